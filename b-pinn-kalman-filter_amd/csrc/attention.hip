// Channel self-attention of the score networks' attention blocks (AttnBlockpp, reference
// models/layerspp.py:75-91; AttnBlock, models/layers.py:549-573) in one kernel on the f32
// MFMA (v_mfma_f32_16x16x4_f32) for gfx950:
//     out[b, c, i] = sum_j v[b, c, j] * softmax_j( scale * sum_c' q[b, c', i] k[b, c', j] )
// q, k, v are the three channel blocks of the stacked 1x1 projection qkv [B, 3, C, P]
// (P = H*W positions), out is [B, C, P] -- the layout the reference's einsum / bmm pair
// produces before NIN_3.  The reference runs this as two batched GEMMs with the [P, P]
// logits written to and re-read from HBM around a softmax kernel; here a workgroup owns 64
// queries of one sample and keeps their logits on chip:
//   1. S = Q^T K: each of the 4 waves accumulates 16 queries x P keys in registers over
//      C / 4 MFMA k-steps, K and Q staged through LDS 32 channels at a time;
//   2. row softmax in registers (max / sum over the 16 lanes of a row by xor shuffles),
//      probabilities to LDS (the PV product needs them as A operands);
//   3. O = P V^T: 32 output channels per pass, V staged through LDS, each lane storing 4
//      consecutive queries of one channel (16-byte stores along P).
// LDS pitches are padded so that the 16 lanes of an MFMA operand row hit distinct banks.
#include "bpk_common.h"

namespace {

using f4 = __attribute__((ext_vector_type(4))) float;

constexpr int kQB = 64;  // queries per workgroup: 4 waves x 16
constexpr int kCC = 32;  // channels per staged chunk

// Key split (nsplit > 1, small batches: B x P / 64 workgroups would leave most CUs idle):
// workgroup (b, query block, s) takes keys [s PK, (s + 1) PK) only and writes its
// unnormalised partial output exp(S - m_s) V to out + s * B * C * P with the row statistics
// (m_s, l_s = sum exp(S - m_s)) to stats; attn_combine_kernel merges the splits.
template <int NKB>  // key blocks of 16 per workgroup: PK = 16 NKB keys
__global__ __launch_bounds__(256) void attn_fwd_kernel(const float* __restrict__ qkv,
                                                       float* __restrict__ out, int C,
                                                       float scale, int P, int nsplit,
                                                       float2* __restrict__ stats) {
  constexpr int PK = 16 * NKB;
  constexpr int kKP = PK + 16;   // Kc pitch: bank 16 kq + jj
  constexpr int kQP = kQB + 16;  // Qc pitch
  constexpr int kPP = PK + 4;    // probability rows: bank 4 jj + kq
  constexpr int kVP = PK + 4;    // Vc pitch
  constexpr int kStage1 = kCC * kKP + kCC * kQP;
  constexpr int kStage3 = kQB * kPP + kCC * kVP;
  __shared__ __attribute__((aligned(16))) float smem[kStage1 > kStage3 ? kStage1 : kStage3];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int kq = lane >> 4, jj = lane & 15;
  const int nqb = P / kQB;
  const int split = blockIdx.x % nsplit;
  const int b = blockIdx.x / (nqb * nsplit);
  const int q0 = ((blockIdx.x / nsplit) % nqb) * kQB;
  const int k0 = split * PK;
  const int64_t cp = (int64_t)C * P;
  const float* qp = qkv + (int64_t)b * 3 * cp;
  const float* kp = qp + cp + k0;
  const float* vp = qp + 2 * cp + k0;

  // 1. logits S[16 queries of this wave][P keys]
  f4 s[NKB];
#pragma unroll
  for (int nb = 0; nb < NKB; ++nb) s[nb] = f4{0.f, 0.f, 0.f, 0.f};
  float* Kc = smem;
  float* Qc = smem + kCC * kKP;
  for (int c0 = 0; c0 < C; c0 += kCC) {
    __syncthreads();
    for (int e = tid; e < kCC * PK / 4; e += 256) {
      const int r = e / (PK / 4), col = e - r * (PK / 4);
      *reinterpret_cast<f4*>(&Kc[r * kKP + 4 * col]) =
          *reinterpret_cast<const f4*>(&kp[(int64_t)(c0 + r) * P + 4 * col]);
    }
    for (int e = tid; e < kCC * kQB / 4; e += 256) {
      const int r = e / (kQB / 4), col = e - r * (kQB / 4);
      *reinterpret_cast<f4*>(&Qc[r * kQP + 4 * col]) =
          *reinterpret_cast<const f4*>(&qp[(int64_t)(c0 + r) * P + q0 + 4 * col]);
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < kCC / 4; ++kk) {
      const float a = Qc[(4 * kk + kq) * kQP + wave * 16 + jj];
#pragma unroll
      for (int nb = 0; nb < NKB; ++nb)
        s[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, Kc[(4 * kk + kq) * kKP + nb * 16 + jj],
                                                     s[nb], 0, 0, 0);
    }
  }

  // 2. softmax over the keys of each query row: lane (kq, jj) holds rows 4 kq + r, keys
  // 16 nb + jj; a row's 16 lanes differ in the low four lane bits
  float mx[4], sm[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float m = -INFINITY;
#pragma unroll
    for (int nb = 0; nb < NKB; ++nb) {
      s[nb][r] *= scale;
      m = fmaxf(m, s[nb][r]);
    }
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
    mx[r] = m;
    float z = 0.f;
#pragma unroll
    for (int nb = 0; nb < NKB; ++nb) {
      s[nb][r] = expf(s[nb][r] - m);
      z += s[nb][r];
    }
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) z += __shfl_xor(z, off, 64);
    sm[r] = z;
  }
  const int nb_all = gridDim.x / (nsplit * nqb);  // batch size
  if (nsplit > 1 && jj == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      stats[((int64_t)split * nb_all + b) * P + q0 + wave * 16 + 4 * kq + r] =
          make_float2(mx[r], sm[r]);
  }
  __syncthreads();  // stage-1 buffers are reused below
  float* Pm = smem;
  float* Vc = smem + kQB * kPP;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float inv = nsplit > 1 ? 1.f : 1.f / sm[r];
#pragma unroll
    for (int nb = 0; nb < NKB; ++nb)
      Pm[(wave * 16 + 4 * kq + r) * kPP + nb * 16 + jj] = s[nb][r] * inv;
  }

  // 3. O[query][channel] = sum_key P[query][key] V[channel][key], 32 channels per pass
  float* op = out + ((int64_t)split * nb_all + b) * cp;
  for (int c0 = 0; c0 < C; c0 += kCC) {
    __syncthreads();  // Pm written / previous Vc reads done
    for (int e = tid; e < kCC * PK / 4; e += 256) {
      const int r = e / (PK / 4), col = e - r * (PK / 4);
      *reinterpret_cast<f4*>(&Vc[r * kVP + 4 * col]) =
          *reinterpret_cast<const f4*>(&vp[(int64_t)(c0 + r) * P + 4 * col]);
    }
    __syncthreads();
    f4 o[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll 8
    for (int kk = 0; kk < PK / 4; ++kk) {
      const float a = Pm[(wave * 16 + jj) * kPP + 4 * kk + kq];
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
        o[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, Vc[(nb * 16 + jj) * kVP + 4 * kk + kq],
                                                     o[nb], 0, 0, 0);
    }
    // lane (kq, jj) holds queries 4 kq + r of channel 16 nb + jj: one 16-byte store each
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
      *reinterpret_cast<f4*>(&op[(int64_t)(c0 + nb * 16 + jj) * P + q0 + wave * 16 + 4 * kq]) = o[nb];
  }
}

// out[b][c][q] = sum_s e^{m_s - M} O_s[b][c][q] / sum_s e^{m_s - M} l_s, M = max_s m_s
// (the key splits of attn_fwd_kernel merged in a fixed order); 4 queries per thread
__global__ __launch_bounds__(256) void attn_combine_kernel(const float* __restrict__ part,
                                                           const float2* __restrict__ stats,
                                                           float* __restrict__ out, int B,
                                                           int C, int P, int nsplit) {
  const int64_t i4 = (int64_t)blockIdx.x * 256 + threadIdx.x;  // index of 4 outputs
  const int64_t n4 = (int64_t)B * C * P / 4;
  if (i4 >= n4) return;
  const int q = (int)((i4 * 4) % P);
  const int b = (int)(i4 * 4 / ((int64_t)C * P));
  const int64_t slab = (int64_t)B * C * P;
  f4 num = f4{0.f, 0.f, 0.f, 0.f}, den = num, mm;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float m = -INFINITY;
    for (int s = 0; s < nsplit; ++s) m = fmaxf(m, stats[((int64_t)s * B + b) * P + q + e].x);
    mm[e] = m;
  }
  for (int s = 0; s < nsplit; ++s) {
    const f4 o = reinterpret_cast<const f4*>(part + s * slab)[i4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float2 st = stats[((int64_t)s * B + b) * P + q + e];
      const float w = expf(st.x - mm[e]);
      num[e] = fmaf(w, o[e], num[e]);
      den[e] = fmaf(w, st.y, den[e]);
    }
  }
  reinterpret_cast<f4*>(out)[i4] = f4{num[0] / den[0], num[1] / den[1], num[2] / den[2],
                                      num[3] / den[3]};
}

// key splits for a launch of B x P / 64 workgroups: up to 4 (at least 64 keys each) while the
// grid stays within one workgroup per CU
int attn_splits(int B, int P) {
  static const int cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  const int64_t wg = (int64_t)B * (P / kQB);
  int S = 1;
  while (S < 4 && P / (2 * S) >= 64 && wg * S * 2 <= cus) S *= 2;
  return S;
}

template <int NKB>
void launch_fwd(const float* qkv, float* out, int B, int C, int P, float scale, int S,
                float2* stats, hipStream_t st) {
  const dim3 grid((unsigned)((int64_t)B * (P / kQB) * S));
  hipLaunchKernelGGL(attn_fwd_kernel<NKB>, grid, dim3(256), 0, st, qkv, out, C, scale, P, S,
                     stats);
}

int attention_impl(const float* qkv, float* out, float* ws, int B, int C, int P, float scale,
                   int S, hipStream_t st) {
  BPK_REQUIRE((int64_t)B * (P / kQB) * S < (1LL << 31), "attention: grid too large");
  float* o = S > 1 ? ws : out;
  float2* stats = S > 1 ? reinterpret_cast<float2*>(ws + (int64_t)S * B * C * P) : nullptr;
  switch (P / S) {
    case 256: launch_fwd<16>(qkv, o, B, C, P, scale, S, stats, st); break;
    case 128: launch_fwd<8>(qkv, o, B, C, P, scale, S, stats, st); break;
    default: launch_fwd<4>(qkv, o, B, C, P, scale, S, stats, st); break;
  }
  BPK_LAUNCH_CHECK("attention");
  if (S > 1) {
    const int64_t n4 = (int64_t)B * C * P / 4;
    hipLaunchKernelGGL(attn_combine_kernel, dim3((unsigned)bpk::ceil_div(n4, 256)), dim3(256), 0,
                       st, ws, stats, out, B, C, P, S);
    BPK_LAUNCH_CHECK("attention_combine");
  }
  return BPK_OK;
}

}  // namespace

extern "C" int bpk_attention_supported(int B, int C, int P) {
  return B > 0 && C > 0 && C % kCC == 0 && (P == 64 || P == 128 || P == 256);
}

extern "C" int bpk_attention_f32(const float* qkv, float* out, int B, int C, int P, float scale,
                                 void* stream) {
  BPK_REQUIRE(bpk_attention_supported(B, C, P),
              "attention: unsupported shape B=%d C=%d P=%d (need C %% 32 == 0, P in {64, 128, 256})",
              B, C, P);
  return attention_impl(qkv, out, nullptr, B, C, P, scale, 1, bpk::as_stream(stream));
}

extern "C" int64_t bpk_attention_workspace_bytes(int B, int C, int P) {
  if (!bpk_attention_supported(B, C, P)) return 0;
  const int S = attn_splits(B, P);
  return S > 1 ? (int64_t)S * B * P * (C + 2) * (int64_t)sizeof(float) : 0;
}

extern "C" int bpk_attention_ex_f32(const float* qkv, float* out, float* workspace, int B, int C,
                                    int P, float scale, void* stream) {
  BPK_REQUIRE(bpk_attention_supported(B, C, P),
              "attention: unsupported shape B=%d C=%d P=%d (need C %% 32 == 0, P in {64, 128, 256})",
              B, C, P);
  const int S = attn_splits(B, P);
  BPK_REQUIRE(S == 1 || workspace != nullptr, "attention: workspace is NULL");
  return attention_impl(qkv, out, workspace, B, C, P, scale, S, bpk::as_stream(stream));
}
