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

template <int NKB>  // key blocks of 16: P = 16 NKB
__global__ __launch_bounds__(256) void attn_fwd_kernel(const float* __restrict__ qkv,
                                                       float* __restrict__ out, int C,
                                                       float scale) {
  constexpr int P = 16 * NKB;
  constexpr int kKP = P + 16;    // Kc pitch: bank 16 kq + jj
  constexpr int kQP = kQB + 16;  // Qc pitch
  constexpr int kPP = P + 4;     // probability rows: bank 4 jj + kq
  constexpr int kVP = P + 4;     // Vc pitch
  constexpr int kStage1 = kCC * kKP + kCC * kQP;
  constexpr int kStage3 = kQB * kPP + kCC * kVP;
  __shared__ __attribute__((aligned(16))) float smem[kStage1 > kStage3 ? kStage1 : kStage3];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int kq = lane >> 4, jj = lane & 15;
  constexpr int nqb = P / kQB;
  const int b = blockIdx.x / nqb;
  const int q0 = (blockIdx.x % nqb) * kQB;
  const int64_t cp = (int64_t)C * P;
  const float* qp = qkv + (int64_t)b * 3 * cp;
  const float* kp = qp + cp;
  const float* vp = qp + 2 * cp;

  // 1. logits S[16 queries of this wave][P keys]
  f4 s[NKB];
#pragma unroll
  for (int nb = 0; nb < NKB; ++nb) s[nb] = f4{0.f, 0.f, 0.f, 0.f};
  float* Kc = smem;
  float* Qc = smem + kCC * kKP;
  for (int c0 = 0; c0 < C; c0 += kCC) {
    __syncthreads();
    for (int e = tid; e < kCC * P / 4; e += 256) {
      const int r = e / (P / 4), col = e - r * (P / 4);
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
  __syncthreads();  // stage-1 buffers are reused below
  float* Pm = smem;
  float* Vc = smem + kQB * kPP;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float inv = 1.f / sm[r];
#pragma unroll
    for (int nb = 0; nb < NKB; ++nb)
      Pm[(wave * 16 + 4 * kq + r) * kPP + nb * 16 + jj] = s[nb][r] * inv;
  }

  // 3. O[query][channel] = sum_key P[query][key] V[channel][key], 32 channels per pass
  float* op = out + (int64_t)b * cp;
  for (int c0 = 0; c0 < C; c0 += kCC) {
    __syncthreads();  // Pm written / previous Vc reads done
    for (int e = tid; e < kCC * P / 4; e += 256) {
      const int r = e / (P / 4), col = e - r * (P / 4);
      *reinterpret_cast<f4*>(&Vc[r * kVP + 4 * col]) =
          *reinterpret_cast<const f4*>(&vp[(int64_t)(c0 + r) * P + 4 * col]);
    }
    __syncthreads();
    f4 o[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll 8
    for (int kk = 0; kk < P / 4; ++kk) {
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

}  // namespace

extern "C" int bpk_attention_supported(int B, int C, int P) {
  return B > 0 && C > 0 && C % kCC == 0 && (P == 64 || P == 128 || P == 256);
}

extern "C" int bpk_attention_f32(const float* qkv, float* out, int B, int C, int P, float scale,
                                 void* stream) {
  BPK_REQUIRE(bpk_attention_supported(B, C, P),
              "attention: unsupported shape B=%d C=%d P=%d (need C %% 32 == 0, P in {64, 128, 256})",
              B, C, P);
  BPK_REQUIRE((int64_t)B * (P / kQB) < (1LL << 31), "attention: grid too large");
  const dim3 grid((unsigned)(B * (P / kQB)));
  hipStream_t st = bpk::as_stream(stream);
  if (P == 256)
    hipLaunchKernelGGL(attn_fwd_kernel<16>, grid, dim3(256), 0, st, qkv, out, C, scale);
  else if (P == 128)
    hipLaunchKernelGGL(attn_fwd_kernel<8>, grid, dim3(256), 0, st, qkv, out, C, scale);
  else
    hipLaunchKernelGGL(attn_fwd_kernel<4>, grid, dim3(256), 0, st, qkv, out, C, scale);
  BPK_LAUNCH_CHECK("attention");
  return BPK_OK;
}
