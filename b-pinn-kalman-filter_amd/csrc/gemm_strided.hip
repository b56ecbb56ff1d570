// Strided batched f32 GEMM on the MFMA (v_mfma_f32_16x16x4_f32) for gfx950:
//     C[b](m, n) = alpha * sum_k A[b](m, k) B[b](k, n) (+ bias)
// with every operand addressed by element strides, so one kernel serves the small GEMMs the
// score networks still ran on rocBLAS / hipBLASLt: the time-embedding MLP and the residual
// blocks' Dense_0 projections (nn.Linear: x W^T + b and its two gradients, reference
// models/ncsnpp.py:86-89, layerspp.py:232-262) and the attention block's two batched products
// under autograd (q^T k and v w^T with their gradients, reference layerspp.py:84-88) -- any
// transpose is a choice of strides, no copies.
//
// Workgroup = 64 x 64 outputs of one batch entry, 4 waves in a 2 x 2 grid of 32 x 32 (2 x 2
// MFMA blocks, 16 accumulators per lane).  K runs in chunks of 16 staged through LDS as
// As[k][m] and Bs[k][n] (row pitch 68: the 16 lanes of an operand row hit distinct banks);
// the global loads of chunk c + 1 are issued before chunk c's MFMAs.  Global loads follow
// whichever index of an operand is contiguous (4 consecutive elements per thread along it),
// so both a row-major and a transposed operand read whole cache lines.
// Deterministic (fixed k order, no atomics).
#include "bpk_common.h"

namespace {

using f4 = __attribute__((ext_vector_type(4))) float;

constexpr int kT = 64, kKC = 16, kLP = kT + 4;

struct SbGeo {
  int M, N, K;
  int64_t sab, sam, sak;  // A(b, m, k) = A[b sab + m sam + k sak]
  int64_t sbb, sbk, sbn;  // B(b, k, n) = B[b sbb + k sbk + n sbn]
  int64_t scb, scm, scn;  // C(b, m, n) = C[b scb + m scm + n scn]
  int tiles_m, tiles_n;
  float alpha;
  int bias_mode;          // 0 none, 1 bias[n], 2 bias[m]
  int beta1;              // 1: C += result (accumulate into C)
};

__global__ __launch_bounds__(256) void gemm_sb_kernel(const float* __restrict__ A,
                                                      const float* __restrict__ B,
                                                      const float* __restrict__ bias,
                                                      float* __restrict__ C, SbGeo g) {
  __shared__ __attribute__((aligned(16))) float sA[2][kKC * kLP];
  __shared__ __attribute__((aligned(16))) float sB[2][kKC * kLP];
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int kq = lane >> 4, jj = lane & 15;
  const int wm = wave >> 1, wn = wave & 1;
  int64_t blk = blockIdx.x;
  const int tn = (int)(blk % g.tiles_n);
  blk /= g.tiles_n;
  const int tm = (int)(blk % g.tiles_m);
  const int64_t b = blk / g.tiles_m;
  const int m0 = tm * kT, n0 = tn * kT;
  const float* Ab = A + b * g.sab;
  const float* Bb = B + b * g.sbb;

  // staging map: 4 consecutive elements per thread along the operand's contiguous index
  const bool a_kc = g.sak == 1 && g.sam != 1;  // A contiguous along k (row-major x, W)
  const bool b_nc = g.sbn == 1;                // B contiguous along n
  // A: (m, k0..k0+3) or (m0..m0+3, k)
  const int a_m = a_kc ? tid >> 2 : (tid & 15) * 4;
  const int a_k = a_kc ? (tid & 3) * 4 : tid >> 4;
  // B: (k, n0..n0+3) or (k0..k0+3, n)
  const int b_k = b_nc ? tid >> 4 : (tid & 3) * 4;
  const int b_n = b_nc ? (tid & 15) * 4 : tid >> 2;
  float ra[4], rb[4];
  auto load = [&](int kc) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = m0 + a_m + (a_kc ? 0 : e), k = kc + a_k + (a_kc ? e : 0);
      ra[e] = (m < g.M && k < g.K) ? Ab[(int64_t)m * g.sam + (int64_t)k * g.sak] : 0.f;
      const int kb = kc + b_k + (b_nc ? 0 : e), n = n0 + b_n + (b_nc ? e : 0);
      rb[e] = (kb < g.K && n < g.N) ? Bb[(int64_t)kb * g.sbk + (int64_t)n * g.sbn] : 0.f;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      sA[buf][(a_k + (a_kc ? e : 0)) * kLP + a_m + (a_kc ? 0 : e)] = ra[e];
      sB[buf][(b_k + (b_nc ? 0 : e)) * kLP + b_n + (b_nc ? e : 0)] = rb[e];
    }
  };

  f4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  const int nch = (g.K + kKC - 1) / kKC;
  load(0);
  store(0);
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const int buf = c & 1;
    if (c + 1 < nch) load((c + 1) * kKC);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int k = 4 * ks + kq;
      float a[2], bb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = sA[buf][k * kLP + wm * 32 + i * 16 + jj];
#pragma unroll
      for (int j = 0; j < 2; ++j) bb[j] = sB[buf][k * kLP + wn * 32 + j * 16 + jj];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], bb[j], acc[i][j], 0, 0, 0);
    }
    if (c + 1 < nch) store(buf ^ 1);
    __syncthreads();
  }

  // acc[i][j][r] = C(m0 + 32 wm + 16 i + 4 kq + r, n0 + 32 wn + 16 j + jj)
  float* Cb = C + b * g.scb;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + 32 * wn + 16 * j + jj;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + 32 * wm + 16 * i + 4 * kq + r;
        if (m >= g.M || n >= g.N) continue;
        float v = g.alpha * acc[i][j][r];
        if (g.bias_mode == 1) v += bias[n];
        if (g.bias_mode == 2) v += bias[m];
        float* o = Cb + (int64_t)m * g.scm + (int64_t)n * g.scn;
        *o = g.beta1 ? *o + v : v;
      }
    }
}

}  // namespace

extern "C" int bpk_gemm_sb_f32(const float* A, int64_t sab, int64_t sam, int64_t sak,
                               const float* B, int64_t sbb, int64_t sbk, int64_t sbn, float* C,
                               int64_t scb, int64_t scm, int64_t scn, const float* bias,
                               int bias_mode, float alpha, int accumulate, int batch, int M,
                               int N, int K, void* stream) {
  BPK_REQUIRE(batch >= 0 && M >= 0 && N >= 0 && K >= 0, "gemm_sb: negative size");
  BPK_REQUIRE(bias_mode >= 0 && bias_mode <= 2 && (bias_mode == 0 || bias != nullptr),
              "gemm_sb: bad bias mode %d", bias_mode);
  if (batch == 0 || M == 0 || N == 0) return BPK_OK;
  SbGeo g{M, N, K, sab, sam, sak, sbb, sbk, sbn, scb, scm, scn,
          (M + kT - 1) / kT, (N + kT - 1) / kT, alpha, bias_mode, accumulate ? 1 : 0};
  const int64_t blocks = (int64_t)batch * g.tiles_m * g.tiles_n;
  BPK_REQUIRE(blocks < (1LL << 31), "gemm_sb: grid too large");
  hipLaunchKernelGGL(gemm_sb_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     bpk::as_stream(stream), A, B, bias, C, g);
  BPK_LAUNCH_CHECK("gemm_sb");
  return BPK_OK;
}
