// 1x1 convolution of NCHW tensors as an f32 MFMA GEMM (v_mfma_f32_16x16x4_f32), with an
// optional second source along K:
//     Y[n] (M x P) = W1 (M x K1) X1[n] (K1 x P) + W2 (M x K2) X2[n] (K2 x P) + bias
// where P = H * W pixels.  The score networks' 1x1 convs (the residual blocks' Conv_2 skip
// projection and the attention NINs, models/layerspp.py / layers.py) run on it; the second
// source lets the up path's skip projection read [h, skip] without materialising their
// channel concatenation (W2 = the weight's trailing K2 columns, same row stride).
//
// Workgroup = 128 output channels x 128 pixels of one image, 4 waves in a 2 x 2 grid of
// 64 x 64 (4 x 4 MFMA blocks, 64 accumulators per lane).  K runs in chunks of 16:
//   * A tile W[m][k] in LDS at row stride 20 (lane (j, kq) reads its 4 k values
//     4 kq .. 4 kq + 3 of row m with one 16-byte read, conflict-free);
//   * B tile X[k][p] in LDS at row stride 132 (lane (j, kq) reads X[4 kq + ks][p + j]:
//     the two kq halves of a 32-lane group sit 16 banks apart);
//   * MFMA k-step ks multiplies k = 4 kq + ks (any k order is fine as long as A and B agree);
//   * global loads of chunk c + 2 in registers, LDS stores of chunk c + 1 behind chunk c's
//     64 MFMAs per wave, double-buffered tiles, one barrier per chunk;
//   * epilogue straight from the accumulators: 16 consecutive pixels (64 B) per row.
#include "bpk_common.h"

#include <algorithm>

namespace {

using f4 = __attribute__((ext_vector_type(4))) float;

constexpr int kBM = 128, kBP = 128, kKC = 16;
constexpr int kAS = 20;    // A row stride (floats)
constexpr int kBS = 132;   // B row stride (floats)

struct GemmGeo {
  int N, M, P, K1, K2, ldw;
  int tiles_m, tiles_p;
};

__global__ __launch_bounds__(256, 2) void gemm_nchw_kernel(
    const float* __restrict__ W1, const float* __restrict__ X1, const float* __restrict__ W2,
    const float* __restrict__ X2, const float* __restrict__ bias, float* __restrict__ Y,
    GemmGeo g, int xcd_remap) {
  __shared__ __attribute__((aligned(16))) float sA[2][kBM * kAS];  // 2 x 10 KB
  __shared__ __attribute__((aligned(16))) float sB[2][kKC * kBS];  // 2 x 8.4 KB

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int kq = lane >> 4, jj = lane & 15;
  const int wm = wave >> 1, wp = wave & 1;
  int64_t nblk = (int64_t)gridDim.x;
  int64_t b = blockIdx.x;
  if (xcd_remap) b = (b % 8) * (nblk / 8) + b / 8;
  // logical order: the M tiles of one pixel tile are consecutive (they share X in L2)
  const int tm = (int)(b % g.tiles_m);
  int64_t r = b / g.tiles_m;
  const int tp = (int)(r % g.tiles_p);
  const int n = (int)(r / g.tiles_p);
  const int m0 = tm * kBM, p0 = tp * kBP;
  const int nch1 = g.K1 / kKC, nch = nch1 + g.K2 / kKC;

  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  // global loads of one chunk: A 128 x 16 (2 f4 per thread), B 16 x 128 (2 f4 per thread)
  const int am = tid >> 2, ak = (tid & 3) * 4;       // A rows am, am + 64; k offset ak
  const int bk = tid >> 5, bp = (tid & 31) * 4;      // B rows bk, bk + 8; pixel offset bp
  f4 ra[2], rb[2];
  auto load = [&](int c) {
    c = min(c, nch - 1);  // past the end: re-load the last chunk (never consumed)
    const bool second = c >= nch1;
    const int k0 = (second ? c - nch1 : c) * kKC;
    const float* Wp = second ? W2 : W1;
    const float* Xp = second ? X2 : X1;
    const int K = second ? g.K2 : g.K1;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      ra[i] = *reinterpret_cast<const f4*>(&Wp[(int64_t)(m0 + am + 64 * i) * g.ldw + k0 + ak]);
    const float* xb = Xp + ((int64_t)n * K + k0) * g.P + p0 + bp;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      rb[i] = *reinterpret_cast<const f4*>(&xb[(int64_t)(bk + 8 * i) * g.P]);
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      *reinterpret_cast<f4*>(&sA[buf][(am + 64 * i) * kAS + ak]) = ra[i];
      *reinterpret_cast<f4*>(&sB[buf][(bk + 8 * i) * kBS + bp]) = rb[i];
    }
  };

  load(0);
  store(0);
  load(1);
  __syncthreads();

  for (int c = 0; c < nch; ++c) {
    const int buf = c & 1;
    // operands of this chunk
    f4 a[4];
    float bv[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      a[i] = *reinterpret_cast<const f4*>(&sA[buf][(64 * wm + 16 * i + jj) * kAS + 4 * kq]);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        bv[j][ks] = sB[buf][(4 * kq + ks) * kBS + 64 * wp + 16 * j + jj];
    // next chunk's tiles into the other buffer, the one after into registers
    if (c + 1 < nch) store(buf ^ 1);
    load(c + 2);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][ks], bv[j][ks], acc[i][j], 0, 0,
                                                           0);
    __syncthreads();
  }

  // acc[i][j][rr] = Y[m0 + 64 wm + 16 i + 4 kq + rr][p0 + 64 wp + 16 j + jj]
  float* yn = Y + (int64_t)n * g.M * g.P;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int m = m0 + 64 * wm + 16 * i + 4 * kq + rr;
      const float bb = bias ? bias[m] : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) yn[(int64_t)m * g.P + p0 + 64 * wp + 16 * j + jj] = acc[i][j][rr] + bb;
    }
}

}  // namespace

extern "C" int bpk_gemm_nchw_supported(int N, int M, int P, int K1, int K2) {
  return N > 0 && M > 0 && P > 0 && K1 > 0 && K2 >= 0 && M % kBM == 0 && P % kBP == 0 &&
         K1 % kKC == 0 && K2 % kKC == 0;
}

extern "C" int bpk_gemm_nchw_f32(const float* W, int ldw, const float* X1, int K1,
                                 const float* X2, int K2, const float* bias, float* Y, int N,
                                 int M, int P, void* stream) {
  BPK_REQUIRE(bpk_gemm_nchw_supported(N, M, P, K1, K2),
              "gemm_nchw: unsupported shape N=%d M=%d P=%d K1=%d K2=%d (need M %% 128, "
              "P %% 128, K %% 16 == 0)", N, M, P, K1, K2);
  BPK_REQUIRE(ldw >= K1 + K2 && ldw % 4 == 0, "gemm_nchw: bad weight row stride %d", ldw);
  BPK_REQUIRE(K2 == 0 || X2 != nullptr, "gemm_nchw: K2 > 0 needs X2");
  GemmGeo g{N, M, P, K1, K2, ldw, M / kBM, P / kBP};
  const int64_t blocks = (int64_t)N * g.tiles_m * g.tiles_p;
  BPK_REQUIRE(blocks < (1LL << 31), "gemm_nchw: grid too large");
  const int remap = (blocks % 8 == 0) ? 1 : 0;
  hipLaunchKernelGGL(gemm_nchw_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     bpk::as_stream(stream), W, X1, K2 ? W + K1 : W, K2 ? X2 : X1, bias, Y, g,
                     remap);
  BPK_LAUNCH_CHECK("gemm_nchw");
  return BPK_OK;
}
