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
  int ksplit;  // > 1: split-K; workgroup slice s contracts chunks [s, s + 1) * nch / ksplit and
               // stores its raw partial to Y + s * N * M * P (gemm_splitk_reduce_kernel adds)
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
  r /= g.tiles_p;
  const int n = (int)(r % g.N);
  const int ks_idx = (int)(r / g.N);  // split-K slice (0 unless ksplit > 1)
  const int m0 = tm * kBM, p0 = tp * kBP;
  const int nch1 = g.K1 / kKC;
  const int ncs = (nch1 + g.K2 / kKC) / max(g.ksplit, 1);  // chunks of this workgroup
  const int cb = ks_idx * ncs;                              // its first chunk
  const int nch = cb + ncs;                                 // one past its last

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
    for (int i = 0; i < 2; ++i)  // rows past M (M % 128 != 0): zero
      ra[i] = m0 + am + 64 * i < g.M
                  ? *reinterpret_cast<const f4*>(&Wp[(int64_t)(m0 + am + 64 * i) * g.ldw + k0 + ak])
                  : f4{0.f, 0.f, 0.f, 0.f};
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

  load(cb);
  store(0);
  load(cb + 1);
  __syncthreads();

  for (int c = cb; c < nch; ++c) {
    const int buf = (c - cb) & 1;
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
  float* yn = Y + ((int64_t)ks_idx * g.N + n) * g.M * g.P;
  // the 16 bias values of this lane requested together (loaded per row before a store
  // group, the compiler waited for each in turn: 16 exposed latencies per workgroup)
  float bbv[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int m = m0 + 64 * wm + 16 * i + 4 * kq + rr;
      bbv[i][rr] = (bias && m < g.M) ? bias[m] : 0.f;
    }
  // a whole 128-row tile in range (every NCSN++ / DDPM++ shape): one straight-line store
  // block -- the per-row guard put each store group in its own branch, and the wait counter
  // (vmcnt counts stores on gfx9) was drained to 0 at every one of them
  if (m0 + kBM <= g.M) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int m = m0 + 64 * wm + 16 * i + 4 * kq + rr;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          yn[(int64_t)m * g.P + p0 + 64 * wp + 16 * j + jj] = acc[i][j][rr] + bbv[i][rr];
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int m = m0 + 64 * wm + 16 * i + 4 * kq + rr;
      if (m >= g.M) continue;
      const float bb = bbv[i][rr];
#pragma unroll
      for (int j = 0; j < 4; ++j) yn[(int64_t)m * g.P + p0 + 64 * wp + 16 * j + jj] = acc[i][j][rr] + bb;
    }
}


// y[n][m][p] = sum_s part[s][n][m][p] + bias[m] (fixed order), 4 pixels per thread
__global__ __launch_bounds__(256) void gemm_splitk_reduce_kernel(const f4* __restrict__ part,
                                                                 int S, int64_t slab4,
                                                                 const float* __restrict__ bias,
                                                                 f4* __restrict__ y, int M,
                                                                 int P4) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= slab4) return;
  f4 v = part[i];
  for (int s = 1; s < S; ++s) v += part[s * slab4 + i];
  if (bias) {
    const float b = bias[(int)((i / P4) % M)];
    v += f4{b, b, b, b};
  }
  y[i] = v;
}


// ---------------------------------------------------------------- weight gradient
// dW (M x K) = sum_n GY[n] (M x P) X[n]^T (P x K)  and  db[m] = sum_{n,p} GY[n][m][p]:
// the 1x1 conv's weight / bias gradient.  The reduction runs over the N * P pixels in
// chunks of 16; both operands keep pixels contiguous, so both tiles sit in LDS as
// [row][pixel] at stride 20 and every lane reads its four k-step values with one 16-byte
// read.  Split-K over pixel ranges (deterministic: per-split partial slabs, summed in a
// fixed order by gemm_wgrad_reduce_kernel).
struct WgGeo {
  int N, M, K, P;
  int tiles_m, tiles_k, splits, cps;  // chunks per split
};

__global__ __launch_bounds__(256, 2) void gemm_nchw_wgrad_kernel(
    const float* __restrict__ GY, const float* __restrict__ X, float* __restrict__ part,
    float* __restrict__ part_b, WgGeo g, int xcd_remap) {
  __shared__ __attribute__((aligned(16))) float sA[2][kBM * kAS];  // GY tile [m][p]
  __shared__ __attribute__((aligned(16))) float sB[2][kBM * kAS];  // X tile  [k][p]

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int kq = lane >> 4, jj = lane & 15;
  const int wm = wave >> 1, wk = wave & 1;
  int b = blockIdx.x;
  const int nblk = gridDim.x;
  if (xcd_remap) b = (b % 8) * (nblk / 8) + b / 8;
  const int tiles = g.tiles_m * g.tiles_k;
  const int s = b / tiles, t = b % tiles;
  const int tm = t / g.tiles_k, tk = t % g.tiles_k;
  const int m0 = tm * kBM, k0 = tk * kBM;
  const int cpi = g.P / kKC;                           // chunks per image
  const int c0 = s * g.cps;
  const int nch = min(g.cps, g.N * cpi - c0);          // >= 1 by construction

  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  float bsum[4] = {0.f, 0.f, 0.f, 0.f};

  // loads: rows r, r + 64 of both tiles, pixels 4 (tid & 3) .. + 3 of the chunk
  const int lr = tid >> 2, lp = (tid & 3) * 4;
  int ln = c0 / cpi, lpc = c0 % cpi, left = nch;       // load cursor (image, chunk in image)
  f4 ra[2], rb[2];
  auto load = [&]() {
    const float* gy = GY + ((int64_t)ln * g.M + m0 + lr) * g.P + lpc * kKC + lp;
    const float* xx = X + ((int64_t)ln * g.K + k0 + lr) * g.P + lpc * kKC + lp;
#pragma unroll
    for (int i = 0; i < 2; ++i) {  // rows past M / K: zero
      ra[i] = m0 + lr + 64 * i < g.M ? *reinterpret_cast<const f4*>(gy + (int64_t)(64 * i) * g.P)
                                     : f4{0.f, 0.f, 0.f, 0.f};
      rb[i] = k0 + lr + 64 * i < g.K ? *reinterpret_cast<const f4*>(xx + (int64_t)(64 * i) * g.P)
                                     : f4{0.f, 0.f, 0.f, 0.f};
    }
    if (--left > 0 && ++lpc == cpi) { lpc = 0; ++ln; }  // past the end: re-load the last chunk
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      *reinterpret_cast<f4*>(&sA[buf][(lr + 64 * i) * kAS + lp]) = ra[i];
      *reinterpret_cast<f4*>(&sB[buf][(lr + 64 * i) * kAS + lp]) = rb[i];
    }
  };

  load();
  store(0);
  load();
  __syncthreads();

  for (int c = 0; c < nch; ++c) {
    const int buf = c & 1;
    f4 a[4], bv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[i] = *reinterpret_cast<const f4*>(&sA[buf][(64 * wm + 16 * i + jj) * kAS + 4 * kq]);
      bv[i] = *reinterpret_cast<const f4*>(&sB[buf][(64 * wk + 16 * i + jj) * kAS + 4 * kq]);
    }
    if (c + 1 < nch) store(buf ^ 1);
    load();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][ks], bv[j][ks], acc[i][j], 0, 0,
                                                           0);
#pragma unroll
    for (int i = 0; i < 4; ++i) bsum[i] += (a[i].x + a[i].y) + (a[i].z + a[i].w);
    __syncthreads();
  }

  // acc[i][j][rr] = dW[m0 + 64 wm + 16 i + 4 kq + rr][k0 + 64 wk + 16 j + jj]
  float* ps = part + (int64_t)s * g.M * g.K;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int m = m0 + 64 * wm + 16 * i + 4 * kq + rr;
      if (m >= g.M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = k0 + 64 * wk + 16 * j + jj;
        if (k < g.K) ps[(int64_t)m * g.K + k] = acc[i][j][rr];
      }
    }
  if (part_b != nullptr && tk == 0 && wk == 0) {  // bias: rows of this wave, summed over kq
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v = bsum[i];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      if (kq == 0 && m0 + 64 * wm + 16 * i + jj < g.M)
        part_b[(int64_t)s * g.M + m0 + 64 * wm + 16 * i + jj] = v;
    }
  }
}

// out[i] = sum_s part[s][i] for i < n4 float4s (fixed order; 4 split groups per column,
// combined through LDS), and ob[m] = sum_s part_b[s][m].
__global__ __launch_bounds__(256) void gemm_wgrad_reduce_kernel(
    const f4* __restrict__ part, f4* __restrict__ out, const float* __restrict__ part_b,
    float* __restrict__ ob, int64_t n4, int M, int splits) {
  __shared__ f4 red[4][64];
  const int col = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + col;
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
  if (i < n4) {
    // eight loads in flight per thread (the adds stay in split order: the same sum); one at a
    // time, hundreds of splits made this kernel latency-bound (~90 us on PressureNet shapes)
    int s = grp;
    for (; s + 28 < splits; s += 32) {
      f4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(s + 4 * u) * n4 + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; s < splits; s += 4) acc += part[(int64_t)s * n4 + i];
  }
  red[grp][col] = acc;
  __syncthreads();
  if (grp == 0 && i < n4) out[i] = ((red[0][col] + red[1][col]) + red[2][col]) + red[3][col];
  if (ob != nullptr && blockIdx.x == 0)
    for (int m = threadIdx.x; m < M; m += 256) {
      float v = 0.f;
      int s = 0;
      for (; s + 7 < splits; s += 8) {
        float t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = part_b[(int64_t)(s + u) * M + m];
#pragma unroll
        for (int u = 0; u < 8; ++u) v += t[u];
      }
      for (; s < splits; ++s) v += part_b[(int64_t)s * M + m];
      ob[m] = v;
    }
}

WgGeo wgrad_geo(int N, int M, int K, int P) {
  WgGeo g{N, M, K, P, (M + kBM - 1) / kBM, (K + kBM - 1) / kBM, 1, 0};
  const int64_t chunks = (int64_t)N * (P / kKC);
  const int tiles = g.tiles_m * g.tiles_k;
  // ~1024 workgroups (4 per CU), at least 8 chunks (128 pixels) per split, at most 256 splits
  // (PressureNet's 1x1 shortcuts, tools/bench_wgrad1x1.py, round 6: 64 chunks per split left
  // 32-128 workgroups on the chip at B = 8, ~95 us a call; now 20-34 us; B = 64 1.66 -> ~1.0
  // ms over the shapes)
  int64_t splits = std::max<int64_t>(
      1, std::min<int64_t>(std::min<int64_t>(bpk::ceil_div(1024, tiles), 256), chunks / 8));
  g.cps = (int)bpk::ceil_div(chunks, splits);
  g.splits = (int)bpk::ceil_div(chunks, (int64_t)g.cps);  // every split non-empty
  return g;
}

}  // namespace

extern "C" int bpk_gemm_nchw_supported(int N, int M, int P, int K1, int K2) {
  return N > 0 && M > 0 && P > 0 && K1 > 0 && K2 >= 0 && M % 16 == 0 && P % kBP == 0 &&
         K1 % kKC == 0 && K2 % kKC == 0;
}

extern "C" int bpk_gemm_nchw_f32(const float* W, int ldw, const float* X1, int K1,
                                 const float* X2, int K2, const float* bias, float* Y, int N,
                                 int M, int P, void* stream) {
  BPK_REQUIRE(bpk_gemm_nchw_supported(N, M, P, K1, K2),
              "gemm_nchw: unsupported shape N=%d M=%d P=%d K1=%d K2=%d (need M %% 16, "
              "P %% 128, K %% 16 == 0)", N, M, P, K1, K2);
  BPK_REQUIRE(ldw >= K1 + K2 && ldw % 4 == 0, "gemm_nchw: bad weight row stride %d", ldw);
  BPK_REQUIRE(K2 == 0 || X2 != nullptr, "gemm_nchw: K2 > 0 needs X2");
  GemmGeo g{N, M, P, K1, K2, ldw, (M + kBM - 1) / kBM, P / kBP, 1};
  const int64_t blocks = (int64_t)N * g.tiles_m * g.tiles_p;
  BPK_REQUIRE(blocks < (1LL << 31), "gemm_nchw: grid too large");
  const int remap = (blocks % 8 == 0) ? 1 : 0;
  hipLaunchKernelGGL(gemm_nchw_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     bpk::as_stream(stream), W, X1, K2 ? W + K1 : W, K2 ? X2 : X1, bias, Y, g,
                     remap);
  BPK_LAUNCH_CHECK("gemm_nchw");
  return BPK_OK;
}

// Split-K for launches that leave most of the chip idle (the 16^2 / 32^2 levels at the
// per-GPU batch of a batch-sharded run: M = 256, P = 256, N = 8 -> 32 workgroups): S slices of
// at least 4 K-chunks, S a power of two, items x S up to the resident workgroups (2 per CU).
static int gemm_splits(int N, int M, int P, int K1, int K2) {
  static const int slots = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return 2 * (n > 0 ? n : 256);
  }();
  if (!bpk_gemm_nchw_supported(N, M, P, K1, K2) || P % 4) return 1;
  const int64_t items = (int64_t)N * ((M + kBM - 1) / kBM) * (P / kBP);
  const int nch = (K1 + K2) / kKC;
  int S = 1;
  while (items * S * 2 <= slots && nch % (2 * S) == 0 && nch / (2 * S) >= 4) S *= 2;
  return S;
}

extern "C" int64_t bpk_gemm_nchw_splitk_bytes(int N, int M, int P, int K1, int K2) {
  const int S = gemm_splits(N, M, P, K1, K2);
  return S > 1 ? (int64_t)S * N * M * P * (int64_t)sizeof(float) : 0;
}

extern "C" int bpk_gemm_nchw_splitk_f32(const float* W, int ldw, const float* X1, int K1,
                                        const float* X2, int K2, const float* bias, float* Y,
                                        float* workspace, int N, int M, int P, void* stream) {
  const int S = gemm_splits(N, M, P, K1, K2);
  if (S <= 1) return bpk_gemm_nchw_f32(W, ldw, X1, K1, X2, K2, bias, Y, N, M, P, stream);
  BPK_REQUIRE(ldw >= K1 + K2 && ldw % 4 == 0, "gemm_nchw: bad weight row stride %d", ldw);
  BPK_REQUIRE(K2 == 0 || X2 != nullptr, "gemm_nchw: K2 > 0 needs X2");
  BPK_REQUIRE(workspace != nullptr, "gemm_nchw_splitk: workspace is NULL");
  GemmGeo g{N, M, P, K1, K2, ldw, (M + kBM - 1) / kBM, P / kBP, S};
  const int64_t blocks = (int64_t)N * g.tiles_m * g.tiles_p * S;
  BPK_REQUIRE(blocks < (1LL << 31), "gemm_nchw: grid too large");
  hipStream_t st = bpk::as_stream(stream);
  hipLaunchKernelGGL(gemm_nchw_kernel, dim3((unsigned)blocks), dim3(256), 0, st, W, X1,
                     K2 ? W + K1 : W, K2 ? X2 : X1, nullptr, workspace, g,
                     (blocks % 8 == 0) ? 1 : 0);
  BPK_LAUNCH_CHECK("gemm_nchw_splitk");
  const int64_t slab4 = (int64_t)N * M * P / 4;
  hipLaunchKernelGGL(gemm_splitk_reduce_kernel, dim3((unsigned)bpk::ceil_div(slab4, 256)),
                     dim3(256), 0, st, reinterpret_cast<const f4*>(workspace), S, slab4, bias,
                     reinterpret_cast<f4*>(Y), M, P / 4);
  BPK_LAUNCH_CHECK("gemm_nchw_splitk_reduce");
  return BPK_OK;
}

extern "C" int bpk_gemm_nchw_wgrad_supported(int N, int M, int K, int P) {
  return N > 0 && M > 0 && K > 0 && P > 0 && M % 16 == 0 && K % 16 == 0 && P % kKC == 0 &&
         (int64_t)N * (P / kKC) < (1LL << 31);
}

extern "C" int64_t bpk_gemm_nchw_wgrad_workspace_bytes(int N, int M, int K, int P) {
  if (!bpk_gemm_nchw_wgrad_supported(N, M, K, P)) return 0;
  const WgGeo g = wgrad_geo(N, M, K, P);
  if (g.splits == 1) return 0;
  return (int64_t)g.splits * ((int64_t)M * K + M) * (int64_t)sizeof(float);
}

extern "C" int bpk_gemm_nchw_wgrad_f32(const float* GY, const float* X, float* dW, float* db,
                                       void* workspace, int N, int M, int K, int P,
                                       void* stream) {
  BPK_REQUIRE(bpk_gemm_nchw_wgrad_supported(N, M, K, P),
              "gemm_nchw_wgrad: unsupported shape N=%d M=%d K=%d P=%d (need M %% 16, K %% 16, "
              "P %% 16 == 0)", N, M, K, P);
  const WgGeo g = wgrad_geo(N, M, K, P);
  BPK_REQUIRE(g.splits == 1 || workspace != nullptr, "gemm_nchw_wgrad: workspace required");
  const int64_t blocks = (int64_t)g.splits * g.tiles_m * g.tiles_k;
  BPK_REQUIRE(blocks < (1LL << 31), "gemm_nchw_wgrad: grid too large");
  float* part = g.splits == 1 ? dW : static_cast<float*>(workspace);
  float* part_b = db == nullptr ? nullptr
                  : g.splits == 1 ? db : part + (int64_t)g.splits * M * K;
  hipStream_t st = bpk::as_stream(stream);
  hipLaunchKernelGGL(gemm_nchw_wgrad_kernel, dim3((unsigned)blocks), dim3(256), 0, st, GY, X,
                     part, part_b, g, (blocks % 8 == 0) ? 1 : 0);
  BPK_LAUNCH_CHECK("gemm_nchw_wgrad");
  if (g.splits > 1) {
    const int64_t n4 = (int64_t)M * K / 4;
    hipLaunchKernelGGL(gemm_wgrad_reduce_kernel, dim3((unsigned)bpk::ceil_div(n4, 64)),
                       dim3(256), 0, st, reinterpret_cast<const f4*>(part),
                       reinterpret_cast<f4*>(dW), part_b, db, n4, M, g.splits);
    BPK_LAUNCH_CHECK("gemm_nchw_wgrad_reduce");
  }
  return BPK_OK;
}
