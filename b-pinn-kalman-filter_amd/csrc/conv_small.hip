// 3x3 / stride 1 / pad 1 fp32 convolution for a small channel count on one side, on the
// VALU (gfx950).
//
// NCSN++ / DDPM++ have per score evaluation one conv with Cin = 1 (conv_in: image -> nf
// channels, models/ncsnpp.py conv_in) and, with progressive = 'output_skip', one conv with
// Cout = 1 per resolution (the pyramid heads: GroupNorm -> SiLU -> conv3x3(C -> 1)).  Neither
// is GEMM-shaped (one GEMM dimension is 1): the work is 9 * Cin * Cout FMAs per pixel against
// one full read (Cout small) or one full write (Cin small) of a [B, C, H, W] tensor, so both
// are HBM-bound.  (MIOpen runs them as Winograd at ~1 ms each for B = 64 @ 128^2, 10-15x the
// byte time.)
//
//   * small_cout_kernel<COUT>: a workgroup owns a 16 x 64 output tile of one image; the
//     18 x 66 input patch of 8 channels at a time is staged in LDS (the next 8 prefetched into registers meanwhile) (GroupNorm affine + SiLU
//     applied on the way in when `pre` is given; the zero padding stays zero), every thread
//     accumulates a 1 x 4 pixel strip for all COUT outputs from a 3 x 6 register window;
//     weights are workgroup-uniform (scalar loads).
//   * small_cin_kernel<CIN>: the CIN x 18 x 66 patch is loaded once, each thread keeps its
//     3 x 6 x CIN window in registers and loops over the output channels, storing one
//     16-byte strip per channel (coalesced rows of the output planes).
// Backward-data of one form is the other form with the flipped, transposed filter
// (op/conv.py), so training and the DPS input gradient use the same two kernels.
#include "bpk_common.h"

#include <algorithm>

namespace {

constexpr int kTH = 16, kTW = 64;         // output tile
constexpr int kPH = kTH + 2, kPW = kTW + 2;  // 18 x 66 input patch
constexpr int kPWp = kPW + 1;             // padded LDS row

using f4 = __attribute__((ext_vector_type(4))) float;

__device__ inline float silu_f(float z) { return z * __builtin_amdgcn_rcpf(1.f + __expf(-z)); }

struct SmallGeo {
  int N, Cin, Cout, H, W, tiles_x, tiles_y;
};

// stage channels [c0, c0 + nc) of image n into s[c][row][col] (zero outside the image)
template <bool PRE>
__device__ inline void stage_patch(float* s, const float* __restrict__ xn,
                                   const float2* __restrict__ pre_n, int c0, int nc, int oy0,
                                   int ox0, const SmallGeo& g) {
  const int64_t plane = (int64_t)g.H * g.W;
  const int total = nc * kPH * kPW;
  for (int i = threadIdx.x; i < total; i += blockDim.x) {
    const int c = i / (kPH * kPW);
    const int r = i - c * (kPH * kPW);
    const int py = r / kPW, px = r - py * kPW;
    const int iy = oy0 - 1 + py, ix = ox0 - 1 + px;
    float v = 0.f;
    if (iy >= 0 && iy < g.H && ix >= 0 && ix < g.W) {
      v = xn[(int64_t)(c0 + c) * plane + (int64_t)iy * g.W + ix];
      if (PRE) {
        const float2 st = pre_n[c0 + c];
        v = silu_f(v * st.x + st.y);
      }
    }
    s[(c * kPH + py) * kPWp + px] = v;
  }
}

// small-Cout form: channels staged kCC at a time; each thread owns fixed patch positions
// (their global / LDS offsets computed once), the next chunk's values are loaded into
// registers while the current chunk is computed (one load latency per chunk hidden)
constexpr int kCC = 8;                                 // channels per chunk
constexpr int kPP = (kPH * kPW + 255) / 256;           // patch positions per thread (5)

template <int COUT, bool PRE>
__global__ __launch_bounds__(256) void small_cout_kernel(const float* __restrict__ x,
                                                         const float2* __restrict__ pre,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ bias,
                                                         float* __restrict__ y, SmallGeo g) {
  __shared__ float s_patch[kCC * kPH * kPWp];  // 38.6 KB
  const int tile = blockIdx.x;
  const int tx = tile % g.tiles_x;
  const int ty = (tile / g.tiles_x) % g.tiles_y;
  const int n = tile / (g.tiles_x * g.tiles_y);
  const int oy0 = ty * kTH, ox0 = tx * kTW;
  const int lr = threadIdx.x >> 4, lc = (threadIdx.x & 15) * 4;  // strip (lr, lc..lc+3)
  const int64_t plane = (int64_t)g.H * g.W;
  const float* xn = x + (int64_t)n * g.Cin * plane;
  const float2* pre_n = PRE ? pre + (int64_t)n * g.Cin : nullptr;

  // this thread's patch positions: global offset within a plane (-1: padding / unused) and
  // LDS offset within a channel slab
  int goff[kPP], loff[kPP];
#pragma unroll
  for (int k = 0; k < kPP; ++k) {
    const int p = threadIdx.x + 256 * k;
    const int py = p / kPW, px = p - (p / kPW) * kPW;
    const int iy = oy0 - 1 + py, ix = ox0 - 1 + px;
    const bool in = p < kPH * kPW && iy >= 0 && iy < g.H && ix >= 0 && ix < g.W;
    goff[k] = in ? iy * g.W + ix : -1;
    loff[k] = p < kPH * kPW ? py * kPWp + px : -1;
  }
  float pf[kCC][kPP];
  auto load = [&](int c0) {
#pragma unroll
    for (int c = 0; c < kCC; ++c)
#pragma unroll
      for (int k = 0; k < kPP; ++k)
        pf[c][k] = (goff[k] >= 0 && c0 + c < g.Cin) ? xn[(int64_t)(c0 + c) * plane + goff[k]]
                                                    : 0.f;
  };
  auto store = [&](int c0) {
#pragma unroll
    for (int c = 0; c < kCC; ++c) {
      float2 st = make_float2(1.f, 0.f);
      if (PRE && c0 + c < g.Cin) st = pre_n[c0 + c];
#pragma unroll
      for (int k = 0; k < kPP; ++k) {
        if (loff[k] < 0) continue;
        float v = pf[c][k];
        if (PRE && goff[k] >= 0) v = silu_f(v * st.x + st.y);  // padding stays zero
        s_patch[c * kPH * kPWp + loff[k]] = v;
      }
    }
  };

  float acc[COUT][4];
#pragma unroll
  for (int co = 0; co < COUT; ++co)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[co][j] = 0.f;

  load(0);
  for (int c0 = 0; c0 < g.Cin; c0 += kCC) {
    const int nc = min(kCC, g.Cin - c0);
    __syncthreads();
    store(c0);
    __syncthreads();
    if (c0 + kCC < g.Cin) load(c0 + kCC);
    for (int c = 0; c < nc; ++c) {
      float win[3][6];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int j = 0; j < 6; ++j) win[r][j] = s_patch[(c * kPH + lr + r) * kPWp + lc + j];
#pragma unroll
      for (int co = 0; co < COUT; ++co) {
        const float* wk = w + ((int64_t)co * g.Cin + c0 + c) * 9;  // uniform
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
          for (int s = 0; s < 3; ++s) {
            const float wv = wk[r * 3 + s];
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[co][j] = fmaf(win[r][j + s], wv, acc[co][j]);
          }
      }
    }
  }
  const int oy = oy0 + lr, ox = ox0 + lc;
  if (oy < g.H && ox < g.W) {  // W % 4 == 0: a strip is all in or all out
#pragma unroll
    for (int co = 0; co < COUT; ++co) {
      const float b = bias ? bias[co] : 0.f;
      *reinterpret_cast<f4*>(&y[((int64_t)n * g.Cout + co) * plane + (int64_t)oy * g.W + ox]) =
          f4{acc[co][0] + b, acc[co][1] + b, acc[co][2] + b, acc[co][3] + b};
    }
  }
}

template <int CIN>
__global__ __launch_bounds__(256) void small_cin_kernel(const float* __restrict__ x,
                                                        const float* __restrict__ w,
                                                        const float* __restrict__ bias,
                                                        float* __restrict__ y, SmallGeo g) {
  __shared__ float s_patch[CIN * kPH * kPWp];
  const int tile = blockIdx.x;
  const int tx = tile % g.tiles_x;
  const int ty = (tile / g.tiles_x) % g.tiles_y;
  const int n = tile / (g.tiles_x * g.tiles_y);
  const int oy0 = ty * kTH, ox0 = tx * kTW;
  const int lr = threadIdx.x >> 4, lc = (threadIdx.x & 15) * 4;
  const int64_t plane = (int64_t)g.H * g.W;
  stage_patch<false>(s_patch, x + (int64_t)n * CIN * plane, nullptr, 0, CIN, oy0, ox0, g);
  __syncthreads();
  float win[CIN][3][6];
#pragma unroll
  for (int c = 0; c < CIN; ++c)
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int j = 0; j < 6; ++j) win[c][r][j] = s_patch[(c * kPH + lr + r) * kPWp + lc + j];
  const int oy = oy0 + lr, ox = ox0 + lc;
  if (oy >= g.H || ox >= g.W) return;  // no barrier below
  float* yo = y + (int64_t)n * g.Cout * plane + (int64_t)oy * g.W + ox;
  for (int co = 0; co < g.Cout; ++co) {
    const float b = bias ? bias[co] : 0.f;
    float a[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < CIN; ++c) {
      const float* wk = w + ((int64_t)co * CIN + c) * 9;  // uniform
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const float wv = wk[r * 3 + s];
#pragma unroll
          for (int j = 0; j < 4; ++j) a[j] = fmaf(win[c][r][j + s], wv, a[j]);
        }
    }
    *reinterpret_cast<f4*>(&yo[(int64_t)co * plane]) = f4{a[0] + b, a[1] + b, a[2] + b, a[3] + b};
  }
}

// Weight gradient of a conv with few output channels (Cout <= 4; K x K, stride 1, pad K / 2,
// K = 1 or 3):  dw[co][c][r][s] = sum_{n, p} gy[n][co][p] x[n][c][p + (r, s) - K / 2],
// db[co] = sum gy[n][co].  The network output convs (NCSN++ conv_out 128 -> 1 at 128^2, the
// PINN heads into 1-4 channels) have one GEMM dimension of 1-4 against a K = pixels reduction,
// which the implicit-GEMM kernel runs on mostly idle 64-row MFMA tiles while gathering every
// x element 9 times (2.3 ms for B = 64, 128 -> 1 at 128^2).  Here it is a single streaming
// pass over x (HBM-bound): one workgroup per (channel c, image n) walks the image in row bands,
// stages each band's rows with their halo in LDS, and every thread accumulates the COUT x K^2
// products of its pixels in registers (gy read coalesced, L2-resident across the channels);
// the workgroup's sums (wave butterflies, then the waves in order) go to a per-image partial,
// and small_cout_wgrad_reduce_kernel adds the images in order: deterministic.
template <int COUT, int K>
__global__ __launch_bounds__(256) void small_cout_wgrad_kernel(const float* __restrict__ x,
                                                               const float* __restrict__ gy,
                                                               float* __restrict__ part,
                                                               float* __restrict__ partb, int Cin,
                                                               int H, int W, int RB) {
  extern __shared__ float s_x[];  // (RB + K - 1) x (W + K - 1)
  constexpr int KK = K * K, P = K / 2;
  const int tid = threadIdx.x;
  const int c = blockIdx.x, n = blockIdx.y;
  const int64_t plane = (int64_t)H * W;
  const float* xp = x + ((int64_t)n * Cin + c) * plane;
  const float* gp = gy + (int64_t)n * COUT * plane;
  const int Wp = W + K - 1;
  float acc[COUT][KK], accb[COUT];
#pragma unroll
  for (int co = 0; co < COUT; ++co) {
    accb[co] = 0.f;
#pragma unroll
    for (int k = 0; k < KK; ++k) acc[co][k] = 0.f;
  }
  // this thread's pixels in a band: q = tid + 256 j -> (row, col), stepped without division
  const int dr = 256 / W, dc = 256 - dr * W;
  const int r_first = tid / W, c_first = tid - r_first * W;
  for (int y0 = 0; y0 < H; y0 += RB) {
    const int rows = min(RB, H - y0);
    __syncthreads();  // the previous band's LDS reads are done
    for (int i = tid; i < (rows + K - 1) * Wp; i += 256) {
      const int rr = i / Wp, cc = i - rr * Wp;
      const int iy = y0 - P + rr, ix = cc - P;
      s_x[i] = (iy >= 0 && iy < H && ix >= 0 && ix < W) ? xp[(int64_t)iy * W + ix] : 0.f;
    }
    __syncthreads();
    int r = r_first, col = c_first;
    while (r < rows) {
      float g[COUT];
#pragma unroll
      for (int co = 0; co < COUT; ++co) g[co] = gp[co * plane + (int64_t)(y0 + r) * W + col];
#pragma unroll
      for (int a = 0; a < K; ++a)
#pragma unroll
        for (int b = 0; b < K; ++b) {
          const float xv = s_x[(r + a) * Wp + col + b];
#pragma unroll
          for (int co = 0; co < COUT; ++co) acc[co][a * K + b] = fmaf(g[co], xv, acc[co][a * K + b]);
        }
#pragma unroll
      for (int co = 0; co < COUT; ++co) accb[co] += g[co];
      r += dr;
      col += dc;
      if (col >= W) {
        col -= W;
        ++r;
      }
    }
  }
  // workgroup sums: butterflies within each wave, then the four waves in order
  __shared__ float red[4][COUT * (KK + 1)];
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int co = 0; co < COUT; ++co)
#pragma unroll
    for (int k = 0; k <= KK; ++k) {
      float v = k < KK ? acc[co][k] : accb[co];
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
      if (lane == 0) red[wave][co * (KK + 1) + k] = v;
    }
  __syncthreads();
  if (tid < COUT * (KK + 1)) {
    const float v = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
    const int co = tid / (KK + 1), k = tid - co * (KK + 1);
    if (k < KK)
      part[(((int64_t)n * COUT + co) * Cin + c) * KK + k] = v;
    else if (c == 0 && partb)
      partb[n * COUT + co] = v;
  }
}

// dw = sum over images of the partials, in image order (db likewise)
__global__ __launch_bounds__(256) void small_cout_wgrad_reduce_kernel(
    const float* __restrict__ part, const float* __restrict__ partb, float* __restrict__ dw,
    float* __restrict__ db, int N, int Cout, int per_co) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int total = Cout * per_co;
  if (i < total) {
    const int co = i / per_co, rest = i - co * per_co;
    float v = 0.f;
#pragma unroll 8
    for (int n = 0; n < N; ++n) v += part[((int64_t)n * Cout + co) * per_co + rest];
    dw[i] = v;
  } else if (db && i < total + Cout) {
    const int co = i - total;
    float v = 0.f;
    for (int n = 0; n < N; ++n) v += partb[n * Cout + co];
    db[co] = v;
  }
}

int wgrad_rows_per_band(int H, int W) { return std::max(1, std::min(H, 1024 / W)); }

}  // namespace

extern "C" int bpk_conv2d_wgrad_small_cout_supported(int N, int Cin, int Cout, int H, int W,
                                                     int K) {
  return N > 0 && Cin > 0 && Cout >= 1 && Cout <= 4 && H > 0 && W > 0 && (K == 1 || K == 3) &&
         (int64_t)N * Cin < (1LL << 31) && (int64_t)N * std::max(Cin, Cout) * H * W < (1LL << 40) &&
         (int64_t)(wgrad_rows_per_band(H, W) + K - 1) * (W + K - 1) * 4 <= 64 * 1024;
}

extern "C" int64_t bpk_conv2d_wgrad_small_cout_workspace_bytes(int N, int Cin, int Cout, int K) {
  return ((int64_t)N * Cout * Cin * K * K + (int64_t)N * Cout) * 4;
}

extern "C" int bpk_conv2d_wgrad_small_cout_f32(const float* x, const float* gy, float* dw,
                                               float* db, void* ws, int N, int Cin, int Cout,
                                               int H, int W, int K, void* stream) {
  BPK_REQUIRE(bpk_conv2d_wgrad_small_cout_supported(N, Cin, Cout, H, W, K),
              "conv2d_wgrad_small_cout: unsupported shape N=%d Cin=%d Cout=%d %dx%d K=%d", N, Cin,
              Cout, H, W, K);
  BPK_REQUIRE(x && gy && dw && ws, "conv2d_wgrad_small_cout: null pointer");
  float* part = static_cast<float*>(ws);
  float* partb = db ? part + (int64_t)N * Cout * Cin * K * K : nullptr;
  const int RB = wgrad_rows_per_band(H, W);
  const size_t lds = (size_t)(RB + K - 1) * (W + K - 1) * 4;
  hipStream_t st = bpk::as_stream(stream);
  const dim3 grid((unsigned)Cin, (unsigned)N);
#define WG(C_, K_)                                                                                hipLaunchKernelGGL((small_cout_wgrad_kernel<C_, K_>), grid, dim3(256), lds, st, x, gy, part,                      partb, Cin, H, W, RB)
#define WGK(C_)   do {              if (K == 3)       WG(C_, 3);     else              WG(C_, 1);   } while (0)
  switch (Cout) {
    case 1: WGK(1); break;
    case 2: WGK(2); break;
    case 3: WGK(3); break;
    default: WGK(4); break;
  }
#undef WGK
#undef WG
  BPK_LAUNCH_CHECK("conv2d_wgrad_small_cout");
  const int per_co = Cin * K * K;
  const int total = Cout * per_co + (db ? Cout : 0);
  hipLaunchKernelGGL(small_cout_wgrad_reduce_kernel, dim3((unsigned)bpk::ceil_div(total, 256)),
                     dim3(256), 0, st, part, partb, dw, db, N, Cout, per_co);
  BPK_LAUNCH_CHECK("conv2d_wgrad_small_cout_reduce");
  return BPK_OK;
}

extern "C" int bpk_conv3x3_small_supported(int N, int Cin, int Cout, int H, int W) {
  return N > 0 && Cin > 0 && Cout > 0 && H > 0 && W > 0 && W % 4 == 0 &&
         (Cout <= 4 || Cin <= 4);
}

extern "C" int bpk_conv3x3_small_f32(const float* x, const float* pre, const float* weight,
                                     const float* bias, float* y, int N, int Cin, int Cout, int H,
                                     int W, void* stream) {
  BPK_REQUIRE(bpk_conv3x3_small_supported(N, Cin, Cout, H, W),
              "conv3x3_small: unsupported shape N=%d Cin=%d Cout=%d H=%d W=%d (need W %% 4 == 0 "
              "and Cin <= 4 or Cout <= 4)", N, Cin, Cout, H, W);
  SmallGeo g{N, Cin, Cout, H, W, (int)bpk::ceil_div(W, kTW), (int)bpk::ceil_div(H, kTH)};
  const int64_t blocks = (int64_t)N * g.tiles_x * g.tiles_y;
  BPK_REQUIRE(blocks < (1LL << 31), "conv3x3_small: grid too large");
  hipStream_t st = bpk::as_stream(stream);
  const float2* pre2 = reinterpret_cast<const float2*>(pre);
  const dim3 grid((unsigned)blocks), block(256);
  if (Cout <= 4 && (Cout <= Cin || pre)) {
#define SC(C_)                                                                           \
  do {                                                                                   \
    if (pre)                                                                             \
      hipLaunchKernelGGL((small_cout_kernel<C_, true>), grid, block, 0, st, x, pre2, weight, \
                         bias, y, g);                                                    \
    else                                                                                 \
      hipLaunchKernelGGL((small_cout_kernel<C_, false>), grid, block, 0, st, x, pre2,    \
                         weight, bias, y, g);                                            \
  } while (0)
    switch (Cout) {
      case 1: SC(1); break;
      case 2: SC(2); break;
      case 3: SC(3); break;
      default: SC(4); break;
    }
#undef SC
  } else {
    BPK_REQUIRE(pre == nullptr, "conv3x3_small: the GroupNorm prologue needs Cout <= 4");
    switch (Cin) {
      case 1: hipLaunchKernelGGL((small_cin_kernel<1>), grid, block, 0, st, x, weight, bias, y, g); break;
      case 2: hipLaunchKernelGGL((small_cin_kernel<2>), grid, block, 0, st, x, weight, bias, y, g); break;
      case 3: hipLaunchKernelGGL((small_cin_kernel<3>), grid, block, 0, st, x, weight, bias, y, g); break;
      default: hipLaunchKernelGGL((small_cin_kernel<4>), grid, block, 0, st, x, weight, bias, y, g); break;
    }
  }
  BPK_LAUNCH_CHECK("conv3x3_small");
  return BPK_OK;
}
