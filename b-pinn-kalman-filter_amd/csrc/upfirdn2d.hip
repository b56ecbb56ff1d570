// upfirdn2d for gfx950: zero-insert upsample -> pad/crop -> FIR (true convolution)
// -> decimate, on [major, H, W, minor] planes.
//
// Semantics follow the reference's CPU oracle `upfirdn2d_native`
// (op/upfirdn2d.py:159-200) and its CUDA op (op/upfirdn2d_kernel.cu:50-207):
//   out[p, oy, ox, m] = sum_{i<kh, j<kw} U[oy*dy + i - py0, ox*dx + j - px0, m]
//                                         * k[kh-1-i, kw-1-j]
//   U[a, b] = x[a/uy, b/ux] when a % uy == 0, b % ux == 0 and in range, else 0.
//
// Design (MI355X-first, HBM-bound op):
//  * minor == 1 (NCHW planes, every NCSN++ call site) goes to an LDS-tiled
//    kernel: a workgroup owns a TH x TW output tile of one plane, stages the
//    input window (with the zero halo) into LDS with 16-byte row loads from an
//    aligned origin, and each of the 256 threads produces 4-wide output strips
//    written with 16-byte stores.  Tile width adapts to the plane width
//    (16/32/64) so 16x16 and 32x32 planes do not idle lanes.  The taps are read
//    once into registers (flipped, zero-extended to KxK).
//  * anything else (minor > 1, factors > 2, kernels > 4x4) uses a grid-stride
//    direct kernel; L1/L2 absorb the tap overlap.
#include "bpk_common.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace {

// LDS-tiled kernel.  A workgroup produces a TH x TW output tile of one plane: it stages the
// input window (zero halo included) into LDS -- 16-byte loads from an aligned origin when
// VEC -- then each thread produces 4-wide output strips (one 16-byte store each when VEC).
template <typename T, int UP, int DOWN, int K, int TH, int TW, bool VEC_>
__global__ __launch_bounds__(256) void upfirdn2d_tiled(const T* __restrict__ x,
                                                        const T* __restrict__ kern,
                                                        T* __restrict__ out, int in_h, int in_w,
                                                        int kh, int kw, int px0, int py0,
                                                        int out_h, int out_w, int tiles_x,
                                                        int tiles_y) {
  constexpr bool VEC = VEC_ && std::is_same<T, float>::value;
  constexpr int TIH = ((TH - 1) * DOWN + K - 1) / UP + 2;
  constexpr int TIW_RAW = ((TW - 1) * DOWN + K - 1) / UP + 2;
  constexpr int TIW = (TIW_RAW + 3 + 3) / 4 * 4;  // + room for the 0..3 alignment shift
  constexpr int LD = TIW + 4;                     // row pitch (16-byte multiple, skews banks)
  constexpr int QW = TIW / 4;
  __shared__ __attribute__((aligned(16))) T sx[TIH * LD];

  const int tid = threadIdx.x;
  int bid = blockIdx.x;
  const int tx_i = bid % tiles_x;
  bid /= tiles_x;
  const int ty_i = bid % tiles_y;
  const int plane = bid / tiles_y;

  const int oy0 = ty_i * TH;
  const int ox0 = tx_i * TW;
  const int iy0 = bpk::floordiv(oy0 * DOWN - py0, UP);
  const int ix0 = bpk::floordiv(ox0 * DOWN - px0, UP);
  const int ixa = VEC ? bpk::floordiv(ix0, 4) * 4 : ix0;  // aligned load origin
  const int shift = ix0 - ixa;

  const T* xp = x + (int64_t)plane * in_h * in_w;
  for (int e = tid; e < TIH * QW; e += 256) {
    const int r = e / QW;
    const int q = e - r * QW;
    const int iy = iy0 + r;
    const int ix = ixa + 4 * q;
    T v[4];
    const bool row_ok = iy >= 0 && iy < in_h;
    bool loaded = false;
    if constexpr (VEC) {
      if (row_ok && ix >= 0 && ix + 3 < in_w) {
        const float4 f = *reinterpret_cast<const float4*>(xp + (int64_t)iy * in_w + ix);
        v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
        loaded = true;
      }
    }
    if (!loaded) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        v[j] = (row_ok && ix + j >= 0 && ix + j < in_w) ? xp[(int64_t)iy * in_w + ix + j] : T(0);
    }
    if constexpr (VEC) {
      *reinterpret_cast<float4*>(&sx[r * LD + 4 * q]) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) sx[r * LD + 4 * q + j] = v[j];
    }
  }

  // flipped taps, zero-extended to K x K
  T w[K][K];
#pragma unroll
  for (int i = 0; i < K; ++i)
#pragma unroll
    for (int j = 0; j < K; ++j)
      w[i][j] = (i < kh && j < kw) ? kern[(kh - 1 - i) * kw + (kw - 1 - j)] : T(0);

  __syncthreads();

  constexpr int SPR = TW / 4;           // strips per output row
  constexpr int ROWS_PER_PASS = 256 / SPR;
  const int sx0 = (tid % SPR) * 4;
#pragma unroll
  for (int pass = 0; pass < TH / ROWS_PER_PASS; ++pass) {
    const int ty = pass * ROWS_PER_PASS + tid / SPR;
    const int oy = oy0 + ty;
    T acc[4] = {T(0), T(0), T(0), T(0)};
#pragma unroll
    for (int i = 0; i < K; ++i) {
      const int a = oy * DOWN + i - py0;
      const int r = bpk::floordiv(a, UP) - iy0;
      const bool row_ok = (UP == 1) || (bpk::floormod(a, UP) == 0);
      const T* srow = sx + r * LD + shift;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int ox = ox0 + sx0 + s;
#pragma unroll
        for (int j = 0; j < K; ++j) {
          const int b = ox * DOWN + j - px0;
          const int c = bpk::floordiv(b, UP) - ix0;
          const bool ok = row_ok && ((UP == 1) || (bpk::floormod(b, UP) == 0));
          acc[s] += srow[c] * (ok ? w[i][j] : T(0));
        }
      }
    }
    const int ox = ox0 + sx0;
    if (oy < out_h) {
      T* op = out + ((int64_t)plane * out_h + oy) * out_w + ox;
      bool stored = false;
      if constexpr (VEC) {
        if (ox + 3 < out_w) {
          *reinterpret_cast<float4*>(op) = make_float4(acc[0], acc[1], acc[2], acc[3]);
          stored = true;
        }
      }
      if (!stored) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
          if (ox + s < out_w) op[s] = acc[s];
      }
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void upfirdn2d_direct(
    const T* __restrict__ x, const T* __restrict__ kern, T* __restrict__ out, int in_h, int in_w,
    int minor, int kh, int kw, int ux, int uy, int dx, int dy, int px0, int py0, int out_h,
    int out_w, int64_t total) {
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int64_t t = idx;
    const int m = (int)(t % minor);
    t /= minor;
    const int ox = (int)(t % out_w);
    t /= out_w;
    const int oy = (int)(t % out_h);
    const int64_t p = t / out_h;
    const T* xp = x + p * in_h * in_w * minor + m;
    T acc = T(0);
    for (int i = 0; i < kh; ++i) {
      const int a = oy * dy + i - py0;
      if (a < 0 || (a % uy) != 0) continue;
      const int iy = a / uy;
      if (iy >= in_h) continue;
      for (int j = 0; j < kw; ++j) {
        const int b = ox * dx + j - px0;
        if (b < 0 || (b % ux) != 0) continue;
        const int ix = b / ux;
        if (ix >= in_w) continue;
        acc += xp[((int64_t)iy * in_w + ix) * minor] * kern[(kh - 1 - i) * kw + (kw - 1 - j)];
      }
    }
    out[idx] = acc;
  }
}

template <typename T, int UP, int DOWN, int K, int TH, int TW>
int launch_tiled(const T* x, const T* k, T* out, int major, int in_h, int in_w, int kh, int kw,
                 int px0, int py0, int out_h, int out_w, hipStream_t st) {
  const int tiles_x = (int)bpk::ceil_div(out_w, TW);
  const int tiles_y = (int)bpk::ceil_div(out_h, TH);
  const int64_t blocks = (int64_t)major * tiles_x * tiles_y;
  if (blocks <= 0) return BPK_OK;
  BPK_REQUIRE(blocks < (int64_t)INT32_MAX, "upfirdn2d: grid too large (%lld blocks)",
              (long long)blocks);
  const bool vec = std::is_same<T, float>::value && in_w % 4 == 0 && out_w % 4 == 0 &&
                   ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out)) & 15) == 0;
  if (vec)
    hipLaunchKernelGGL((upfirdn2d_tiled<T, UP, DOWN, K, TH, TW, true>), dim3((unsigned)blocks),
                       dim3(256), 0, st, x, k, out, in_h, in_w, kh, kw, px0, py0, out_h, out_w,
                       tiles_x, tiles_y);
  else
    hipLaunchKernelGGL((upfirdn2d_tiled<T, UP, DOWN, K, TH, TW, false>), dim3((unsigned)blocks),
                       dim3(256), 0, st, x, k, out, in_h, in_w, kh, kw, px0, py0, out_h, out_w,
                       tiles_x, tiles_y);
  BPK_LAUNCH_CHECK("upfirdn2d_tiled");
  return BPK_OK;
}

// tile shapes (TH x TW outputs, 4..8 per thread) by plane width
template <typename T, int UP, int DOWN>
int launch_tiled_w(const T* x, const T* k, T* out, int major, int in_h, int in_w, int kh, int kw,
                   int px0, int py0, int out_h, int out_w, hipStream_t st) {
  if (out_w <= 16)
    return launch_tiled<T, UP, DOWN, 4, 64, 16>(x, k, out, major, in_h, in_w, kh, kw, px0, py0,
                                                out_h, out_w, st);
  if (out_w <= 32)
    return launch_tiled<T, UP, DOWN, 4, 32, 32>(x, k, out, major, in_h, in_w, kh, kw, px0, py0,
                                                out_h, out_w, st);
  return launch_tiled<T, UP, DOWN, 4, 32, 64>(x, k, out, major, in_h, in_w, kh, kw, px0, py0,
                                              out_h, out_w, st);
}

// Register-streaming kernel for the FIR modes NCSN++ uses (and their adjoints):
// (up, down) in {(1,2), (1,1), (2,1)}, taps <= 4x4, pad0 = P0 on both axes.  A lane segment of
// SEGW lanes (SEGW = 64 / 32 / 16 / 8, matched to the plane width so no lane idles) owns a
// strip of SEGW*NOC output columns x R output rows of one plane.  Per input row each lane
// loads LV consecutive floats (8-byte loads when LV = 2) and takes its +-1 neighbours'
// values with cross-lane shuffles inside the segment, so there is no LDS staging and no
// workgroup barrier; short strips (R = 4..8) keep many waves in flight, which is what an
// HBM-bound stencil needs on MI355X.  All tap bookkeeping is compile-time: input row t of
// the strip feeds output row r through vertical tap i = t*UP - r*DOWN, and output column oc
// of a lane reads relative input column q = (oc*DOWN + j - P0) / UP.
// TAIL: the plane is one strip wide plus one column (odd widths 2^k + 1: the FIR pad(2, 2)
// of conv_downsample_2d, 64 -> 65): the segment's last lane also produces the plane's last
// column from the values it already holds, so a 65-wide row takes a 32-lane segment
// instead of a half-idle 64-lane one.
#ifndef UPFIRDN_WPE
#define UPFIRDN_WPE 1
#endif
template <int UP, int DOWN, int P0, int R, int SEGW, int NOCD = 0, bool TAIL = false>
__global__ __launch_bounds__(256, UPFIRDN_WPE) void upfirdn2d_stream(const float* __restrict__ x,
                                                         const float* __restrict__ kern,
                                                         float* __restrict__ out, int in_h,
                                                         int in_w, int kh, int kw, int out_h,
                                                         int out_w, int strips_x, int strips_y,
                                                         int64_t n_strips) {
  // output columns per lane: NOCD, or the default 1 (down2) / 2
  constexpr int NOC = NOCD > 0 ? NOCD : ((UP == 1 && DOWN == 2) ? 1 : 2);
  constexpr int LV = NOC * DOWN / UP;                      // input columns loaded per lane
  constexpr int NIR = ((R - 1) * DOWN + 3) / UP + 1;    // input rows feeding R output rows
  constexpr int SEGS = 64 / SEGW;
  const int lane = threadIdx.x & 63;
  const int sl = lane % SEGW;  // lane within its segment
  const int64_t strip = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * SEGS + lane / SEGW;
  const bool active = strip < n_strips;
  const int64_t sidx = active ? strip : 0;
  const int sxi = (int)(sidx % strips_x);
  const int syi = (int)((sidx / strips_x) % strips_y);
  const int64_t plane = sidx / ((int64_t)strips_x * strips_y);
  const int ox0 = sxi * SEGW * NOC;
  const int oyb = syi * R;  // R even -> (oyb*DOWN - P0) divisible by UP when UP = 2, P0 = 2
  const int ixbase = ox0 * DOWN / UP;
  const int iy_lo = bpk::floordiv(oyb * DOWN - P0, UP);
  const int mycol = ixbase + LV * sl;

  float w[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w[i][j] = (i < kh && j < kw) ? kern[(kh - 1 - i) * kw + (kw - 1 - j)] : 0.f;

  constexpr int NOCT = NOC + (TAIL ? 1 : 0);  // columns computed (the tail one on the last lane)
  float acc[R][NOCT];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int oc = 0; oc < NOCT; ++oc) acc[r][oc] = 0.f;

  const float* xp = x + plane * in_h * in_w;
#pragma unroll
  for (int t = 0; t < NIR; ++t) {
    const int iy = iy_lo + t;
    const bool row_ok = active && iy >= 0 && iy < in_h;
    const float* row = xp + (int64_t)iy * in_w;
    float own[LV], left[LV], right[LV];
    if constexpr (LV == 4) {  // 16-byte row loads (in_w % 4 == 0, 16-byte aligned x)
      if (row_ok && mycol + 3 < in_w) {
        const float4 v = *reinterpret_cast<const float4*>(row + mycol);
        own[0] = v.x;
        own[1] = v.y;
        own[2] = v.z;
        own[3] = v.w;
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) own[c] = (row_ok && mycol + c < in_w) ? row[mycol + c] : 0.f;
      }
    } else if constexpr (LV == 2) {
      if (row_ok && mycol + 1 < in_w) {
        const float2 v = *reinterpret_cast<const float2*>(row + mycol);
        own[0] = v.x;
        own[1] = v.y;
      } else {
        own[0] = (row_ok && mycol < in_w) ? row[mycol] : 0.f;
        own[1] = 0.f;
      }
    } else {
      own[0] = (row_ok && mycol < in_w) ? row[mycol] : 0.f;
    }
#pragma unroll
    for (int c = 0; c < LV; ++c) {
      left[c] = __shfl_up(own[c], 1, SEGW);
      right[c] = __shfl_down(own[c], 1, SEGW);
    }
    if (sl == 0) {
#pragma unroll
      for (int c = 0; c < LV; ++c) {
        const int col = mycol - LV + c;
        left[c] = (row_ok && col >= 0 && col < in_w) ? row[col] : 0.f;
      }
    }
    if (sl == SEGW - 1) {
#pragma unroll
      for (int c = 0; c < LV; ++c) {
        const int col = mycol + LV + c;
        right[c] = (row_ok && col < in_w) ? row[col] : 0.f;
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int i = t * UP - r * DOWN;
      if (i < 0 || i >= 4) continue;
#pragma unroll
      for (int oc = 0; oc < NOCT; ++oc) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int u = oc * DOWN + j - P0;
          if (bpk::floormod(u, UP) != 0) continue;
          const int q = bpk::floordiv(u, UP);
          const int lo = bpk::floordiv(q, LV);
          const int comp = bpk::floormod(q, LV);
          const float v = lo < 0 ? left[comp] : (lo == 0 ? own[comp] : right[comp]);
          acc[r][oc] += v * w[i][j];
        }
      }
    }
  }
  if (!active) return;
  const int oxl = ox0 + NOC * sl;
  float* op = out + plane * out_h * out_w;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int oy = oyb + r;
    float* orow = op + (int64_t)oy * out_w;
    if (oy < out_h) {
      if constexpr (NOC == 4 && TAIL) {  // odd row pitch: the widest store the address allows
        const int64_t e0 = (plane * out_h + oy) * (int64_t)out_w + oxl;  // element index
        if ((e0 & 3) == 0) {
          *reinterpret_cast<float4*>(orow + oxl) =
              make_float4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
        } else if ((e0 & 1) == 0) {
          *reinterpret_cast<float2*>(orow + oxl) = make_float2(acc[r][0], acc[r][1]);
          *reinterpret_cast<float2*>(orow + oxl + 2) = make_float2(acc[r][2], acc[r][3]);
        } else {
#pragma unroll
          for (int oc = 0; oc < 4; ++oc) orow[oxl + oc] = acc[r][oc];
        }
      } else if constexpr (NOC == 4) {  // out_w % 4 == 0 (host check): 16-byte aligned quads
        if (oxl + 3 < out_w) {
          *reinterpret_cast<float4*>(orow + oxl) =
              make_float4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
        } else {
#pragma unroll
          for (int oc = 0; oc < 4; ++oc)
            if (oxl + oc < out_w) orow[oxl + oc] = acc[r][oc];
        }
      } else if constexpr (NOC == 2) {
        // 8-byte store when the pair is aligned (odd out_w makes every other row odd)
        if (oxl + 1 < out_w && (((int64_t)oy * out_w + oxl) & 1) == 0 && (out_h * out_w) % 2 == 0) {
          *reinterpret_cast<float2*>(orow + oxl) = make_float2(acc[r][0], acc[r][1]);
        } else {
          if (oxl < out_w) orow[oxl] = acc[r][0];
          if (oxl + 1 < out_w) orow[oxl + 1] = acc[r][1];
        }
      } else {
        if (oxl < out_w) orow[oxl] = acc[r][0];
      }
      if constexpr (TAIL) {
        if (sl == SEGW - 1) orow[out_w - 1] = acc[r][NOC];
      }
    }
  }
}

template <int UP, int DOWN, int P0, int R, int SEGW, int NOCD, bool TAIL = false>
int launch_stream_seg(const float* x, const float* k, float* out, int major, int in_h, int in_w,
                      int kh, int kw, int out_h, int out_w, hipStream_t st) {
  constexpr int NOC = NOCD > 0 ? NOCD : ((UP == 1 && DOWN == 2) ? 1 : 2);
  const int strips_x = TAIL ? 1 : (int)bpk::ceil_div(out_w, SEGW * NOC);
  const int strips_y = (int)bpk::ceil_div(out_h, R);
  const int64_t n = (int64_t)major * strips_x * strips_y;
  if (n <= 0) return BPK_OK;
  const int64_t blocks = bpk::ceil_div(n, 4 * (64 / SEGW));
  BPK_REQUIRE(blocks < (int64_t)INT32_MAX, "upfirdn2d: grid too large");
  hipLaunchKernelGGL((upfirdn2d_stream<UP, DOWN, P0, R, SEGW, NOCD, TAIL>), dim3((unsigned)blocks), dim3(256),
                     0, st, x, k, out, in_h, in_w, kh, kw, out_h, out_w, strips_x, strips_y, n);
  BPK_LAUNCH_CHECK("upfirdn2d_stream");
  return BPK_OK;
}

// segment width = lanes needed for one output row of the plane (power of two, 8..64)
template <int UP, int DOWN, int P0, int R, int NOCD = 0>
int launch_stream(const float* x, const float* k, float* out, int major, int in_h, int in_w,
                  int kh, int kw, int out_h, int out_w, hipStream_t st) {
  constexpr int NOC = NOCD > 0 ? NOCD : ((UP == 1 && DOWN == 2) ? 1 : 2);
  const int lanes = (int)bpk::ceil_div(out_w, NOC);
  if (lanes <= 8)
    return launch_stream_seg<UP, DOWN, P0, R, 8, NOCD>(x, k, out, major, in_h, in_w, kh, kw, out_h, out_w, st);
  if (lanes <= 16)
    return launch_stream_seg<UP, DOWN, P0, R, 16, NOCD>(x, k, out, major, in_h, in_w, kh, kw, out_h, out_w, st);
  if (lanes <= 32)
    return launch_stream_seg<UP, DOWN, P0, R, 32, NOCD>(x, k, out, major, in_h, in_w, kh, kw, out_h, out_w, st);
  return launch_stream_seg<UP, DOWN, P0, R, 64, NOCD>(x, k, out, major, in_h, in_w, kh, kw, out_h, out_w, st);
}

// Row-rolling kernel for the UP = 1 modes (down2 and the 1:1 FIR), taps <= 4x4: a lane segment
// owns a column strip of SEGW*NOC output columns (as upfirdn2d_stream) but walks DOWN the plane
// over `rows` output rows, one input row at a time, keeping only the output rows in flight
// (2 accumulators for DOWN = 2, 4 for DOWN = 1) instead of the whole strip -- so strips can be
// tall (the vertical halo is re-read once per strip: (rows*DOWN + 3) / (rows*DOWN) instead of
// 10 / 8 rows for the 4-row strips) at ~half the registers.  The next input row's loads are
// issued before the current row's arithmetic (one row of prefetch).
//   out row oy reads input rows oy*DOWN - P0 + i, i < 4: input row t feeds tap i = t - oy*DOWN + P0.
template <int DOWN, int P0, int SEGW, int NOC, bool TAIL, int RB = 0>
__global__ __launch_bounds__(256) void upfirdn2d_roll(const float* __restrict__ x,
                                                       const float* __restrict__ kern,
                                                       float* __restrict__ out, int in_h,
                                                       int in_w, int kh, int kw, int out_h,
                                                       int out_w, int rows, int strips_x,
                                                       int strips_y, int64_t n_strips) {
  static_assert(DOWN == 1 || DOWN == 2, "upfirdn2d_roll: down 1 or 2");
  constexpr int LV = NOC * DOWN;                 // input columns loaded per lane
  constexpr int NOCT = NOC + (TAIL ? 1 : 0);     // columns computed (tail on the last lane)
  constexpr int NA = 4 / DOWN;                   // output rows in flight
  constexpr int SEGS = 64 / SEGW;
  const int lane = threadIdx.x & 63;
  const int sl = lane % SEGW;
  const int64_t strip = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * SEGS + lane / SEGW;
  const bool active = strip < n_strips;
  const int64_t sidx = active ? strip : 0;
  const int sxi = (int)(sidx % strips_x);
  const int syi = (int)((sidx / strips_x) % strips_y);
  const int64_t plane = sidx / ((int64_t)strips_x * strips_y);
  const int ox0 = sxi * SEGW * NOC;
  const int oyb = syi * rows;
  const int oye = min(oyb + rows, out_h);
  const int mycol = ox0 * DOWN + LV * sl;

  float w[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w[i][j] = (i < kh && j < kw) ? kern[(kh - 1 - i) * kw + (kw - 1 - j)] : 0.f;

  const float* xp = x + plane * in_h * in_w;
  // one input row: own LV columns (vector load), the neighbours' by segment shuffles, the
  // segment edges' by direct loads (zero outside the plane)
  auto load_row = [&](int iy, float (&own)[LV]) {
    const bool row_ok = active && iy >= 0 && iy < in_h;
    const float* row = xp + (int64_t)(row_ok ? iy : 0) * in_w;
    if constexpr (LV == 4) {
      if (row_ok && mycol + 3 < in_w) {
        const float4 v = *reinterpret_cast<const float4*>(row + mycol);
        own[0] = v.x; own[1] = v.y; own[2] = v.z; own[3] = v.w;
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) own[c] = (row_ok && mycol + c < in_w) ? row[mycol + c] : 0.f;
      }
    } else if constexpr (LV == 2) {
      if (row_ok && mycol + 1 < in_w) {
        const float2 v = *reinterpret_cast<const float2*>(row + mycol);
        own[0] = v.x; own[1] = v.y;
      } else {
        own[0] = (row_ok && mycol < in_w) ? row[mycol] : 0.f;
        own[1] = (row_ok && mycol + 1 < in_w) ? row[mycol + 1] : 0.f;
      }
    } else {
      own[0] = (row_ok && mycol < in_w) ? row[mycol] : 0.f;
    }
  };
  auto edges = [&](int iy, const float (&own)[LV], float (&left)[LV], float (&right)[LV]) {
#pragma unroll
    for (int c = 0; c < LV; ++c) {
      left[c] = __shfl_up(own[c], 1, SEGW);
      right[c] = __shfl_down(own[c], 1, SEGW);
    }
    const bool row_ok = active && iy >= 0 && iy < in_h;
    const float* row = xp + (int64_t)(row_ok ? iy : 0) * in_w;
    if (sl == 0) {
#pragma unroll
      for (int c = 0; c < LV; ++c) {
        const int col = mycol - LV + c;
        left[c] = (row_ok && col >= 0 && col < in_w) ? row[col] : 0.f;
      }
    }
    if (sl == SEGW - 1) {
#pragma unroll
      for (int c = 0; c < LV; ++c) {
        const int col = mycol + LV + c;
        right[c] = (row_ok && col < in_w) ? row[col] : 0.f;
      }
    }
  };
  // acc[oc] += (horizontal taps of row `i` applied to this input row)
  auto hsum = [&](int i, const float (&own)[LV], const float (&left)[LV],
                  const float (&right)[LV], float (&acc)[NOCT]) {
#pragma unroll
    for (int oc = 0; oc < NOCT; ++oc)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = oc * DOWN + j - P0;
        const int lo = bpk::floordiv(q, LV);
        const int comp = bpk::floormod(q, LV);
        const float v = lo < 0 ? left[comp] : (lo == 0 ? own[comp] : right[comp]);
        acc[oc] = fmaf(v, w[i][j], acc[oc]);
      }
  };
  const int oxl = ox0 + NOC * sl;
  float* op = out + plane * out_h * out_w;
  auto store = [&](int oy, const float (&acc)[NOCT]) {
    if (!active || oy < oyb || oy >= oye) return;
    float* orow = op + (int64_t)oy * out_w;
    if constexpr (NOC == 4 && TAIL) {  // odd row pitch: the widest store the address allows
      const int64_t e0 = (plane * out_h + oy) * (int64_t)out_w + oxl;
      if ((e0 & 3) == 0) {
        *reinterpret_cast<float4*>(orow + oxl) = make_float4(acc[0], acc[1], acc[2], acc[3]);
      } else if ((e0 & 1) == 0) {
        *reinterpret_cast<float2*>(orow + oxl) = make_float2(acc[0], acc[1]);
        *reinterpret_cast<float2*>(orow + oxl + 2) = make_float2(acc[2], acc[3]);
      } else {  // odd: one float, an aligned pair, one float
        orow[oxl] = acc[0];
        *reinterpret_cast<float2*>(orow + oxl + 1) = make_float2(acc[1], acc[2]);
        orow[oxl + 3] = acc[3];
      }
    } else if constexpr (NOC == 2 && TAIL) {
      const int64_t e0 = (plane * out_h + oy) * (int64_t)out_w + oxl;
      if ((e0 & 1) == 0) {
        *reinterpret_cast<float2*>(orow + oxl) = make_float2(acc[0], acc[1]);
      } else {
        orow[oxl] = acc[0];
        orow[oxl + 1] = acc[1];
      }
    } else if constexpr (NOC == 4) {
      if (oxl + 3 < out_w) {
        *reinterpret_cast<float4*>(orow + oxl) = make_float4(acc[0], acc[1], acc[2], acc[3]);
      } else {
#pragma unroll
        for (int oc = 0; oc < 4; ++oc)
          if (oxl + oc < out_w) orow[oxl + oc] = acc[oc];
      }
    } else if constexpr (NOC == 2) {
      if (oxl + 1 < out_w && (((int64_t)oy * out_w + oxl) & 1) == 0 && (out_h * out_w) % 2 == 0) {
        *reinterpret_cast<float2*>(orow + oxl) = make_float2(acc[0], acc[1]);
      } else {
        if (oxl < out_w) orow[oxl] = acc[0];
        if (oxl + 1 < out_w) orow[oxl + 1] = acc[1];
      }
    } else {
      if (oxl < out_w) orow[oxl] = acc[0];
    }
    if constexpr (TAIL) {
      if (sl == SEGW - 1) orow[out_w - 1] = acc[NOC];
    }
  };

  float acc[NA][NOCT];
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int oc = 0; oc < NOCT; ++oc) acc[a][oc] = 0.f;
  // input rows t0 .. t1 feed output rows oyb .. oye - 1
  const int t0 = oyb * DOWN - P0;
  const int t1 = (oye - 1) * DOWN - P0 + 3;
  float cur[LV], nxt[LV], left[LV], right[LV];
  load_row(t0, cur);
  if constexpr (DOWN == 1 && RB > 0) {
    // RB = rows (compile time): the strip's output rows stay in registers and are stored
    // after its last input row, so no row load is issued behind a store (gfx9 counts stores in
    // vmcnt: waiting for such a load also waited for the store before it)
    float ob[RB][NOCT];
#pragma unroll
    for (int it = 0; it < RB + 3; ++it) {
      const int t = t0 + it;
      if (t <= t1) {
        if (t < t1) load_row(t + 1, nxt);
        edges(t, cur, left, right);
#pragma unroll
        for (int k = 0; k < 4; ++k) hsum(3 - k, cur, left, right, acc[k]);
      }
      if (it >= 3) {
#pragma unroll
        for (int oc = 0; oc < NOCT; ++oc) ob[it >= 3 ? it - 3 : 0][oc] = acc[0][oc];
      }
#pragma unroll
      for (int oc = 0; oc < NOCT; ++oc) {
        acc[0][oc] = acc[1][oc];
        acc[1][oc] = acc[2][oc];
        acc[2][oc] = acc[3][oc];
        acc[3][oc] = 0.f;
      }
#pragma unroll
      for (int c = 0; c < LV; ++c) cur[c] = nxt[c];
    }
#pragma unroll
    for (int r = 0; r < RB; ++r) store(oyb + r, ob[r]);
  } else if constexpr (DOWN == 1) {
    // acc[k] = output row t + P0 - 3 + k (tap 3 - k of input row t); after row t, acc[0] is
    // complete
    for (int t = t0; t <= t1; ++t) {
      if (t < t1) load_row(t + 1, nxt);
      edges(t, cur, left, right);
#pragma unroll
      for (int k = 0; k < 4; ++k) hsum(3 - k, cur, left, right, acc[k]);
      store(t + P0 - 3, acc[0]);
#pragma unroll
      for (int oc = 0; oc < NOCT; ++oc) {
        acc[0][oc] = acc[1][oc];
        acc[1][oc] = acc[2][oc];
        acc[2][oc] = acc[3][oc];
        acc[3][oc] = 0.f;
      }
#pragma unroll
      for (int c = 0; c < LV; ++c) cur[c] = nxt[c];
    }
  } else {
    // rows in pairs: row t = oy*2 - P0 + 2 (taps 2 of oy, 0 of oy + 1) and t + 1 (taps 3, 1);
    // acc[0] = output oy, acc[1] = oy + 1.  Prologue: rows t0, t0 + 1 (taps 0, 1 of oyb).
    // (Holding the strip's rows in registers and storing them after its last input row, as
    // the FIR form does, measured slower here: 0.60 -> 0.44 of HBM on [64,128,128,128],
    // 0.63 -> 0.47 on [64,256,64,64], round 4 -- the two in-flight accumulators already keep
    // the stores off the loads' critical path.)
    load_row(t0 + 1, nxt);
    edges(t0, cur, left, right);
    hsum(0, cur, left, right, acc[0]);
#pragma unroll
    for (int c = 0; c < LV; ++c) cur[c] = nxt[c];
    int t = t0 + 1;
    if (t + 1 <= t1) load_row(t + 1, nxt);
    edges(t, cur, left, right);
    hsum(1, cur, left, right, acc[0]);
#pragma unroll
    for (int c = 0; c < LV; ++c) cur[c] = nxt[c];
    for (int oy = oyb; oy < oye; ++oy) {
      t = oy * 2 - P0 + 2;  // cur holds row t
      load_row(t + 1, nxt);
      edges(t, cur, left, right);
      hsum(2, cur, left, right, acc[0]);
      hsum(0, cur, left, right, acc[1]);
#pragma unroll
      for (int c = 0; c < LV; ++c) cur[c] = nxt[c];
      if (oy + 1 < oye) load_row(t + 2, nxt);
      edges(t + 1, cur, left, right);
      hsum(3, cur, left, right, acc[0]);
      hsum(1, cur, left, right, acc[1]);
      store(oy, acc[0]);
#pragma unroll
      for (int oc = 0; oc < NOCT; ++oc) {
        acc[0][oc] = acc[1][oc];
        acc[1][oc] = 0.f;
      }
#pragma unroll
      for (int c = 0; c < LV; ++c) cur[c] = nxt[c];
    }
  }
}

template <int DOWN, int P0, int SEGW, int NOC, bool TAIL = false, int RB = 0>
int launch_roll(const float* x, const float* k, float* out, int major, int in_h, int in_w, int kh,
                int kw, int out_h, int out_w, int rows, hipStream_t st) {
  const int strips_x = TAIL ? 1 : (int)bpk::ceil_div(out_w, SEGW * NOC);
  const int strips_y = (int)bpk::ceil_div(out_h, rows);
  const int64_t n = (int64_t)major * strips_x * strips_y;
  if (n <= 0) return BPK_OK;
  const int64_t blocks = bpk::ceil_div(n, 4 * (64 / SEGW));
  BPK_REQUIRE(blocks < (int64_t)INT32_MAX, "upfirdn2d: grid too large");
  hipLaunchKernelGGL((upfirdn2d_roll<DOWN, P0, SEGW, NOC, TAIL, RB>), dim3((unsigned)blocks), dim3(256),
                     0, st, x, k, out, in_h, in_w, kh, kw, out_h, out_w, rows, strips_x, strips_y, n);
  BPK_LAUNCH_CHECK("upfirdn2d_roll");
  return BPK_OK;
}

// Strip height of the rolling kernel: down2 -> about 32 k waves (tools/gpu_upfirdn_roll.sh on
// MI355X: [64,128,128,128] best at 8 rows, [64,256,64,64] at 4, i.e. 32 k waves both), the
// odd-width 1:1 FIR -> the divisor of the height in 5..8 (65 = 13 x 5; 5 and 6 rows: 0.59 of
// HBM vs 0.45 for the 4-row stream strips).
int roll_rows_down2(int major, int out_h, int strips_x, int segs) {
  const double per = (double)major * out_h * strips_x / (32768.0 * segs);
  return std::max(3, std::min(64, (int)(per + 0.5)));
}

int roll_rows_fir(int out_h) {
  for (int c = 5; c <= 8; ++c)
    if (out_h % c == 0) return c;
  return 6;
}

bool try_roll(const float* x, const float* k, float* out, int major, int in_h, int in_w, int kh,
              int kw, int down, int p0, int out_h, int out_w, hipStream_t st, int* rc) {
  const bool a16 = (reinterpret_cast<uintptr_t>(x) & 15) == 0 && in_w % 4 == 0;
  if (down == 2 && a16 && (p0 == 1 || p0 == 2)) {
    const int lanes = (int)bpk::ceil_div(out_w, 2);  // two output columns per lane
    const int sw = lanes <= 8 ? 8 : lanes <= 16 ? 16 : lanes <= 32 ? 32 : 64;
    const int rows = roll_rows_down2(major, out_h, (int)bpk::ceil_div(out_w, 2 * sw), 64 / sw);
#define BPK_ROLL2(P, SW) \
  return (*rc = launch_roll<2, P, SW, 2>(x, k, out, major, in_h, in_w, kh, kw, out_h, out_w, rows, st), true)
    if (p0 == 1) {
      if (sw == 8) BPK_ROLL2(1, 8);
      if (sw == 16) BPK_ROLL2(1, 16);
      if (sw == 32) BPK_ROLL2(1, 32);
      BPK_ROLL2(1, 64);
    }
    if (sw == 8) BPK_ROLL2(2, 8);
    if (sw == 16) BPK_ROLL2(2, 16);
    if (sw == 32) BPK_ROLL2(2, 32);
    BPK_ROLL2(2, 64);
#undef BPK_ROLL2
  }
  if (down == 1 && p0 == 2 && (out_w & 1) && kw == 4 && a16) {
    const int rows = roll_rows_fir(out_h);
    const int lanes4 = (out_w - 1) / 4;  // 2^k + 1 wide: four columns per lane + the tail
    // output rows kept in registers and stored after the strip's last input row: [64,128,64,64]
    // 0.559 -> 0.610 of the HBM peak (round 3, one box, twice)
    if (rows == 5 && out_h % 5 == 0) {
#define BPK_ROLLTB(SW) \
  return (*rc = launch_roll<1, 2, SW, 4, true, 5>(x, k, out, major, in_h, in_w, kh, kw, out_h, out_w, rows, st), true)
      if (lanes4 == 64) BPK_ROLLTB(64);
      if (lanes4 == 32) BPK_ROLLTB(32);
      if (lanes4 == 16) BPK_ROLLTB(16);
      if (lanes4 == 8) BPK_ROLLTB(8);
#undef BPK_ROLLTB
    }
#define BPK_ROLLT(SW) \
  return (*rc = launch_roll<1, 2, SW, 4, true>(x, k, out, major, in_h, in_w, kh, kw, out_h, out_w, rows, st), true)
    if (lanes4 == 64) BPK_ROLLT(64);
    if (lanes4 == 32) BPK_ROLLT(32);
    if (lanes4 == 16) BPK_ROLLT(16);
    if (lanes4 == 8) BPK_ROLLT(8);
#undef BPK_ROLLT
  }
  return false;
}

// returns true (and sets *rc) when a streaming specialisation applies
bool try_stream(const float* x, const float* k, float* out, int major, int in_h, int in_w,
                int kh, int kw, int up, int down, int p0, int out_h, int out_w, hipStream_t st,
                int* rc) {
  if (kh > 4 || kw > 4 || (reinterpret_cast<uintptr_t>(x) & 7) ||
      (reinterpret_cast<uintptr_t>(out) & 7))
    return false;
#define BPK_STREAM(U, D, P, RR) \
  (*rc = launch_stream<U, D, P, RR>(x, k, out, major, in_h, in_w, kh, kw, out_h, out_w, st), true)
  // strip heights measured on MI355X (tools/ab_upfirdn.sh): R = 4 (down2), 16 (up2), 8 (1x1)
  if (in_w % 2 != 0) return false;  // 8-byte row loads need an even row pitch
  if (up == 1 && try_roll(x, k, out, major, in_h, in_w, kh, kw, down, p0, out_h, out_w, st, rc))
    return true;
  if (up == 1 && down == 2) {
    // two output columns per lane (16-byte input loads) where rows allow it
    if (in_w % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
      if (p0 == 1) return (*rc = launch_stream<1, 2, 1, 4, 2>(x, k, out, major, in_h, in_w, kh, kw, out_h, out_w, st), true);
      if (p0 == 2) return (*rc = launch_stream<1, 2, 2, 4, 2>(x, k, out, major, in_h, in_w, kh, kw, out_h, out_w, st), true);
    }
    if (p0 == 1) return BPK_STREAM(1, 2, 1, 4);
    if (p0 == 2) return BPK_STREAM(1, 2, 2, 4);
  }
  if (up == 1 && down == 1) {
    if (p0 == 2 && (out_w & 1) && kw == 4) {
      // odd width 2^k + 1 (the FIR pad(2, 2) of conv_downsample_2d): a segment of
      // (out_w - 1) / 2 lanes with the tail column on its last lane
      // (reached only when the rolling kernel above does not apply: a misaligned input).
      // 4-row strips with 4 columns per lane (16-byte row loads), else 8 rows with 2 columns
      // per lane; round 1 on [64,128,64,64] -> 65^2: 39.8 % / 32.6 % of the HBM peak
      const int lanes = (out_w - 1) / 2;
#define BPK_TAIL2(SW) \
  return (*rc = launch_stream_seg<1, 1, 2, 8, SW, 0, true>(x, k, out, major, in_h, in_w, kh, kw, out_h, out_w, st), true)
#define BPK_TAIL4(SW, RR) \
  return (*rc = launch_stream_seg<1, 1, 2, RR, SW, 4, true>(x, k, out, major, in_h, in_w, kh, kw, out_h, out_w, st), true)
      const int lanes4 = (out_w - 1) / 4;
      if ((reinterpret_cast<uintptr_t>(x) & 15) == 0 && in_w % 4 == 0) {
        if (lanes4 == 64) BPK_TAIL4(64, 4);
        if (lanes4 == 32) BPK_TAIL4(32, 4);
        if (lanes4 == 16) BPK_TAIL4(16, 4);
        if (lanes4 == 8) BPK_TAIL4(8, 4);
      }
      if (lanes == 64) BPK_TAIL2(64);
      if (lanes == 32) BPK_TAIL2(32);
      if (lanes == 16) BPK_TAIL2(16);  // 33-wide
      if (lanes == 8) BPK_TAIL2(8);    // 17-wide
#undef BPK_TAIL2
#undef BPK_TAIL4
    }
    if (p0 == 1) return BPK_STREAM(1, 1, 1, 8);
    if (p0 == 2) return BPK_STREAM(1, 1, 2, 8);
  }
  if (up == 2 && down == 1 && p0 == 2) {
    // four output columns per lane (8-byte input loads, 16-byte stores) when rows allow it
    if (out_w % 4 == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0)
      return (*rc = launch_stream<2, 1, 2, 16, 4>(x, k, out, major, in_h, in_w, kh, kw, out_h, out_w, st), true);
    return BPK_STREAM(2, 1, 2, 16);
  }
#undef BPK_STREAM
  return false;
}

template <typename T>
int upfirdn2d_impl(const T* x, const T* k, T* out, int major, int in_h, int in_w, int minor,
                   int kh, int kw, int ux, int uy, int dx, int dy, int px0, int px1, int py0,
                   int py1, int out_h, int out_w, void* stream) {
  BPK_REQUIRE(major >= 0 && in_h > 0 && in_w > 0 && minor > 0, "upfirdn2d: bad input shape");
  BPK_REQUIRE(kh > 0 && kw > 0, "upfirdn2d: empty kernel");
  BPK_REQUIRE(ux > 0 && uy > 0 && dx > 0 && dy > 0, "upfirdn2d: factors must be positive");
  const int exp_h = (in_h * uy + py0 + py1 - kh) / dy + 1;
  const int exp_w = (in_w * ux + px0 + px1 - kw) / dx + 1;
  BPK_REQUIRE(out_h == exp_h && out_w == exp_w,
              "upfirdn2d: out shape (%d,%d) != expected (%d,%d)", out_h, out_w, exp_h, exp_w);
  BPK_REQUIRE(out_h > 0 && out_w > 0, "upfirdn2d: empty output");
  if (major == 0) return BPK_OK;
  hipStream_t st = bpk::as_stream(stream);
  if constexpr (std::is_same<T, float>::value) {
    if (minor == 1 && ux == uy && dx == dy && px0 == py0) {
      int rc = BPK_OK;
      if (try_stream(x, k, out, major, in_h, in_w, kh, kw, ux, dx, px0, out_h, out_w, st, &rc))
        return rc;
    }
  }
  const bool tiled = minor == 1 && ux == uy && dx == dy && kh <= 4 && kw <= 4 &&
                     ((ux == 1 && dx == 1) || (ux == 2 && dx == 1) || (ux == 1 && dx == 2));
  if (tiled) {
    if (ux == 2)
      return launch_tiled_w<T, 2, 1>(x, k, out, major, in_h, in_w, kh, kw, px0, py0, out_h, out_w,
                                     st);
    if (dx == 2)
      return launch_tiled_w<T, 1, 2>(x, k, out, major, in_h, in_w, kh, kw, px0, py0, out_h, out_w,
                                     st);
    return launch_tiled_w<T, 1, 1>(x, k, out, major, in_h, in_w, kh, kw, px0, py0, out_h, out_w,
                                   st);
  }
  const int64_t total = (int64_t)major * out_h * out_w * minor;
  const int64_t blocks = std::min<int64_t>(bpk::ceil_div(total, 256), 256 * 32);
  hipLaunchKernelGGL(upfirdn2d_direct<T>, dim3((unsigned)blocks), dim3(256), 0, st, x, k, out,
                     in_h, in_w, minor, kh, kw, ux, uy, dx, dy, px0, py0, out_h, out_w, total);
  BPK_LAUNCH_CHECK("upfirdn2d_direct");
  return BPK_OK;
}

}  // namespace

extern "C" int bpk_upfirdn2d_f32(const float* x, const float* kernel, float* out, int major,
                                 int in_h, int in_w, int minor, int kernel_h, int kernel_w,
                                 int up_x, int up_y, int down_x, int down_y, int pad_x0,
                                 int pad_x1, int pad_y0, int pad_y1, int out_h, int out_w,
                                 void* stream) {
  return upfirdn2d_impl<float>(x, kernel, out, major, in_h, in_w, minor, kernel_h, kernel_w, up_x,
                               up_y, down_x, down_y, pad_x0, pad_x1, pad_y0, pad_y1, out_h, out_w,
                               stream);
}

extern "C" int bpk_upfirdn2d_f64(const double* x, const double* kernel, double* out, int major,
                                 int in_h, int in_w, int minor, int kernel_h, int kernel_w,
                                 int up_x, int up_y, int down_x, int down_y, int pad_x0,
                                 int pad_x1, int pad_y0, int pad_y1, int out_h, int out_w,
                                 void* stream) {
  return upfirdn2d_impl<double>(x, kernel, out, major, in_h, in_w, minor, kernel_h, kernel_w, up_x,
                                up_y, down_x, down_y, pad_x0, pad_x1, pad_y0, pad_y1, out_h, out_w,
                                stream);
}
