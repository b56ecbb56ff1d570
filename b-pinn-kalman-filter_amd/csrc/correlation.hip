// FlowNet cost volume ("correlation") for gfx950: forward and both input grads.
//
// Semantics (op/correlation.py:13-231, the CuPy kernels of the reference):
//   out[b, d, oy, ox] = (1/C) * sum_c first[b, c, y, x] * second[b, c, y + dy*s, x + dx*s]
//   with (y, x) = (oy*s, ox*s), d = (dy + 3) * 7 + (dx + 3), dx, dy in [-3, 3],
//   zero outside the image (the reference zero-pads by 3*s, :296-306), and an
//   output of ceil(H/s) x ceil(W/s) (:317-321).
//   grad_first[b, c, y, x]  = (1/C) sum_d gout[b, d, y/s, x/s] * second[b, c, y+dy*s, x+dx*s]
//                             (only on the stride grid, :104-165)
//   grad_second[b, c, y, x] = (1/C) sum_d gout[b, d, y/s - dy, x/s - dx] * first[b, c, y-dy*s, x-dx*s]
//                             (:167-231)
// The displacement sums run in the reference's order (dy outer, dx inner).
//
// MI355X design: no NHWC "rearrange" copies and no padded scratch (the reference
// materialises two padded [B, H+6s, W+6s, C] tensors per call).  NCHW is read
// directly; x is the fastest thread index, so every load/store is a coalesced row
// segment, and the 7x7 neighbourhood re-reads are served from L1/L2.  The forward
// runs one thread per (b, dy, oy, ox) with the 7 dx partial sums in registers; the
// reference's block-shared 32-way reduction (which races on `sum[]`, :69,89-100) is
// replaced by a per-thread sequential channel sum.
#include "bpk_common.h"

#include <algorithm>

namespace {

constexpr int kDisp = 3;
constexpr int kWin = 2 * kDisp + 1;  // 7
constexpr int kD = kWin * kWin;      // 49

struct CorrGeo {
  int B, C, H, W, Ho, Wo, s;
};

__global__ __launch_bounds__(256) void corr_fwd_kernel(const float* __restrict__ first,
                                                       const float* __restrict__ second,
                                                       float* __restrict__ out, CorrGeo g) {
  const int64_t total = (int64_t)g.B * kWin * g.Ho * g.Wo;
  const int64_t plane = (int64_t)g.H * g.W;
  const float inv_c = 1.0f / (float)g.C;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int ox = (int)(i % g.Wo);
    int64_t r = i / g.Wo;
    const int oy = (int)(r % g.Ho);
    r /= g.Ho;
    const int p = (int)(r % kWin);  // dy + 3
    const int b = (int)(r / kWin);
    const int y = oy * g.s, x = ox * g.s;
    const int y2 = y + (p - kDisp) * g.s;
    float acc[kWin];
#pragma unroll
    for (int o = 0; o < kWin; ++o) acc[o] = 0.f;
    if (y2 >= 0 && y2 < g.H) {
      const float* f1 = first + (int64_t)b * g.C * plane + (int64_t)y * g.W + x;
      const float* f2 = second + (int64_t)b * g.C * plane + (int64_t)y2 * g.W;
      bool ok[kWin];
#pragma unroll
      for (int o = 0; o < kWin; ++o) {
        const int x2 = x + (o - kDisp) * g.s;
        ok[o] = x2 >= 0 && x2 < g.W;
      }
      for (int c = 0; c < g.C; ++c) {
        const float a = f1[(int64_t)c * plane];
        const float* row = f2 + (int64_t)c * plane;
#pragma unroll
        for (int o = 0; o < kWin; ++o) {
          const int x2 = x + (o - kDisp) * g.s;
          const float v = ok[o] ? row[x2] : 0.f;
          acc[o] += a * v;
        }
      }
    }
    float* dst = out + (((int64_t)b * kD + p * kWin) * g.Ho + oy) * g.Wo + ox;
    const int64_t dstride = (int64_t)g.Ho * g.Wo;
#pragma unroll
    for (int o = 0; o < kWin; ++o) dst[o * dstride] = acc[o] * inv_c;
  }
}

// One thread per (b, c, y, x) of the input planes; computes grad_first and/or
// grad_second for that element.
__global__ __launch_bounds__(256) void corr_bwd_kernel(const float* __restrict__ first,
                                                       const float* __restrict__ second,
                                                       const float* __restrict__ gout,
                                                       float* __restrict__ grad_first,
                                                       float* __restrict__ grad_second,
                                                       CorrGeo g) {
  const int64_t plane = (int64_t)g.H * g.W;
  const int64_t total = (int64_t)g.B * g.C * plane;
  const int64_t oplane = (int64_t)g.Ho * g.Wo;
  const float inv_c = 1.0f / (float)g.C;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(i % g.W);
    int64_t r = i / g.W;
    const int y = (int)(r % g.H);
    r /= g.H;
    const int c = (int)(r % g.C);
    const int b = (int)(r / g.C);
    const bool on_grid = (x % g.s == 0) && (y % g.s == 0);
    const int oy0 = y / g.s, ox0 = x / g.s;
    const float* go = gout + (int64_t)b * kD * oplane;
    const float* f1 = first + ((int64_t)b * g.C + c) * plane;
    const float* f2 = second + ((int64_t)b * g.C + c) * plane;
    if (grad_first) {
      float sum = 0.f;
      if (on_grid && oy0 < g.Ho && ox0 < g.Wo) {
        for (int p = 0; p < kWin; ++p) {
          const int y2 = y + (p - kDisp) * g.s;
#pragma unroll
          for (int o = 0; o < kWin; ++o) {
            const int x2 = x + (o - kDisp) * g.s;
            const float v = (y2 >= 0 && y2 < g.H && x2 >= 0 && x2 < g.W)
                                ? f2[(int64_t)y2 * g.W + x2] : 0.f;
            sum += go[(int64_t)(p * kWin + o) * oplane + (int64_t)oy0 * g.Wo + ox0] * v;
          }
        }
      }
      grad_first[i] = sum * inv_c;
    }
    if (grad_second) {
      float sum = 0.f;
      if (on_grid) {
        for (int p = 0; p < kWin; ++p) {
          const int oy = oy0 - (p - kDisp);
          if (oy < 0 || oy >= g.Ho) continue;
#pragma unroll
          for (int o = 0; o < kWin; ++o) {
            const int ox = ox0 - (o - kDisp);
            if (ox < 0 || ox >= g.Wo) continue;
            const float v = f1[(int64_t)(oy * g.s) * g.W + ox * g.s];
            sum += go[(int64_t)(p * kWin + o) * oplane + (int64_t)oy * g.Wo + ox] * v;
          }
        }
      }
      grad_second[i] = sum * inv_c;
    }
  }
}

unsigned blocks_for(int64_t n) { return (unsigned)std::min<int64_t>(bpk::ceil_div(n, 256), 65536); }

}  // namespace

extern "C" int bpk_correlation_fwd_f32(const float* first, const float* second, float* out, int B,
                                       int C, int H, int W, int stride, void* stream) {
  BPK_REQUIRE(B >= 0 && C > 0 && H > 0 && W > 0, "correlation: bad shape B=%d C=%d H=%d W=%d", B,
              C, H, W);
  BPK_REQUIRE(stride >= 1, "correlation: stride must be >= 1 (got %d)", stride);
  const CorrGeo g{B, C, H, W, (H + stride - 1) / stride, (W + stride - 1) / stride, stride};
  const int64_t n = (int64_t)B * kWin * g.Ho * g.Wo;
  if (n == 0) return BPK_OK;
  hipLaunchKernelGGL(corr_fwd_kernel, dim3(blocks_for(n)), dim3(256), 0, bpk::as_stream(stream),
                     first, second, out, g);
  BPK_LAUNCH_CHECK("correlation_fwd");
  return BPK_OK;
}

extern "C" int bpk_correlation_bwd_f32(const float* first, const float* second,
                                       const float* grad_out, float* grad_first,
                                       float* grad_second, int B, int C, int H, int W, int stride,
                                       void* stream) {
  BPK_REQUIRE(B >= 0 && C > 0 && H > 0 && W > 0, "correlation: bad shape B=%d C=%d H=%d W=%d", B,
              C, H, W);
  BPK_REQUIRE(stride >= 1, "correlation: stride must be >= 1 (got %d)", stride);
  const CorrGeo g{B, C, H, W, (H + stride - 1) / stride, (W + stride - 1) / stride, stride};
  const int64_t n = (int64_t)B * C * H * W;
  if (n == 0 || (!grad_first && !grad_second)) return BPK_OK;
  hipLaunchKernelGGL(corr_bwd_kernel, dim3(blocks_for(n)), dim3(256), 0, bpk::as_stream(stream),
                     first, second, grad_out, grad_first, grad_second, g);
  BPK_LAUNCH_CHECK("correlation_bwd");
  return BPK_OK;
}
