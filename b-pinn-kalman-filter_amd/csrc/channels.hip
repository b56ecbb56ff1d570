// Flow-component swap + scale of FlowNet's `project` (reference models/flownet.py:8-25):
// out[n, 0] = u[n, 1] / c0, out[n, 1] = u[n, 0] / c1 for a two-channel flow u [N, 2, P].
// The map is linear and its adjoint is the same map with c0 and c1 exchanged, so every
// derivative order of the PINN residual (pinn_kalman/pinn.py:72-111) runs this one kernel
// (op.channels.swap_scale) -- aten needed two divisions into slices of an empty output per
// call.  Division by a scalar as aten performs it -- multiplication by the fp32 reciprocal
// 1.f / c -- so the results are bit-identical.
#include "bpk_common.h"

#include <algorithm>
#include <type_traits>

namespace {

template <int V>
__global__ __launch_bounds__(256) void swap_scale_kernel(const float* __restrict__ u,
                                                         float* __restrict__ out, int64_t units,
                                                         int64_t pv, float c0, float c1) {
  const float r0 = 1.f / c0, r1 = 1.f / c1;
  using vec = typename std::conditional<V == 4, float4, float>::type;
  const vec* uv = reinterpret_cast<const vec*>(u);
  vec* ov = reinterpret_cast<vec*>(out);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < units;
       i += (int64_t)gridDim.x * 256) {
    const int64_t n = i / pv, p = i - n * pv;
    const int64_t a = 2 * n * pv + p, b = a + pv;  // channel 0 / channel 1 element
    const vec x0 = uv[a], x1 = uv[b];
    if constexpr (V == 4) {
      ov[a] = make_float4(x1.x * r0, x1.y * r0, x1.z * r0, x1.w * r0);
      ov[b] = make_float4(x0.x * r1, x0.y * r1, x0.z * r1, x0.w * r1);
    } else {
      ov[a] = x1 * r0;
      ov[b] = x0 * r1;
    }
  }
}

// the channels-last layout [N, P, 2] (the gradients the PINN residual sends back through
// project's NHWC grid view): two pixels' (c0, c1) pairs per float4
__global__ __launch_bounds__(256) void swap_scale_pairs_kernel(const float4* __restrict__ u,
                                                               float4* __restrict__ out,
                                                               int64_t units, float c0, float c1) {
  const float r0 = 1.f / c0, r1 = 1.f / c1;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < units;
       i += (int64_t)gridDim.x * 256) {
    const float4 x = u[i];
    out[i] = make_float4(x.y * r0, x.x * r1, x.w * r0, x.z * r1);
  }
}

__global__ __launch_bounds__(256) void swap_scale_pair_kernel(const float2* __restrict__ u,
                                                              float2* __restrict__ out,
                                                              int64_t units, float c0, float c1) {
  const float r0 = 1.f / c0, r1 = 1.f / c1;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < units;
       i += (int64_t)gridDim.x * 256) {
    const float2 x = u[i];
    out[i] = make_float2(x.y * r0, x.x * r1);
  }
}

// y[p][i][j] = (x[p][2i][2j] + x[p][2i][2j+1]) + (x[p][2i+1][2j] + x[p][2i+1][2j+1]) over planes
// p: the adjoint of the nearest x2 upsample (the `ddpm` net's Upsample under autograd, DPS:
// op.conv._ConvUp2's input gradient).  aten ran it as a strided reduction over a 6-D view
// (≈470 us per call at 256^2); one pass here, two output pixels per thread from two float4 rows
template <bool V4>
__global__ __launch_bounds__(256) void sum2x2_kernel(const float* __restrict__ x,
                                                     float* __restrict__ y, int64_t units,
                                                     int H, int W) {
  const int Wq = V4 ? W / 2 : W;  // units per output row: pairs of output pixels (V4) or pixels
  for (int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x; u < units;
       u += (int64_t)gridDim.x * 256) {
    const int64_t row = u / Wq;  // output row index over all planes
    const int c = (int)(u - row * Wq);
    const int64_t p = row / H;
    const int i = (int)(row - p * H);
    const float* r0 = x + (p * 2 * H + 2 * i) * (int64_t)(2 * W);
    const float* r1 = r0 + 2 * W;
    if constexpr (V4) {
      const float4 a = reinterpret_cast<const float4*>(r0)[c];
      const float4 b = reinterpret_cast<const float4*>(r1)[c];
      reinterpret_cast<float2*>(y + row * W)[c] =
          make_float2((a.x + a.y) + (b.x + b.y), (a.z + a.w) + (b.z + b.w));
    } else {
      y[row * W + c] = (r0[2 * c] + r0[2 * c + 1]) + (r1[2 * c] + r1[2 * c + 1]);
    }
  }
}

}  // namespace

extern "C" int bpk_sum2x2_f32(const float* x, float* y, int64_t planes, int H, int W,
                              void* stream) {
  BPK_REQUIRE(planes >= 0 && H > 0 && W > 0, "sum2x2: bad shape");
  BPK_REQUIRE(x && y, "sum2x2: null pointer");
  if (planes == 0) return BPK_OK;
  const bool v4 = W % 2 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(y) & 7) == 0;
  const int64_t units = planes * H * (v4 ? W / 2 : W);
  const unsigned blocks = (unsigned)std::min<int64_t>(bpk::ceil_div(units, 256), 8192);
  if (v4)
    hipLaunchKernelGGL(sum2x2_kernel<true>, dim3(blocks), dim3(256), 0, bpk::as_stream(stream), x,
                       y, units, H, W);
  else
    hipLaunchKernelGGL(sum2x2_kernel<false>, dim3(blocks), dim3(256), 0, bpk::as_stream(stream), x,
                       y, units, H, W);
  BPK_LAUNCH_CHECK("sum2x2");
  return BPK_OK;
}

extern "C" int bpk_swap_scale_f32(const float* u, float* out, int64_t N, int64_t P, float c0,
                                  float c1, int channels_last, void* stream) {
  BPK_REQUIRE(N >= 0 && P >= 0, "swap_scale: bad shape N=%lld P=%lld", (long long)N,
              (long long)P);
  BPK_REQUIRE(u && out && u != out, "swap_scale: null or aliased pointers");
  if (N == 0 || P == 0) return BPK_OK;
  hipStream_t st = bpk::as_stream(stream);
  const bool al = (reinterpret_cast<uintptr_t>(u) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(out) & 15) == 0;
  if (channels_last) {
    const int64_t pix = N * P;
    const bool v4 = al && pix % 2 == 0;
    const int64_t units = v4 ? pix / 2 : pix;
    const unsigned blocks = (unsigned)std::min<int64_t>(bpk::ceil_div(units, 256), 4096);
    if (v4)
      hipLaunchKernelGGL(swap_scale_pairs_kernel, dim3(blocks), dim3(256), 0, st,
                         reinterpret_cast<const float4*>(u), reinterpret_cast<float4*>(out),
                         units, c0, c1);
    else
      hipLaunchKernelGGL(swap_scale_pair_kernel, dim3(blocks), dim3(256), 0, st,
                         reinterpret_cast<const float2*>(u), reinterpret_cast<float2*>(out),
                         units, c0, c1);
    BPK_LAUNCH_CHECK("swap_scale");
    return BPK_OK;
  }
  const bool v4 = P % 4 == 0 && al;
  const int64_t pv = v4 ? P / 4 : P, units = N * pv;
  const unsigned blocks = (unsigned)std::min<int64_t>(bpk::ceil_div(units, 256), 4096);
  if (v4)
    hipLaunchKernelGGL(swap_scale_kernel<4>, dim3(blocks), dim3(256), 0, st, u, out, units, pv,
                       c0, c1);
  else
    hipLaunchKernelGGL(swap_scale_kernel<1>, dim3(blocks), dim3(256), 0, st, u, out, units, pv,
                       c0, c1);
  BPK_LAUNCH_CHECK("swap_scale");
  return BPK_OK;
}
