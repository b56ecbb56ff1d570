// fused bias + activation (+ derivative mask), and the residual rescale used by
// every BigGAN/DDPM++ block.
//
// fused_bias_act semantics: op/fused_bias_act_kernel.cu:18-49 (GPU path of the
// reference).  y = scale * act(x + b[(i / step_b) % size_b]);
//   act 1 (linear): grad 0/1 -> x, grad 2 -> 0
//   act 3 (lrelu) : grad 0 -> x > 0 ? x : alpha x ; grad 1 -> ref > 0 ? x : alpha x ; grad 2 -> 0
// Grid-stride elementwise kernel, 4 elements per thread per iteration.
#include "bpk_common.h"

#include <algorithm>

namespace {

template <typename T>
__global__ __launch_bounds__(256) void fused_bias_act_kernel(
    const T* __restrict__ x, const T* __restrict__ b, const T* __restrict__ ref, T* __restrict__ out,
    int64_t n, int64_t step_b, int64_t size_b, int act, int grad, T alpha, T scale) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    T v = x[i];
    if (b) v += b[(i / step_b) % size_b];
    const T r = ref ? ref[i] : T(0);
    T y;
    switch (act * 10 + grad) {
      default:
      case 10:
      case 11: y = v; break;
      case 12: y = T(0); break;
      case 30: y = (v > T(0)) ? v : v * alpha; break;
      case 31: y = (r > T(0)) ? v : v * alpha; break;
      case 32: y = T(0); break;
    }
    out[i] = y * scale;
  }
}

// no bias, float32, 16-B aligned, n % 4 == 0 (FlowNet's LeakyReLU(0.1) and its derivative
// mask, 242 launches per PINN step at B = 8): four elements per thread, the act / grad case
// resolved at compile time -- the same per-element arithmetic as above
template <int CASE>
__global__ __launch_bounds__(256) void lrelu4_kernel(const float4* __restrict__ x,
                                                     const float4* __restrict__ ref,
                                                     float4* __restrict__ out, int64_t n4,
                                                     float alpha, float scale) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = x[i];
    const float4 r = CASE == 31 ? ref[i] : v;
    float4 y;
    y.x = ((CASE == 30 ? v.x : r.x) > 0.f ? v.x : v.x * alpha) * scale;
    y.y = ((CASE == 30 ? v.y : r.y) > 0.f ? v.y : v.y * alpha) * scale;
    y.z = ((CASE == 30 ? v.z : r.z) > 0.f ? v.z : v.z * alpha) * scale;
    y.w = ((CASE == 30 ? v.w : r.w) > 0.f ? v.w : v.w * alpha) * scale;
    out[i] = y;
  }
}

template <typename T>
int fba_impl(const T* x, const T* bias, const T* refer, T* out, int64_t n, int64_t step_b,
             int64_t size_b, int act, int grad, T alpha, T scale, void* stream) {
  BPK_REQUIRE(n >= 0, "fused_bias_act: negative size");
  BPK_REQUIRE(act == 1 || act == 3, "fused_bias_act: act must be 1 (linear) or 3 (lrelu), got %d",
              act);
  BPK_REQUIRE(grad >= 0 && grad <= 2, "fused_bias_act: grad must be 0, 1 or 2");
  if (bias) BPK_REQUIRE(step_b > 0 && size_b > 0, "fused_bias_act: bad bias geometry");
  if (n == 0) return BPK_OK;
  const bool al = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(refer) |
                    reinterpret_cast<uintptr_t>(out)) & 15) == 0;
  if (sizeof(T) == 4 && !bias && act == 3 && (grad == 0 || (grad == 1 && refer)) && n % 4 == 0 &&
      al) {
    const int64_t n4 = n / 4;
    const int64_t blocks = std::min<int64_t>(bpk::ceil_div(n4, 256), 256 * 16);
    const float4* x4 = reinterpret_cast<const float4*>(x);
    const float4* r4 = reinterpret_cast<const float4*>(refer);
    float4* o4 = reinterpret_cast<float4*>(out);
    if (grad == 0)
      hipLaunchKernelGGL(lrelu4_kernel<30>, dim3((unsigned)blocks), dim3(256), 0,
                         bpk::as_stream(stream), x4, r4, o4, n4, (float)alpha, (float)scale);
    else
      hipLaunchKernelGGL(lrelu4_kernel<31>, dim3((unsigned)blocks), dim3(256), 0,
                         bpk::as_stream(stream), x4, r4, o4, n4, (float)alpha, (float)scale);
    BPK_LAUNCH_CHECK("fused_bias_act");
    return BPK_OK;
  }
  const int64_t blocks = std::min<int64_t>(bpk::ceil_div(n, 256), 256 * 16);
  hipLaunchKernelGGL(fused_bias_act_kernel<T>, dim3((unsigned)blocks), dim3(256), 0,
                     bpk::as_stream(stream), x, bias, refer, out, n, step_b, size_b, act, grad,
                     alpha, scale);
  BPK_LAUNCH_CHECK("fused_bias_act");
  return BPK_OK;
}

// out = (x + (h + bias[c])) / div over [N, C, HW]; float4 along HW when possible
template <int W>
__global__ __launch_bounds__(256) void residual_rescale_kernel(const float* __restrict__ x,
                                                               const float* __restrict__ h,
                                                               const float* __restrict__ bias,
                                                               float* __restrict__ out,
                                                               int64_t n, int C, int64_t HW,
                                                               float div) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * W; i < n; i += stride * W) {
    const float b = bias ? bias[(i / HW) % C] : 0.f;
    if constexpr (W == 4) {
      const float4 a = *reinterpret_cast<const float4*>(x + i);
      const float4 c = *reinterpret_cast<const float4*>(h + i);
      *reinterpret_cast<float4*>(out + i) =
          make_float4((a.x + (c.x + b)) / div, (a.y + (c.y + b)) / div, (a.z + (c.z + b)) / div,
                      (a.w + (c.w + b)) / div);
    } else {
      out[i] = (x[i] + (h[i] + b)) / div;
    }
  }
}

}  // namespace

extern "C" int bpk_fused_bias_act_f32(const float* x, const float* bias, const float* refer,
                                      float* out, int64_t n, int64_t step_b, int64_t size_b,
                                      int act, int grad, float alpha, float scale, void* stream) {
  return fba_impl<float>(x, bias, refer, out, n, step_b, size_b, act, grad, alpha, scale, stream);
}

extern "C" int bpk_fused_bias_act_f64(const double* x, const double* bias, const double* refer,
                                      double* out, int64_t n, int64_t step_b, int64_t size_b,
                                      int act, int grad, double alpha, double scale,
                                      void* stream) {
  return fba_impl<double>(x, bias, refer, out, n, step_b, size_b, act, grad, alpha, scale, stream);
}

extern "C" int bpk_residual_rescale_f32(const float* x, const float* h, const float* bias,
                                        float* out, int N, int C, int64_t HW, float div,
                                        void* stream) {
  BPK_REQUIRE(N >= 0 && C > 0 && HW > 0, "residual_rescale: bad shape");
  const int64_t n = (int64_t)N * C * HW;
  if (n == 0) return BPK_OK;
  hipStream_t st = bpk::as_stream(stream);
  const bool vec = HW % 4 == 0 && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(h) |
                                    reinterpret_cast<uintptr_t>(out)) & 15) == 0;
  const int W = vec ? 4 : 1;
  const int64_t blocks = std::min<int64_t>(bpk::ceil_div(n / W, 256), 256 * 32);
  if (vec)
    hipLaunchKernelGGL(residual_rescale_kernel<4>, dim3((unsigned)blocks), dim3(256), 0, st, x, h,
                       bias, out, n, C, HW, div);
  else
    hipLaunchKernelGGL(residual_rescale_kernel<1>, dim3((unsigned)blocks), dim3(256), 0, st, x, h,
                       bias, out, n, C, HW, div);
  BPK_LAUNCH_CHECK("residual_rescale");
  return BPK_OK;
}
