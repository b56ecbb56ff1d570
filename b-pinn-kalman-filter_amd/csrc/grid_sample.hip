// Bilinear 2-D grid_sample forward / backward / double-backward for gfx950.
//
// Forward and backward follow ATen's grid_sampler_2d semantics that the
// reference calls (op/grid_sample.py:39-60: F.grid_sample and
// aten::grid_sampler_2d_backward, interpolation = bilinear, padding zeros or
// border).  The double-backward is the reference's custom kernel
// (op/grid_sample_kernel.cu:27-210): given (g2_input, g2_grid) -- the incoming
// gradients w.r.t. the first backward's outputs -- it produces the gradients
// w.r.t. (grad_output, input, grid).  This is what makes the PINN residual's
// second derivatives possible (pinn_kalman/pinn.py:89-92).
//
// Forward: one thread per output location (n, h, w) looping over channels; backward and
// double backward: each location's channels split over S threads (see gs_bwd); grad_input
// accumulation uses hardware float atomics.
#include "bpk_common.h"

#include <algorithm>
#include <cstdlib>

namespace {

template <typename T>
__device__ inline T unnormalize(T coord, int size, bool align, T* mult) {
  if (align) {
    *mult = T(size - 1) / T(2);
    return ((coord + T(1)) / T(2)) * T(size - 1);
  }
  *mult = T(size) / T(2);
  return ((coord + T(1)) * T(size) - T(1)) / T(2);
}

// ATen clip_coordinates_set_grad: borders count as out of range for the grad
template <typename T>
__device__ inline T clip_set_grad(T in, int size, T* g) {
  if (in <= T(0)) {
    *g = T(0);
    return T(0);
  }
  const T mx = T(size - 1);
  if (in >= mx) {
    *g = T(0);
    return mx;
  }
  *g = T(1);
  return in;
}

template <typename T>
__device__ inline T source_index_set_grad(T coord, int size, int padding, bool align, T* gmult) {
  T m;
  coord = unnormalize(coord, size, align, &m);
  if (padding == 1) {  // border
    T gc;
    coord = clip_set_grad(coord, size, &gc);
    m = m * gc;
  }
  *gmult = m;
  return coord;
}

__device__ inline bool inb(int y, int x, int H, int W) { return y >= 0 && y < H && x >= 0 && x < W; }

template <typename T>
struct Corners {
  T ix, iy;
  int ix_nw, iy_nw, ix_ne, iy_ne, ix_sw, iy_sw, ix_se, iy_se;
  T nw, ne, sw, se;
  T gix_mult, giy_mult;
};

template <typename T>
__device__ inline Corners<T> corners(T gx, T gy, int H, int W, int padding, bool align) {
  Corners<T> c;
  c.ix = source_index_set_grad(gx, W, padding, align, &c.gix_mult);
  c.iy = source_index_set_grad(gy, H, padding, align, &c.giy_mult);
  c.ix_nw = (int)floor(c.ix);
  c.iy_nw = (int)floor(c.iy);
  c.ix_ne = c.ix_nw + 1;
  c.iy_ne = c.iy_nw;
  c.ix_sw = c.ix_nw;
  c.iy_sw = c.iy_nw + 1;
  c.ix_se = c.ix_nw + 1;
  c.iy_se = c.iy_nw + 1;
  c.nw = (c.ix_se - c.ix) * (c.iy_se - c.iy);
  c.ne = (c.ix - c.ix_sw) * (c.iy_sw - c.iy);
  c.sw = (c.ix_ne - c.ix) * (c.iy - c.iy_ne);
  c.se = (c.ix - c.ix_nw) * (c.iy - c.iy_nw);
  return c;
}

template <typename T>
__global__ __launch_bounds__(256) void gs_fwd(const T* __restrict__ inp, const T* __restrict__ grid,
                                              T* __restrict__ out, int N, int C, int H, int W,
                                              int Ho, int Wo, int padding, int align) {
  const int64_t total = (int64_t)N * Ho * Wo;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int w = (int)(idx % Wo);
    const int h = (int)((idx / Wo) % Ho);
    const int64_t n = idx / ((int64_t)Ho * Wo);
    const T gx = grid[idx * 2], gy = grid[idx * 2 + 1];
    const Corners<T> q = corners(gx, gy, H, W, padding, align != 0);
    const T* ip = inp + n * C * H * W;
    T* op = out + n * C * Ho * Wo + (int64_t)h * Wo + w;
    for (int c = 0; c < C; ++c, ip += (int64_t)H * W, op += (int64_t)Ho * Wo) {
      T acc = T(0);
      if (inb(q.iy_nw, q.ix_nw, H, W)) acc += ip[q.iy_nw * W + q.ix_nw] * q.nw;
      if (inb(q.iy_ne, q.ix_ne, H, W)) acc += ip[q.iy_ne * W + q.ix_ne] * q.ne;
      if (inb(q.iy_sw, q.ix_sw, H, W)) acc += ip[q.iy_sw * W + q.ix_sw] * q.sw;
      if (inb(q.iy_se, q.ix_se, H, W)) acc += ip[q.iy_se * W + q.ix_se] * q.se;
      *op = acc;
    }
  }
}

template <typename T>
__device__ inline void safe_add(T* base, int y, int x, int H, int W, T v) {
  if (inb(y, x, H, W)) atomicAdd(base + (int64_t)y * W + x, v);
}

// Backward: a block is P = 256 / S output locations x S channel slices (thread (p, s) runs
// channels s, s + S, ...): S x the parallelism of one thread per location -- the PINN
// warps [64, 16..128, 2..32, 2..32] feature maps, where a per-location channel loop of
// atomics left the chip latency-bound (186 us per call).  grad_grid's channel sum is
// combined over the slices in LDS in a fixed order.
template <typename T, int S>
__global__ __launch_bounds__(256) void gs_bwd(const T* __restrict__ gout,
                                              const T* __restrict__ inp,
                                              const T* __restrict__ grid, T* grad_inp,
                                              T* __restrict__ grad_grid, int N, int C, int H, int W,
                                              int Ho, int Wo, int padding, int align) {
  constexpr int P = 256 / S;
  __shared__ T red[2][S][P];
  const int lp = threadIdx.x % P, sl = threadIdx.x / P;
  const int64_t total = (int64_t)N * Ho * Wo;
  const int64_t idx = (int64_t)blockIdx.x * P + lp;
  const bool valid = idx < total;
  T gix = T(0), giy = T(0);
  Corners<T> q{};
  if (valid) {
    const int w = (int)(idx % Wo);
    const int h = (int)((idx / Wo) % Ho);
    const int64_t n = idx / ((int64_t)Ho * Wo);
    const T gx = grid[idx * 2], gy = grid[idx * 2 + 1];
    q = corners(gx, gy, H, W, padding, align != 0);
    const int64_t hw = (int64_t)H * W, howo = (int64_t)Ho * Wo;
    const T* ip = inp + n * C * hw + sl * hw;
    T* gp = grad_inp ? grad_inp + n * C * hw + sl * hw : nullptr;
    const T* go = gout + n * C * howo + (int64_t)h * Wo + w + sl * howo;
    for (int c = sl; c < C; c += S, ip += S * hw, go += S * howo) {
      const T g = *go;
      if (gp) {
        T* gpc = gp + (int64_t)(c - sl) * hw;
        safe_add(gpc, q.iy_nw, q.ix_nw, H, W, q.nw * g);
        safe_add(gpc, q.iy_ne, q.ix_ne, H, W, q.ne * g);
        safe_add(gpc, q.iy_sw, q.ix_sw, H, W, q.sw * g);
        safe_add(gpc, q.iy_se, q.ix_se, H, W, q.se * g);
      }
      if (grad_grid) {
        if (inb(q.iy_nw, q.ix_nw, H, W)) {
          const T v = ip[q.iy_nw * W + q.ix_nw];
          gix -= v * (q.iy_se - q.iy) * g;
          giy -= v * (q.ix_se - q.ix) * g;
        }
        if (inb(q.iy_ne, q.ix_ne, H, W)) {
          const T v = ip[q.iy_ne * W + q.ix_ne];
          gix += v * (q.iy_sw - q.iy) * g;
          giy -= v * (q.ix - q.ix_sw) * g;
        }
        if (inb(q.iy_sw, q.ix_sw, H, W)) {
          const T v = ip[q.iy_sw * W + q.ix_sw];
          gix -= v * (q.iy - q.iy_ne) * g;
          giy += v * (q.ix_ne - q.ix) * g;
        }
        if (inb(q.iy_se, q.ix_se, H, W)) {
          const T v = ip[q.iy_se * W + q.ix_se];
          gix += v * (q.iy - q.iy_nw) * g;
          giy += v * (q.ix - q.ix_nw) * g;
        }
      }
    }
  }
  if (!grad_grid) return;
  if (S > 1) {
    red[0][sl][lp] = gix;
    red[1][sl][lp] = giy;
    __syncthreads();
    if (sl != 0) return;
#pragma unroll
    for (int k = 1; k < S; ++k) {
      gix += red[0][k][lp];
      giy += red[1][k][lp];
    }
  }
  if (valid) {
    grad_grid[idx * 2] = q.gix_mult * gix;
    grad_grid[idx * 2 + 1] = q.giy_mult * giy;
  }
}

// op/grid_sample_kernel.cu:27-210; P output locations x S channel slices per block as gs_bwd
template <typename T, int S>
__global__ __launch_bounds__(256) void gs_grad2(
    const T* __restrict__ g2_inp, const T* __restrict__ g2_grid, const T* __restrict__ gout,
    const T* __restrict__ inp, const T* __restrict__ grid, T* __restrict__ gg_out, T* grad_inp,
    T* __restrict__ grad_grid, int N, int C, int H, int W, int Ho, int Wo, int padding,
    int align) {
  constexpr int P = 256 / S;
  __shared__ T red[2][S][P];
  const int lp = threadIdx.x % P, sl = threadIdx.x / P;
  const int64_t total = (int64_t)N * Ho * Wo;
  const int64_t idx = (int64_t)blockIdx.x * P + lp;
  const bool valid = idx < total;
  T gix = T(0), giy = T(0);
  Corners<T> q{};
  if (valid) {
    const int w = (int)(idx % Wo);
    const int h = (int)((idx / Wo) % Ho);
    const int64_t n = idx / ((int64_t)Ho * Wo);
    const T gx = grid[idx * 2], gy = grid[idx * 2 + 1];
    q = corners(gx, gy, H, W, padding, align != 0);
    // a NULL g2_grid / g2_inp is an all-zero incoming gradient (autograd passes None for an
    // output nothing depends on; materialising zeros cost a fill launch and a read)
    const T dx = g2_grid ? g2_grid[idx * 2] * q.gix_mult : T(0);
    const T dy = g2_grid ? g2_grid[idx * 2 + 1] * q.giy_mult : T(0);
    const T* ip = inp + n * C * H * W;
    const T* g2p = g2_inp ? g2_inp + n * C * H * W : nullptr;
    T* gip = grad_inp + n * C * H * W;
    const int64_t oofs = n * C * Ho * Wo + (int64_t)h * Wo + w;
    const bool b_nw = inb(q.iy_nw, q.ix_nw, H, W), b_ne = inb(q.iy_ne, q.ix_ne, H, W),
               b_sw = inb(q.iy_sw, q.ix_sw, H, W), b_se = inb(q.iy_se, q.ix_se, H, W);
    const T nw_tmp = -dx * (q.iy_se - q.iy) - dy * (q.ix_se - q.ix);
    const T ne_tmp = +dx * (q.iy_sw - q.iy) - dy * (q.ix - q.ix_sw);
    const T sw_tmp = -dx * (q.iy - q.iy_ne) + dy * (q.ix_ne - q.ix);
    const T se_tmp = +dx * (q.iy - q.iy_nw) + dy * (q.ix - q.ix_nw);
    for (int c = sl; c < C; c += S) {
      const int64_t pc = (int64_t)c * H * W;
      const T nw_v = b_nw ? ip[pc + q.iy_nw * W + q.ix_nw] : T(0);
      const T ne_v = b_ne ? ip[pc + q.iy_ne * W + q.ix_ne] : T(0);
      const T sw_v = b_sw ? ip[pc + q.iy_sw * W + q.ix_sw] : T(0);
      const T se_v = b_se ? ip[pc + q.iy_se * W + q.ix_se] : T(0);
      const T g2_nw = g2p && b_nw ? g2p[pc + q.iy_nw * W + q.ix_nw] : T(0);
      const T g2_ne = g2p && b_ne ? g2p[pc + q.iy_ne * W + q.ix_ne] : T(0);
      const T g2_sw = g2p && b_sw ? g2p[pc + q.iy_sw * W + q.ix_sw] : T(0);
      const T g2_se = g2p && b_se ? g2p[pc + q.iy_se * W + q.ix_se] : T(0);
      T ggo = T(0);
      ggo += g2_nw * q.nw + g2_ne * q.ne + g2_sw * q.sw + g2_se * q.se;
      ggo += nw_v * nw_tmp + ne_tmp * ne_v + sw_tmp * sw_v + se_tmp * se_v;
      gg_out[oofs + (int64_t)c * Ho * Wo] = ggo;
      const T g = gout[oofs + (int64_t)c * Ho * Wo];
      T* gic = gip + pc;
      safe_add(gic, q.iy_nw, q.ix_nw, H, W, nw_tmp * g);
      safe_add(gic, q.iy_ne, q.ix_ne, H, W, ne_tmp * g);
      safe_add(gic, q.iy_sw, q.ix_sw, H, W, sw_tmp * g);
      safe_add(gic, q.iy_se, q.ix_se, H, W, se_tmp * g);
      const T dxy = nw_v - ne_v - sw_v + se_v;
      gix += g * (-g2_nw * (q.iy_se - q.iy) + g2_ne * (q.iy_sw - q.iy) - g2_sw * (q.iy - q.iy_ne) +
                  g2_se * (q.iy - q.iy_nw));
      gix += g * dy * dxy;
      giy += g * (-g2_nw * (q.ix_se - q.ix) - g2_ne * (q.ix - q.ix_sw) + g2_sw * (q.ix_ne - q.ix) +
                  g2_se * (q.ix - q.ix_nw));
      giy += g * dx * dxy;
    }
  }
  if (S > 1) {
    red[0][sl][lp] = gix;
    red[1][sl][lp] = giy;
    __syncthreads();
    if (sl != 0) return;
#pragma unroll
    for (int k = 1; k < S; ++k) {
      gix += red[0][k][lp];
      giy += red[1][k][lp];
    }
  }
  if (valid) {
    grad_grid[idx * 2] = gix * q.gix_mult;
    grad_grid[idx * 2 + 1] = giy * q.giy_mult;
  }
}

// channel slices per block: S x the threads of one-per-location where C allows (one thread
// per location took 186 us vs ~25 us per call on the PINN shapes, round 2)
inline int slices_for(int C) { return C >= 16 ? 8 : (C >= 4 ? 4 : 1); }

unsigned blocks_for(int64_t total) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(bpk::ceil_div(total, 256), 256 * 32));
}

#define GS_CHECK()                                                                            \
  BPK_REQUIRE(N >= 0 && C >= 0 && H_in > 0 && W_in > 0 && H_out >= 0 && W_out >= 0,           \
              "grid_sample: bad shape");                                                      \
  BPK_REQUIRE(padding_mode == 0 || padding_mode == 1,                                         \
              "grid_sample: padding_mode must be 0 (zeros) or 1 (border), got %d", padding_mode)

template <typename T>
int fwd_impl(const T* input, const T* grid, T* out, int N, int C, int H_in, int W_in, int H_out,
             int W_out, int padding_mode, int align_corners, void* stream) {
  GS_CHECK();
  const int64_t total = (int64_t)N * H_out * W_out;
  if (total == 0 || C == 0) return BPK_OK;
  hipLaunchKernelGGL(gs_fwd<T>, dim3(blocks_for(total)), dim3(256), 0, bpk::as_stream(stream),
                     input, grid, out, N, C, H_in, W_in, H_out, W_out, padding_mode, align_corners);
  BPK_LAUNCH_CHECK("grid_sample2d_fwd");
  return BPK_OK;
}

template <typename T>
int bwd_impl(const T* gout, const T* input, const T* grid, T* gin, T* ggrid, int N, int C,
             int H_in, int W_in, int H_out, int W_out, int padding_mode, int align_corners,
             void* stream) {
  GS_CHECK();
  const int64_t total = (int64_t)N * H_out * W_out;
  if (total == 0) return BPK_OK;
  const int S = slices_for(C);
  const unsigned blocks = (unsigned)bpk::ceil_div(total, 256 / S);
  BPK_REQUIRE(bpk::ceil_div(total, 256 / S) < (1ll << 31), "grid_sample2d_bwd: too many locations");
  auto k = S == 8 ? gs_bwd<T, 8> : (S == 4 ? gs_bwd<T, 4> : gs_bwd<T, 1>);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, bpk::as_stream(stream), gout, input, grid,
                     gin, ggrid, N, C, H_in, W_in, H_out, W_out, padding_mode, align_corners);
  BPK_LAUNCH_CHECK("grid_sample2d_bwd");
  return BPK_OK;
}

template <typename T>
int grad2_impl(const T* g2i, const T* g2g, const T* gout, const T* input, const T* grid, T* ggo,
               T* gin, T* ggrid, int N, int C, int H_in, int W_in, int H_out, int W_out,
               int padding_mode, int align_corners, void* stream) {
  GS_CHECK();
  BPK_REQUIRE(ggo && gin && ggrid, "grid_sample2d_grad2: all outputs required");
  const int64_t total = (int64_t)N * H_out * W_out;
  if (total == 0) return BPK_OK;
  const int S = slices_for(C);
  const unsigned blocks = (unsigned)bpk::ceil_div(total, 256 / S);
  BPK_REQUIRE(bpk::ceil_div(total, 256 / S) < (1ll << 31), "grid_sample2d_grad2: too many locations");
  auto k = S == 8 ? gs_grad2<T, 8> : (S == 4 ? gs_grad2<T, 4> : gs_grad2<T, 1>);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, bpk::as_stream(stream), g2i, g2g, gout, input,
                     grid, ggo, gin, ggrid, N, C, H_in, W_in, H_out, W_out, padding_mode,
                     align_corners);
  BPK_LAUNCH_CHECK("grid_sample2d_grad2");
  return BPK_OK;
}

}  // namespace

extern "C" {
int bpk_grid_sample2d_fwd_f32(const float* input, const float* grid, float* out, int N, int C,
                              int H_in, int W_in, int H_out, int W_out, int padding_mode,
                              int align_corners, void* stream) {
  return fwd_impl(input, grid, out, N, C, H_in, W_in, H_out, W_out, padding_mode, align_corners,
                  stream);
}
int bpk_grid_sample2d_fwd_f64(const double* input, const double* grid, double* out, int N, int C,
                              int H_in, int W_in, int H_out, int W_out, int padding_mode,
                              int align_corners, void* stream) {
  return fwd_impl(input, grid, out, N, C, H_in, W_in, H_out, W_out, padding_mode, align_corners,
                  stream);
}
int bpk_grid_sample2d_bwd_f32(const float* grad_out, const float* input, const float* grid,
                              float* grad_input, float* grad_grid, int N, int C, int H_in,
                              int W_in, int H_out, int W_out, int padding_mode, int align_corners,
                              void* stream) {
  return bwd_impl(grad_out, input, grid, grad_input, grad_grid, N, C, H_in, W_in, H_out, W_out,
                  padding_mode, align_corners, stream);
}
int bpk_grid_sample2d_bwd_f64(const double* grad_out, const double* input, const double* grid,
                              double* grad_input, double* grad_grid, int N, int C, int H_in,
                              int W_in, int H_out, int W_out, int padding_mode, int align_corners,
                              void* stream) {
  return bwd_impl(grad_out, input, grid, grad_input, grad_grid, N, C, H_in, W_in, H_out, W_out,
                  padding_mode, align_corners, stream);
}
int bpk_grid_sample2d_grad2_f32(const float* g2_input, const float* g2_grid,
                                const float* grad_out, const float* input, const float* grid,
                                float* grad_grad_out, float* grad_input, float* grad_grid, int N,
                                int C, int H_in, int W_in, int H_out, int W_out, int padding_mode,
                                int align_corners, void* stream) {
  return grad2_impl(g2_input, g2_grid, grad_out, input, grid, grad_grad_out, grad_input, grad_grid,
                    N, C, H_in, W_in, H_out, W_out, padding_mode, align_corners, stream);
}
int bpk_grid_sample2d_grad2_f64(const double* g2_input, const double* g2_grid,
                                const double* grad_out, const double* input, const double* grid,
                                double* grad_grad_out, double* grad_input, double* grad_grid,
                                int N, int C, int H_in, int W_in, int H_out, int W_out,
                                int padding_mode, int align_corners, void* stream) {
  return grad2_impl(g2_input, g2_grid, grad_out, input, grid, grad_grad_out, grad_input, grad_grid,
                    N, C, H_in, W_in, H_out, W_out, padding_mode, align_corners, stream);
}
}
