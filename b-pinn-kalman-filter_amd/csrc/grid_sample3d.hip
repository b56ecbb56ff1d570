// Trilinear 3-D grid_sample forward / backward / double-backward for gfx950.
//
// Forward and backward follow ATen's grid_sampler_3d (bilinear = trilinear, padding zeros
// or border) that the reference calls (op/grid_sample.py:79-113: F.grid_sample on 5-D
// tensors and aten::grid_sampler_3d_backward); the double-backward restates the
// reference's custom kernel (op/grid_sample_kernel.cu:212-533).  The eight corners are
// indexed c = 4 bz + 2 by + bx (bz: t/b = z0/z1, by: n/s = y0/y1, bx: w/e = x0/x1 in the
// reference's names); corner c's weight is Wx(bx) Wy(by) Wz(bz) with W(0) = (i0 + 1 - i),
// W(1) = (i - i0) and dW/di = -1 / +1 -- the reference's per-corner products, in its
// operation order (x * y) * z.
#include "bpk_common.h"

#include <algorithm>

namespace {

template <typename T>
__device__ inline T src_index(T coord, int size, int padding, bool align, T* gmult) {
  T m, c;
  if (align) {
    m = T(size - 1) / T(2);
    c = ((coord + T(1)) / T(2)) * T(size - 1);
  } else {
    m = T(size) / T(2);
    c = ((coord + T(1)) * T(size) - T(1)) / T(2);
  }
  if (padding == 1) {  // border: ATen clip_coordinates_set_grad
    if (c <= T(0)) {
      c = T(0);
      m = T(0);
    } else if (c >= T(size - 1)) {
      c = T(size - 1);
      m = T(0);
    }
  }
  *gmult = m;
  return c;
}

template <typename T>
struct Tri {
  int x0, y0, z0;
  T wx[2], wy[2], wz[2];  // W(0), W(1) per axis
  T gx, gy, gz;           // gradient multipliers
};

template <typename T>
__device__ inline Tri<T> tri(const T* g, int D, int H, int W, int padding, bool align) {
  Tri<T> t;
  const T ix = src_index(g[0], W, padding, align, &t.gx);
  const T iy = src_index(g[1], H, padding, align, &t.gy);
  const T iz = src_index(g[2], D, padding, align, &t.gz);
  t.x0 = (int)floor(ix);
  t.y0 = (int)floor(iy);
  t.z0 = (int)floor(iz);
  t.wx[0] = T(t.x0 + 1) - ix;
  t.wx[1] = ix - T(t.x0);
  t.wy[0] = T(t.y0 + 1) - iy;
  t.wy[1] = iy - T(t.y0);
  t.wz[0] = T(t.z0 + 1) - iz;
  t.wz[1] = iz - T(t.z0);
  return t;
}

__device__ inline bool inb3(int z, int y, int x, int D, int H, int W) {
  return z >= 0 && z < D && y >= 0 && y < H && x >= 0 && x < W;
}

#define CORNER(c) const int bx = (c) & 1, by = ((c) >> 1) & 1, bz = (c) >> 2; \
  const int zz = q.z0 + bz, yy = q.y0 + by, xx = q.x0 + bx;                        \
  const bool ok = inb3(zz, yy, xx, D, H, W);                                      \
  const int64_t off = ((int64_t)zz * H + yy) * W + xx;                             \
  const T sx = bx ? T(1) : T(-1), sy = by ? T(1) : T(-1), sz = bz ? T(1) : T(-1); \
  (void)sx; (void)sy; (void)sz

template <typename T>
__global__ __launch_bounds__(256) void gs3_fwd(const T* __restrict__ inp, const T* __restrict__ grid,
                                               T* __restrict__ out, int N, int C, int D, int H, int W,
                                               int Do, int Ho, int Wo, int padding, int align) {
  const int64_t so = (int64_t)Do * Ho * Wo, si = (int64_t)D * H * W;
  const int64_t total = (int64_t)N * so;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = idx / so, s = idx - n * so;
    const Tri<T> q = tri(grid + idx * 3, D, H, W, padding, align != 0);
    const T* ip = inp + n * C * si;
    T* op = out + n * C * so + s;
    for (int c = 0; c < C; ++c, ip += si, op += so) {
      T acc = T(0);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        CORNER(k);
        if (ok) acc += ip[off] * (q.wx[bx] * q.wy[by] * q.wz[bz]);
      }
      *op = acc;
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void gs3_bwd(const T* __restrict__ gout, const T* __restrict__ inp,
                                               const T* __restrict__ grid, T* grad_inp,
                                               T* __restrict__ grad_grid, int N, int C, int D, int H,
                                               int W, int Do, int Ho, int Wo, int padding, int align) {
  const int64_t so = (int64_t)Do * Ho * Wo, si = (int64_t)D * H * W;
  const int64_t total = (int64_t)N * so;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = idx / so, s = idx - n * so;
    const Tri<T> q = tri(grid + idx * 3, D, H, W, padding, align != 0);
    const T* ip = inp + n * C * si;
    const T* go = gout + n * C * so + s;
    T* gp = grad_inp ? grad_inp + n * C * si : nullptr;
    T gix = T(0), giy = T(0), giz = T(0);
    for (int c = 0; c < C; ++c, ip += si, go += so) {
      const T g = *go;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        CORNER(k);
        if (!ok) continue;
        if (gp) atomicAdd(gp + (int64_t)c * si + off, (q.wx[bx] * q.wy[by] * q.wz[bz]) * g);
        if (grad_grid) {
          const T v = ip[off];
          gix += sx * v * q.wy[by] * q.wz[bz] * g;
          giy += sy * v * q.wx[bx] * q.wz[bz] * g;
          giz += sz * v * q.wx[bx] * q.wy[by] * g;
        }
      }
    }
    if (grad_grid) {
      grad_grid[idx * 3] = q.gx * gix;
      grad_grid[idx * 3 + 1] = q.gy * giy;
      grad_grid[idx * 3 + 2] = q.gz * giz;
    }
  }
}

// op/grid_sample_kernel.cu:212-533
template <typename T>
__global__ __launch_bounds__(256) void gs3_grad2(
    const T* __restrict__ g2_inp, const T* __restrict__ g2_grid, const T* __restrict__ gout,
    const T* __restrict__ inp, const T* __restrict__ grid, T* __restrict__ gg_out, T* grad_inp,
    T* __restrict__ grad_grid, int N, int C, int D, int H, int W, int Do, int Ho, int Wo,
    int padding, int align) {
  const int64_t so = (int64_t)Do * Ho * Wo, si = (int64_t)D * H * W;
  const int64_t total = (int64_t)N * so;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = idx / so, s = idx - n * so;
    const Tri<T> q = tri(grid + idx * 3, D, H, W, padding, align != 0);
    const T dx = g2_grid[idx * 3] * q.gx, dy = g2_grid[idx * 3 + 1] * q.gy,
            dz = g2_grid[idx * 3 + 2] * q.gz;
    T tmp[8];  // dx dw/dix + dy dw/diy + dz dw/diz per corner
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      CORNER(k);
      (void)ok;
      (void)off;
      tmp[k] = sx * dx * q.wy[by] * q.wz[bz] + sy * dy * q.wx[bx] * q.wz[bz] +
               sz * dz * q.wx[bx] * q.wy[by];
    }
    const T* ip = inp + n * C * si;
    const T* g2p = g2_inp + n * C * si;
    T* gip = grad_inp + n * C * si;
    const int64_t oofs = n * C * so + s;
    T gix = T(0), giy = T(0), giz = T(0);
    for (int c = 0; c < C; ++c) {
      const int64_t pc = (int64_t)c * si;
      const T g = gout[oofs + c * so];
      T ggo = T(0), dxy = T(0), dxz = T(0), dyz = T(0), ax = T(0), ay = T(0), az = T(0);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        CORNER(k);
        if (!ok) continue;
        const T v = ip[pc + off], g2 = g2p[pc + off];
        ggo += g2 * (q.wx[bx] * q.wy[by] * q.wz[bz]) + v * tmp[k];
        atomicAdd(gip + pc + off, tmp[k] * g);
        dxy += sx * sy * v * q.wz[bz];
        dxz += sx * sz * v * q.wy[by];
        dyz += sy * sz * v * q.wx[bx];
        ax += sx * g2 * q.wy[by] * q.wz[bz];
        ay += sy * g2 * q.wx[bx] * q.wz[bz];
        az += sz * g2 * q.wx[bx] * q.wy[by];
      }
      gg_out[oofs + c * so] = ggo;
      gix += g * ax + g * (dz * dxz + dy * dxy);
      giy += g * ay + g * (dx * dxy + dz * dyz);
      giz += g * az + g * (dx * dxz + dy * dyz);
    }
    grad_grid[idx * 3] = gix * q.gx;
    grad_grid[idx * 3 + 1] = giy * q.gy;
    grad_grid[idx * 3 + 2] = giz * q.gz;
  }
}
#undef CORNER

unsigned blocks3(int64_t total) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(bpk::ceil_div(total, 256), 256 * 32));
}

#define GS3_CHECK()                                                                                   \
  BPK_REQUIRE(N >= 0 && C >= 0 && D > 0 && H > 0 && W > 0 && Do >= 0 && Ho >= 0 && Wo >= 0,          \
              "grid_sample3d: bad shape");                                                           \
  BPK_REQUIRE(padding_mode == 0 || padding_mode == 1,                                                \
              "grid_sample3d: padding_mode must be 0 (zeros) or 1 (border), got %d", padding_mode)

template <typename T>
int fwd3(const T* input, const T* grid, T* out, int N, int C, int D, int H, int W, int Do, int Ho,
         int Wo, int padding_mode, int align_corners, void* stream) {
  GS3_CHECK();
  const int64_t total = (int64_t)N * Do * Ho * Wo;
  if (total == 0 || C == 0) return BPK_OK;
  hipLaunchKernelGGL(gs3_fwd<T>, dim3(blocks3(total)), dim3(256), 0, bpk::as_stream(stream), input,
                     grid, out, N, C, D, H, W, Do, Ho, Wo, padding_mode, align_corners);
  BPK_LAUNCH_CHECK("grid_sample3d_fwd");
  return BPK_OK;
}

template <typename T>
int bwd3(const T* gout, const T* input, const T* grid, T* gin, T* ggrid, int N, int C, int D, int H,
         int W, int Do, int Ho, int Wo, int padding_mode, int align_corners, void* stream) {
  GS3_CHECK();
  const int64_t total = (int64_t)N * Do * Ho * Wo;
  if (total == 0) return BPK_OK;
  hipLaunchKernelGGL(gs3_bwd<T>, dim3(blocks3(total)), dim3(256), 0, bpk::as_stream(stream), gout,
                     input, grid, gin, ggrid, N, C, D, H, W, Do, Ho, Wo, padding_mode, align_corners);
  BPK_LAUNCH_CHECK("grid_sample3d_bwd");
  return BPK_OK;
}

template <typename T>
int grad2_3(const T* g2i, const T* g2g, const T* gout, const T* input, const T* grid, T* ggo,
            T* gin, T* ggrid, int N, int C, int D, int H, int W, int Do, int Ho, int Wo,
            int padding_mode, int align_corners, void* stream) {
  GS3_CHECK();
  BPK_REQUIRE(ggo && gin && ggrid, "grid_sample3d_grad2: all outputs required");
  const int64_t total = (int64_t)N * Do * Ho * Wo;
  if (total == 0) return BPK_OK;
  hipLaunchKernelGGL(gs3_grad2<T>, dim3(blocks3(total)), dim3(256), 0, bpk::as_stream(stream), g2i,
                     g2g, gout, input, grid, ggo, gin, ggrid, N, C, D, H, W, Do, Ho, Wo,
                     padding_mode, align_corners);
  BPK_LAUNCH_CHECK("grid_sample3d_grad2");
  return BPK_OK;
}

}  // namespace

#define GS3_EXPORTS(T, S)                                                                             \
  extern "C" int bpk_grid_sample3d_fwd_##S(const T* input, const T* grid, T* out, int N, int C,      \
                                            int D, int H, int W, int Do, int Ho, int Wo,              \
                                            int padding_mode, int align_corners, void* stream) {     \
    return fwd3(input, grid, out, N, C, D, H, W, Do, Ho, Wo, padding_mode, align_corners, stream);  \
  }                                                                                                  \
  extern "C" int bpk_grid_sample3d_bwd_##S(const T* grad_out, const T* input, const T* grid,        \
                                            T* grad_input, T* grad_grid, int N, int C, int D, int H, \
                                            int W, int Do, int Ho, int Wo, int padding_mode,         \
                                            int align_corners, void* stream) {                       \
    return bwd3(grad_out, input, grid, grad_input, grad_grid, N, C, D, H, W, Do, Ho, Wo,            \
                padding_mode, align_corners, stream);                                               \
  }                                                                                                  \
  extern "C" int bpk_grid_sample3d_grad2_##S(const T* g2_input, const T* g2_grid, const T* grad_out, \
                                              const T* input, const T* grid, T* grad_grad_out,       \
                                              T* grad_input, T* grad_grid, int N, int C, int D,      \
                                              int H, int W, int Do, int Ho, int Wo,                  \
                                              int padding_mode, int align_corners, void* stream) {   \
    return grad2_3(g2_input, g2_grid, grad_out, input, grid, grad_grad_out, grad_input, grad_grid,  \
                   N, C, D, H, W, Do, Ho, Wo, padding_mode, align_corners, stream);                 \
  }

GS3_EXPORTS(float, f32)
GS3_EXPORTS(double, f64)
