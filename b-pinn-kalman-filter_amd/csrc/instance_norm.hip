// InstanceNorm2d (affine=False) + ELU(alpha=1), twice differentiable, for PressureNet's
// ResidualBlocks (reference models/layers.py:438-491: conv(act(normalize(x))) with
// normalization=nn.InstanceNorm2d, act=nn.ELU()).
//
// The PINN residual differentiates PressureNet w.r.t. its inputs with create_graph=True and
// then backpropagates through that derivative, so each norm+act runs forward, backward and
// double backward every step.  On aten that is batch_norm statistics / transform, the ELU,
// native_batch_norm_backward, elu_backward and a composite batchnorm double backward of
// ~25 small kernels per norm; here it is one kernel per order.
//
// Per plane p = (n, c) of M = H*W elements: mu = mean(x), r = 1 / sqrt(var + eps) (biased
// variance), z = (x - mu) r, y = e(z) with e = ELU (act = 1) or identity (act = 0).
//   backward     g = dy e'(z);  dx = r (g - mean(g) - z mean(g z))
//   double bwd   for v = dL/d(dx):  w = r (v - mean(v) - z mean(v z))
//                d/d(dy) = w e'(z)
//                q = dy e''(z) w - r (g mean(v z) + v mean(g z))
//                S = mean(g v) - mean(g) mean(v) - mean(g z) mean(v z)
//                d/dx = r (q - mean(q) - z mean(q z)) - r^2 z S
// (derivation: DESIGN.md section 4b; e'(z) = exp(z), e''(z) = exp(z) for z <= 0, else 1, 0,
// the branch aten's elu_backward takes at z = 0.)
//
// Small planes (<= 256 elements) and very large ones: one wave per plane (4 planes per
// 256-thread block), reductions lane-strided sums in a fixed order followed by a butterfly;
// 257..4096 elements: one workgroup per plane (below).  Deterministic either way.
#include "bpk_common.h"

#include <cmath>

namespace {

constexpr int kWaves = 4;

template <typename T>
__device__ inline T wsum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T>
__device__ inline T act_f(T z, int act) {
  if (!act) return z;
  return z <= T(0) ? expm1(z) : z;
}
template <typename T>
__device__ inline T act_d1(T z, int act) {
  if (!act) return T(1);
  return z <= T(0) ? exp(z) : T(1);
}
template <typename T>
__device__ inline T act_d2(T z, int act) {
  if (!act) return T(0);
  return z <= T(0) ? exp(z) : T(0);
}

template <typename T>
__global__ __launch_bounds__(256) void in_fwd(const T* __restrict__ x, T* __restrict__ y,
                                              T* __restrict__ mean, T* __restrict__ rstd,
                                              int64_t planes, int64_t M, T eps, int act) {
  const int lane = threadIdx.x & 63;
  const int64_t p = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (p >= planes) return;
  const T* xp = x + p * M;
  T s = T(0);
  for (int64_t i = lane; i < M; i += 64) s += xp[i];
  const T mu = wsum(s) / T(M);
  T s2 = T(0);
  for (int64_t i = lane; i < M; i += 64) {
    const T d = xp[i] - mu;
    s2 += d * d;
  }
  const T r = T(1) / sqrt(wsum(s2) / T(M) + eps);
  T* yp = y + p * M;
  for (int64_t i = lane; i < M; i += 64) yp[i] = act_f((xp[i] - mu) * r, act);
  if (lane == 0) {
    mean[p] = mu;
    rstd[p] = r;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void in_bwd(const T* __restrict__ dy, const T* __restrict__ x,
                                              const T* __restrict__ mean,
                                              const T* __restrict__ rstd, T* __restrict__ dx,
                                              int64_t planes, int64_t M, int act,
                                              const T* __restrict__ add) {
  const int lane = threadIdx.x & 63;
  const int64_t p = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (p >= planes) return;
  const T* xp = x + p * M;
  const T* dp = dy + p * M;
  const T mu = mean[p], r = rstd[p];
  T sg = T(0), sgz = T(0);
  for (int64_t i = lane; i < M; i += 64) {
    const T z = (xp[i] - mu) * r;
    const T g = dp[i] * act_d1(z, act);
    sg += g;
    sgz += g * z;
  }
  const T mg = wsum(sg) / T(M), mgz = wsum(sgz) / T(M);
  T* op = dx + p * M;
  for (int64_t i = lane; i < M; i += 64) {
    const T z = (xp[i] - mu) * r;
    const T g = dp[i] * act_d1(z, act);
    const T o = r * (g - mg - z * mgz);
    op[i] = add ? o + add[p * M + i] : o;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void in_bwd2(const T* __restrict__ v, const T* __restrict__ dy,
                                               const T* __restrict__ x,
                                               const T* __restrict__ mean,
                                               const T* __restrict__ rstd, T* __restrict__ gdy,
                                               T* __restrict__ gx, int64_t planes, int64_t M,
                                               int act) {
  const int lane = threadIdx.x & 63;
  const int64_t p = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (p >= planes) return;
  const T* xp = x + p * M;
  const T* dp = dy + p * M;
  const T* vp = v + p * M;
  const T mu = mean[p], r = rstd[p];
  // pass 1: mean(v), mean(v z), mean(g), mean(g z), mean(g v)
  T sv = T(0), svz = T(0), sg = T(0), sgz = T(0), sgv = T(0);
  for (int64_t i = lane; i < M; i += 64) {
    const T z = (xp[i] - mu) * r;
    const T g = dp[i] * act_d1(z, act);
    const T vi = vp[i];
    sv += vi;
    svz += vi * z;
    sg += g;
    sgz += g * z;
    sgv += g * vi;
  }
  const T inv = T(1) / T(M);
  const T mv = wsum(sv) * inv, mvz = wsum(svz) * inv, mg = wsum(sg) * inv;
  const T mgz = wsum(sgz) * inv, mgv = wsum(sgv) * inv;
  const T S = mgv - mg * mv - mgz * mvz;
  // pass 2: mean(q), mean(q z)  (only when d/dx is wanted)
  T mq = T(0), mqz = T(0);
  if (gx) {
    T sq = T(0), sqz = T(0);
    for (int64_t i = lane; i < M; i += 64) {
      const T z = (xp[i] - mu) * r;
      const T d1 = act_d1(z, act);
      const T g = dp[i] * d1;
      const T vi = vp[i];
      const T w = r * (vi - mv - z * mvz);
      const T q = dp[i] * act_d2(z, act) * w - r * (g * mvz + vi * mgz);
      sq += q;
      sqz += q * z;
    }
    mq = wsum(sq) * inv;
    mqz = wsum(sqz) * inv;
  }
  // pass 3: outputs
  for (int64_t i = lane; i < M; i += 64) {
    const T z = (xp[i] - mu) * r;
    const T d1 = act_d1(z, act);
    const T vi = vp[i];
    const T w = r * (vi - mv - z * mvz);
    if (gdy) gdy[p * M + i] = w * d1;
    if (gx) {
      const T g = dp[i] * d1;
      const T q = dp[i] * act_d2(z, act) * w - r * (g * mvz + vi * mgz);
      gx[p * M + i] = r * (q - mq - z * mqz) - r * r * z * S;
    }
  }
}

// Planes of 257..4096 elements (PressureNet at 32^2 and 64^2): one 256-thread workgroup per
// plane holding it in registers, so every pass after the first reads registers instead of
// re-reading HBM and the plane's loads are all in flight at once (the one-wave kernels above
// walk a 64^2 plane in 64 dependent steps per pass).  A thread owns V runs of W consecutive
// elements (W = 4: 16-byte accesses, fp32 planes of M % 4 == 0), run k at (thread + 256 k) W.
// Sums: per-thread in element order, wave butterfly, then the four wave sums in order
// (deterministic).
template <typename T>
__device__ inline T bsum(T v, T* sh) {
  v = wsum(v);
  __syncthreads();  // the previous sum's readers are done with sh
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  return ((sh[0] + sh[1]) + sh[2]) + sh[3];
}

template <typename T, int W>
__device__ inline void ld(const T* p, T* v) {
  static_assert(W == 1 || sizeof(T) == 4, "16-byte runs are fp32 only");
  if constexpr (W == 4) {
    const float4 q = *reinterpret_cast<const float4*>(p);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else {
    v[0] = *p;
  }
}
template <typename T, int W>
__device__ inline void st(T* p, const T* v) {
  if constexpr (W == 4)
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  else
    *p = v[0];
}

template <typename T, int V, int W>
__global__ __launch_bounds__(256) void in_fwd_blk(const T* __restrict__ x, T* __restrict__ y,
                                                  T* __restrict__ mean, T* __restrict__ rstd,
                                                  int64_t M, T eps, int act) {
  __shared__ T sh[4];
  const int64_t p = blockIdx.x;
  T xv[V][W];
  T s = T(0);
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t e = (threadIdx.x + 256 * (int64_t)k) * W;
    if (e < M) ld<T, W>(x + p * M + e, xv[k]);
    else
#pragma unroll
      for (int j = 0; j < W; ++j) xv[k][j] = T(0);
#pragma unroll
    for (int j = 0; j < W; ++j) s += xv[k][j];
  }
  const T mu = bsum(s, sh) / T(M);
  T s2 = T(0);
#pragma unroll
  for (int k = 0; k < V; ++k)
    if ((threadIdx.x + 256 * (int64_t)k) * W < M)
#pragma unroll
      for (int j = 0; j < W; ++j) {
        const T d = xv[k][j] - mu;
        s2 += d * d;
      }
  const T r = T(1) / sqrt(bsum(s2, sh) / T(M) + eps);
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t e = (threadIdx.x + 256 * (int64_t)k) * W;
    if (e >= M) continue;
    T o[W];
#pragma unroll
    for (int j = 0; j < W; ++j) o[j] = act_f((xv[k][j] - mu) * r, act);
    st<T, W>(y + p * M + e, o);
  }
  if (threadIdx.x == 0) {
    mean[p] = mu;
    rstd[p] = r;
  }
}

template <typename T, int V, int W>
__global__ __launch_bounds__(256) void in_bwd_blk(const T* __restrict__ dy, const T* __restrict__ x,
                                                  const T* __restrict__ mean,
                                                  const T* __restrict__ rstd, T* __restrict__ dx,
                                                  int64_t M, int act, const T* __restrict__ add) {
  __shared__ T sh[4];
  const int64_t p = blockIdx.x;
  const T mu = mean[p], r = rstd[p];
  T z[V][W], g[V][W];
  T sg = T(0), sgz = T(0);
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t e = (threadIdx.x + 256 * (int64_t)k) * W;
    T xv[W], dv[W];
    if (e < M) {
      ld<T, W>(x + p * M + e, xv);
      ld<T, W>(dy + p * M + e, dv);
    } else {
#pragma unroll
      for (int j = 0; j < W; ++j) xv[j] = dv[j] = T(0);
    }
#pragma unroll
    for (int j = 0; j < W; ++j) {
      z[k][j] = e < M ? (xv[j] - mu) * r : T(0);
      g[k][j] = e < M ? dv[j] * act_d1(z[k][j], act) : T(0);
      sg += g[k][j];
      sgz += g[k][j] * z[k][j];
    }
  }
  const T mg = bsum(sg, sh) / T(M);
  const T mgz = bsum(sgz, sh) / T(M);
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t e = (threadIdx.x + 256 * (int64_t)k) * W;
    if (e >= M) continue;
    T o[W];
#pragma unroll
    for (int j = 0; j < W; ++j) o[j] = r * (g[k][j] - mg - z[k][j] * mgz);
    if (add) {  // the identity-skip gradient of the residual block, added in the same pass
      T a[W];
      ld<T, W>(add + p * M + e, a);
#pragma unroll
      for (int j = 0; j < W; ++j) o[j] = o[j] + a[j];
    }
    st<T, W>(dx + p * M + e, o);
  }
}

template <typename T, int V, int W>
__global__ __launch_bounds__(256) void in_bwd2_blk(const T* __restrict__ v,
                                                   const T* __restrict__ dy,
                                                   const T* __restrict__ x,
                                                   const T* __restrict__ mean,
                                                   const T* __restrict__ rstd,
                                                   T* __restrict__ gdy, T* __restrict__ gx,
                                                   int64_t M, int act) {
  __shared__ T sh[4];
  const int64_t p = blockIdx.x;
  const T mu = mean[p], r = rstd[p];
  T z[V][W], d[V][W], vv[V][W];  // z, dy, v
  T sv = T(0), svz = T(0), sg = T(0), sgz = T(0), sgv = T(0);
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t e = (threadIdx.x + 256 * (int64_t)k) * W;
    T xv[W];
    if (e < M) {
      ld<T, W>(x + p * M + e, xv);
      ld<T, W>(dy + p * M + e, d[k]);
      ld<T, W>(v + p * M + e, vv[k]);
    } else {
#pragma unroll
      for (int j = 0; j < W; ++j) xv[j] = d[k][j] = vv[k][j] = T(0);
    }
#pragma unroll
    for (int j = 0; j < W; ++j) {
      z[k][j] = e < M ? (xv[j] - mu) * r : T(0);
      const T gj = d[k][j] * act_d1(z[k][j], act);
      sv += vv[k][j];
      svz += vv[k][j] * z[k][j];
      sg += gj;
      sgz += gj * z[k][j];
      sgv += gj * vv[k][j];
    }
  }
  const T inv = T(1) / T(M);
  const T mv = bsum(sv, sh) * inv, mvz = bsum(svz, sh) * inv, mg = bsum(sg, sh) * inv;
  const T mgz = bsum(sgz, sh) * inv, mgv = bsum(sgv, sh) * inv;
  const T S = mgv - mg * mv - mgz * mvz;
  T mq = T(0), mqz = T(0);
  if (gx) {
    T sq = T(0), sqz = T(0);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      if ((threadIdx.x + 256 * (int64_t)k) * W >= M) continue;
#pragma unroll
      for (int j = 0; j < W; ++j) {
        const T d1 = act_d1(z[k][j], act);
        const T gj = d[k][j] * d1;
        const T w = r * (vv[k][j] - mv - z[k][j] * mvz);
        const T q = d[k][j] * act_d2(z[k][j], act) * w - r * (gj * mvz + vv[k][j] * mgz);
        sq += q;
        sqz += q * z[k][j];
      }
    }
    mq = bsum(sq, sh) * inv;
    mqz = bsum(sqz, sh) * inv;
  }
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t e = (threadIdx.x + 256 * (int64_t)k) * W;
    if (e >= M) continue;
    T o1[W], o2[W];
#pragma unroll
    for (int j = 0; j < W; ++j) {
      const T d1 = act_d1(z[k][j], act);
      const T w = r * (vv[k][j] - mv - z[k][j] * mvz);
      o1[j] = w * d1;
      const T gj = d[k][j] * d1;
      const T q = d[k][j] * act_d2(z[k][j], act) * w - r * (gj * mvz + vv[k][j] * mgz);
      o2[j] = r * (q - mq - z[k][j] * mqz) - r * r * z[k][j] * S;
    }
    if (gdy) st<T, W>(gdy + p * M + e, o1);
    if (gx) st<T, W>(gx + p * M + e, o2);
  }
}

unsigned blocks_for(int64_t planes) { return (unsigned)bpk::ceil_div(planes, kWaves); }

// runs per thread of the workgroup-per-plane kernels (0: the one-wave kernels); W = 4 when
// the planes are whole 16-byte vectors
int blk_runs(int64_t M, int W) {
  if (M <= 256 || M > 256 * 16) return 0;
  const int64_t v = bpk::ceil_div(M, 256 * (int64_t)W);
  return v <= 1 ? 1 : v <= 2 ? 2 : v <= 4 ? 4 : v <= 8 ? 8 : 16;
}
template <typename T>
int blk_w(const void* a, const void* b, const void* c, int64_t M) {
  const auto al = [](const void* q) { return q == nullptr || (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  return (sizeof(T) == 4 && M % 4 == 0 && al(a) && al(b) && al(c)) ? 4 : 1;
}
#define IN_BLK_V(KERNEL, T, W, ...)                                                              \
  switch (blk_runs(M, W)) {                                                                      \
    case 1: hipLaunchKernelGGL((KERNEL<T, 1, W>), dim3((unsigned)planes), dim3(256), 0, st, __VA_ARGS__); break; \
    case 2: hipLaunchKernelGGL((KERNEL<T, 2, W>), dim3((unsigned)planes), dim3(256), 0, st, __VA_ARGS__); break; \
    case 4: hipLaunchKernelGGL((KERNEL<T, 4, W>), dim3((unsigned)planes), dim3(256), 0, st, __VA_ARGS__); break; \
    case 8: hipLaunchKernelGGL((KERNEL<T, 8, W>), dim3((unsigned)planes), dim3(256), 0, st, __VA_ARGS__); break; \
    default: hipLaunchKernelGGL((KERNEL<T, 16, W>), dim3((unsigned)planes), dim3(256), 0, st, __VA_ARGS__); break; \
  }
#define IN_BLK(KERNEL, T, WSEL, ...)                                                             \
  if constexpr (sizeof(T) == 4) {                                                                \
    if ((WSEL) == 4) {                                                                           \
      IN_BLK_V(KERNEL, T, 4, __VA_ARGS__)                                                        \
    } else {                                                                                     \
      IN_BLK_V(KERNEL, T, 1, __VA_ARGS__)                                                        \
    }                                                                                            \
  } else {                                                                                       \
    IN_BLK_V(KERNEL, T, 1, __VA_ARGS__)                                                          \
  }

#define IN_CHECK(what)                                                                   \
  BPK_REQUIRE(planes >= 0 && M > 0, "%s: bad geometry planes=%lld M=%lld", what,         \
              (long long)planes, (long long)M);                                          \
  BPK_REQUIRE(act == 0 || act == 1, "%s: act must be 0 (none) or 1 (ELU), got %d", what, act); \
  BPK_REQUIRE(bpk::ceil_div(planes, kWaves) < (1ll << 31), "%s: too many planes", what)

template <typename T>
int fwd_impl(const T* x, T* y, T* mean, T* rstd, int64_t planes, int64_t M, double eps, int act,
             void* stream) {
  IN_CHECK("instance_norm_act_fwd");
  BPK_REQUIRE(x && y && mean && rstd, "instance_norm_act_fwd: null pointer");
  if (planes == 0) return BPK_OK;
  hipStream_t st = bpk::as_stream(stream);
  if (blk_runs(M, 1) && planes < (1ll << 31)) {
    IN_BLK(in_fwd_blk, T, (blk_w<T>(x, y, nullptr, M)), x, y, mean, rstd, M, (T)eps, act)
  } else {
    hipLaunchKernelGGL(in_fwd<T>, dim3(blocks_for(planes)), dim3(256), 0, st, x, y, mean, rstd,
                       planes, M, (T)eps, act);
  }
  BPK_LAUNCH_CHECK("instance_norm_act_fwd");
  return BPK_OK;
}

template <typename T>
int bwd_impl(const T* dy, const T* x, const T* mean, const T* rstd, T* dx, int64_t planes,
             int64_t M, int act, void* stream, const T* add = nullptr) {
  IN_CHECK("instance_norm_act_bwd");
  BPK_REQUIRE(dy && x && mean && rstd && dx, "instance_norm_act_bwd: null pointer");
  if (planes == 0) return BPK_OK;
  hipStream_t st = bpk::as_stream(stream);
  if (blk_runs(M, 1) && planes < (1ll << 31)) {
    const int w = blk_w<T>(dy, x, dx, M) == 4 && blk_w<T>(add, nullptr, nullptr, M) == 4 ? 4 : 1;
    IN_BLK(in_bwd_blk, T, w, dy, x, mean, rstd, dx, M, act, add)
  } else {
    hipLaunchKernelGGL(in_bwd<T>, dim3(blocks_for(planes)), dim3(256), 0, st, dy, x, mean, rstd,
                       dx, planes, M, act, add);
  }
  BPK_LAUNCH_CHECK("instance_norm_act_bwd");
  return BPK_OK;
}

template <typename T>
int bwd2_impl(const T* v, const T* dy, const T* x, const T* mean, const T* rstd, T* gdy, T* gx,
              int64_t planes, int64_t M, int act, void* stream) {
  IN_CHECK("instance_norm_act_bwd2");
  BPK_REQUIRE(v && dy && x && mean && rstd, "instance_norm_act_bwd2: null input pointer");
  if (planes == 0 || (!gdy && !gx)) return BPK_OK;
  hipStream_t st = bpk::as_stream(stream);
  if (blk_runs(M, 1) && planes < (1ll << 31)) {
    const int w = blk_w<T>(v, dy, x, M) == 4 && blk_w<T>(gdy, gx, nullptr, M) == 4 ? 4 : 1;
    IN_BLK(in_bwd2_blk, T, w, v, dy, x, mean, rstd, gdy, gx, M, act)
  } else {
    hipLaunchKernelGGL(in_bwd2<T>, dim3(blocks_for(planes)), dim3(256), 0, st, v, dy, x, mean,
                       rstd, gdy, gx, planes, M, act);
  }
  BPK_LAUNCH_CHECK("instance_norm_act_bwd2");
  return BPK_OK;
}

}  // namespace

extern "C" {

int bpk_instance_norm_act_fwd_f32(const float* x, float* y, float* mean, float* rstd,
                                  int64_t planes, int64_t M, double eps, int act, void* stream) {
  return fwd_impl(x, y, mean, rstd, planes, M, eps, act, stream);
}
int bpk_instance_norm_act_fwd_f64(const double* x, double* y, double* mean, double* rstd,
                                  int64_t planes, int64_t M, double eps, int act, void* stream) {
  return fwd_impl(x, y, mean, rstd, planes, M, eps, act, stream);
}
int bpk_instance_norm_act_bwd_f32(const float* dy, const float* x, const float* mean,
                                  const float* rstd, float* dx, int64_t planes, int64_t M, int act,
                                  void* stream) {
  return bwd_impl(dy, x, mean, rstd, dx, planes, M, act, stream);
}
int bpk_instance_norm_act_bwd_f64(const double* dy, const double* x, const double* mean,
                                  const double* rstd, double* dx, int64_t planes, int64_t M,
                                  int act, void* stream) {
  return bwd_impl(dy, x, mean, rstd, dx, planes, M, act, stream);
}
int bpk_instance_norm_act_bwd_add_f32(const float* dy, const float* x, const float* mean,
                                      const float* rstd, const float* add, float* dx,
                                      int64_t planes, int64_t M, int act, void* stream) {
  BPK_REQUIRE(add, "instance_norm_act_bwd_add: null addend");
  return bwd_impl(dy, x, mean, rstd, dx, planes, M, act, stream, add);
}
int bpk_instance_norm_act_bwd2_f32(const float* v, const float* dy, const float* x,
                                   const float* mean, const float* rstd, float* gdy, float* gx,
                                   int64_t planes, int64_t M, int act, void* stream) {
  return bwd2_impl(v, dy, x, mean, rstd, gdy, gx, planes, M, act, stream);
}
int bpk_instance_norm_act_bwd2_f64(const double* v, const double* dy, const double* x,
                                   const double* mean, const double* rstd, double* gdy, double* gx,
                                   int64_t planes, int64_t M, int act, void* stream) {
  return bwd2_impl(v, dy, x, mean, rstd, gdy, gx, planes, M, act, stream);
}

}  // extern "C"
