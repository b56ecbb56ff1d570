// Spatial embedding of the PINN nets (reference models/layers.py:517-521,
// get_spatial_embedding) with its first and second derivatives, for the PINN residual
// (pinn_kalman/pinn.py:72-111), which differentiates FlowNet / PressureNet w.r.t. the
// coordinate channels x, y three times over:
//     f(x, y) = (sin(w r1) + sin(w r2)) / s,   r1 = |(x, y)|,   r2 = |(mx - x, my - y)|,
// mx = max(x), my = max(y) over one batch ("copy": the batch may hold k stacked copies of one
// batch, each with its own max -- pinn.PINN.forward_residual_copies).  As aten ops the chain
// is ~15 launches forward and 20-60 per derivative pass (pow, sqrt, sin, their backwards and
// double backwards, the max's evenly-distributed gradient, the fan-in adds); here each order
// is one reduction launch (per-copy sums, fixed order: deterministic) + one elementwise launch.
//
// Derivatives.  With A(r) = w cos(w r) / (r s), B(r) = (-w^2 sin(w r) r - w cos(w r)) / (r^3 s)
// and p = mx - x, q = my - y:  F1 = sin(w r1)/s has F1_a = A1 x, F1_aa = A1 + B1 x^2,
// F1_ab = B1 x y, ...; F2 = sin(w r2)/s has F2_p = A2 p, F2_pp = A2 + B2 p^2, F2_pq = B2 p q.
// The max enters as mx = x_a (a = argmax; ties share the gradient evenly, as torch's max()):
//   VJP   gx_j = g_j (A1 x - A2 p)_j + [x_j = mx] / cnt_x * sum_i g_i A2_i p_i      (y alike)
//   VJP2  for cotangents (hx, hy) of (gx, gy), with Hx = sum_{x_j = mx} hx_j / cnt_x:
//         dg = hx (A1 x - A2 p) + hy (A1 y - A2 q) + Hx A2 p + Hy A2 q
//         dx = g [hx (F1_aa + F2_pp) + hy (F1_ab + F2_pq) - Hx F2_pp - Hy F2_pq]
//              + [x = mx] / cnt_x * (Hx T_pp - sum g hx F2_pp + Hy T_pq - sum g hy F2_pq)
//         dy likewise (T_.. = sum g F2_..).
// The forward keeps the reference's float32 operation order (x*x + y*y, sqrt, w * r, sin,
// e1 + e2, times the fp32 reciprocal of s as aten's division by a scalar): bit-identical.
#include "bpk_common.h"

#include <algorithm>

// no FMA contraction: the forward must round like the reference's separate aten ops
#pragma clang fp contract(off)

namespace {

constexpr int kThreads = 256;
constexpr int kMaxS = 11;  // sums per copy (VJP2)
constexpr int kMaxNb = 32;  // reduce blocks per copy

struct EmbGeo {
  int64_t per;  // elements per copy
  int k, nb;    // copies, reduce blocks per copy
  float w, s, rs;
};

struct Terms {
  float A1, B1, A2, B2, p, q;
};

__device__ inline Terms terms(float x, float y, float mx, float my, const EmbGeo& g, bool second) {
  Terms t;
  const float r1 = sqrtf(x * x + y * y);
  t.p = mx - x;
  t.q = my - y;
  const float r2 = sqrtf(t.p * t.p + t.q * t.q);
  const float c1 = cosf(g.w * r1), c2 = cosf(g.w * r2);
  t.A1 = g.w * c1 / (r1 * g.s);
  t.A2 = g.w * c2 / (r2 * g.s);
  if (second) {
    const float s1 = sinf(g.w * r1), s2 = sinf(g.w * r2);
    t.B1 = (-g.w * g.w * s1 * r1 - g.w * c1) / (r1 * r1 * r1 * g.s);
    t.B2 = (-g.w * g.w * s2 * r2 - g.w * c2) / (r2 * r2 * r2 * g.s);
  } else {
    t.B1 = t.B2 = 0.f;
  }
  return t;
}

// block-wide sum of S values per thread (fixed tree order) into red[0..S)
template <int S>
__device__ inline void block_sum(float (&v)[S], float* red) {
  __shared__ float sm[S][kThreads];
  for (int j = 0; j < S; ++j) sm[j][threadIdx.x] = v[j];
  __syncthreads();
  for (int w = kThreads / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
      for (int j = 0; j < S; ++j) sm[j][threadIdx.x] += sm[j][threadIdx.x + w];
    __syncthreads();
  }
  if ((int)threadIdx.x < S) red[threadIdx.x] = sm[threadIdx.x][0];
}

// MODE 0: block max of x, y.  MODE 1: sum g A2 p, sum g A2 q, #(x == mx), #(y == my).
// MODE 2: Hx', Hy' (hx / hy summed over the argmax sets), the two counts and the seven sums of
// the VJP2 formulas.  part[(c * nb + j) * S + s].
template <int MODE>
__global__ __launch_bounds__(kThreads) void emb_reduce_kernel(
    const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ mxy,
    const float* __restrict__ gr, const float* __restrict__ hx, const float* __restrict__ hy,
    float* __restrict__ part, EmbGeo g) {
  constexpr int S = MODE == 0 ? 2 : (MODE == 1 ? 4 : 11);
  const int j = blockIdx.x, c = blockIdx.y;
  const int64_t chunk = (g.per + g.nb - 1) / g.nb;
  const int64_t b0 = (int64_t)c * g.per + (int64_t)j * chunk;
  const int64_t b1 = (int64_t)c * g.per + std::min<int64_t>(g.per, (int64_t)(j + 1) * chunk);
  float v[S];
  for (int s = 0; s < S; ++s) v[s] = MODE == 0 ? -INFINITY : 0.f;
  const float mx = MODE == 0 ? 0.f : mxy[2 * c], my = MODE == 0 ? 0.f : mxy[2 * c + 1];
  for (int64_t i = b0 + threadIdx.x; i < b1; i += kThreads) {
    const float xi = x[i], yi = y[i];
    if constexpr (MODE == 0) {
      v[0] = fmaxf(v[0], xi);
      v[1] = fmaxf(v[1], yi);
    } else {
      const bool ax = xi == mx, ay = yi == my;
      const Terms t = terms(xi, yi, mx, my, g, MODE == 2);
      const float gi = gr[i];
      if constexpr (MODE == 1) {
        v[0] += gi * t.A2 * t.p;
        v[1] += gi * t.A2 * t.q;
        v[2] += ax ? 1.f : 0.f;
        v[3] += ay ? 1.f : 0.f;
      } else {
        const float hxi = hx ? hx[i] : 0.f, hyi = hy ? hy[i] : 0.f;
        const float f2pp = t.A2 + t.B2 * t.p * t.p, f2pq = t.B2 * t.p * t.q;
        const float f2qq = t.A2 + t.B2 * t.q * t.q;
        v[0] += ax ? hxi : 0.f;
        v[1] += ay ? hyi : 0.f;
        v[2] += ax ? 1.f : 0.f;
        v[3] += ay ? 1.f : 0.f;
        v[4] += gi * f2pp;
        v[5] += gi * f2pq;
        v[6] += gi * f2qq;
        v[7] += gi * hxi * f2pp;
        v[8] += gi * hyi * f2pq;
        v[9] += gi * hxi * f2pq;
        v[10] += gi * hyi * f2qq;
      }
    }
  }
  if constexpr (MODE == 0) {
    __shared__ float sm[2][kThreads];
    sm[0][threadIdx.x] = v[0];
    sm[1][threadIdx.x] = v[1];
    __syncthreads();
    for (int w = kThreads / 2; w > 0; w >>= 1) {
      if ((int)threadIdx.x < w) {
        sm[0][threadIdx.x] = fmaxf(sm[0][threadIdx.x], sm[0][threadIdx.x + w]);
        sm[1][threadIdx.x] = fmaxf(sm[1][threadIdx.x], sm[1][threadIdx.x + w]);
      }
      __syncthreads();
    }
    if (threadIdx.x < 2) part[((int64_t)c * g.nb + j) * S + threadIdx.x] = sm[threadIdx.x][0];
  } else {
    __shared__ float red[S];
    block_sum<S>(v, red);
    __syncthreads();
    if ((int)threadIdx.x < S) part[((int64_t)c * g.nb + j) * S + threadIdx.x] = red[threadIdx.x];
  }
}

// the copy's combined partials (fixed order) in LDS; blocks never straddle copies (per % 256)
template <int MODE>
__device__ inline void combine(const float* __restrict__ part, int c, const EmbGeo& g, float* tot) {
  constexpr int S = MODE == 0 ? 2 : (MODE == 1 ? 4 : 11);
  if ((int)threadIdx.x < S) {
    float a = MODE == 0 ? -INFINITY : 0.f;
    for (int j = 0; j < g.nb; ++j) {
      const float v = part[((int64_t)c * g.nb + j) * S + threadIdx.x];
      a = MODE == 0 ? fmaxf(a, v) : a + v;
    }
    tot[threadIdx.x] = a;
  }
  __syncthreads();
}

__global__ __launch_bounds__(kThreads) void emb_fwd_kernel(const float* __restrict__ x,
                                                          const float* __restrict__ y,
                                                          const float* __restrict__ part,
                                                          float* __restrict__ out,
                                                          float* __restrict__ mxy, EmbGeo g) {
  __shared__ float tot[2];
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const int c = (int)(((int64_t)blockIdx.x * kThreads) / g.per);
  combine<0>(part, c, g, tot);
  const float mx = tot[0], my = tot[1];
  if ((int64_t)blockIdx.x * kThreads == (int64_t)c * g.per && threadIdx.x == 0) {
    mxy[2 * c] = mx;
    mxy[2 * c + 1] = my;
  }
  const float xi = x[i], yi = y[i];
  const float e1 = sinf(g.w * sqrtf(xi * xi + yi * yi));
  const float p = mx - xi, q = my - yi;
  const float e2 = sinf(g.w * sqrtf(p * p + q * q));
  out[i] = (e1 + e2) * g.rs;
}

__global__ __launch_bounds__(kThreads) void emb_vjp_kernel(
    const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ mxy,
    const float* __restrict__ gr, const float* __restrict__ part, float* __restrict__ gx,
    float* __restrict__ gy, EmbGeo g) {
  __shared__ float tot[4];
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const int c = (int)(((int64_t)blockIdx.x * kThreads) / g.per);
  combine<1>(part, c, g, tot);
  const float mx = mxy[2 * c], my = mxy[2 * c + 1];
  const float xi = x[i], yi = y[i], gi = gr[i];
  const Terms t = terms(xi, yi, mx, my, g, false);
  float vx = gi * (t.A1 * xi - t.A2 * t.p);
  float vy = gi * (t.A1 * yi - t.A2 * t.q);
  if (xi == mx) vx += tot[0] / tot[2];
  if (yi == my) vy += tot[1] / tot[3];
  gx[i] = vx;
  gy[i] = vy;
}

__global__ __launch_bounds__(kThreads) void emb_vjp2_kernel(
    const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ mxy,
    const float* __restrict__ gr, const float* __restrict__ hx, const float* __restrict__ hy,
    const float* __restrict__ part, float* __restrict__ dg, float* __restrict__ dx,
    float* __restrict__ dy, EmbGeo g) {
  __shared__ float tot[kMaxS];
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const int c = (int)(((int64_t)blockIdx.x * kThreads) / g.per);
  combine<2>(part, c, g, tot);
  const float mx = mxy[2 * c], my = mxy[2 * c + 1];
  const float Hx = tot[0] / tot[2], Hy = tot[1] / tot[3];
  const float xi = x[i], yi = y[i], gi = gr[i];
  const float hxi = hx ? hx[i] : 0.f, hyi = hy ? hy[i] : 0.f;
  const Terms t = terms(xi, yi, mx, my, g, true);
  const float f1aa = t.A1 + t.B1 * xi * xi, f1ab = t.B1 * xi * yi, f1bb = t.A1 + t.B1 * yi * yi;
  const float f2pp = t.A2 + t.B2 * t.p * t.p, f2pq = t.B2 * t.p * t.q;
  const float f2qq = t.A2 + t.B2 * t.q * t.q;
  if (dg)
    dg[i] = hxi * (t.A1 * xi - t.A2 * t.p) + hyi * (t.A1 * yi - t.A2 * t.q) + Hx * t.A2 * t.p +
            Hy * t.A2 * t.q;
  float vx = gi * (hxi * (f1aa + f2pp) + hyi * (f1ab + f2pq) - Hx * f2pp - Hy * f2pq);
  float vy = gi * (hxi * (f1ab + f2pq) + hyi * (f1bb + f2qq) - Hx * f2pq - Hy * f2qq);
  if (xi == mx) vx += (Hx * tot[4] - tot[7] + Hy * tot[5] - tot[8]) / tot[2];
  if (yi == my) vy += (Hx * tot[5] - tot[9] + Hy * tot[6] - tot[10]) / tot[3];
  if (dx) dx[i] = vx;
  if (dy) dy[i] = vy;
}

EmbGeo make_geo(int64_t n, int k, float omega, float s) {
  EmbGeo g;
  g.k = k;
  g.per = n / k;
  g.nb = (int)std::min<int64_t>(kMaxNb, std::max<int64_t>(1, bpk::ceil_div(g.per, kThreads * 16)));
  g.w = omega;
  g.s = s;
  g.rs = 1.0f / s;
  return g;
}

}  // namespace

extern "C" int bpk_spatial_emb_supported(int64_t n, int k) {
  return n > 0 && k > 0 && n % k == 0 && (n / k) % kThreads == 0 && n / kThreads < (1LL << 31);
}

extern "C" int64_t bpk_spatial_emb_workspace_bytes(int64_t n, int k) {
  if (!bpk_spatial_emb_supported(n, k)) return 0;
  return (int64_t)k * kMaxNb * kMaxS * (int64_t)sizeof(float);
}

#define EMB_CHECK(n, k, ws)                                                                   \
  BPK_REQUIRE(bpk_spatial_emb_supported(n, k), "spatial_emb: need n %% k == 0 and (n / k) %% " \
              "256 == 0 (n=%lld k=%d)", (long long)(n), (k));                                 \
  BPK_REQUIRE((ws) != nullptr, "spatial_emb: workspace is NULL")

extern "C" int bpk_spatial_emb_fwd_f32(const float* x, const float* y, float* out, float* mxy,
                                       float* workspace, int64_t n, int k, float omega, float s,
                                       void* stream) {
  EMB_CHECK(n, k, workspace);
  const EmbGeo g = make_geo(n, k, omega, s);
  hipStream_t st = bpk::as_stream(stream);
  hipLaunchKernelGGL(emb_reduce_kernel<0>, dim3(g.nb, k), dim3(kThreads), 0, st, x, y, nullptr,
                     nullptr, nullptr, nullptr, workspace, g);
  BPK_LAUNCH_CHECK("spatial_emb_fwd(reduce)");
  hipLaunchKernelGGL(emb_fwd_kernel, dim3((unsigned)(n / kThreads)), dim3(kThreads), 0, st, x, y,
                     workspace, out, mxy, g);
  BPK_LAUNCH_CHECK("spatial_emb_fwd");
  return BPK_OK;
}

extern "C" int bpk_spatial_emb_vjp_f32(const float* x, const float* y, const float* mxy,
                                       const float* gr, float* gx, float* gy, float* workspace,
                                       int64_t n, int k, float omega, float s, void* stream) {
  EMB_CHECK(n, k, workspace);
  const EmbGeo g = make_geo(n, k, omega, s);
  hipStream_t st = bpk::as_stream(stream);
  hipLaunchKernelGGL(emb_reduce_kernel<1>, dim3(g.nb, k), dim3(kThreads), 0, st, x, y, mxy, gr,
                     nullptr, nullptr, workspace, g);
  BPK_LAUNCH_CHECK("spatial_emb_vjp(reduce)");
  hipLaunchKernelGGL(emb_vjp_kernel, dim3((unsigned)(n / kThreads)), dim3(kThreads), 0, st, x, y,
                     mxy, gr, workspace, gx, gy, g);
  BPK_LAUNCH_CHECK("spatial_emb_vjp");
  return BPK_OK;
}

extern "C" int bpk_spatial_emb_vjp2_f32(const float* x, const float* y, const float* mxy,
                                        const float* gr, const float* hx, const float* hy,
                                        float* dg, float* dx, float* dy, float* workspace,
                                        int64_t n, int k, float omega, float s, void* stream) {
  EMB_CHECK(n, k, workspace);
  const EmbGeo g = make_geo(n, k, omega, s);
  hipStream_t st = bpk::as_stream(stream);
  hipLaunchKernelGGL(emb_reduce_kernel<2>, dim3(g.nb, k), dim3(kThreads), 0, st, x, y, mxy, gr,
                     hx, hy, workspace, g);
  BPK_LAUNCH_CHECK("spatial_emb_vjp2(reduce)");
  hipLaunchKernelGGL(emb_vjp2_kernel, dim3((unsigned)(n / kThreads)), dim3(kThreads), 0, st, x,
                     y, mxy, gr, hx, hy, workspace, dg, dx, dy, g);
  BPK_LAUNCH_CHECK("spatial_emb_vjp2");
  return BPK_OK;
}
