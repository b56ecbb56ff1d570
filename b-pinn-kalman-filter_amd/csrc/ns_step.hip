// Navier-Stokes explicit step (ns_step) for gfx950.
//
// Bit-level restatement of op/ns_step_kernel.cu:30-234 + the op sequencing of
// op/ns_step.cpp:45-102.  Every expression keeps the reference's operation
// order and its float/double promotions (`2.0`, `3.0`, `0.25`, `8.0` are double
// literals in the reference, so those sub-expressions run in double there too);
// FMA contraction is disabled for this file so the result is bit-identical to
// the gcc-compiled C oracle (oracle/ns_step_ref.c).
//
// Layout (reference convention, op/ns_step_kernel.cu:30-37): a plane is
// field[y * nx + x], x in [0, nx) (contiguous, nx = size(2)), y in [0, ny)
// (ny = size(3)); velocity planes u/v of sample b at 2b / 2b+1.
//
// What changes vs the reference (MI355X-first):
//  * one thread per site with x fastest (coalesced 256-B rows) instead of one
//    block per site with the batch on threadIdx.x (uncoalesced, B <= 1024);
//  * the whole simulator step (velocity -> pressure -> density) runs as two
//    fused kernels that recompute the intermediate fields from cached inputs
//    instead of 7+ launches that round-trip every intermediate through HBM.
#include "bpk_common.h"

#pragma clang fp contract(off)

namespace {

struct Geo {
  int nx, ny;
  int64_t hw;
};

__device__ inline int clampx(int x, int n) { return x < 0 ? -x : (x > n - 1 ? 2 * n - 2 - x : x); }

template <typename T>
__device__ inline int sgn(T v) {
  if (v < 0.0) return -1;
  if (v > 0.0) return 1;
  return 0;
}

// CIP advection of one site (op/ns_step_kernel.cu:115-158), operands passed as
// plane pointers so callers can supply stored or recomputed fields.
struct CipIn {
  float f_c, f_ym, f_xm, f_xmym;  // f(x,y) f(x,ym) f(xm,y) f(xm,ym)
  float fx_c, fx_xm, fx_ym;       // fx(x,y) fx(xm,y) fx(x,ym)
  float fy_c, fy_xm, fy_ym;       // fy(x,y) fy(xm,y) fy(x,ym)
};

// Correctly rounded division without the IEEE divide sequence.  For b != 0 with
// r = RN(1/b) and q = RN(a*r) (within 1 ulp of a/b), the residual a - b*q is exact
// (one FMA) and RN(q + r*(a - b*q)) == RN(a/b) (Markstein's theorem) -- so these are
// bit-identical to `a / b` while costing a multiply and two FMAs.  The theorem needs
// every intermediate in the normal range: the fast path is taken only for
// 1e-25 < |a| < 1e25 and a denominator in [1e-10, 1e10] (`ok`, decided once per
// launch); everything else -- including exact zeros (sign of a zero quotient), inf
// and NaN -- takes the true division.
// The rare true divisions live out of line so the compiler cannot if-convert (and so
// always execute) the IEEE divide sequence next to the fast path.
__device__ __attribute__((noinline)) float div_true(float a, float b) { return a / b; }
__device__ __attribute__((noinline)) double div_true(double a, double b) { return a / b; }

__device__ inline float div_rn(float a, float b, float rb, bool ok) {
  const float aa = fabsf(a);
  if (__builtin_expect(!(ok && aa > 1e-25f && aa < 1e25f), 0)) return div_true(a, b);
  const float q = a * rb;
  const float rem = __builtin_fmaf(-q, b, a);
  return __builtin_fmaf(rem, rb, q);
}
__device__ inline double div_rn(double a, double b, double rb, bool ok) {
  const double aa = fabs(a);
  if (__builtin_expect(!(ok && aa > 1e-200 && aa < 1e200), 0)) return div_true(a, b);
  const double q = a * rb;
  const double rem = __builtin_fma(-q, b, a);
  return __builtin_fma(rem, rb, q);
}

__device__ inline bool denom_ok(float b) {
  const float ab = fabsf(b);
  return ab >= 1e-10f && ab <= 1e10f;
}

// Per-launch constants of the fast path: dx, dx^3 as the reference rounds them, and
// their correctly rounded reciprocals (computed once per thread with true divisions).
struct NsConst {
  float dt, dx, rdx;       // 1/dx
  float d3, rd3;           // (dx*dx)*dx, 1/d3 (float)
  double dxd, rdxd;        // (double)dx, 1/(double)dx
  double d3d, rd3d;        // (double)d3, 1/(double)d3
  bool ok_dx, ok_d3;
  __device__ explicit NsConst(float dt_, float dx_) : dt(dt_), dx(dx_) {
    rdx = 1.0f / dx;
    d3 = dx * dx * dx;
    rd3 = 1.0f / d3;
    dxd = (double)dx;
    rdxd = 1.0 / dxd;
    d3d = (double)d3;
    rd3d = 1.0 / d3d;
    ok_dx = denom_ok(dx);
    ok_d3 = denom_ok(d3);
  }
  // reference (d / dx) for a float difference d
  __device__ float over_dx(float d) const { return div_rn(d, dx, rdx, ok_dx); }
  // reference central difference (d / dx / 2); /2 == *0.5 exactly
  __device__ float over_2dx(float d) const { return div_rn(d, dx, rdx, ok_dx) * 0.5f; }
};

// d / (s * dx^3) in float for s = sgn(...) (the reference's x_s_denom); s == 0 keeps the
// reference's division by zero (inf/nan)
__device__ inline float div_sd3(float d, int s, const NsConst& k) {
  if (s == 0) return div_true(d, (float)s * k.dx * k.dx * k.dx);
  const float q = div_rn(d, k.d3, k.rd3, k.ok_d3);
  return s > 0 ? q : -q;
}
__device__ inline double div_sd3(double d, int s, const NsConst& k) {
  if (s == 0) return div_true(d, (double)((float)s * k.dx * k.dx * k.dx));
  const double q = div_rn(d, k.d3d, k.rd3d, k.ok_d3);
  return s > 0 ? q : -q;
}

// cip_site (op/ns_step_kernel.cu:115-158) with the cheap exact divisions; every
// expression keeps the reference's float/double types and operation order.
__device__ inline float cip_site_fast(const CipIn& q, float u, float v, const NsConst& k) {
  const int x_s = sgn(u);
  const int y_s = sgn(v);
  const float dx = k.dx;
  float tmp1 = q.f_c - q.f_ym - q.f_xm + q.f_xmym;
  float tmp2 = q.f_xm - q.f_c;
  float tmp3 = q.f_ym - q.f_c;
  float a = (float)div_sd3((double)(x_s * (q.fx_xm + q.fx_c) * dx) - 2.0 * (-tmp2), x_s, k);
  float b = (float)div_sd3((double)(y_s * (q.fy_ym + q.fy_c) * dx) - 2.0 * (-tmp3), y_s, k);
  float c = div_sd3(-tmp1 - x_s * (q.fx_ym - q.fx_c) * dx, y_s, k);
  float d = div_sd3(-tmp1 - y_s * (q.fy_xm - q.fy_c) * dx, x_s, k);
  double en = 3.0 * tmp2 + x_s * (q.fx_xm + 2.0 * q.fx_c) * (double)dx;
  double fn = 3.0 * tmp3 + y_s * (q.fy_ym + 2.0 * q.fy_c) * (double)dx;
  float e = (float)div_rn(div_rn(en, k.dxd, k.rdxd, k.ok_dx), k.dxd, k.rdxd, k.ok_dx);
  float f = (float)div_rn(div_rn(fn, k.dxd, k.rdxd, k.ok_dx), k.dxd, k.rdxd, k.ok_dx);
  float gn = -(q.fy_xm - q.fy_c) + c * dx * dx;
  float g;
  if (x_s == 0) {
    g = div_true(gn, x_s * dx);
  } else {
    const float gq = div_rn(gn, dx, k.rdx, k.ok_dx);
    g = x_s > 0 ? gq : -gq;
  }
  float X = -u * k.dt;
  float Y = -v * k.dt;
  return ((a * X + c * Y + e) * X + g * Y + q.fx_c) * X + ((b * Y + d * X + f) * Y + q.fy_c) * Y +
         q.f_c;
}


// ---- reference device helpers (op/ns_step_kernel.cu:50-75), exact fast division
__device__ inline float ddx(const float* f, int x, int y, const Geo& g, const NsConst& c) {
  const float* r = f + (int64_t)y * g.nx;
  if (x == 0) return c.over_dx(r[x + 1] - r[x]);
  if (x == g.nx - 1) return c.over_dx(r[x] - r[x - 1]);
  return c.over_2dx(r[x + 1] - r[x - 1]);
}
__device__ inline float ddy(const float* f, int x, int y, const Geo& g, const NsConst& c) {
  if (y == 0) return c.over_dx(f[(int64_t)(y + 1) * g.nx + x] - f[(int64_t)y * g.nx + x]);
  if (y == g.ny - 1) return c.over_dx(f[(int64_t)y * g.nx + x] - f[(int64_t)(y - 1) * g.nx + x]);
  return c.over_2dx(f[(int64_t)(y + 1) * g.nx + x] - f[(int64_t)(y - 1) * g.nx + x]);
}

// pressure update of one site (op/ns_step_kernel.cu:205-234):
// sub_x = V(xu) - V(xd), sub_y = V(yu) - V(yd)
__device__ inline float pres_site(float p_xd, float p_xu, float p_yd, float p_yu, float u_xu,
                                  float u_xd, float v_xu, float v_xd, float u_yu, float u_yd,
                                  float v_yu, float v_yd, float dt, float dx, float r8dt,
                                  bool ok8) {
  const float sxx = u_xu - u_xd, sxy = v_xu - v_xd;
  const float syx = u_yu - u_yd, syy = v_yu - v_yd;
  const float aver_p = 0.25 * (p_xd + p_xu + p_yd + p_yu);
  const float pred_p = aver_p + (sxx * sxx + syy * syy + (syx * sxy)) / 8.0 -
                       div_rn(dx * (sxx + syy), 8 * dt, r8dt, ok8);
  return pred_p;
}

// ---------------------------------------------------------------- low-level kernels

__global__ __launch_bounds__(256) void k_gradient(const float* __restrict__ f, int64_t fstride,
                                                  float* __restrict__ fx, float* __restrict__ fy,
                                                  int B, Geo g, float dx) {
  const NsConst c(1.0f, dx);
  const int64_t total = (int64_t)B * g.hw;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / g.hw;
    const int s = (int)(i - b * g.hw);
    const int y = s / g.nx, x = s - y * g.nx;
    const float* fp = f + b * fstride;
    fx[i] = ddx(fp, x, y, g, c);
    fy[i] = ddy(fp, x, y, g, c);
  }
}

__device__ inline CipIn gather_cip(const float* fp, const float* fxp, const float* fyp, int x,
                                   int y, int xm, int ym, int nx) {
  CipIn q;
  const int64_t c = (int64_t)y * nx + x, cxm = (int64_t)y * nx + xm, cym = (int64_t)ym * nx + x,
                cxy = (int64_t)ym * nx + xm;
  q.f_c = fp[c];
  q.f_ym = fp[cym];
  q.f_xm = fp[cxm];
  q.f_xmym = fp[cxy];
  q.fx_c = fxp[c];
  q.fx_xm = fxp[cxm];
  q.fx_ym = fxp[cym];
  q.fy_c = fyp[c];
  q.fy_xm = fyp[cxm];
  q.fy_ym = fyp[cym];
  return q;
}

// out[b] (plane stride ostride) = CIP(f[b] with stride fstride, fx/fy contiguous, vel[b])
__global__ __launch_bounds__(256) void k_cip(const float* __restrict__ f, int64_t fstride,
                                             const float* __restrict__ fx,
                                             const float* __restrict__ fy,
                                             const float* __restrict__ vel,
                                             float* __restrict__ out, int64_t ostride, int B,
                                             Geo g, float dt, float dx) {
  const NsConst c(dt, dx);
  const int64_t total = (int64_t)B * g.hw;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / g.hw;
    const int s = (int)(i - b * g.hw);
    const int y = s / g.nx, x = s - y * g.nx;
    const float u = vel[(2 * b) * g.hw + s];
    const float v = vel[(2 * b + 1) * g.hw + s];
    const int xm = clampx(x - sgn(u), g.nx);
    const int ym = clampx(y - sgn(v), g.ny);
    const CipIn q = gather_cip(f + b * fstride, fx + b * g.hw, fy + b * g.hw, x, y, xm, ym, g.nx);
    out[b * ostride + s] = cip_site_fast(q, u, v, c);
  }
}

__global__ __launch_bounds__(256) void k_advect(const float* __restrict__ f, int64_t fstride,
                                                const float* __restrict__ fx,
                                                const float* __restrict__ fy,
                                                const float* __restrict__ vel,
                                                float* __restrict__ out, int B, Geo g, float dt) {
  const int64_t total = (int64_t)B * g.hw;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / g.hw;
    const int64_t s = i - b * g.hw;
    float advect = vel[(2 * b) * g.hw + s] * fx[i] + vel[(2 * b + 1) * g.hw + s] * fy[i];
    out[i] = f[b * fstride + s] - dt * advect;
  }
}

__global__ __launch_bounds__(256) void k_vel_update(const float* __restrict__ vel,
                                                    const float* __restrict__ px,
                                                    const float* __restrict__ py,
                                                    float* __restrict__ vel_n, int B, Geo g,
                                                    float dt) {
  const int64_t total = (int64_t)B * g.hw;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / g.hw;
    const int64_t s = i - b * g.hw;
    vel_n[(2 * b) * g.hw + s] = vel[(2 * b) * g.hw + s] - px[i] * dt;
    vel_n[(2 * b + 1) * g.hw + s] = vel[(2 * b + 1) * g.hw + s] - py[i] * dt;
  }
}

__global__ __launch_bounds__(256) void k_pres_update(const float* __restrict__ pres,
                                                     const float* __restrict__ vel,
                                                     float* __restrict__ pres_n, int B, Geo g,
                                                     float dt, float dx) {
  const float r8dt = 1.0f / (8 * dt);
  const bool ok8 = denom_ok(8 * dt);
  const int64_t total = (int64_t)B * g.hw;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / g.hw;
    const int s = (int)(i - b * g.hw);
    const int y = s / g.nx, x = s - y * g.nx;
    const int xu = clampx(x + 1, g.nx), xd = clampx(x - 1, g.nx);
    const int yu = clampx(y + 1, g.ny), yd = clampx(y - 1, g.ny);
    const float* p = pres + b * g.hw;
    const float* u = vel + (2 * b) * g.hw;
    const float* v = vel + (2 * b + 1) * g.hw;
    const int64_t ixu = (int64_t)y * g.nx + xu, ixd = (int64_t)y * g.nx + xd,
                  iyu = (int64_t)yu * g.nx + x, iyd = (int64_t)yd * g.nx + x;
    pres_n[i] = pres_site(p[ixd], p[ixu], p[iyd], p[iyu], u[ixu], u[ixd], v[ixu], v[ixd], u[iyu],
                          u[iyd], v[iyu], v[iyd], dt, dx, r8dt, ok8);
  }
}

// ---------------------------------------------------------------- fused full step
// Stage A: vel' = CIP advection of the vel_n planes, where vel_n = vel - dt grad(p).
// The advected "u" field of sample b is vel_n plane uplane(b) and the "v" field plane
// vplane(b):  compat -> (b, b+1)  (reference unbind quirk), else (2b, 2b+1); the
// advecting velocity is vel_n planes (2b, 2b+1) at the site.
//
// LDS-tiled: a block owns a TX x TY tile of one sample.  It computes vel_n of the two
// field planes over the tile + 2-site halo into LDS once, then their x/y differences
// over the tile + 1-site halo, then the CIP update of every site from LDS -- instead
// of recomputing each vel_n value ~16 times per site from HBM.
constexpr int kTX = 64, kTY = 4;
constexpr int kFW = kTX + 4, kFH = kTY + 4;  // field tile (+2 halo)
constexpr int kGW = kTX + 2, kGH = kTY + 2;  // gradient tile (+1 halo)

__device__ inline float veln_at(const float* __restrict__ vel, const float* __restrict__ pres,
                                int64_t k, int x, int y, const Geo& g, const NsConst& c) {
  const float* p = pres + (k >> 1) * g.hw;
  float grad;
  if (k & 1) {
    if (y == 0) grad = c.over_dx(p[(int64_t)(y + 1) * g.nx + x] - p[(int64_t)y * g.nx + x]);
    else if (y == g.ny - 1) grad = c.over_dx(p[(int64_t)y * g.nx + x] - p[(int64_t)(y - 1) * g.nx + x]);
    else grad = c.over_2dx(p[(int64_t)(y + 1) * g.nx + x] - p[(int64_t)(y - 1) * g.nx + x]);
  } else {
    const float* r = p + (int64_t)y * g.nx;
    if (x == 0) grad = c.over_dx(r[x + 1] - r[x]);
    else if (x == g.nx - 1) grad = c.over_dx(r[x] - r[x - 1]);
    else grad = c.over_2dx(r[x + 1] - r[x - 1]);
  }
  return vel[k * g.hw + (int64_t)y * g.nx + x] - grad * c.dt;
}

__global__ __launch_bounds__(256) void k_fused_velocity_lds(const float* __restrict__ vel,
                                                            const float* __restrict__ pres,
                                                            float* __restrict__ vel_out,
                                                            int B, Geo g, float dt, float dx,
                                                            int compat, int tiles_x,
                                                            int tiles_y) {
  __shared__ float sF[2][kFH][kFW];
  __shared__ float sFx[2][kGH][kGW];
  __shared__ float sFy[2][kGH][kGW];
  const NsConst c(dt, dx);
  const int tid = threadIdx.x;
  const int64_t tiles_per_sample = (int64_t)tiles_x * tiles_y;
  // consecutive tiles on one XCD (shared halo rows hit its L2): bpk::xcd_tile
  const int64_t first = bpk::xcd_tile(blockIdx.x, gridDim.x);
  for (int64_t tile = first; tile < (int64_t)B * tiles_per_sample; tile += gridDim.x) {
    const int b = (int)(tile / tiles_per_sample);
    const int tr = (int)(tile - (int64_t)b * tiles_per_sample);
    const int x0 = (tr % tiles_x) * kTX, y0 = (tr / tiles_x) * kTY;
    const int64_t plane_k[2] = {compat ? (int64_t)b : 2 * (int64_t)b,
                                compat ? (int64_t)b + 1 : 2 * (int64_t)b + 1};
    __syncthreads();  // previous tile's readers are done with LDS
    // 1. vel_n of both field planes over the tile + 2 halo (in-domain points only)
    for (int i = tid; i < 2 * kFH * kFW; i += blockDim.x) {
      const int pl = i / (kFH * kFW);
      const int r = i - pl * (kFH * kFW);
      const int ly = r / kFW, lx = r - ly * kFW;
      const int gx = x0 - 2 + lx, gy = y0 - 2 + ly;
      if (gx >= 0 && gx < g.nx && gy >= 0 && gy < g.ny)
        sF[pl][ly][lx] = veln_at(vel, pres, plane_k[pl], gx, gy, g, c);
    }
    __syncthreads();
    // 2. reference diff_x / diff_y of the field planes over the tile + 1 halo
    for (int i = tid; i < 2 * kGH * kGW; i += blockDim.x) {
      const int pl = i / (kGH * kGW);
      const int r = i - pl * (kGH * kGW);
      const int ly = r / kGW, lx = r - ly * kGW;
      const int gx = x0 - 1 + lx, gy = y0 - 1 + ly;
      if (gx >= 0 && gx < g.nx && gy >= 0 && gy < g.ny) {
        const int fy = ly + 1, fx = lx + 1;  // position in sF
        float dxv, dyv;
        if (gx == 0) dxv = c.over_dx(sF[pl][fy][fx + 1] - sF[pl][fy][fx]);
        else if (gx == g.nx - 1) dxv = c.over_dx(sF[pl][fy][fx] - sF[pl][fy][fx - 1]);
        else dxv = c.over_2dx(sF[pl][fy][fx + 1] - sF[pl][fy][fx - 1]);
        if (gy == 0) dyv = c.over_dx(sF[pl][fy + 1][fx] - sF[pl][fy][fx]);
        else if (gy == g.ny - 1) dyv = c.over_dx(sF[pl][fy][fx] - sF[pl][fy - 1][fx]);
        else dyv = c.over_2dx(sF[pl][fy + 1][fx] - sF[pl][fy - 1][fx]);
        sFx[pl][ly][lx] = dxv;
        sFy[pl][ly][lx] = dyv;
      }
    }
    __syncthreads();
    // 3. CIP update of the tile's sites, both components
    {
      const int lx = tid % kTX, ly = tid / kTX;
      const int x = x0 + lx, y = y0 + ly;
      if (ly < kTY && x < g.nx && y < g.ny) {
        const float u = veln_at(vel, pres, 2 * (int64_t)b, x, y, g, c);
        const float v = veln_at(vel, pres, 2 * (int64_t)b + 1, x, y, g, c);
        const int xm = clampx(x - sgn(u), g.nx);
        const int ym = clampx(y - sgn(v), g.ny);
        // LDS coordinates: field tile origin (x0-2, y0-2), gradient tile origin (x0-1, y0-1)
        const int fxc = x - x0 + 2, fyc = y - y0 + 2, fxm = xm - x0 + 2, fym = ym - y0 + 2;
        const int gxc = x - x0 + 1, gyc = y - y0 + 1, gxm = xm - x0 + 1, gym = ym - y0 + 1;
        const int64_t s = (int64_t)y * g.nx + x;
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) {
          CipIn q;
          q.f_c = sF[pl][fyc][fxc];
          q.f_ym = sF[pl][fym][fxc];
          q.f_xm = sF[pl][fyc][fxm];
          q.f_xmym = sF[pl][fym][fxm];
          q.fx_c = sFx[pl][gyc][gxc];
          q.fx_xm = sFx[pl][gyc][gxm];
          q.fx_ym = sFx[pl][gym][gxc];
          q.fy_c = sFy[pl][gyc][gxc];
          q.fy_xm = sFy[pl][gyc][gxm];
          q.fy_ym = sFy[pl][gym][gxc];
          vel_out[(2 * (int64_t)b + pl) * g.hw + s] = cip_site_fast(q, u, v, c);
        }
      }
    }
  }
}

// Stage B: pres' = pressure update with vel'; dens' = CIP(dens) with vel'.
__global__ __launch_bounds__(256) void k_fused_pres_dens(const float* __restrict__ dens,
                                                         const float* __restrict__ pres,
                                                         const float* __restrict__ vel1,
                                                         float* __restrict__ dens_out,
                                                         float* __restrict__ pres_out, int B,
                                                         Geo g, float dt, float dx) {
  const NsConst c(dt, dx);
  const float r8dt = 1.0f / (8 * dt);
  const bool ok8 = denom_ok(8 * dt);
  const int64_t total = (int64_t)B * g.hw;
  // rows y-2 .. y+2 of a block's sites are read by its neighbours too: keep those on one XCD
  const int64_t lb = bpk::xcd_tile(blockIdx.x, gridDim.x);
  for (int64_t i = lb * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / g.hw;
    const int s = (int)(i - b * g.hw);
    const int y = s / g.nx, x = s - y * g.nx;
    const float* p = pres + b * g.hw;
    const float* u = vel1 + (2 * b) * g.hw;
    const float* v = vel1 + (2 * b + 1) * g.hw;
    {
      const int xu = clampx(x + 1, g.nx), xd = clampx(x - 1, g.nx);
      const int yu = clampx(y + 1, g.ny), yd = clampx(y - 1, g.ny);
      const int64_t ixu = (int64_t)y * g.nx + xu, ixd = (int64_t)y * g.nx + xd,
                    iyu = (int64_t)yu * g.nx + x, iyd = (int64_t)yd * g.nx + x;
      pres_out[i] = pres_site(p[ixd], p[ixu], p[iyd], p[iyu], u[ixu], u[ixd], v[ixu], v[ixd],
                              u[iyu], u[iyd], v[iyu], v[iyd], dt, dx, r8dt, ok8);
    }
    const float uc = u[s], vc = v[s];
    const int xm = clampx(x - sgn(uc), g.nx);
    const int ym = clampx(y - sgn(vc), g.ny);
    const float* f = dens + b * g.hw;
    CipIn q;
    q.f_c = f[s];
    q.f_ym = f[(int64_t)ym * g.nx + x];
    q.f_xm = f[(int64_t)y * g.nx + xm];
    q.f_xmym = f[(int64_t)ym * g.nx + xm];
    q.fx_c = ddx(f, x, y, g, c);
    q.fx_xm = ddx(f, xm, y, g, c);
    q.fx_ym = ddx(f, x, ym, g, c);
    q.fy_c = ddy(f, x, y, g, c);
    q.fy_xm = ddy(f, xm, y, g, c);
    q.fy_ym = ddy(f, x, ym, g, c);
    dens_out[i] = cip_site_fast(q, uc, vc, c);
  }
}

// out[x] = sum_j coef(j, x) g[j] for the 1-D stencil D of diff_x: interior rows j give
// +-1/(2dx) to x = j+-1, border rows give +-1/dx (one-sided differences)
__device__ inline float adj1d(const float* g, int64_t stride, int x, int n, float dx) {
  float acc = 0.f;
  auto coef = [&](int j, int xx) -> float {  // coefficient of f[xx] in (D f)[j]
    if (j == 0) return xx == 1 ? 1.0f / dx : (xx == 0 ? -1.0f / dx : 0.f);
    if (j == n - 1) return xx == n - 1 ? 1.0f / dx : (xx == n - 2 ? -1.0f / dx : 0.f);
    return xx == j + 1 ? 0.5f / dx : (xx == j - 1 ? -0.5f / dx : 0.f);
  };
  for (int j = x - 1; j <= x + 1; ++j)
    if (j >= 0 && j < n) acc += coef(j, x) * g[(int64_t)j * stride];
  return acc;
}

__global__ __launch_bounds__(256) void k_gradient_adjoint(const float* __restrict__ gx,
                                                          const float* __restrict__ gy,
                                                          float* __restrict__ out, int B, Geo g,
                                                          float dx) {
  const int64_t total = (int64_t)B * g.hw;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / g.hw;
    const int s = (int)(i - b * g.hw);
    const int y = s / g.nx, x = s - y * g.nx;
    const float* rx = gx + b * g.hw + (int64_t)y * g.nx;  // row y of gx, stride 1 in x
    const float* cy = gy + b * g.hw + x;                   // column x of gy, stride nx in y
    out[i] = adj1d(rx, 1, x, g.nx, dx) + adj1d(cy, g.nx, y, g.ny, dx);
  }
}

unsigned grid_for(int64_t total) {
  return (unsigned)std::min<int64_t>(bpk::ceil_div(total, 256), 256 * 64);
}

#define NS_GEO_CHECK(B, nx, ny)                                                            \
  BPK_REQUIRE((B) >= 0 && (nx) >= 2 && (ny) >= 2, "ns_step: need B >= 0 and planes >= 2x2 " \
                                                  "(got B=%d nx=%d ny=%d)",               \
              (B), (nx), (ny))

}  // namespace

extern "C" int bpk_ns_gradient_f32(const float* f, int64_t f_plane_stride, float* fx, float* fy,
                                   int B, int nx, int ny, float dx, void* stream) {
  NS_GEO_CHECK(B, nx, ny);
  const Geo g{nx, ny, (int64_t)nx * ny};
  if (B == 0) return BPK_OK;
  hipLaunchKernelGGL(k_gradient, dim3(grid_for(B * g.hw)), dim3(256), 0, bpk::as_stream(stream), f,
                     f_plane_stride, fx, fy, B, g, dx);
  BPK_LAUNCH_CHECK("ns_gradient");
  return BPK_OK;
}

extern "C" int bpk_ns_gradient_adjoint_f32(const float* gx, const float* gy, float* out, int B,
                                           int nx, int ny, float dx, void* stream) {
  NS_GEO_CHECK(B, nx, ny);
  const Geo g{nx, ny, (int64_t)nx * ny};
  if (B == 0) return BPK_OK;
  hipLaunchKernelGGL(k_gradient_adjoint, dim3(grid_for(B * g.hw)), dim3(256), 0,
                     bpk::as_stream(stream), gx, gy, out, B, g, dx);
  BPK_LAUNCH_CHECK("ns_gradient_adjoint");
  return BPK_OK;
}

extern "C" int bpk_ns_cip_advect_f32(const float* f, int64_t f_plane_stride, const float* fx,
                                     const float* fy, const float* vel, float* out, int B, int nx,
                                     int ny, float dt, float dx, void* stream) {
  NS_GEO_CHECK(B, nx, ny);
  const Geo g{nx, ny, (int64_t)nx * ny};
  if (B == 0) return BPK_OK;
  hipLaunchKernelGGL(k_cip, dim3(grid_for(B * g.hw)), dim3(256), 0, bpk::as_stream(stream), f,
                     f_plane_stride, fx, fy, vel, out, g.hw, B, g, dt, dx);
  BPK_LAUNCH_CHECK("ns_cip_advect");
  return BPK_OK;
}

extern "C" int bpk_ns_advect_f32(const float* f, int64_t f_plane_stride, const float* fx,
                                 const float* fy, const float* vel, float* out, int B, int nx,
                                 int ny, float dt, void* stream) {
  NS_GEO_CHECK(B, nx, ny);
  const Geo g{nx, ny, (int64_t)nx * ny};
  if (B == 0) return BPK_OK;
  hipLaunchKernelGGL(k_advect, dim3(grid_for(B * g.hw)), dim3(256), 0, bpk::as_stream(stream), f,
                     f_plane_stride, fx, fy, vel, out, B, g, dt);
  BPK_LAUNCH_CHECK("ns_advect");
  return BPK_OK;
}

extern "C" int bpk_ns_vel_update_f32(const float* vel, const float* px, const float* py,
                                     float* vel_n, int B, int nx, int ny, float dt,
                                     void* stream) {
  NS_GEO_CHECK(B, nx, ny);
  const Geo g{nx, ny, (int64_t)nx * ny};
  if (B == 0) return BPK_OK;
  hipLaunchKernelGGL(k_vel_update, dim3(grid_for(B * g.hw)), dim3(256), 0, bpk::as_stream(stream),
                     vel, px, py, vel_n, B, g, dt);
  BPK_LAUNCH_CHECK("ns_vel_update");
  return BPK_OK;
}

extern "C" int bpk_ns_pres_update_f32(const float* pres, const float* vel, float* pres_n, int B,
                                      int nx, int ny, float dt, float dx, void* stream) {
  NS_GEO_CHECK(B, nx, ny);
  const Geo g{nx, ny, (int64_t)nx * ny};
  if (B == 0) return BPK_OK;
  hipLaunchKernelGGL(k_pres_update, dim3(grid_for(B * g.hw)), dim3(256), 0,
                     bpk::as_stream(stream), pres, vel, pres_n, B, g, dt, dx);
  BPK_LAUNCH_CHECK("ns_pres_update");
  return BPK_OK;
}

extern "C" int64_t bpk_ns_workspace_bytes(int op, int B, int nx, int ny) {
  const int64_t plane = (int64_t)nx * ny * (int64_t)sizeof(float);
  if (B <= 0 || nx <= 0 || ny <= 0) return 0;
  switch (op) {
    case 0: return 2 * B * plane;  // fx, fy
    case 1: return 8 * B * plane;  // px, py, vel_n (2), du/dv gradients (4)
    default: return 0;
  }
}

extern "C" int bpk_ns_update_density_f32(const float* dens, const float* vel, float* out,
                                         void* workspace, int B, int nx, int ny, float dt,
                                         float dx, void* stream) {
  NS_GEO_CHECK(B, nx, ny);
  if (B == 0) return BPK_OK;
  BPK_REQUIRE(workspace, "ns_update_density: workspace required");
  const int64_t hw = (int64_t)nx * ny;
  float* fx = static_cast<float*>(workspace);
  float* fy = fx + B * hw;
  int rc = bpk_ns_gradient_f32(dens, hw, fx, fy, B, nx, ny, dx, stream);
  if (rc) return rc;
  return bpk_ns_cip_advect_f32(dens, hw, fx, fy, vel, out, B, nx, ny, dt, dx, stream);
}

extern "C" int bpk_ns_update_velocity_f32(const float* vel, const float* pres, float* out,
                                          void* workspace, int B, int nx, int ny, float dt,
                                          float dx, int compat, void* stream) {
  NS_GEO_CHECK(B, nx, ny);
  if (B == 0) return BPK_OK;
  BPK_REQUIRE(workspace, "ns_update_velocity: workspace required");
  const Geo g{nx, ny, (int64_t)nx * ny};
  const int64_t hw = g.hw;
  float* px = static_cast<float*>(workspace);
  float* py = px + B * hw;
  float* vel_n = py + B * hw;
  float* dudx = vel_n + 2 * B * hw;
  float* dudy = dudx + B * hw;
  float* dvdx = dudy + B * hw;
  float* dvdy = dvdx + B * hw;
  int rc = bpk_ns_gradient_f32(pres, hw, px, py, B, nx, ny, dx, stream);
  if (rc) return rc;
  rc = bpk_ns_vel_update_f32(vel, px, py, vel_n, B, nx, ny, dt, stream);
  if (rc) return rc;
  // op/ns_step.cpp:70 -- unbind(vel_n, 1) views read with batch stride hw (compat)
  const int64_t fstride = compat ? hw : 2 * hw;
  const float* ufield = vel_n;
  const float* vfield = vel_n + hw;
  hipStream_t st = bpk::as_stream(stream);
  rc = bpk_ns_gradient_f32(ufield, fstride, dudx, dudy, B, nx, ny, dx, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(k_cip, dim3(grid_for(B * hw)), dim3(256), 0, st, ufield, fstride, dudx, dudy,
                     vel_n, out, 2 * hw, B, g, dt, dx);
  BPK_LAUNCH_CHECK("ns_update_velocity(u)");
  rc = bpk_ns_gradient_f32(vfield, fstride, dvdx, dvdy, B, nx, ny, dx, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(k_cip, dim3(grid_for(B * hw)), dim3(256), 0, st, vfield, fstride, dvdx, dvdy,
                     vel_n, out + hw, 2 * hw, B, g, dt, dx);
  BPK_LAUNCH_CHECK("ns_update_velocity(v)");
  return BPK_OK;
}

extern "C" int bpk_ns_update_pressure_f32(const float* pres, const float* vel, float* out, int B,
                                          int nx, int ny, float dt, float dx, void* stream) {
  return bpk_ns_pres_update_f32(pres, vel, out, B, nx, ny, dt, dx, stream);
}

extern "C" int64_t bpk_ns_full_step_workspace_bytes(int B, int nx, int ny) {
  (void)B;
  (void)nx;
  (void)ny;
  return 0;
}

extern "C" int bpk_ns_full_step_f32(const float* dens, const float* vel, const float* pres,
                                    float* dens_out, float* vel_out, float* pres_out,
                                    void* workspace, int B, int nx, int ny, float dt, float dx,
                                    int compat, void* stream) {
  (void)workspace;
  NS_GEO_CHECK(B, nx, ny);
  if (B == 0) return BPK_OK;
  const Geo g{nx, ny, (int64_t)nx * ny};
  hipStream_t st = bpk::as_stream(stream);
  const int tiles_x = (int)bpk::ceil_div(nx, kTX), tiles_y = (int)bpk::ceil_div(ny, kTY);
  const int64_t tiles = (int64_t)B * tiles_x * tiles_y;
  hipLaunchKernelGGL(k_fused_velocity_lds, dim3((unsigned)std::min<int64_t>(tiles, 1 << 20)),
                     dim3(256), 0, st, vel, pres, vel_out, B, g, dt, dx, compat, tiles_x,
                     tiles_y);
  BPK_LAUNCH_CHECK("ns_full_step(velocity)");
  hipLaunchKernelGGL(k_fused_pres_dens, dim3(grid_for(B * g.hw)), dim3(256), 0, st, dens, pres,
                     vel_out, dens_out, pres_out, B, g, dt, dx);
  BPK_LAUNCH_CHECK("ns_full_step(pressure+density)");
  return BPK_OK;
}
