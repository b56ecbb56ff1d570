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

// ---- reference device helpers (op/ns_step_kernel.cu:50-75) ----
__device__ inline float ddx(const float* f, int x, int y, const Geo& g, float dx) {
  const float* r = f + (int64_t)y * g.nx;
  if (x == 0) return (r[x + 1] - r[x]) / dx;
  if (x == g.nx - 1) return (r[x] - r[x - 1]) / dx;
  return (r[x + 1] - r[x - 1]) / dx / 2;
}
__device__ inline float ddy(const float* f, int x, int y, const Geo& g, float dx) {
  if (y == 0) return (f[(int64_t)(y + 1) * g.nx + x] - f[(int64_t)y * g.nx + x]) / dx;
  if (y == g.ny - 1) return (f[(int64_t)y * g.nx + x] - f[(int64_t)(y - 1) * g.nx + x]) / dx;
  return (f[(int64_t)(y + 1) * g.nx + x] - f[(int64_t)(y - 1) * g.nx + x]) / dx / 2;
}

// CIP advection of one site (op/ns_step_kernel.cu:115-158), operands passed as
// plane pointers so callers can supply stored or recomputed fields.
struct CipIn {
  float f_c, f_ym, f_xm, f_xmym;  // f(x,y) f(x,ym) f(xm,y) f(xm,ym)
  float fx_c, fx_xm, fx_ym;       // fx(x,y) fx(xm,y) fx(x,ym)
  float fy_c, fy_xm, fy_ym;       // fy(x,y) fy(xm,y) fy(x,ym)
};

__device__ inline float cip_site(const CipIn& q, float u, float v, float dt, float dx) {
  const int x_s = sgn(u);
  const int y_s = sgn(v);
  float tmp1 = q.f_c - q.f_ym - q.f_xm + q.f_xmym;
  float tmp2 = q.f_xm - q.f_c;
  float tmp3 = q.f_ym - q.f_c;
  float x_s_denom = x_s * dx * dx * dx;
  float y_s_denom = y_s * dx * dx * dx;
  float a = (x_s * (q.fx_xm + q.fx_c) * dx - 2.0 * (-tmp2)) / x_s_denom;
  float b = (y_s * (q.fy_ym + q.fy_c) * dx - 2.0 * (-tmp3)) / y_s_denom;
  float c = (-tmp1 - x_s * (q.fx_ym - q.fx_c) * dx) / y_s_denom;
  float d = (-tmp1 - y_s * (q.fy_xm - q.fy_c) * dx) / x_s_denom;
  float e = (3.0 * tmp2 + x_s * (q.fx_xm + 2.0 * q.fx_c) * dx) / dx / dx;
  float f = (3.0 * tmp3 + y_s * (q.fy_ym + 2.0 * q.fy_c) * dx) / dx / dx;
  float g = (-(q.fy_xm - q.fy_c) + c * dx * dx) / (x_s * dx);
  float X = -u * dt;
  float Y = -v * dt;
  return ((a * X + c * Y + e) * X + g * Y + q.fx_c) * X + ((b * Y + d * X + f) * Y + q.fy_c) * Y +
         q.f_c;
}

__device__ inline float pres_site(float p_xd, float p_xu, float p_yd, float p_yu, float u_xu,
                                  float u_xd, float v_xu, float v_xd, float u_yu, float u_yd,
                                  float v_yu, float v_yd, float dt, float dx) {
  // sub_x = V(xu) - V(xd), sub_y = V(yu) - V(yd)   (op/ns_step_kernel.cu:219-231)
  float sxx = u_xu - u_xd, sxy = v_xu - v_xd;
  float syx = u_yu - u_yd, syy = v_yu - v_yd;
  float aver_p = 0.25 * (p_xd + p_xu + p_yd + p_yu);
  float pred_p = aver_p + (sxx * sxx + syy * syy + (syx * sxy)) / 8.0 - dx * (sxx + syy) / (8 * dt);
  return pred_p;
}

// ---------------------------------------------------------------- low-level kernels

__global__ __launch_bounds__(256) void k_gradient(const float* __restrict__ f, int64_t fstride,
                                                  float* __restrict__ fx, float* __restrict__ fy,
                                                  int B, Geo g, float dx) {
  const int64_t total = (int64_t)B * g.hw;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / g.hw;
    const int s = (int)(i - b * g.hw);
    const int y = s / g.nx, x = s - y * g.nx;
    const float* fp = f + b * fstride;
    fx[i] = ddx(fp, x, y, g, dx);
    fy[i] = ddy(fp, x, y, g, dx);
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
    out[b * ostride + s] = cip_site(q, u, v, dt, dx);
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
                          u[iyd], v[iyu], v[iyd], dt, dx);
  }
}

// ---------------------------------------------------------------- fused full step
// Stage A (per site of sample b): vel' = CIP advection of the vel_n planes, where
// vel_n = vel - dt grad(p) is recomputed on the fly (bit-identical to storing it).
// The advected "u" field of batch b is vel_n plane  uplane(b) and the "v" field
// plane vplane(b):  compat -> (b, b+1)  (reference unbind quirk), else (2b, 2b+1).

struct VelN {
  const float* vel;
  const float* pres;
  Geo g;
  float dt, dx;
  // vel_n value of memory plane k at (x,y): plane k = sample k>>1, component k&1
  __device__ inline float at(int64_t k, int x, int y) const {
    const float* p = pres + (k >> 1) * g.hw;
    const float grad = (k & 1) ? ddy(p, x, y, g, dx) : ddx(p, x, y, g, dx);
    return vel[k * g.hw + (int64_t)y * g.nx + x] - grad * dt;
  }
  // reference diff_x / diff_y of the vel_n plane k
  __device__ inline float dfx(int64_t k, int x, int y) const {
    if (x == 0) return (at(k, x + 1, y) - at(k, x, y)) / dx;
    if (x == g.nx - 1) return (at(k, x, y) - at(k, x - 1, y)) / dx;
    return (at(k, x + 1, y) - at(k, x - 1, y)) / dx / 2;
  }
  __device__ inline float dfy(int64_t k, int x, int y) const {
    if (y == 0) return (at(k, x, y + 1) - at(k, x, y)) / dx;
    if (y == g.ny - 1) return (at(k, x, y) - at(k, x, y - 1)) / dx;
    return (at(k, x, y + 1) - at(k, x, y - 1)) / dx / 2;
  }
  __device__ inline float cip(int64_t k, int x, int y, float u, float v) const {
    const int xm = clampx(x - sgn(u), g.nx);
    const int ym = clampx(y - sgn(v), g.ny);
    CipIn q;
    q.f_c = at(k, x, y);
    q.f_ym = at(k, x, ym);
    q.f_xm = at(k, xm, y);
    q.f_xmym = at(k, xm, ym);
    q.fx_c = dfx(k, x, y);
    q.fx_xm = dfx(k, xm, y);
    q.fx_ym = dfx(k, x, ym);
    q.fy_c = dfy(k, x, y);
    q.fy_xm = dfy(k, xm, y);
    q.fy_ym = dfy(k, x, ym);
    return cip_site(q, u, v, dt, dx);
  }
};

__global__ __launch_bounds__(256) void k_fused_velocity(const float* __restrict__ vel,
                                                        const float* __restrict__ pres,
                                                        float* __restrict__ vel_out, int B, Geo g,
                                                        float dt, float dx, int compat) {
  const VelN vn{vel, pres, g, dt, dx};
  const int64_t total = (int64_t)B * g.hw;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / g.hw;
    const int s = (int)(i - b * g.hw);
    const int y = s / g.nx, x = s - y * g.nx;
    const float u = vn.at(2 * b, x, y);
    const float v = vn.at(2 * b + 1, x, y);
    const int64_t up = compat ? b : 2 * b;
    const int64_t vp = compat ? b + 1 : 2 * b + 1;
    vel_out[(2 * b) * g.hw + s] = vn.cip(up, x, y, u, v);
    vel_out[(2 * b + 1) * g.hw + s] = vn.cip(vp, x, y, u, v);
  }
}

// Stage B: pres' = pressure update with vel'; dens' = CIP(dens) with vel'.
__global__ __launch_bounds__(256) void k_fused_pres_dens(const float* __restrict__ dens,
                                                         const float* __restrict__ pres,
                                                         const float* __restrict__ vel1,
                                                         float* __restrict__ dens_out,
                                                         float* __restrict__ pres_out, int B,
                                                         Geo g, float dt, float dx) {
  const int64_t total = (int64_t)B * g.hw;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
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
                              u[iyu], u[iyd], v[iyu], v[iyd], dt, dx);
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
    q.fx_c = ddx(f, x, y, g, dx);
    q.fx_xm = ddx(f, xm, y, g, dx);
    q.fx_ym = ddx(f, x, ym, g, dx);
    q.fy_c = ddy(f, x, y, g, dx);
    q.fy_xm = ddy(f, xm, y, g, dx);
    q.fy_ym = ddy(f, x, ym, g, dx);
    dens_out[i] = cip_site(q, uc, vc, dt, dx);
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
  hipLaunchKernelGGL(k_fused_velocity, dim3(grid_for(B * g.hw)), dim3(256), 0, st, vel, pres,
                     vel_out, B, g, dt, dx, compat);
  BPK_LAUNCH_CHECK("ns_full_step(velocity)");
  hipLaunchKernelGGL(k_fused_pres_dens, dim3(grid_for(B * g.hw)), dim3(256), 0, st, dens, pres,
                     vel_out, dens_out, pres_out, B, g, dt, dx);
  BPK_LAUNCH_CHECK("ns_full_step(pressure+density)");
  return BPK_OK;
}
