/*
 * ORACLE (test infrastructure only) -- ns_step restated in plain C.
 *
 * Follows op/ns_step_kernel.cu:30-234 (device helpers and kernels) and the op
 * sequencing of op/ns_step.cpp:45-102, expression for expression, including the
 * double-precision promotions caused by the reference's `2.0`, `3.0`, `0.25`
 * and `8.0` literals.  Build with -ffp-contract=off (oracle/Makefile) so every
 * operation rounds exactly once, as IEEE-754 prescribes; the gfx950 kernels
 * (csrc/ns_step.hip) are compiled the same way and must match bit for bit.
 *
 * Plane convention (reference): f[y * nx + x], x < nx = size(2), y < ny = size(3).
 * No runnable reference exists here (CUDA-only extension); pinned by analytic
 * known-answer tests in tests/test_oracle_ns_step.py.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  int nx, ny;
} geo_t;

static float get(const float* f, int x, int y, geo_t g) { return f[(int64_t)y * g.nx + x]; }

static float diff_x(const float* f, int x, int y, geo_t g, float dx) {
  if (x == 0) return (get(f, x + 1, y, g) - get(f, x, y, g)) / dx;
  if (x == g.nx - 1) return (get(f, x, y, g) - get(f, x - 1, y, g)) / dx;
  return (get(f, x + 1, y, g) - get(f, x - 1, y, g)) / dx / 2;
}

static float diff_y(const float* f, int x, int y, geo_t g, float dx) {
  if (y == 0) return (get(f, x, y + 1, g) - get(f, x, y, g)) / dx;
  if (y == g.ny - 1) return (get(f, x, y, g) - get(f, x, y - 1, g)) / dx;
  return (get(f, x, y + 1, g) - get(f, x, y - 1, g)) / dx / 2;
}

static int mirror(int v, int n) { return v < 0 ? -v : (v > n - 1 ? 2 * n - 2 - v : v); }

static int sign_of(float v) {
  if (v < 0.0) return -1;
  if (v > 0.0) return 1;
  return 0;
}

/* gradient of B planes of f (plane stride fs) into contiguous fx, fy */
void ns_ref_gradient(const float* f, int64_t fs, float* fx, float* fy, int B, int nx, int ny,
                     float dx) {
  geo_t g = {nx, ny};
  int64_t hw = (int64_t)nx * ny;
  for (int b = 0; b < B; ++b)
    for (int y = 0; y < ny; ++y)
      for (int x = 0; x < nx; ++x) {
        fx[b * hw + (int64_t)y * nx + x] = diff_x(f + b * fs, x, y, g, dx);
        fy[b * hw + (int64_t)y * nx + x] = diff_y(f + b * fs, x, y, g, dx);
      }
}

/* CIP advection (op/ns_step_kernel.cu:115-158): out[b] (plane stride os) */
void ns_ref_cip(const float* fc, int64_t fs, const float* fdx, const float* fdy, const float* vel,
                float* out, int64_t os, int B, int nx, int ny, float dt, float dx) {
  geo_t g = {nx, ny};
  int64_t hw = (int64_t)nx * ny;
  for (int b = 0; b < B; ++b) {
    const float* f = fc + b * fs;
    const float* gx = fdx + b * hw;
    const float* gy = fdy + b * hw;
    const float* u = vel + (int64_t)(2 * b) * hw;
    const float* v = vel + (int64_t)(2 * b + 1) * hw;
    for (int y = 0; y < ny; ++y)
      for (int x = 0; x < nx; ++x) {
        int x_s = sign_of(get(u, x, y, g));
        int y_s = sign_of(get(v, x, y, g));
        int x_m = mirror(x - x_s, nx);
        int y_m = mirror(y - y_s, ny);
        float tmp1 = get(f, x, y, g) - get(f, x, y_m, g) - get(f, x_m, y, g) + get(f, x_m, y_m, g);
        float tmp2 = get(f, x_m, y, g) - get(f, x, y, g);
        float tmp3 = get(f, x, y_m, g) - get(f, x, y, g);
        float x_s_denom = x_s * dx * dx * dx;
        float y_s_denom = y_s * dx * dx * dx;
        float a = (x_s * (get(gx, x_m, y, g) + get(gx, x, y, g)) * dx - 2.0 * (-tmp2)) / x_s_denom;
        float bb = (y_s * (get(gy, x, y_m, g) + get(gy, x, y, g)) * dx - 2.0 * (-tmp3)) / y_s_denom;
        float c = (-tmp1 - x_s * (get(gx, x, y_m, g) - get(gx, x, y, g)) * dx) / y_s_denom;
        float d = (-tmp1 - y_s * (get(gy, x_m, y, g) - get(gy, x, y, g)) * dx) / x_s_denom;
        float e = (3.0 * tmp2 + x_s * (get(gx, x_m, y, g) + 2.0 * get(gx, x, y, g)) * dx) / dx / dx;
        float ff = (3.0 * tmp3 + y_s * (get(gy, x, y_m, g) + 2.0 * get(gy, x, y, g)) * dx) / dx / dx;
        float gg = (-(get(gy, x_m, y, g) - get(gy, x, y, g)) + c * dx * dx) / (x_s * dx);
        float X = -get(u, x, y, g) * dt;
        float Y = -get(v, x, y, g) * dt;
        out[b * os + (int64_t)y * nx + x] =
            ((a * X + c * Y + e) * X + gg * Y + get(gx, x, y, g)) * X +
            ((bb * Y + d * X + ff) * Y + get(gy, x, y, g)) * Y + get(f, x, y, g);
      }
  }
}

/* velocity_update_kernel (:181-202) */
void ns_ref_vel_update(const float* vel, const float* px, const float* py, float* vel_n, int B,
                       int nx, int ny, float dt) {
  int64_t hw = (int64_t)nx * ny;
  for (int b = 0; b < B; ++b)
    for (int64_t s = 0; s < hw; ++s) {
      vel_n[(2 * b) * hw + s] = vel[(2 * b) * hw + s] - px[b * hw + s] * dt;
      vel_n[(2 * b + 1) * hw + s] = vel[(2 * b + 1) * hw + s] - py[b * hw + s] * dt;
    }
}

/* pressure_update_kernel (:205-234) */
void ns_ref_pressure(const float* pres, const float* vel, float* out, int B, int nx, int ny,
                     float dt, float dx) {
  geo_t g = {nx, ny};
  int64_t hw = (int64_t)nx * ny;
  for (int b = 0; b < B; ++b) {
    const float* p = pres + b * hw;
    const float* u = vel + (int64_t)(2 * b) * hw;
    const float* v = vel + (int64_t)(2 * b + 1) * hw;
    for (int y = 0; y < ny; ++y)
      for (int x = 0; x < nx; ++x) {
        int x_u = mirror(x + 1, nx), x_d = mirror(x - 1, nx);
        int y_u = mirror(y + 1, ny), y_d = mirror(y - 1, ny);
        float sub_x_x = get(u, x_u, y, g) - get(u, x_d, y, g);
        float sub_x_y = get(v, x_u, y, g) - get(v, x_d, y, g);
        float sub_y_x = get(u, x, y_u, g) - get(u, x, y_d, g);
        float sub_y_y = get(v, x, y_u, g) - get(v, x, y_d, g);
        float aver_p = 0.25 * (get(p, x_d, y, g) + get(p, x_u, y, g) + get(p, x, y_d, g) +
                               get(p, x, y_u, g));
        float pred_p = aver_p + (sub_x_x * sub_x_x + sub_y_y * sub_y_y + (sub_y_x * sub_x_y)) / 8.0 -
                       dx * (sub_x_x + sub_y_y) / (8 * dt);
        out[b * hw + (int64_t)y * nx + x] = pred_p;
      }
  }
}

/* ns_step.cpp:45-57 */
void ns_ref_update_density(const float* dens, const float* vel, float* out, int B, int nx, int ny,
                           float dt, float dx) {
  int64_t hw = (int64_t)nx * ny;
  float* fx = (float*)malloc(sizeof(float) * B * hw);
  float* fy = (float*)malloc(sizeof(float) * B * hw);
  ns_ref_gradient(dens, hw, fx, fy, B, nx, ny, dx);
  ns_ref_cip(dens, hw, fx, fy, vel, out, hw, B, nx, ny, dt, dx);
  free(fx);
  free(fy);
}

/* ns_step.cpp:59-92; compat = 1 reproduces the unbind-stride read of :70 */
void ns_ref_update_velocity(const float* vel, const float* pres, float* out, int B, int nx, int ny,
                            float dt, float dx, int compat) {
  int64_t hw = (int64_t)nx * ny;
  float* px = (float*)malloc(sizeof(float) * B * hw);
  float* py = (float*)malloc(sizeof(float) * B * hw);
  float* vel_n = (float*)malloc(sizeof(float) * 2 * B * hw);
  float* gx = (float*)malloc(sizeof(float) * B * hw);
  float* gy = (float*)malloc(sizeof(float) * B * hw);
  ns_ref_gradient(pres, hw, px, py, B, nx, ny, dx);
  ns_ref_vel_update(vel, px, py, vel_n, B, nx, ny, dt);
  int64_t fs = compat ? hw : 2 * hw;
  ns_ref_gradient(vel_n, fs, gx, gy, B, nx, ny, dx);
  ns_ref_cip(vel_n, fs, gx, gy, vel_n, out, 2 * hw, B, nx, ny, dt, dx);
  ns_ref_gradient(vel_n + hw, fs, gx, gy, B, nx, ny, dx);
  ns_ref_cip(vel_n + hw, fs, gx, gy, vel_n, out + hw, 2 * hw, B, nx, ny, dt, dx);
  free(px);
  free(py);
  free(vel_n);
  free(gx);
  free(gy);
}

/* advect_kernel (:161-178), method 1 -- never selected by the reference ops */
void ns_ref_advect(const float* f, const float* fx, const float* fy, const float* vel, float* out,
                   int B, int nx, int ny, float dt) {
  int64_t hw = (int64_t)nx * ny;
  for (int b = 0; b < B; ++b)
    for (int64_t s = 0; s < hw; ++s) {
      float advect = vel[(2 * b) * hw + s] * fx[b * hw + s] + vel[(2 * b + 1) * hw + s] * fy[b * hw + s];
      out[b * hw + s] = f[b * hw + s] - dt * advect;
    }
}
