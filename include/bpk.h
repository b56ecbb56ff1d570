/*
 * bpk.h -- C ABI of the MI355X-native (gfx950) hot-path library `libbpk.so`.
 *
 * This is the drop-in boundary for the hot path of XDzzzzzZyq/b-pinn-kalman-filter
 * (score-SDE training / PC sampling + PINN / Navier-Stokes stencil).  Each entry
 * point replaces one native op of the reference's `op/` package; the citation on
 * each block names the reference interface it replaces (paths relative to the
 * reference repository root).
 *
 * Conventions (all entry points):
 *   - plain device pointers, element counts / sizes, and a `hipStream_t` passed as
 *     `void* stream` (the caller's current stream; 0 = legacy default stream);
 *   - all ops are out-of-place and asynchronous on `stream`; nothing allocates;
 *     where scratch memory is needed the caller passes it (size queried with the
 *     matching `*_workspace_bytes` function) -- so every call is graph-capturable;
 *   - return BPK_OK (0) on success; otherwise an error code, and
 *     bpk_last_error() returns a thread-local human-readable message.  The
 *     reference raised c10::Error -> Python RuntimeError from TORCH_CHECK
 *     (op/upfirdn2d.cpp:8,15-16); the Python host maps a nonzero status to
 *     RuntimeError the same way.
 *   - tensors are dense row-major (C-contiguous) unless a stride argument says
 *     otherwise.
 */
#ifndef BPK_H_
#define BPK_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BPK_OK 0
#define BPK_ERR_ARG 1
#define BPK_ERR_LAUNCH 2
#define BPK_ERR_UNSUPPORTED 3

#define BPK_ABI_VERSION 1

/* Thread-local message of the last failed call on this thread. */
const char* bpk_last_error(void);
/* Returns BPK_ABI_VERSION. */
int bpk_abi_version(void);


/* ------------------------------------------------------------------------- *
 * upfirdn2d: zero-insert upsample by (up_x, up_y), pad (negative = crop),
 * true 2-D convolution with `kernel` [kernel_h, kernel_w] (i.e. correlation with
 * the flipped taps), then keep every (down_x, down_y)-th sample.
 *   x   : [major, in_h, in_w, minor]
 *   out : [major, out_h, out_w, minor],
 *         out_h = (in_h*up_y + pad_y0 + pad_y1 - kernel_h) / down_y + 1 (same for w)
 * Replaces `upfirdn2d_op.upfirdn2d(input, kernel, up_x, up_y, down_x, down_y,
 * pad_x0, pad_x1, pad_y0, pad_y1)` -- op/upfirdn2d.cpp:12-22 and its CUDA host
 * op/upfirdn2d_kernel.cu:209-369.  The adjoint (backward) is the same entry
 * with up<->down, the flipped kernel and the g_pad of op/upfirdn2d.py:111-116.
 * ------------------------------------------------------------------------- */
int bpk_upfirdn2d_f32(const float* x, const float* kernel, float* out, int major, int in_h,
                      int in_w, int minor, int kernel_h, int kernel_w, int up_x, int up_y,
                      int down_x, int down_y, int pad_x0, int pad_x1, int pad_y0, int pad_y1,
                      int out_h, int out_w, void* stream);
int bpk_upfirdn2d_f64(const double* x, const double* kernel, double* out, int major, int in_h,
                      int in_w, int minor, int kernel_h, int kernel_w, int up_x, int up_y,
                      int down_x, int down_y, int pad_x0, int pad_x1, int pad_y0, int pad_y1,
                      int out_h, int out_w, void* stream);

/* ------------------------------------------------------------------------- *
 * fused_bias_act: out = scale * act(x + bias[(i / step_b) % size_b]), act in
 * {1: linear, 3: leaky-relu(alpha)}; grad = 1 selects the derivative mask from
 * `refer` (out > 0 ? 1 : alpha); grad = 2 writes zeros.  `bias` / `refer` may be
 * NULL (numel 0 in the reference).  Replaces `fused.fused_bias_act(input, bias,
 * refer, act, grad, alpha, scale)` -- op/fused_bias_act.cpp:11-20,
 * op/fused_bias_act_kernel.cu:18-98.
 * ------------------------------------------------------------------------- */
int bpk_fused_bias_act_f32(const float* x, const float* bias, const float* refer, float* out,
                           int64_t n, int64_t step_b, int64_t size_b, int act, int grad,
                           float alpha, float scale, void* stream);
int bpk_fused_bias_act_f64(const double* x, const double* bias, const double* refer, double* out,
                           int64_t n, int64_t step_b, int64_t size_b, int act, int grad,
                           double alpha, double scale, void* stream);

/* ------------------------------------------------------------------------- *
 * grid_sample 2-D, bilinear, padding_mode 0 = zeros / 1 = border.
 *   input [N, C, H_in, W_in], grid [N, H_out, W_out, 2], out [N, C, H_out, W_out]
 * fwd/bwd replace the ATen calls of op/grid_sample.py:39-60; grad2 replaces
 * `gridsample_grad2.grad2_2d(...)` -- op/grid_sample.cpp:26-57,
 * op/grid_sample_kernel.cu:27-210 and 536-599.
 * bwd: grad_input (may be NULL) must be zero-filled by the caller (atomics);
 *      grad_grid (may be NULL) is overwritten.
 * grad2: outputs grad_grad_output (overwritten), grad_input (zero-filled by the
 *      caller, atomics), grad_grid (overwritten); g2_input / g2_grid may be NULL (an
 *      all-zero incoming gradient, the None autograd passes).
 * ------------------------------------------------------------------------- */
int bpk_grid_sample2d_fwd_f32(const float* input, const float* grid, float* out, int N, int C,
                              int H_in, int W_in, int H_out, int W_out, int padding_mode,
                              int align_corners, void* stream);
int bpk_grid_sample2d_bwd_f32(const float* grad_out, const float* input, const float* grid,
                              float* grad_input, float* grad_grid, int N, int C, int H_in,
                              int W_in, int H_out, int W_out, int padding_mode, int align_corners,
                              void* stream);
int bpk_grid_sample2d_grad2_f32(const float* g2_input, const float* g2_grid,
                                const float* grad_out, const float* input, const float* grid,
                                float* grad_grad_out, float* grad_input, float* grad_grid, int N,
                                int C, int H_in, int W_in, int H_out, int W_out, int padding_mode,
                                int align_corners, void* stream);
int bpk_grid_sample2d_fwd_f64(const double* input, const double* grid, double* out, int N, int C,
                              int H_in, int W_in, int H_out, int W_out, int padding_mode,
                              int align_corners, void* stream);
int bpk_grid_sample2d_bwd_f64(const double* grad_out, const double* input, const double* grid,
                              double* grad_input, double* grad_grid, int N, int C, int H_in,
                              int W_in, int H_out, int W_out, int padding_mode, int align_corners,
                              void* stream);
int bpk_grid_sample2d_grad2_f64(const double* g2_input, const double* g2_grid,
                                const double* grad_out, const double* input, const double* grid,
                                double* grad_grad_out, double* grad_input, double* grad_grid, int N,
                                int C, int H_in, int W_in, int H_out, int W_out, int padding_mode,
                                int align_corners, void* stream);

/* ------------------------------------------------------------------------- *
 * grid_sample_3d (trilinear) -- replaces F.grid_sample on 5-D tensors and
 * aten::grid_sampler_3d_backward as op/grid_sample.py:79-113 calls them, and
 * gridsample_grad2.grad2_3d (op/grid_sample.cpp:42-57, op/grid_sample_kernel.cu:212-533,
 * host 601-666).  input [N, C, D, H, W], grid [N, Do, Ho, Wo, 3] (x, y, z), contiguous;
 * same output conventions as the 2-D entries (grad_input zero-filled by the caller).
 * ------------------------------------------------------------------------- */
int bpk_grid_sample3d_fwd_f32(const float* input, const float* grid, float* out, int N, int C,
                              int D, int H, int W, int Do, int Ho, int Wo, int padding_mode,
                              int align_corners, void* stream);
int bpk_grid_sample3d_bwd_f32(const float* grad_out, const float* input, const float* grid,
                              float* grad_input, float* grad_grid, int N, int C, int D, int H,
                              int W, int Do, int Ho, int Wo, int padding_mode, int align_corners,
                              void* stream);
int bpk_grid_sample3d_grad2_f32(const float* g2_input, const float* g2_grid, const float* grad_out,
                                const float* input, const float* grid, float* grad_grad_out,
                                float* grad_input, float* grad_grid, int N, int C, int D, int H,
                                int W, int Do, int Ho, int Wo, int padding_mode, int align_corners,
                                void* stream);
int bpk_grid_sample3d_fwd_f64(const double* input, const double* grid, double* out, int N, int C,
                              int D, int H, int W, int Do, int Ho, int Wo, int padding_mode,
                              int align_corners, void* stream);
int bpk_grid_sample3d_bwd_f64(const double* grad_out, const double* input, const double* grid,
                              double* grad_input, double* grad_grid, int N, int C, int D, int H,
                              int W, int Do, int Ho, int Wo, int padding_mode, int align_corners,
                              void* stream);
int bpk_grid_sample3d_grad2_f64(const double* g2_input, const double* g2_grid,
                                const double* grad_out, const double* input, const double* grid,
                                double* grad_grad_out, double* grad_input, double* grad_grid,
                                int N, int C, int D, int H, int W, int Do, int Ho, int Wo,
                                int padding_mode, int align_corners, void* stream);

/* ------------------------------------------------------------------------- *
 * ns_step: explicit 2-D incompressible-flow step on B planes.
 * Memory convention follows the reference exactly (op/ns_step_kernel.cu:30-37):
 * a plane is addressed as field[y * nx + x] with nx = tensor.size(2) (the
 * contiguous axis) and ny = tensor.size(3); scalar fields [B,1,.,.] have plane
 * stride nx*ny, velocity [B,2,.,.] has its u / v planes at (2b) / (2b+1).
 * Arithmetic mirrors op/ns_step_kernel.cu:50-234 operation for operation
 * (including the double-precision promotions of its `2.0`, `3.0`, `0.25`,
 * `8.0` literals), compiled without FMA contraction, so it is bit-identical to
 * the C oracle restatement (oracle/ns_step_ref.c).
 *
 * Low-level kernels (replace the device kernels of op/ns_step_kernel.cu):
 *   gradient  : fx, fy <- central differences of f          (:97-112)
 *   cip_advect: out <- CIP advection of f by vel            (:115-158)
 *   advect    : out <- f - dt (u fx + v fy)                 (:161-178)
 *   vel_update: vel_n <- vel - dt grad(p)                   (:181-202)
 *   pres_update: pres_n <- Jacobi-like pressure update      (:205-234)
 * `f_plane_stride` is the element distance between consecutive batch planes of f.
 *
 * High-level ops (replace ns_step_forward.update_{density,velocity,pressure},
 * op/ns_step.cpp:45-102).  update_velocity with compat = 1 reproduces the
 * reference's unbind-stride quirk (op/ns_step.cpp:70: the u / v views of vel_n
 * are read with batch stride nx*ny instead of 2*nx*ny); compat = 0 reads the
 * intended planes.  Scratch: bpk_ns_workspace_bytes(op, B, nx, ny) bytes
 * (op: 0 = density, 1 = velocity, 2 = pressure).
 * ------------------------------------------------------------------------- */
int bpk_ns_gradient_f32(const float* f, int64_t f_plane_stride, float* fx, float* fy, int B, int nx,
                        int ny, float dx, void* stream);
int bpk_ns_cip_advect_f32(const float* f, int64_t f_plane_stride, const float* fx, const float* fy,
                          const float* vel, float* out, int B, int nx, int ny, float dt, float dx,
                          void* stream);
int bpk_ns_advect_f32(const float* f, int64_t f_plane_stride, const float* fx, const float* fy,
                      const float* vel, float* out, int B, int nx, int ny, float dt, void* stream);
int bpk_ns_vel_update_f32(const float* vel, const float* px, const float* py, float* vel_n, int B,
                          int nx, int ny, float dt, void* stream);
int bpk_ns_pres_update_f32(const float* pres, const float* vel, float* pres_n, int B, int nx, int ny,
                           float dt, float dx, void* stream);
/* Adjoint of bpk_ns_gradient_f32 (the reference's diff_x / diff_y stencil, one-sided at
 * the borders): out = Dx^T gx + Dy^T gy on B contiguous planes.  Lets autograd
 * differentiate through the stencil (the PINN finite-difference residual,
 * pinn_kalman/pinn.py equation_mse_fd); no reference counterpart. */
int bpk_ns_gradient_adjoint_f32(const float* gx, const float* gy, float* out, int B, int nx,
                                int ny, float dx, void* stream);
int64_t bpk_ns_workspace_bytes(int op, int B, int nx, int ny);
int bpk_ns_update_density_f32(const float* dens, const float* vel, float* out, void* workspace,
                              int B, int nx, int ny, float dt, float dx, void* stream);
int bpk_ns_update_velocity_f32(const float* vel, const float* pres, float* out, void* workspace,
                               int B, int nx, int ny, float dt, float dx, int compat, void* stream);
int bpk_ns_update_pressure_f32(const float* pres, const float* vel, float* out, int B, int nx,
                               int ny, float dt, float dx, void* stream);
/* One whole simulator step (pinn_kalman/simulator.py:55-57): vel' =
 * update_velocity(vel, pres); pres' = update_pressure(pres, vel'); dens' =
 * update_density(dens, vel'), fused into LDS-tiled kernels.  Results equal the
 * three calls above bit for bit. */
int64_t bpk_ns_full_step_workspace_bytes(int B, int nx, int ny);
int bpk_ns_full_step_f32(const float* dens, const float* vel, const float* pres, float* dens_out,
                         float* vel_out, float* pres_out, void* workspace, int B, int nx, int ny,
                         float dt, float dx, int compat, void* stream);

/* ------------------------------------------------------------------------- *
 * GroupNorm (+ optional fused per-(n,c) bias before the norm and SiLU after).
 * The build's fusion of nn.GroupNorm + act + `h += Dense(temb)[:, :, None, None]`
 * of models/layerspp.py:242-274 (ResnetBlockBigGANpp) and :200-209.
 *   x [N, C, HW] (NCHW), bias_nc [N, C] or NULL, gamma/beta [C] or NULL,
 *   y [N, C, HW]; mean/rstd [N, G] (may be NULL in fwd).  act: 0 none, 1 silu.
 * bwd: dx [N,C,HW]; dgamma_nc / dbeta_nc [N, C] per-sample partial sums
 * (reduce over N on the host); may be NULL.
 * ------------------------------------------------------------------------- */
int64_t bpk_group_norm_workspace_bytes(int N, int C, int64_t HW, int G);
int bpk_group_norm_fwd_f32(const float* x, const float* bias_nc, const float* gamma,
                           const float* beta, float* y, float* mean, float* rstd, void* workspace,
                           int N, int C, int64_t HW, int G, float eps, int act, void* stream);
/* Statistics of GroupNorm(x + bias_nc) folded into a per-(n, c) affine form:
 * scale_shift[n][c] = (s, t) with act(GN(x + b)) == act(x * s + t); s = rstd * gamma[c],
 * t = beta[c] + (b[n, c] - mean) * s.  One read of x.  Consumed by the Winograd conv's
 * fused prologue (bpk_conv3x3_wino_pre_f32) so the normalized tensor is never stored.
 * workspace: bpk_group_norm_workspace_bytes(N, C, HW, G). */
int bpk_group_norm_affine_f32(const float* x, const float* bias_nc, const float* gamma,
                              const float* beta, float* scale_shift, void* workspace, int N, int C,
                              int64_t HW, int G, float eps, void* stream);
/* Same, also writing the group statistics mean / rstd [N, G] the affine form was built from
 * (may be NULL): the GroupNorm backward (bpk_group_norm_bwd_f32) of a conv that applied the
 * normalization in its input load under autograd (op.norm_act.group_norm_affine_stats). */
int bpk_group_norm_affine_stats_f32(const float* x, const float* bias_nc, const float* gamma,
                                    const float* beta, float* scale_shift, float* mean,
                                    float* rstd, void* workspace, int N, int C, int64_t HW, int G,
                                    float eps, void* stream);
/* The same affine form from per-(n, channel, region) partial statistics written by the
 * producer of x (bpk_conv3x3_wino_ex_f32): part [N, C, R, 2] = (mean, M2) of cnt values
 * each; no pass over x.  Deterministic (fixed reduction order). */
int bpk_group_norm_affine_partials_f32(const float* part, int R, int cnt, const float* bias_nc,
                                       const float* gamma, const float* beta, float* scale_shift,
                                       int N, int C, int G, float eps, void* stream);
/* Same, also writing mean / rstd [N, G] (may be NULL). */
int bpk_group_norm_affine_partials_stats_f32(const float* part, int R, int cnt,
                                             const float* bias_nc, const float* gamma,
                                             const float* beta, float* scale_shift, float* mean,
                                             float* rstd, int N, int C, int G, float eps,
                                             void* stream);
/* Same for the channel concatenation [x1 (C1 channels), x2 (C - C1)] from the two tensors'
 * own partials (part [N, C1, R, 2], part2 [N, C - C1, R, 2]) -- the up path's
 * torch.cat([h, hs.pop()], 1) (reference models/ncsnpp.py:318) without concatenating
 * either; bit-identical to the single-source entry on the concatenated partials. */
int bpk_group_norm_affine_partials2_f32(const float* part, int C1, const float* part2, int R,
                                        int cnt, const float* bias_nc, const float* gamma,
                                        const float* beta, float* scale_shift, int N, int C,
                                        int G, float eps, void* stream);
/* Partial statistics for a tensor whose producer wrote none: part [N, C, HW / 128, 2] =
 * (mean, M2) of each run of 128 consecutive pixels (HW % 128 == 0), the form both entries
 * above consume (R = HW / 128, cnt = 128).  One read of x. */
int bpk_group_norm_chunk_partials_f32(const float* x, float* part, int N, int C, int64_t HW,
                                      void* stream);
/* y = silu(x * s + t) with scale_shift[n][c] = (s, t): the activation the Winograd conv's
 * GroupNorm prologue computes, materialised for the conv's weight gradient under autograd
 * (same arithmetic as the prologue). */
int bpk_affine_silu_f32(const float* x, const float* scale_shift, float* y, int N, int C,
                        int64_t HW, void* stream);
int bpk_group_norm_bwd_f32(const float* dy, const float* x, const float* bias_nc,
                           const float* gamma, const float* beta, const float* mean,
                           const float* rstd, float* dx, float* dgamma_nc, float* dbeta_nc,
                           void* workspace, int N, int C, int64_t HW, int G, int act,
                           void* stream);
/* The same backward with dx = addend + (the GroupNorm backward) when addend [N, C, HW] is not
 * NULL: another consumer's gradient of x (a residual block's identity skip) added in the same
 * pass instead of by a separate accumulation -- the same fp32 sum the autograd engine forms. */
int bpk_group_norm_bwd_add_f32(const float* dy, const float* x, const float* bias_nc,
                               const float* gamma, const float* beta, const float* mean,
                               const float* rstd, const float* addend, float* dx, float* dgamma_nc,
                               float* dbeta_nc, void* workspace, int N, int C, int64_t HW, int G,
                               int act, void* stream);
/* The parameter gradients behind that backward in one launch (NULL outputs skipped):
 * d_bias_nc [N, C] = sum over the plane of dx [N, C, HW]; dgamma / dbeta [C] = sum over n of
 * its dgamma_nc / dbeta_nc [N, C].  Fixed summation order. */
int bpk_group_norm_param_grads_f32(const float* dx, const float* dgamma_nc, const float* dbeta_nc,
                                   float* d_bias_nc, float* dgamma, float* dbeta, int N, int C,
                                   int64_t HW, void* stream);

/* out[n, 0] = u[n, 1] / c0, out[n, 1] = u[n, 0] / c1 for u, out [N, 2, P] (distinct buffers;
 * channels_last != 0: both stored [N, P, 2]):
 * the flow-component swap + scale of FlowNet's project (reference models/flownet.py:8-25,
 * torch.cat([u[:, 1:2] / c0, u[:, 0:1] / c1], 1)); a tensor-by-scalar division as aten runs it
 * (times the fp32 reciprocal 1.f / c): bit-identical. */
int bpk_swap_scale_f32(const float* u, float* out, int64_t N, int64_t P, float c0, float c1,
                       int channels_last, void* stream);
/* y [planes, H, W] = the 2 x 2 block sums of x [planes, 2H, 2W]: the adjoint of the nearest
 * x2 upsample (the `ddpm` net's Upsample(with_conv=True), reference layers.py:576-590, under
 * autograd -- the input gradient of bpk_conv3x3_wino_up2_f32's fused upsample + conv). */
int bpk_sum2x2_f32(const float* x, float* y, int64_t planes, int H, int W, void* stream);

/* The PINN nets' spatial embedding f = (sin(w |(x, y)|) + sin(w |(mx - x, my - y)|)) / s,
 * mx / my the max of x / y over each of k copies of the batch (reference models/layers.py:
 * 517-521, get_spatial_embedding; copies: pinn.PINN.forward_residual_copies), with its first
 * (vjp: (g f_x, g f_y) + the max's evenly shared gradient) and second derivatives (vjp2: the
 * cotangent (hx, hy) of the vjp's outputs mapped to (dg, dx, dy); hx / hy / dg / dx / dy may be
 * NULL) -- one reduction launch + one elementwise launch each, the forward bit-identical to the
 * reference's aten op sequence.  x, y, out, g, ... hold n floats; n / k must be a multiple of
 * 256 (bpk_spatial_emb_supported); mxy [k][2] is written by the forward and read by the
 * derivatives; workspace: bpk_spatial_emb_workspace_bytes(n, k). */
int bpk_spatial_emb_supported(int64_t n, int k);
int64_t bpk_spatial_emb_workspace_bytes(int64_t n, int k);
int bpk_spatial_emb_fwd_f32(const float* x, const float* y, float* out, float* mxy,
                            float* workspace, int64_t n, int k, float omega, float s,
                            void* stream);
int bpk_spatial_emb_vjp_f32(const float* x, const float* y, const float* mxy, const float* g,
                            float* gx, float* gy, float* workspace, int64_t n, int k, float omega,
                            float s, void* stream);
int bpk_spatial_emb_vjp2_f32(const float* x, const float* y, const float* mxy, const float* g,
                             const float* hx, const float* hy, float* dg, float* dx, float* dy,
                             float* workspace, int64_t n, int k, float omega, float s,
                             void* stream);

/* out[n,c,:] = (x + (h + bias[c])) / div -- the skip_rescale residual of the
 * BigGAN / DDPM++ blocks with Conv_1's bias folded in (models/layerspp.py:266-274,
 * :200-209).  bias may be NULL.  x, h, out: [N, C, HW]. */
int bpk_residual_rescale_f32(const float* x, const float* h, const float* bias, float* out, int N,
                             int C, int64_t HW, float div, void* stream);

/* ------------------------------------------------------------------------- *
 * Score-SDE PC-sampler update kernels (sampling.py:176-282) and the counter-
 * based noise source.  Per-step scalars live in a device table `coef`
 * [n_steps, BPK_COEF_STRIDE] built on the host with the reference's float32
 * algorithm; the step index is read from device memory `step_ptr` so a whole
 * PC step can be captured once in a hipGraph and replayed.  Noise: when
 * `noise` is NULL the kernel draws N(0,1) from Philox4x32-10 keyed by `seed`,
 * counter = (global element index / 4, step, draw); global element index =
 * (sample_offset + b) * D + e, so draws are identical however the batch is
 * sharded over ranks.  A non-NULL `noise` [B, D] injects explicit noise (parity
 * hook).  x_mean may alias nothing; x_out may alias x.
 * ------------------------------------------------------------------------- */
#define BPK_COEF_STRIDE 8
/* coef layout per step (float32):
 *  [0] score_div   (std used to turn model output into a score; see score_mode)
 *  [1] drift_coef  (EM: -0.5 beta(t), VE: 0)        / ancestral & RD: beta or sigma^2 - adj^2
 *  [2] diffusion   (EM: g(t))                        / ancestral: sqrt(1-beta) ...
 *  [3] dt          (EM: -1/N as float32)
 *  [4] sqrt_mdt    (EM: float32(sqrt(-dt)))
 *  [5] alpha       (Langevin: alphas[timestep] or 1)
 *  [6], [7] spare
 */
enum {
  BPK_PRED_EULER_MARUYAMA = 0,
  BPK_PRED_REVERSE_DIFFUSION = 1,
  BPK_PRED_ANCESTRAL_VP = 2,
  BPK_PRED_ANCESTRAL_VE = 3,
};
/* score_mode 0: score = (-m) / coef[0]  (VP / subVP);  1: score = m (VE). */
int bpk_philox_normal_f32(float* out, int B, int64_t D, int64_t sample_offset, uint64_t seed,
                          const int* step_ptr, int draw, void* stream);
int bpk_pc_predictor_f32(int kind, const float* x, const float* model_out, const float* noise,
                         float* x_out, float* x_mean, int B, int64_t D, int64_t sample_offset,
                         const float* coef, int coef_bdim, const int* step_ptr, int score_mode,
                         int drift_mul_x, uint64_t seed, int draw, void* stream);
/* Langevin corrector, split in three launches so a 2-float all-reduce can sit
 * between (2) and (3) for batch-sharded runs:
 *   (1) partial: per (sample, chunk) sums of squares of score and noise
 *   (2) reduce : red[0] = sum_b ||score_b||, red[1] = sum_b ||noise_b|| (local batch)
 *   (3) update : step = (snr * (red[1]/B_global) / (red[0]/B_global))^2 * 2 * alpha;
 *                x_mean = x + step*score; x = x_mean + sqrt(2 step) * noise
 * mode 0 = Langevin (sampling.py:253-282), 1 = annealed Langevin dynamics
 * (sampling.py:285-319: step = (snr * std)^2 * 2 * alpha, std = coef[6]).  */
int64_t bpk_langevin_workspace_bytes(int B, int64_t D);
int bpk_langevin_partial_f32(const float* model_out, const float* noise, void* workspace, int B,
                             int64_t D, int64_t sample_offset, const float* coef, int coef_bdim,
                             const int* step_ptr, int score_mode, uint64_t seed, int draw,
                             void* stream);
int bpk_langevin_reduce_f32(void* workspace, float* red, int B, int64_t D, void* stream);
int bpk_langevin_update_f32(int mode, const float* x, const float* model_out, const float* noise,
                            const float* red, float* x_out, float* x_mean, int B, int64_t D,
                            int B_global, int64_t sample_offset, const float* coef,
                            int coef_bdim, const int* step_ptr, int score_mode, float snr,
                            uint64_t seed, int draw, void* stream);
/* step_ptr[0] += 1 (device-side step counter for graph replay) */
int bpk_step_increment(int* step_ptr, void* stream);
/* labels[b] = table[*step_ptr] for b < B (time conditioning for the score net) */
int bpk_fill_step_scalar_f32(float* labels, int B, const float* table, const int* step_ptr,
                             void* stream);

/* ------------------------------------------------------------------------- *
 * FlowNet correlation (cost volume), 7x7 displacements of `stride` pixels.
 *   first, second : [B, C, H, W] (NCHW, contiguous)
 *   out           : [B, 49, ceil(H/stride), ceil(W/stride)]
 *   out[b, (dy+3)*7 + (dx+3), oy, ox] = mean_c first[b,c,oy*s,ox*s] *
 *                                      second[b,c,oy*s+dy*s, ox*s+dx*s]  (0 outside)
 * Replaces the CuPy kernels kernel_Correlation_rearrange/updateOutput of
 * op/correlation.py:13-102 launched by _FunctionCorrelation.forward (:291-370).
 * bwd: grad_first / grad_second (either may be NULL) [B, C, H, W], fully
 * written (zero off the stride grid); replaces kernel_Correlation_updateGrad
 * {First,Second} (op/correlation.py:104-231) launched per sample by
 * _FunctionCorrelation.backward (:374-460).
 * ------------------------------------------------------------------------- */
int bpk_correlation_fwd_f32(const float* first, const float* second, float* out, int B, int C,
                            int H, int W, int stride, void* stream);
int bpk_correlation_bwd_f32(const float* first, const float* second, const float* grad_out,
                            float* grad_first, float* grad_second, int B, int C, int H, int W,
                            int stride, void* stream);

/* ------------------------------------------------------------------------- *
 * 3x3 / stride 1 / pad 1 convolution, fused Winograd F(2x2,3x3) on the f32 MFMA
 * (the score networks' conv3x3: models/layers.py ddpm_conv3x3 / layerspp conv3x3,
 * which the reference runs as torch.nn.Conv2d -> cuDNN).
 *   filter: U [Cin, CoutP, 16] = G w G^T of w [Cout, Cin, 3, 3] (cache while w is fixed);
 *           CoutP = Cout rounded up to 64, the extra couts zero (filter_bytes() sizes it)
 *   conv  : y [N, Cout, H, W] = conv(x [N, Cin, H, W], w) (+ bias[Cout], may be NULL)
 * supported(): Cin % 8 == 0, Cout % 16 == 0, H % 8 == 0, W % 16 == 0 (Cout % 64 != 0: the
 * pipelined kernel computes CoutP couts and stores Cout -- the PINN networks' 16 / 32 / 96 /
 * 192-channel convs).
 * ------------------------------------------------------------------------- */
int64_t bpk_conv3x3_wino_filter_bytes(int Cin, int Cout);
int bpk_conv3x3_wino_filter_f32(const float* weight, float* U, int Cin, int Cout, void* stream);
/* The same transform of flip_t(w) = w[ci][co][2 - r][2 - s] for w [Cin, Cout, 3, 3] (the
 * weight of the conv whose backward-data this is: dx = conv(dy, flip_t(w)), the cuDNN
 * backward-data of nn.Conv2d) -- read in place, no flipped copy of w. */
int bpk_conv3x3_wino_filter_ft_f32(const float* weight, float* U, int Cin, int Cout,
                                   void* stream);
/* Many filter transforms in one launch: jobs (device memory) = n records of six int64
 * (weight ptr, U ptr, Cin, Cout, CoutP, ft) with the meaning of the two entries above (ft = 1:
 * the flipped, transposed filter); max_elems = the largest Cin * CoutP among them. */
int bpk_conv3x3_wino_filter_batch_f32(const int64_t* jobs, int n, int max_elems, void* stream);
int bpk_conv3x3_wino_supported(int N, int Cin, int Cout, int H, int W);
/* The 16-cin kernel's pair form, used by bpk_conv3x3_wino_ex_f32 / _splitk_f32 when W == 8 (and
 * the W % 16 form does not apply): two 8 x 8 images side by side per 8 x 16 region -- N even,
 * H % 8, Cin % 16, Cout % 128 == 0, one source, no statistics (CIFAR-10's 8 x 8 level,
 * reference configs/vp/cifar10_ncsnpp_continuous.py:41-64 ch_mult (1, 2, 2, 2)). */
int bpk_conv3x3_wino_pair_supported(int N, int Cin, int Cout, int H, int W);
int bpk_conv3x3_wino_f32(const float* x, const float* U, const float* bias, float* y, int N,
                         int Cin, int Cout, int H, int W, void* stream);
/* Same conv with the residual-block tail fused into the epilogue (layerspp.py:272-274,
 * ResnetBlockBigGANpp / DDPMpp): y = (skip + (conv(x) + bias)) / div, skip [N, Cout, H, W]
 * (NULL: plain conv) -- bit-identical to bpk_residual_rescale_f32 on the conv output. */
int bpk_conv3x3_wino_residual_f32(const float* x, const float* U, const float* bias,
                                  const float* skip, float div, float* y, int N, int Cin,
                                  int Cout, int H, int W, void* stream);
/* General form: the conv input is silu(x * s + t) with pre[n][cin] = (s, t) from
 * bpk_group_norm_affine_f32 (pre NULL: x itself), i.e. GroupNorm + SiLU + conv (+ residual
 * tail) in one launch without materialising the normalized tensor. */
int bpk_conv3x3_wino_pre_f32(const float* x, const float* pre, const float* U, const float* bias,
                             const float* skip, float div, float* y, int N, int Cin, int Cout,
                             int H, int W, void* stream);
/* Same, and -- stats != NULL -- the GroupNorm partial statistics of the stored output:
 * stats [N, Cout, (H/8) * (W/16), 2] = (mean, M2) of each channel over each 8 x 16 pixel
 * region (bpk_group_norm_affine_partials_f32 turns them into the next GroupNorm's affine
 * form without a statistics pass over y).  x2 != NULL: the input is the channel
 * concatenation [x (C1 channels), x2 (Cin - C1 channels)] without building it (C1 % 8 == 0;
 * the up path's torch.cat([h, hs.pop()]) in models/ncsnpp.py). */
int bpk_conv3x3_wino_ex_f32(const float* x, const float* x2, int C1, const float* pre,
                            const float* U, const float* bias, const float* skip, float div,
                            float* y, float* stats, int N, int Cin, int Cout, int H, int W,
                            void* stream);
/* Split-K form of bpk_conv3x3_wino_ex_f32 for launches that would leave most CUs idle (the
 * 32^2 / 16^2 levels at the per-GPU batch of a batch-sharded run, SURVEY 8(e): 64 -> 8/GPU):
 * the input channels are split into S slices whose raw partial outputs go to `workspace`,
 * then one reduce launch applies bias, the residual tail and the statistics (fixed summation
 * order: deterministic).  splitk_bytes() = the workspace this shape needs, 0 = no split (then
 * the entry is bpk_conv3x3_wino_ex_f32 and workspace may be NULL).  Same contract otherwise. */
int64_t bpk_conv3x3_wino_splitk_bytes(int N, int Cin, int C1, int Cout, int H, int W);
int bpk_conv3x3_wino_splitk_f32(const float* x, const float* x2, int C1, const float* pre,
                                const float* U, const float* bias, const float* skip, float div,
                                float* y, float* stats, float* workspace, int N, int Cin, int Cout,
                                int H, int W, void* stream);
/* y = conv3x3(nearest_x2(x)) + bias (bias may be NULL) for x [N, Cin, H/2, W/2] and y
 * [N, Cout, H, W]: F.interpolate(x, scale_factor=2, mode='nearest') followed by Conv_0 of the
 * ddpm net's Upsample (reference models/layers.py:576-590), with the upsample read inside the
 * Winograd kernel's patch load (the full-resolution input is never materialised).  U from
 * bpk_conv3x3_wino_filter_f32.  Needs Cin % 16 == 0, Cout % 128 == 0, H % 8, W % 16 == 0
 * (bpk_conv3x3_wino_up2_supported). */
int bpk_conv3x3_wino_up2_supported(int N, int Cin, int Cout, int H, int W);
int bpk_conv3x3_wino_up2_f32(const float* x, const float* U, const float* bias, float* y, int N,
                             int Cin, int Cout, int H, int W, void* stream);
/* Weight gradient of the same conv (the backward-filter convolution cuDNN / MIOpen runs
 * for nn.Conv2d's autograd): dw [Cout, Cin, 3, 3] = d(sum y * gy)/dw for x [N, Cin, H, W],
 * gy [N, Cout, H, W].  Winograd F(2x2,3x3): per transform position a split-K GEMM
 * dU_pos = sum_tiles V_pos^T (A gy A^T)_pos, then dw = G^T dU G.  `workspace` holds the
 * split-K partial slabs (bpk_conv3x3_wino_wgrad_workspace_bytes, device memory).
 * supported(): Cin % 32 == 0, Cout % 16 == 0, H % 2 == 0, W % 16 == 0 (or W == 8, N even:
 * two images per strip).  Deterministic. */
int bpk_conv3x3_wino_wgrad_supported(int N, int Cin, int Cout, int H, int W);
int64_t bpk_conv3x3_wino_wgrad_workspace_bytes(int N, int Cin, int Cout, int H, int W);
int bpk_conv3x3_wino_wgrad_f32(const float* x, const float* gy, float* dw, float* workspace,
                               int N, int Cin, int Cout, int H, int W, void* stream);
/* Same, plus the bias gradient db [Cout] = sum of gy over (n, h, w), accumulated from the
 * gradient tiles the weight-gradient kernel loads anyway (replaces a separate reduction of
 * gy; deterministic). */
int bpk_conv3x3_wino_wgrad_bias_f32(const float* x, const float* gy, float* dw, float* db,
                                    float* workspace, int N, int Cin, int Cout, int H, int W,
                                    void* stream);
/* Same with the convolved input silu(x * s + t), pre[n][cin] = (s, t) (may be NULL: x itself):
 * the weight gradient of the GroupNorm+SiLU-prologue conv (bpk_conv3x3_wino_ex_f32 with pre)
 * without materialising the activation. */
int bpk_conv3x3_wino_wgrad_pre_f32(const float* x, const float* pre, const float* gy, float* dw,
                                   float* db, float* workspace, int N, int Cin, int Cout, int H,
                                   int W, void* stream);
/* The weight gradient summed over two (x, gy) sources in one launch: dw = wgrad(x, gy) +
 * wgrad(x2, gy2) with x2 [N2, Cin, H, W], gy2 [N2, Cout, H, W]; db (optional) = the FIRST
 * source's bias gradient.  Workspace: bpk_conv3x3_wino_wgrad_workspace_bytes(N + N2, ...).
 * 8-wide images need N even.  The deferred weight gradients of the PINN backward (a conv and
 * its first-order backward-data conv share the weight): one launch and one reduce instead of
 * two each plus autograd's accumulation add -- no reference interface of its own. */
int bpk_conv3x3_wino_wgrad2_f32(const float* x, const float* gy, const float* x2, const float* gy2,
                                int N2, float* dw, float* db, float* workspace, int N, int Cin,
                                int Cout, int H, int W, void* stream);

/* 3x3 / stride 1 / pad 1 conv with a small channel count on one side (VALU, HBM-bound):
 * the score networks' conv_in (Cin = image channels, models/ncsnpp.py) and output_skip
 * pyramid heads (Cout = image channels), which the reference runs through nn.Conv2d ->
 * cuDNN.  y [N, Cout, H, W] = conv(a, w [Cout, Cin, 3, 3]) (+ bias, may be NULL) with
 * a = x, or a = silu(x * s + t) for pre[n][cin] = (s, t) (bpk_group_norm_affine_f32;
 * Cout <= 4 only).  supported(): W % 4 == 0 and (Cin <= 4 or Cout <= 4). */
int bpk_conv3x3_small_supported(int N, int Cin, int Cout, int H, int W);
int bpk_conv3x3_small_f32(const float* x, const float* pre, const float* weight,
                          const float* bias, float* y, int N, int Cin, int Cout, int H, int W,
                          void* stream);

/* Weight (+ bias) gradient of a K x K / stride 1 / pad K/2 conv (K = 1 or 3) into few output
 * channels (Cout <= 4): dw [Cout, Cin, K, K] = sum_{n,p} gy[n][co][p] x[n][c][p + (r, s) - K/2],
 * db [Cout] = sum gy (db may be NULL).  The networks' output convs (NCSN++ conv_out, the PINN
 * heads; reference nn.Conv2d -> cuDNN backward-weights).  One streaming pass over x, per-image
 * partials in `workspace` (workspace_bytes()), summed in image order: deterministic. */
int bpk_conv2d_wgrad_small_cout_supported(int N, int Cin, int Cout, int H, int W, int K);
int64_t bpk_conv2d_wgrad_small_cout_workspace_bytes(int N, int Cin, int Cout, int K);
int bpk_conv2d_wgrad_small_cout_f32(const float* x, const float* gy, float* dw, float* db,
                                    void* workspace, int N, int Cin, int Cout, int H, int W,
                                    int K, void* stream);

/* 1x1 convolution of NCHW tensors as an f32 MFMA GEMM with an optional second source
 * along K (the score networks' Conv_2 skip projections and attention NINs, which the
 * reference runs through nn.Conv2d / einsum):
 *   Y[n] (M x P) = W[:, :K1] X1[n] (K1 x P) + W[:, K1:K1+K2] X2[n] (K2 x P) + bias[M]
 * W row-major [M, ldw], X1 [N, K1, P], X2 [N, K2, P] (NULL when K2 = 0), Y [N, M, P], P = H*W;
 * reading [X1, X2] this way replaces the channel concatenation torch.cat([X1, X2], 1).
 * supported(): M % 16 == 0, P % 128 == 0, K1 % 16 == 0, K2 % 16 == 0 (M tiles of 128,
 * rows past M masked). */
int bpk_gemm_nchw_supported(int N, int M, int P, int K1, int K2);
int bpk_gemm_nchw_f32(const float* W, int ldw, const float* X1, int K1, const float* X2, int K2,
                      const float* bias, float* Y, int N, int M, int P, void* stream);
/* Split-K form for launches too small to fill the chip (the 16^2 / 32^2 levels at the per-GPU
 * batch of a batch-sharded run): S slices of K write raw partials to `workspace`, one reduce
 * launch sums them in a fixed order and adds the bias.  splitk_bytes() = the workspace this
 * shape needs, 0 = no split (then the entry is bpk_gemm_nchw_f32, workspace may be NULL). */
int64_t bpk_gemm_nchw_splitk_bytes(int N, int M, int P, int K1, int K2);
int bpk_gemm_nchw_splitk_f32(const float* W, int ldw, const float* X1, int K1, const float* X2,
                             int K2, const float* bias, float* Y, float* workspace, int N, int M,
                             int P, void* stream);
/* Strided batched GEMM on the f32 MFMA: C(b, m, n) = alpha * sum_k A(b, m, k) B(b, k, n)
 * (+ bias[n] for bias_mode 1, bias[m] for 2; accumulate != 0: C += instead of C =), each operand
 * addressed by element strides (A(b, m, k) = A[b sab + m sam + k sak], ...), so transposes
 * are strides, not copies.  Replaces the rocBLAS / hipBLASLt GEMMs behind nn.Linear (the
 * time-embedding MLP and Dense_0 projections, reference models/ncsnpp.py:86-89,
 * layerspp.py:232-262) and torch.bmm in the attention block under autograd (reference
 * layerspp.py:84-88), forward and both gradients.  Deterministic. */
int bpk_gemm_sb_f32(const float* A, int64_t sab, int64_t sam, int64_t sak, const float* B,
                    int64_t sbb, int64_t sbk, int64_t sbn, float* C, int64_t scb, int64_t scm,
                    int64_t scn, const float* bias, int bias_mode, float alpha, int accumulate,
                    int batch, int M, int N, int K, void* stream);

/* Channel self-attention of the score networks' attention blocks at inference, one kernel:
 *   out[b, c, i] = sum_j V[b, c, j] softmax_j(scale * sum_c' Q[b, c', i] K[b, c', j])
 * qkv [B, 3, C, P] (Q, K, V = the three channel blocks of the stacked NIN_0/1/2 projection),
 * out [B, C, P], P = H*W.  Replaces the einsum / bmm + softmax + bmm of AttnBlockpp
 * (models/layerspp.py:75-91) and AttnBlock (models/layers.py:549-573).
 * supported(): C % 32 == 0, P in {64, 128, 256}. */
int bpk_attention_supported(int B, int C, int P);
int bpk_attention_f32(const float* qkv, float* out, int B, int C, int P, float scale, void* stream);
/* Same, with the keys split over up to 4 workgroups per query block when B x P / 64
 * workgroups would leave most CUs idle (the per-GPU batch of a batch-sharded run: B = 8 ->
 * 32 workgroups at 16^2): each split's unnormalised partial output and row statistics go to
 * `workspace` (workspace_bytes(), 0 = no split: workspace may be NULL) and a combine launch
 * merges them in a fixed order. */
int64_t bpk_attention_workspace_bytes(int B, int C, int P);
int bpk_attention_ex_f32(const float* qkv, float* out, float* workspace, int B, int C, int P,
                         float scale, void* stream);

/* Weight / bias gradient of that 1x1 conv (replaces the conv2d backward-weights MIOpen
 * runs for the reference's nn.Conv2d 1x1 layers -- ddpm_conv1x1 (models/layers.py:96), the
 * BigGAN blocks' Conv_2 skip projection (models/layerspp.py:235) -- under loss.backward(),
 * losses.py:210):
 *   dW (M x K) = sum_n GY[n] (M x P) X[n]^T (P x K),   db[m] = sum_{n,p} GY[n][m][p]
 * GY [N, M, P], X [N, K, P], dW row-major [M, K], db [M] or NULL.  Split-K over pixel
 * ranges with per-split partial slabs summed in a fixed order (deterministic); workspace of
 * workspace_bytes() (0: none needed).  supported(): M % 16, K % 16, P % 16 == 0. */
int bpk_gemm_nchw_wgrad_supported(int N, int M, int K, int P);
int64_t bpk_gemm_nchw_wgrad_workspace_bytes(int N, int M, int K, int P);
int bpk_gemm_nchw_wgrad_f32(const float* GY, const float* X, float* dW, float* db,
                            void* workspace, int N, int M, int K, int P, void* stream);

/* General convolution (any KH x KW, stride, zero padding; groups = 1, dilation = 1) as
 * implicit GEMM on the f32 MFMA: the forward, its adjoint (backward-data = conv transpose)
 * and the weight (+ bias) gradient.  Replaces the cuDNN convolutions the reference runs
 * for every conv the Winograd / small-channel / 1x1 kernels above do not take: the
 * stride-2 convs of FIR downsampling (models/up_or_down_sampling.py:144-178, F.conv2d) and
 * of the PINN feature pyramid (models/flownet.py:27-33), the PINN / CIFAR-10 3x3 convs at
 * 2^2..8^2 and with Cin % 8 != 0 (flownet.py:42-58, 93-138), ConvTranspose2d
 * (flownet.py:97, 229-231: forward == this dgrad), under loss.backward() and the PINN
 * residual's create_graph derivatives (pinn_kalman/pinn.py:72-111).
 *   x [N, Cin, H, W], w [Cout, Cin, KH, KW], y / gy [N, Cout, Ho, Wo] with
 *   Ho = (H + 2 ph - KH) / sh + 1 (same for Wo); dw like w, db [Cout] or NULL.
 * fwd: y = conv(x, w) + bias (bias NULL = none); dgrad: gx = conv^T(gy) (gx fully written);
 * wgrad: dw (and db = sum over n, oy, ox of gy when db != NULL).  Split-K partials in a
 * caller-provided workspace of workspace_bytes(mode 0 / 1 / 2, ..., bias_grad) bytes
 * (0: none needed; -1: unsupported shape), summed in a fixed order (deterministic). */
int64_t bpk_conv2d_igemm_workspace_bytes(int mode, int N, int Cin, int H, int W, int Cout,
                                         int KH, int KW, int sh, int sw, int ph, int pw, int Ho,
                                         int Wo, int bias_grad);
int bpk_conv2d_igemm_fwd_f32(const float* x, const float* w, const float* bias, float* y,
                             void* workspace, int N, int Cin, int H, int W, int Cout, int KH,
                             int KW, int sh, int sw, int ph, int pw, int Ho, int Wo,
                             void* stream);
int bpk_conv2d_igemm_dgrad_f32(const float* gy, const float* w, float* gx, void* workspace,
                               int N, int Cin, int H, int W, int Cout, int KH, int KW, int sh,
                               int sw, int ph, int pw, int Ho, int Wo, void* stream);
int bpk_conv2d_igemm_wgrad_f32(const float* x, const float* gy, float* dw, float* db,
                               void* workspace, int N, int Cin, int H, int W, int Cout, int KH,
                               int KW, int sh, int sw, int ph, int pw, int Ho, int Wo,
                               void* stream);
/* The weight gradient summed over two (x, gy) sources of the same geometry in one launch:
 * dw = wgrad(x, gy) + wgrad(x2, gy2), x [N, Cin, H, W], x2 [N2, Cin, H, W] (gy, gy2 likewise);
 * db (optional) = the bias gradient of the FIRST source only.  The K sum runs over the images
 * of x then x2 (workspace: bpk_conv2d_igemm_workspace_bytes(2, N + N2, ...)).  Replaces the
 * second weight-gradient launch, its reduce and autograd's accumulation add for a weight that
 * two convs of one backward pass use (the PINN residual: each conv and its backward-data conv
 * of the first-order pass) -- no reference interface of its own. */
int bpk_conv2d_igemm_wgrad2_f32(const float* x, const float* gy, const float* x2, const float* gy2,
                                int N2, float* dw, float* db, void* workspace, int N, int Cin,
                                int H, int W, int Cout, int KH, int KW, int sh, int sw, int ph,
                                int pw, int Ho, int Wo, void* stream);

/* ------------------------------------------------------------------------- *
 * InstanceNorm2d (affine=False) + activation, forward / backward / double backward:
 * replaces aten's batch_norm statistics + transform, ELU, native_batch_norm_backward,
 * elu_backward and the composite batchnorm double backward behind PressureNet's
 * ResidualBlock `conv(act(normalize(x)))` (reference models/layers.py:438-491, used by
 * models/flownet.py:219-224 get_double_res), differentiated twice by the PINN residual
 * (pinn_kalman/pinn.py:72-111).  x [planes = N*C, M = H*W] contiguous; act 0 = identity,
 * 1 = ELU(alpha=1).  fwd writes y and per-plane mean / rstd (1/sqrt(biased var + eps));
 * bwd: dx for upstream dy; bwd2: for v = dL/d(dx), gdy = dL/d(dy) and gx = dL/dx (either
 * may be NULL).  Deterministic (fixed-order per-plane reductions). */
int bpk_instance_norm_act_fwd_f32(const float* x, float* y, float* mean, float* rstd,
                                  int64_t planes, int64_t M, double eps, int act, void* stream);
int bpk_instance_norm_act_fwd_f64(const double* x, double* y, double* mean, double* rstd,
                                  int64_t planes, int64_t M, double eps, int act, void* stream);
int bpk_instance_norm_act_bwd_f32(const float* dy, const float* x, const float* mean,
                                  const float* rstd, float* dx, int64_t planes, int64_t M, int act,
                                  void* stream);
int bpk_instance_norm_act_bwd_f64(const double* dy, const double* x, const double* mean,
                                  const double* rstd, double* dx, int64_t planes, int64_t M,
                                  int act, void* stream);
/* dx = the backward above + add (same shapes): the residual block's skip gradient added in the
 * same pass (PressureNet's ResidualBlock input feeds its first norm and its skip; autograd
 * would add the two gradients in a separate launch). */
int bpk_instance_norm_act_bwd_add_f32(const float* dy, const float* x, const float* mean,
                                      const float* rstd, const float* add, float* dx,
                                      int64_t planes, int64_t M, int act, void* stream);
int bpk_instance_norm_act_bwd2_f32(const float* v, const float* dy, const float* x,
                                   const float* mean, const float* rstd, float* gdy, float* gx,
                                   int64_t planes, int64_t M, int act, void* stream);
int bpk_instance_norm_act_bwd2_f64(const double* v, const double* dy, const double* x,
                                   const double* mean, const double* rstd, double* gdy, double* gx,
                                   int64_t planes, int64_t M, int act, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* BPK_H_ */
