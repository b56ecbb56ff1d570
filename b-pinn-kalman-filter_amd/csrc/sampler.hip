// Score-SDE Predictor-Corrector update kernels + counter-based Gaussian noise.
//
// Restates the per-step arithmetic of sampling.py (EulerMaruyamaPredictor
// :176-187, ReverseDiffusionPredictor :190-200, AncestralSamplingPredictor
// :203-239, LangevinCorrector :253-282, AnnealedLangevinDynamics :285-319) and
// of the reverse SDE (sde_lib.py:81-119) as fused elementwise kernels.  Each
// kernel keeps the reference's float32 operation order (FMA contraction off),
// so with the same model output and noise it is bit-identical to the torch-CPU
// restatement in oracle/score_sde_ref.py.
//
// Per-step scalars come from a device table built once on the host (float32,
// reference algorithm) and the step index from a device counter, so one PC step
// is a fixed launch sequence that a hipGraph can capture and replay N times.
//
// Noise: Philox4x32-10 keyed by `seed`; counter = (q_lo, q_hi, step, draw) with
// q = global_element / 4, global_element = (sample_offset + b) * D + e; 4 normals
// per counter via Box-Muller.  Identical values for any batch sharding.
#include "bpk_common.h"

#include <algorithm>

#pragma clang fp contract(off)

namespace {

__device__ inline uint4 philox4x32_10(uint4 ctr, uint2 key) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  constexpr uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(M0, ctr.x), lo0 = M0 * ctr.x;
    const uint32_t hi1 = __umulhi(M1, ctr.z), lo1 = M1 * ctr.z;
    ctr = make_uint4(hi1 ^ ctr.y ^ key.x, lo1, hi0 ^ ctr.w ^ key.y, lo0);
    key.x += W0;
    key.y += W1;
  }
  return ctr;
}

__device__ inline float u01(uint32_t r) {  // (0, 1]
  return ((float)(r >> 8) + 1.0f) * (1.0f / 16777216.0f);
}

// normal of global element index ge (4 per Philox block)
__device__ inline void normal4(uint64_t q, int step, int draw, uint64_t seed, float out[4]) {
  const uint4 r = philox4x32_10(make_uint4((uint32_t)q, (uint32_t)(q >> 32), (uint32_t)step,
                                           (uint32_t)draw),
                                make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
  const float two_pi = 6.283185307179586f;
  const float r0 = sqrtf(-2.0f * logf(u01(r.x)));
  const float r1 = sqrtf(-2.0f * logf(u01(r.z)));
  float s0, c0, s1, c1;
  sincosf(two_pi * u01(r.y), &s0, &c0);
  sincosf(two_pi * u01(r.w), &s1, &c1);
  out[0] = r0 * c0;
  out[1] = r0 * s0;
  out[2] = r1 * c1;
  out[3] = r1 * s1;
}

__device__ inline float noise_at(const float* noise, int64_t i, int64_t ge, int step, int draw,
                                 uint64_t seed) {
  if (noise) return noise[i];
  float z[4];
  normal4((uint64_t)ge >> 2, step, draw, seed, z);
  return z[ge & 3];
}

__device__ inline float score_of(float m, float sdiv, int score_mode) {
  return score_mode == 0 ? (-m) / sdiv : m;
}

// every kernel handles 4 consecutive elements of one sample per thread so the
// Philox block is computed once per 4 outputs when D % 4 == 0
struct Idx {
  int64_t b, e;
};

__global__ __launch_bounds__(256) void k_philox(float* out, int B, int64_t D, int64_t sample_offset,
                                                uint64_t seed, const int* step_ptr, int draw) {
  const int step = step_ptr ? *step_ptr : 0;
  const int64_t total = (int64_t)B * D;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / D;
    const int64_t ge = (sample_offset + b) * D + (i - b * D);
    out[i] = noise_at(nullptr, i, ge, step, draw, seed);
  }
}

// coef index helpers
#define C_SDIV 0
#define C_DRIFT 1
#define C_DIFF 2
#define C_DT 3
#define C_SQRT_MDT 4
#define C_ALPHA 5
#define C_AUX 6

// coefficient row of local sample b at `step`: table [n_steps, coef_bdim, STRIDE]
__device__ inline const float* coef_row(const float* coef, int coef_bdim, int step, int64_t b) {
  return coef + ((int64_t)step * coef_bdim + (coef_bdim == 1 ? 0 : b)) * BPK_COEF_STRIDE;
}

__global__ __launch_bounds__(256) void k_predictor(int kind, const float* __restrict__ x,
                                                   const float* __restrict__ m,
                                                   const float* __restrict__ noise,
                                                   float* x_out, float* __restrict__ x_mean,
                                                   int B, int64_t D, int64_t sample_offset,
                                                   const float* __restrict__ coef, int coef_bdim,
                                                   const int* __restrict__ step_ptr,
                                                   int score_mode, int drift_mul_x,
                                                   uint64_t seed, int draw) {
  const int step = *step_ptr;
  const int64_t total = (int64_t)B * D;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / D;
    const float* cf = coef_row(coef, coef_bdim, step, b);
    const float sdiv = cf[C_SDIV];
    const int64_t ge = (sample_offset + b) * D + (i - b * D);
    const float xv = x[i];
    const float score = score_of(m[i], sdiv, score_mode);
    const float z = noise_at(noise, i, ge, step, draw, seed);
    float xm, xn;
    if (kind == BPK_PRED_EULER_MARUYAMA) {
      // drift, diffusion = sde(x,t); drift = drift - diffusion**2 * score * 1.
      // x_mean = x + drift*dt; x = x_mean + (diffusion*sqrt(-dt)) * z
      const float diff = cf[C_DIFF];
      float drift = drift_mul_x ? cf[C_DRIFT] * xv : cf[C_DRIFT];
      const float diff2 = diff * diff;
      drift = drift - diff2 * score * 1.0f;
      xm = xv + drift * cf[C_DT];
      xn = xm + (diff * cf[C_SQRT_MDT]) * z;
    } else if (kind == BPK_PRED_REVERSE_DIFFUSION) {
      // VP: f = sqrt(alpha)*x - x ; VE: f = 0.  G = coef[DIFF]
      // rev_f = f - G**2 * score * 1. ; x_mean = x - rev_f ; x = x_mean + G*z
      const float G = cf[C_DIFF];
      const float f = drift_mul_x ? cf[C_DRIFT] * xv - xv : 0.0f;
      const float G2 = G * G;
      const float rev_f = f - G2 * score * 1.0f;
      xm = xv - rev_f;
      xn = xm + G * z;
    } else if (kind == BPK_PRED_ANCESTRAL_VP) {
      // x_mean = (x + beta*score) / sqrt(1-beta) ; x = x_mean + sqrt(beta)*noise
      xm = (xv + cf[C_DRIFT] * score) / cf[C_DIFF];
      xn = xm + cf[C_SQRT_MDT] * z;
    } else {  // ANCESTRAL_VE
      // x_mean = x + score*(sigma^2 - adj^2) ; x = x_mean + std*noise
      xm = xv + score * cf[C_DRIFT];
      xn = xm + cf[C_DIFF] * z;
    }
    if (x_mean) x_mean[i] = xm;
    x_out[i] = xn;
  }
}

// ---- Langevin corrector
constexpr int kLgvThreads = 256;
constexpr int64_t kLgvChunk = 256 * 16;  // elements per (sample, chunk) workgroup

__global__ __launch_bounds__(kLgvThreads) void k_lgv_partial(
    const float* __restrict__ m, const float* __restrict__ noise, float* __restrict__ part,
    int64_t D, int chunks, int64_t sample_offset, const float* __restrict__ coef, int coef_bdim,
    const int* __restrict__ step_ptr, int score_mode, uint64_t seed, int draw) {
  __shared__ float sg[kLgvThreads / 64], sn[kLgvThreads / 64];
  const int step = *step_ptr;
  const int chunk = blockIdx.x;
  const int64_t b = blockIdx.y;
  const float sdiv = coef_row(coef, coef_bdim, step, b)[C_SDIV];
  const int64_t e0 = chunk * kLgvChunk;
  const int64_t e1 = std::min<int64_t>(D, e0 + kLgvChunk);
  float ag = 0.f, an = 0.f;
  for (int64_t e = e0 + threadIdx.x; e < e1; e += kLgvThreads) {
    const int64_t i = b * D + e;
    const float g = score_of(m[i], sdiv, score_mode);
    const float z = noise_at(noise, i, (sample_offset + b) * D + e, step, draw, seed);
    ag += g * g;
    an += z * z;
  }
  for (int off = 32; off > 0; off >>= 1) {
    ag += __shfl_xor(ag, off, 64);
    an += __shfl_xor(an, off, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    sg[threadIdx.x >> 6] = ag;
    sn[threadIdx.x >> 6] = an;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float tg = 0.f, tn = 0.f;
    for (int w = 0; w < kLgvThreads / 64; ++w) {
      tg += sg[w];
      tn += sn[w];
    }
    part[(b * chunks + chunk) * 2] = tg;
    part[(b * chunks + chunk) * 2 + 1] = tn;
  }
}

__global__ __launch_bounds__(256) void k_lgv_reduce(const float* __restrict__ part,
                                                    float* __restrict__ red, int B, int chunks) {
  __shared__ float sg[256], sn[256];
  float tg = 0.f, tn = 0.f;
  for (int b = threadIdx.x; b < B; b += 256) {
    float g = 0.f, n = 0.f;
    for (int c = 0; c < chunks; ++c) {
      g += part[((int64_t)b * chunks + c) * 2];
      n += part[((int64_t)b * chunks + c) * 2 + 1];
    }
    tg += sqrtf(g);
    tn += sqrtf(n);
  }
  sg[threadIdx.x] = tg;
  sn[threadIdx.x] = tn;
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f, c = 0.f;
    for (int i = 0; i < 256; ++i) {
      a += sg[i];
      c += sn[i];
    }
    red[0] = a;
    red[1] = c;
  }
}

__global__ __launch_bounds__(256) void k_lgv_update(
    int mode, const float* __restrict__ x, const float* __restrict__ m,
    const float* __restrict__ noise, const float* __restrict__ red, float* x_out,
    float* __restrict__ x_mean, int B, int64_t D, int B_global, int64_t sample_offset,
    const float* __restrict__ coef, int coef_bdim, const int* __restrict__ step_ptr,
    int score_mode, float snr, uint64_t seed, int draw) {
  const int step = *step_ptr;
  const int64_t total = (int64_t)B * D;
  float grad_norm = 0.f, noise_norm = 0.f;
  if (mode == 0) {
    grad_norm = red[0] / (float)B_global;
    noise_norm = red[1] / (float)B_global;
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / D;
    const float* cf = coef_row(coef, coef_bdim, step, b);
    const float alpha = cf[C_ALPHA];
    float step_size;
    if (mode == 0) {
      // (snr * noise_norm / grad_norm) ** 2 * 2 * alpha
      const float r = snr * noise_norm / grad_norm;
      step_size = r * r * 2.0f * alpha;
    } else {
      // (snr * std) ** 2 * 2 * alpha
      const float r = snr * cf[C_AUX];
      step_size = r * r * 2.0f * alpha;
    }
    const float nscale = sqrtf(step_size * 2.0f);
    const float g = score_of(m[i], cf[C_SDIV], score_mode);
    const float z = noise_at(noise, i, (sample_offset + b) * D + (i - b * D), step, draw, seed);
    const float xm = x[i] + step_size * g;
    if (x_mean) x_mean[i] = xm;
    x_out[i] = xm + nscale * z;
  }
}

__global__ void k_step_inc(int* step_ptr) { step_ptr[0] += 1; }

__global__ void k_fill(float* labels, int B, const float* table, const int* step_ptr) {
  const float v = table[*step_ptr];
  for (int b = threadIdx.x; b < B; b += blockDim.x) labels[b] = v;
}

unsigned blocks_for(int64_t total) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(bpk::ceil_div(total, 256), 256 * 32));
}

}  // namespace

extern "C" int bpk_philox_normal_f32(float* out, int B, int64_t D, int64_t sample_offset,
                                     uint64_t seed, const int* step_ptr, int draw, void* stream) {
  BPK_REQUIRE(B >= 0 && D >= 0, "philox_normal: bad shape");
  if ((int64_t)B * D == 0) return BPK_OK;
  hipLaunchKernelGGL(k_philox, dim3(blocks_for((int64_t)B * D)), dim3(256), 0,
                     bpk::as_stream(stream), out, B, D, sample_offset, seed, step_ptr, draw);
  BPK_LAUNCH_CHECK("philox_normal");
  return BPK_OK;
}

extern "C" int bpk_pc_predictor_f32(int kind, const float* x, const float* model_out,
                                    const float* noise, float* x_out, float* x_mean, int B,
                                    int64_t D, int64_t sample_offset, const float* coef,
                                    int coef_bdim, const int* step_ptr, int score_mode,
                                    int drift_mul_x, uint64_t seed, int draw, void* stream) {
  BPK_REQUIRE(kind >= 0 && kind <= 3, "pc_predictor: unknown kind %d", kind);
  BPK_REQUIRE(score_mode == 0 || score_mode == 1, "pc_predictor: bad score_mode");
  BPK_REQUIRE(coef && step_ptr, "pc_predictor: coef table and step counter required");
  BPK_REQUIRE(B >= 0 && D >= 0, "pc_predictor: bad shape");
  if ((int64_t)B * D == 0) return BPK_OK;
  hipLaunchKernelGGL(k_predictor, dim3(blocks_for((int64_t)B * D)), dim3(256), 0,
                     bpk::as_stream(stream), kind, x, model_out, noise, x_out, x_mean, B, D,
                     sample_offset, coef, coef_bdim, step_ptr, score_mode, drift_mul_x, seed,
                     draw);
  BPK_LAUNCH_CHECK("pc_predictor");
  return BPK_OK;
}

extern "C" int64_t bpk_langevin_workspace_bytes(int B, int64_t D) {
  if (B <= 0 || D <= 0) return 0;
  return (int64_t)B * bpk::ceil_div(D, kLgvChunk) * 2 * (int64_t)sizeof(float);
}

extern "C" int bpk_langevin_partial_f32(const float* model_out, const float* noise,
                                        void* workspace, int B, int64_t D, int64_t sample_offset,
                                        const float* coef, int coef_bdim, const int* step_ptr,
                                        int score_mode, uint64_t seed, int draw, void* stream) {
  BPK_REQUIRE(workspace && coef && step_ptr, "langevin_partial: workspace/coef/step required");
  BPK_REQUIRE(B > 0 && D > 0 && B <= 65535, "langevin_partial: bad shape");
  const int chunks = (int)bpk::ceil_div(D, kLgvChunk);
  hipLaunchKernelGGL(k_lgv_partial, dim3(chunks, B), dim3(kLgvThreads), 0, bpk::as_stream(stream),
                     model_out, noise, static_cast<float*>(workspace), D, chunks, sample_offset,
                     coef, coef_bdim, step_ptr, score_mode, seed, draw);
  BPK_LAUNCH_CHECK("langevin_partial");
  return BPK_OK;
}

extern "C" int bpk_langevin_reduce_f32(void* workspace, float* red, int B, int64_t D,
                                       void* stream) {
  BPK_REQUIRE(workspace && red, "langevin_reduce: workspace/red required");
  BPK_REQUIRE(B > 0 && D > 0, "langevin_reduce: bad shape");
  const int chunks = (int)bpk::ceil_div(D, kLgvChunk);
  hipLaunchKernelGGL(k_lgv_reduce, dim3(1), dim3(256), 0, bpk::as_stream(stream),
                     static_cast<const float*>(workspace), red, B, chunks);
  BPK_LAUNCH_CHECK("langevin_reduce");
  return BPK_OK;
}

extern "C" int bpk_langevin_update_f32(int mode, const float* x, const float* model_out,
                                       const float* noise, const float* red, float* x_out,
                                       float* x_mean, int B, int64_t D, int B_global,
                                       int64_t sample_offset, const float* coef, int coef_bdim,
                                       const int* step_ptr, int score_mode, float snr,
                                       uint64_t seed, int draw, void* stream) {
  BPK_REQUIRE(mode == 0 || mode == 1, "langevin_update: mode must be 0 or 1");
  BPK_REQUIRE(coef && step_ptr && (mode == 1 || red), "langevin_update: missing inputs");
  BPK_REQUIRE(B >= 0 && D >= 0 && B_global > 0, "langevin_update: bad shape");
  if ((int64_t)B * D == 0) return BPK_OK;
  hipLaunchKernelGGL(k_lgv_update, dim3(blocks_for((int64_t)B * D)), dim3(256), 0,
                     bpk::as_stream(stream), mode, x, model_out, noise, red, x_out, x_mean, B, D,
                     B_global, sample_offset, coef, coef_bdim, step_ptr, score_mode, snr, seed,
                     draw);
  BPK_LAUNCH_CHECK("langevin_update");
  return BPK_OK;
}

extern "C" int bpk_step_increment(int* step_ptr, void* stream) {
  BPK_REQUIRE(step_ptr, "step_increment: null counter");
  hipLaunchKernelGGL(k_step_inc, dim3(1), dim3(1), 0, bpk::as_stream(stream), step_ptr);
  BPK_LAUNCH_CHECK("step_increment");
  return BPK_OK;
}

extern "C" int bpk_fill_step_scalar_f32(float* labels, int B, const float* table,
                                        const int* step_ptr, void* stream) {
  BPK_REQUIRE(labels && table && step_ptr && B >= 0, "fill_step_scalar: bad args");
  if (B == 0) return BPK_OK;
  hipLaunchKernelGGL(k_fill, dim3(1), dim3(256), 0, bpk::as_stream(stream), labels, B, table,
                     step_ptr);
  BPK_LAUNCH_CHECK("fill_step_scalar");
  return BPK_OK;
}
