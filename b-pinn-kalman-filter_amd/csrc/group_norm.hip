// GroupNorm (+ fused per-(n,c) bias before the norm, + fused SiLU after) for gfx950.
//
// Replaces the nn.GroupNorm -> act chains of the NCSN++ / DDPM++ residual blocks
// (models/layerspp.py:242-274, :200-209; models/ncsnpp.py:371-377) and folds in the
// time-embedding bias `h += Dense_0(act(temb))[:, :, None, None]` that sits right
// before GroupNorm_1 (layerspp.py:263-265).
//
// NCHW makes every (sample, group) a contiguous slab of S = (C/G)*HW floats, so:
//  * resident path (S <= 64K floats): one workgroup per slab, the slab is loaded
//    ONCE into registers with 16-byte loads, mean and variance are exact two-pass
//    reductions over the registers, and the normalized output is written once:
//    1 read + 1 write of HBM per element (the algorithmic minimum).
//  * split path (larger slabs): per-chunk (count, mean, M2) partials combined with
//    Chan's formula in a fixed order (deterministic), then a normalize pass.
// Backward mirrors this (resident: x and dy read once; dgamma/dbeta emitted as
// per-(n,c) partial sums that the host reduces over n).
#include "bpk_common.h"

#include <algorithm>

namespace {

constexpr int kWave = 64;

template <int T>
__device__ inline float block_sum(float v, float* sbuf) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  const int wid = threadIdx.x / kWave;
  const int lane = threadIdx.x % kWave;
  __syncthreads();
  if (lane == 0) sbuf[wid] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < T / kWave; ++i) r += sbuf[i];
  return r;
}

__device__ inline float act_fwd(float z, int act) {
  return act == 1 ? z / (1.f + expf(-z)) : z;
}
// d act / dz
__device__ inline float act_bwd(float z, int act) {
  if (act != 1) return 1.f;
  const float s = 1.f / (1.f + expf(-z));
  return s * (1.f + z * (1.f - s));
}

// Element access for a slab: W = 4 (float4 path) or 1 (scalar path).
template <int W>
struct Vec;
template <>
struct Vec<4> {
  static __device__ inline void load(const float* p, float* v) {
    const float4 q = *reinterpret_cast<const float4*>(p);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  }
  static __device__ inline void store(float* p, const float* v) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
};
template <>
struct Vec<1> {
  static __device__ inline void load(const float* p, float* v) { v[0] = *p; }
  static __device__ inline void store(float* p, const float* v) { *p = v[0]; }
};

// ---------------------------------------------------------------- forward

template <int T, int VPT, int W>
__global__ __launch_bounds__(T) void gn_fwd_resident(const float* __restrict__ x,
                                                     const float* __restrict__ bias_nc,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ beta,
                                                     float* __restrict__ y, float* mean_out,
                                                     float* rstd_out, int C, int HW, int G,
                                                     float eps, int act) {
  __shared__ float sbuf[T / kWave];
  const int ng = blockIdx.x;
  const int n = ng / G;
  const int g = ng - n * G;
  const int cpg = C / G;
  const int S = cpg * HW;
  const int64_t base = ((int64_t)n * C + (int64_t)g * cpg) * HW;
  const int tid = threadIdx.x;

  float v[VPT][W];
  float lsum = 0.f;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int e = (k * T + tid) * W;
    if (e < S) {
      Vec<W>::load(x + base + e, v[k]);
      if (bias_nc) {
        const float b = bias_nc[(int64_t)n * C + g * cpg + e / HW];
#pragma unroll
        for (int q = 0; q < W; ++q) v[k][q] += b;
      }
#pragma unroll
      for (int q = 0; q < W; ++q) lsum += v[k][q];
    }
  }
  const float mean = block_sum<T>(lsum, sbuf) / (float)S;
  float lm2 = 0.f;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int e = (k * T + tid) * W;
    if (e < S) {
#pragma unroll
      for (int q = 0; q < W; ++q) {
        const float d = v[k][q] - mean;
        lm2 += d * d;
      }
    }
  }
  const float var = block_sum<T>(lm2, sbuf) / (float)S;
  const float rstd = 1.f / sqrtf(var + eps);
  if (tid == 0) {
    if (mean_out) mean_out[ng] = mean;
    if (rstd_out) rstd_out[ng] = rstd;
  }
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int e = (k * T + tid) * W;
    if (e < S) {
      const int c = g * cpg + e / HW;
      const float ga = gamma ? gamma[c] : 1.f;
      const float be = beta ? beta[c] : 0.f;
      float o[W];
#pragma unroll
      for (int q = 0; q < W; ++q) o[q] = act_fwd((v[k][q] - mean) * rstd * ga + be, act);
      Vec<W>::store(y + base + e, o);
    }
  }
}

// split path, stage 1: per-chunk (mean, M2) of CHUNK = T*VPT*W elements
template <int T, int VPT, int W>
__global__ __launch_bounds__(T) void gn_fwd_partial(const float* __restrict__ x,
                                                    const float* __restrict__ bias_nc,
                                                    float* __restrict__ part, int C, int HW,
                                                    int G, int splits) {
  __shared__ float sbuf[T / kWave];
  const int split = blockIdx.x;
  const int ng = blockIdx.y;
  const int n = ng / G;
  const int g = ng - n * G;
  const int cpg = C / G;
  const int S = cpg * HW;
  constexpr int CHUNK = T * VPT * W;
  const int e0 = split * CHUNK;
  const int cnt = min(CHUNK, S - e0);
  const int64_t base = ((int64_t)n * C + (int64_t)g * cpg) * HW;
  const int tid = threadIdx.x;
  float v[VPT][W];
  float lsum = 0.f;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int e = e0 + (k * T + tid) * W;
    if (e < S) {
      Vec<W>::load(x + base + e, v[k]);
      if (bias_nc) {
        const float b = bias_nc[(int64_t)n * C + g * cpg + e / HW];
#pragma unroll
        for (int q = 0; q < W; ++q) v[k][q] += b;
      }
#pragma unroll
      for (int q = 0; q < W; ++q) lsum += v[k][q];
    }
  }
  const float m = block_sum<T>(lsum, sbuf) / (float)cnt;
  float lm2 = 0.f;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int e = e0 + (k * T + tid) * W;
    if (e < S) {
#pragma unroll
      for (int q = 0; q < W; ++q) {
        const float d = v[k][q] - m;
        lm2 += d * d;
      }
    }
  }
  const float m2 = block_sum<T>(lm2, sbuf);
  if (tid == 0) {
    float* p = part + ((int64_t)ng * splits + split) * 3;
    p[0] = (float)cnt;
    p[1] = m;
    p[2] = m2;
  }
}

// Chan et al. parallel combination, fixed order -> deterministic
__device__ inline void combine_partials(const float* p, int splits, float& mean, float& m2,
                                        float& count) {
  count = p[0];
  mean = p[1];
  m2 = p[2];
  for (int s = 1; s < splits; ++s) {
    const float nb = p[3 * s];
    const float mb = p[3 * s + 1];
    const float m2b = p[3 * s + 2];
    const float nn = count + nb;
    const float d = mb - mean;
    mean += d * (nb / nn);
    m2 += m2b + d * d * (count * nb / nn);
    count = nn;
  }
}

template <int W>
__global__ __launch_bounds__(256) void gn_fwd_apply(const float* __restrict__ x,
                                                    const float* __restrict__ bias_nc,
                                                    const float* __restrict__ gamma,
                                                    const float* __restrict__ beta,
                                                    const float* __restrict__ part,
                                                    float* __restrict__ y, float* mean_out,
                                                    float* rstd_out, int C, int HW, int G,
                                                    int splits, int chunk, float eps, int act) {
  __shared__ float s_stat[2];
  const int split = blockIdx.x;
  const int ng = blockIdx.y;
  const int n = ng / G;
  const int g = ng - n * G;
  const int cpg = C / G;
  const int S = cpg * HW;
  if (threadIdx.x == 0) {
    float mean, m2, count;
    combine_partials(part + (int64_t)ng * splits * 3, splits, mean, m2, count);
    const float rstd = 1.f / sqrtf(m2 / count + eps);
    s_stat[0] = mean;
    s_stat[1] = rstd;
    if (split == 0) {
      if (mean_out) mean_out[ng] = mean;
      if (rstd_out) rstd_out[ng] = rstd;
    }
  }
  __syncthreads();
  const float mean = s_stat[0];
  const float rstd = s_stat[1];
  const int64_t base = ((int64_t)n * C + (int64_t)g * cpg) * HW;
  const int e_end = min(S, (split + 1) * chunk);
  for (int e = split * chunk + threadIdx.x * W; e < e_end; e += 256 * W) {
    float v[W];
    Vec<W>::load(x + base + e, v);
    const int c = g * cpg + e / HW;
    const float b = bias_nc ? bias_nc[(int64_t)n * C + c] : 0.f;
    const float ga = gamma ? gamma[c] : 1.f;
    const float be = beta ? beta[c] : 0.f;
    float o[W];
#pragma unroll
    for (int q = 0; q < W; ++q) o[q] = act_fwd((v[q] + b - mean) * rstd * ga + be, act);
    Vec<W>::store(y + base + e, o);
  }
}

// per-(n, c) affine form of act(GroupNorm(x + bias_nc)): act(x * s + t) with
// s = rstd * gamma[c], t = beta[c] + (bias_nc[n, c] - mean) * s -- consumed by the
// Winograd conv's patch load so the normalized tensor never round-trips HBM
__global__ __launch_bounds__(64) void gn_affine_kernel(const float* __restrict__ part,
                                                       const float* __restrict__ bias_nc,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta,
                                                       float2* __restrict__ ss,
                                                       float* __restrict__ mean_out,
                                                       float* __restrict__ rstd_out, int C, int G,
                                                       int splits, float eps) {
  __shared__ float s_stat[2];
  const int ng = blockIdx.x;
  const int n = ng / G;
  const int g = ng - n * G;
  const int cpg = C / G;
  if (threadIdx.x == 0) {
    float mean, m2, count;
    combine_partials(part + (int64_t)ng * splits * 3, splits, mean, m2, count);
    s_stat[0] = mean;
    s_stat[1] = 1.f / sqrtf(m2 / count + eps);
    if (mean_out) mean_out[ng] = mean;
    if (rstd_out) rstd_out[ng] = s_stat[1];
  }
  __syncthreads();
  for (int j = threadIdx.x; j < cpg; j += blockDim.x) {
    const int c = g * cpg + j;
    const float sc = s_stat[1] * (gamma ? gamma[c] : 1.f);
    const float b = bias_nc ? bias_nc[(int64_t)n * C + c] : 0.f;
    ss[(int64_t)n * C + c] = make_float2(sc, (beta ? beta[c] : 0.f) + (b - s_stat[0]) * sc);
  }
}

// ---------------------------------------------------------------- backward

template <int T, int VPT, int W>
__global__ __launch_bounds__(T) void gn_bwd_resident(
    const float* __restrict__ dy, const float* __restrict__ x, const float* __restrict__ bias_nc,
    const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in, float* __restrict__ dx,
    float* __restrict__ dgamma_nc, float* __restrict__ dbeta_nc, int C, int HW, int G, int act,
    const float* __restrict__ addend) {
  // [T/64] reduce buffer + 2*cpg channel partials + 2 * VPT * T/64 wave-slice partials
  extern __shared__ float sdyn[];
  float* sbuf = sdyn;
  float* s_dg = sdyn + T / kWave;
  const int ng = blockIdx.x;
  const int n = ng / G;
  const int g = ng - n * G;
  const int cpg = C / G;
  const int S = cpg * HW;
  float* s_sl = s_dg + 2 * cpg;
  const int64_t base = ((int64_t)n * C + (int64_t)g * cpg) * HW;
  const int tid = threadIdx.x;
  const float mean = mean_in[ng];
  const float rstd = rstd_in[ng];
  // gamma / beta partials per channel in a fixed order (the result must not depend on the
  // order waves finish in): L = units of W elements per channel plane.  L % 64 == 0: every
  // (k, wave) slice of 64 units lies in one channel -- butterfly sum per slice, then the
  // slices of a channel in slice order; L < 64 dividing 64: a channel is one aligned lane
  // segment of one slice -- a butterfly within the segment gives its sum.  Other planes
  // (H W not a power-of-two multiple): LDS atomics, order-dependent in the last bits.
  const int L = HW / W;
  const bool slice_mode = L % kWave == 0;
  const bool seg_mode = !slice_mode && L < kWave && kWave % L == 0;
  for (int i = tid; i < 2 * cpg; i += T) s_dg[i] = 0.f;
  __syncthreads();

  float xh[VPT][W], dxh[VPT][W];
  float la = 0.f, lb = 0.f;
  const int lane = tid & (kWave - 1), wave = tid / kWave;
  const bool ordered = (dgamma_nc || dbeta_nc) && (slice_mode || seg_mode);
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int e = (k * T + tid) * W;
    float pg = 0.f, pb = 0.f;
    if (e < S) {
      const int cl = e / HW;
      const int c = g * cpg + cl;
      const float b = bias_nc ? bias_nc[(int64_t)n * C + c] : 0.f;
      const float ga = gamma ? gamma[c] : 1.f;
      const float be = beta ? beta[c] : 0.f;
      float xv[W], gv[W];
      Vec<W>::load(x + base + e, xv);
      Vec<W>::load(dy + base + e, gv);
#pragma unroll
      for (int q = 0; q < W; ++q) {
        const float xhat = (xv[q] + b - mean) * rstd;
        const float dz = gv[q] * act_bwd(xhat * ga + be, act);
        pg += dz * xhat;
        pb += dz;
        xh[k][q] = xhat;
        dxh[k][q] = dz * ga;
        la += dxh[k][q];
        lb += dxh[k][q] * xhat;
      }
      if ((dgamma_nc || dbeta_nc) && !ordered) {
        atomicAdd(&s_dg[cl], pg);
        atomicAdd(&s_dg[cpg + cl], pb);
      }
    }
    if (ordered) {  // every lane takes part (zeros past the slab)
      const int span = slice_mode ? kWave : L;
      for (int off = span >> 1; off > 0; off >>= 1) {
        pg += __shfl_xor(pg, off, kWave);
        pb += __shfl_xor(pb, off, kWave);
      }
      if (slice_mode) {
        if (lane == 0) {
          s_sl[2 * (k * (T / kWave) + wave)] = pg;
          s_sl[2 * (k * (T / kWave) + wave) + 1] = pb;
        }
      } else if (lane % L == 0) {
        const int cl = (k * T + tid) / L;  // the segment is channel cl's whole plane
        if (cl < cpg) {
          s_dg[cl] = pg;
          s_dg[cpg + cl] = pb;
        }
      }
    }
  }
  if (ordered) {
    __syncthreads();
    if (slice_mode) {  // channel c = slices [c L / 64, (c + 1) L / 64), summed in order
      const int per = L / kWave;
      for (int i = tid; i < 2 * cpg; i += T) {
        const int c = i % cpg, which = i / cpg;
        float acc = 0.f;
        for (int j = c * per; j < (c + 1) * per; ++j) acc += s_sl[2 * j + which];
        s_dg[i] = acc;
      }
    }
  }
  const float A = block_sum<T>(la, sbuf) / (float)S;
  const float Bm = block_sum<T>(lb, sbuf) / (float)S;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int e = (k * T + tid) * W;
    if (e < S) {
      float o[W];
#pragma unroll
      for (int q = 0; q < W; ++q) o[q] = rstd * (dxh[k][q] - A - xh[k][q] * Bm);
      if (addend) {  // another consumer's gradient of x, added where the autograd engine would
        float ad[W];
        Vec<W>::load(addend + base + e, ad);
#pragma unroll
        for (int q = 0; q < W; ++q) o[q] = ad[q] + o[q];
      }
      Vec<W>::store(dx + base + e, o);
    }
  }
  // block_sum's barriers ordered every LDS atomic before this read
  for (int i = tid; i < cpg; i += T) {
    if (dgamma_nc) dgamma_nc[(int64_t)n * C + g * cpg + i] = s_dg[i];
    if (dbeta_nc) dbeta_nc[(int64_t)n * C + g * cpg + i] = s_dg[cpg + i];
  }
}

// split backward (deterministic, no atomics): the blocks of a group are laid on channel
// boundaries -- a block covers one slice of one channel plane (HW >= CH) or a run of whole
// planes (HW < CH) -- so the channel's bias / gamma / beta are loop constants, and the
// per-channel dgamma / dbeta sums are per-block partials reduced in a fixed order by the
// apply kernel (float atomics into one address per channel serialise and are not
// bit-reproducible).
struct BwdBlk {
  int c0, nc, h0, h1, s;
};
__host__ __device__ inline int bwd_spc(int HW, int CH) { return HW >= CH ? (HW + CH - 1) / CH : 1; }
__host__ __device__ inline int bwd_bpg(int HW, int cpg, int CH) {
  if (HW >= CH) return cpg * bwd_spc(HW, CH);
  const int cpb = CH / HW;
  return (cpg + cpb - 1) / cpb;
}
__device__ inline BwdBlk bwd_block(int bi, int HW, int cpg, int CH) {
  BwdBlk r;
  if (HW >= CH) {
    const int spc = bwd_spc(HW, CH);
    r.c0 = bi / spc;
    r.s = bi - r.c0 * spc;
    r.nc = 1;
    r.h0 = r.s * CH;
    r.h1 = min(HW, r.h0 + CH);
  } else {
    const int cpb = CH / HW;
    r.c0 = bi * cpb;
    r.nc = min(cpb, cpg - r.c0);
    r.s = 0;
    r.h0 = 0;
    r.h1 = HW;
  }
  return r;
}

template <int W>
__global__ __launch_bounds__(256) void gn_bwd_partial2(
    const float* __restrict__ dy, const float* __restrict__ x, const float* __restrict__ bias_nc,
    const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    float2* __restrict__ part_ab, float2* __restrict__ part_c, int want_c, int C, int HW, int G,
    int CH, int act) {
  __shared__ float sbuf[256 / kWave];
  const int bi = blockIdx.x, bpg = gridDim.x;
  const int ng = blockIdx.y;
  const int n = ng / G;
  const int g = ng - n * G;
  const int cpg = C / G;
  const BwdBlk blk = bwd_block(bi, HW, cpg, CH);
  const int spc = bwd_spc(HW, CH);
  const float mean = mean_in[ng];
  const float rstd = rstd_in[ng];
  float la = 0.f, lb = 0.f;
  for (int k = 0; k < blk.nc; ++k) {
    const int c = g * cpg + blk.c0 + k;
    const float b = bias_nc ? bias_nc[(int64_t)n * C + c] : 0.f;
    const float ga = gamma ? gamma[c] : 1.f;
    const float be = beta ? beta[c] : 0.f;
    const int64_t base = ((int64_t)n * C + c) * HW;
    float pg = 0.f, pb = 0.f;
    // two strides per iteration, loads first; same accumulation order as one stride at a
    // time (bit-identical partials)
    for (int e = blk.h0 + threadIdx.x * W; e < blk.h1; e += 2 * 256 * W) {
      const int e2 = e + 256 * W;
      const bool two = e2 < blk.h1;
      float xv[2][W], gv[2][W];
      Vec<W>::load(x + base + e, xv[0]);
      Vec<W>::load(dy + base + e, gv[0]);
      if (two) {
        Vec<W>::load(x + base + e2, xv[1]);
        Vec<W>::load(dy + base + e2, gv[1]);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (u == 1 && !two) break;
#pragma unroll
        for (int q = 0; q < W; ++q) {
          const float xhat = (xv[u][q] + b - mean) * rstd;
          const float dz = gv[u][q] * act_bwd(xhat * ga + be, act);
          pg += dz * xhat;
          pb += dz;
        }
      }
    }
    la += pb * ga;
    lb += pg * ga;
    if (want_c) {
      const float PG = block_sum<256>(pg, sbuf);
      const float PB = block_sum<256>(pb, sbuf);
      if (threadIdx.x == 0) part_c[((int64_t)n * C + c) * spc + blk.s] = make_float2(PG, PB);
    }
  }
  const float A = block_sum<256>(la, sbuf);
  const float B = block_sum<256>(lb, sbuf);
  if (threadIdx.x == 0) part_ab[(int64_t)ng * bpg + bi] = make_float2(A, B);
}

template <int W>
__global__ __launch_bounds__(256) void gn_bwd_apply2(
    const float* __restrict__ dy, const float* __restrict__ x, const float* __restrict__ bias_nc,
    const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    const float2* __restrict__ part_ab, const float2* __restrict__ part_c, float* __restrict__ dx,
    float* __restrict__ dgamma_nc, float* __restrict__ dbeta_nc, int C, int HW, int G, int CH,
    int act, const float* __restrict__ addend) {
  const int bi = blockIdx.x, bpg = gridDim.x;
  const int ng = blockIdx.y;
  const int n = ng / G;
  const int g = ng - n * G;
  const int cpg = C / G;
  const BwdBlk blk = bwd_block(bi, HW, cpg, CH);
  const int spc = bwd_spc(HW, CH);
  const float mean = mean_in[ng];
  const float rstd = rstd_in[ng];
  float A = 0.f, B = 0.f;
  for (int i = 0; i < bpg; ++i) {
    const float2 p = part_ab[(int64_t)ng * bpg + i];
    A += p.x;
    B += p.y;
  }
  const float S = (float)cpg * (float)HW;
  A /= S;
  B /= S;
  for (int k = 0; k < blk.nc; ++k) {
    const int c = g * cpg + blk.c0 + k;
    const float b = bias_nc ? bias_nc[(int64_t)n * C + c] : 0.f;
    const float ga = gamma ? gamma[c] : 1.f;
    const float be = beta ? beta[c] : 0.f;
    const int64_t base = ((int64_t)n * C + c) * HW;
    // two strides per iteration, all four loads issued before any use (more bytes in
    // flight per thread: the pass is HBM-bound)
    for (int e = blk.h0 + threadIdx.x * W; e < blk.h1; e += 2 * 256 * W) {
      const int e2 = e + 256 * W;
      const bool two = e2 < blk.h1;
      float xv[2][W], gv[2][W], o[W];
      Vec<W>::load(x + base + e, xv[0]);
      Vec<W>::load(dy + base + e, gv[0]);
      if (two) {
        Vec<W>::load(x + base + e2, xv[1]);
        Vec<W>::load(dy + base + e2, gv[1]);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (u == 1 && !two) break;
#pragma unroll
        for (int q = 0; q < W; ++q) {
          const float xhat = (xv[u][q] + b - mean) * rstd;
          const float dxhat = gv[u][q] * act_bwd(xhat * ga + be, act) * ga;
          o[q] = rstd * (dxhat - A - xhat * B);
        }
        if (addend) {
          float ad[W];
          Vec<W>::load(addend + base + (u ? e2 : e), ad);
#pragma unroll
          for (int q = 0; q < W; ++q) o[q] = ad[q] + o[q];
        }
        Vec<W>::store(dx + base + (u ? e2 : e), o);
      }
    }
    if (blk.s == 0 && threadIdx.x == 0 && (dgamma_nc || dbeta_nc)) {
      float pg = 0.f, pb = 0.f;
      for (int i = 0; i < spc; ++i) {
        const float2 p = part_c[((int64_t)n * C + c) * spc + i];
        pg += p.x;
        pb += p.y;
      }
      if (dgamma_nc) dgamma_nc[(int64_t)n * C + c] = pg;
      if (dbeta_nc) dbeta_nc[(int64_t)n * C + c] = pb;
    }
  }
}

// The reductions behind the backward's parameter gradients, one launch: d bias_nc[n, c] =
// sum over the plane of dx (the per-(n, c) bias added before the norm: the time-embedding
// Dense_0 output), dgamma[c] / dbeta[c] = sum over n of the kernels' per-(n, c) partials.
// Blocks [0, rows): one (n, c) plane each; the rest: 64 channels each.
// Fixed summation orders (deterministic); replaced three aten reductions per backward.
__global__ __launch_bounds__(256) void gn_param_grads_kernel(
    const float* __restrict__ dx, const float* __restrict__ dg_nc, const float* __restrict__ db_nc,
    float* __restrict__ d_bnc, float* __restrict__ dgamma, float* __restrict__ dbeta, int N,
    int C, int HW, int rows) {
  __shared__ float sbuf[256 / kWave];
  if ((int)blockIdx.x < rows) {
    const float* p = dx + (int64_t)blockIdx.x * HW;
    float v = 0.f;
    if ((HW & 3) == 0 && (reinterpret_cast<uintptr_t>(p) & 15) == 0) {
      const float4* p4 = reinterpret_cast<const float4*>(p);
      for (int i = threadIdx.x; i < HW / 4; i += 256) {
        const float4 q = p4[i];
        v += (q.x + q.y) + (q.z + q.w);
      }
    } else {
      for (int i = threadIdx.x; i < HW; i += 256) v += p[i];
    }
    v = block_sum<256>(v, sbuf);
    if (threadIdx.x == 0) d_bnc[blockIdx.x] = v;
    return;
  }
  // 64 channels per block (one per lane); wave w adds n in [w nq, (w + 1) nq) in order, eight
  // loads in flight at a time (a serial chain of N dependent loads took ~N load latencies),
  // then the four wave partials in wave order
  __shared__ float red[2][4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = ((int)blockIdx.x - rows) * 64 + lane;
  const int nq = (N + 3) / 4, n0 = w * nq, n1 = min(N, n0 + nq);
  float sg = 0.f, sb = 0.f;
  if (c < C) {
    for (int n = n0; n < n1; n += 8) {
      float tg[8], tb[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const bool in = n + u < n1;
        tg[u] = dgamma && in ? dg_nc[(int64_t)(n + u) * C + c] : 0.f;
        tb[u] = dbeta && in ? db_nc[(int64_t)(n + u) * C + c] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        sg += tg[u];
        sb += tb[u];
      }
    }
  }
  red[0][w][lane] = sg;
  red[1][w][lane] = sb;
  __syncthreads();
  if (w != 0 || c >= C) return;
  if (dgamma) dgamma[c] = ((red[0][0][lane] + red[0][1][lane]) + red[0][2][lane]) + red[0][3][lane];
  if (dbeta) dbeta[c] = ((red[1][0][lane] + red[1][1][lane]) + red[1][2][lane]) + red[1][3][lane];
}

// ---------------------------------------------------------------- dispatch

constexpr int kSplitChunk = 256 * 16 * 4;  // floats per split-path chunk (W = 4)

struct Plan {
  bool resident;
  int W;
  int splits;
  int chunk;
};

Plan make_plan(int64_t S, int64_t HW, bool aligned, int64_t resident_max) {
  Plan p{};
  p.W = (HW % 4 == 0 && aligned) ? 4 : 1;
  p.resident = S <= resident_max;
  p.chunk = kSplitChunk / (4 / p.W);
  p.splits = (int)bpk::ceil_div(S, p.chunk);
  return p;
}

template <int W>
int fwd_resident_dispatch(int64_t S, const float* x, const float* bias, const float* gamma,
                          const float* beta, float* y, float* mean, float* rstd, int N, int C,
                          int HW, int G, float eps, int act, hipStream_t st) {
  const int64_t units = bpk::ceil_div(S, W);
  dim3 grid(N * G);
#define GN_FWD(T_, V_)                                                                         \
  if (units <= (int64_t)(T_) * (V_)) {                                                         \
    hipLaunchKernelGGL((gn_fwd_resident<T_, V_, W>), grid, dim3(T_), 0, st, x, bias, gamma,   \
                       beta, y, mean, rstd, C, HW, G, eps, act);                               \
    BPK_LAUNCH_CHECK("group_norm_fwd_resident");                                              \
    return BPK_OK;                                                                             \
  }
  GN_FWD(256, 1)
  GN_FWD(256, 2)
  GN_FWD(256, 4)
  GN_FWD(256, 8)
  GN_FWD(512, 8)
  GN_FWD(1024, 8)
  GN_FWD(1024, 16)
#undef GN_FWD
  bpk::set_error("group_norm: slab too large for resident path");
  return BPK_ERR_ARG;
}

template <int W>
int bwd_resident_dispatch(int64_t S, const float* dy, const float* x, const float* bias,
                          const float* gamma, const float* beta, const float* mean,
                          const float* rstd, float* dx, float* dg, float* db, int N, int C, int HW,
                          int G, int act, const float* addend, hipStream_t st) {
  const int64_t units = bpk::ceil_div(S, W);
  const int cpg = C / G;
  dim3 grid(N * G);
#define GN_BWD(T_, V_)                                                                         \
  if (units <= (int64_t)(T_) * (V_)) {                                                         \
    const size_t sh = sizeof(float) * ((T_) / kWave + 2 * cpg + 2 * (V_) * ((T_) / kWave)); \
    hipLaunchKernelGGL((gn_bwd_resident<T_, V_, W>), grid, dim3(T_), sh, st, dy, x, bias,     \
                       gamma, beta, mean, rstd, dx, dg, db, C, HW, G, act, addend);            \
    BPK_LAUNCH_CHECK("group_norm_bwd_resident");                                              \
    return BPK_OK;                                                                             \
  }
  GN_BWD(256, 1)
  GN_BWD(256, 2)
  GN_BWD(256, 4)
  GN_BWD(256, 8)
  GN_BWD(512, 8)
  GN_BWD(1024, 8)
#undef GN_BWD
  bpk::set_error("group_norm: slab too large for resident backward");
  return BPK_ERR_ARG;
}

constexpr int64_t kFwdResidentMax = 1024 * 16 * 4;
constexpr int64_t kBwdResidentMax = 1024 * 8 * 4;

bool is_aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" int64_t bpk_group_norm_workspace_bytes(int N, int C, int64_t HW, int G) {
  if (N <= 0 || G <= 0 || C % G != 0) return 0;
  const int64_t S = (int64_t)(C / G) * HW;
  const int64_t splits = bpk::ceil_div(S, kSplitChunk / 4);  // worst case W = 1
  // backward split path: per-block (A, B) partials + per-(channel, slice) (dgamma, dbeta)
  const int64_t bpg = splits + C / G, spc = bpk::ceil_div(HW, kSplitChunk / 4);
  const int64_t bwd = ((int64_t)N * G * bpg + (int64_t)N * C * spc) * 2;
  return std::max<int64_t>((int64_t)N * G * splits * 3, bwd) * (int64_t)sizeof(float);
}

extern "C" int bpk_group_norm_fwd_f32(const float* x, const float* bias_nc, const float* gamma,
                                      const float* beta, float* y, float* mean, float* rstd,
                                      void* workspace, int N, int C, int64_t HW, int G, float eps,
                                      int act, void* stream) {
  BPK_REQUIRE(N >= 0 && C > 0 && HW > 0 && G > 0, "group_norm: bad shape");
  BPK_REQUIRE(C % G == 0, "group_norm: C (%d) not divisible by G (%d)", C, G);
  BPK_REQUIRE(act == 0 || act == 1, "group_norm: act must be 0 (none) or 1 (silu)");
  BPK_REQUIRE(HW < (1ll << 31) / 64, "group_norm: plane too large");
  if (N == 0) return BPK_OK;
  const int64_t S = (int64_t)(C / G) * HW;
  BPK_REQUIRE(S < (1ll << 31), "group_norm: slab too large");
  hipStream_t st = bpk::as_stream(stream);
  const Plan p = make_plan(S, HW, is_aligned16(x) && is_aligned16(y), kFwdResidentMax);
  if (p.resident) {
    if (p.W == 4)
      return fwd_resident_dispatch<4>(S, x, bias_nc, gamma, beta, y, mean, rstd, N, C, (int)HW, G,
                                      eps, act, st);
    return fwd_resident_dispatch<1>(S, x, bias_nc, gamma, beta, y, mean, rstd, N, C, (int)HW, G,
                                    eps, act, st);
  }
  BPK_REQUIRE(workspace != nullptr, "group_norm: split path needs a workspace");
  float* part = static_cast<float*>(workspace);
  dim3 grid(p.splits, N * G);
  if (p.W == 4) {
    hipLaunchKernelGGL((gn_fwd_partial<256, 16, 4>), grid, dim3(256), 0, st, x, bias_nc, part, C,
                       (int)HW, G, p.splits);
    BPK_LAUNCH_CHECK("group_norm_fwd_partial");
    hipLaunchKernelGGL((gn_fwd_apply<4>), grid, dim3(256), 0, st, x, bias_nc, gamma, beta, part, y,
                       mean, rstd, C, (int)HW, G, p.splits, p.chunk, eps, act);
  } else {
    hipLaunchKernelGGL((gn_fwd_partial<256, 16, 1>), grid, dim3(256), 0, st, x, bias_nc, part, C,
                       (int)HW, G, p.splits);
    BPK_LAUNCH_CHECK("group_norm_fwd_partial");
    hipLaunchKernelGGL((gn_fwd_apply<1>), grid, dim3(256), 0, st, x, bias_nc, gamma, beta, part, y,
                       mean, rstd, C, (int)HW, G, p.splits, p.chunk, eps, act);
  }
  BPK_LAUNCH_CHECK("group_norm_fwd_apply");
  return BPK_OK;
}

extern "C" int bpk_group_norm_bwd_f32(const float* dy, const float* x, const float* bias_nc,
                                      const float* gamma, const float* beta, const float* mean,
                                      const float* rstd, float* dx, float* dgamma_nc,
                                      float* dbeta_nc, void* workspace, int N, int C, int64_t HW,
                                      int G, int act, void* stream) {
  return bpk_group_norm_bwd_add_f32(dy, x, bias_nc, gamma, beta, mean, rstd, nullptr, dx,
                                    dgamma_nc, dbeta_nc, workspace, N, C, HW, G, act, stream);
}

extern "C" int bpk_group_norm_bwd_add_f32(const float* dy, const float* x, const float* bias_nc,
                                          const float* gamma, const float* beta,
                                          const float* mean, const float* rstd,
                                          const float* addend, float* dx, float* dgamma_nc,
                                          float* dbeta_nc, void* workspace, int N, int C,
                                          int64_t HW, int G, int act, void* stream) {
  BPK_REQUIRE(N >= 0 && C > 0 && HW > 0 && G > 0, "group_norm_bwd: bad shape");
  BPK_REQUIRE(C % G == 0, "group_norm_bwd: C (%d) not divisible by G (%d)", C, G);
  BPK_REQUIRE(act == 0 || act == 1, "group_norm_bwd: act must be 0 or 1");
  BPK_REQUIRE(mean && rstd, "group_norm_bwd: mean/rstd required");
  if (N == 0) return BPK_OK;
  const int64_t S = (int64_t)(C / G) * HW;
  BPK_REQUIRE(S < (1ll << 31), "group_norm_bwd: slab too large");
  hipStream_t st = bpk::as_stream(stream);
  const bool al = is_aligned16(x) && is_aligned16(dy) && is_aligned16(dx) &&
                  (!addend || is_aligned16(addend));
  const Plan p = make_plan(S, HW, al, kBwdResidentMax);
  if (p.resident) {
    if (p.W == 4)
      return bwd_resident_dispatch<4>(S, dy, x, bias_nc, gamma, beta, mean, rstd, dx, dgamma_nc,
                                      dbeta_nc, N, C, (int)HW, G, act, addend, st);
    return bwd_resident_dispatch<1>(S, dy, x, bias_nc, gamma, beta, mean, rstd, dx, dgamma_nc,
                                    dbeta_nc, N, C, (int)HW, G, act, addend, st);
  }
  BPK_REQUIRE(workspace != nullptr, "group_norm_bwd: split path needs a workspace");
  const int cpg = C / G;
  const int CH = p.chunk;
  const int bpg = bwd_bpg((int)HW, cpg, CH);
  float2* part_ab = static_cast<float2*>(workspace);
  float2* part_c = part_ab + (int64_t)N * G * bpg;
  const int want_c = (dgamma_nc || dbeta_nc) ? 1 : 0;
  dim3 grid(bpg, N * G);
  if (p.W == 4) {
    hipLaunchKernelGGL(gn_bwd_partial2<4>, grid, dim3(256), 0, st, dy, x, bias_nc, gamma, beta,
                       mean, rstd, part_ab, part_c, want_c, C, (int)HW, G, CH, act);
    BPK_LAUNCH_CHECK("group_norm_bwd_partial");
    hipLaunchKernelGGL(gn_bwd_apply2<4>, grid, dim3(256), 0, st, dy, x, bias_nc, gamma, beta,
                       mean, rstd, part_ab, part_c, dx, dgamma_nc, dbeta_nc, C, (int)HW, G, CH,
                       act, addend);
  } else {
    hipLaunchKernelGGL(gn_bwd_partial2<1>, grid, dim3(256), 0, st, dy, x, bias_nc, gamma, beta,
                       mean, rstd, part_ab, part_c, want_c, C, (int)HW, G, CH, act);
    BPK_LAUNCH_CHECK("group_norm_bwd_partial");
    hipLaunchKernelGGL(gn_bwd_apply2<1>, grid, dim3(256), 0, st, dy, x, bias_nc, gamma, beta,
                       mean, rstd, part_ab, part_c, dx, dgamma_nc, dbeta_nc, C, (int)HW, G, CH,
                       act, addend);
  }
  BPK_LAUNCH_CHECK("group_norm_bwd_apply");
  return BPK_OK;
}

extern "C" int bpk_group_norm_param_grads_f32(const float* dx, const float* dgamma_nc,
                                              const float* dbeta_nc, float* d_bias_nc,
                                              float* dgamma, float* dbeta, int N, int C,
                                              int64_t HW, void* stream) {
  BPK_REQUIRE(N > 0 && C > 0 && HW > 0 && HW < (1ll << 31), "group_norm_param_grads: bad shape");
  BPK_REQUIRE(!d_bias_nc || dx, "group_norm_param_grads: d_bias_nc needs dx");
  BPK_REQUIRE(!dgamma || dgamma_nc, "group_norm_param_grads: dgamma needs dgamma_nc");
  BPK_REQUIRE(!dbeta || dbeta_nc, "group_norm_param_grads: dbeta needs dbeta_nc");
  const int rows = d_bias_nc ? N * C : 0;
  const int cols = (dgamma || dbeta) ? (int)bpk::ceil_div(C, 64) : 0;
  if (rows + cols == 0) return BPK_OK;
  hipLaunchKernelGGL(gn_param_grads_kernel, dim3(rows + cols), dim3(256), 0,
                     bpk::as_stream(stream), dx, dgamma_nc, dbeta_nc, d_bias_nc, dgamma, dbeta, N,
                     C, (int)HW, rows);
  BPK_LAUNCH_CHECK("group_norm_param_grads");
  return BPK_OK;
}

extern "C" int bpk_group_norm_affine_stats_f32(const float* x, const float* bias_nc,
                                               const float* gamma, const float* beta,
                                               float* scale_shift, float* mean, float* rstd,
                                               void* workspace, int N, int C, int64_t HW, int G,
                                               float eps, void* stream) {
  BPK_REQUIRE(N >= 0 && C > 0 && HW > 0 && G > 0, "group_norm_affine: bad shape");
  BPK_REQUIRE(C % G == 0, "group_norm_affine: C (%d) not divisible by G (%d)", C, G);
  BPK_REQUIRE(workspace != nullptr, "group_norm_affine: workspace required");
  if (N == 0) return BPK_OK;
  const int64_t S = (int64_t)(C / G) * HW;
  BPK_REQUIRE(S < (1ll << 31), "group_norm_affine: slab too large");
  hipStream_t st = bpk::as_stream(stream);
  const Plan p = make_plan(S, HW, is_aligned16(x), 0);
  float* part = static_cast<float*>(workspace);
  dim3 grid(p.splits, N * G);
  if (p.W == 4)
    hipLaunchKernelGGL((gn_fwd_partial<256, 16, 4>), grid, dim3(256), 0, st, x, bias_nc, part, C,
                       (int)HW, G, p.splits);
  else
    hipLaunchKernelGGL((gn_fwd_partial<256, 16, 1>), grid, dim3(256), 0, st, x, bias_nc, part, C,
                       (int)HW, G, p.splits);
  BPK_LAUNCH_CHECK("group_norm_affine(partial)");
  hipLaunchKernelGGL(gn_affine_kernel, dim3(N * G), dim3(64), 0, st, part, bias_nc, gamma, beta,
                     reinterpret_cast<float2*>(scale_shift), mean, rstd, C, G, p.splits, eps);
  BPK_LAUNCH_CHECK("group_norm_affine");
  return BPK_OK;
}

extern "C" int bpk_group_norm_affine_f32(const float* x, const float* bias_nc, const float* gamma,
                                         const float* beta, float* scale_shift, void* workspace,
                                         int N, int C, int64_t HW, int G, float eps,
                                         void* stream) {
  return bpk_group_norm_affine_stats_f32(x, bias_nc, gamma, beta, scale_shift, nullptr, nullptr,
                                         workspace, N, C, HW, G, eps, stream);
}

// ---------------------------------------------------------------- statistics from partials
// GroupNorm (s, t) from per-(n, channel, region) partial statistics written by the producer
// of x (the Winograd conv's epilogue, bpk_conv3x3_wino_ex_f32): part[n][c][r] = (mean, M2) of
// `cnt` values each.  Equal counts, so the group mean is the mean of the partial means
// (+ the per-channel bias) and M2 = sum(M2_i + cnt (mean_i + b_c - mean)^2) -- two passes
// over the partials, fixed reduction order (deterministic).
namespace {
__global__ __launch_bounds__(256) void gn_affine_partials_kernel(
    const float2* __restrict__ part, const float2* __restrict__ part2, int C1, int R, float cnt,
    const float* __restrict__ bias_nc, const float* __restrict__ gamma,
    const float* __restrict__ beta, float2* __restrict__ ss, float* __restrict__ mean_out,
    float* __restrict__ rstd_out, int C, int G, float eps) {
  __shared__ float sbuf[256 / kWave];
  __shared__ float s_stat[2];
  const int ng = blockIdx.x;
  const int n = ng / G;
  const int g = ng - n * G;
  const int cpg = C / G;
  const int K = cpg * R;
  // partials of channel c: part [N, C1, R] for c < C1, part2 [N, C - C1, R] after (the two
  // halves of a channel concatenation, read in place)
  const int c0 = g * cpg;
  auto at = [&](int i) -> float2 {
    const int c = c0 + i / R, r = i - (i / R) * R;
    return c < C1 ? part[((int64_t)n * C1 + c) * R + r]
                  : part2[((int64_t)n * (C - C1) + (c - C1)) * R + r];
  };
  const float* bn = bias_nc ? bias_nc + (int64_t)n * C + c0 : nullptr;
  float ls = 0.f;
  for (int i = threadIdx.x; i < K; i += blockDim.x) ls += at(i).x + (bn ? bn[i / R] : 0.f);
  const float mean = block_sum<256>(ls, sbuf) / (float)K;
  float lm2 = 0.f;
  for (int i = threadIdx.x; i < K; i += blockDim.x) {
    const float2 p = at(i);
    const float d = p.x + (bn ? bn[i / R] : 0.f) - mean;
    lm2 += p.y + cnt * d * d;
  }
  const float m2 = block_sum<256>(lm2, sbuf);
  if (threadIdx.x == 0) {
    s_stat[0] = mean;
    s_stat[1] = 1.f / sqrtf(m2 / ((float)K * cnt) + eps);
    if (mean_out) mean_out[ng] = mean;
    if (rstd_out) rstd_out[ng] = s_stat[1];
  }
  __syncthreads();
  for (int j = threadIdx.x; j < cpg; j += blockDim.x) {
    const int c = g * cpg + j;
    const float sc = s_stat[1] * (gamma ? gamma[c] : 1.f);
    const float b = bias_nc ? bias_nc[(int64_t)n * C + c] : 0.f;
    ss[(int64_t)n * C + c] = make_float2(sc, (beta ? beta[c] : 0.f) + (b - s_stat[0]) * sc);
  }
}

// (mean, M2) of every 128 consecutive values of x: one wave per chunk, one float2 per lane.
// For a plane of H*W % 128 == 0 pixels these are the GroupNorm partial statistics of
// bpk_group_norm_affine_partials_f32 (R = H*W / 128 per (n, c), cnt = 128) for a tensor
// whose producer wrote none.
__global__ __launch_bounds__(256) void gn_chunk_partials_kernel(const float* __restrict__ x,
                                                                float2* __restrict__ part,
                                                                int64_t nchunks) {
  const int64_t ch = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (ch >= nchunks) return;  // wave-uniform
  const int lane = threadIdx.x & 63;
  const float2 v = reinterpret_cast<const float2*>(x + ch * 128)[lane];
  float s = v.x + v.y;
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, kWave);
  const float mean = s * (1.f / 128.f);
  const float a = v.x - mean, b = v.y - mean;
  float m2 = a * a + b * b;
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) m2 += __shfl_xor(m2, off, kWave);
  if (lane == 0) part[ch] = make_float2(mean, m2);
}
}  // namespace

extern "C" int bpk_group_norm_affine_partials_stats_f32(const float* part, int R, int cnt,
                                                        const float* bias_nc, const float* gamma,
                                                        const float* beta, float* scale_shift,
                                                        float* mean, float* rstd, int N, int C,
                                                        int G, float eps, void* stream) {
  BPK_REQUIRE(N >= 0 && C > 0 && G > 0 && R > 0 && cnt > 0,
              "group_norm_affine_partials: bad shape");
  BPK_REQUIRE(C % G == 0, "group_norm_affine_partials: C (%d) not divisible by G (%d)", C, G);
  BPK_REQUIRE((int64_t)(C / G) * R < (1ll << 31), "group_norm_affine_partials: too many partials");
  if (N == 0) return BPK_OK;
  hipLaunchKernelGGL(gn_affine_partials_kernel, dim3(N * G), dim3(256), 0, bpk::as_stream(stream),
                     reinterpret_cast<const float2*>(part), nullptr, C, R, (float)cnt, bias_nc,
                     gamma, beta, reinterpret_cast<float2*>(scale_shift), mean, rstd, C, G, eps);
  BPK_LAUNCH_CHECK("group_norm_affine_partials");
  return BPK_OK;
}

extern "C" int bpk_group_norm_affine_partials_f32(const float* part, int R, int cnt,
                                                  const float* bias_nc, const float* gamma,
                                                  const float* beta, float* scale_shift, int N,
                                                  int C, int G, float eps, void* stream) {
  return bpk_group_norm_affine_partials_stats_f32(part, R, cnt, bias_nc, gamma, beta,
                                                  scale_shift, nullptr, nullptr, N, C, G, eps,
                                                  stream);
}

extern "C" int bpk_group_norm_affine_partials2_f32(const float* part, int C1, const float* part2,
                                                   int R, int cnt, const float* bias_nc,
                                                   const float* gamma, const float* beta,
                                                   float* scale_shift, int N, int C, int G,
                                                   float eps, void* stream) {
  BPK_REQUIRE(N >= 0 && C > 0 && G > 0 && R > 0 && cnt > 0 && C1 > 0 && C1 < C,
              "group_norm_affine_partials2: bad shape");
  BPK_REQUIRE(C % G == 0, "group_norm_affine_partials2: C (%d) not divisible by G (%d)", C, G);
  BPK_REQUIRE((int64_t)(C / G) * R < (1ll << 31), "group_norm_affine_partials2: too many partials");
  if (N == 0) return BPK_OK;
  hipLaunchKernelGGL(gn_affine_partials_kernel, dim3(N * G), dim3(256), 0, bpk::as_stream(stream),
                     reinterpret_cast<const float2*>(part), reinterpret_cast<const float2*>(part2),
                     C1, R, (float)cnt, bias_nc, gamma, beta,
                     reinterpret_cast<float2*>(scale_shift), nullptr, nullptr, C, G, eps);
  BPK_LAUNCH_CHECK("group_norm_affine_partials2");
  return BPK_OK;
}

extern "C" int bpk_group_norm_chunk_partials_f32(const float* x, float* part, int N, int C,
                                                 int64_t HW, void* stream) {
  BPK_REQUIRE(N >= 0 && C > 0 && HW > 0 && HW % 128 == 0,
              "group_norm_chunk_partials: need H*W %% 128 == 0 (got %lld)", (long long)HW);
  const int64_t nchunks = (int64_t)N * C * (HW / 128);
  if (nchunks == 0) return BPK_OK;
  BPK_REQUIRE(bpk::ceil_div(nchunks, 4) < (1LL << 31), "group_norm_chunk_partials: too large");
  hipLaunchKernelGGL(gn_chunk_partials_kernel, dim3((unsigned)bpk::ceil_div(nchunks, 4)),
                     dim3(256), 0, bpk::as_stream(stream), x, reinterpret_cast<float2*>(part),
                     nchunks);
  BPK_LAUNCH_CHECK("group_norm_chunk_partials");
  return BPK_OK;
}

// ---------------------------------------------------------------- per-(n, c) affine + SiLU
// y = silu(x * s + t), (s, t) = scale_shift[n][c]: the activation the Winograd conv's
// GroupNorm prologue computes in its patch load, materialised when a weight gradient needs it
// (op.norm_act.affine_silu; the same expression as the prologue: one FMA, __expf, rcp).
namespace {
__global__ __launch_bounds__(256) void affine_silu_kernel(const float* __restrict__ x,
                                                          const float2* __restrict__ ss,
                                                          float* __restrict__ y, int64_t planes,
                                                          int HW, int vec) {
  const int64_t pl = blockIdx.y + (int64_t)blockIdx.z * 65535;
  if (pl >= planes) return;
  const float2 st = ss[pl];
  const int64_t base = pl * HW;
  if (vec) {
    for (int e = (blockIdx.x * 256 + threadIdx.x) * 4; e < HW; e += gridDim.x * 256 * 4) {
      const float4 v = *reinterpret_cast<const float4*>(x + base + e);
      float o[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float z = o[q] * st.x + st.y;
        o[q] = z * __builtin_amdgcn_rcpf(1.f + __expf(-z));
      }
      *reinterpret_cast<float4*>(y + base + e) = make_float4(o[0], o[1], o[2], o[3]);
    }
  } else {
    for (int e = blockIdx.x * 256 + threadIdx.x; e < HW; e += gridDim.x * 256) {
      const float z = x[base + e] * st.x + st.y;
      y[base + e] = z * __builtin_amdgcn_rcpf(1.f + __expf(-z));
    }
  }
}
}  // namespace

extern "C" int bpk_affine_silu_f32(const float* x, const float* scale_shift, float* y, int N,
                                   int C, int64_t HW, void* stream) {
  BPK_REQUIRE(N >= 0 && C > 0 && HW > 0 && HW < (1ll << 31), "affine_silu: bad shape");
  BPK_REQUIRE(x && scale_shift && y, "affine_silu: null pointer");
  const int64_t planes = (int64_t)N * C;
  if (planes == 0) return BPK_OK;
  const int vec = (HW % 4 == 0 && is_aligned16(x) && is_aligned16(y)) ? 1 : 0;
  const int64_t per = vec ? bpk::ceil_div(HW, 4) : HW;
  const unsigned bx = (unsigned)std::min<int64_t>(bpk::ceil_div(per, 256), 64);
  const dim3 grid(bx, (unsigned)std::min<int64_t>(planes, 65535),
                  (unsigned)bpk::ceil_div(planes, 65535));
  hipLaunchKernelGGL(affine_silu_kernel, grid, dim3(256), 0, bpk::as_stream(stream), x,
                     reinterpret_cast<const float2*>(scale_shift), y, planes, (int)HW, vec);
  BPK_LAUNCH_CHECK("affine_silu");
  return BPK_OK;
}
