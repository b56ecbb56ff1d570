// 3x3 / stride 1 / pad 1 fp32 convolution as fused Winograd F(2x2, 3x3) on the
// f32-input MFMA (v_mfma_f32_16x16x4_f32) for gfx950.
//
// The score networks' convolutions (models/layerspp.py, layers.py: every 3x3 conv of
// NCSN++ / DDPM++) are ~99 % of their FLOPs.  Winograd F(2,3) computes a 2x2 output
// tile from a 4x4 input tile with 16 multiplies per (cin, cout) instead of 36:
//     Y = A^T [ sum_cin (G g G^T) .* (B^T d B) ] A
// so for each of the 16 transform positions the contraction over cin is a GEMM
//     M_pos[tile, cout] = sum_cin V_pos[tile, cin] * U_pos[cin, cout]
// which runs on MFMA with exact f32 products (a k-ordered fma chain).
//
// Kernel shape (one workgroup = 4 waves, 256 threads):
//   * output region: 4 x 8 tiles (8 x 16 pixels) of one image -> M = 32 tiles,
//     64 output channels (wave w owns couts [16w, 16w + 16));
//   * K loop over cin in chunks of 8: the 8 x 10 x 18 input patch is loaded to LDS,
//     each thread transforms one (cin, tile) pair into its 16 V values (LDS), then every
//     wave issues 16 positions x 2 M-blocks x 2 k-steps = 64 MFMAs 16x16x4 against its
//     U operands, prefetched from global one chunk ahead;
//   * accumulators: 16 positions x 2 M-blocks x 4 = 128 f32 per lane; the output
//     transform is lane-local (all 16 positions of a (tile, cout) sit in one lane), the
//     result goes through LDS so every global store is a 64-B row segment;
//   * XCD-aware block order: the cout-blocks of one spatial region are consecutive in
//     the logical order, which is dealt to one XCD, so they share the input patch in L2.
// Filter transform U = G g G^T (16 x cin x cout) is a separate, tiny kernel; callers
// cache U while the weights do not change (sampling).
#include "bpk_common.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace {

using f4 = __attribute__((ext_vector_type(4))) float;

constexpr int kTR = 4, kTC = 8;          // tiles per region (rows, cols)
constexpr int kM = kTR * kTC;            // 32 tiles
constexpr int kPR = 2 * kTR + 2;         // 10 patch rows
constexpr int kPC = 2 * kTC + 2;         // 18 patch cols
// LDS row pitch of the input patch: 24 floats.  The V transform reads each 4 x 4 input tile
// as 8 ds_read_b64 at dword offsets 24 (2 ty + i) + 2 tx: per 32-lane group (one cin, 32
// tiles) the four tile rows land on dword banks {0-15, 48-63, 32-47, 16-31} (48 ty mod 64)
// -- all 64 banks once, conflict-free (a pitch of 19 with 16 ds_read_b32 was 2-way)
constexpr int kPCp = 24;
constexpr int kCK = 8;                   // cin per chunk
constexpr int kOutRows = 2 * kTR, kOutCols = 2 * kTC;  // 8 x 16 pixels

// U[cin][cout][pos] = (G g G^T)[pos] with G = [[1,0,0],[.5,.5,.5],[.5,-.5,.5],[0,0,1]]
// (the 16 positions of one (cin, cout) pair are contiguous: one lane of the GEMM loads
// its B operands for all positions with four 16-B loads)
// Cout not a multiple of 64: U is laid out for CoutP = Cout rounded up to 64 couts, the
// extra couts zero (the conv computes them and never stores them).
__device__ inline void wino_filter_range(const float* __restrict__ w, float* __restrict__ U,
                                         int Cin, int Cout, int CoutP, int ft, int64_t first,
                                         int64_t stride) {
  const int64_t total = (int64_t)Cin * CoutP;
  for (int64_t i = first; i < total; i += stride) {
    const int co = (int)(i % CoutP);
    const int ci = (int)(i / CoutP);
    if (co >= Cout) {
      f4* u = reinterpret_cast<f4*>(U + ((int64_t)ci * CoutP + co) * 16);
#pragma unroll
      for (int r = 0; r < 4; ++r) u[r] = f4{0.f, 0.f, 0.f, 0.f};
      continue;
    }
    // ft: the filter is flip_t(w) for w [Cin, Cout, 3, 3] (backward-data of the conv with
    // w): element (co, ci, r, s) = w[ci][co][2 - r][2 - s], read in place
    const float* g = ft ? w + ((int64_t)ci * Cout + co) * 9 : w + ((int64_t)co * Cin + ci) * 9;
    auto gv = [&](int k) { return ft ? g[8 - k] : g[k]; };
    float t[4][3];  // G g
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float g0 = gv(c), g1 = gv(3 + c), g2 = gv(6 + c);
      t[0][c] = g0;
      t[1][c] = 0.5f * (g0 + g1 + g2);
      t[2][c] = 0.5f * (g0 - g1 + g2);
      t[3][c] = g2;
    }
    float* u = U + ((int64_t)ci * CoutP + co) * 16;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float a0 = t[r][0], a1 = t[r][1], a2 = t[r][2];
      u[4 * r + 0] = a0;
      u[4 * r + 1] = 0.5f * (a0 + a1 + a2);
      u[4 * r + 2] = 0.5f * (a0 - a1 + a2);
      u[4 * r + 3] = a2;
    }
  }
}

__global__ __launch_bounds__(256) void wino_filter_kernel(const float* __restrict__ w,
                                                          float* __restrict__ U, int Cin,
                                                          int Cout, int CoutP, int ft) {
  wino_filter_range(w, U, Cin, Cout, CoutP, ft, (int64_t)blockIdx.x * blockDim.x + threadIdx.x,
                    (int64_t)gridDim.x * blockDim.x);
}

// many filters in one launch (op.conv.FilterBatch: every 3x3 conv weight of a model, forward
// and flipped, refreshed once per training step instead of one launch per conv call): job j =
// jobs[6 j .. 6 j + 5] = (w, U, Cin, Cout, CoutP, ft), blockIdx.y = j
__global__ __launch_bounds__(256) void wino_filter_batch_kernel(const int64_t* __restrict__ jobs) {
  const int64_t* jb = jobs + 6 * (int64_t)blockIdx.y;
  wino_filter_range(reinterpret_cast<const float*>(jb[0]), reinterpret_cast<float*>(jb[1]),
                    (int)jb[2], (int)jb[3], (int)jb[4], (int)jb[5],
                    (int64_t)blockIdx.x * blockDim.x + threadIdx.x,
                    (int64_t)gridDim.x * blockDim.x);
}

struct WinoGeo {
  int N, Cin, Cout, H, W;
  int regions_x, regions_y, cout_blocks;
  float div;  // fused residual: y = (skip + (conv + bias)) / div when skip != nullptr
  int C1;     // input channels [0, C1) from x, [C1, Cin) from x2 (pipelined kernel only)
  int CoutS;  // couts stored (y, skip, stats channel count); Cout = CoutS rounded up to 64
  int up;     // 16-cin kernel only: 1 = x is [N, Cin, H/2, W/2], convolved as its nearest x2
              // upsample (the ddpm net's Upsample + Conv_0, reference layers.py:576-590)
  int ksplit; // 16-cin kernel only: > 1 = split-K over the input channels; workgroup s of a tile
              // contracts chunks [s, s + 1) * nch / ksplit and writes its raw partial output to
              // y + s * N * CoutS * H * W (no bias / tail / statistics: wino_splitk_reduce_kernel)
  int pair;   // 16-cin kernel only: 1 = W == 8, a region is two 8 x 8 images side by side
              // (images 2p, 2p + 1; regions_x = 1, N even, one source, no statistics)
};

constexpr int kVS = 20;                  // LDS stride of one (cin, tile) V record (16 + pad)
constexpr int kOS = kOutRows * kOutCols + 4;  // LDS stride of one staged output channel
constexpr int kPatchPerThread = (kCK * kPR * kPC + 255) / 256;  // 6
constexpr int kPreMaxCin = 1024;        // pipelined kernel: GroupNorm affine table in LDS

// NB = MFMA N-blocks (16 couts each) per wave: NB = 2 -> 256 accumulator registers, one
// workgroup per CU; NB = 1 -> 128, two workgroups per CU whose phases interleave.
// PRE: the conv input is act(GroupNorm(x + b)) given as x and its per-(n, cin) affine form
// pre[n][cin] = (s, t) (bpk_group_norm_affine_f32): the patch load applies silu(x s + t)
// (zero padding stays zero), so the normalized tensor is never written to HBM.
// fast exp / reciprocal: a few ulp, far inside the network tolerance (1e-4)

__device__ inline float silu_f(float z) { return z * __builtin_amdgcn_rcpf(1.f + __expf(-z)); }

// q = a / d, r = a % d for a block index: a shift when d is a power of two (every NCSN++ /
// DDPM++ shape), else a 32-bit unsigned division -- the 64-bit forms were ~600 scalar
// instructions of the workgroup prologue
__device__ inline unsigned udivmod(unsigned a, unsigned d, unsigned& r) {
  if ((d & (d - 1)) == 0) {
    r = a & (d - 1);
    return a >> __builtin_ctz(d);
  }
  const unsigned q = a / d;
  r = a - q * d;
  return q;
}

// a / b correctly rounded (== IEEE division, bit for bit) from r = 1 / b (correctly rounded,
// computed once): q = a r, then one Markstein correction with the exact residual a - b q.
// 3 VALU instead of the ~10 of a full-range division (the residual tail divides by sqrt 2).
__device__ inline float div_rn(float a, float b, float r) {
  const float q = a * r;
  return fmaf(fmaf(-q, b, a), r, q);
}

// Coalesced stores of one wave's staged output (kWN couts x 8 rows x 16 cols, LDS s_w[co]
// at stride kOS), with the residual-block tail, and -- stats != nullptr -- the GroupNorm
// partial statistics of the stored values: stats[n][cout][region] = (mean, M2) of the
// region's 128 pixels (bpk_group_norm_affine_partials_f32 consumes them, so the next
// GroupNorm needs no statistics pass over this tensor).  Per iteration the 32 lanes of a
// half-wave hold one channel's 128 values; the butterfly merge (equal counts) gives every
// lane the same bits.
template <int CTRL>
__device__ inline float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Chan merge of two equal-count partials (count c each); symmetric in its arguments, so both
// partners of a butterfly get the same bits
__device__ inline void merge_stats(float& m, float& m2, float mo, float m2o, float c) {
  const float d = mo - m;
  m2 = (m2 + m2o) + d * d * (0.5f * c);
  m = 0.5f * (m + mo);
}

template <int kWN>
__device__ inline void store_tile(const float* s_w, const float* __restrict__ skip,
                                  float* __restrict__ y, float2* __restrict__ stats,
                                  const WinoGeo& g, int n, int cout_w, int oy0, int ox0, int lane) {
  if (cout_w >= g.CoutS) return;  // padded couts (wave-uniform: CoutS % 16 == 0)
  const int64_t plane = (int64_t)g.H * g.W;
  constexpr int kIt = kWN / 2;
  float mm[kIt], qq[kIt];
  auto out_off = [&](int it) {
    const int q = it * 64 + lane;
    const int co = q >> 5;                 // 32 float4 per cout (8 rows x 4)
    const int rem = q & 31;
    const int row = rem >> 2, c4 = rem & 3;
    return (int64_t)n * g.CoutS * plane + (int64_t)(cout_w + co) * plane +
           (int64_t)(oy0 + row) * g.W + ox0 + 4 * c4;
  };
  // residual tail: every skip vector of the tile requested before the first is used (one
  // exposed memory latency, as the 16-cin kernel's epilogue)
  f4 skv[kIt];
  if (skip) {
#pragma unroll
    for (int it = 0; it < kIt; ++it) skv[it] = *reinterpret_cast<const f4*>(&skip[out_off(it)]);
  }
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const int q = it * 64 + lane;
    const int co = q >> 5;
    const int rem = q & 31;
    const int row = rem >> 2, c4 = rem & 3;
    f4 v = *reinterpret_cast<const f4*>(&s_w[co * kOS + row * kOutCols + 4 * c4]);
    const int64_t o = out_off(it);
    if (skip) {  // residual block tail, same operation order as bpk_residual_rescale_f32
      const f4 sk = skv[it];
      v = f4{(sk[0] + v[0]) / g.div, (sk[1] + v[1]) / g.div, (sk[2] + v[2]) / g.div,
             (sk[3] + v[3]) / g.div};
    }
    *reinterpret_cast<f4*>(&y[o]) = v;
    mm[it] = ((v[0] + v[1]) + (v[2] + v[3])) * 0.25f;
    float m2 = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) m2 = fmaf(v[e] - mm[it], v[e] - mm[it], m2);
    qq[it] = m2;
  }
  if (!stats) return;
  // 32-lane reductions (one channel per half-wave and iteration), all iterations interleaved:
  // xor 1, xor 2 (quad_perm), 8-lane and 16-lane mirrors (DPP), then xor 16 (bpermute)
#pragma unroll
  for (int it = 0; it < kIt; ++it)
    merge_stats(mm[it], qq[it], dpp_f<0xB1>(mm[it]), dpp_f<0xB1>(qq[it]), 4.f);
#pragma unroll
  for (int it = 0; it < kIt; ++it)
    merge_stats(mm[it], qq[it], dpp_f<0x4E>(mm[it]), dpp_f<0x4E>(qq[it]), 8.f);
#pragma unroll
  for (int it = 0; it < kIt; ++it)
    merge_stats(mm[it], qq[it], dpp_f<0x141>(mm[it]), dpp_f<0x141>(qq[it]), 16.f);
#pragma unroll
  for (int it = 0; it < kIt; ++it)
    merge_stats(mm[it], qq[it], dpp_f<0x140>(mm[it]), dpp_f<0x140>(qq[it]), 32.f);
#pragma unroll
  for (int it = 0; it < kIt; ++it)
    merge_stats(mm[it], qq[it], __shfl_xor(mm[it], 16, 64), __shfl_xor(qq[it], 16, 64), 64.f);
  const int R = g.regions_x * g.regions_y;
  const int region = (oy0 / kOutRows) * g.regions_x + ox0 / kOutCols;
  if ((lane & 31) == 0) {
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int co = (it * 64 + lane) >> 5;
      stats[((int64_t)n * g.CoutS + cout_w + co) * R + region] = make_float2(mm[it], qq[it]);
    }
  }
}

template <int NB, bool PRE>
__global__ __launch_bounds__(256, NB == 1 ? 2 : 1) void wino_f23_kernel(const float* __restrict__ x,
                                                          const float* __restrict__ U,
                                                          const float* __restrict__ bias,
                                                          const float* __restrict__ skip,
                                                          const float2* __restrict__ pre,
                                                          float* __restrict__ y,
                                                          float2* __restrict__ stats, WinoGeo g,
                                                          int xcd_remap) {
  __shared__ float2 s_ss[2][kCK];  // PRE: (s, t) of the chunk's input channels
  // patch [cin][row][col] + a tail that absorbs the writes of out-of-patch slots (so the
  // stores are branch-free, like the loads)
  __shared__ float s_patch_raw[kCK * kPR * kPCp + 256];  //  7.1 KB
  float(*s_patch)[kPR][kPCp] = reinterpret_cast<float(*)[kPR][kPCp]>(s_patch_raw);
  __shared__ __attribute__((aligned(16))) float s_v[kCK * kM * kVS];  // 20.5 KB
  __shared__ __attribute__((aligned(16))) float s_out[4 * 16 * NB * kOS];  // 33.8 KB per NB

  constexpr int kWN = 16 * NB;  // couts per wave
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;

  // logical block index: blocks b and b + 8 share an XCD under round-robin placement,
  // so consecutive logical blocks (the cout-blocks of one region) read one input patch
  int64_t nblk = (int64_t)gridDim.x;
  int64_t b = blockIdx.x;
  if (xcd_remap) b = (b % 8) * (nblk / 8) + b / 8;
  const int cb = (int)(b % g.cout_blocks);
  int64_t r = b / g.cout_blocks;
  const int rx = (int)(r % g.regions_x);
  r /= g.regions_x;
  const int ry = (int)(r % g.regions_y);
  const int n = (int)(r / g.regions_y);
  const int oy0 = ry * kOutRows, ox0 = rx * kOutCols;
  const int cout_w = cb * (4 * kWN) + wave * kWN;  // first cout of this wave

  f4 acc[16][2][NB];
#pragma unroll
  for (int p = 0; p < 16; ++p)
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) acc[p][mb][nb] = f4{0.f, 0.f, 0.f, 0.f};

  const int64_t plane = (int64_t)g.H * g.W;
  const float* xn = x + (int64_t)n * g.Cin * plane;
  const int kq = lane >> 4, jj = lane & 15;

  // patch element i of this thread: (cin, row, col) of the 8 x 10 x 18 patch
  float pv[kPatchPerThread];
  // branch-free: every lane issues every load (out-of-image / tail elements read a valid
  // in-plane address and are zeroed after), so the outstanding-load count is static and
  // the compiler's vmcnt waits stay exact -- the prefetch really overlaps the MFMAs
  // the zero-padding select is applied when the values are stored to LDS (next chunk),
  // not here: a select right after a load would wait for that load immediately
  unsigned pmask = 0;
  auto load_patch = [&](int c0) {
    pmask = 0;
#pragma unroll
    for (int e = 0; e < kPatchPerThread; ++e) {
      const int i = tid + 256 * e;
      const bool in_patch = i < kCK * kPR * kPC;
      const int ii = in_patch ? i : 0;
      const int c = ii / (kPR * kPC);
      const int rr = ii - c * (kPR * kPC);
      const int py = rr / kPC, px = rr - py * kPC;
      const int iy = oy0 - 1 + py, ix = ox0 - 1 + px;
      const bool inb = in_patch && iy >= 0 && iy < g.H && ix >= 0 && ix < g.W;
      const int cy = min(max(iy, 0), g.H - 1), cx = min(max(ix, 0), g.W - 1);
      pv[e] = xn[(int64_t)(c0 + c) * plane + (int64_t)cy * g.W + cx];
      pmask |= inb ? (1u << e) : 0u;
    }
  };
  load_patch(0);

  // B operands: uo[ks][nb][q] = U[c0 + 4ks + kq][cout_w + 16nb + jj][4q..4q+3]; the next
  // chunk's are loaded right after this chunk's MFMAs have issued, so their latency
  // overlaps the patch store, the V transform and both barriers of the next chunk
  f4 uo[2][NB][4];
  auto load_u = [&](int c0) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const f4* src = reinterpret_cast<const f4*>(
            U + ((int64_t)(c0 + 4 * ks + kq) * g.Cout + cout_w + 16 * nb + jj) * 16);
#pragma unroll
        for (int q = 0; q < 4; ++q) uo[ks][nb][q] = src[q];
      }
  };
  load_u(0);
  const float2* pre_n = PRE ? pre + (int64_t)n * g.Cin : nullptr;
  float2 ss_next = make_float2(1.f, 0.f);
  if (PRE) {
    if (tid < kCK) s_ss[0][tid] = pre_n[tid];
    __syncthreads();
  }

  for (int c0 = 0; c0 < g.Cin; c0 += kCK) {
    const int sbuf = (c0 / kCK) & 1;
    // 1. patch registers -> LDS
#pragma unroll
    for (int e = 0; e < kPatchPerThread; ++e) {
      const int i = tid + 256 * e;
      const int c = i / (kPR * kPC);
      const int rr = i - c * (kPR * kPC);
      const int py = rr / kPC, px = rr - py * kPC;
      const int dst = i < kCK * kPR * kPC ? (c * kPR + py) * kPCp + px : kCK * kPR * kPCp + tid;
      float v = pv[e];
      if (PRE) {
        const float2 st = s_ss[sbuf][min(c, kCK - 1)];
        v = silu_f(v * st.x + st.y);
      }
      s_patch_raw[dst] = ((pmask >> e) & 1u) ? v : 0.f;
    }
    __syncthreads();
    // 2. V = B^T d B for one (cin, tile) per thread -> s_v[(c * 32 + m) * kVS + pos]
    {
      const int c = tid >> 5, m = tid & 31;
      const int ty = m / kTC, tx = m - ty * kTC;
      float d[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) d[i][j] = s_patch[c][2 * ty + i][2 * tx + j];
      float t[4][4];  // B^T d   (B^T = [[1,0,-1,0],[0,1,1,0],[0,-1,1,0],[0,1,0,-1]])
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        t[0][j] = d[0][j] - d[2][j];
        t[1][j] = d[1][j] + d[2][j];
        t[2][j] = d[2][j] - d[1][j];
        t[3][j] = d[1][j] - d[3][j];
      }
      f4* dst = reinterpret_cast<f4*>(&s_v[(c * kM + m) * kVS]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        dst[i] = f4{t[i][0] - t[i][2], t[i][1] + t[i][2], t[i][2] - t[i][1], t[i][1] - t[i][3]};
    }
    __syncthreads();
    // 3. next chunk's patch in flight during the MFMAs
    // (unconditional: the last chunk re-loads itself, so every iteration issues the same
    // loads and the compiler's vmcnt bookkeeping across the back edge stays exact)
    load_patch(min(c0 + kCK, g.Cin - kCK));
    if (PRE && tid < kCK) ss_next = pre_n[min(c0 + kCK, g.Cin - kCK) + tid];
    // 4. MFMAs: acc[p][mb][nb] += V_p[mb*16 + i][4ks + k] * U_p[4ks + k][16nb + j]
    // A operands (16 positions of one (ks, mb) group = 4 x 16 B) are read one group
    // ahead, so each group's LDS latency hides behind the previous group's MFMAs.
    {
      auto a_src = [&](int grp) {  // grp = 2 ks + mb
        const int ks = grp >> 1, mb = grp & 1;
        return reinterpret_cast<const f4*>(&s_v[((4 * ks + kq) * kM + mb * 16 + jj) * kVS]);
      };
      f4 a_cur[4], a_nxt[4];
      {
        const f4* src = a_src(0);
#pragma unroll
        for (int q = 0; q < 4; ++q) a_cur[q] = src[q];
      }
#pragma unroll
      for (int grp = 0; grp < 4; ++grp) {
        if (grp < 3) {
          const f4* src = a_src(grp + 1);
#pragma unroll
          for (int q = 0; q < 4; ++q) a_nxt[q] = src[q];
        }
        const int ks = grp >> 1, mb = grp & 1;
#pragma unroll
        for (int p = 0; p < 16; ++p)
#pragma unroll
          for (int nb = 0; nb < NB; ++nb)
            acc[p][mb][nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                a_cur[p >> 2][p & 3], uo[ks][nb][p >> 2][p & 3], acc[p][mb][nb], 0, 0, 0);
        if (grp < 3) {
#pragma unroll
          for (int q = 0; q < 4; ++q) a_cur[q] = a_nxt[q];
        }
        // keep the next group's 4 LDS reads ahead of this group's MFMAs
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 16 * NB, 0);
      }
    }
    load_u(min(c0 + kCK, g.Cin - kCK));
    if (PRE && tid < kCK) s_ss[sbuf ^ 1][tid] = ss_next;
    __syncthreads();
  }

  // 5. output transform (lane-local) -> per-wave LDS staging [cout][8 x 16 pixels]
  // acc element (mb, nb, reg): tile m = mb*16 + 4*kq + reg, cout = cout_w + 16nb + jj
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    float* so = &s_out[(wave * kWN + 16 * nb + jj) * kOS];
    const float bv = (bias && cout_w + 16 * nb + jj < g.CoutS) ? bias[cout_w + 16 * nb + jj] : 0.f;
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        const int m = mb * 16 + 4 * kq + rg;
        const int ty = m / kTC, tx = m - ty * kTC;
        float t0[4], t1[4];  // A^T M with A^T = [[1,1,1,0],[0,1,-1,-1]]
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          t0[j] = acc[j][mb][nb][rg] + acc[4 + j][mb][nb][rg] + acc[8 + j][mb][nb][rg];
          t1[j] = acc[4 + j][mb][nb][rg] - acc[8 + j][mb][nb][rg] - acc[12 + j][mb][nb][rg];
        }
        so[(2 * ty) * kOutCols + 2 * tx] = t0[0] + t0[1] + t0[2] + bv;
        so[(2 * ty) * kOutCols + 2 * tx + 1] = t0[1] - t0[2] - t0[3] + bv;
        so[(2 * ty + 1) * kOutCols + 2 * tx] = t1[0] + t1[1] + t1[2] + bv;
        so[(2 * ty + 1) * kOutCols + 2 * tx + 1] = t1[1] - t1[2] - t1[3] + bv;
      }
    }
  }
  __syncthreads();
  // 6. coalesced stores: per wave kWN couts x 8 rows x 16 cols = 32 kWN float4
  store_tile<kWN>(&s_out[wave * kWN * kOS], skip, y, stats, g, n, cout_w, oy0, ox0, lane);
}

// Per-workgroup phase timestamps (diagnostic build only, -DWINO_TIMING; tools/wino_timing.py):
// wall clock (100 MHz) at entry, once the prologue's loads have landed, after the first patch
// stores, at the start of the chunk loop, after it and after the epilogue (wave 0's view), the
// shader clock at entry and exit (s_memtime, for the clock rate), and the XCC / SE / CU.
#ifdef WINO_TIMING
constexpr unsigned kTsMax = 1u << 17;
__device__ long long g_wino_ts[kTsMax][8];
__device__ unsigned g_wino_cu[kTsMax];
#define WINO_TS(slot)                                                              \
  do {                                                                             \
    if (threadIdx.x == 0 && blockIdx.x < kTsMax) {                                 \
      g_wino_ts[blockIdx.x][slot] = wall_clock64();                                \
      if (slot == 0) g_wino_cu[blockIdx.x] = __smid();                             \
      if (slot == 0 || slot == 5)                                                  \
        g_wino_ts[blockIdx.x][6 + slot / 5] = (long long)__builtin_amdgcn_s_memtime(); \
    }                                                                              \
  } while (0)
#else
#define WINO_TS(slot) \
  do {                \
  } while (0)
#endif

// Software-pipelined form (one workgroup per CU, 4 waves x 32 couts = 128 couts, 32 tiles).
// The serial form above runs store-patch | barrier | transform | barrier | MFMAs per chunk,
// so a wave's MFMA pipe idles through the transform phase unless a second workgroup
// happens to be out of phase.  Here the work of three chunks overlaps inside each wave:
// while the MFMAs of chunk k read V(k) from one LDS buffer, the same wave transforms
// patch(k+1) (already in LDS) into the other V buffer, stores patch(k+2) (in registers)
// into the free patch buffer and issues the global loads of patch(k+3) and of U(k+1) into
// a second register set -- one barrier per chunk.  The VALU / LDS work (~70 instructions
// per chunk) fills MFMA issue gaps (128 MFMAs of 32 cycles per chunk per wave).
// WG = waves per workgroup: 4 (64 couts, two workgroups per CU) or 8 (128 couts, one
// workgroup per CU, NB = 1): the eight waves share one patch / V stream, so the GroupNorm+SiLU
// patch stores (4 channels per thread instead of 8: half the SiLU work per SIMD per MFMA of the
// two-workgroup form).
// TAIL (nch = Cin / 8 even and >= 4): the last three chunks are peeled so they skip the side
// work of chunks that do not exist (patch loads / stores, the V transform and the filter
// prefetch past the last chunk, and the last barrier) instead of redoing the last chunk's.
template <int NB, bool PRE, int WG = 4, bool TAIL = false>
__global__ __launch_bounds__(64 * WG, WG == 8 ? 1 : (NB == 1 ? 2 : 1)) void wino_f23_pipe_kernel(
    const float* __restrict__ x, const float* __restrict__ U, const float* __restrict__ bias,
    const float* __restrict__ skip, const float2* __restrict__ pre, float* __restrict__ y,
    float2* __restrict__ stats, WinoGeo g, int xcd_remap, const float* __restrict__ x2) {
  constexpr int kWN = 16 * NB;  // couts per wave
  constexpr int kPatch = kCK * kPR * kPCp;
  __shared__ __attribute__((aligned(16))) float s_patch_raw[2][kPatch];     // 2 x 7.5 KB
  constexpr int kVBuf = kCK * kM * kVS;                                      // 20.5 KB
  __shared__ __attribute__((aligned(16))) float s_v[2][kVBuf];              // V double buffer
  __shared__ float2 s_ss[PRE ? kPreMaxCin : 1];  // PRE: (s, t) of every input channel

  WINO_TS(0);
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  // grid < 2^31 blocks (host check): 32-bit block arithmetic
  const unsigned nblk = gridDim.x;
  unsigned b = blockIdx.x;
  if (xcd_remap) b = (b & 7u) * (nblk >> 3) + (b >> 3);
  unsigned cb, rx, ry;
  unsigned r = udivmod(b, (unsigned)g.cout_blocks, cb);
  r = udivmod(r, (unsigned)g.regions_x, rx);
  const int n = (int)udivmod(r, (unsigned)g.regions_y, ry);
  const int oy0 = (int)ry * kOutRows, ox0 = (int)rx * kOutCols;
  const int cout_w = (int)cb * (WG * kWN) + wave * kWN;
  static_assert(WG == 4 || (WG == 8 && NB == 1), "8-wave form: NB = 1");
  // 8 waves: waves 0-3 stage channels 0-3 of a chunk and transform V, waves 4-7 stage
  // channels 4-7 (wave-uniform, in SGPRs).  Every wave transforms (waves w and w + 4 write the
  // same V records, identical values): a wave-uniform branch around the transform, or waves
  // with split roles, made the compiler spill
  constexpr int kCT = kCK * 4 / WG;  // channels staged per thread
  const int phc = WG == 8 ? __builtin_amdgcn_readfirstlane(tid >> 8) : 0;

  // accumulators: the first chunk's k-step 0 MFMAs take an inline-constant zero C operand
  // (no 128 register clears in the prologue)
  f4 acc[16][2][NB];

  const int64_t plane = (int64_t)g.H * g.W;
  const int C2 = g.Cin - g.C1;
  const float* xn = x + (int64_t)n * g.C1 * plane;
  const float2* pre_n = PRE ? pre + (int64_t)n * g.Cin : nullptr;
  const int kq = lane >> 4, jj = lane & 15;
  const int nch = g.Cin / kCK;

  // Global loads go through buffer descriptors (base in SGPRs, 32-bit per-lane offsets,
  // the chunk offset in soffset): no 64-bit address registers next to the accumulators.
  // Two sources (the up path's [h, skip] without their concatenation): channels [0, C1)
  // from x, [C1, Cin) from x2; a chunk never straddles (C1 % 8 == 0).
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(xn), 0, (int)(g.C1 * plane * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t xrs2 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(C2 > 0 ? x2 + (int64_t)n * C2 * plane : xn), 0,
      (int)((C2 > 0 ? C2 : g.C1) * plane * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t urs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(U), 0, (int)((int64_t)g.Cin * g.Cout * 64), 0x00020000);

  // patch loads, position-major: thread t < 180 owns patch position (py, px) = (t / 18,
  // t % 18) for all 8 channels of a chunk (one in-plane offset, one LDS slot, one
  // in-image bit per thread; the channel stride goes into soffset / the LDS immediate).
  // Threads >= 180 duplicate thread 0 (same loads, same values to the same LDS words), so
  // every lane runs the same branch-free code.
  constexpr int kPos = kPR * kPC;  // 180
  int poff, pdst;
  bool pin;
  {
    const int t8 = tid & 255;
    const int t = t8 < kPos ? t8 : 0;
    const int py = t / kPC, px = t - py * kPC;
    const int iy = oy0 - 1 + py, ix = ox0 - 1 + px;
    pin = iy >= 0 && iy < g.H && ix >= 0 && ix < g.W;
    const int cy = min(max(iy, 0), g.H - 1), cx = min(max(ix, 0), g.W - 1);
    poff = (cy * g.W + cx) * 4;
    pdst = py * kPCp + px + phc * kCT * (kPR * kPCp);
  }
  float pv[kCT];
  auto load_patch = [&](int k) {
    const int cc = min(k, nch - 1) * kCK;
    const bool second = cc >= g.C1;
    const int soff = ((second ? cc - g.C1 : cc) + phc * kCT) * (int)plane * 4;
#pragma unroll
    for (int c = 0; c < kCT; ++c)
      pv[c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
          second ? xrs2 : xrs, poff, soff + c * (int)plane * 4, 0));
  };
  auto store_patch_from = [&](const float* src, float* sp, int k) {
    const int c0 = min(k, nch - 1) * kCK + phc * kCT;
#pragma unroll
    for (int c = 0; c < kCT; ++c) {
      float v = src[c];
      if (PRE) {
        const float2 st = s_ss[c0 + c];
        v = silu_f(v * st.x + st.y);
      }
      sp[pdst + c * (kPR * kPCp)] = pin ? v : 0.f;
    }
  };
  auto store_patch = [&](float* sp, int k) { store_patch_from(pv, sp, k); };
  // B operands of one k-step half: uo[ks][nb][q] = U[c0 + 4ks + kq][cout_w + 16nb + jj][4q..]
  f4 uo[2][NB][4];
  const int uoff = ((kq * g.Cout + cout_w + jj) * 16) * 4;
  auto load_u = [&](int ks, int k) {
    const int soff = ((min(k, nch - 1) * kCK + 4 * ks) * g.Cout) * 64;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        using u4 = __attribute__((ext_vector_type(4))) unsigned;
        const u4 w = __builtin_amdgcn_raw_buffer_load_b128(urs, uoff + nb * 1024 + q * 16, soff, 0);
        uo[ks][nb][q] = __builtin_bit_cast(f4, w);
      }
  };
  // V = B^T d B of one (cin, tile) per thread
  const int tc = (tid & 255) >> 5, tm = tid & 31;
  const int tty = tm / kTC, ttx = tm - tty * kTC;
  float d[4][4];
  auto read_d = [&](const float* sp) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; j += 2) {
        const float2 v2 =
            *reinterpret_cast<const float2*>(&sp[(tc * kPR + 2 * tty + i) * kPCp + 2 * ttx + j]);
        d[i][j] = v2.x;
        d[i][j + 1] = v2.y;
      }
  };
  auto write_v = [&](float* sv) {
    float t[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      t[0][j] = d[0][j] - d[2][j];
      t[1][j] = d[1][j] + d[2][j];
      t[2][j] = d[2][j] - d[1][j];
      t[3][j] = d[1][j] - d[3][j];
    }
    f4* dst = reinterpret_cast<f4*>(&sv[(tc * kM + tm) * kVS]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      dst[i] = f4{t[i][0] - t[i][2], t[i][1] + t[i][2], t[i][2] - t[i][1], t[i][1] - t[i][3]};
  };

  // prologue: V(0) in s_v[0], patch(1) in s_patch[1], patch(2) and U(0) in flight.  The
  // global loads of patches 0-2, U(0) and the GroupNorm table are all issued before the
  // first wait, so a workgroup pays one memory latency here, not four.
  float pv0[kCT], pv1[kCT];
  load_patch(0);
#pragma unroll
  for (int c = 0; c < kCT; ++c) pv0[c] = pv[c];
  load_patch(1);
#pragma unroll
  for (int c = 0; c < kCT; ++c) pv1[c] = pv[c];
  load_patch(2);
  load_u(0, 0);
  load_u(1, 0);
  if (PRE) {
    for (int c = tid; c < g.Cin; c += 64 * WG) s_ss[c] = pre_n[c];
    __syncthreads();
  }
  WINO_TS(1);
  store_patch_from(pv0, s_patch_raw[0], 0);
  store_patch_from(pv1, s_patch_raw[1], 1);
  __syncthreads();
  WINO_TS(2);
  read_d(s_patch_raw[0]);
  write_v(s_v[0]);
  __syncthreads();

  // A operands a[q] = V[pos 4q..4q+3] of (ks, mb) = this lane's tile row of one LDS record;
  // each a[q] / uo[ks][nb][q] register is refilled (next group's A, next chunk's U) right
  // after the last MFMA that reads it, so A needs 16 registers and U 64, and every load
  // has most of a group (>= 24 MFMAs) to land
  f4 a[4];
  auto a_src = [&](const float* sv, int grp) {  // grp = 2 ks + mb
    const int ks = grp >> 1, mb = grp & 1;
    return reinterpret_cast<const f4*>(&sv[((4 * ks + kq) * kM + mb * 16 + jj) * kVS]);
  };
  {
    const f4* src = a_src(s_v[0], 0);
#pragma unroll
    for (int q = 0; q < 4; ++q) a[q] = src[q];
  }
  // TM: 0 = full side work, 1 = no patch load (chunk nch - 3), 2 = no patch load / store
  // (nch - 2), 3 = the last chunk: no side work, no filter prefetch, no barrier
  auto step = [&](int k, auto sb_c, auto first_c, auto tm_c) __attribute__((always_inline)) {
    constexpr int SB = decltype(sb_c)::value;
    constexpr bool FIRST = decltype(first_c)::value;
    constexpr int TM = decltype(tm_c)::value;
    const float* sv = s_v[SB];
#pragma unroll
    for (int grp = 0; grp < 4; ++grp) {
      const int ks = grp >> 1, mb = grp & 1;
      // side work of the next chunks, spread over the four MFMA groups and fenced off from
      // the MFMAs (free / interleaved schedules measured slower, round 2)
      __builtin_amdgcn_sched_barrier(0);
      if (TM < 3 && grp == 0) read_d(s_patch_raw[SB ^ 1]);  // patch(k+1)
      if (TM < 3 && grp == 1) write_v(s_v[SB ^ 1]);         // V(k+1)
      if (TM < 2 && grp == 2) store_patch(s_patch_raw[SB], k + 2);  // patch(k+2)
      if (TM < 1 && grp == 3) load_patch(k + 3);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int pp = 0; pp < 4; ++pp)
#pragma unroll
          for (int nb = 0; nb < NB; ++nb)
            acc[4 * q + pp][mb][nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                a[q][pp], uo[ks][nb][q][pp],
                (FIRST && ks == 0) ? f4{0.f, 0.f, 0.f, 0.f} : acc[4 * q + pp][mb][nb], 0, 0, 0);
        // refill: A of the next group (the next chunk's group 0 comes after the barrier)
        if (grp < 3) a[q] = a_src(sv, grp + 1)[q];
        if (TM < 3 && mb == 1) {
          const int soff = ((min(k + 1, nch - 1) * kCK + 4 * ks) * g.Cout) * 64;
#pragma unroll
          for (int nb = 0; nb < NB; ++nb) {
            using u4 = __attribute__((ext_vector_type(4))) unsigned;
            const u4 w = __builtin_amdgcn_raw_buffer_load_b128(urs, uoff + nb * 1024 + q * 16,
                                                               soff, 0);
            uo[ks][nb][q] = __builtin_bit_cast(f4, w);
          }
        }
      }
    }
    if constexpr (TM < 3) {
      __syncthreads();
      const f4* src = a_src(s_v[SB ^ 1], 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) a[q] = src[q];
    }
  };
  using C0 = std::integral_constant<int, 0>;
  using C1 = std::integral_constant<int, 1>;
  using F = std::false_type;
  WINO_TS(3);
  using T0 = std::integral_constant<int, 0>;
  auto run = [&]() __attribute__((always_inline)) {
    step(0, C0{}, std::true_type{}, T0{});
    int k = 1;
    if constexpr (TAIL) {  // nch even, >= 4: chunks nch - 3, nch - 2, nch - 1 have SB 1, 0, 1
      for (; k + 1 <= nch - 4; k += 2) {
        step(k, C1{}, F{}, T0{});
        step(k + 1, C0{}, F{}, T0{});
      }
      step(k, C1{}, F{}, std::integral_constant<int, 1>{});
      step(k + 1, C0{}, F{}, std::integral_constant<int, 2>{});
      step(k + 2, C1{}, F{}, std::integral_constant<int, 3>{});
    } else {
      for (; k + 1 < nch; k += 2) {
        step(k, C1{}, F{}, T0{});
        step(k + 1, C0{}, F{}, T0{});
      }
      if (k < nch) step(k, C1{}, F{}, T0{});
    }
  };
  // (one call site per instantiation: a second, dead one stopped the inliner and put the
  // accumulators in scratch)
  run();
  WINO_TS(4);

  // output transform straight from registers to global memory (no LDS staging, no
  // barrier).  Per M-block a lane holds tiles m = 16 mb + 4 kq + rg, rg = 0..3: tile row
  // 2 mb + kq / 2, tile cols 4 (kq & 1) + rg -- 2 output rows x 8 pixels of channel
  // cout_w + 16 nb + jj, stored as two 16-B strips per row (lanes kq, kq ^ 1 cover a whole
  // 64-B row).  GroupNorm partial statistics: a running Chan merge over the lane's 32
  // values, then the 4 lanes jj + 16 kq (equal counts, symmetric butterfly: same bits).
  const float rdiv = 1.f / g.div;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    if (cout_w + 16 * nb >= g.CoutS) continue;  // padded couts (wave-uniform: CoutS % 16 == 0)
    const int co = cout_w + 16 * nb + jj;
    const float bv = bias ? bias[co] : 0.f;
    const int64_t obase = ((int64_t)n * g.CoutS + co) * plane;
    float lm = 0.f, lm2 = 0.f;
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
      const int oy = oy0 + 2 * (2 * mb + (kq >> 1));
      const int ox = ox0 + 8 * (kq & 1);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          f4 v;
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const int rg = 2 * e + u;
            float t[4];  // row h of A^T M, A^T = [[1,1,1,0],[0,1,-1,-1]]
#pragma unroll
            for (int j = 0; j < 4; ++j)
              t[j] = h == 0 ? acc[j][mb][nb][rg] + acc[4 + j][mb][nb][rg] + acc[8 + j][mb][nb][rg]
                            : acc[4 + j][mb][nb][rg] - acc[8 + j][mb][nb][rg] - acc[12 + j][mb][nb][rg];
            v[2 * u] = t[0] + t[1] + t[2] + bv;
            v[2 * u + 1] = t[1] - t[2] - t[3] + bv;
          }
          const int64_t o = obase + (int64_t)(oy + h) * g.W + ox + 4 * e;
          if (skip) {  // residual block tail, bit-identical to bpk_residual_rescale_f32
            const f4 sk = *reinterpret_cast<const f4*>(&skip[o]);
#pragma unroll
            for (int c = 0; c < 4; ++c) v[c] = div_rn(sk[c] + v[c], g.div, rdiv);
          }
          *reinterpret_cast<f4*>(&y[o]) = v;
          if (stats) {  // strip s = 4 mb + 2 h + e joins the s strips (4 s values) before it
            const float sm = ((v[0] + v[1]) + (v[2] + v[3])) * 0.25f;
            float sm2 = 0.f;
#pragma unroll
            for (int c = 0; c < 4; ++c) sm2 = fmaf(v[c] - sm, v[c] - sm, sm2);
            constexpr float kW[8] = {1.f, 1.f / 2, 1.f / 3, 1.f / 4, 1.f / 5, 1.f / 6, 1.f / 7, 1.f / 8};
            const int st = 4 * mb + 2 * h + e;
            const float d = sm - lm;
            lm = lm + d * kW[st];
            lm2 = (lm2 + sm2) + d * d * (4.f * st * kW[st]);
          }
        }
      }
    }
    if (stats) {
      merge_stats(lm, lm2, __shfl_xor(lm, 16, 64), __shfl_xor(lm2, 16, 64), 32.f);
      merge_stats(lm, lm2, __shfl_xor(lm, 32, 64), __shfl_xor(lm2, 32, 64), 64.f);
      if (kq == 0) {
        const int R = g.regions_x * g.regions_y;
        const int region = (oy0 / kOutRows) * g.regions_x + ox0 / kOutCols;
        stats[((int64_t)n * g.CoutS + co) * R + region] = make_float2(lm, lm2);
      }
    }
  }
  WINO_TS(5);
}

// 16-cin chunk form of the 8-wave pipelined kernel (one workgroup per CU, 8 waves x 16 couts =
// 128 couts, 32 tiles).  With 8-cin chunks the 8 waves transform the 256 (cin, tile) records of
// a chunk twice (waves w and w + 4 write identical V records: a wave-uniform branch around the
// transform made the compiler spill) and meet at a barrier every 64 MFMAs per wave.  Here a
// chunk is 16 input channels: the 512 threads own one (cin, tile) record each (no duplicate
// transform), every thread stages 8 channels of the patch (as the 4-wave form), and each wave
// issues 128 MFMAs per barrier; the side work of a chunk spreads over 8 MFMA groups.  The B
// operands (U) keep two k-step slots in registers: the slot a group has just finished is
// refilled with the k-step two ahead (next chunk's for the last two), one group pair before use.
// LDS: 2 x 15 KB patches + 2 x 40 KB V + the GroupNorm table (8 KB) = 118 KB.
// PAIR (images 8 pixels wide: CIFAR-10's 8 x 8 level): the 8 x 16-pixel region holds the same
// 8 rows of two images side by side -- tile columns 0-3 of image 2p, 4-7 of image 2p + 1 --
// and the patch is 10 x 20 (each image with its own one-pixel halo: columns 0-9 and 10-19), so
// the 3x3 convs of 8 x 8 feature maps run at the full 32-tile region instead of on the
// implicit GEMM.
template <bool PRE, bool PAIR>
__device__ __forceinline__ void k16_item(
    unsigned b, const float* __restrict__ x, const float* __restrict__ U,
    const float* __restrict__ bias, const float* __restrict__ skip,
    const float2* __restrict__ pre, float* __restrict__ y, float2* __restrict__ stats,
    const WinoGeo& g, const float* __restrict__ x2) {
  constexpr int CK = 16;
  constexpr int kPatch = CK * kPR * kPCp;
  __shared__ __attribute__((aligned(16))) float s_patch_raw[2][kPatch];
  constexpr int kVBuf = CK * kM * kVS;
  __shared__ __attribute__((aligned(16))) float s_v[2][kVBuf];
  __shared__ float2 s_ss[PRE ? kPreMaxCin : 1];

  WINO_TS(0);
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  unsigned cb, rx, ry;
  unsigned r = udivmod(b, (unsigned)g.cout_blocks, cb);
  r = udivmod(r, (unsigned)g.regions_x, rx);
  r = udivmod(r, (unsigned)g.regions_y, ry);
  unsigned nn;
  // split-K slice (0 unless ksplit > 1); PAIR: nn = the image pair, n its first image
  const int ks_idx = (int)udivmod(r, (unsigned)(PAIR ? g.N >> 1 : g.N), nn);
  const int n = PAIR ? (int)nn * 2 : (int)nn;
  const int oy0 = (int)ry * kOutRows, ox0 = (int)rx * kOutCols;
  const int cout_w = (int)cb * 128 + wave * 16;
  const int ph = __builtin_amdgcn_readfirstlane(tid >> 8);  // channels 8 ph .. 8 ph + 7

  f4 acc[16][2];
  const int64_t plane = (int64_t)g.H * g.W;
  const int up = g.up;  // nearest x2 input: the patch reads x[iy >> 1][ix >> 1] of an H/2 x W/2 plane
  const int64_t xplane = plane >> (2 * up);
  const int C2 = g.Cin - g.C1;
  const float* xn = x + (int64_t)n * g.C1 * xplane;
  const float2* pre_n = PRE ? pre + (int64_t)n * g.Cin : nullptr;
  const int kq = lane >> 4, jj = lane & 15;
  const int nch = g.Cin / CK / max(g.ksplit, 1);  // chunks of this workgroup
  const int kb = ks_idx * nch;                    // its first chunk

  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(xn), 0, (int)(g.C1 * xplane * 4) << (PAIR ? 1 : 0), 0x00020000);
  const __amdgpu_buffer_rsrc_t xrs2 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(C2 > 0 ? x2 + (int64_t)n * C2 * plane : xn), 0,
      (int)((C2 > 0 ? C2 : g.C1) * plane * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t urs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(U), 0, (int)((int64_t)g.Cin * g.Cout * 64), 0x00020000);

  // 180 patch positions (PAIR: 200); threads beyond them in a half duplicate position 0
  constexpr int kCols = PAIR ? 2 * (kOutCols / 2 + 2) : kPC;
  constexpr int kPos = kPR * kCols;
  static_assert(kCols <= kPCp && kPos <= 256, "patch layout");
  int poff, pdst;
  bool pin;
  {
    const int t8 = tid & 255;
    const int t = t8 < kPos ? t8 : 0;
    const int py = t / kCols, px = t - py * kCols;
    const int img = PAIR && px >= kCols / 2;        // PAIR: second image of the region
    const int iy = oy0 - 1 + py, ix = ox0 - 1 + px - img * (kCols / 2);
    pin = iy >= 0 && iy < g.H && ix >= 0 && ix < g.W;
    const int cy = min(max(iy, 0), g.H - 1), cx = min(max(ix, 0), g.W - 1);
    poff = ((cy >> up) * (g.W >> up) + (cx >> up)) * 4 + img * (int)(g.C1 * xplane * 4);
    pdst = py * kPCp + px + ph * 8 * (kPR * kPCp);
  }
  float pv[8];
  auto load_patch_part = [&](float* dst, int k, int c0, int cn) {
    const int cc = (kb + min(k, nch - 1)) * CK;
    const bool second = cc >= g.C1;
    const int soff = ((second ? cc - g.C1 : cc) + ph * 8) * (int)xplane * 4;
#pragma unroll
    for (int c = c0; c < c0 + cn; ++c)
      dst[c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
          second ? xrs2 : xrs, poff, soff + c * (int)xplane * 4, 0));
  };
  // PAIR: the second image's GroupNorm table follows the first's in LDS
  const int ssoff = PAIR ? ((tid & 255) < kPos && ((tid & 255) % kCols) >= kCols / 2) * g.Cin : 0;
  auto store_patch_part = [&](const float* src, float* sp, int k, int c0, int cn) {
    const int cb0 = (kb + min(k, nch - 1)) * CK + ph * 8;
#pragma unroll
    for (int c = c0; c < c0 + cn; ++c) {
      float v = src[c];
      if (PRE) {
        const float2 st = s_ss[ssoff + cb0 + c];
        v = silu_f(v * st.x + st.y);
      }
      sp[pdst + c * (kPR * kPCp)] = pin ? v : 0.f;
    }
  };
  // B operands: uo[ks & 1][q] = U[c0 + 4 ks + kq][cout_w + jj][4q..4q + 3]
  f4 uo[2][4];
  const int uoff = ((kq * g.Cout + cout_w + jj) * 16) * 4;
  auto u_soff = [&](int k, int ks) {
    return (((kb + min(k, nch - 1)) * CK + 4 * ks) * g.Cout) * 64;
  };
  auto load_u = [&](int slot, int k, int ks) {
    const int soff = u_soff(k, ks);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      using u4 = __attribute__((ext_vector_type(4))) unsigned;
      const u4 w = __builtin_amdgcn_raw_buffer_load_b128(urs, uoff + q * 16, soff, 0);
      uo[slot][q] = __builtin_bit_cast(f4, w);
    }
  };
  // V = B^T d B of one (cin, tile) per thread (512 records = 16 cin x 32 tiles)
  const int tc = tid >> 5, tm = tid & 31;
  const int tty = tm / kTC, ttx = tm - tty * kTC;
  const int tcol = 2 * ttx + (PAIR ? 2 * (ttx >= kTC / 2) : 0);  // PAIR: past the first halo
  float d[4][4];
  auto read_d = [&](const float* sp) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; j += 2) {
        const float2 v2 =
            *reinterpret_cast<const float2*>(&sp[(tc * kPR + 2 * tty + i) * kPCp + tcol + j]);
        d[i][j] = v2.x;
        d[i][j + 1] = v2.y;
      }
  };
  auto write_v = [&](float* sv) {
    float t[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      t[0][j] = d[0][j] - d[2][j];
      t[1][j] = d[1][j] + d[2][j];
      t[2][j] = d[2][j] - d[1][j];
      t[3][j] = d[1][j] - d[3][j];
    }
    f4* dst = reinterpret_cast<f4*>(&sv[(tc * kM + tm) * kVS]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      dst[i] = f4{t[i][0] - t[i][2], t[i][1] + t[i][2], t[i][2] - t[i][1], t[i][1] - t[i][3]};
  };

  // prologue: V(0) in s_v[0], patch(1) in s_patch[1], patch(2) and U(0) in flight
  {
    float pv0[8], pv1[8];
    load_patch_part(pv0, 0, 0, 8);
    load_patch_part(pv1, 1, 0, 8);
    load_patch_part(pv, 2, 0, 8);
    load_u(0, 0, 0);
    load_u(1, 0, 1);
    if (PRE) {
      for (int c = tid; c < (g.Cin << (PAIR ? 1 : 0)); c += 512) s_ss[c] = pre_n[c];
      __syncthreads();
    }
    WINO_TS(1);
    store_patch_part(pv0, s_patch_raw[0], 0, 0, 8);
    store_patch_part(pv1, s_patch_raw[1], 1, 0, 8);
  }
  __syncthreads();
  WINO_TS(2);
  read_d(s_patch_raw[0]);
  write_v(s_v[0]);
  __syncthreads();

  f4 a[4];
  auto a_src = [&](const float* sv, int grp) {  // grp = 2 ks + mb
    const int ks = grp >> 1, mb = grp & 1;
    return reinterpret_cast<const f4*>(&sv[((4 * ks + kq) * kM + mb * 16 + jj) * kVS]);
  };
  {
    const f4* src = a_src(s_v[0], 0);
#pragma unroll
    for (int q = 0; q < 4; ++q) a[q] = src[q];
  }
  auto step = [&](int k, auto sb_c, auto first_c) __attribute__((always_inline)) {
    constexpr int SB = decltype(sb_c)::value;
    constexpr bool FIRST = decltype(first_c)::value;
    const float* sv = s_v[SB];
#pragma unroll
    for (int grp = 0; grp < 8; ++grp) {
      const int ks = grp >> 1, mb = grp & 1;
      __builtin_amdgcn_sched_barrier(0);
      if (grp == 0) read_d(s_patch_raw[SB ^ 1]);                        // patch(k+1)
      if (grp == 1) write_v(s_v[SB ^ 1]);                               // V(k+1)
      if (grp == 2) store_patch_part(pv, s_patch_raw[SB], k + 2, 0, 4);  // patch(k+2)
      if (grp == 3) store_patch_part(pv, s_patch_raw[SB], k + 2, 4, 4);
      if (grp == 4) load_patch_part(pv, k + 3, 0, 4);
      if (grp == 5) load_patch_part(pv, k + 3, 4, 4);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int pp = 0; pp < 4; ++pp)
          acc[4 * q + pp][mb] = __builtin_amdgcn_mfma_f32_16x16x4f32(
              a[q][pp], uo[ks & 1][q][pp],
              (FIRST && ks == 0) ? f4{0.f, 0.f, 0.f, 0.f} : acc[4 * q + pp][mb], 0, 0, 0);
        if (grp < 7) a[q] = a_src(sv, grp + 1)[q];
        if (mb == 1) {  // k-step ks + 2 of this chunk, or ks - 2 of the next
          const int soff = ks < 2 ? u_soff(k, ks + 2) : u_soff(k + 1, ks - 2);
          using u4 = __attribute__((ext_vector_type(4))) unsigned;
          const u4 w = __builtin_amdgcn_raw_buffer_load_b128(urs, uoff + q * 16, soff, 0);
          uo[ks & 1][q] = __builtin_bit_cast(f4, w);
        }
      }
    }
    __syncthreads();
    const f4* src = a_src(s_v[SB ^ 1], 0);
#pragma unroll
    for (int q = 0; q < 4; ++q) a[q] = src[q];
  };
  using C0 = std::integral_constant<int, 0>;
  using C1 = std::integral_constant<int, 1>;
  WINO_TS(3);
  step(0, C0{}, std::true_type{});
  int k = 1;
  for (; k + 1 < nch; k += 2) {
    step(k, C1{}, std::false_type{});
    step(k + 1, C0{}, std::false_type{});
  }
  if (k < nch) step(k, C1{}, std::false_type{});
  WINO_TS(4);

  // output transform straight from registers (as wino_f23_pipe_kernel, NB = 1).  PAIR: a
  // lane's tile columns 4 (kq & 1) + rg all lie in image n + (kq & 1), at x 0..7
  const float rdiv = 1.f / g.div;
  if (cout_w < g.CoutS) {
    const int co = cout_w + jj;
    const float bv = bias ? bias[co] : 0.f;
    const int oimg = PAIR ? n + (kq & 1) : n;
    const int oxl = PAIR ? 0 : ox0 + 8 * (kq & 1);
    const int64_t obase = ((int64_t)(ks_idx * g.N + oimg) * g.CoutS + co) * plane;
    float lm = 0.f, lm2 = 0.f;
    // residual tail: all eight skip vectors of this lane requested before the first is used
    // (one exposed memory latency; loaded per store, the compiler waited for each in turn)
    f4 skv[2][2][2];
    if (skip) {
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int e = 0; e < 2; ++e)
            skv[mb][h][e] = *reinterpret_cast<const f4*>(
                &skip[obase + (int64_t)(oy0 + 2 * (2 * mb + (kq >> 1)) + h) * g.W + oxl + 4 * e]);
    }
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
      const int oy = oy0 + 2 * (2 * mb + (kq >> 1));
      const int ox = oxl;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          f4 v;
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const int rg = 2 * e + u;
            float t[4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
              t[j] = h == 0 ? acc[j][mb][rg] + acc[4 + j][mb][rg] + acc[8 + j][mb][rg]
                            : acc[4 + j][mb][rg] - acc[8 + j][mb][rg] - acc[12 + j][mb][rg];
            v[2 * u] = t[0] + t[1] + t[2] + bv;
            v[2 * u + 1] = t[1] - t[2] - t[3] + bv;
          }
          const int64_t o = obase + (int64_t)(oy + h) * g.W + ox + 4 * e;
          if (skip) {
            const f4 sk = skv[mb][h][e];
#pragma unroll
            for (int c = 0; c < 4; ++c) v[c] = div_rn(sk[c] + v[c], g.div, rdiv);
          }
          *reinterpret_cast<f4*>(&y[o]) = v;
          if (!PAIR && stats) {
            const float sm = ((v[0] + v[1]) + (v[2] + v[3])) * 0.25f;
            float sm2 = 0.f;
#pragma unroll
            for (int c = 0; c < 4; ++c) sm2 = fmaf(v[c] - sm, v[c] - sm, sm2);
            constexpr float kW[8] = {1.f, 1.f / 2, 1.f / 3, 1.f / 4, 1.f / 5, 1.f / 6, 1.f / 7, 1.f / 8};
            const int st = 4 * mb + 2 * h + e;
            const float dd = sm - lm;
            lm = lm + dd * kW[st];
            lm2 = (lm2 + sm2) + dd * dd * (4.f * st * kW[st]);
          }
        }
      }
    }
    if (!PAIR && stats) {
      merge_stats(lm, lm2, __shfl_xor(lm, 16, 64), __shfl_xor(lm2, 16, 64), 32.f);
      merge_stats(lm, lm2, __shfl_xor(lm, 32, 64), __shfl_xor(lm2, 32, 64), 64.f);
      if (kq == 0) {
        const int R = g.regions_x * g.regions_y;
        const int region = (oy0 / kOutRows) * g.regions_x + ox0 / kOutCols;
        stats[((int64_t)n * g.CoutS + co) * R + region] = make_float2(lm, lm2);
      }
    }
  }
  WINO_TS(5);
}

// Persistent form (round 6): gridDim.x workgroups (one per CU, k16_grid) walk the items, so the
// dispatcher's workgroup turnaround (~1 us between one workgroup's exit and the next one's start
// on a CU, the round-4 timeline) is paid once per CU instead of once per item.  With xcd_remap
// the workgroups sharing an XCD (w, w + 8, ...: blocks are dealt round-robin over the 8 XCDs)
// walk one contiguous eighth of the items together, in order -- the order the dispatcher gave
// the one-workgroup-per-item launch: the cout blocks of a region and the neighbouring regions
// (their patch halos) are processed close in time on one XCD's L2.  Items do not overlap inside
// a workgroup (the register-staged overlap spilled); the barrier between
// items keeps the next prologue's LDS stores behind every wave's last reads of the previous one.
template <bool PRE, bool PAIR = false>
__global__ __launch_bounds__(512, 1) void wino_f23_k16_kernel(
    const float* __restrict__ x, const float* __restrict__ U, const float* __restrict__ bias,
    const float* __restrict__ skip, const float2* __restrict__ pre, float* __restrict__ y,
    float2* __restrict__ stats, WinoGeo g, int xcd_remap, const float* __restrict__ x2,
    unsigned items) {
  const unsigned G = gridDim.x, w = blockIdx.x;
  unsigned first = w, stride = G, end = items;
  if (xcd_remap) {  // G % 8 == 0: XCD label w % 8 owns items [start, start + count)
    const unsigned xc = w & 7u, q = items >> 3, r = items & 7u;
    const unsigned start = xc * q + min(xc, r);
    first = start + (w >> 3);
    stride = G >> 3;
    end = start + q + (xc < r ? 1u : 0u);
  }
  for (unsigned b = first; b < end; b += stride) {
    if (b != first) __syncthreads();
    k16_item<PRE, PAIR>(b, x, U, bias, skip, pre, y, stats, g, x2);
  }
}

// Split-K epilogue: y = sum_s part[s] + bias, or (skip + that) / div, and the GroupNorm partial
// statistics of the stored values, as the 16-cin kernel's own epilogue (the partial slabs are
// summed in a fixed order: deterministic).  One workgroup = 8 channels x one 8 x 16 region of
// one image; a half-wave holds one channel's 128 values (the store_tile mapping).
__global__ __launch_bounds__(256) void wino_splitk_reduce_kernel(
    const float* __restrict__ part, int S, const float* __restrict__ bias,
    const float* __restrict__ skip, float* __restrict__ y, float2* __restrict__ stats,
    WinoGeo g) {
  const int lane = threadIdx.x & 63;
  const int q = threadIdx.x;
  unsigned b = blockIdx.x, reg, cg;
  const unsigned R = (unsigned)(g.regions_x * g.regions_y);
  unsigned r = udivmod(b, R, reg);
  int n = (int)udivmod(r, (unsigned)(g.CoutS / 8), cg);
  const int co = (int)cg * 8 + (q >> 5);
  const int rem = q & 31;
  const int row = rem >> 2;
  int c4 = rem & 3;
  if (g.pair) {  // region = image pair n: columns 0-7 of image 2n, 8-15 of image 2n + 1
    n = 2 * n + (c4 >> 1);
    c4 &= 1;
  }
  const int oy0 = (int)(reg / g.regions_x) * kOutRows, ox0 = (int)(reg % g.regions_x) * kOutCols;
  const int64_t plane = (int64_t)g.H * g.W;
  const int64_t slab = (int64_t)g.N * g.CoutS * plane;
  const int64_t o = ((int64_t)n * g.CoutS + co) * plane + (int64_t)(oy0 + row) * g.W + ox0 + 4 * c4;
  f4 v = *reinterpret_cast<const f4*>(&part[o]);
  for (int s = 1; s < S; ++s) v += *reinterpret_cast<const f4*>(&part[s * slab + o]);
  const float bv = bias ? bias[co] : 0.f;
  v += f4{bv, bv, bv, bv};
  if (skip) {
    const f4 sk = *reinterpret_cast<const f4*>(&skip[o]);
    const float rdiv = 1.f / g.div;
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = div_rn(sk[c] + v[c], g.div, rdiv);
  }
  *reinterpret_cast<f4*>(&y[o]) = v;
  if (!stats || g.pair) return;
  float mm = ((v[0] + v[1]) + (v[2] + v[3])) * 0.25f;
  float qq = 0.f;
#pragma unroll
  for (int e = 0; e < 4; ++e) qq = fmaf(v[e] - mm, v[e] - mm, qq);
  merge_stats(mm, qq, dpp_f<0xB1>(mm), dpp_f<0xB1>(qq), 4.f);
  merge_stats(mm, qq, dpp_f<0x4E>(mm), dpp_f<0x4E>(qq), 8.f);
  merge_stats(mm, qq, dpp_f<0x141>(mm), dpp_f<0x141>(qq), 16.f);
  merge_stats(mm, qq, dpp_f<0x140>(mm), dpp_f<0x140>(qq), 32.f);
  merge_stats(mm, qq, __shfl_xor(mm, 16, 64), __shfl_xor(qq, 16, 64), 64.f);
  if ((lane & 31) == 0) stats[((int64_t)n * g.CoutS + co) * R + reg] = make_float2(mm, qq);
}

}  // namespace

static int cout_padded(int Cout) { return (Cout + 63) / 64 * 64; }

// grid of the persistent 16-cin kernel: one workgroup per CU (its launch bound), at most one
// per item; WINO_PERSIST=0 builds launch one workgroup per item (the round-5 form, for A/B)
#ifndef WINO_PERSIST
#define WINO_PERSIST 1
#endif
static unsigned k16_grid(int64_t items) {
  static const int cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  return (unsigned)(WINO_PERSIST ? std::min<int64_t>(items, cus) : items);
}

extern "C" int64_t bpk_conv3x3_wino_filter_bytes(int Cin, int Cout) {
  return (int64_t)16 * Cin * cout_padded(Cout) * (int64_t)sizeof(float);
}

static int wino_filter(const float* weight, float* U, int Cin, int Cout, int ft,
                       void* stream) {
  BPK_REQUIRE(Cin > 0 && Cout > 0, "conv3x3_wino_filter: bad channels %d -> %d", Cin, Cout);
  const int64_t total = (int64_t)Cin * cout_padded(Cout);
  hipLaunchKernelGGL(wino_filter_kernel, dim3((unsigned)std::min<int64_t>(bpk::ceil_div(total, 256), 4096)),
                     dim3(256), 0, bpk::as_stream(stream), weight, U, Cin, Cout,
                     cout_padded(Cout), ft);
  BPK_LAUNCH_CHECK("conv3x3_wino_filter");
  return BPK_OK;
}

extern "C" int bpk_conv3x3_wino_filter_f32(const float* weight, float* U, int Cin, int Cout,
                                           void* stream) {
  return wino_filter(weight, U, Cin, Cout, 0, stream);
}

extern "C" int bpk_conv3x3_wino_filter_ft_f32(const float* weight, float* U, int Cin, int Cout,
                                              void* stream) {
  return wino_filter(weight, U, Cin, Cout, 1, stream);
}

extern "C" int bpk_conv3x3_wino_filter_batch_f32(const int64_t* jobs, int n, int max_elems,
                                                 void* stream) {
  BPK_REQUIRE(n >= 0 && n < 65536 && max_elems >= 0, "conv3x3_wino_filter_batch: bad job count");
  if (n == 0 || max_elems == 0) return BPK_OK;
  BPK_REQUIRE(jobs != nullptr, "conv3x3_wino_filter_batch: jobs is NULL");
  const dim3 grid((unsigned)std::min<int64_t>(bpk::ceil_div(max_elems, 256), 64), (unsigned)n);
  hipLaunchKernelGGL(wino_filter_batch_kernel, grid, dim3(256), 0, bpk::as_stream(stream), jobs);
  BPK_LAUNCH_CHECK("conv3x3_wino_filter_batch");
  return BPK_OK;
}

// The PAIR form of the 16-cin kernel (8-pixel-wide images, two per region): one source, no
// GroupNorm statistics, N even; a GroupNorm prologue needs both images' tables in LDS.
static bool wino_pair_ok(int N, int Cin, int Cout, int H, int W) {
  return N > 0 && N % 2 == 0 && W == 8 && H > 0 && H % kOutRows == 0 && Cin % 16 == 0 &&
         Cout % 16 == 0 && cout_padded(Cout) % 128 == 0;
}

extern "C" int bpk_conv3x3_wino_pair_supported(int N, int Cin, int Cout, int H, int W) {
  return wino_pair_ok(N, Cin, Cout, H, W);
}

static int wino_pair_launch(const float* x, const float* pre, const float* U, const float* bias,
                            const float* skip, float div, float* y, int N, int Cin, int Cout,
                            int H, int W, int S, void* stream) {
  BPK_REQUIRE(wino_pair_ok(N, Cin, Cout, H, W),
              "conv3x3_wino pair form: unsupported shape N=%d Cin=%d Cout=%d H=%d W=%d (need "
              "W == 8, N even, H %% 8, Cin %% 16, Cout %% 128 == 0)", N, Cin, Cout, H, W);
  BPK_REQUIRE(!pre || 2 * Cin <= kPreMaxCin, "conv3x3_wino pair form: GroupNorm prologue over "
              "%d > %d channels", Cin, kPreMaxCin / 2);
  const int CoutP = cout_padded(Cout);
  WinoGeo gk{N, Cin, CoutP, H, W, 1, H / kOutRows, CoutP / 128, div, Cin, Cout, 0, S, 1};
  const int64_t items = (int64_t)(N / 2) * gk.regions_y * gk.cout_blocks * S;
  BPK_REQUIRE(items < (1LL << 31), "conv3x3_wino pair form: grid too large");
  const float2* kpre = reinterpret_cast<const float2*>(pre);
  hipStream_t st = bpk::as_stream(stream);
  const unsigned kg = k16_grid(items);
  const int remap = (kg % 8 == 0) ? 1 : 0;
  const float* kb = S > 1 ? nullptr : bias;
  const float* ks = S > 1 ? nullptr : skip;
  if (pre)
    hipLaunchKernelGGL((wino_f23_k16_kernel<true, true>), dim3(kg), dim3(512), 0, st,
                       x, U, kb, ks, kpre, y, nullptr, gk, remap, nullptr, (unsigned)items);
  else
    hipLaunchKernelGGL((wino_f23_k16_kernel<false, true>), dim3(kg), dim3(512), 0, st,
                       x, U, kb, ks, kpre, y, nullptr, gk, remap, nullptr, (unsigned)items);
  BPK_LAUNCH_CHECK("conv3x3_wino_pair");
  return BPK_OK;
}

extern "C" int bpk_conv3x3_wino_supported(int N, int Cin, int Cout, int H, int W) {
  // Cout % 64 != 0 (multiples of 16): padded to 64 couts, software-pipelined kernel
  return N > 0 && Cin > 0 && Cin % kCK == 0 && Cout % 16 == 0 && H % kOutRows == 0 &&
         W % kOutCols == 0;
}

extern "C" int bpk_conv3x3_wino_ex_f32(const float* x, const float* x2, int C1, const float* pre,
                                       const float* U, const float* bias, const float* skip,
                                       float div, float* y, float* stats, int N, int Cin,
                                       int Cout, int H, int W, void* stream) {
  float2* stats2 = reinterpret_cast<float2*>(stats);
  if (!x2) C1 = Cin;
  if (W == 8 && !bpk_conv3x3_wino_supported(N, Cin, Cout, H, W)) {
    BPK_REQUIRE(!x2 && !stats, "conv3x3_wino pair form (W == 8): one source, no statistics");
    return wino_pair_launch(x, pre, U, bias, skip, div, y, N, Cin, Cout, H, W, 1, stream);
  }
  BPK_REQUIRE(C1 > 0 && C1 <= Cin && C1 % kCK == 0,
              "conv3x3_wino: bad channel split C1=%d of Cin=%d", C1, Cin);
  BPK_REQUIRE(bpk_conv3x3_wino_supported(N, Cin, Cout, H, W),
              "conv3x3_wino: unsupported shape N=%d Cin=%d Cout=%d H=%d W=%d (need Cin %% 8, "
              "Cout %% 16, H %% 8, W %% 16 == 0)", N, Cin, Cout, H, W);
  const int CoutP = cout_padded(Cout);
  // Kernel choice (each form measured against the others on the NCSN++ / DDPM++ shapes;
  // the rejected variants -- two persistent forms (register- and LDS-DMA-staged), 128-cout
  // NB = 2 blocks, the 4-wave residual tail -- are gone, numbers in DESIGN.md section 4):
  //   * wino_f23_k16_kernel: CoutP % 128 == 0 and 16-cin chunks (every NCSN++ conv);
  //   * wino_f23_pipe_kernel: the other shapes (8-wave / 128-cout form for the GroupNorm
  //     prologue convs without a residual tail, 4 waves / 64 couts otherwise);
  //   * wino_f23_kernel: a GroupNorm prologue over more than kPreMaxCin input channels.
  const bool pipe_ok = !pre || Cin <= kPreMaxCin;
  BPK_REQUIRE(!x2 || pipe_ok,
              "conv3x3_wino: a second input source needs the pipelined kernel");
  BPK_REQUIRE(Cout == CoutP || pipe_ok,
              "conv3x3_wino: Cout %% 64 != 0 needs the pipelined kernel (Cin <= %d with pre)",
              kPreMaxCin);
  if (pipe_ok) {
    const int wg = (pre && !skip && CoutP % 128 == 0) ? 8 : 4;
#ifdef WINO_NO_K16  // variant builds only (tools/build_variant.sh): the 8-cin forms everywhere
    const bool k16 = false;
#else
    const bool k16 = CoutP % 128 == 0 && Cin % 16 == 0 && C1 % 16 == 0;
#endif
    if (k16) {
      WinoGeo gk{N, Cin, CoutP, H, W, W / kOutCols, H / kOutRows, CoutP / 128, div, C1, Cout};
      const int64_t items = (int64_t)N * gk.regions_x * gk.regions_y * gk.cout_blocks;
      BPK_REQUIRE(items < (1LL << 31), "conv3x3_wino: grid too large");
      const float2* kpre = reinterpret_cast<const float2*>(pre);
      hipStream_t kst = bpk::as_stream(stream);
      const unsigned kg = k16_grid(items);
      const int kremap = (kg % 8 == 0) ? 1 : 0;
      if (pre)
        hipLaunchKernelGGL((wino_f23_k16_kernel<true>), dim3(kg), dim3(512), 0, kst,
                           x, U, bias, skip, kpre, y, stats2, gk, kremap, x2, (unsigned)items);
      else
        hipLaunchKernelGGL((wino_f23_k16_kernel<false>), dim3(kg), dim3(512), 0, kst,
                           x, U, bias, skip, kpre, y, stats2, gk, kremap, x2, (unsigned)items);
      BPK_LAUNCH_CHECK("conv3x3_wino_k16");
      return BPK_OK;
    }
    WinoGeo g{N, Cin, CoutP, H, W, W / kOutCols, H / kOutRows, CoutP / (64 * wg / 4), div,
              C1, Cout};
    const int64_t blocks = (int64_t)N * g.regions_x * g.regions_y * g.cout_blocks;
    BPK_REQUIRE(blocks < (1LL << 31), "conv3x3_wino: grid too large");
    const int remap = (blocks % 8 == 0) ? 1 : 0;
    const float2* pre2 = reinterpret_cast<const float2*>(pre);
    hipStream_t st = bpk::as_stream(stream);
#define WINO_PIPE(NB_, PRE_, TAIL_)                                                           \
  hipLaunchKernelGGL((wino_f23_pipe_kernel<NB_, PRE_, 4, TAIL_>), dim3((unsigned)blocks), dim3(256), 0, st, \
                     x, U, bias, skip, pre2, y, stats2, g, remap, x2)
    const int nch = Cin / kCK;
    // peeled tail chunks (GroupNorm-prologue form only: the plain form spills with them)
    const bool tail = pre && nch % 2 == 0 && nch >= 4;
#define WINO_PIPE8(PRE_, TAIL_)                                                                 \
  hipLaunchKernelGGL((wino_f23_pipe_kernel<1, PRE_, 8, TAIL_>), dim3((unsigned)blocks), dim3(512), \
                     0, st, x, U, bias, skip, pre2, y, stats2, g, remap, x2)
    if (wg == 8) {
      if (pre) {
        if (tail) WINO_PIPE8(true, true); else WINO_PIPE8(true, false);
      } else {
        WINO_PIPE8(false, false);
      }
    } else if (tail) {
      WINO_PIPE(1, true, true);
    } else {
      if (pre) WINO_PIPE(1, true, false); else WINO_PIPE(1, false, false);
    }
#undef WINO_PIPE8
#undef WINO_PIPE
    BPK_LAUNCH_CHECK("conv3x3_wino_pipe");
    return BPK_OK;
  }
  WinoGeo g{N, Cin, Cout, H, W, W / kOutCols, H / kOutRows, Cout / 64, div, Cin, Cout};
  const int64_t blocks = (int64_t)N * g.regions_x * g.regions_y * g.cout_blocks;
  BPK_REQUIRE(blocks < (1LL << 31), "conv3x3_wino: grid too large");
  const int remap = (blocks % 8 == 0) ? 1 : 0;
  const float2* pre2 = reinterpret_cast<const float2*>(pre);
  hipStream_t st = bpk::as_stream(stream);
#define WINO_LAUNCH(NB_, PRE_)                                                                 \
  hipLaunchKernelGGL((wino_f23_kernel<NB_, PRE_>), dim3((unsigned)blocks), dim3(256), 0, st, x, \
                     U, bias, skip, pre2, y, stats2, g, remap)
  if (pre) WINO_LAUNCH(1, true); else WINO_LAUNCH(1, false);
#undef WINO_LAUNCH
  BPK_LAUNCH_CHECK("conv3x3_wino");
  return BPK_OK;
}

// Split-K for 16-cin launches that leave most CUs idle (the 32^2 / 16^2 levels at the small
// per-GPU batches of a batch-sharded run: B = 8 -> 128 / 32 workgroups on 256 CUs): the input
// channels are split into S slices (S a power of two, at least 2 chunks per slice), so that
// items x S is at most one workgroup per CU, then a reduce kernel applies the epilogue.
static int wino_splits(int N, int Cin, int C1, int Cout, int H, int W) {
  static const int cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  const int CoutP = cout_padded(Cout);
  const bool pair = W == 8 && C1 == Cin && wino_pair_ok(N, Cin, Cout, H, W);
  if (!pair && (!bpk_conv3x3_wino_supported(N, Cin, Cout, H, W) || CoutP % 128 || Cin % 16 ||
                C1 % 16))
    return 1;
  const int64_t items = pair ? (int64_t)(N / 2) * (H / kOutRows) * (CoutP / 128)
                             : (int64_t)N * (H / kOutRows) * (W / kOutCols) * (CoutP / 128);
  const int nch = Cin / 16;
  int S = 1;
  while (items * S * 2 <= cus && nch % (2 * S) == 0 && nch / (2 * S) >= 2) S *= 2;
  return S;
}

extern "C" int64_t bpk_conv3x3_wino_splitk_bytes(int N, int Cin, int C1, int Cout, int H, int W) {
  const int S = wino_splits(N, Cin, C1, Cout, H, W);
  return S > 1 ? (int64_t)S * N * Cout * H * W * (int64_t)sizeof(float) : 0;
}

extern "C" int bpk_conv3x3_wino_splitk_f32(const float* x, const float* x2, int C1,
                                           const float* pre, const float* U, const float* bias,
                                           const float* skip, float div, float* y, float* stats,
                                           float* workspace, int N, int Cin, int Cout, int H,
                                           int W, void* stream) {
  const int S = wino_splits(N, Cin, x2 ? C1 : Cin, Cout, H, W);
  if (S <= 1)
    return bpk_conv3x3_wino_ex_f32(x, x2, C1, pre, U, bias, skip, div, y, stats, N, Cin, Cout, H,
                                   W, stream);
  if (!x2) C1 = Cin;
  BPK_REQUIRE(workspace != nullptr, "conv3x3_wino_splitk: workspace is NULL");
  BPK_REQUIRE(Cout % 16 == 0, "conv3x3_wino_splitk: Cout %% 16 != 0");
  const int CoutP = cout_padded(Cout);
  if (W == 8 && !bpk_conv3x3_wino_supported(N, Cin, Cout, H, W)) {
    BPK_REQUIRE(!x2 && !stats, "conv3x3_wino pair form (W == 8): one source, no statistics");
    const int rc = wino_pair_launch(x, pre, U, bias, skip, div, workspace, N, Cin, Cout, H, W,
                                    S, stream);
    if (rc != BPK_OK) return rc;
    WinoGeo gr{N, Cin, CoutP, H, W, 1, H / kOutRows, CoutP / 128, div, Cin, Cout, 0, S, 1};
    const int64_t rblocks = (int64_t)(N / 2) * (Cout / 8) * gr.regions_y;
    hipLaunchKernelGGL(wino_splitk_reduce_kernel, dim3((unsigned)rblocks), dim3(256), 0,
                       bpk::as_stream(stream), workspace, S, bias, skip, y, nullptr, gr);
    BPK_LAUNCH_CHECK("conv3x3_wino_pair_splitk_reduce");
    return BPK_OK;
  }
  WinoGeo gk{N, Cin, CoutP, H, W, W / kOutCols, H / kOutRows, CoutP / 128, div, C1, Cout, 0, S};
  const int64_t items = (int64_t)N * gk.regions_x * gk.regions_y * gk.cout_blocks * S;
  BPK_REQUIRE(items < (1LL << 31), "conv3x3_wino_splitk: grid too large");
  const float2* kpre = reinterpret_cast<const float2*>(pre);
  hipStream_t st = bpk::as_stream(stream);
  const unsigned kg = k16_grid(items);
  const int remap = (kg % 8 == 0) ? 1 : 0;
  if (pre)
    hipLaunchKernelGGL((wino_f23_k16_kernel<true>), dim3(kg), dim3(512), 0, st, x, U,
                       nullptr, nullptr, kpre, workspace, nullptr, gk, remap, x2, (unsigned)items);
  else
    hipLaunchKernelGGL((wino_f23_k16_kernel<false>), dim3(kg), dim3(512), 0, st, x,
                       U, nullptr, nullptr, kpre, workspace, nullptr, gk, remap, x2, (unsigned)items);
  BPK_LAUNCH_CHECK("conv3x3_wino_splitk");
  const int64_t rblocks = (int64_t)N * (Cout / 8) * gk.regions_x * gk.regions_y;
  BPK_REQUIRE(Cout % 8 == 0 && rblocks < (1LL << 31), "conv3x3_wino_splitk: reduce grid");
  hipLaunchKernelGGL(wino_splitk_reduce_kernel, dim3((unsigned)rblocks), dim3(256), 0, st,
                     workspace, S, bias, skip, y, reinterpret_cast<float2*>(stats), gk);
  BPK_LAUNCH_CHECK("conv3x3_wino_splitk_reduce");
  return BPK_OK;
}

extern "C" int bpk_conv3x3_wino_up2_supported(int N, int Cin, int Cout, int H, int W) {
  return bpk_conv3x3_wino_supported(N, Cin, Cout, H, W) && Cin % 16 == 0 &&
         cout_padded(Cout) % 128 == 0;
}

// y = conv3x3(nearest_x2(x)) + bias for x [N, Cin, H/2, W/2], y [N, Cout, H, W]: the 16-cin
// kernel reads the half-resolution input inside its patch load, so the upsampled tensor is
// never written (reference layers.py:576-590, Upsample(with_conv=True)).
extern "C" int bpk_conv3x3_wino_up2_f32(const float* x, const float* U, const float* bias,
                                        float* y, int N, int Cin, int Cout, int H, int W,
                                        void* stream) {
  BPK_REQUIRE(bpk_conv3x3_wino_up2_supported(N, Cin, Cout, H, W),
              "conv3x3_wino_up2: unsupported shape N=%d Cin=%d Cout=%d H=%d W=%d (need Cin %% 16, "
              "Cout %% 128, H %% 8, W %% 16 == 0)", N, Cin, Cout, H, W);
  const int CoutP = cout_padded(Cout);
  WinoGeo gk{N, Cin, CoutP, H, W, W / kOutCols, H / kOutRows, CoutP / 128, 1.0f, Cin, Cout, 1};
  const int64_t items = (int64_t)N * gk.regions_x * gk.regions_y * gk.cout_blocks;
  BPK_REQUIRE(items < (1LL << 31), "conv3x3_wino_up2: grid too large");
  const unsigned kg = k16_grid(items);
  hipLaunchKernelGGL((wino_f23_k16_kernel<false>), dim3(kg), dim3(512), 0,
                     bpk::as_stream(stream), x, U, bias, nullptr, nullptr, y, nullptr, gk,
                     (kg % 8 == 0) ? 1 : 0, nullptr, (unsigned)items);
  BPK_LAUNCH_CHECK("conv3x3_wino_up2");
  return BPK_OK;
}

extern "C" int bpk_conv3x3_wino_pre_f32(const float* x, const float* pre, const float* U,
                                        const float* bias, const float* skip, float div, float* y,
                                        int N, int Cin, int Cout, int H, int W, void* stream) {
  return bpk_conv3x3_wino_ex_f32(x, nullptr, Cin, pre, U, bias, skip, div, y, nullptr, N, Cin,
                                 Cout, H, W, stream);
}

extern "C" int bpk_conv3x3_wino_residual_f32(const float* x, const float* U, const float* bias,
                                             const float* skip, float div, float* y, int N,
                                             int Cin, int Cout, int H, int W, void* stream) {
  return bpk_conv3x3_wino_pre_f32(x, nullptr, U, bias, skip, div, y, N, Cin, Cout, H, W, stream);
}

extern "C" int bpk_conv3x3_wino_f32(const float* x, const float* U, const float* bias, float* y,
                                    int N, int Cin, int Cout, int H, int W, void* stream) {
  return bpk_conv3x3_wino_pre_f32(x, nullptr, U, bias, nullptr, 1.0f, y, N, Cin, Cout, H, W,
                                  stream);
}

#ifdef WINO_TIMING
extern "C" int bpk_wino_timing_read(long long* ts, unsigned* cu, int n) {
  if (n > (int)kTsMax) n = (int)kTsMax;
  if (hipMemcpyFromSymbol(ts, HIP_SYMBOL(g_wino_ts), sizeof(long long) * 8 * n) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(cu, HIP_SYMBOL(g_wino_cu), sizeof(unsigned) * n) != hipSuccess) return -1;
  return n;
}
#endif
