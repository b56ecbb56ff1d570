// Weight gradient of the 3x3 / stride 1 / pad 1 conv as Winograd F(2x2, 3x3) on the f32
// MFMA (gfx950) -- the backward-filter half of the score networks' conv3x3 (the reference
// gets it from cuDNN through torch.nn.Conv2d's autograd; here it replaces MIOpen's
// backward-weights convolution, which ran at ~100 TFLOP/s on the NCSN++ shapes).
//
// The forward conv is Y = A^T [ U .* V ] A per 2x2 output tile with U = G w G^T and
// V = B^T d B, linear in U, so
//     dL/dU_pos[cin][cout] = sum_{n, tiles} V_pos[tile][cin] * Gbar_pos[tile][cout],
//     Gbar = A dY A^T (the 2x2 output-gradient tile lifted to 4x4),
//     dL/dw = G^T (dL/dU) G.
// For each of the 16 positions that is a GEMM with M = Cin, N = Cout and a long
// K = N * tiles, computed split-K:
//   * one workgroup = 32 cin x 64 cout (4 waves x 16 couts, 2 M-blocks each) over a
//     contiguous range of K-chunks; a K-chunk = 8 tiles = a 2 x 16 pixel strip of one
//     image: the 32 x 4 x 18 input patch and the 64 x 2 x 16 gradient strip are loaded
//     (prefetched in registers during the previous chunk's MFMAs), transformed into V / Gbar
//     records (16 positions contiguous, LDS) and contracted with 16 positions x 2 M-blocks
//     x 2 k-steps = 64 v_mfma_f32_16x16x4_f32 per wave;
//   * partial dU slabs [split][Cin][Cout][16] (deterministic: no atomics) are summed and
//     back-transformed (G^T dU G) by a second small kernel straight into dw [Cout][Cin][3][3].
#include "bpk_common.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace {

using f4 = __attribute__((ext_vector_type(4))) float;

constexpr int kCB = 32;              // cin per workgroup
constexpr int kOB = 64;              // cout per workgroup per N-block of the waves (NB)
constexpr int kT = 8;                // tiles per K-chunk (1 tile row x 8 tile cols)
constexpr int kXR = 4;               // input patch rows
constexpr int kRec = 24;             // LDS stride of one 16-position record

struct WgradGeo {
  int N, Cin, Cout, H, W;
  int strips_x, strips_y;  // W / 16, H / 2 (PAIR: 1, H / 2; a strip = 2 rows of two images)
  int cin_blocks, cout_blocks, splits;
  int64_t chunks;          // N * strips_y * strips_x
  int N1;                  // TWO: images n >= N1 are image n - N1 of (x2, gy2)
};

// Software-pipelined weight gradient (workgroup = 32 cin x 64 cout over a K-range of 8-tile
// chunks; round 1's unpipelined form of the same decomposition was 1.3x slower and is gone),
// organized like the forward pipe kernel:
//   * the B operands (Gbar = A dY A^T, one (tile, cout) record per lane and k-step) are
//     built in registers by the lane that consumes them, from a 2 x 2 gradient tile it
//     loads itself (two 8-byte loads), one chunk ahead -- no LDS traffic for the gradient;
//   * chunk c's input patch is loaded at step c-3 (2 x 16 B + one halo word per thread and
//     (cin, row)), stored to LDS at step c-2, transformed into V records at step c-1 while
//     the MFMAs of the previous chunk run (double-buffered patch and V), one barrier per chunk;
//   * V records of tile t sit at t * 772 + cin * 24 floats: conflict-free 16-B writes and
//     16-B operand reads (a 20-float record made the operand reads 2-way: 45% of LDS cycles
//     were bank-conflict cycles, SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE, round 5).
constexpr int kXRS = 24;                     // LDS patch row: halo at 3, interior at 4..19, halo 20
constexpr int kXCS = kXR * kXRS + 16;        // per-cin stride (2-way transform reads)
constexpr int kVT = kCB * kRec + 4;          // per-tile stride of the V records (772)

// NB = 16-cout blocks per wave: NB = 1 -> 64 couts per workgroup, two workgroups per CU (the
// form that runs).  NB = 2 (128 couts per workgroup, 256 accumulators per lane, one workgroup
// per CU: the V transform, the patch staging and every A operand read serve twice the couts)
// was measured slower on every NCSN++ shape, round 4 (1.85 vs 1.50 ms at 128->128 @128^2,
// 7.06 vs 5.20 at 256->256 @128^2; DSM train 2.59 vs 2.87 steps/s, same box) -- the halved
// residency exposes the per-chunk barrier and load latency that two co-resident workgroups
// hide -- and is not launched.
// PAIR (8-pixel-wide images, CIFAR-10's 8 x 8 level): a chunk's 2 x 16 strip is the same two
// rows of images 2p (tiles 0-3) and 2p + 1 (tiles 4-7); each image's halo columns are padding
// (always zero), so a patch row is [0 | A x0..7 | 0 0 | B x0..7 | 0] and the gradient tiles of
// k-step ks come from image 2p + ks.  Strip cursor: n = pair, strips_x = 1.
// PRE: the convolved input is silu(x * s + t) with pre[n][cin] = (s, t) -- the GroupNorm+SiLU
// the forward conv applied in its input load (op.conv.gn_silu_conv3x3_ad) -- applied here in
// the patch store with the forward prologue's arithmetic; the zero padding stays zero.
// TWO: the K range runs over the images of two (x, gy) sources (x2, gy2 from image N1 on; PAIR
// needs N1 even) -- the weight gradient of one weight used by two convs in one launch; the
// bias gradient sums the first source's gradient tiles only.
template <int NB, bool PAIR = false, bool PRE = false, bool TWO = false>
__global__ __launch_bounds__(256, NB == 1 ? 2 : 1) void wino_wgrad_pipe_kernel(
    const float* __restrict__ x, const float* __restrict__ gy, float* __restrict__ part,
    float* __restrict__ part_b, WgradGeo g, int xcd_remap, const float2* __restrict__ pre,
    const float* __restrict__ x2, const float* __restrict__ gy2) {
  __shared__ __attribute__((aligned(16))) float s_x[2][kCB * kXCS];   // 2 x 14.3 KB
  __shared__ __attribute__((aligned(16))) float s_v[2][kT * kVT];     // 2 x 24.7 KB

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int kq = lane >> 4, jj = lane & 15;
  int64_t nblk = (int64_t)gridDim.x;
  int64_t b = blockIdx.x;
  if (xcd_remap) b = (b % 8) * (nblk / 8) + b / 8;
  const int ob = (int)(b % g.cout_blocks);
  const int cbk = (int)((b / g.cout_blocks) % g.cin_blocks);
  const int split = (int)(b / ((int64_t)g.cout_blocks * g.cin_blocks));
  const int cin0 = cbk * kCB, cout0 = ob * kOB * NB;
  const int64_t k_begin = g.chunks * split / g.splits;
  const int64_t k_end = g.chunks * (split + 1) / g.splits;
  const int nk = (int)(k_end - k_begin);
  const int plane = g.H * g.W;  // < 2^29 (host check)

  f4 acc[16][2][NB];
#pragma unroll
  for (int p = 0; p < 16; ++p)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[p][0][nb] = acc[p][1][nb] = f4{0.f, 0.f, 0.f, 0.f};
  // bias gradient (sum of dy over n, h, w): the cin-block-0 workgroups add up the gradient
  // tiles they load anyway; per-(split, cout) partials, reduced with dw
  const bool want_b = part_b != nullptr && cbk == 0;
  // Cout % 64 != 0 (multiples of 16): the last cout block's waves past Cout skip their gradient
  // loads, MFMAs and stores (wave-uniform); they still stage and transform the shared patch
  const bool wvalid = __builtin_amdgcn_readfirstlane(cout0 + 16 * NB * (tid >> 6)) < g.Cout;
  float bsum[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) bsum[nb] = 0.f;
  if (nk <= 0) {  // empty K-range: zero partial slabs (no barrier below)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int co = cout0 + 16 * NB * wave + 16 * nb + jj;
      if (!wvalid) continue;
      if (want_b && kq == 0) part_b[(int64_t)split * g.Cout + co] = 0.f;
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          f4* dst = reinterpret_cast<f4*>(
              part + (((int64_t)split * g.Cin + cin0 + 16 * mb + 4 * kq + r) * g.Cout + co) * 16);
#pragma unroll
          for (int q = 0; q < 4; ++q) dst[q] = f4{0.f, 0.f, 0.f, 0.f};
        }
    }
    return;
  }

  // chunk geometry (strip of 2 x 16 output pixels) as an incremental cursor: one division
  // at the start, then scalar increments; past the end of the K-range a cursor stays on the
  // last chunk (those loads are re-loads, never consumed)
  struct Strip { int n, sy, sx, j; };
  auto strip_at = [&](int j) {
    const unsigned ck = (unsigned)(k_begin + min(j, nk - 1));
    const unsigned r = ck / (unsigned)g.strips_x;
    Strip s;
    s.sx = __builtin_amdgcn_readfirstlane((int)(ck - r * (unsigned)g.strips_x));
    s.sy = __builtin_amdgcn_readfirstlane((int)(r % (unsigned)g.strips_y));
    s.n = __builtin_amdgcn_readfirstlane((int)(r / (unsigned)g.strips_y));
    s.j = min(j, nk - 1);
    return s;
  };
  auto advance = [&](Strip& s) {
    if (s.j + 1 >= nk) return;
    ++s.j;
    if (++s.sx == g.strips_x) {
      s.sx = 0;
      if (++s.sy == g.strips_y) {
        s.sy = 0;
        ++s.n;
      }
    }
  };

  // ---- input patch: thread -> (cin c, row py, half h): 2 x f4 interior + 1 halo word
  const int xp = tid >> 1, xh = tid & 1;
  const int xc = xp >> 2, xpy = xp & 3;
  float xv[9];
  float2 xst = make_float2(1.f, 0.f);  // PRE: the patch channel's (s, t)
  bool xrow_ok, xhalo_ok;
  Strip xcur = strip_at(0);
  auto load_x = [&]() {  // patch of chunk xcur, then advance
    const Strip s = xcur;
    advance(xcur);
    const int oy0 = 2 * s.sy, ox0 = PAIR ? -8 * xh : 16 * s.sx;  // PAIR: half xh = image 2n + xh
    int img = PAIR ? 2 * s.n + xh : s.n;
    const float* xsrc = x;
    if (TWO && img >= g.N1) {
      xsrc = x2;
      img -= g.N1;
    }
    const float* base = xsrc + ((int64_t)img * g.Cin + cin0) * plane;
    if (PRE) xst = pre[(int64_t)img * g.Cin + cin0 + xc];
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(base), 0, kCB * plane * 4, 0x00020000);
    const int iy = oy0 - 1 + xpy;
    xrow_ok = iy >= 0 && iy < g.H;
    const int iyc = min(max(iy, 0), g.H - 1);
    const int hx = xh ? ox0 + 16 : ox0 - 1;
    xhalo_ok = hx >= 0 && hx < g.W;
    const int hxc = min(max(hx, 0), g.W - 1);
    // without the prologue, rows / halo columns outside the image read as zero through the
    // buffer's range check (offsets past num_records = kCB * plane * 4 < 2^31 return 0): no
    // zeroing multiplies in store_x.  With it, silu(0 * s + t) != 0, so store_x masks.
    constexpr unsigned kOOB = 0x80000000u;
    const unsigned rowoff = (!PRE && !xrow_ok) ? kOOB : (unsigned)((xc * plane + iyc * g.W) * 4);
    const unsigned hoff = (!PRE && !(xrow_ok && xhalo_ok)) ? kOOB : rowoff + (unsigned)(hxc * 4);
    using u4 = __attribute__((ext_vector_type(4))) unsigned;
    const u4 a = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(rowoff + (unsigned)((ox0 + 8 * xh) * 4)), 0, 0);
    const u4 c = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(rowoff + (unsigned)((ox0 + 8 * xh + 4) * 4)), 0, 0);
    const unsigned hv = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)hoff, 0, 0);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      xv[e] = __uint_as_float(a[e]);
      xv[4 + e] = __uint_as_float(c[e]);
    }
    xv[8] = __uint_as_float(hv);
  };
  auto store_x = [&](float* sx) {
    float* row = sx + xc * kXCS + xpy * kXRS;
    if (PRE) {  // padding stays zero after the activation: mask here
      const float z = xrow_ok ? 1.f : 0.f;
#pragma unroll
      for (int e = 0; e < 9; ++e) {
        const float u = xv[e] * xst.x + xst.y;
        xv[e] = u * __builtin_amdgcn_rcpf(1.f + __expf(-u));
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) xv[e] *= z;
      xv[8] = (xrow_ok && xhalo_ok) ? xv[8] : 0.f;
    }
    if (PAIR) {  // image xh's 8 pixels at columns 4 + 10 xh (8-byte aligned for xh = 1)
      float2* r2 = reinterpret_cast<float2*>(row + 4 + 10 * xh);
#pragma unroll
      for (int e = 0; e < 4; ++e) r2[e] = make_float2(xv[2 * e], xv[2 * e + 1]);
      return;
    }
    *reinterpret_cast<f4*>(row + 4 + 8 * xh) = f4{xv[0], xv[1], xv[2], xv[3]};
    *reinterpret_cast<f4*>(row + 8 + 8 * xh) = f4{xv[4], xv[5], xv[6], xv[7]};
    row[xh ? 20 : 3] = xv[8];
  };

  // ---- V = B^T d B of one (tile, cin) per thread: c = tid >> 3, tile = tid & 7
  const int vc = tid >> 3, vt = tid & 7;
  const int vcol = 3 + 2 * vt + (PAIR && vt >= 4 ? 2 : 0);  // PAIR: past image A's right halo
  float d[4][4];
  auto read_d = [&](const float* sx) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) d[i][j] = sx[vc * kXCS + i * kXRS + vcol + j];
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
    f4* dst = reinterpret_cast<f4*>(&sv[vt * kVT + vc * kRec]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      dst[i] = f4{t[i][0] - t[i][2], t[i][1] + t[i][2], t[i][2] - t[i][1], t[i][1] - t[i][3]};
  };

  // ---- gradient tiles: lane (kq, jj) of wave w needs, per k-step ks and N-block nb, the
  // 2 x 2 tile (4 ks + kq) of channel cout0 + 16 NB w + 16 nb + jj
  const int gco = cout0 + 16 * NB * wave + jj;
  float2 gq[NB][2][2];  // [nb][ks][row], one chunk ahead
  Strip gcur = strip_at(0);
  // buffer loads: the chunk's base (image, this wave's first cout, strip origin) is uniform --
  // a scalar resource and soffset -- and the lane's part (cout jj + 16 nb, tile column) a
  // fixed 32-bit voffset: no per-chunk 64-bit address arithmetic on the vector unit
  const int gwave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int gvo0 = (jj * plane + 2 * kq) * 4;  // + 16 nb planes; + W floats for row 1
  bool g_src1 = true;  // TWO: the gradient tiles in gq are the first source's (bias gradient)
  auto load_g = [&](float2 (&dst)[NB][2][2]) {  // gradient tiles of chunk gcur, then advance
    const Strip s = gcur;
    advance(gcur);
    if (TWO) g_src1 = (PAIR ? 2 * s.n : s.n) < g.N1;
    if (!wvalid) return;  // past Cout: its MFMAs run on stale registers, never stored
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      {
        // tile 4 ks + kq; PAIR: k-step ks is image 2n + ks, tile column kq
        int img = PAIR ? 2 * s.n + ks : s.n;
        const float* gsrc = gy;
        if (TWO && img >= g.N1) {
          gsrc = gy2;
          img -= g.N1;
        }
        const float* base = gsrc + ((int64_t)img * g.Cout + cout0 + 16 * NB * gwave) * plane;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(base), 0, 16 * NB * plane * 4, 0x00020000);
        const int so = (2 * s.sy * g.W + (PAIR ? 0 : 16 * s.sx + 8 * ks)) * 4;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          using u2 = __attribute__((ext_vector_type(2))) unsigned;
          const int vo = gvo0 + 16 * nb * plane * 4;
          const u2 r0 = __builtin_amdgcn_raw_buffer_load_b64(rs, vo, so, 0);
          const u2 r1 = __builtin_amdgcn_raw_buffer_load_b64(rs, vo + g.W * 4, so, 0);
          dst[nb][ks][0] = make_float2(__uint_as_float(r0[0]), __uint_as_float(r0[1]));
          dst[nb][ks][1] = make_float2(__uint_as_float(r1[0]), __uint_as_float(r1[1]));
        }
      }
    }
  };
  // Gbar' = A' dY A'^T with A' = [[1,0],[1,1],[1,-1],[0,1]]: 16 values, position 4 i + j.
  // A' is the transform's A = [[1,0],[1,1],[1,-1],[0,-1]] with its last row negated, so
  // Gbar' = D Gbar D (D = diag(1,1,1,-1)) and the partial sums come out as D M D; the reduce
  // kernel's output transform absorbs D (G' = D G, exact sign flips: bit-identical dw) and the
  // 16 negations per k-step leave the MFMA loop
  auto gbar = [&](const float2 (&t)[2], f4 (&bq)[4]) {
    const float a = t[0].x, bb = t[0].y, c = t[1].x, dd = t[1].y;
    const float rows[4][2] = {{a, bb}, {a + c, bb + dd}, {a - c, bb - dd}, {c, dd}};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float p = rows[i][0], q = rows[i][1];
      bq[i] = f4{p, p + q, p - q, q};
    }
  };

  // ---- prologue
  if (PAIR) {  // the padding columns 3, 12, 13, 22 of every patch row, both buffers: zero once
    for (int i = tid; i < 2 * kCB * kXR; i += 256) {
      float* row = s_x[i / (kCB * kXR)] + ((i % (kCB * kXR)) / kXR) * kXCS + (i % kXR) * kXRS;
      row[3] = row[12] = row[13] = row[22] = 0.f;
    }
  }
  float xv0[9], xv1[9];
  float2 st0, st1;
  bool ok0r, ok0h, ok1r, ok1h;
  load_x();
#pragma unroll
  for (int e = 0; e < 9; ++e) xv0[e] = xv[e];
  ok0r = xrow_ok; ok0h = xhalo_ok; st0 = xst;
  load_x();
#pragma unroll
  for (int e = 0; e < 9; ++e) xv1[e] = xv[e];
  ok1r = xrow_ok; ok1h = xhalo_ok; st1 = xst;
  load_x();
  load_g(gq);
  {
    float keep[9];
    bool kr = xrow_ok, kh = xhalo_ok;
    const float2 kst = xst;
#pragma unroll
    for (int e = 0; e < 9; ++e) { keep[e] = xv[e]; xv[e] = xv0[e]; }
    xrow_ok = ok0r; xhalo_ok = ok0h; xst = st0;
    store_x(s_x[0]);
#pragma unroll
    for (int e = 0; e < 9; ++e) xv[e] = xv1[e];
    xrow_ok = ok1r; xhalo_ok = ok1h; xst = st1;
    store_x(s_x[1]);
#pragma unroll
    for (int e = 0; e < 9; ++e) xv[e] = keep[e];
    xrow_ok = kr; xhalo_ok = kh; xst = kst;
  }
  __syncthreads();
  read_d(s_x[0]);
  write_v(s_v[0]);
  __syncthreads();

  // step j: MFMAs of chunk j (V in s_v[SB], Gbar from gq); side work: V(j+1) from
  // s_x[SB^1], patch(j+2) -> s_x[SB], patch(j+3) and gradient(j+1) loads
  auto step = [&](auto sb_c) {
    constexpr int SB = decltype(sb_c)::value;
    const float* sv = s_v[SB];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      f4 bq[NB][4];
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        gbar(gq[nb][ks], bq[nb]);
        if (want_b && (!TWO || g_src1))
          bsum[nb] += (gq[nb][ks][0].x + gq[nb][ks][0].y) + (gq[nb][ks][1].x + gq[nb][ks][1].y);
      }
      if (ks == 1) load_g(gq);  // chunk j + 1 (both k-steps' tiles consumed)
      const int tile = 4 * ks + kq;
#pragma unroll
      for (int mb = 0; mb < 2; ++mb) {
        __builtin_amdgcn_sched_barrier(0);
        if (ks == 0 && mb == 0) read_d(s_x[SB ^ 1]);
        if (ks == 0 && mb == 1) write_v(s_v[SB ^ 1]);
        if (ks == 1 && mb == 0) store_x(s_x[SB]);
        if (ks == 1 && mb == 1) load_x();  // chunk j + 3
        __builtin_amdgcn_sched_barrier(0);
        const f4* as = reinterpret_cast<const f4*>(&sv[tile * kVT + (16 * mb + jj) * kRec]);
        f4 a[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) a[q] = as[q];
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
#pragma unroll
          for (int p = 0; p < 16; ++p)
            acc[p][mb][nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                a[p >> 2][p & 3], bq[nb][p >> 2][p & 3], acc[p][mb][nb], 0, 0, 0);
      }
    }
    __syncthreads();
  };
  int j = 0;
  for (; j + 1 < nk; j += 2) {
    step(std::integral_constant<int, 0>{});
    step(std::integral_constant<int, 1>{});
  }
  if (j < nk) step(std::integral_constant<int, 0>{});

  if (!wvalid) return;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int co = gco + 16 * nb;
    if (want_b) {  // lanes jj, jj + 16, jj + 32, jj + 48 hold one channel's tiles
      float bs = bsum[nb];
      bs += __shfl_xor(bs, 16, 64);
      bs += __shfl_xor(bs, 32, 64);
      if (kq == 0) part_b[(int64_t)split * g.Cout + co] = bs;
    }
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ci = cin0 + 16 * mb + 4 * kq + r;
        f4* dst = reinterpret_cast<f4*>(part + (((int64_t)split * g.Cin + ci) * g.Cout + co) * 16);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          dst[q] = f4{acc[4 * q][mb][nb][r], acc[4 * q + 1][mb][nb][r], acc[4 * q + 2][mb][nb][r],
                      acc[4 * q + 3][mb][nb][r]};
      }
  }
}

// dw[cout][cin] = G'^T (sum_s part[s][cin][cout]) G',  G'^T = [[1,.5,.5,0],[0,.5,-.5,0],[0,.5,.5,-1]]
// (G' = D G: the partials are D M D, see gbar in wino_wgrad_pipe_kernel)
// Block = 16 (cin, cout) pairs x 4 float4 columns of their 16 partial values x 4 groups of
// splits (group g sums splits g, g + 4, ...; the groups combine in a fixed order in LDS):
// deterministic, and 16x the parallelism of one thread per pair (the PINN shapes have few
// pairs and hundreds of splits).
__global__ __launch_bounds__(256) void wino_wgrad_reduce_kernel(const float* __restrict__ part,
                                                                float* __restrict__ dw,
                                                                const float* __restrict__ part_b,
                                                                float* __restrict__ db, int Cin,
                                                                int Cout, int splits) {
  __shared__ f4 red[4][64];
  const int64_t pairs = (int64_t)Cin * Cout;
  if (db && blockIdx.x == 0) {  // db[cout] = sum over splits, fixed order
    for (int i = threadIdx.x; i < Cout; i += blockDim.x) {
      float acc = 0.f;
      int sp = 0;
      for (; sp + 7 < splits; sp += 8) {
        float t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = part_b[(int64_t)(sp + u) * Cout + i];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += t[u];
      }
      for (; sp < splits; ++sp) acc += part_b[(int64_t)sp * Cout + i];
      db[i] = acc;
    }
  }
  const int col = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 16 + (col >> 2);  // pair
  const int q = col & 3;
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
  if (i < pairs) {
    // eight loads in flight per thread, added in split order (the same sum)
    int s = grp;
    for (; s + 28 < splits; s += 32) {
      f4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = *reinterpret_cast<const f4*>(part + ((int64_t)(s + 4 * u) * pairs + i) * 16 + 4 * q);
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; s < splits; s += 4)
      acc += *reinterpret_cast<const f4*>(part + ((int64_t)s * pairs + i) * 16 + 4 * q);
  }
  red[grp][col] = acc;
  __syncthreads();
  if (grp == 0) red[0][col] = ((red[0][col] + red[1][col]) + red[2][col]) + red[3][col];
  __syncthreads();
  if (threadIdx.x < 16) {
    const int64_t pi = (int64_t)blockIdx.x * 16 + threadIdx.x;
    if (pi < pairs) {
      f4 u[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) u[r] = red[0][4 * threadIdx.x + r];
      float t[3][4];  // G'^T dU (rows of dU = u[row])
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        t[0][j] = u[0][j] + 0.5f * (u[1][j] + u[2][j]);
        t[1][j] = 0.5f * (u[1][j] - u[2][j]);
        t[2][j] = 0.5f * (u[1][j] + u[2][j]) - u[3][j];
      }
      const int ci = (int)(pi / Cout), co = (int)(pi % Cout);
      float* o = dw + ((int64_t)co * Cin + ci) * 9;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        o[3 * r + 0] = t[r][0] + 0.5f * (t[r][1] + t[r][2]);
        o[3 * r + 1] = 0.5f * (t[r][1] - t[r][2]);
        o[3 * r + 2] = 0.5f * (t[r][1] + t[r][2]) - t[r][3];
      }
    }
  }
}

constexpr int kNB = 1;  // N-blocks per wave (see wino_wgrad_pipe_kernel)

static bool wgrad_pair(int N, int W) { return W == 8 && N % 2 == 0; }

WgradGeo make_geo(int N, int Cin, int Cout, int H, int W) {
  WgradGeo g{};
  const int nb = kNB;
  g.N = N; g.Cin = Cin; g.Cout = Cout; g.H = H; g.W = W;
  const bool pair = wgrad_pair(N, W);
  g.strips_x = pair ? 1 : W / 16;
  g.strips_y = H / 2;
  g.cin_blocks = Cin / kCB;
  g.cout_blocks = (Cout + kOB * nb - 1) / (kOB * nb);  // Cout % 16 == 0; the last may be partial
  g.chunks = (int64_t)(pair ? N / 2 : N) * g.strips_y * g.strips_x;
  // ~512 resident workgroups' worth (two per CU at NB = 1, one at NB = 2, twice the work
  // each): enough K-splits to fill the chip, no more (each split adds a [Cin][Cout][16]
  // partial slab to write and re-read)
  const int64_t tiles = (int64_t)g.cin_blocks * g.cout_blocks;
  const int64_t target = nb == 1 ? 512 : 256;
  const int64_t want = std::max<int64_t>(1, (target + tiles - 1) / tiles);
  // at least 8 chunks per split: with 1-2 per split the small-image shapes (the PINN's 64^2
  // levels at 8 samples per GPU) were all prologue and partial-slab traffic -- round 6,
  // tools/bench_wgrad3x3.py: B = 8 shapes 776 -> 654 us in sum, B = 64 unchanged
  g.splits = (int)std::max<int64_t>(1, std::min<int64_t>(want, g.chunks / 8));
  return g;
}

}  // namespace

extern "C" int bpk_conv3x3_wino_wgrad_supported(int N, int Cin, int Cout, int H, int W) {
  return N > 0 && Cin > 0 && Cout > 0 && Cin % kCB == 0 && Cout % 16 == 0 && H % 2 == 0 &&
         (W % 16 == 0 || wgrad_pair(N, W)) && (int64_t)H * W * kCB * 4 < (1LL << 31);
}

extern "C" int64_t bpk_conv3x3_wino_wgrad_workspace_bytes(int N, int Cin, int Cout, int H,
                                                          int W) {
  if (!bpk_conv3x3_wino_wgrad_supported(N, Cin, Cout, H, W)) return 0;
  const WgradGeo g = make_geo(N, Cin, Cout, H, W);
  return ((int64_t)g.splits * Cin * Cout * 16 + (int64_t)g.splits * Cout) * (int64_t)sizeof(float);
}

extern "C" int bpk_conv3x3_wino_wgrad_f32(const float* x, const float* gy, float* dw,
                                          float* workspace, int N, int Cin, int Cout, int H,
                                          int W, void* stream) {
  return bpk_conv3x3_wino_wgrad_bias_f32(x, gy, dw, nullptr, workspace, N, Cin, Cout, H, W,
                                         stream);
}

extern "C" int bpk_conv3x3_wino_wgrad_bias_f32(const float* x, const float* gy, float* dw,
                                               float* db, float* workspace, int N, int Cin,
                                               int Cout, int H, int W, void* stream) {
  return bpk_conv3x3_wino_wgrad_pre_f32(x, nullptr, gy, dw, db, workspace, N, Cin, Cout, H, W,
                                        stream);
}

namespace {

int wgrad_launch(const float* x, const float* pre, const float* gy, const float* x2,
                 const float* gy2, int N2, float* dw, float* db, float* workspace, int N, int Cin,
                 int Cout, int H, int W, void* stream);

}  // namespace

extern "C" int bpk_conv3x3_wino_wgrad_pre_f32(const float* x, const float* pre, const float* gy,
                                              float* dw, float* db, float* workspace, int N,
                                              int Cin, int Cout, int H, int W, void* stream) {
  return wgrad_launch(x, pre, gy, nullptr, nullptr, 0, dw, db, workspace, N, Cin, Cout, H, W,
                      stream);
}

extern "C" int bpk_conv3x3_wino_wgrad2_f32(const float* x, const float* gy, const float* x2,
                                           const float* gy2, int N2, float* dw, float* db,
                                           float* workspace, int N, int Cin, int Cout, int H,
                                           int W, void* stream) {
  BPK_REQUIRE(N > 0 && N2 > 0 && x2 && gy2, "conv3x3_wino_wgrad2: second source missing (N2=%d)",
              N2);
  BPK_REQUIRE(!wgrad_pair(N + N2, W) || N % 2 == 0,
              "conv3x3_wino_wgrad2: 8-wide images need an even first source (N=%d)", N);
  return wgrad_launch(x, nullptr, gy, x2, gy2, N2, dw, db, workspace, N, Cin, Cout, H, W, stream);
}

namespace {

int wgrad_launch(const float* x, const float* pre, const float* gy, const float* x2,
                 const float* gy2, int N2, float* dw, float* db, float* workspace, int N1, int Cin,
                 int Cout, int H, int W, void* stream) {
  const int N = N1 + N2;
  BPK_REQUIRE(bpk_conv3x3_wino_wgrad_supported(N, Cin, Cout, H, W),
              "conv3x3_wino_wgrad: unsupported shape N=%d Cin=%d Cout=%d H=%d W=%d (need Cin "
              "%% 32, Cout %% 16, H %% 2, W %% 16 == 0 or W == 8 with N even)", N, Cin, Cout,
              H, W);
  BPK_REQUIRE(workspace != nullptr, "conv3x3_wino_wgrad: workspace is NULL");
  WgradGeo g = make_geo(N, Cin, Cout, H, W);
  g.N1 = N1;
  const int64_t blocks = (int64_t)g.splits * g.cin_blocks * g.cout_blocks;
  BPK_REQUIRE(blocks < (1LL << 31), "conv3x3_wino_wgrad: grid too large");
  hipStream_t st = bpk::as_stream(stream);
  const int remap = (blocks % 8 == 0) ? 1 : 0;
  float* part_b = db ? workspace + (int64_t)g.splits * Cin * Cout * 16 : nullptr;
  const float2* kp = reinterpret_cast<const float2*>(pre);
#define BPK_WG(PAIR_, PRE_, TWO_)                                                                \
  hipLaunchKernelGGL((wino_wgrad_pipe_kernel<kNB, PAIR_, PRE_, TWO_>), dim3((unsigned)blocks),  \
                     dim3(256), 0, st, x, gy, workspace, part_b, g, remap, kp, x2, gy2)
  if (N2 > 0) {  // two sources (no prologue)
    if (wgrad_pair(N, W)) BPK_WG(true, false, true); else BPK_WG(false, false, true);
  } else if (wgrad_pair(N, W)) {
    if (pre) BPK_WG(true, true, false); else BPK_WG(true, false, false);
  } else {
    if (pre) BPK_WG(false, true, false); else BPK_WG(false, false, false);
  }
#undef BPK_WG
  BPK_LAUNCH_CHECK("conv3x3_wino_wgrad");
  const int64_t pairs = (int64_t)Cin * Cout;
  BPK_REQUIRE(bpk::ceil_div(pairs, 16) < (1LL << 31), "conv3x3_wino_wgrad: too many pairs");
  hipLaunchKernelGGL(wino_wgrad_reduce_kernel, dim3((unsigned)bpk::ceil_div(pairs, 16)),
                     dim3(256), 0, st, workspace, dw, part_b, db, Cin, Cout, g.splits);
  BPK_LAUNCH_CHECK("conv3x3_wino_wgrad_reduce");
  return BPK_OK;
}

}  // namespace
