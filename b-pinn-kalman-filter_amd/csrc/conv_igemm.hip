// General 2-D convolution (any kernel size, stride, zero padding; groups = 1, dilation = 1)
// as implicit GEMM on the f32-input MFMA (v_mfma_f32_16x16x4_f32), NCHW fp32, gfx950.
//
// The Winograd kernel (conv_winograd.hip) covers the score networks' big 3x3 / stride-1
// convs; everything else the networks run -- the PINN's convs at 2^2..8^2 and with Cin not a
// multiple of 8 (FlowNet's 49- and 2f+2-channel inputs), every stride-2 conv, the CIFAR nets'
// 8^2 / 4^2 levels, the ConvTranspose2d layers (PressureNet up path, FlowNet flow upsample) --
// ran on MIOpen (plus its NHWC transposes and per-call host search).  One kernel family
// covers all three products of a conv:
//
//   MODE 0  forward        C[co][p]      = sum_{ci,r,s} w[co][ci][r][s] x[n][ci][oy s_h - p_h + r][ox s_w - p_w + s]
//                          (p = (n, oy, ox) over the whole batch: small images do not
//                          starve the grid)
//   MODE 1  backward-data  C[ci][p_in]   = sum_{co,r,s} w[co][ci][r][s] gy[n][co][oy][ox]
//                          with oy = (iy + p_h - r) / s_h when that divides exactly (the
//                          conv transpose; also ConvTranspose2d's forward)
//   MODE 2  weight grad    C[co][(ci,r,s)] = sum_p gy[n][co][oy][ox] x[n][ci][iy][ix], plus
//                          one extra column of ones: the bias gradient sum_p gy[co][p]
//   MODE 3  backward-data of a strided conv, one input-pixel class per launch: the pixels
//                          (iy, ix) = (cy + s_h iyc, cx + s_w ixc) only receive the taps
//                          r = rc0 + s_h i, s = sc0 + s_w j (r = (cy + p_h) mod s_h ...), so
//                          each class is a dense GEMM over Cout * KHc * KWc instead of MODE 1's
//                          K = Cout * KH * KW of which 3/4 are structural zeros at stride 2
//
// Tile: 64 x 64 (or, when those alone fill the chip, 128 x 128) outputs per workgroup (4
// waves, 2 x 2 of 32 x 32 / 64 x 64, each 2 x 2 / 4 x 4 MFMA blocks),
// K in chunks of 16 staged through double-buffered LDS (operands gathered with the
// convolution's index arithmetic and zero padding; the next chunk's global loads are in
// flight while the current chunk's 16 MFMAs per wave run).  Split-K over grid.z when the
// output tiles alone cannot fill the chip (tiny images, the weight gradient's long pixel
// sum): partials go to a workspace and a second kernel adds them in a fixed order, so
// results are deterministic (no atomics).
#include "bpk_common.h"

#include <algorithm>

namespace {

using f4 = __attribute__((ext_vector_type(4))) float;

constexpr int BK = 16;

// n / d for 0 <= n < 2^31 by multiply-high and shift (d > 0 fixed per launch): the runtime
// divisors (pixels per image, row width, stride, generic tap counts) would otherwise cost a
// ~40-instruction integer division per gathered element
struct FDiv {
  unsigned d, m, s;
};
FDiv make_fdiv(unsigned d) {
  unsigned s = 0;
  while ((1u << s) < d) ++s;
  const uint64_t m = ((uint64_t(1) << 32) * ((uint64_t(1) << s) - d)) / d + 1;
  return FDiv{d, (unsigned)m, s};
}
__device__ inline int fdiv(int n, const FDiv& f) {
  return (int)((__umulhi((unsigned)n, f.m) + (unsigned)n) >> f.s);
}

struct IgGeo {
  int N, Cin, H, W, Cout, Ho, Wo, KH, KW, sh, sw, ph, pw;
  int M, Ncol, K;  // GEMM shape
  int KHW, HW, HoWo;
  int nchunk, chunks_per_split, splits, tile;  // tile: 0 = 64x64, 1 = 128x128, 2 = 16x256
  int wcols;  // MODE 2: Cin * KH * KW (the column Ncol - 1 == wcols is the bias column)
  FDiv f_howo, f_wo, f_hw, f_w, f_khw, f_kw, f_sh, f_sw;
  // MODE 3: the input-pixel class (cy, cx), its grid Hc x Wc and sub-filter KHc x KWc whose
  // taps start at (rc0, sc0) and step by the stride
  int cy, cx, Hc, Wc, KHc, KWc, rc0, sc0;
  FDiv f_hwc, f_wc, f_khwc, f_kwc;
  // tap-major K order (forward, stride-1 backward-data of 3x3 filters with Cc % 16 == 0):
  // k = (r * KW + s) * Cc + c, Cc = Cin (forward) or Cout (backward-data), so a 16-wide
  // K-chunk is 16 channels of ONE tap
  int tap, Cc;
  FDiv f_cc;
  // MODE 2 over two (x, gy) sources: images n < N1 of the K range come from (B0, A0), the
  // others from (B1, A1) as image n - N1 (the weight gradient of one weight used by two convs
  // in one launch); the bias column counts images n < Nb only
  const float* A1;
  const float* B1;
  int N1, Nb;
};

// k -> (co, r, s) of a MODE 3 class sub-filter tap
__device__ inline void split_tap_class(int k, const IgGeo& g, int& co, int& r, int& s) {
  co = fdiv(k, g.f_khwc);
  const int t = k - co * (g.KHc * g.KWc);
  const int ri = fdiv(t, g.f_kwc);
  r = g.rc0 + ri * g.sh;
  s = g.sc0 + (t - ri * g.KWc) * g.sw;
}

// MODE 3 column -> output offset of its input pixel (n, cy + sh iyc, cx + sw ixc)
__device__ inline int64_t class_pixel_offset(int col, const IgGeo& g) {
  const int n = fdiv(col, g.f_hwc), pix = col - n * (g.Hc * g.Wc);
  const int iyc = fdiv(pix, g.f_wc), ixc = pix - iyc * g.Wc;
  return (int64_t)n * g.Cin * g.HW + (int64_t)(g.cy + iyc * g.sh) * g.W + g.cx + ixc * g.sw;
}

// k -> (c, r, s) of a filter tap index k = (c * KH + r) * KW + s; compile-time KH, KW turn
// the divisions into multiplies
template <int KH_, int KW_>
__device__ inline void split_tap(int k, const IgGeo& g, int& c, int& r, int& s) {
  const int khw = KH_ ? KH_ * KW_ : g.KHW;
  const int kw = KW_ ? KW_ : g.KW;
  c = KH_ ? k / khw : fdiv(k, g.f_khw);
  const int rs = k - c * khw;
  r = KW_ ? rs / kw : fdiv(rs, g.f_kw);
  s = rs - r * kw;
}

// TM x TN outputs per workgroup of 4 waves (WMW along M x 4 / WMW along N; each wave
// NBM x NBN MFMA blocks of 16 x 16), K chunks of 16 through double-buffered LDS
template <int MODE, int KH_, int KW_, int TM, int TN, int WMW, bool TAP>
__global__ __launch_bounds__(256) void igemm_kernel(const float* __restrict__ A0,
                                                    const float* __restrict__ B0,
                                                    const float* __restrict__ bias,
                                                    float* __restrict__ out,
                                                    float* __restrict__ out2,
                                                    float* __restrict__ ws, IgGeo g) {
  constexpr int WNW = 4 / WMW;
  constexpr int WTM = TM / WMW, WTN = TN / WNW;  // wave tile
  constexpr int NBM = WTM / 16, NBN = WTN / 16;  // MFMA blocks per wave
  constexpr int NLA = TM / 16, NLB = TN / 16;    // A / B elements each thread stages per chunk
  constexpr int kAP = BK + 1;                    // LDS pitch of the A tile [m][k]
  // LDS pitch of the B tile [k][n]: TN + 16 makes the MFMA operand reads conflict-free; the
  // weight gradient stores the tile k-fastest (16 lanes = 16 k), where that pitch put 8 lanes
  // on one bank -- TN + 18 (= 18 mod 32: 16 distinct even banks per half-wave) leaves its
  // stores conflict-free and 2 of 32 lanes of each operand read 2-way
  constexpr int kBP = TN + (MODE == 2 ? 18 : 16);
  __shared__ float s_a[2][TM * kAP];
  __shared__ float s_b[2][BK * kBP];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int kq = lane >> 4, jj = lane & 15;
  const int n0 = blockIdx.x * TN, m0 = blockIdx.y * TM;
  const int kc0 = blockIdx.z * g.chunks_per_split;
  const int kc1 = min(g.nchunk, kc0 + g.chunks_per_split);

  // ---- A loads: thread -> (k = tid & 15, m = tid / 16 + 16 j)
  const int ak = tid & 15, am = tid >> 4;
  // ---- B loads: MODE 0/1 thread -> (n = tid % TN, k = tid / TN + (256 / TN) j)
  //      (pixels coalesced); MODE 2 thread -> (k = tid & 15, n = tid / 16 + 16 j) (k = pixels)
  constexpr int kBStep = TN >= 256 ? 1 : 256 / TN;
  const int bn = MODE == 2 ? (tid >> 4) : (tid % TN);
  const int bk = MODE == 2 ? (tid & 15) : (tid / TN);

  // per-thread fixed part of the B gather
  int64_t bbase = 0;  // MODE 0/1: image base of this thread's pixel column
  int py = 0, px = 0;
  bool pvalid = false;
  int bc[NLB], br[NLB], bs[NLB];  // MODE 2: the (c, r, s) of this thread's columns
  bool bcol_ok[NLB], bcol_one[NLB];
  // MODE 2 with a compile-time filter (<= 16 taps): column j's element offset from the tap
  // origin (c HW + r W + s) and its bit in the chunk's valid-tap mask (bit 16: the bias column,
  // 0: past the last column), so a gathered element costs a mask test and an add
  constexpr bool kMask2 = MODE == 2 && KH_ > 0 && KH_ * KW_ <= 16;
  int boff[NLB];
  unsigned bbit[NLB];
  if (MODE != 2) {
    const int p = n0 + bn;
    pvalid = p < g.Ncol;
    const int pp = pvalid ? p : 0;
    if (MODE == 0) {
      const int n = fdiv(pp, g.f_howo), pix = pp - n * g.HoWo;
      const int oy = fdiv(pix, g.f_wo), ox = pix - oy * g.Wo;
      py = oy * g.sh - g.ph;
      px = ox * g.sw - g.pw;
      bbase = (int64_t)n * g.Cin * g.HW;
    } else if (MODE == 3) {
      const int n = fdiv(pp, g.f_hwc), pix = pp - n * (g.Hc * g.Wc);
      const int iyc = fdiv(pix, g.f_wc), ixc = pix - iyc * g.Wc;
      py = g.cy + iyc * g.sh + g.ph;
      px = g.cx + ixc * g.sw + g.pw;
      bbase = (int64_t)n * g.Cout * g.HoWo;
    } else {
      const int n = fdiv(pp, g.f_hw), pix = pp - n * g.HW;
      const int iy = fdiv(pix, g.f_w), ix = pix - iy * g.W;
      py = iy + g.ph;
      px = ix + g.pw;
      bbase = (int64_t)n * g.Cout * g.HoWo;
    }
  } else {
#pragma unroll
    for (int j = 0; j < NLB; ++j) {
      const int col = n0 + bn + 16 * j;
      bcol_ok[j] = col < g.Ncol;
      bcol_one[j] = col == g.wcols;
      int c, r, s;
      split_tap<KH_, KW_>(bcol_ok[j] && !bcol_one[j] ? col : 0, g, c, r, s);
      bc[j] = c;
      br[j] = r;
      bs[j] = s;
      if (kMask2) {
        boff[j] = c * g.HW + r * g.W + s;
        bbit[j] = !bcol_ok[j] ? 0u : bcol_one[j] ? (1u << 16) : (1u << (r * KW_ + s));
      }
    }
  }

  float ra[NLA], rb[NLB];
  auto gload = [&](int kc) {
    const int kb = kc * BK;
    // tap-major chunk: one tap (r, s) for channels c0 .. c0 + 15 -- the gathers below need
    // one bounds test and one address per chunk instead of a (c, r, s) split per element
    int tap_rs = 0, tap_c0 = 0, tap_r = 0, tap_s = 0;
    if (TAP) {
      tap_rs = fdiv(kb, g.f_cc);
      tap_c0 = kb - tap_rs * g.Cc;
      tap_r = tap_rs / KW_;
      tap_s = tap_rs - tap_r * KW_;
    }
    // A
    if (TAP) {
#pragma unroll
      for (int j = 0; j < NLA; ++j) {
        const int m = m0 + am + 16 * j;
        float v = 0.f;
        if (m < g.M) {
          if (MODE == 0)  // w[m][c][r][s]
            v = A0[((int64_t)m * g.Cin + tap_c0 + ak) * (KH_ * KW_) + tap_rs];
          else            // w[co][m][r][s]
            v = A0[((int64_t)(tap_c0 + ak) * g.Cin + m) * (KH_ * KW_) + tap_rs];
        }
        ra[j] = v;
      }
    } else {
      const int k = kb + ak;
      int a_co = 0, a_rs = 0, a_n = 0, a_pix = 0;
      if (MODE == 1) {
        const int khw = KH_ ? KH_ * KW_ : g.KHW;
        a_co = KH_ ? k / khw : fdiv(k, g.f_khw);
        a_rs = k - a_co * khw;
      } else if (MODE == 3) {
        int r, s;
        split_tap_class(k < g.K ? k : 0, g, a_co, r, s);
        a_rs = r * g.KW + s;
      } else if (MODE == 2) {
        a_n = fdiv(k < g.K ? k : 0, g.f_howo);
        a_pix = k - a_n * g.HoWo;
      }
#pragma unroll
      for (int j = 0; j < NLA; ++j) {
        const int m = m0 + am + 16 * j;
        float v = 0.f;
        if (m < g.M && k < g.K) {
          if (MODE == 0) {
            v = A0[(int64_t)m * g.K + k];
          } else if (MODE == 1) {  // m = ci, k = (co, r, s)
            const int khw = KH_ ? KH_ * KW_ : g.KHW;
            v = A0[((int64_t)a_co * g.Cin + m) * khw + a_rs];
          } else if (MODE == 3) {  // m = ci, k = (co, class tap)
            v = A0[((int64_t)a_co * g.Cin + m) * g.KHW + a_rs];
          } else {  // m = co, k = pixel
            const bool s2 = a_n >= g.N1;
            v = (s2 ? g.A1 : A0)[((int64_t)(s2 ? a_n - g.N1 : a_n) * g.Cout + m) * g.HoWo + a_pix];
          }
        }
        ra[j] = v;
      }
    }
    // B
    if (TAP) {
      int ty, tx, hh, ww;
      if (MODE == 0) {
        ty = py + tap_r; tx = px + tap_s; hh = g.H; ww = g.W;
      } else {  // stride 1: the output pixel is the input pixel shifted back by the tap
        ty = py - tap_r; tx = px - tap_s; hh = g.Ho; ww = g.Wo;
      }
      const bool ok = pvalid && ty >= 0 && ty < hh && tx >= 0 && tx < ww;
      const int64_t cstride = (int64_t)hh * ww;
      const float* bp = B0 + bbase + (int64_t)ty * ww + tx + (int64_t)(tap_c0 + bk) * cstride;
#pragma unroll
      for (int j = 0; j < NLB; ++j) rb[j] = ok ? bp[(int64_t)(kBStep * j) * cstride] : 0.f;
    } else if (MODE != 2) {
#pragma unroll
      for (int j = 0; j < NLB; ++j) {
        const int k = kb + bk + kBStep * j;
        float v = 0.f;
        int c, r, s;
        if (MODE == 3)
          split_tap_class(k < g.K ? k : 0, g, c, r, s);
        else
          split_tap<KH_, KW_>(k < g.K ? k : 0, g, c, r, s);
        if (MODE == 0) {
          const int iy = py + r, ix = px + s;
          if (pvalid && k < g.K && iy >= 0 && iy < g.H && ix >= 0 && ix < g.W)
            v = B0[bbase + ((int64_t)c * g.H + iy) * g.W + ix];
        } else {
          const int ty = py - r, tx = px - s;  // MODE 3: multiples of the stride by construction
          if (pvalid && k < g.K && ty >= 0 && tx >= 0) {
            const int oy = fdiv(ty, g.f_sh), ox = fdiv(tx, g.f_sw);
            if ((MODE == 3 || (oy * g.sh == ty && ox * g.sw == tx)) && oy < g.Ho && ox < g.Wo)
              v = B0[bbase + ((int64_t)c * g.Ho + oy) * g.Wo + ox];
          }
        }
        rb[j] = v;
      }
    } else if (kMask2) {
      const int k = kb + bk;  // pixel
      const bool kv = k < g.K;
      const int kk = kv ? k : 0;
      const int n = fdiv(kk, g.f_howo), pix = kk - n * g.HoWo;
      const int oy = fdiv(pix, g.f_wo), ox = pix - oy * g.Wo;
      const int iy0 = oy * g.sh - g.ph, ix0 = ox * g.sw - g.pw;
      unsigned rm = 0, sm = 0, vm = 0;
#pragma unroll
      for (int r = 0; r < KH_; ++r) rm |= (unsigned)((unsigned)(iy0 + r) < (unsigned)g.H) << r;
#pragma unroll
      for (int q = 0; q < KW_; ++q) sm |= (unsigned)((unsigned)(ix0 + q) < (unsigned)g.W) << q;
#pragma unroll
      for (int r = 0; r < KH_; ++r) vm |= ((rm >> r) & 1u) ? sm << (r * KW_) : 0u;
      vm = kv ? vm | (n < g.Nb ? 1u << 16 : 0u) : 0u;
      // the tap origin's element offset; negative only where the mask excludes the tap
      const bool s2 = n >= g.N1;
      const float* bsrc = s2 ? g.B1 : B0;
      const int pb = (s2 ? n - g.N1 : n) * g.Cin * g.HW + iy0 * g.W + ix0;
#pragma unroll
      for (int j = 0; j < NLB; ++j) {
        float v = 0.f;
        if (vm & bbit[j]) v = bcol_one[j] ? 1.f : bsrc[(unsigned)(pb + boff[j])];
        rb[j] = v;
      }
    } else {
      const int k = kb + bk;  // pixel
      const bool kv = k < g.K;
      const int kk = kv ? k : 0;
      const int n = fdiv(kk, g.f_howo), pix = kk - n * g.HoWo;
      const int oy = fdiv(pix, g.f_wo), ox = pix - oy * g.Wo;
      const int iy0 = oy * g.sh - g.ph, ix0 = ox * g.sw - g.pw;
      const bool s2 = n >= g.N1;
      const float* bsrc = s2 ? g.B1 : B0;
      const int64_t xb = (int64_t)(s2 ? n - g.N1 : n) * g.Cin * g.HW;
#pragma unroll
      for (int j = 0; j < NLB; ++j) {
        float v = 0.f;
        if (kv && bcol_ok[j]) {
          if (bcol_one[j]) {
            v = n < g.Nb ? 1.f : 0.f;
          } else {
            const int iy = iy0 + br[j], ix = ix0 + bs[j];
            if (iy >= 0 && iy < g.H && ix >= 0 && ix < g.W)
              v = bsrc[xb + ((int64_t)bc[j] * g.H + iy) * g.W + ix];
          }
        }
        rb[j] = v;
      }
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int j = 0; j < NLA; ++j) s_a[buf][(am + 16 * j) * kAP + ak] = ra[j];
#pragma unroll
    for (int j = 0; j < NLB; ++j) {
      if (MODE == 2)
        s_b[buf][bk * kBP + bn + 16 * j] = rb[j];
      else
        s_b[buf][(bk + kBStep * j) * kBP + bn] = rb[j];
    }
  };

  const int wm = wave % WMW, wn = wave / WMW;
  f4 acc[NBM][NBN];
#pragma unroll
  for (int i = 0; i < NBM; ++i)
#pragma unroll
    for (int j = 0; j < NBN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  if (kc0 < kc1) {
    gload(kc0);
    sstore(0);
    __syncthreads();
    for (int kc = kc0; kc < kc1; ++kc) {
      const int buf = (kc - kc0) & 1;
      const bool more = kc + 1 < kc1;
      if (more) gload(kc + 1);
      const float* sa = s_a[buf];
      const float* sb = s_b[buf];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        float a[NBM], b[NBN];
#pragma unroll
        for (int mb = 0; mb < NBM; ++mb) a[mb] = sa[(wm * WTM + mb * 16 + jj) * kAP + 4 * ks + kq];
#pragma unroll
        for (int nb = 0; nb < NBN; ++nb) b[nb] = sb[(4 * ks + kq) * kBP + wn * WTN + nb * 16 + jj];
#pragma unroll
        for (int mb = 0; mb < NBM; ++mb)
#pragma unroll
          for (int nb = 0; nb < NBN; ++nb)
            acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mb], b[nb], acc[mb][nb], 0, 0, 0);
      }
      if (more) sstore(buf ^ 1);
      __syncthreads();
    }
  }

  // epilogue: acc[mb][nb][i] = C[m0 + WTM wm + 16 mb + 4 kq + i][n0 + WTN wn + 16 nb + jj]
  // forward bias: the lane's NBM x 4 values requested together before the stores (loaded per
  // store, each was waited for in turn)
  float bbv[NBM][4];
#pragma unroll
  for (int mb = 0; mb < NBM; ++mb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wm * WTM + mb * 16 + 4 * kq + i;
      bbv[mb][i] = (MODE == 0 && g.splits == 1 && bias && m < g.M) ? bias[m] : 0.f;
    }
  // a whole tile in range (MODE 0 / 1, or split-K slabs): straight-line stores.  With the
  // per-element guards below every store sat in its own branch and the wait counter (vmcnt
  // counts stores on gfx9) was drained to 0 before each one.
  if (MODE != 2 && m0 + TM <= g.M && n0 + TN <= g.Ncol) {
#pragma unroll
    for (int nb = 0; nb < NBN; ++nb) {
      const int col = n0 + wn * WTN + nb * 16 + jj;
      int64_t obase, ostride;
      if (g.splits > 1) {
        obase = (int64_t)blockIdx.z * g.M * g.Ncol + col;
        ostride = g.Ncol;
      } else if (MODE == 0) {
        const int n = fdiv(col, g.f_howo), pix = col - n * g.HoWo;
        obase = (int64_t)n * g.Cout * g.HoWo + pix;
        ostride = g.HoWo;
      } else if (MODE == 3) {
        obase = class_pixel_offset(col, g);
        ostride = g.HW;
      } else {
        const int n = fdiv(col, g.f_hw), pix = col - n * g.HW;
        obase = (int64_t)n * g.Cin * g.HW + pix;
        ostride = g.HW;
      }
      float* dst = g.splits > 1 ? ws : out;
#pragma unroll
      for (int mb = 0; mb < NBM; ++mb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = m0 + wm * WTM + mb * 16 + 4 * kq + i;
          dst[obase + (int64_t)m * ostride] = acc[mb][nb][i] + bbv[mb][i];
        }
    }
    return;
  }
#pragma unroll
  for (int nb = 0; nb < NBN; ++nb) {
    const int col = n0 + wn * WTN + nb * 16 + jj;
    if (col >= g.Ncol) continue;
    int64_t obase = 0;
    int64_t ostride = 0;  // output offset step per row m
    if (g.splits > 1) {
      obase = (int64_t)blockIdx.z * g.M * g.Ncol + col;
      ostride = g.Ncol;
    } else if (MODE == 0) {
      const int n = fdiv(col, g.f_howo), pix = col - n * g.HoWo;
      obase = (int64_t)n * g.Cout * g.HoWo + pix;
      ostride = g.HoWo;
    } else if (MODE == 1) {
      const int n = fdiv(col, g.f_hw), pix = col - n * g.HW;
      obase = (int64_t)n * g.Cin * g.HW + pix;
      ostride = g.HW;
    } else if (MODE == 3) {
      obase = class_pixel_offset(col, g);
      ostride = g.HW;
    } else {
      obase = col;
      ostride = g.wcols;
    }
#pragma unroll
    for (int mb = 0; mb < NBM; ++mb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm * WTM + mb * 16 + 4 * kq + i;
        if (m >= g.M) continue;
        float v = acc[mb][nb][i];
        if (g.splits > 1) {
          ws[obase + (int64_t)m * ostride] = v;
        } else if (MODE == 2) {
          if (col == g.wcols)
            out2[m] = v;
          else
            out[obase + (int64_t)m * ostride] = v;
        } else {
          if (MODE == 0 && bias) v += bbv[mb][i];
          out[obase + (int64_t)m * ostride] = v;
        }
      }
  }
}

// Many splits (a weight gradient over a long pixel sum into few outputs: the PINN's 1-32
// channel convs at 64^2 x 64 images run 2048 splits into a few hundred outputs): first
// partial sums of kRedG consecutive splits, each workgroup 64 outputs (one per lane,
// coalesced) x kRedG splits (16 per wave, all 16 loads in flight), the four waves' sums added
// in wave order.  The final pass then adds S / kRedG of these.  With one serial pass each
// thread waited for 2048 dependent loads in turn (~0.5 ms for 330 outputs).
constexpr int kRedG = 64;

__global__ __launch_bounds__(256) void igemm_reduce_partial_kernel(const float* __restrict__ ws,
                                                                   float* __restrict__ ws2,
                                                                   int64_t total, int S) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + lane;
  const int s0 = blockIdx.y * kRedG + wave * 16;
  float v = 0.f;
  if (i < total) {
    float t[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) t[j] = s0 + j < S ? ws[(int64_t)(s0 + j) * total + i] : 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) v += t[j];
  }
  red[wave][lane] = v;
  __syncthreads();
  if (wave == 0 && i < total)
    ws2[(int64_t)blockIdx.y * total + i] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

// sum of the S split-K partials (or partial sums) in split order, scattered to the output
// layout
template <int MODE>
__global__ __launch_bounds__(256) void igemm_reduce_kernel(const float* __restrict__ ws, int S,
                                                           const float* __restrict__ bias,
                                                           float* __restrict__ out,
                                                           float* __restrict__ out2, IgGeo g) {
  const int64_t total = (int64_t)g.M * g.Ncol;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int m = (int)(i / g.Ncol), col = (int)(i - (int64_t)m * g.Ncol);
    float v = ws[i];
#pragma unroll 8
    for (int z = 1; z < S; ++z) v += ws[(int64_t)z * total + i];
    if (MODE == 0) {
      const int n = fdiv(col, g.f_howo), pix = col - n * g.HoWo;
      if (bias) v += bias[m];
      out[((int64_t)n * g.Cout + m) * g.HoWo + pix] = v;
    } else if (MODE == 1) {
      const int n = fdiv(col, g.f_hw), pix = col - n * g.HW;
      out[((int64_t)n * g.Cin + m) * g.HW + pix] = v;
    } else if (MODE == 3) {
      out[class_pixel_offset(col, g) + (int64_t)m * g.HW] = v;
    } else {
      if (col == g.wcols)
        out2[m] = v;
      else
        out[(int64_t)m * g.wcols + col] = v;
    }
  }
}

int g_num_cus = 0;
int num_cus() {
  if (g_num_cus == 0) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
    g_num_cus = cus;
  }
  return g_num_cus;
}

constexpr int64_t kMaxWorkspace = 64ll << 20;  // split-K partials (bytes): their round trip stays small

void choose_tiling(IgGeo& g, int mode);

// geometry, tile and split-K choice; false when the shape is out of range
bool make_geo(int mode, int N, int Cin, int H, int W, int Cout, int KH, int KW, int sh, int sw,
              int ph, int pw, int Ho, int Wo, int bias_col, IgGeo& g) {
  if (N <= 0 || Cin <= 0 || H <= 0 || W <= 0 || Cout <= 0 || KH <= 0 || KW <= 0 || sh <= 0 ||
      sw <= 0 || ph < 0 || pw < 0 || Ho <= 0 || Wo <= 0)
    return false;
  // element offsets are 64-bit per image; the flattened GEMM indices (n, pixel) are 32-bit
  const int64_t xin = (int64_t)N * Cin * H * W, yout = (int64_t)N * Cout * Ho * Wo;
  const int64_t wsz = (int64_t)Cout * Cin * KH * KW;
  if (xin >= (1ll << 31) || yout >= (1ll << 31) || wsz >= (1ll << 31)) return false;
  g = IgGeo{};
  g.N = N; g.Cin = Cin; g.H = H; g.W = W; g.Cout = Cout; g.Ho = Ho; g.Wo = Wo;
  g.KH = KH; g.KW = KW; g.sh = sh; g.sw = sw; g.ph = ph; g.pw = pw;
  g.KHW = KH * KW; g.HW = H * W; g.HoWo = Ho * Wo;
  g.wcols = Cin * KH * KW;
  g.f_howo = make_fdiv(g.HoWo); g.f_wo = make_fdiv(Wo); g.f_hw = make_fdiv(g.HW);
  g.f_w = make_fdiv(W); g.f_khw = make_fdiv(g.KHW); g.f_kw = make_fdiv(KW);
  g.f_sh = make_fdiv(sh); g.f_sw = make_fdiv(sw);
  if (mode == 0) {
    g.M = Cout; g.Ncol = N * Ho * Wo; g.K = Cin * g.KHW;
  } else if (mode == 1) {
    g.M = Cin; g.Ncol = N * H * W; g.K = Cout * g.KHW;
  } else {
    g.M = Cout; g.Ncol = g.wcols + (bias_col ? 1 : 0); g.K = N * Ho * Wo;
  }
  g.N1 = g.Nb = N;
  g.Cc = mode == 0 ? Cin : Cout;
  g.tap = (mode == 0 || (mode == 1 && sh == 1 && sw == 1)) && KH == 3 && KW == 3 &&
          g.Cc % BK == 0;
  g.f_cc = make_fdiv(g.Cc);
  choose_tiling(g, mode);
  return true;
}

// MODE 3 geometry of input-pixel class (cy, cx) of a strided backward-data; false when the
// class holds no pixel
bool make_geo_class(const IgGeo& base, int cy, int cx, IgGeo& g) {
  g = base;
  g.tap = 0;
  g.cy = cy; g.cx = cx;
  g.Hc = (int)bpk::ceil_div(base.H - cy, base.sh);
  g.Wc = (int)bpk::ceil_div(base.W - cx, base.sw);
  if (g.Hc <= 0 || g.Wc <= 0) return false;
  g.rc0 = (cy + base.ph) % base.sh;
  g.sc0 = (cx + base.pw) % base.sw;
  g.KHc = (int)bpk::ceil_div(base.KH - g.rc0, base.sh);  // >= 1: KH >= sh (class_dgrad_ok)
  g.KWc = (int)bpk::ceil_div(base.KW - g.sc0, base.sw);
  g.f_hwc = make_fdiv(g.Hc * g.Wc); g.f_wc = make_fdiv(g.Wc);
  g.f_khwc = make_fdiv(g.KHc * g.KWc); g.f_kwc = make_fdiv(g.KWc);
  g.M = base.Cin; g.Ncol = base.N * g.Hc * g.Wc; g.K = base.Cout * g.KHc * g.KWc;
  choose_tiling(g, 3);
  return true;
}

int64_t grid_size(const IgGeo& g) {
  const int tm = g.tile == 1 ? 128 : g.tile == 2 ? 16 : 64;
  const int tn = g.tile == 1 ? 128 : g.tile == 2 ? 256 : 64;
  return bpk::ceil_div(g.M, tm) * bpk::ceil_div(g.Ncol, tn) * g.splits;
}

// strided backward-data runs class by class (MODE 3) when every class has a tap and every
// class launch still fills the chip (small images: the classes' launches of a few dozen
// workgroups each ran longer than the one MODE 1 launch with its structural zeros, e.g. the
// PINN's 32^2 stride-2 convs, 73 vs 45 us)
bool class_dgrad_ok(const IgGeo& g) {
  if (!((g.sh > 1 || g.sw > 1) && g.KH >= g.sh && g.KW >= g.sw)) return false;
  IgGeo gc;
  for (int cy = 0; cy < g.sh; ++cy)
    for (int cx = 0; cx < g.sw; ++cx)
      if (make_geo_class(g, cy, cx, gc) && grid_size(gc) < num_cus()) return false;
  return true;
}

int64_t ws_bytes(const IgGeo& g) {
  if (g.splits <= 1) return 0;
  const int64_t S2 = g.splits > kRedG ? bpk::ceil_div(g.splits, kRedG) : 0;
  return (g.splits + S2) * (int64_t)g.M * g.Ncol * 4;
}

void choose_tiling(IgGeo& g, int mode) {
  g.nchunk = (g.K + BK - 1) / BK;
  const int64_t cus = num_cus();
  // 16 x 256 tiles for M <= 16 (a conv into 1-16 channels, or the weight gradient of one:
  // no 64-row tile three-quarters idle -- the PINN's 16-channel weight gradients over 64^2 x 64
  // pixels); 128 x 128 (4x the MFMA work per staged chunk) when M, N are large; else 64 x 64
  // the weight gradient decides on its filter columns alone (the bias column would change
  // the split count, and with it the summation order: dw must not depend on bias_grad)
  const int ncol = mode == 2 ? g.wcols : g.Ncol;
  int tm, tn;
  if (g.M <= 16) {
    g.tile = 2; tm = 16; tn = 256;
  } else if (g.M >= 128 && (int64_t)g.M * ncol >= 128ll * 128 * cus / 2) {
    g.tile = 1; tm = tn = 128;
  } else {
    g.tile = 0; tm = tn = 64;
  }
  const int64_t tiles = bpk::ceil_div(g.M, tm) * bpk::ceil_div(ncol, tn);
  // split K until ~4 (64 x 64: 8) workgroups per CU for latency hiding, >= 8 chunks (128
  // of K) per split, partials within the workspace cap
  const int64_t want = (g.tile == 0 ? 8 : 4) * cus;
  int64_t splits = 1;
  if (tiles < want) splits = std::min<int64_t>(bpk::ceil_div(want, tiles), g.nchunk / 8);
  const int64_t cap = kMaxWorkspace / ((int64_t)g.M * (mode == 2 ? g.wcols + 1 : g.Ncol) * 4);
  splits = std::max<int64_t>(1, std::min<int64_t>(splits, std::min<int64_t>(cap, 4096)));
  g.chunks_per_split = (int)bpk::ceil_div(g.nchunk, splits);
  g.splits = (int)bpk::ceil_div(g.nchunk, g.chunks_per_split);
}

template <int MODE, int TM, int TN, int WMW>
void launch_tile(const IgGeo& g, const float* A0, const float* B0, const float* bias,
                 float* out, float* out2, float* wsp, hipStream_t st) {
  const dim3 grid((unsigned)bpk::ceil_div(g.Ncol, TN), (unsigned)bpk::ceil_div(g.M, TM),
                  (unsigned)g.splits);
#define BPK_IG(KH_, KW_) \
  igemm_kernel<MODE, KH_, KW_, TM, TN, WMW, false><<<grid, 256, 0, st>>>(A0, B0, bias, out, out2, wsp, g)
  if (MODE == 3)  // class sub-filters: runtime tap arithmetic (split_tap_class)
    BPK_IG(0, 0);
  else if ((MODE == 0 || MODE == 1) && g.tap)
    igemm_kernel<(MODE == 0 ? 0 : 1), 3, 3, TM, TN, WMW, true><<<grid, 256, 0, st>>>(
        A0, B0, bias, out, out2, wsp, g);
  else if (g.KH == 3 && g.KW == 3)
    BPK_IG(3, 3);
  else if (g.KH == 1 && g.KW == 1)
    BPK_IG(1, 1);
  else if (g.KH == 2 && g.KW == 2)
    BPK_IG(2, 2);
  else if (g.KH == 4 && g.KW == 4)
    BPK_IG(4, 4);
  else
    BPK_IG(0, 0);
#undef BPK_IG
}

template <int MODE>
int launch(const IgGeo& g, const float* A0, const float* B0, const float* bias, float* out,
           float* out2, float* ws, hipStream_t st) {
  float* wsp = g.splits > 1 ? ws : nullptr;
  if (g.tile == 1)
    launch_tile<MODE, 128, 128, 2>(g, A0, B0, bias, out, out2, wsp, st);
  else if (g.tile == 2)
    launch_tile<MODE, 16, 256, 1>(g, A0, B0, bias, out, out2, wsp, st);
  else
    launch_tile<MODE, 64, 64, 2>(g, A0, B0, bias, out, out2, wsp, st);
  BPK_LAUNCH_CHECK("conv2d_igemm");
  if (g.splits > 1) {
    const int64_t total = (int64_t)g.M * g.Ncol;
    const float* src = ws;
    int S = g.splits;
    if (S > kRedG) {  // partial sums behind the partials (workspace_bytes counts them)
      float* ws2 = ws + (int64_t)S * total;
      const dim3 grid((unsigned)bpk::ceil_div(total, 64), (unsigned)bpk::ceil_div(S, kRedG));
      igemm_reduce_partial_kernel<<<grid, 256, 0, st>>>(ws, ws2, total, S);
      BPK_LAUNCH_CHECK("conv2d_igemm_reduce_partial");
      src = ws2;
      S = (int)bpk::ceil_div(S, kRedG);
    }
    const unsigned blocks = (unsigned)std::min<int64_t>(bpk::ceil_div(total, 256), 4096);
    igemm_reduce_kernel<MODE><<<blocks, 256, 0, st>>>(src, S, bias, out, out2, g);
    BPK_LAUNCH_CHECK("conv2d_igemm_reduce");
  }
  return BPK_OK;
}

}  // namespace

extern "C" int64_t bpk_conv2d_igemm_workspace_bytes(int mode, int N, int Cin, int H, int W,
                                                    int Cout, int KH, int KW, int sh, int sw,
                                                    int ph, int pw, int Ho, int Wo,
                                                    int bias_grad) {
  IgGeo g;
  if (mode < 0 || mode > 2 ||
      !make_geo(mode, N, Cin, H, W, Cout, KH, KW, sh, sw, ph, pw, Ho, Wo, bias_grad, g))
    return -1;
  if (mode == 1 && class_dgrad_ok(g)) {  // the largest class's partials (classes run in turn)
    int64_t b = 0;
    IgGeo gc;
    for (int cy = 0; cy < sh; ++cy)
      for (int cx = 0; cx < sw; ++cx)
        if (make_geo_class(g, cy, cx, gc)) b = std::max(b, ws_bytes(gc));
    return b;
  }
  return ws_bytes(g);
}

extern "C" int bpk_conv2d_igemm_fwd_f32(const float* x, const float* w, const float* bias,
                                        float* y, void* wsv, int N, int Cin, int H, int W,
                                        int Cout, int KH, int KW, int sh, int sw, int ph, int pw,
                                        int Ho, int Wo, void* stream) {
  IgGeo g;
  float* ws = static_cast<float*>(wsv);
  BPK_REQUIRE(make_geo(0, N, Cin, H, W, Cout, KH, KW, sh, sw, ph, pw, Ho, Wo, 0, g),
              "conv2d_igemm_fwd: bad shape N=%d Cin=%d %dx%d Cout=%d k=%dx%d", N, Cin, H, W,
              Cout, KH, KW);
  BPK_REQUIRE(Ho == (H + 2 * ph - KH) / sh + 1 && Wo == (W + 2 * pw - KW) / sw + 1,
              "conv2d_igemm_fwd: output %dx%d inconsistent", Ho, Wo);
  BPK_REQUIRE(x && w && y && (g.splits == 1 || ws), "conv2d_igemm_fwd: null pointer");
  return launch<0>(g, w, x, bias, y, nullptr, ws, bpk::as_stream(stream));
}

extern "C" int bpk_conv2d_igemm_dgrad_f32(const float* gy, const float* w, float* gx, void* wsv,
                                          int N, int Cin, int H, int W, int Cout, int KH, int KW,
                                          int sh, int sw, int ph, int pw, int Ho, int Wo,
                                          void* stream) {
  IgGeo g;
  float* ws = static_cast<float*>(wsv);
  BPK_REQUIRE(make_geo(1, N, Cin, H, W, Cout, KH, KW, sh, sw, ph, pw, Ho, Wo, 0, g),
              "conv2d_igemm_dgrad: bad shape N=%d Cin=%d %dx%d Cout=%d k=%dx%d", N, Cin, H, W,
              Cout, KH, KW);
  BPK_REQUIRE((H + 2 * ph - KH) / sh + 1 == Ho && (W + 2 * pw - KW) / sw + 1 == Wo,
              "conv2d_igemm_dgrad: output %dx%d inconsistent with input %dx%d", Ho, Wo, H, W);
  hipStream_t st = bpk::as_stream(stream);
  if (class_dgrad_ok(g)) {
    BPK_REQUIRE(gy && w && gx, "conv2d_igemm_dgrad: null pointer");
    IgGeo gc;
    for (int cy = 0; cy < sh; ++cy)
      for (int cx = 0; cx < sw; ++cx) {
        if (!make_geo_class(g, cy, cx, gc)) continue;
        BPK_REQUIRE(gc.splits == 1 || ws, "conv2d_igemm_dgrad: null workspace");
        const int rc = launch<3>(gc, w, gy, nullptr, gx, nullptr, ws, st);
        if (rc != BPK_OK) return rc;
      }
    return BPK_OK;
  }
  BPK_REQUIRE(gy && w && gx && (g.splits == 1 || ws), "conv2d_igemm_dgrad: null pointer");
  return launch<1>(g, w, gy, nullptr, gx, nullptr, ws, st);
}

extern "C" int bpk_conv2d_igemm_wgrad_f32(const float* x, const float* gy, float* dw, float* db,
                                          void* wsv, int N, int Cin, int H, int W, int Cout,
                                          int KH, int KW, int sh, int sw, int ph, int pw, int Ho,
                                          int Wo, void* stream) {
  IgGeo g;
  float* ws = static_cast<float*>(wsv);
  BPK_REQUIRE(make_geo(2, N, Cin, H, W, Cout, KH, KW, sh, sw, ph, pw, Ho, Wo, db != nullptr, g),
              "conv2d_igemm_wgrad: bad shape N=%d Cin=%d %dx%d Cout=%d k=%dx%d", N, Cin, H, W,
              Cout, KH, KW);
  BPK_REQUIRE((H + 2 * ph - KH) / sh + 1 == Ho && (W + 2 * pw - KW) / sw + 1 == Wo,
              "conv2d_igemm_wgrad: output %dx%d inconsistent with input %dx%d", Ho, Wo, H, W);
  BPK_REQUIRE(x && gy && dw && (g.splits == 1 || ws), "conv2d_igemm_wgrad: null pointer");
  return launch<2>(g, gy, x, nullptr, dw, db, ws, bpk::as_stream(stream));
}

extern "C" int bpk_conv2d_igemm_wgrad2_f32(const float* x, const float* gy, const float* x2,
                                           const float* gy2, int N2, float* dw, float* db,
                                           void* wsv, int N, int Cin, int H, int W, int Cout,
                                           int KH, int KW, int sh, int sw, int ph, int pw,
                                           int Ho, int Wo, void* stream) {
  IgGeo g;
  float* ws = static_cast<float*>(wsv);
  BPK_REQUIRE(N > 0 && N2 >= 0, "conv2d_igemm_wgrad2: bad image counts %d, %d", N, N2);
  BPK_REQUIRE(make_geo(2, N + N2, Cin, H, W, Cout, KH, KW, sh, sw, ph, pw, Ho, Wo,
                       db != nullptr, g),
              "conv2d_igemm_wgrad2: bad shape N=%d+%d Cin=%d %dx%d Cout=%d k=%dx%d", N, N2, Cin,
              H, W, Cout, KH, KW);
  BPK_REQUIRE((H + 2 * ph - KH) / sh + 1 == Ho && (W + 2 * pw - KW) / sw + 1 == Wo,
              "conv2d_igemm_wgrad2: output %dx%d inconsistent with input %dx%d", Ho, Wo, H, W);
  BPK_REQUIRE(x && gy && dw && (N2 == 0 || (x2 && gy2)) && (g.splits == 1 || ws),
              "conv2d_igemm_wgrad2: null pointer");
  g.N1 = g.Nb = N;
  g.A1 = gy2;
  g.B1 = x2;
  return launch<2>(g, gy, x, nullptr, dw, db, ws, bpk::as_stream(stream));
}
