// Problem policies for every GEMM-shaped op of the MNIST CNN.
//
// Activations NHWC fp32, weights HWIO flattened to [25*Cin, Cout] (model.py:24-86).
// Each policy = per-thread gather info (prepA/prepB, fixed across K tiles) + 4-wide
// gathers at a wave-uniform tile base k0 (loadA/loadB, raw buffer loads: padding and
// tile edges read as 0 via the hardware range check) + fused epilogue for
// ddl::gemm_f32_kernel (gemm.h).  Tiles are BK = 32 deep and every Cin/Cout >= 32 is a
// multiple of 32, so a K tile never straddles two 5x5 taps: tap = k0 / C is uniform.
#pragma once
#include <math.h>
#include "gemm.h"

namespace ddl {

constexpr int kBK = 32;

// SAME-conv halo.  The 5x5 convolutions' inputs (p1..p3) and the pre-pool gradient maps their
// data gradients read (d2..d4) are stored with a 2-pixel zero border, [B, H+4, H+4, C]: the
// workspace is zeroed once at allocation and no kernel ever writes a border element, so an
// im2col gather is one buffer load at (per-lane voffset fixed for the whole K loop, per-K-tile
// tap offset in the instruction's SGPR soffset) — no range checks, no per-load VALU, and the
// per-row (b, y, x, valid) state collapses into one VGPR.  The image (conv1 input), d1 (read
// only by conv1's weight gradient) and p4 (fc1's input) stay unpadded.
constexpr int kHalo = 2;
constexpr int halo_w(int h) { return h + 2 * kHalo; }
// element offset of (b, y, x, c) in a [B, H, H, C] map, with or without the halo
template <int H, int C, bool PAD>
DDL_DEV int map_off(int b, int y, int x, int c) {
  if constexpr (PAD) return ((b * halo_w(H) + y + kHalo) * halo_w(H) + x + kHalo) * C + c;
  else return ((b * H + y) * H + x) * C + c;
}

// Tap skipping (gemm.h K maps).  On the 4x4 / 7x7 / 14x14 maps 51 / 31 / 16 % of the 5x5 taps of
// a SAME conv land in the zero halo.  With M enumerated position-major (all images of one pixel /
// pool window adjacent) a 32-row tile covers one or two positions, so its useful taps are a
// rectangle [ty0, ty0+nty) x [tx0, tx0+ntx) of the 5x5 grid and its K loop runs only over those
// (virtual tap t -> (ty0 + t / ntx, tx0 + t % ntx); rx = ceil(2^16 / ntx) divides exactly for t < 25).
struct TapWin {
  int ty0, nty, tx0, ntx, rx;
};
DDL_HD TapWin tap_win(int ty0, int ty1, int tx0, int tx1) {  // inclusive bounds
  const int nx = tx1 - tx0 + 1;
  return {ty0, ty1 - ty0 + 1, tx0, nx, (65536 + nx - 1) / nx};
}
DDL_DEV int tap_of(const TapWin& w, int t) {
  const int ty = (t * w.rx) >> 16;
  return (w.ty0 + ty) * 5 + w.tx0 + (t - ty * w.ntx);
}

struct LinInfo {   // linear operand: element offset of (row, k = 0 + kk), validity
  int off;
  int kk;
  bool ok;
};

// ---------------------------------------------------------------------------------------------
// conv 5x5 SAME + bias + ReLU + max-pool 2x2/2 SAME, forward (model.py:28-31 etc.)
// M enumerates conv output positions pool-window-major, in groups of 4 rows: a lane's 4
// consecutive C rows are one 2x2 pool window (q = dy*2+dx), so the epilogue pools in registers.
// Even maps (28, 14, 4): m = ((b*HP+py)*HP+px)*4 + q.  Odd maps (7, SAME pool 7->4) in
// compact order: the (HP-1)^2 full windows, then the 2(HP-1) edge windows (2 valid positions
// each, two windows per 4-row group), then the corner window (1 valid row of 4) — 52 rows
// per image instead of 64 (the padded enumeration computed 15 rows of the 64 that pool away).
// N = COUT, K = 25*CIN (k = tap*CIN + ci, tap = ky*5+kx).  Epilogue writes the pooled output
// and a 1-byte code: argmax q, or 0xFF when the max is <= 0 (ReLU inactive => no gradient).
// ---------------------------------------------------------------------------------------------
// KM: the K map (tap skipping, group-major rows) — on by default for the small maps (H <= 7);
// the eval forward also takes it for conv2 (ConvFwd<14, 32, 64, true>: its border pool windows
// skip 11 % of the taps, and at 10k images the group-major tiles keep their parallelism)
template <int H, int CIN, int COUT, bool KM = (H <= 7)>
struct ConvFwd {
  static constexpr int HP = (H + 1) / 2;
  static constexpr bool ODD = (H % 2) == 1;
  static constexpr int FULLW = ODD ? (HP - 1) * (HP - 1) : HP * HP;  // full 2x2 windows
  static constexpr int EDGEW = ODD ? HP - 1 : 0;                       // per edge
  static constexpr int GROUPS = ODD ? FULLW + EDGEW + 1 : FULLW;       // 4-row groups per image
  static constexpr int RP = 4 * GROUPS;                                // GEMM rows per image
  static constexpr bool A_KCONTIG = true;
  static constexpr bool B_KCONTIG = false;
  static_assert(CIN == 1 || CIN % kBK == 0, "tap must be tile-uniform");
  static_assert(COUT % kBK == 0, "weight columns need no range check");
  // input with halo (conv2-4; conv1 reads the image); output with halo when a conv reads it
  static constexpr bool PADIN = CIN % kBK == 0;
  static constexpr bool PADOUT = H > 4;
  static constexpr int HI = halo_w(H);
  static constexpr int rows(int batch) { return batch * RP; }
  // conv3-4: M group-major, m = (g*B + b)*4 + q (every image's pool window g adjacent), and a
  // K map over the taps that reach the image from the tile's pixels.  conv1 (K = 25: one
  // tile) and conv2 (14x14: only 16 % of the taps fall in the halo, while the group-major
  // order spreads a tile's gathers over 32 images: 26.1 -> 26.6 us) keep the image-major
  // order m = b*RP + 4g + q.
  static constexpr bool KMAP = PADIN && KM;
  using KWin = TapWin;
  int M, N, K;
  const float* __restrict__ x;     // [B,H,H,CIN] (+ halo when PADIN)
  const float* __restrict__ w;     // [25*CIN, COUT]
  const float* __restrict__ bias;  // [COUT]
  float* __restrict__ out;         // [B,HP,HP,COUT] (+ halo when PADOUT)
  uint8_t* __restrict__ code;      // [B,HP,HP,COUT] or nullptr

  struct AInfo {
    int base;   // element offset of the image
    int y, x;
    int kk;
    bool ok;
    int voff;   // PADIN: byte offset of tap (0, 0) of the row (row without a position: image 0)
  };
  using BInfo = LinInfo;

  // position (y, x) of row r (0..3) of 4-row group g of an image; false = no position
  static DDL_HD bool group_row(int g, int r, int& y, int& x) {
    if (!ODD || g < FULLW) {
      const int w = ODD ? HP - 1 : HP;
      y = 2 * (g / w) + (r >> 1);
      x = 2 * (g % w) + (r & 1);
      return true;
    }
    if (g < FULLW + EDGEW) {
      const int e = 2 * (g - FULLW) + (r >> 1), j = r & 1;
      if (e < EDGEW) { y = H - 1; x = 2 * e + j; }              // bottom edge window
      else { y = 2 * (e - EDGEW) + j; x = H - 1; }               // right edge window
      return true;
    }
    y = x = H - 1;  // corner window: row 0 only
    return r == 0;
  }

  DDL_DEV uint32_t x_bytes() const {
    return (uint32_t)((M / RP) * (PADIN ? HI * HI : H * H) * CIN) * 4u;
  }
  // image b and 4-row group g of row m
  DDL_DEV void row_bg(int m, int& b, int& g) const {
    if constexpr (KMAP) {
      const int nimg = M / RP, gb = m >> 2;
      g = gb / nimg;
      b = gb - g * nimg;
    } else {
      b = m / RP;
      g = (m - b * RP) >> 2;
    }
  }
  DDL_DEV KWin kfull() const { return tap_win(0, 4, 0, 4); }
  // input row y + ky - 2 is inside the image for ky in [2 - y, H + 1 - y]
  DDL_HD KWin kwin(int m_lo, int m_hi) const {
    const int nimg = M / RP;
    const int g0 = (m_lo >> 2) / nimg, g1 = ((m_hi - 1) >> 2) / nimg;
    int ylo = H, yhi = 0, xlo = H, xhi = 0;
    for (int g = g0; g <= g1; ++g)
      for (int q = 0; q < 4; ++q) {
        int y, xx;
        if (group_row(g, q, y, xx) && y < H && xx < H) {
          ylo = min(ylo, y); yhi = max(yhi, y);
          xlo = min(xlo, xx); xhi = max(xhi, xx);
        }
      }
    return tap_win(max(0, 2 - yhi), min(4, H + 1 - ylo), max(0, 2 - xhi), min(4, H + 1 - xlo));
  }
  DDL_HD int kvlen(const KWin& w) const { return w.nty * w.ntx * CIN; }
  DDL_DEV int kreal(const KWin& w, int kv) const {
    const int t = kv / CIN;
    return tap_of(w, t) * CIN + (kv - t * CIN);
  }

  DDL_DEV AInfo prepA(int m, int kk) const {
    AInfo a;
    int b, g;
    row_bg(m, b, g);
    a.ok = group_row(g, m & 3, a.y, a.x) && m < M && a.y < H && a.x < H;
    a.base = b * H * H * CIN;
    a.kk = kk;
    // halo coordinates of input pixel (y + ky - 2, x + kx - 2) are (y + ky, x + kx); a row
    // without a position gathers image 0 (its MFMA row is never stored)
    a.voff = (a.ok ? (b * HI + a.y) * HI * CIN + a.x * CIN + kk : kk) * 4;
    return a;
  }
  // the 16-byte gather of the halo-input forms (also the LDS-DMA source, gemm.h mainloop_dma)
  static constexpr bool DMA = PADIN;
  DDL_DEV Gather16 srcA(const AInfo& a, int k0) const {
    const int tap = k0 / CIN, cib = k0 - tap * CIN;
    const int ky = tap / 5, kx = tap - ky * 5;
    return {make_rsrc(x, x_bytes()), a.voff, ((ky * HI + kx) * CIN + cib) * 4};
  }
  DDL_DEV Gather16 srcA(const AInfo& a, int kv, const KWin& win) const {
    return srcA(a, kreal(win, kv));
  }
  DDL_DEV Gather16 srcB(const BInfo& b, int k0) const {
    return {make_rsrc(w, 25u * CIN * COUT * 4u), b.ok ? b.off * 4 : kOOB, k0 * COUT * 4};
  }
  DDL_DEV Gather16 srcB(const BInfo& b, int kv, const KWin& win) const {
    return srcB(b, kreal(win, kv));
  }
  DDL_DEV float4 loadA(const AInfo& a, int k0) const {
    const brsrc_t r = make_rsrc(x, x_bytes());
    if constexpr (PADIN) {
      const Gather16 g = srcA(a, k0);
      return bload4_so(g.r, g.voff, g.soff);
    } else {  // CIN == 1: k = tap, 4 taps per float4
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = k0 + a.kk + j;
        const int ky = k / 5, kx = k - ky * 5;
        const int iy = a.y + ky - 2, ix = a.x + kx - 2;
        const bool good =
            a.ok && k < K && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)H;
        v[j] = bload1(r, good ? (a.base + iy * H + ix) * 4 : kOOB);
      }
      return make_float4(v[0], v[1], v[2], v[3]);
    }
  }
  DDL_DEV float4 loadA(const AInfo& a, int kv, const KWin& win) const {
    return loadA(a, kreal(win, kv));
  }
  DDL_DEV BInfo prepB(int n, int kk) const { return {kk * COUT + n, kk, n < N}; }
  DDL_DEV float4 loadB(const BInfo& b, int kv, const KWin& win) const {
    return loadB(b, kreal(win, kv));
  }
  DDL_DEV float4 loadB(const BInfo& b, int k0) const {
    const brsrc_t r = make_rsrc(w, 25u * CIN * COUT * 4u);
    if constexpr (PADIN) {  // K = 25*CIN is a whole number of tiles (loop-invariant guard)
      const Gather16 g = srcB(b, k0);
      return bload4_so(g.r, g.voff, g.soff);
    } else {
      const bool good = b.ok && k0 + b.kk < K;
      return bload4(r, good ? (b.off + k0 * COUT) * 4 : kOOB);
    }
  }
  // pooled output (halo layout when a conv reads it) and its pool code (no halo)
  DDL_DEV void store_pooled(int b, int py, int px, int n, float best, int arg) const {
    out[map_off<HP, COUT, PADOUT>(b, py, px, n)] = best > 0.f ? best : 0.f;
    if (code)
      code[((size_t)(b * HP + py) * HP + px) * COUT + n] = best > 0.f ? (uint8_t)arg : (uint8_t)0xFF;
  }
  // max-pool + bias + ReLU of the rows [lo, hi) of the group as one window whose rows have
  // pool codes q(r); writes pooled output (py, px)
  DDL_DEV void pool_out(int b, int py, int px, int n, float bb, const float* v, const int* qs,
                        int cnt) const {
    float best = -INFINITY;
    int arg = 0;
    for (int i = 0; i < cnt; ++i) {
      const float val = v[i] + bb;
      if (val > best) { best = val; arg = qs[i]; }
    }
    store_pooled(b, py, px, n, best, arg);
  }
  DDL_DEV void epi(int m0, int n, f32x4 v) const {
    const float bb = bias[n];
    int b, g;
    row_bg(m0, b, g);
    const float vv[4] = {v[0], v[1], v[2], v[3]};
    if (!ODD || g < FULLW) {
      const int w = ODD ? HP - 1 : HP;
      const int py = g / w, px = g % w;
      float best = -INFINITY;
      int arg = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int y = 2 * py + (q >> 1), xx = 2 * px + (q & 1);
        if (y < H && xx < H) {
          const float val = vv[q] + bb;
          if (val > best) { best = val; arg = q; }
        }
      }
      store_pooled(b, py, px, n, best, arg);
    } else if (g < FULLW + EDGEW) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int e = 2 * (g - FULLW) + h;
        const bool bottom = e < EDGEW;
        const int qs[2] = {0, bottom ? 1 : 2};  // (dy, dx) = (0, j) bottom, (j, 0) right
        pool_out(b, bottom ? HP - 1 : e - EDGEW, bottom ? e : HP - 1, n, bb, vv + 2 * h, qs, 2);
      }
    } else {
      const int qs[1] = {0};
      pool_out(b, HP - 1, HP - 1, n, bb, vv, qs, 1);
    }
  }
};

// Scatter one pooled-output gradient g into the 2x2 window of the pre-pool gradient:
// dpre[b, 2y+dy, 2x+dx, c] = (code == dy*2+dx) ? g : 0  (ReLU folded in via code 0xFF).
// dpre has the halo layout when a data gradient reads it (HPREV < 28: d2..d4).
template <int HPREV, int C>
DDL_DEV void pool_bwd_scatter(float* __restrict__ dpre, int b, int y, int x, int c, uint8_t code,
                              float g) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int yy = 2 * y + (q >> 1), xx = 2 * x + (q & 1);
    if (yy < HPREV && xx < HPREV)
      dpre[map_off<HPREV, C, (HPREV < 28)>(b, yy, xx, c)] = (code == q) ? g : 0.f;
  }
}

// ---------------------------------------------------------------------------------------------
// conv data gradient (Conv2DBackpropInput) fused with the previous
// layer's MaxPoolGrad + ReluGrad (B7/B8): M = B*H*H (b,y,x), N = CIN, K = 25*COUT
// (k = tap*COUT + co).  dX[b,y,x,ci] = sum dpre[b, y-ky+2, x-kx+2, co] * W[ky,kx,ci,co];
// the epilogue scatters dX through the previous pool's codes into dpre_prev.
// ---------------------------------------------------------------------------------------------
template <int H, int CIN, int COUT, int HPREV>
struct ConvDgrad {
  static constexpr bool A_KCONTIG = true;
  static constexpr bool B_KCONTIG = true;
  static_assert(COUT % kBK == 0, "tap must be tile-uniform");
  static constexpr int HI = halo_w(H);
  // conv3-4 (H <= 7): M pixel-major, m = (y*H + x)*B + b, and a K map over the taps whose
  // output-gradient pixel (y - ky + 2, x - kx + 2) is inside the map for some row of the tile.
  // conv2 (14x14, 16 % of the taps in the halo) keeps m = (b*H + y)*H + x: the pixel-major
  // order made its dual launch 50.6 -> 58.4 us (gathers spread over 32 images per tile).
  static constexpr bool KMAP = H <= 7;
  using KWin = TapWin;
  int M, N, K;
  const float* __restrict__ dpre;        // [B,H+4,H+4,COUT] (halo)
  const float* __restrict__ w;           // [25*CIN, COUT]
  const uint8_t* __restrict__ code_prev; // [B,H,H,CIN]
  float* __restrict__ dpre_prev;         // [B,HPREV,HPREV,CIN] (+ halo if HPREV < 28)

  struct AInfo {
    int voff;  // byte offset of halo pixel (y, x) + kk (row m >= M: image 0's)
  };
  using BInfo = LinInfo;

  // image and pixel of row m
  DDL_DEV void row_pix(int m, int& b, int& y, int& x) const {
    if constexpr (KMAP) {
      const int nimg = M / (H * H);
      const int pos = m / nimg;
      b = m - pos * nimg;
      y = pos / H;
      x = pos - y * H;
    } else {
      x = m % H;
      const int t = m / H;
      y = t % H;
      b = t / H;
    }
  }
  DDL_DEV KWin kfull() const { return tap_win(0, 4, 0, 4); }
  // oy = y - ky + 2 in [0, H) for ky in [y + 3 - H, y + 2]
  DDL_HD KWin kwin(int m_lo, int m_hi) const {
    const int nimg = M / (H * H);
    const int p0 = m_lo / nimg, p1 = (m_hi - 1) / nimg;
    const int ylo = p0 / H, yhi = p1 / H;
    const int xlo = ylo == yhi ? p0 - ylo * H : 0, xhi = ylo == yhi ? p1 - yhi * H : H - 1;
    return tap_win(max(0, ylo + 3 - H), min(4, yhi + 2), max(0, xlo + 3 - H), min(4, xhi + 2));
  }
  DDL_HD int kvlen(const KWin& w) const { return w.nty * w.ntx * COUT; }
  DDL_DEV int kreal(const KWin& w, int kv) const {
    const int t = kv / COUT;
    return tap_of(w, t) * COUT + (kv - t * COUT);
  }
  DDL_DEV AInfo prepA(int m, int kk) const {
    int b, y, x;
    row_pix(m < M ? m : 0, b, y, x);
    return {(((b * HI + y) * HI + x) * COUT + kk) * 4};
  }
  // output gradient at (y - ky + 2, x - kx + 2) = halo pixel (y + 4 - ky, x + 4 - kx); the
  // 16-byte gathers are the LDS-DMA sources of the 16x16x4 tile (CFG_MF16; on the 32x32x2 tile
  // the data gradients stage through registers: DMA there measured slower inside the dual)
  DDL_DEV Gather16 srcA(const AInfo& a, int k0) const {
    const int tap = k0 / COUT, cob = k0 - tap * COUT;
    const int ky = tap / 5, kx = tap - ky * 5;
    return {make_rsrc(dpre, (uint32_t)(M / (H * H)) * HI * HI * COUT * 4u), a.voff,
            (((2 * kHalo - ky) * HI + (2 * kHalo - kx)) * COUT + cob) * 4};
  }
  DDL_DEV BInfo prepB(int n, int kk) const { return {n * COUT + kk, kk, n < N}; }
  DDL_DEV Gather16 srcB(const BInfo& b, int k0) const {
    const int tap = k0 / COUT, cob = k0 - tap * COUT;
    return {make_rsrc(w, 25u * CIN * COUT * 4u), b.ok ? b.off * 4 : kOOB,
            (tap * CIN * COUT + cob) * 4};
  }
  DDL_DEV Gather16 srcA(const AInfo& a, int kv, const KWin& win) const {
    return srcA(a, kreal(win, kv));
  }
  DDL_DEV Gather16 srcB(const BInfo& b, int kv, const KWin& win) const {
    return srcB(b, kreal(win, kv));
  }
  DDL_DEV float4 loadA(const AInfo& a, int k0) const {
    const Gather16 g = srcA(a, k0);
    return bload4_so(g.r, g.voff, g.soff);
  }
  DDL_DEV float4 loadB(const BInfo& b, int k0) const {
    const Gather16 g = srcB(b, k0);
    return bload4_so(g.r, g.voff, g.soff);
  }
  DDL_DEV float4 loadA(const AInfo& a, int kv, const KWin& win) const {
    return loadA(a, kreal(win, kv));
  }
  DDL_DEV float4 loadB(const BInfo& b, int kv, const KWin& win) const {
    return loadB(b, kreal(win, kv));
  }
  DDL_DEV void epi(int m0, int n, f32x4 v) const {
    // one row decode per group of 4 (its runtime division by the image count), then a carry:
    // the pixel-major K-map order puts 4 images of one pixel in a group (wrapping at most once)
    int b, y, xx;
    row_pix(m0 < M ? m0 : 0, b, y, xx);
    const int nimg = M / (H * H);
    uint8_t cd[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {  // every code load issued before the first store
      int br = b, yr = y, xr = xx;
      step_row(br, yr, xr, r, nimg);
      cd[r] = m0 + r < M ? code_prev[((size_t)(br * H + yr) * H + xr) * CIN + n] : 0;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (m0 + r >= M) break;
      int br = b, yr = y, xr = xx;
      step_row(br, yr, xr, r, nimg);
      pool_bwd_scatter<HPREV, CIN>(dpre_prev, br, yr, xr, n, cd[r], v[r]);
    }
  }
  // row m, columns n0 .. n0 + 3 (the tile epilogue's quad transpose, gemm.h HasEpiT): one
  // 4-byte load of the four codes, then one 16-byte store per pool-window position
  DDL_DEV void epi_t(int m, int n0, float4 v) const {
    int b, y, xx;
    row_pix(m, b, y, xx);
    const size_t px = (size_t)(b * H + y) * H + xx;
    const uint32_t cw = *reinterpret_cast<const uint32_t*>(code_prev + px * CIN + n0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int yy = 2 * y + (q >> 1), x2 = 2 * xx + (q & 1);
      if (yy >= HPREV || x2 >= HPREV) continue;
      const uint32_t qq = (uint32_t)q;
      float4 o;
      o.x = (cw & 0xFFu) == qq ? v.x : 0.f;
      o.y = ((cw >> 8) & 0xFFu) == qq ? v.y : 0.f;
      o.z = ((cw >> 16) & 0xFFu) == qq ? v.z : 0.f;
      o.w = (cw >> 24) == qq ? v.w : 0.f;
      *reinterpret_cast<float4*>(dpre_prev + map_off<HPREV, CIN, (HPREV < 28)>(b, yy, x2, n0)) = o;
    }
  }
  // (b, y, x) of row m0 + r from that of m0 (r < 4)
  DDL_DEV void step_row(int& b, int& y, int& x, int r, int nimg) const {
    if constexpr (KMAP) {  // m = (y*H + x)*nimg + b: image fastest
      b += r;
      while (b >= nimg) {  // (once for batches >= 4)
        b -= nimg;
        if (++x == H) { x = 0; ++y; }
      }
    } else {  // m = (b*H + y)*H + x: pixel fastest
      x += r;
      if (x >= H) {
        x -= H;
        if (++y == H) { y = 0; ++b; }
      }
    }
  }
};

// ---------------------------------------------------------------------------------------------
// conv weight gradient (Conv2DBackpropFilter + bias grad, B10/B8): dW_aug[25*CIN+1, COUT].
// M = 25*CIN + 1 (row 25*CIN is a row of ones -> db), N = COUT.
// K enumerates positions row by row with a row width WP >= H: k = (b*H + y)*WP + x,
// K = B*H*WP (columns x >= H read 0).  The row index of a K tile's first element comes from
// the tile base (uniform: scalar unit) and a thread's (row, column) offset inside the tile is
// fixed (prepA/prepB), so a gather needs a column carry and a row wrap (compare-selects)
// instead of the per-element position decode k / H, k % H, k / (H*H) (~20 VALU per gather).
// WP = H (exact rows) is the default; WP = next power of two (no carry, but WP/H more MFMA
// work on the H = 7, 14, 28 layers) measured 2 us/step slower (kWgradRowPad).
// A[m=(tap,ci)][k=(b,y,x)] = x[b, y+ky-2, x+kx-2, ci] (ci contiguous => MN-contiguous),
// B[n=co][k] = dpre[((b*H + y)*H + x)*COUT + co] (MN-contiguous).
// ---------------------------------------------------------------------------------------------
constexpr int wgrad_wp(int h) { return h <= 4 ? 4 : h <= 8 ? 8 : h <= 16 ? 16 : 32; }
constexpr int ilog2(int v) { return v <= 1 ? 0 : 1 + ilog2(v / 2); }

// WP: row width of the K enumeration — wgrad_wp(H) (padded to a power of two) or H (exact;
// a thread's column then may wrap into the next row, one compare-select per gather)
template <int H, int CIN, int COUT, int WP = wgrad_wp(H)>
struct ConvWgrad {
  static constexpr bool A_KCONTIG = false;
  static constexpr bool B_KCONTIG = false;
  static constexpr int KW = 25 * CIN;
  // x = p1..p3 and dpre = d2..d4 carry the halo; conv1's image and d1 do not
  static constexpr bool PADX = CIN >= kBK;
  static constexpr bool PADD = H < 28;
  static constexpr int HI = halo_w(H);
  static_assert(WP >= H, "row width below the map width");
  // tiles start at multiples of BK (16 or 32): a thread's column offset never carries into
  // the next row when WP divides 16 or is a multiple of 32
  static constexpr bool XWRAP = !(16 % WP == 0 || WP % 32 == 0);
  // rows a thread's offset can add to the tile's first row, plus a column carry
  static_assert((H & (H - 1)) == 0 || 32 / WP + 1 < H, "one row wrap at most");
  static constexpr int padded_k(int batch) { return batch * H * WP; }
  int M, N, K;                     // K = padded_k(batch)
  const float* __restrict__ x;     // [B,H,H,CIN]
  const float* __restrict__ dpre;  // [B,H,H,COUT]
  float* __restrict__ gw;          // [25*CIN, COUT]
  float* __restrict__ gb;          // [COUT]

  struct Pos {  // a thread's fixed position offset inside every K tile
    int dr;     // rows past the tile's first row
    int xk;     // column offset (added to the tile's first column)
  };
  struct AInfo {
    int m;      // first of the 4 rows
    int dy, dx; // tap offsets of row m (vector path)
    int ci;
    Pos p;
    bool vec;   // all 4 rows are weight rows of one tap
  };
  struct BInfo {
    int n;
    Pos p;
    bool ok;
  };

  static DDL_DEV Pos pos(int kk) { return {kk / WP, kk % WP}; }
  // (b, y, x, valid) of a thread's element in the K tile at k0 (a multiple of BK); the
  // divisions by the constants WP, H of the uniform k0 run on the scalar unit
  DDL_DEV void decode(int k0, const Pos& p, int& b, int& y, int& xx, bool& ok) const {
    const int r0 = k0 / WP;
    int dr = p.dr;
    xx = k0 % WP + p.xk;
    if constexpr (XWRAP) {
      const bool cx = xx >= WP;
      xx -= cx ? WP : 0;
      dr += cx ? 1 : 0;
    }
    int yy = r0 % H + dr;
    b = r0 / H;
    if constexpr ((H & (H - 1)) == 0) {
      b += yy >> ilog2(H);
      yy &= H - 1;
    } else {
      const bool wrap = yy >= H;
      yy -= wrap ? H : 0;
      b += wrap ? 1 : 0;
    }
    y = yy;
    ok = xx < H && (r0 + dr) * WP < K;
  }

  DDL_DEV AInfo prepA(int m, int kk) const {
    AInfo a;
    a.m = m;
    const int tap = m / CIN;
    a.ci = m - tap * CIN;
    a.dy = tap / 5 - 2;
    a.dx = tap % 5 - 2;
    a.p = pos(kk);
    a.vec = (CIN % 4 == 0) && (m + 3 < KW);
    return a;
  }
  DDL_DEV float4 loadA(const AInfo& a, int k0) const {
    const int nimg = K / (WP * H);
    const brsrc_t r = make_rsrc(x, (uint32_t)nimg * (PADX ? HI * HI : H * H) * CIN * 4u);
    int b, y, xx;
    bool kin;
    decode(k0, a.p, b, y, xx, kin);
    if constexpr (CIN % 4 == 0) {
      // KW = 25*CIN is a multiple of 4, so a 4-row group is either all weight rows (one
      // 16-B gather) or starts at row >= KW: the ones row (db) then zeros.  Branch-free.
      const int iy = y + a.dy, ix = xx + a.dx;
      bool good = a.vec && kin;
      if constexpr (!PADX) good = good && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)H;
      float4 v = bload4(r, good ? map_off<H, CIN, PADX>(b, iy, ix, a.ci) * 4 : kOOB);
      if (a.m == KW) v.x = kin ? 1.f : 0.f;
      return v;
    }
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int e = a.m + j;
      const int tap = e / CIN, ci = e - tap * CIN;
      const int iy = y + tap / 5 - 2, ix = xx + tap % 5 - 2;
      const bool good = kin && e < KW && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)H;
      const float val = bload1(r, good ? (((b * H + iy) * H + ix) * CIN + ci) * 4 : kOOB);
      v[j] = (e == KW && kin) ? 1.f : val;
    }
    return make_float4(v[0], v[1], v[2], v[3]);
  }
  DDL_DEV BInfo prepB(int n, int kk) const { return {n, pos(kk), n < N}; }
  DDL_DEV float4 loadB(const BInfo& bi, int k0) const {
    const int nimg = K / (WP * H);
    const brsrc_t r = make_rsrc(dpre, (uint32_t)nimg * (PADD ? HI * HI : H * H) * COUT * 4u);
    int b, y, xx;
    bool kin;
    decode(k0, bi.p, b, y, xx, kin);
    const bool good = bi.ok && kin;
    return bload4(r, good ? map_off<H, COUT, PADD>(b, y, xx, bi.n) * 4 : kOOB);
  }
  DDL_DEV void epi(int m0, int n, f32x4 v) const {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + r;
      if (m < KW) gw[(size_t)m * COUT + n] = v[r];
      else if (m == KW) gb[n] = v[r];
    }
  }
};

// ---------------------------------------------------------------------------------------------
// conv weight gradient of conv2-4 (inputs and output gradients in the halo layout), K
// enumerated batch-minor: k = pos * NB + b, pos = y*H + x, NB = max(B, 32) images per position
// (b >= B reads 0).  A K tile (<= 32 deep) then spans at most two positions, so a slot's image
// and pixel are the tile's scalar (b0, pos0) plus one per-lane carry, and its pixel offset is
// one of two scalars: a gather costs an add, a compare, three selects and a multiply-add, shared
// between the A and B slots of the same k, instead of a per-load (b, y, x) decode with column,
// row and image carries (~17 VALU per load in the row-major enumeration of ConvWgrad).
// A[m=(tap,ci)][k] = x[b, y+ky-2, x+kx-2, ci] = halo x[b, y+ky, x+kx, ci],
// B[n=co][k] = halo dpre[b, y+2, x+2, co]; both MN-contiguous (ci / co innermost).
// ---------------------------------------------------------------------------------------------
template <int H, int CIN, int COUT>
struct ConvWgradBM {
  static constexpr bool A_KCONTIG = false;
  static constexpr bool B_KCONTIG = false;
  static constexpr int KW = 25 * CIN;
  static constexpr int HI = halo_w(H);
  static_assert(CIN % kBK == 0 && COUT % 4 == 0, "halo-layout conv layers only");
  static constexpr int nb(int batch) { return batch < kBK ? kBK : batch; }
  static constexpr int k_of(int batch) { return H * H * nb(batch); }
  // floor(2^32 / NB) + 1: k0 / NB == umulhi(k0, mag) exactly while k0 * NB < 2^32
  static uint32_t magic(int nbv) { return (uint32_t)((1ull << 32) / (uint64_t)nbv) + 1u; }
  // K map: a tile's rows are (one or two) taps; only the output positions whose input pixel
  // (y + ky - 2, x + kx - 2) is inside the image contribute.  The window is a rectangle of
  // positions [y0, y0+ny) x [x0, x0+nx); virtual position v -> (y0 + v / nx, x0 + v % nx)
  // (rx = ceil(2^16 / nx): exact for v <= 196).
  static constexpr bool KMAP = true;
  struct KWin {
    int y0, ny, x0, nx, rx;
  };
  int M, N, K;                     // K = k_of(B)
  const float* __restrict__ x;     // [B,H+4,H+4,CIN]
  const float* __restrict__ dpre;  // [B,H+4,H+4,COUT]
  float* __restrict__ gw;          // [25*CIN, COUT]
  float* __restrict__ gb;          // [COUT]
  int nimg;                        // B
  int NB;                          // nb(B)
  uint32_t mag;                    // magic(NB)

  struct AInfo {
    int m;       // first of the 4 rows
    int tapoff;  // (ky*HI + kx)*CIN + ci of row m
    int kk;
    bool vec;    // all 4 rows are weight rows of one tap
  };
  struct BInfo {
    int n;
    int kk;
    bool ok;
  };
  static DDL_HD KWin pos_win(int y0, int y1, int x0, int x1) {  // inclusive bounds
    const int nx = x1 - x0 + 1;
    return {y0, y1 - y0 + 1, x0, nx, (65536 + nx - 1) / nx};
  }
  DDL_HD KWin kfull() const { return pos_win(0, H - 1, 0, H - 1); }
  DDL_HD KWin kwin(int m_lo, int m_hi) const {
    if (m_hi > KW) return kfull();  // the ones row (bias gradient) sums every position
    const int t0 = m_lo / CIN, t1 = (m_hi - 1) / CIN;
    const int kylo = t0 / 5, kyhi = t1 / 5;
    const int kxlo = kylo == kyhi ? t0 - kylo * 5 : 0, kxhi = kylo == kyhi ? t1 - kyhi * 5 : 4;
    // input row y + ky - 2 is inside the image for y in [2 - ky, H + 1 - ky]
    return pos_win(max(0, 2 - kyhi), min(H - 1, H + 1 - kylo), max(0, 2 - kxhi),
                   min(H - 1, H + 1 - kxlo));
  }
  DDL_HD int kvlen(const KWin& w) const { return w.ny * w.nx * NB; }
  static DDL_DEV void vpos(const KWin& w, int v, int& y, int& xx) {
    const int r = (v * w.rx) >> 16;
    y = w.y0 + r;
    xx = w.x0 + v - r * w.nx;
  }
  // image b and position carry w of virtual slot k0 + kk; kin = inside the window's K range
  // and b < B.  Bitwise logic only: a short-circuit && becomes an exec-mask branch per load.
  DDL_DEV void slot(int k0, int kk, int nvp, int& b, bool& w, bool& kin) const {
    const int pos0 = (int)__umulhi((uint32_t)k0, mag);
    const bool c0 = pos0 < nvp, c1 = pos0 + 1 < nvp;  // scalar
    const int t = k0 - pos0 * NB + kk;
    w = t >= NB;
    b = t - (w ? NB : 0);
    kin = (w ? c1 : c0) & (b < nimg);
  }
  DDL_DEV AInfo prepA(int m, int kk) const {
    const int tap = m / CIN, ci = m - tap * CIN;
    const int ky = tap / 5, kx = tap - ky * 5;
    return {m, (ky * HI + kx) * CIN + ci, kk, m + 3 < KW};
  }
  // the 16-byte gathers (also the LDS-DMA sources of the 16x16x4 tile, CFG_MF16); A's ones row
  // (the bias gradient) is not in memory: the group starting at row KW gathers zeros and its .x
  // is patched — in registers by loadA, in the LDS image by the DMA loop (ones_group /
  // ones_value).  (LDS-DMA on the 32x32x2 tile measured neutral: registers staging kept.)
  DDL_DEV Gather16 srcA(const AInfo& a, int k0, const KWin& win) const {
    const int pos0 = (int)__umulhi((uint32_t)k0, mag);
    int y0, x0, y1, x1;
    vpos(win, pos0, y0, x0);
    vpos(win, pos0 + 1, y1, x1);
    const int p0 = (y0 * HI + x0) * CIN, p1 = (y1 * HI + x1) * CIN;  // scalar
    int b;
    bool w, kin;
    slot(k0, a.kk, win.ny * win.nx, b, w, kin);
    // the offset is computed unconditionally and pushed out of range by an add (a select of
    // the whole address lets hipcc branch around its computation per load)
    const int off = ((int)__umul24(b, HI * HI * CIN) + (w ? p1 : p0) + a.tapoff) * 4;
    return {make_rsrc(x, (uint32_t)nimg * HI * HI * CIN * 4u), off + ((a.vec & kin) ? 0 : kOOB),
            0};
  }
  DDL_DEV bool ones_group(const AInfo& a) const { return a.m == KW; }
  DDL_DEV float ones_value(const AInfo& a, int k0, const KWin& win) const {
    int b;
    bool w, kin;
    slot(k0, a.kk, win.ny * win.nx, b, w, kin);
    return kin ? 1.f : 0.f;
  }
  DDL_DEV float4 loadA(const AInfo& a, int k0, const KWin& win) const {
    const Gather16 g = srcA(a, k0, win);
    float4 v = bload4(g.r, g.voff);
    if (a.m == KW) v.x = ones_value(a, k0, win);  // ones row: bias gradient
    return v;
  }
  DDL_DEV BInfo prepB(int n, int kk) const { return {n, kk, n < N}; }
  DDL_DEV Gather16 srcB(const BInfo& bi, int k0, const KWin& win) const {
    const int pos0 = (int)__umulhi((uint32_t)k0, mag);
    int y0, x0, y1, x1;
    vpos(win, pos0, y0, x0);
    vpos(win, pos0 + 1, y1, x1);
    const int q0 = ((y0 + kHalo) * HI + x0 + kHalo) * COUT;
    const int q1 = ((y1 + kHalo) * HI + x1 + kHalo) * COUT;
    int b;
    bool w, kin;
    slot(k0, bi.kk, win.ny * win.nx, b, w, kin);
    const int off = ((int)__umul24(b, HI * HI * COUT) + (w ? q1 : q0) + bi.n) * 4;
    return {make_rsrc(dpre, (uint32_t)nimg * HI * HI * COUT * 4u),
            off + ((bi.ok & kin) ? 0 : kOOB), 0};
  }
  DDL_DEV float4 loadB(const BInfo& bi, int k0, const KWin& win) const {
    const Gather16 g = srcB(bi, k0, win);
    return bload4(g.r, g.voff);
  }
  DDL_DEV void epi(int m0, int n, f32x4 v) const {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + r;
      if (m < KW) gw[(size_t)m * COUT + n] = v[r];
      else if (m == KW) gb[n] = v[r];
    }
  }
};

// The four conv weight-gradient GEMMs (conv4 .. conv1); conv1 (image input, d1 without halo)
// keeps the row-major enumeration with exact rows.
using WgradConv4 = ConvWgradBM<4, 128, 256>;
using WgradConv3 = ConvWgradBM<7, 64, 128>;
using WgradConv2 = ConvWgradBM<14, 32, 64>;
using WgradConv1 = ConvWgrad<28, 1, 32, 28>;

// A ConvWgrad whose reduce epilogue also runs the optimizer (Adam, TF1 form, common.h adam1)
// on every element it has just summed: with one worker the update of conv1 (the step's last
// gradients) needs no launch of its own (gemm.h splitk_wide_reduce_tail).  The gradient is
// still stored.  w/m/v: conv1's weight [25*CIN*COUT] and bias [COUT] parameter / Adam-state
// spans, in the same layout as gw / gb.
template <class P>
struct WgradAdam : P {
  float *w_w, *w_m, *w_v;  // weight span
  float *b_w, *b_m, *b_v;  // bias span
  float lr_t, c1, c2, eps, scale;
  DDL_DEV void epi(int m0, int n, f32x4 v) const {
    constexpr int KW = P::KW;  // gw is [KW, N] (N = COUT)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + r;
      float *pw, *pm, *pv;
      size_t i;
      if (m < KW) {
        i = (size_t)m * this->N + n; pw = w_w; pm = w_m; pv = w_v;
        this->gw[i] = v[r];
      } else if (m == KW) {
        i = (size_t)n; pw = b_w; pm = b_m; pv = b_v;
        this->gb[i] = v[r];
      } else {
        continue;
      }
      float W = pw[i], M = pm[i], V = pv[i];
      adam1(W, v[r] * scale, M, V, lr_t, c1, c2, eps);
      pw[i] = W; pm[i] = M; pv[i] = V;
    }
  }
};

// ---------------------------------------------------------------------------------------------
// fully connected forward (model.py:70 fc1: +b, ReLU, dropout; :79,82 fc2: +b, dropout)
// M = B, N = NOUT, K = KIN.  Dropout key derived on device from *seed (graph-replayable),
// or from seed_v when no seed word is given (the native step runner: no seed-upload kernel).
// ---------------------------------------------------------------------------------------------
template <bool RELU>
struct FcFwd {
  static constexpr bool A_KCONTIG = true;
  static constexpr bool B_KCONTIG = false;
  int M, N, K;
  const float* __restrict__ in;    // [B,KIN]
  const float* __restrict__ w;     // [KIN,NOUT]
  const float* __restrict__ bias;  // [NOUT]
  float* __restrict__ out;         // [B,NOUT]
  const uint32_t* __restrict__ seed;
  uint32_t layer;
  uint32_t thr24;                  // 0 => no dropout
  float inv_keep;
  uint32_t seed_v;                 // dropout seed by value when `seed` is null

  using AInfo = LinInfo;
  using BInfo = LinInfo;
  DDL_DEV AInfo prepA(int m, int kk) const { return {m * K + kk, kk, m < M}; }
  DDL_DEV float4 loadA(const AInfo& a, int k0) const {
    const brsrc_t r = make_rsrc(in, (uint32_t)M * K * 4u);
    return bload4(r, a.ok && k0 + a.kk < K ? (a.off + k0) * 4 : kOOB);
  }
  DDL_DEV BInfo prepB(int n, int kk) const { return {kk * N + n, kk, n < N}; }
  DDL_DEV float4 loadB(const BInfo& b, int k0) const {
    const brsrc_t r = make_rsrc(w, (uint32_t)K * N * 4u);
    return bload4(r, b.ok && k0 + b.kk < K ? (b.off + k0 * N) * 4 : kOOB);
  }
  DDL_DEV void epi(int m0, int n, f32x4 v) const {
    const float bb = bias[n];
    uint32_t key = 0;
    if (thr24) key = ddl_mix32((seed ? *seed : seed_v) + layer * 0x9E3779B9u);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + r;
      if (m >= M) break;
      float val = v[r] + bb;
      if (RELU) val = val > 0.f ? val : 0.f;
      const uint32_t idx = (uint32_t)(m * N + n);
      if (thr24) val = ddl_keep(key, idx, thr24) ? val * inv_keep : 0.f;
      out[idx] = val;
    }
  }
};

// fc data gradient dX = dY W^T (B2/B4/B6).  A = dY [B,NOUT] (K-contig), B[n=i][k=o] =
// W[i][o] (K-contig).  Epilogue variants:
//   FcDgradAct  : previous layer was ReLU+dropout (fc1): dpre = hpost > 0 ? g/keep : 0
//   FcDgradPool : previous layer was the conv4 max-pool (flatten of [B,2,2,256])
struct FcDgradBase {
  static constexpr bool A_KCONTIG = true;
  static constexpr bool B_KCONTIG = true;
  int M, N, K;
  const float* __restrict__ dy;     // [B,K]
  const float* __restrict__ w;      // [N,K]
  using AInfo = LinInfo;
  using BInfo = LinInfo;
  DDL_DEV AInfo prepA(int m, int kk) const { return {m * K + kk, kk, m < M}; }
  DDL_DEV float4 loadA(const AInfo& a, int k0) const {
    const brsrc_t r = make_rsrc(dy, (uint32_t)M * K * 4u);
    return bload4(r, a.ok && k0 + a.kk < K ? (a.off + k0) * 4 : kOOB);
  }
  DDL_DEV BInfo prepB(int n, int kk) const { return {n * K + kk, kk, n < N}; }
  DDL_DEV float4 loadB(const BInfo& b, int k0) const {
    const brsrc_t r = make_rsrc(w, (uint32_t)N * K * 4u);
    return bload4(r, b.ok && k0 + b.kk < K ? (b.off + k0) * 4 : kOOB);
  }
};

struct FcDgradAct : FcDgradBase {
  const float* __restrict__ hpost;  // [B,N] post ReLU+dropout activation
  float inv_keep;
  float* __restrict__ dx;           // [B,N]
  DDL_DEV void epi(int m0, int n, f32x4 v) const {
    const int M = this->M, N = this->N;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + r;
      if (m >= M) break;
      const size_t o = (size_t)m * N + n;
      dx[o] = hpost[o] > 0.f ? v[r] * inv_keep : 0.f;
    }
  }
  // row m, columns n0 .. n0 + 3 (gemm.h HasEpiT): 16-byte load and store
  DDL_DEV void epi_t(int m, int n0, float4 v) const {
    const size_t o = (size_t)m * this->N + n0;
    const float4 h = *reinterpret_cast<const float4*>(hpost + o);
    float4 d;
    d.x = h.x > 0.f ? v.x * inv_keep : 0.f;
    d.y = h.y > 0.f ? v.y * inv_keep : 0.f;
    d.z = h.z > 0.f ? v.z * inv_keep : 0.f;
    d.w = h.w > 0.f ? v.w * inv_keep : 0.f;
    *reinterpret_cast<float4*>(dx + o) = d;
  }
};

template <int HP, int C>
struct FcDgradPool : FcDgradBase {
  static constexpr int HPREV = 2 * HP;
  const uint8_t* __restrict__ code;    // [B,HP,HP,C] == [B,N]
  float* __restrict__ dpre_prev;       // [B,HPREV,HPREV,C] + halo
  DDL_DEV void epi(int m0, int n, f32x4 v) const {
    const int M = this->M, N = this->N;
    const int c = n % C;
    const int t = n / C;
    const int px = t % HP, py = t / HP;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + r;
      if (m >= M) break;
      pool_bwd_scatter<HPREV, C>(dpre_prev, m, py, px, c, code[(size_t)m * N + n], v[r]);
    }
  }
  // row m, columns n0 .. n0 + 3 (gemm.h HasEpiT): one 4-byte code load, four 16-byte stores
  DDL_DEV void epi_t(int m, int n0, float4 v) const {
    const int c0 = n0 % C, t = n0 / C;
    const int px = t % HP, py = t / HP;
    const uint32_t cw = *reinterpret_cast<const uint32_t*>(code + (size_t)m * this->N + n0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t qq = (uint32_t)q;
      float4 o;
      o.x = (cw & 0xFFu) == qq ? v.x : 0.f;
      o.y = ((cw >> 8) & 0xFFu) == qq ? v.y : 0.f;
      o.z = ((cw >> 16) & 0xFFu) == qq ? v.z : 0.f;
      o.w = (cw >> 24) == qq ? v.w : 0.f;
      *reinterpret_cast<float4*>(
          dpre_prev + map_off<HPREV, C, true>(m, 2 * py + (q >> 1), 2 * px + (q & 1), c0)) = o;
    }
  }
};

// fc weight gradient dW_aug[KIN+1, NOUT] = [X;1]^T dY (B2/B4/B6): M = KIN+1, N = NOUT, K = B.
struct FcWgrad {
  static constexpr bool A_KCONTIG = false;
  static constexpr bool B_KCONTIG = false;
  int M, N, K;
  int KIN;
  const float* __restrict__ in;  // [B,KIN]
  const float* __restrict__ dy;  // [B,NOUT]
  float* __restrict__ gw;        // [KIN,NOUT]
  float* __restrict__ gb;        // [NOUT]

  using AInfo = LinInfo;
  using BInfo = LinInfo;
  // A info: off = first row m, kk = k offset, ok = the 4 rows are all weight rows
  DDL_DEV AInfo prepA(int m, int kk) const { return {m, kk, m + 3 < KIN}; }
  DDL_DEV float4 loadA(const AInfo& a, int k0) const {
    const brsrc_t r = make_rsrc(in, (uint32_t)K * KIN * 4u);
    const int k = k0 + a.kk;
    const bool kin = k < K;
    if ((KIN & 3) == 0) {  // group = all weight rows, or [ones row, 0, 0, 0] / zeros: branch-free
      float4 v = bload4(r, (a.ok && kin) ? (k * KIN + a.off) * 4 : kOOB);
      if (a.off == KIN) v.x = kin ? 1.f : 0.f;
      return v;
    }
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int e = a.off + j;
      const float val = bload1(r, kin && e < KIN ? (k * KIN + e) * 4 : kOOB);
      v[j] = (e == KIN && kin) ? 1.f : val;
    }
    return make_float4(v[0], v[1], v[2], v[3]);
  }
  DDL_DEV BInfo prepB(int n, int kk) const { return {kk * N + n, kk, n < N}; }
  DDL_DEV float4 loadB(const BInfo& b, int k0) const {
    const brsrc_t r = make_rsrc(dy, (uint32_t)K * N * 4u);
    return bload4(r, b.ok && k0 + b.kk < K ? (b.off + k0 * N) * 4 : kOOB);
  }
  DDL_DEV void epi(int m0, int n, f32x4 v) const {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + r;
      if (m < KIN) gw[(size_t)m * N + n] = v[r];
      else if (m == KIN) gb[n] = v[r];
    }
  }
};

// ops the 16x16x4 LDS-DMA tile (CFG_MF16, gemm.h mainloop_dma16) is instantiated for: the
// halo-layout convolutions, whose 16-byte gathers srcA / srcB are the DMA sources
template <class P>
struct Mf16OK : std::false_type {};
template <int H, int CIN, int COUT, bool KM>
struct Mf16OK<ConvFwd<H, CIN, COUT, KM>> : std::bool_constant<CIN % kBK == 0> {};
template <int H, int CIN, int COUT, int HPREV>
struct Mf16OK<ConvDgrad<H, CIN, COUT, HPREV>> : std::true_type {};
template <int H, int CIN, int COUT>
struct Mf16OK<ConvWgradBM<H, CIN, COUT>> : std::true_type {};

// ops the 16-row K-wave launch (kwave16.h gemm_kw16_kernel, CFG_KW16) is instantiated for: the fc
// forwards (fc2 on it writes h2 itself and the head reads h2 instead of fc2's split-K partials).
// (The fc data gradients on its body inside the packed launches measured equal or slower,
// profiles/r6_sched_ab_kw16_dgrad.log, and were not kept.)
template <class P>
struct KW16OK : std::false_type {};
template <bool R>
struct KW16OK<FcFwd<R>> : std::true_type {};

// ops the K-wave launch (gemm.h gemm_kwave_kernel, CFG_KWAVE) is instantiated for
template <class P>
struct KWaveOK : std::false_type {};
template <bool R>
struct KWaveOK<FcFwd<R>> : std::true_type {};
template <>
struct KWaveOK<FcDgradAct> : std::true_type {};
template <int HP, int C>
struct KWaveOK<FcDgradPool<HP, C>> : std::true_type {};
// (the conv2-4 forwards as K-wave launches — the K split inside one workgroup instead of the
// split-K partials, tickets and last arriver — measured 277.9-288.6 us/step against 278.3 for
// 4 / 8 / 16 waves: no gain, not instantiated; profiles/r6_sched_ab_kwave_fwd.log)
// (the conv backward as K-wave tiles lost to the dual launches in every variant, 312-402 vs
// 289.5 us/step, and was removed: docs/DESIGN.md round 5)

}  // namespace ddl
