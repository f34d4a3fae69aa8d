// Kernel-instantiating half of the CNN step engine (engine.hip holds the host logic).
//
// Every GEMM op instantiates its tile configs x schedules and every dual launch the cross
// product of its two ops' one-wave configs, so the templates live here and are explicitly
// instantiated in several translation units (engine_ops_*.hip) that compile in parallel.
#pragma once
#include <stdexcept>
#include <type_traits>

#include "api.h"
#include "layers.h"
#include "head.h"
#include "conv1.h"
#include "kwave16.h"
#include "engine_decl.h"

namespace ddl {

#define TILE_0 64, 64, 32, 1, 1
#define TILE_1 128, 64, 32, 2, 1
#define TILE_2 64, 32, 32, 1, 1
#define TILE_3 32, 32, 32, 1, 1
#define TILE_4 32, 64, 32, 1, 1
#define TILE_5 32, 32, 16, 1, 1   // software-pipelined main loop (gemm.h GemmTile::PIPE)
#define TILE_6 64, 64, 32, 2, 2   // 4 waves of 32x32 sharing one LDS-staged 64x64 block tile
#define TILE_7 64, 32, 32, 2, 1   // 2 waves of 32x32 along M
#define TILE_8 32, 64, 32, 1, 2   // 2 waves of 32x32 along N
// eval-only (conv forward, large M)
#define TILE_9 128, 128, 32, 2, 2
#define TILE_10 128, 64, 32, 2, 2
#define TILE_11 256, 64, 32, 4, 1
#define TILE_12 128, 128, 32, 4, 1
// training: one-wave 32x32x32 on 16x16x4 MFMAs with LDS-DMA staging (CFG_MF16)
#define TILE_14 32, 32, 32, 1, 1, 1

template <class P>
inline void launch_cfg(int c, const P& p, int s, int wide_thr, const SplitScratch& sc,
                       hipStream_t st) {
  if (c == CFG_KWAVE) {
    if constexpr (KWaveOK<P>::value) {
      launch_gemm_kwave<32>(p, s < 0 ? -s : s, st);
      return;
    }
    c = 3;  // not instantiated for this op: the one-wave 32x32 tile
  }
  if (c == CFG_KW16) {
    if constexpr (KW16OK<P>::value) {
      launch_gemm_kw16(p, s < 0 ? -s : s, st);
      return;
    }
    c = 3;
  }
  if (c == CFG_MF16) {
    if constexpr (Mf16OK<P>::value) {
      launch_gemm<TILE_14>(p, s, wide_thr, sc, st);
      return;
    }
    c = 3;
  }
  switch (c) {
    case 0: launch_gemm<TILE_0>(p, s, wide_thr, sc, st); break;
    case 1: launch_gemm<TILE_1>(p, s, wide_thr, sc, st); break;
    case 2: launch_gemm<TILE_2>(p, s, wide_thr, sc, st); break;
    case 3: launch_gemm<TILE_3>(p, s, wide_thr, sc, st); break;
    case 4: launch_gemm<TILE_4>(p, s, wide_thr, sc, st); break;
    case 5: launch_gemm<TILE_5>(p, s, wide_thr, sc, st); break;
    case 6: launch_gemm<TILE_6>(p, s, wide_thr, sc, st); break;
    case 7: launch_gemm<TILE_7>(p, s, wide_thr, sc, st); break;
    default: launch_gemm<TILE_8>(p, s, wide_thr, sc, st); break;
  }
}

template <class W>
inline W wgrad_bm(int M, int N, int K, const float* x, const float* dpre, float* gw, float* gb,
                  int B) {
  const int nb = W::nb(B);
  if ((uint64_t)K * (uint64_t)nb >= (1ull << 32))  // W::magic's exactness bound
    throw std::runtime_error("weight-gradient batch too large for the batch-minor enumeration");
  return W{M, N, K, x, dpre, gw, gb, B, nb, W::magic(nb)};
}

// Problem policy of op OP (layers.h) bound to this engine's buffers, at batch B.
template <int OP>
inline auto make_policy(const Engine& e, int B, const float* x, const uint32_t* seed,
                        bool train) {
  int M, N, K;
  Engine::op_shape(OP, B, &M, &N, &K);
  const uint32_t thr = train ? e.thr24 : 0u;
  const float* const* P = e.P;
  float* const* G = e.G;
  // pool / ReLU codes only feed the backward: an eval forward skips their stores
  if constexpr (OP == OP_CONV1_FWD)
    return ConvFwd<28, 1, 32>{M, N, K, x, P[0], P[1], e.p1, train ? e.c1 : nullptr};
  else if constexpr (OP == OP_CONV2_FWD)
    return ConvFwd<14, 32, 64>{M, N, K, e.p1, P[2], P[3], e.p2, train ? e.c2 : nullptr};
  else if constexpr (OP == OP_CONV3_FWD)
    return ConvFwd<7, 64, 128>{M, N, K, e.p2, P[4], P[5], e.p3, train ? e.c3 : nullptr};
  else if constexpr (OP == OP_CONV4_FWD)
    return ConvFwd<4, 128, 256>{M, N, K, e.p3, P[6], P[7], e.p4, train ? e.c4 : nullptr};
  else if constexpr (OP == OP_FC1_FWD)
    return FcFwd<true>{M, N, K, e.p4, P[8], P[9], e.h1, seed, 1u, thr, e.inv_keep, e.seed_value};
  else if constexpr (OP == OP_FC2_FWD)
    return FcFwd<false>{M, N, K, e.h1, P[10], P[11], e.h2, seed, 2u, thr, e.inv_keep, e.seed_value};
  else if constexpr (OP == OP_FC2_DGRAD)
    return FcDgradAct{{M, N, K, e.dpre2fc, P[10]}, e.h1, e.inv_keep, e.dpre1fc};
  else if constexpr (OP == OP_FC2_WGRAD)
    return FcWgrad{M, N, K, 1024, e.h1, e.dpre2fc, G[10], G[11]};
  else if constexpr (OP == OP_FC1_DGRAD)
    return FcDgradPool<2, 256>{{M, N, K, e.dpre1fc, P[8]}, e.c4, e.d4};
  else if constexpr (OP == OP_FC1_WGRAD)
    return FcWgrad{M, N, K, 1024, e.p4, e.dpre1fc, G[8], G[9]};
  else if constexpr (OP == OP_CONV4_DGRAD)
    return ConvDgrad<4, 128, 256, 7>{M, N, K, e.d4, P[6], e.c3, e.d3};
  else if constexpr (OP == OP_CONV4_WGRAD)
    return wgrad_bm<WgradConv4>(M, N, K, e.p3, e.d4, G[6], G[7], B);
  else if constexpr (OP == OP_CONV3_DGRAD)
    return ConvDgrad<7, 64, 128, 14>{M, N, K, e.d3, P[4], e.c2, e.d2};
  else if constexpr (OP == OP_CONV3_WGRAD)
    return wgrad_bm<WgradConv3>(M, N, K, e.p2, e.d3, G[4], G[5], B);
  else if constexpr (OP == OP_CONV2_DGRAD)
    return ConvDgrad<14, 32, 64, 28>{M, N, K, e.d2, P[2], e.c1, e.d1};
  else if constexpr (OP == OP_CONV2_WGRAD)
    return wgrad_bm<WgradConv2>(M, N, K, e.p1, e.d2, G[2], G[3], B);
  else
    return WgradConv1{M, N, K, x, e.d1, G[0], G[1]};
}

template <int OP>
void run_op_inst(Engine& e, const float* x, int B, const uint32_t* seed, bool train,
                     hipStream_t st, int si) {
  const auto p = make_policy<OP>(e, B, x, seed, train);
  if constexpr (OP == OP_CONV2_FWD) {
    // eval: conv2 on the tap-skipping K map (group-major rows), one-wave 64x64 tiles
    if (!train && e.eval_kmap2 && e.eval_cfg[OP] == 0) {
      const ConvFwd<14, 32, 64, true> pk{p.M, p.N, p.K, p.x, p.w, p.bias, p.out, p.code};
      launch_gemm<TILE_0>(pk, 1, 1, e.scratch[si], st);
      return;
    }
  }
  if constexpr (OP == OP_CONV2_FWD || OP == OP_CONV3_FWD || OP == OP_CONV4_FWD) {
    if (!train && e.eval_cfg[OP] >= NUM_TILE_CFGS) {  // eval-only large tiles, no split
      switch (e.eval_cfg[OP]) {
        case 9: launch_gemm<TILE_9>(p, 1, 1, e.scratch[si], st); break;
        case 10: launch_gemm<TILE_10>(p, 1, 1, e.scratch[si], st); break;
        case 11: launch_gemm<TILE_11>(p, 1, 1, e.scratch[si], st); break;
        default: launch_gemm<TILE_12>(p, 1, 1, e.scratch[si], st); break;
      }
      return;
    }
  }
  launch_cfg(train ? e.cfg[OP] : e.eval_cfg[OP], p, train ? e.splits[OP] : 1, e.wide[OP],
             e.scratch[si], st);
}

// ---- dual launches: data- and weight-gradient GEMM of one layer in one kernel -----------------
// dual launches are instantiated for the one-wave configs: 32x32 (3), 32x32 BK 16 pipelined (5)
// and the 16x16x4 tile (CFG_MF16) (the register-staged one-wave 64x64 / 32x64 tiles, 180-230
// VGPRs, never won a dual launch in the real-step tuner)
inline bool one_wave_cfg(int c) { return c == 3 || c == 5 || c == CFG_MF16; }

template <int C> struct CfgOf;
template <> struct CfgOf<3> { using T = TileCfg<TILE_3>; };
template <> struct CfgOf<5> { using T = TileCfg<TILE_5>; };
template <> struct CfgOf<CFG_MF16> { using T = TileCfg<TILE_14>; };
template <int C> using IC = std::integral_constant<int, C>;

// f(IC<c'>) for the one-wave config c' that op policy P runs for run-time config c (configs P
// has no instantiation for fall back to 3; anything but 5 / MF16 likewise)
template <class P, class F>
inline void with_one_wave_cfg(int c, F&& f) {
  if constexpr (Mf16OK<P>::value) {
    if (c == CFG_MF16) return f(IC<CFG_MF16>{});
  }
  if (c == 5) return f(IC<5>{});
  f(IC<3>{});
}
// every pairing of the one-wave configs is instantiated
constexpr bool dual_pair_ok(int, int) { return true; }

// The fc1 / fc2 weight gradients as extra blocks of the conv4 dual launch:
// dW1 / dW2 feed only the optimizer, so they leave the fc backward's packed launches (which then
// carry only the data-gradient chain to conv4) and fill the conv4 dual's idle SIMD slots.  The
// tiles are the packs' (one-wave 32x32, BK 32, unsplit over K = batch): the same bits.  The
// segment's optimizer tail (tail.h) follows them.  models/__init__.py HIP_SEGMENTS lists fc1 / fc2
// in segment 1 accordingly.
struct FcWgradAux {
  using T = GemmTile<32, 32, 32, 1, 1, FcWgrad>;
  static constexpr int LDS_F4 = T::LDS_F4;
  FcWgrad p2{}, p1{};           // fc2, fc1
  int n2 = 0, n1 = 0, gx2 = 1, gx1 = 1;
  UpdTail t;
  int nblk = 0;
  int first_ = 0;
  static DDL_DEV void tile(const FcWgrad& p, int i, int gx, float* lds) {
    const int m_blk = (i % gx) * 32, n_blk = (i / gx) * 32;
    f32x16 acc[1][1];
    T::mainloop(p, m_blk, n_blk, 0, p.K, lds, acc);
    T::epilogue(p, m_blk, n_blk, acc);
  }
  DDL_DEV void run(int b, float* lds) const {
    if (b < n2) tile(p2, b, gx2, lds);
    else if (b < n2 + n1) tile(p1, b - n2, gx1, lds);
    else tail_body(t, b - n2 - n1);
  }
};

inline FcWgradAux fc_wgrad_aux(Engine& e, int B, const float* x, const uint32_t* seed) {
  FcWgradAux a;
  if (e.fc_wgrad_pending & 1) {
    a.p2 = make_policy<OP_FC2_WGRAD>(e, B, x, seed, true);
    a.gx2 = (a.p2.M + 31) / 32;
    a.n2 = a.gx2 * ((a.p2.N + 31) / 32);
  }
  if (e.fc_wgrad_pending & 2) {
    a.p1 = make_policy<OP_FC1_WGRAD>(e, B, x, seed, true);
    a.gx1 = (a.p1.M + 31) / 32;
    a.n1 = a.gx1 * ((a.p1.N + 31) / 32);
  }
  e.fc_wgrad_pending = 0;
  a.t = e.tail;
  e.tail = UpdTail();
  a.first_ = 0;  // (tiles, then the tail, after the GEMM blocks)
  a.nblk = a.n2 + a.n1 + a.t.nblocks;
  return a;
}

// fc3's weight gradient as aux blocks (head.h), pending after the fused head kernel
inline HeadWgradAux head_aux(Engine& e, int B) {
  HeadWgradAux a;
  if (e.head_wgrad_pending) {
    a.h2 = e.h2;
    a.dlog = e.dlog;
    a.B = B;
    a.gw = e.G[12];
    a.gb = e.G[13];
    a.nblk = HK + 1;
  }
  e.head_wgrad_pending = 0;
  return a;
}

template <int OA, int OB>
inline void run_back_to_back(Engine& e, const float* x, int B, const uint32_t* seed,
                             hipStream_t st) {
  e.flush_tail(st);
  if constexpr (OA == OP_FC2_DGRAD) e.flush_head_wgrad(B, st);
  run_op_inst<OA>(e, x, B, seed, true, st, 0);
  run_op_inst<OB>(e, x, B, seed, true, st, 0);
}

template <class CA, class CB, int OA, int OB, class PA, class PB>
inline void dual_b(Engine& e, const PA& pa, const PB& pb, int B, hipStream_t st) {
  auto go = [&](const auto& aux) {
    launch_gemm_dual<CA, PA, CB, PB>(pa, e.splits[OA], e.scratch[0], e.wide[OA], pb,
                                     e.splits[OB], e.scratch[1], e.wide[OB], st, aux, nullptr,
                                     e.dual_order(OA));
  };
  // the fc2 dual carries fc3's weight gradient; the conv4 dual the deferred fc weight
  // gradients (if any) and the pending optimizer tail; the others the tail
  if constexpr (OA == OP_FC2_DGRAD) {
    e.flush_tail(st);
    go(head_aux(e, B));
  } else if constexpr (OA == OP_CONV4_DGRAD) {
    if (e.fc_wgrad_pending) {
      go(fc_wgrad_aux(e, B, nullptr, nullptr));
    } else {
      go(TailAux(e.tail));
      e.tail = UpdTail();
    }
  } else {
    go(TailAux(e.tail));
    e.tail = UpdTail();
  }
}

// Ops OA and OB (independent) in one launch if both use one-wave tiles, else back to back.
// OA on the K-wave config (fc data gradients) with OB on a one-wave 32x32 config: one packed
// launch (gemm.h gemm_pack_kernel; OB's tiles run BK 32 there).
// (fc only: the packed launch runs OB's tiles unsplit over the raw K range, which the conv weight
// gradients' tap-window K maps do not support; a conv pair with a K-wave op runs back to back)
template <int OA, int OB>
void run_dual_inst(Engine& e, const float* x, int B, const uint32_t* seed, hipStream_t st) {
  constexpr bool fc_pair = OA == OP_FC2_DGRAD || OA == OP_FC1_DGRAD;
  if (fc_pair && e.dual && e.cfg[OA] == CFG_KWAVE && (e.cfg[OB] == 3 || e.cfg[OB] == 5)) {
    const auto pa = make_policy<OA>(e, B, x, seed, true);
    auto pb = make_policy<OB>(e, B, x, seed, true);
    if constexpr (fc_pair && KWaveOK<std::decay_t<decltype(pa)>>::value) {
      // the weight gradient left to the conv4 dual launch (FcWgradAux): the pack carries the
      // data gradient (and its aux work) only
      if (e.fc_wgrad_defer) {
        e.fc_wgrad_pending |= OA == OP_FC2_DGRAD ? 1 : 2;
        pb.M = 0;
      }
      if constexpr (OA == OP_FC2_DGRAD) {
        e.flush_tail(st);
        launch_gemm_pack(pa, e.splits[OA], pb, head_aux(e, B), st);
      } else {
        launch_gemm_pack(pa, e.splits[OA], pb, TailAux(e.tail), st);
        e.tail = UpdTail();
      }
      return;
    }
  }
  if (!e.dual || !one_wave_cfg(e.cfg[OA]) || !one_wave_cfg(e.cfg[OB])) {
    run_back_to_back<OA, OB>(e, x, B, seed, st);
    return;
  }
  const auto pa = make_policy<OA>(e, B, x, seed, true);
  const auto pb = make_policy<OB>(e, B, x, seed, true);
  using PA = std::decay_t<decltype(pa)>;
  using PB = std::decay_t<decltype(pb)>;
  with_one_wave_cfg<PA>(e.cfg[OA], [&](auto ca) {
    with_one_wave_cfg<PB>(e.cfg[OB], [&](auto cb) {
      constexpr int A = decltype(ca)::value, Bc = decltype(cb)::value;
      if constexpr (dual_pair_ok(A, Bc))
        dual_b<typename CfgOf<A>::T, typename CfgOf<Bc>::T, OA, OB>(e, pa, pb, B, st);
      else
        run_back_to_back<OA, OB>(e, x, B, seed, st);
    });
  });
}

// Split the last segment's update `in` into conv1's weight / bias spans (applied by the
// epilogue of conv1's weight-gradient reduce: `pa`) and the remaining ranges (`rest`, tail
// blocks of that launch).  false: the layout does not allow it (the caller keeps `in`).
template <class PN>
inline bool final_split(const Engine& e, const UpdTail& in, const PN& pn, WgradAdam<PN>& pa,
                        UpdTail& rest) {
  struct Span { const float* w; int64_t n; float *pw = nullptr, *pm = nullptr, *pv = nullptr;
                float lr_t = 0.f; };
  Span sp[2] = {{e.P[0], (int64_t)PN::KW * pn.N}, {e.P[1], (int64_t)pn.N}};
  rest = in;
  rest.npieces = 0;
  int blk = 0;
  auto a16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  auto keep = [&](const UpdPiece& p, int64_t lo, int64_t hi) {
    if (hi <= lo) return true;
    if ((hi - lo) % 4 || rest.npieces >= kTailPieces) return false;
    UpdPiece q = p;
    q.w = p.w + lo; q.g = p.g + lo; q.m = p.m + lo; q.v = p.v + lo;
    if (!a16(q.w) || !a16(q.g) || !a16(q.m) || !a16(q.v)) return false;
    q.n = hi - lo;
    q.blk0 = blk;
    blk += (int)((q.n / 4 + in.f4_per_block - 1) / in.f4_per_block);
    rest.p[rest.npieces++] = q;
    return true;
  };
  for (int i = 0; i < in.npieces; ++i) {
    const UpdPiece& p = in.p[i];
    // the spans inside this piece, in address order
    int64_t cuts[2][2];
    int nc = 0;
    for (Span& s : sp) {
      const int64_t o = s.w - p.w;
      if (o + s.n <= 0 || o >= p.n) continue;       // disjoint
      if (o < 0 || o + s.n > p.n) return false;      // straddles the piece edge
      s.pw = p.w + o; s.pm = p.m + o; s.pv = p.v + o; s.lr_t = p.lr_t;
      cuts[nc][0] = o; cuts[nc][1] = o + s.n; ++nc;
    }
    if (nc == 2 && cuts[1][0] < cuts[0][0]) {
      std::swap(cuts[0][0], cuts[1][0]);
      std::swap(cuts[0][1], cuts[1][1]);
    }
    int64_t at = 0;
    for (int c = 0; c < nc; ++c) {
      if (!keep(p, at, cuts[c][0])) return false;
      at = cuts[c][1];
    }
    if (!keep(p, at, p.n)) return false;
  }
  if (!sp[0].pw || !sp[1].pw || sp[0].lr_t != sp[1].lr_t) return false;
  rest.nblocks = blk;
  static_cast<PN&>(pa) = pn;
  pa.w_w = sp[0].pw; pa.w_m = sp[0].pm; pa.w_v = sp[0].pv;
  pa.b_w = sp[1].pw; pa.b_m = sp[1].pm; pa.b_v = sp[1].pv;
  pa.lr_t = sp[0].lr_t;
  pa.c1 = in.c1; pa.c2 = in.c2; pa.eps = in.eps; pa.scale = in.scale;
  return true;
}

// The Adam spans (parameter, m, v, lr_t) of [w, w + n) inside the update pieces of `t`.
inline bool find_span(const UpdTail& t, const float* w, int64_t n, float*& pw, float*& pm,
                      float*& pv, float& lr) {
  for (int i = 0; i < t.npieces; ++i) {
    const UpdPiece& p = t.p[i];
    const int64_t o = w - p.w;
    if (o >= 0 && o + n <= p.n) {
      pw = p.w + o; pm = p.m + o; pv = p.v + o; lr = p.lr_t;
      return true;
    }
  }
  return false;
}

// Split the last segment's update into conv2's (weight-gradient reduce epilogue: `pa`) and
// conv1's (final reduce level of the direct kernel: `ad`); false unless the pieces are exactly
// those four tensors with one step size.
template <class PB>
inline bool final_split_conv12(const Engine& e, const UpdTail& in, const PB& pb,
                               WgradAdam<PB>& pa, C1Adam& ad) {
  const int64_t n2w = (int64_t)PB::KW * pb.N, n2b = pb.N, n1w = 800, n1b = 32;
  // every element of the pieces is one of the four tensors or the alignment padding that
  // follows a tensor in the plan buffer (< kPad elements: zero gradient and state, so skipping
  // its update changes nothing; flat plans at W > 1 end the bucket on a 256-float boundary)
  constexpr int64_t kPad = 256;
  const float* sw[4] = {e.P[0], e.P[1], e.P[2], e.P[3]};
  const int64_t sn[4] = {n1w, n1b, n2w, n2b};
  for (int i = 0; i < in.npieces; ++i) {
    const UpdPiece& p = in.p[i];
    int64_t pos = 0;
    bool first = true;
    while (pos < p.n) {
      int k = -1;
      for (int j = 0; j < 4; ++j) {
        const int64_t o = sw[j] - p.w;
        if (o >= pos && o + sn[j] <= p.n && (k < 0 || o < sw[k] - p.w)) k = j;
      }
      if (k < 0) break;
      const int64_t gap = (sw[k] - p.w) - pos;
      if (gap >= kPad || (first && gap != 0)) return false;
      pos = (sw[k] - p.w) + sn[k];
      first = false;
    }
    if (first || p.n - pos >= kPad) return false;
  }
  float lr[4];
  static_cast<PB&>(pa) = pb;
  if (!find_span(in, e.P[2], n2w, pa.w_w, pa.w_m, pa.w_v, lr[0]) ||
      !find_span(in, e.P[3], n2b, pa.b_w, pa.b_m, pa.b_v, lr[1]) ||
      !find_span(in, e.P[0], n1w, ad.w_w, ad.w_m, ad.w_v, lr[2]) ||
      !find_span(in, e.P[1], n1b, ad.b_w, ad.b_m, ad.b_v, lr[3]))
    return false;
  if (lr[1] != lr[0] || lr[2] != lr[0] || lr[3] != lr[0]) return false;
  pa.lr_t = ad.lr_t = lr[0];
  pa.c1 = ad.c1 = in.c1;
  pa.c2 = ad.c2 = in.c2;
  pa.eps = ad.eps = in.eps;
  pa.scale = ad.scale = in.scale;
  ad.on = 1;
  return true;
}

// Dual launch OA + OB, then op ON with OB's wide split-K reduce fused into ON's launch (both
// need only what the dual wrote; saves one dependent boundary: conv2 dual -> [conv2 wgrad
// reduce | conv1 wgrad GEMM]).  Instantiated for the tuned configs (OA: 32x32, OB: 32x32
// BK 16 pipelined, ON: 32x32 split-K); any other schedule takes the unfused sequence.
template <int OA, int OB, int ON, class CA, class CB>
void dual_then_b(Engine& e, const float* x, int B, const uint32_t* seed, hipStream_t st) {
  const auto pa = make_policy<OA>(e, B, x, seed, true);
  const auto pb = make_policy<OB>(e, B, x, seed, true);
  const auto pn = make_policy<ON>(e, B, x, seed, true);
  using PA = std::decay_t<decltype(pa)>;
  using PB = std::decay_t<decltype(pb)>;
  using PN = std::decay_t<decltype(pn)>;
  using CN = TileCfg<TILE_3>;
  SubGrid gb;
  launch_gemm_dual<CA, PA, CB, PB>(pa, e.splits[OA], e.scratch[0], e.wide[OA], pb,
                                   e.splits[OB], e.scratch[1], e.wide[OB], st, TailAux(e.tail),
                                   &gb, e.dual_order(OA));
  e.tail = UpdTail();
  constexpr bool kFinal = ON == OP_CONV1_WGRAD;
  if constexpr (kFinal) {
    // conv1's weight gradient on the direct kernel (conv1.h), sharing its launch with OB's
    // pending reduce; scratch[0] is free here (OA's split-K finished inside the dual launch
    // or in its own reduce before this point)
    const bool direct =
        e.conv1_wgrad_direct && conv1_wgrad_direct_ok(B, e.slab_floats, e.scratch[0].max_tiles);
    if (direct) {
      float* part = static_cast<float*>(e.scratch[0].slab);
      // the last segment's update (W = 1 tail path) inside this launch: conv2's in its weight-
      // gradient reduce epilogue, conv1's in the final reduce level; no Adam launch follows
      if (e.final_upd.npieces > 0 && gb.mode == 2) {
        WgradAdam<PB> pa;
        C1Adam ad;
        if (final_split_conv12(e, e.final_upd, pb, pa, ad)) {
          launch_conv1_wgrad<CB, WgradAdam<PB>>(pa, gb, x, e.d1, B, e.G[0], e.G[1], part,
                                                e.scratch[0].tickets, st, ad);
          e.final_upd = UpdTail();
          return;
        }
      }
      launch_conv1_wgrad<CB, PB>(pb, gb, x, e.d1, B, e.G[0], e.G[1], part, e.scratch[0].tickets,
                                 st);
      return;
    }
  }
  const bool fin = kFinal && e.final_upd.npieces > 0;
  SubGrid gn;
  if (!launch_reduce_with_gemm<CB, PB, CN, PN>(pb, gb, pn, e.splits[ON], e.wide[ON],
                                               e.scratch[0], st,
                                               fin ? &gn : nullptr)) {
    launch_reduce<CB::BM, CB::BN, CB::BK, CB::WM, CB::WN, PB>(pb, gb, st);
    e.run_op(ON, x, B, seed, true, st, 0);
    return;
  }
  if constexpr (kFinal) {
    if (fin) {
      // conv1's weight-gradient reduce applies conv1's update in its epilogue and carries the
      // rest of the last segment's update as tail blocks: no stand-alone optimizer launch
      WgradAdam<PN> pa;
      UpdTail rest;
      if (final_split(e, e.final_upd, pn, pa, rest) &&
          launch_reduce_tail<CN::BM, CN::BN, CN::BK, CN::WM, CN::WN>(pa, gn, rest, st))
        e.final_upd = UpdTail();
      else
        launch_reduce<CN::BM, CN::BN, CN::BK, CN::WM, CN::WN, PN>(pn, gn, st);
    }
  }
}

// Instantiated for OA / OB on the one-wave configs (dual_pair_ok), ON on 32x32 split-K; any
// other schedule takes the unfused sequence.
template <int OA, int OB, int ON>
void run_dual_then_inst(Engine& e, const float* x, int B, const uint32_t* seed, hipStream_t st) {
  const int ca = e.cfg[OA], cb = e.cfg[OB];
  if (!e.dual || (ca != 3 && ca != CFG_MF16) || (cb != 3 && cb != 5 && cb != CFG_MF16) ||
      e.cfg[ON] != 3) {
    run_dual_inst<OA, OB>(e, x, B, seed, st);
    e.run_op(ON, x, B, seed, true, st, 0);
    return;
  }
  using PA = decltype(make_policy<OA>(e, B, x, seed, true));
  using PB = decltype(make_policy<OB>(e, B, x, seed, true));
  with_one_wave_cfg<PA>(ca, [&](auto ia) {
    with_one_wave_cfg<PB>(cb, [&](auto ib) {
      constexpr int A = decltype(ia)::value, Bc = decltype(ib)::value;
      if constexpr (A != 5 && dual_pair_ok(A, Bc)) {
        dual_then_b<OA, OB, ON, typename CfgOf<A>::T, typename CfgOf<Bc>::T>(e, x, B, seed, st);
      } else {
        run_dual_inst<OA, OB>(e, x, B, seed, st);
        e.run_op(ON, x, B, seed, true, st, 0);
      }
    });
  });
}

}  // namespace ddl
