// Generic FP32 MFMA GEMM engine for gfx950: C[M,N] = sum_k A[m,k] * B[k,n].
//
// Every conv / fc forward, data-gradient and weight-gradient of the MNIST CNN is one
// instantiation of this kernel with a *problem* policy P that supplies:
//   * operand gathers: P::prepA(mn) -> per-thread info hoisted out of the K loop, then
//     P::loadA(info, k) returning 4 consecutive elements along the operand's contiguous
//     global direction (A_KCONTIG / B_KCONTIG); same for B.  Implicit-GEMM im2col,
//     transposed weights and pool-window row orders are just address functions — nothing
//     is materialised;
//   * a fused epilogue P::epi(m0, n, f32x4 rows m0..m0+3) (bias / ReLU / max-pool with
//     argmax code / dropout / pool-backward scatter / dW+db split).  The 32x32 MFMA C
//     layout gives each lane 4 groups of 4 consecutive rows of one column; with M
//     enumerated pool-window-major each group is exactly one 2x2 pool window.
//
// Math: v_mfma_f32_32x32x2_f32 (exact fp32; gfx950 has no xf32), 64-cycle issue; a wave
// with a single fragment alternates two accumulator chains.
// Tiling: BM x BN block tile, BK-deep K step, WM x WN waves (wave64), wave tile
// (BM/WM) x (BN/WN) of 32x32 fragments.  One-wave blocks use a single LDS buffer (no
// barriers), multi-wave blocks a double buffer; global loads run two K tiles ahead in
// registers; a whole K tile's fragments are read from LDS in one burst before its MFMAs.  LDS operand images follow global contiguity so the
// global->LDS copy is a straight float4 store:
//   K-contiguous operand -> [mn][BK+4]   one ds_read_b128 per 4 MFMAs: lane half
//                                        h = l>>5 owns k = 8r+4h .. 8r+4h+3 of every
//                                        8-deep sub-step (MFMA s pairs k = 8r+s and
//                                        8r+4+s); stride BK+4 is bank-conflict free for
//                                        the four 16-lane b128 groups
//   MN-contiguous operand -> [BK][mn+4]  ds_read_b32; the two 32-lane halves read rows
//                                        4 apart (separate conflict groups)
//
// The split-K driver runs the per-tile main loop / epilogue (GemmTile):
// Split-K (gridDim.z = S > 1), deterministic, no float atomics:
//   mode 1: every split stores its fp32 partial fragments (float4 per lane, coalesced,
//     write-through sc1) and takes an arrival ticket; the last arriver of a tile sums the S
//     partials in z order with sc1 loads and runs the fused epilogue (MI355X guide §5 /
//     §6 G16 in-launch reduction, sc1 form: no release or acquire fence).
//   mode 2: partials only; splitk_wide_reduce sums them with RL lanes per output element
//     and runs the epilogue.
#pragma once
#include <stdlib.h>

#include <type_traits>

#include "common.h"

// s_setprio 1 around each K tile's MFMA cluster (guide T5; measured 0.3753 -> 0.3747 ms/step)
#define DDL_MFMA_PRIO 1
#include "scratch.h"
#include "stamps.h"
#include "tail.h"

// partials in flight per round of a one-fragment tile's split-K sum (sum_partials)
#ifndef DDL_SPLITK_ZB
#define DDL_SPLITK_ZB 4
#endif

namespace ddl {

// One push-tail block (tail.h kind 1): arrival slice j of piece P — the gradient slice into the
// PS host's inbox (system write-through stores), then, once the wave's stores are
// acknowledged, the slice's word on the arrival board in host memory (the protocol of
// xgmi_async.hip's push kernel; one wave, so vmcnt covers every lane's stores).
DDL_DEV void push_tail_body(const UpdTail& t, const UpdPiece& P, int b) {
  const int j = b - P.blk0;
  if (j >= P.nslice) return;  // padding blocks of the last piece
  const int lane = threadIdx.x & 63;
  const int64_t n4 = P.n >> 2;
  const int64_t s0 = (int64_t)j * P.slice4;
  const int cnt = (int)((s0 + P.slice4 < n4 ? s0 + P.slice4 : n4) - s0);
  const float4* src = reinterpret_cast<const float4*>(P.g) + s0;
  if (P.w) {  // (null: a shard this rank hosts, posted only — xgmi_async.hip AsyncTable::elide)
    const brsrc_t dst = make_rsrc(P.w + s0 * 4, (uint32_t)cnt * 16u);
    for (int i = lane; i < cnt; i += 64) bstore4_sys(dst, i * 16, src[i]);
    drain_vmem();
  }
  if (lane == 0)
    __hip_atomic_store(P.posted + j, t.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One optimizer-tail block (tail.h): kTailF4PerLane float4 of one piece per lane, all loads
// issued before any math (HBM-bound: memory-level parallelism is the whole game).
DDL_DEV void tail_body(const UpdTail& t, int b) {
  int i = 0;
#pragma unroll
  for (int q = 1; q < kTailPieces; ++q)
    if (q < t.npieces && b >= t.p[q].blk0) i = q;
  if (t.kind == 1) {
    push_tail_body(t, t.p[i], b);
    return;
  }
  if (t.kind == 2) {  // ready flag: the launch started, so every earlier launch has completed
    if (b == 0 && (threadIdx.x & 63) == 0)
      __hip_atomic_store(t.p[0].arrive, t.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  const UpdPiece& P = t.p[i];
  const int64_t n4 = P.n >> 2;
  const int64_t blk_base = (int64_t)(b - P.blk0) * t.f4_per_block + (threadIdx.x & 63);
  float4* w = reinterpret_cast<float4*>(P.w);
  const float4* g = reinterpret_cast<const float4*>(P.g);
  float4* m = reinterpret_cast<float4*>(P.m);
  float4* v = reinterpret_cast<float4*>(P.v);
  for (int off = 0; off < t.f4_per_block; off += kTailF4PerBlock) {
    const int64_t base = blk_base + off;
    if (base >= n4) break;
    float4 W[kTailF4PerLane], G[kTailF4PerLane], M[kTailF4PerLane], V[kTailF4PerLane];
#pragma unroll
    for (int j = 0; j < kTailF4PerLane; ++j) {
      const int64_t e = base + j * 64;
      if (e < n4) { W[j] = w[e]; G[j] = g[e]; M[j] = m[e]; V[j] = v[e]; }
    }
#pragma unroll
    for (int j = 0; j < kTailF4PerLane; ++j) {
      const int64_t e = base + j * 64;
      if (e >= n4) continue;
      adam1(W[j].x, G[j].x * t.scale, M[j].x, V[j].x, P.lr_t, t.c1, t.c2, t.eps);
      adam1(W[j].y, G[j].y * t.scale, M[j].y, V[j].y, P.lr_t, t.c1, t.c2, t.eps);
      adam1(W[j].z, G[j].z * t.scale, M[j].z, V[j].z, P.lr_t, t.c1, t.c2, t.eps);
      adam1(W[j].w, G[j].w * t.scale, M[j].w, V[j].w, P.lr_t, t.c1, t.c2, t.eps);
      w[e] = W[j]; m[e] = M[j]; v[e] = V[j];
    }
  }
}

typedef float f32x16 __attribute__((ext_vector_type(16)));

DDL_DEV f32x16 mfma32x32x2(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

template <int BM, int BN, int WM, int WN>
struct TileGeo {
  static constexpr int NW = WM * WN;
  static constexpr int WTM = BM / WM, WTN = BN / WN;
  static constexpr int TM = WTM / 32, TN = WTN / 32;
  static constexpr int FRAGS = TM * TN;
  // float4 elements of one split's partial tile: 4 float4 per fragment per lane
  static constexpr int PART4 = NW * FRAGS * 4 * 64;
};

// ---- K maps: skipping K tiles that only multiply zeros ---------------------------------------
// A policy with `static constexpr bool KMAP = true` enumerates, per block tile, only part of
// its K range: `KWin kwin(m_lo, m_hi)` describes the rows' useful K sub-space (for a SAME
// conv: the 5x5 taps that land inside the image for some row of the tile), `kvlen(win)` is its
// length and the loaders take a *virtual* k (0 .. kvlen) plus the window: loadA(info, kv, win).
// Split-K divides each tile's virtual length (balanced per tile).  Anything a window keeps
// beyond the useful set
// reads zeros (halo layout), so a window only has to be a superset.
template <class P, class = void>
struct KMapOf {
  static constexpr bool value = false;
  struct Win {};
};
template <class P>
struct KMapOf<P, std::void_t<decltype(P::KMAP)>> {
  static constexpr bool value = P::KMAP;
  using Win = typename P::KWin;
};

// LDS-DMA staging of the one-wave 32x32 tiles (mainloop_dma, one 8 KB image per block) for
// policies that opt in with a constexpr DMA and srcA / srcB (the 16-byte gathers of their loadA /
// loadB): the halo-layout conv forwards.  The one-wave MULTI-fragment tiles (64x64 / 32x64,
// BN = 64: the eval forward) stage the same way (mainloop_dma_mf).  The variants measured and
// rejected — two images per block, DMA for the conv data / weight gradients on the 32x32x2 tile,
// direct-to-register fragments, register-gathered B — are recorded in docs/DESIGN.md.
// a policy whose A operand has rows that are not in memory (the weight gradients' ones row)
template <class P, class = void>
struct HasOnesA : std::false_type {};
template <class P>
struct HasOnesA<P, std::void_t<decltype(std::declval<const P&>().ones_group(
                       std::declval<const typename P::AInfo&>()))>> : std::true_type {};
// a policy with a row-wise epilogue epi_t(m, n0, float4 = row m, columns n0 .. n0 + 3): the tile
// epilogue transposes each lane quad's 4 rows x 4 columns first (GemmTile::epilogue)
template <class P, class = void>
struct HasEpiT : std::false_type {};
template <class P>
struct HasEpiT<P, std::void_t<decltype(std::declval<const P&>().epi_t(0, 0, float4{}))>>
    : std::true_type {};
template <class P, class = void>
struct HasDma : std::false_type {};
template <class P>
struct HasDma<P, std::void_t<decltype(P::DMA)>> : std::bool_constant<P::DMA> {};

// ---- per-tile building blocks shared by the split-K and stream-K drivers ---------------------
// V (tile-config variant): 0 = the 32x32x2 MFMA loops below; 1 = the one-wave 32x32x32 tile on
// v_mfma_f32_16x16x4_f32 with LDS-DMA staging (mainloop_dma16)
template <int BM, int BN, int BK, int WM, int WN, class P, int V = 0>
struct GemmTile {
  using G = TileGeo<BM, BN, WM, WN>;
  static constexpr int NT = WM * WN * 64;
  static constexpr bool AK = P::A_KCONTIG;
  static constexpr bool BKC = P::B_KCONTIG;
  static constexpr int SA = AK ? (BK + 4) : (BM + 4);
  static constexpr int A_ELEMS = AK ? BM * SA : BK * SA;
  static constexpr int SB = BKC ? (BK + 4) : (BN + 4);
  static constexpr int B_ELEMS = BKC ? BN * SB : BK * SB;
  static constexpr int WTM = G::WTM, WTN = G::WTN, TM = G::TM, TN = G::TN;
  static constexpr int FA = (BM * BK / 4) / NT;
  static constexpr int FB = (BN * BK / 4) / NT;
  static constexpr int R = BK / 8;
  static_assert(FA >= 1 && FA * NT == BM * BK / 4, "A tile must split evenly over threads");
  static_assert(FB >= 1 && FB * NT == BN * BK / 4, "B tile must split evenly over threads");
  static_assert(TM * 32 == WTM && TN * 32 == WTN, "wave tile must be 32-multiples");
  static_assert(BK % 8 == 0, "BK must be a multiple of 8");
  // One-wave blocks need neither a second LDS buffer nor barriers: a wave's LDS ops execute
  // in order, so the next tile's ds_writes cannot overtake this tile's ds_reads.  Halving
  // the LDS footprint doubles the resident waves per CU (LDS was the occupancy limit).
  static constexpr bool SOLO = (NT == 64);
  static constexpr int NBUF = SOLO ? 1 : 2;
  // 16x16x4 MFMA + LDS-DMA one-wave tile (variant 1; instantiated only for policies with the
  // 16-byte gathers srcA / srcB: layers.h Mf16OK)
  static constexpr bool DMA16 = V == 1 && SOLO && BM == 32 && BN == 32 && BK == 32;
  // (variants 2-4 — generic multi-fragment LDS-DMA tiles and 32x32 rings of 2 / 3 LDS-DMA
  // images — lost to these loops in every launch and were removed: docs/DESIGN.md round 5)
  static_assert(V == 0 || DMA16, "variant 1 is the one-wave 32x32x32 16x16x4 tile");
  // LDS-DMA staging (mainloop_dma): unpadded 32x32 images, swizzled through the gather
  // addresses (the DMA writes lane-linearly), one image of A + B per block
  static constexpr bool DMA = V == 0 && HasDma<P>::value && SOLO && TM * TN == 1 && BM == 32 &&
                              BN == 32 && BK == 32;
  static constexpr bool DMA_MF = V == 0 && HasDma<P>::value && SOLO && TM * TN > 1 && BN == 64 &&
                                 BK == 32 && AK && !BKC && !HasOnesA<P>::value;
  static constexpr int LDS_F4 = (DMA16 || DMA) ? 512
                                : DMA_MF ? (BM * BK + BK * BN) / 4
                                : (NBUF * (A_ELEMS + B_ELEMS)) / 4;
  // A wave with a single 32x32 fragment alternates two accumulator chains (summed at the
  // end) so consecutive MFMAs are independent (one chain: measured 0.3050 -> 0.3070 ms/step)
  static constexpr int NCH = TM * TN == 1 ? 2 : 1;
  static constexpr int WPART = TM * TN * 4 * 64;  // float4 of one wave's partial fragments
  static constexpr bool KM = KMapOf<P>::value;
  using Win = typename KMapOf<P>::Win;
  static DDL_DEV float4 ldA(const P& p, const typename P::AInfo& a, int k, const Win& w) {
    if constexpr (KM) return p.loadA(a, k, w);
    else return p.loadA(a, k);
  }
  static DDL_DEV float4 ldB(const P& p, const typename P::BInfo& b, int k, const Win& w) {
    if constexpr (KM) return p.loadB(b, k, w);
    else return p.loadB(b, k);
  }

  // acc = sum over k in [kb, ke) of the (m_blk, n_blk) block tile; kb is a multiple of BK.
  // One-wave single-fragment tiles with BK = 16 take the software-pipelined loop (its double
  // register sets fit at 3 waves/SIMD only with the 16-deep K step: at BK = 32 it needed
  // 256 VGPRs + 64 AGPRs, one wave per SIMD, and lost to the basic loop); others the basic loop.
  static constexpr bool PIPE = SOLO && TM * TN == 1 && BK == 16;
  // [kb, ke) is virtual (window w) for K-map policies
  static DDL_DEV void mainloop(const P& p, int m_blk, int n_blk, int kb, int ke, float* lds,
                               f32x16 (&acc)[TM][TN], const Win& w = Win()) {
    if constexpr (DMA16) mainloop_dma16(p, m_blk, n_blk, kb, ke, lds, acc, w);
    else if constexpr (DMA) mainloop_dma(p, m_blk, n_blk, kb, ke, lds, acc, w);
    else if constexpr (DMA_MF) mainloop_dma_mf(p, m_blk, n_blk, kb, ke, lds, acc, w);
    else if constexpr (PIPE) mainloop_pipe(p, m_blk, n_blk, kb, ke, lds, acc, w);
    else mainloop_basic(p, m_blk, n_blk, kb, ke, lds, acc, w);
  }

  // Software-pipelined main loop (one wave, one 32x32 fragment, single LDS buffer).
  // Per K tile t the wave's 16 MFMAs on fragments F[t&1] (already in VGPRs) are interleaved
  // with: the LDS store of tile t+1 from global-load registers G[(t+1)&1], the global loads
  // of tile t+3 into that freed register set (two iterations of latency cover), and the LDS
  // fragment reads of tile t+1 into F[(t+1)&1].  The LDS ops of a wave execute in order, so
  // the stores of t+1 cannot overtake the (earlier-issued) reads of t, nor the reads of t+1
  // the stores.  PMC on the unpipelined loop: MFMA pipe ~40 % busy with waves stalled on
  // LDS-read latency and on global loads issued only one tile ahead.
  static DDL_DEV void mainloop_pipe(const P& p, int m_blk, int n_blk, int kb, int ke,
                                    float* lds, f32x16 (&acc)[TM][TN], const Win& w) {
    float* const As = lds;
    float* const Bs = lds + A_ELEMS;
    const int tid = threadIdx.x & (NT - 1);  // a one-wave tile may be one wave of a larger block
    const int lane = tid & 63;
    const int nk = (ke - kb + BK - 1) / BK;
    typename P::AInfo ai[FA];
    typename P::BInfo bi[FB];
    int a_off[FA], b_off[FB];
#pragma unroll
    for (int it = 0; it < FA; ++it) {
      const int idx = tid + it * NT;
      if constexpr (AK) {
        const int kq = idx % (BK / 4), row = idx / (BK / 4);
        ai[it] = p.prepA(m_blk + row, kq * 4);
        a_off[it] = row * SA + kq * 4;
      } else {
        const int mq = idx % (BM / 4), kk = idx / (BM / 4);
        ai[it] = p.prepA(m_blk + mq * 4, kk);
        a_off[it] = kk * SA + mq * 4;
      }
    }
#pragma unroll
    for (int it = 0; it < FB; ++it) {
      const int idx = tid + it * NT;
      if constexpr (BKC) {
        const int kq = idx % (BK / 4), row = idx / (BK / 4);
        bi[it] = p.prepB(n_blk + row, kq * 4);
        b_off[it] = row * SB + kq * 4;
      } else {
        const int nq = idx % (BN / 4), kk = idx / (BN / 4);
        bi[it] = p.prepB(n_blk + nq * 4, kk);
        b_off[it] = kk * SB + nq * 4;
      }
    }
    float4 ga0[FA], gb0[FB], ga1[FA], gb1[FB];     // global staging G[0], G[1]
    float f0a[R][4], f0b[R][4], f1a[R][4], f1b[R][4];  // fragments F[0], F[1]
    auto gload = [&](int k0, float4 (&ra)[FA], float4 (&rb)[FB]) {
#pragma unroll
      for (int it = 0; it < FA; ++it) ra[it] = ldA(p, ai[it], k0, w);
#pragma unroll
      for (int it = 0; it < FB; ++it) rb[it] = ldB(p, bi[it], k0, w);
    };
    auto sstore = [&](const float4 (&ra)[FA], const float4 (&rb)[FB]) {
#pragma unroll
      for (int it = 0; it < FA; ++it) *reinterpret_cast<float4*>(As + a_off[it]) = ra[it];
#pragma unroll
      for (int it = 0; it < FB; ++it) *reinterpret_cast<float4*>(Bs + b_off[it]) = rb[it];
    };
    const int lr = lane & 31, lh = lane >> 5;
    auto fetch = [&](float (&fa)[R][4], float (&fb)[R][4]) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if constexpr (AK) {
          const float4 t = *reinterpret_cast<const float4*>(As + lr * SA + r * 8 + 4 * lh);
          fa[r][0] = t.x; fa[r][1] = t.y; fa[r][2] = t.z; fa[r][3] = t.w;
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) fa[r][s] = As[(r * 8 + 4 * lh + s) * SA + lr];
        }
        if constexpr (BKC) {
          const float4 t = *reinterpret_cast<const float4*>(Bs + lr * SB + r * 8 + 4 * lh);
          fb[r][0] = t.x; fb[r][1] = t.y; fb[r][2] = t.z; fb[r][3] = t.w;
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) fb[r][s] = Bs[(r * 8 + 4 * lh + s) * SB + lr];
        }
      }
    };
    f32x16 c0, c1;  // two independent accumulator chains
#pragma unroll
    for (int q = 0; q < 16; ++q) { c0[q] = 0.f; c1[q] = 0.f; }
    auto mfmas = [&](const float (&fa)[R][4], const float (&fb)[R][4]) {
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          if ((s & 1) && NCH == 2) c1 = mfma32x32x2(fa[r][s], fb[r][s], c1);
          else c0 = mfma32x32x2(fa[r][s], fb[r][s], c0);
        }
    };
    // Interleave pattern of one steady-state iteration (4R MFMAs, 64 cycles each): the DS
    // stores of the next tile between the first FA+FB MFMAs, then the next tile's fragment
    // reads (which must follow those stores) and the global loads between the rest.
    constexpr int NMF = 4 * R, NST = FA + FB;
    static_assert(NMF >= 2 * NST, "pipelined loop needs 2 MFMAs per staged float4");
    auto interleave = [&]() {
#pragma unroll
      for (int i = 0; i < NST; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // DS write
      }
#pragma unroll
      for (int i = 0; i < NMF - NST; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS read
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read
      }
    };

    if (nk > 0) {
      gload(kb, ga0, gb0);
      if (nk > 1) gload(kb + BK, ga1, gb1);
      sstore(ga0, gb0);
      if (nk > 2) gload(kb + 2 * BK, ga0, gb0);
      fetch(f0a, f0b);
    }
    int kt = 0;
    // steady state: tiles kt (F0) and kt+1 (F1) per trip; all of kt+1..kt+4 exist
    for (; kt + 4 < nk; kt += 2) {
      sstore(ga1, gb1);                       // tile kt+1
      gload(kb + (kt + 3) * BK, ga1, gb1);    // tile kt+3
      fetch(f1a, f1b);                        // fragments of kt+1
      mfmas(f0a, f0b);                        // tile kt
      interleave();
      __builtin_amdgcn_sched_barrier(0);
      sstore(ga0, gb0);                       // tile kt+2
      gload(kb + (kt + 4) * BK, ga0, gb0);    // tile kt+4
      fetch(f0a, f0b);                        // fragments of kt+2
      mfmas(f1a, f1b);                        // tile kt+1
      interleave();
      __builtin_amdgcn_sched_barrier(0);
    }
    // tail: at most 4 tiles left (kt .. nk-1), same rotation with guards
    for (; kt < nk; ++kt) {
      const bool odd = (kt & 1) != 0;
      const bool has1 = kt + 1 < nk, has3 = kt + 3 < nk;
      if (!odd) {
        if (has1) sstore(ga1, gb1);
        if (has3) gload(kb + (kt + 3) * BK, ga1, gb1);
        if (has1) fetch(f1a, f1b);
        mfmas(f0a, f0b);
      } else {
        if (has1) sstore(ga0, gb0);
        if (has3) gload(kb + (kt + 3) * BK, ga0, gb0);
        if (has1) fetch(f0a, f0b);
        mfmas(f1a, f1b);
      }
    }
    if constexpr (NCH == 2) acc[0][0] = c0 + c1;
    else acc[0][0] = c0;
  }

  static DDL_DEV Gather16 srcA(const P& p, const typename P::AInfo& a, int k, const Win& w) {
    if constexpr (KM) return p.srcA(a, k, w);
    else return p.srcA(a, k);
  }
  static DDL_DEV Gather16 srcB(const P& p, const typename P::BInfo& b, int k, const Win& w) {
    if constexpr (KM) return p.srcB(b, k, w);
    else return p.srcB(b, k);
  }

  // LDS-DMA loop (one wave, one 32x32 fragment, BK = 32).  Each K tile is 8 DMA instructions
  // (A and B: 4 x 1 KB) straight into an unpadded LDS image; no staging VGPRs and no ds_write.
  // The image is lane-linear, so the conflict-free layout is made on the GATHER side (guide
  // rule 21): a K-contiguous operand's 16-byte quad q of row r sits at quad q ^ ((r >> 1) & 7)
  // (the 16 lanes of a ds_read_b128 pass then hit 16 different bank groups), an MN-contiguous
  // operand's k-row k at row k ^ ((k >> 2) & 1) (the two lane halves of a fragment read, k and
  // k + 4, land in opposite bank halves).  The MFMA order (k pairs, two accumulator chains) is
  // the basic loop's, so both give the same bits.  A's rows that are not in memory (HasOnesA:
  // the weight gradients' ones row) arrive as zeros and are patched in the image with one
  // ds_write per holding lane once the tile has landed, before the fragment reads.  Tile t+1
  // is DMA'd into the one image once tile t's fragments are in registers; completion is
  // counted by hand (vm_wait).  (A second image — tile t+2 in flight during tile t's MFMAs —
  // measured 8 % slower: 152 registers and 16 KB of LDS cap the block at 2.5 waves per SIMD.)
  static DDL_DEV void mainloop_dma(const P& p, int m_blk, int n_blk, int kb, int ke, float* lds,
                                   f32x16 (&acc)[TM][TN], const Win& w) {
    static_assert(FA == 4 && FB == 4 && R == 4, "32x32x32 one-wave tile");
    static_assert(!(HasOnesA<P>::value && AK), "ones-row patch: MN-contiguous A");
    const int lane = threadIdx.x & 63;
    const int lr = lane & 31, lh = lane >> 5;
    const int nk = (ke - kb + BK - 1) / BK;
    typename P::AInfo ai[4];
    typename P::BInfo bi[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int sl = it * 64 + lane, row = sl >> 3, q = sl & 7;
      if constexpr (AK) ai[it] = p.prepA(m_blk + row, (q ^ ((row >> 1) & 7)) * 4);
      else ai[it] = p.prepA(m_blk + q * 4, row ^ ((row >> 2) & 1));
      if constexpr (BKC) bi[it] = p.prepB(n_blk + row, (q ^ ((row >> 1) & 7)) * 4);
      else bi[it] = p.prepB(n_blk + q * 4, row ^ ((row >> 2) & 1));
    }
    // the image float that lane's DMA `it` of A fills first (its .x), for the ones-row patch
    auto patch = [&](int k0) {
      if constexpr (HasOnesA<P>::value) {
#pragma unroll
        for (int it = 0; it < 4; ++it)
          if (p.ones_group(ai[it])) lds[(it * 64 + lane) * 4] = p.ones_value(ai[it], k0, w);
      }
    };
    const uint32_t base = lds_addr(lds);
    auto dma = [&](int k0) {
#pragma unroll
      for (int it = 0; it < 4; ++it) dma16(srcA(p, ai[it], k0, w), base + it * 1024);
#pragma unroll
      for (int it = 0; it < 4; ++it) dma16(srcB(p, bi[it], k0, w), base + 4096 + it * 1024);
    };
    // fragments of K step (r, s): lane half h holds k = 8r + 4h + s (the basic loop's order)
    auto rd = [&](float (&av)[R][4], float (&bv)[R][4]) {
      const float* As = lds;
      const float* Bs = As + 1024;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int q = (2 * r + lh) ^ ((lr >> 1) & 7);
        if constexpr (AK) {
          const float4 t = *reinterpret_cast<const float4*>(As + lr * 32 + q * 4);
          av[r][0] = t.x; av[r][1] = t.y; av[r][2] = t.z; av[r][3] = t.w;
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) av[r][s] = As[((8 * r + 4 * lh + s) ^ lh) * 32 + lr];
        }
        if constexpr (BKC) {
          const float4 u = *reinterpret_cast<const float4*>(Bs + lr * 32 + q * 4);
          bv[r][0] = u.x; bv[r][1] = u.y; bv[r][2] = u.z; bv[r][3] = u.w;
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) bv[r][s] = Bs[((8 * r + 4 * lh + s) ^ lh) * 32 + lr];
        }
      }
    };
    f32x16 acc2;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      acc2[q] = 0.f;
      acc[0][0][q] = 0.f;
    }
    auto mma = [&](const float (&av)[R][4], const float (&bv)[R][4]) {
#if DDL_MFMA_PRIO
      __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          if constexpr (NCH == 2) {
            if (s & 1) acc2 = mfma32x32x2(av[r][s], bv[r][s], acc2);
            else acc[0][0] = mfma32x32x2(av[r][s], bv[r][s], acc[0][0]);
          } else {
            acc[0][0] = mfma32x32x2(av[r][s], bv[r][s], acc[0][0]);
          }
        }
#if DDL_MFMA_PRIO
      __builtin_amdgcn_s_setprio(0);
#endif
    };
    if (nk > 0) {
      float a0[R][4], b0[R][4];
      dma(kb);
      for (int kt = 0; kt < nk; ++kt) {
        vm_wait<0>();   // tile kt is in the image
        patch(kb + kt * BK);
        rd(a0, b0);
        lgkm_wait0();   // its fragments are in registers: the image may be restaged
        if (kt + 1 < nk) dma(kb + (kt + 1) * BK);
        mma(a0, b0);
      }
    }
    if constexpr (NCH == 2) acc[0][0] += acc2;
  }

  // One-wave 32x32x32 tile on v_mfma_f32_16x16x4_f32 (variant 1).  The
  // 32x32 tile is four 16x16 sub-tiles, each with its own 4-register accumulator: 16
  // accumulator registers instead of the 32 of two 32x32 chains, and four independent
  // accumulation chains (consecutive MFMAs never depend on each other), so the wave fits in
  // <= 96 VGPR+AGPR with LDS-DMA staging (no staging registers) — 5 waves per SIMD with the 8 KB
  // image, where the 32x32x2 tiles sit at 3.
  //  * k assignment: MFMA step s (0..7) of a K tile feeds k = 8h + s from lane group h = l >> 4
  //    (the MFMA's own k index is h), so a lane's A / B values of a whole tile are 8
  //    consecutive k — two ds_read_b128 per row for a K-contiguous operand.
  //  * images: K-contiguous operand as mainloop_dma (quad q of row r at q ^ ((r >> 1) & 7): the
  //    16 rows of a read hit 16 distinct bank groups).  MN-contiguous operand [k][32 mn] with
  //    logical k-row k at physical row k ^ ((k >> 4) & 1) and its two 16-column halves swapped
  //    when bit 3 of k is set: the four lane groups of one ds_read_b32 (k = s, 8+s, 16+s, 24+s)
  //    then read four distinct 16-bank windows.  The DMA writes lane-linearly, so both layouts
  //    are made on the gather side (slot (row, quad) fetches the logical element it holds).
  //  * the accumulators are re-laid out through LDS into the 32x32 MFMA layout at the end of
  //    the tile (4 ds_write_b128 + 4 ds_read_b128 per lane, column-major image with pitch 36),
  //    so epilogues, split-K partials and the wide reduce are unchanged.
  static DDL_DEV void mainloop_dma16(const P& p, int m_blk, int n_blk, int kb, int ke, float* lds,
                                     f32x16 (&acc)[TM][TN], const Win& w) {
    static_assert(FA == 4 && FB == 4, "32x32x32 one-wave tile");
    static_assert(!(HasOnesA<P>::value && AK), "ones-row patch: MN-contiguous A");
    const int lane = threadIdx.x & 63;
    const int nk = (ke - kb + BK - 1) / BK;
    // gather side: DMA slot sl = it * 64 + lane is image quad sl (row sl >> 3, quad sl & 7)
    auto kc_of = [](int sl, int& row, int& kk) {  // K-contiguous: (mn row, k offset)
      row = sl >> 3;
      kk = ((sl & 7) ^ ((row >> 1) & 7)) * 4;
    };
    auto mn_of = [](int sl, int& mn, int& k) {  // MN-contiguous: (mn offset, k row)
      const int pr = sl >> 3;
      k = pr ^ ((pr >> 4) & 1);
      mn = ((sl & 7) ^ (((k >> 3) & 1) << 2)) * 4;
    };
    typename P::AInfo ai[4];
    typename P::BInfo bi[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int sl = it * 64 + lane;
      int x, y;
      if constexpr (AK) { kc_of(sl, x, y); ai[it] = p.prepA(m_blk + x, y); }
      else { mn_of(sl, x, y); ai[it] = p.prepA(m_blk + x, y); }
      if constexpr (BKC) { kc_of(sl, x, y); bi[it] = p.prepB(n_blk + x, y); }
      else { mn_of(sl, x, y); bi[it] = p.prepB(n_blk + x, y); }
    }
    auto patch = [&](int k0) {
      if constexpr (HasOnesA<P>::value) {
#pragma unroll
        for (int it = 0; it < 4; ++it)
          if (p.ones_group(ai[it])) lds[(it * 64 + lane) * 4] = p.ones_value(ai[it], k0, w);
      }
    };
    const uint32_t base = lds_addr(lds);
    auto dma = [&](int k0) {
#pragma unroll
      for (int it = 0; it < 4; ++it) dma16(srcA(p, ai[it], k0, w), base + it * 1024);
#pragma unroll
      for (int it = 0; it < 4; ++it) dma16(srcB(p, bi[it], k0, w), base + 4096 + it * 1024);
    };
    // read side: lane (h = lane >> 4, c = lane & 15) of sub-tile row / column block i
    const int h = lane >> 4, c = lane & 15;
    auto rd = [&](const float* img, bool kcontig, float (&v)[2][8]) {
      if (kcontig) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int row = i * 16 + c, sw = (row >> 1) & 7;
          const float4 lo = *reinterpret_cast<const float4*>(img + row * 32 + ((2 * h) ^ sw) * 4);
          const float4 hi =
              *reinterpret_cast<const float4*>(img + row * 32 + ((2 * h + 1) ^ sw) * 4);
          v[i][0] = lo.x; v[i][1] = lo.y; v[i][2] = lo.z; v[i][3] = lo.w;
          v[i][4] = hi.x; v[i][5] = hi.y; v[i][6] = hi.z; v[i][7] = hi.w;
        }
      } else {
        // k = 8h + s sits at physical row 8h + (s ^ (h >> 1)), column (16i + c) ^ 16 (h & 1)
        const int t = h >> 1;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int col = (i * 16 + c) ^ ((h & 1) << 4);
#pragma unroll
          for (int s2 = 0; s2 < 8; ++s2) v[i][s2] = img[(8 * h + (s2 ^ t)) * 32 + col];
        }
      }
    };
    f32x4 c4[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) c4[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (nk > 0) {
      float av[2][8], bv[2][8];
      dma(kb);
      for (int kt = 0; kt < nk; ++kt) {
        vm_wait<0>();  // tile kt is in the image
        patch(kb + kt * BK);
        rd(lds, AK, av);
        rd(lds + 1024, BKC, bv);
        lgkm_wait0();  // its fragments are in registers: the image may be restaged
        if (kt + 1 < nk) dma(kb + (kt + 1) * BK);
#if DDL_MFMA_PRIO
        __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
        for (int s2 = 0; s2 < 8; ++s2)
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) c4[i][j] = mfma16x16x4(av[i][s2], bv[j][s2], c4[i][j]);
#if DDL_MFMA_PRIO
        __builtin_amdgcn_s_setprio(0);
#endif
      }
    }
    // 16x16 layout (lane: column 16j + c, rows 16i + 4h .. +3) -> 32x32 layout (lane: column
    // l & 31, rows 8g + 4 (l >> 5) .. +3), through a column-major [32][36] image
    constexpr int PC = 36;
    lgkm_wait0();
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        *reinterpret_cast<float4*>(lds + (16 * j + c) * PC + 16 * i + 4 * h) =
            make_float4(c4[i][j][0], c4[i][j][1], c4[i][j][2], c4[i][j][3]);
    const int col = lane & 31, lh = lane >> 5;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 t = *reinterpret_cast<const float4*>(lds + col * PC + 8 * g + 4 * lh);
      acc[0][0][4 * g] = t.x; acc[0][0][4 * g + 1] = t.y;
      acc[0][0][4 * g + 2] = t.z; acc[0][0][4 * g + 3] = t.w;
    }
    lgkm_wait0();  // the image is free again (split-K flag word, the next tile's DMA)
  }

  // LDS-DMA loop of a one-wave tile with TM x TN fragments (K-contiguous A: BM rows of 8 quads,
  // quad q of row r at q ^ ((r >> 1) & 7); MN-contiguous B, BN = 64: k-row k of 16 quads, the
  // two 32-column halves swapped on rows with bit 2 set, so the lane halves' reads of rows k and
  // k + 4 land in opposite bank halves).  One image: tile t+1 is DMA'd once tile t's fragments
  // are in registers, under tile t's TM*TN*16 MFMAs.  Same MFMA order as mainloop_basic.
  static DDL_DEV void mainloop_dma_mf(const P& p, int m_blk, int n_blk, int kb, int ke,
                                      float* lds, f32x16 (&acc)[TM][TN], const Win& w) {
    constexpr int NDA = BM * BK / 4 / 64, NDB = BK * BN / 4 / 64;  // 1 KB DMAs per tile
    const int lane = threadIdx.x & 63;
    const int lr = lane & 31, lh = lane >> 5;
    const int nk = (ke - kb + BK - 1) / BK;
    typename P::AInfo ai[NDA];
    typename P::BInfo bi[NDB];
#pragma unroll
    for (int it = 0; it < NDA; ++it) {
      const int sl = it * 64 + lane, row = sl >> 3, q = sl & 7;
      ai[it] = p.prepA(m_blk + row, (q ^ ((row >> 1) & 7)) * 4);
    }
#pragma unroll
    for (int it = 0; it < NDB; ++it) {
      const int sl = it * 64 + lane, k = sl >> 4, q = sl & 15;
      bi[it] = p.prepB(n_blk + (q ^ (((k >> 2) & 1) << 3)) * 4, k);
    }
    const uint32_t base = lds_addr(lds);
    auto dma = [&](int k0) {
#pragma unroll
      for (int it = 0; it < NDA; ++it) dma16(srcA(p, ai[it], k0, w), base + it * 1024);
#pragma unroll
      for (int it = 0; it < NDB; ++it)
        dma16(srcB(p, bi[it], k0, w), base + BM * BK * 4 + it * 1024);
    };
    const float* As = lds;
    const float* Bs = lds + BM * BK;
    float av[R][TM][4], bv[R][TN][4];
    auto rd = [&]() {
#pragma unroll
      for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = i * 32 + lr;
          const int q = (2 * r + lh) ^ ((row >> 1) & 7);
          const float4 t = *reinterpret_cast<const float4*>(As + row * BK + q * 4);
          av[r][i][0] = t.x; av[r][i][1] = t.y; av[r][i][2] = t.z; av[r][i][3] = t.w;
        }
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const int k = 8 * r + 4 * lh + s;
            bv[r][j][s] = Bs[k * BN + ((j * 32 + lr) ^ (((k >> 2) & 1) << 5))];
          }
      }
    };
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
    if (nk <= 0) return;
    dma(kb);
    for (int kt = 0; kt < nk; ++kt) {
      vm_wait<0>();   // tile kt is in the image
      rd();
      lgkm_wait0();   // its fragments are in registers: the image may be restaged
      if (kt + 1 < nk) dma(kb + (kt + 1) * BK);
#if DDL_MFMA_PRIO
      __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = mfma32x32x2(av[r][i][s], bv[r][j][s], acc[i][j]);
#if DDL_MFMA_PRIO
      __builtin_amdgcn_s_setprio(0);
#endif
    }
  }

  static DDL_DEV void mainloop_basic(const P& p, int m_blk, int n_blk, int kb, int ke,
                                     float* lds, f32x16 (&acc)[TM][TN], const Win& w) {
    float* const As0 = lds;
    float* const Bs0 = lds + NBUF * A_ELEMS;
    const int tid = threadIdx.x & (NT - 1);  // a one-wave tile may be one wave of a larger block
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int nk = (ke - kb + BK - 1) / BK;

    // Loader protocol: prepX(mn, kk) fixes a thread's row/column (group) and its k offset
    // inside every K tile; loadX(info, k0) gathers at tile base k0 (wave-uniform, a multiple
    // of BK = 32), so per-tile index math that depends only on k0 runs on the scalar unit.
    typename P::AInfo ai[FA];
    typename P::BInfo bi[FB];
    int a_off[FA], b_off[FB];
#pragma unroll
    for (int it = 0; it < FA; ++it) {
      const int idx = tid + it * NT;
      if constexpr (AK) {
        const int kq = idx % (BK / 4), row = idx / (BK / 4);
        ai[it] = p.prepA(m_blk + row, kq * 4);
        a_off[it] = row * SA + kq * 4;
      } else {
        const int mq = idx % (BM / 4), kk = idx / (BM / 4);
        ai[it] = p.prepA(m_blk + mq * 4, kk);
        a_off[it] = kk * SA + mq * 4;
      }
    }
#pragma unroll
    for (int it = 0; it < FB; ++it) {
      const int idx = tid + it * NT;
      if constexpr (BKC) {
        const int kq = idx % (BK / 4), row = idx / (BK / 4);
        bi[it] = p.prepB(n_blk + row, kq * 4);
        b_off[it] = row * SB + kq * 4;
      } else {
        const int nq = idx % (BN / 4), kk = idx / (BN / 4);
        bi[it] = p.prepB(n_blk + nq * 4, kk);
        b_off[it] = kk * SB + nq * 4;
      }
    }

    // Two register-prefetch stages of the global operands: K tile t+1 is stored to LDS
    // while tile t's fragments are already in VGPRs, and tile t+2 loads during t's MFMAs.
    float4 ra[FA], rb[FB];
    auto gload = [&](int k0) {
#pragma unroll
      for (int it = 0; it < FA; ++it) ra[it] = ldA(p, ai[it], k0, w);
#pragma unroll
      for (int it = 0; it < FB; ++it) rb[it] = ldB(p, bi[it], k0, w);
    };
    auto sstore = [&](int buf) {
      float* As = As0 + buf * A_ELEMS;
      float* Bs = Bs0 + buf * B_ELEMS;
#pragma unroll
      for (int it = 0; it < FA; ++it) *reinterpret_cast<float4*>(As + a_off[it]) = ra[it];
#pragma unroll
      for (int it = 0; it < FB; ++it) *reinterpret_cast<float4*>(Bs + b_off[it]) = rb[it];
    };

    f32x16 acc2;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc2[q] = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;

    const int lr = lane & 31;   // fragment row / column
    const int lh = lane >> 5;   // k half

    // fragment fetch of a whole K tile from LDS buffer (As, Bs), issued as one burst so the
    // LDS latency is paid once per tile
    float av[R][TM][4], bv[R][TN][4];
    auto fetch_all = [&](const float* As, const float* Bs) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wm * WTM + i * 32 + lr;
          if constexpr (AK) {
            const float4 t = *reinterpret_cast<const float4*>(As + row * SA + r * 8 + 4 * lh);
            av[r][i][0] = t.x; av[r][i][1] = t.y; av[r][i][2] = t.z; av[r][i][3] = t.w;
          } else {
#pragma unroll
            for (int s = 0; s < 4; ++s) av[r][i][s] = As[(r * 8 + 4 * lh + s) * SA + row];
          }
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = wn * WTN + j * 32 + lr;
          if constexpr (BKC) {
            const float4 t = *reinterpret_cast<const float4*>(Bs + col * SB + r * 8 + 4 * lh);
            bv[r][j][0] = t.x; bv[r][j][1] = t.y; bv[r][j][2] = t.z; bv[r][j][3] = t.w;
          } else {
#pragma unroll
            for (int s = 0; s < 4; ++s) bv[r][j][s] = Bs[(r * 8 + 4 * lh + s) * SB + col];
          }
        }
      }
    };

    if (nk > 0) {
      gload(kb);
      sstore(0);
      if (nk > 1) gload(kb + BK);
    }
    if constexpr (!SOLO) __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = SOLO ? 0 : (kt & 1);
      fetch_all(As0 + cur * A_ELEMS, Bs0 + cur * B_ELEMS);
      // (SOLO) overwriting the buffer just read is safe: a wave's LDS ops run in order;
      // with two buffers the previous iteration's barrier freed buffer cur^1.
      // One-wave blocks stage tile kt+1 AFTER tile kt's MFMAs (below): issued before them, the
      // LDS writes' vmcnt waits for tile kt+1's global loads sat in front of the MFMA cluster
      // (its lgkmcnt wait covers the writes), so every K tile paid the load latency again
      // (0.3135 -> 0.3098 ms/step).
      if constexpr (!SOLO) {
        if (kt + 1 < nk) sstore(SOLO ? 0 : (cur ^ 1));
        if (kt + 2 < nk) gload(kb + (kt + 2) * BK);
      }
      __builtin_amdgcn_sched_barrier(0);
#if DDL_MFMA_PRIO
      __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          if constexpr (NCH == 2) {
            if (s & 1) acc2 = mfma32x32x2(av[r][0][s], bv[r][0][s], acc2);
            else acc[0][0] = mfma32x32x2(av[r][0][s], bv[r][0][s], acc[0][0]);
          } else {
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
              for (int j = 0; j < TN; ++j)
                acc[i][j] = mfma32x32x2(av[r][i][s], bv[r][j][s], acc[i][j]);
          }
        }
#if DDL_MFMA_PRIO
      __builtin_amdgcn_s_setprio(0);
#endif
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (SOLO) {
        if (kt + 1 < nk) sstore(0);
        if (kt + 2 < nk) gload(kb + (kt + 2) * BK);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (!SOLO) __syncthreads();
    }
    if constexpr (NCH == 2) acc[0][0] += acc2;
  }

  // fused epilogue: each lane owns 4 groups of 4 consecutive rows of one column
  static DDL_DEV void epilogue(const P& p, int m_blk, int n_blk, const f32x16 (&acc)[TM][TN]) {
    const int lane = threadIdx.x & 63, wave = (threadIdx.x & (NT - 1)) >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int lr = lane & 31, lh = lane >> 5;
    if constexpr (HasEpiT<P>::value) {
      // row-wise: lane quad (columns 4k .. 4k+3, one row group) transposed so lane k of the
      // quad holds row m0 + k, columns 4k' .. 4k'+3 — one 16-byte store where the column-wise
      // epilogue issued four 4-byte ones (every lane active here: the guards follow the DPP)
      const int qi = lane & 3;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x16& v = acc[i][j];
            const float4 t = quad_transpose(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3], qi);
            const int n0 = n_blk + wn * WTN + j * 32 + (lr & ~3);
            const int m = m_blk + wm * WTM + i * 32 + 8 * g + 4 * lh + qi;
            if (n0 < p.N && m < p.M) p.epi_t(m, n0, t);
          }
      return;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n_blk + wn * WTN + j * 32 + lr;
        if (n >= p.N) continue;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int m0 = m_blk + wm * WTM + i * 32 + 8 * g + 4 * lh;
          if (m0 < p.M) {
            const f32x16& v = acc[i][j];
            p.epi(m0, n, f32x4{v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]});
          }
        }
      }
    }
  }

  // partial-fragment image of one block: [wave][frag][g][lane] float4 (coalesced per wave),
  // at float4 index `base` of the slab.  Written and read write-through (sc1): see arrive().
  static DDL_DEV void store_partial(brsrc_t slab, size_t base, const f32x16 (&acc)[TM][TN]) {
    const int mine = (int)base + ((threadIdx.x & (NT - 1)) >> 6) * WPART + (threadIdx.x & 63);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x16& v = acc[i][j];
          bstore4_sc1(slab, (mine + ((i * TN + j) * 4 + g) * 64) * 16,
                      make_float4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]));
        }
  }
  static DDL_DEV void add_partial(brsrc_t slab, size_t base, f32x16 (&acc)[TM][TN]) {
    const int src = (int)base + ((threadIdx.x & (NT - 1)) >> 6) * WPART + (threadIdx.x & 63);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 t = bload4_sc1(slab, (src + ((i * TN + j) * 4 + g) * 64) * 16);
          acc[i][j][4 * g] += t.x; acc[i][j][4 * g + 1] += t.y;
          acc[i][j][4 * g + 2] += t.z; acc[i][j][4 * g + 3] += t.w;
        }
  }
  // The last arriver's sum of the gz partials at base0 + z * zstride, in z order (bit-identical
  // to zero() + one add_partial per z) with the loads of ZB partials in flight per round: one
  // add_partial per z waits a full sc1-load latency per partial, so a 12-way split's last
  // arriver spent ~12 load round trips in its epilogue — the longest block of the launch.
  static constexpr int kZB = DDL_SPLITK_ZB;  // partials in flight per round, one-fragment tile
  static constexpr int ZB = TM * TN >= kZB ? 1 : kZB / (TM * TN);
  static DDL_DEV void sum_partials(brsrc_t slab, size_t base0, size_t zstride, int gz,
                                   f32x16 (&acc)[TM][TN]) {
    zero(acc);
    const int lane_off = ((threadIdx.x & (NT - 1)) >> 6) * WPART + (threadIdx.x & 63);
    int z = 0;
    if constexpr (ZB > 1) {
      // the last round is a partial batch too (its missing partials add 0), so a split of up
      // to ZB partials is ONE load round trip and g partials take ceil(g / ZB)
      for (; z < gz; z += ZB) {
        float4 t[ZB][TM][TN][4];
#pragma unroll
        for (int b = 0; b < ZB; ++b) {
          const int src = (int)(base0 + (size_t)(z + b) * zstride) + lane_off;
          const bool have = z + b < gz;  // wave-uniform
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
              for (int g = 0; g < 4; ++g)
                t[b][i][j][g] = have ? bload4_sc1(slab, (src + ((i * TN + j) * 4 + g) * 64) * 16)
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int b = 0; b < ZB; ++b)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
              for (int g = 0; g < 4; ++g) {
                acc[i][j][4 * g] += t[b][i][j][g].x; acc[i][j][4 * g + 1] += t[b][i][j][g].y;
                acc[i][j][4 * g + 2] += t[b][i][j][g].z; acc[i][j][4 * g + 3] += t[b][i][j][g].w;
              }
      }
    }
    for (; z < gz; ++z) add_partial(slab, base0 + (size_t)z * zstride, acc);  // (ZB == 1)
  }
  static DDL_DEV void zero(f32x16 (&acc)[TM][TN]) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
  }

  // In-launch hand-off of partial tiles (MI355X guide §6 Guideline 16, sc1 form): the
  // partials were stored write-through (sc1), so publishing is just every wave draining its
  // stores, the block barrier and ONE relaxed agent-scope ticket add — no release fence
  // (an agent release writes back the XCD's whole L2, which serialised many-worker launches).
  // The last of `count` arrivers reads every partial with sc1 loads (they bypass this CU's
  // L1), so it needs no acquire fence; it re-arms the ticket and tells its block via LDS
  // (the flag lives in the kernel's single __shared__ array: guide §5 trap 4a).
  static DDL_DEV bool arrive(int* ticket, int count, int* flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const int prev = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
      const int last = prev == count - 1;
      if (last) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = last;
    }
    __syncthreads();
    const bool last = *flag != 0;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the slab loads below
    __syncthreads();  // flag may be rewritten by the next arrive of this block
    return last;
  }
};

// ---- drivers ------------------------------------------------------------------------------
// Each driver is a device-function body over a *virtual* block id, so a kernel can host one
// problem (gemm_f32_kernel) or two independent problems side by side
// (gemm_dual_kernel: the data- and weight-gradient GEMMs of one layer in ONE launch — their
// concurrency without a second stream, whose cross-queue event waits cost tens of us).
// `lds` is the block's staging array (>= GemmTile::LDS_F4 float4), `flag` one int of LDS.

// Classic split-K: virtual grid (gx, gy, gz); split bz covers K range
// [bz*kchunk, (bz+1)*kchunk).  mode 0: no split; mode 1: in-launch last-arriver reduction of
// the gz partials (in z order, deterministic); mode 2: partials only (splitk_wide_reduce).
template <int BM, int BN, int BK, int WM, int WN, class P, int V = 0>
DDL_DEV int splitk_body(const P& p, int kchunk, int mode, float4* __restrict__ slab,
                         int* __restrict__ tickets, int bx, int by, int bz, int gx, int gy,
                         int gz, float* lds, int* flag, unsigned long long* mid = nullptr) {
  using T = GemmTile<BM, BN, BK, WM, WN, P, V>;
  using G = typename T::G;
  const int m_blk = bx * BM;
  const int n_blk = by * BN;
  f32x16 acc[T::TM][T::TN];
  int nkt;  // K tiles this block runs (diagnostics)
  if constexpr (T::KM) {
    // this tile's useful K sub-space, divided over the gz splits (whole BK tiles)
    const typename T::Win w = p.kwin(m_blk, min(p.M, m_blk + BM));
    const int kv = p.kvlen(w);
    // (one chunk length sized by the longest window instead, heavy tiles getting more waves
    // than light ones: measured 0.3056 -> 0.3098-0.3167 ms/step, docs/DESIGN.md)
    const int kc = gz > 1 ? ((kv + gz - 1) / gz + BK - 1) / BK * BK : kv;
    const int kb = bz * kc;
    nkt = (max(0, min(kv, kb + kc) - kb) + BK - 1) / BK;
    T::mainloop(p, m_blk, n_blk, kb, min(kv, kb + kc), lds, acc, w);
  } else {
    const int kb = bz * kchunk;
    const int ke = min(p.K, kb + kchunk);
    nkt = (max(0, ke - kb) + BK - 1) / BK;
    T::mainloop(p, m_blk, n_blk, kb, ke, lds, acc);
  }
#if DDL_STAMPS
  if (mid) mid[0] = __builtin_amdgcn_s_memrealtime();  // main loop done
#else
  (void)mid;
#endif
  if (mode != 0) {
    const int tile = by * gx + bx;
    const int ntiles = gx * gy;
    const brsrc_t sr = make_rsrc(slab, (uint32_t)(gz * ntiles * G::PART4 * 16u));
    T::store_partial(sr, ((size_t)bz * ntiles + tile) * G::PART4, acc);
    if (mode == 2) return nkt;
    const bool last = T::arrive(&tickets[tile], gz, flag);
#if DDL_STAMPS
    if (mid) mid[1] = __builtin_amdgcn_s_memrealtime();  // partial stored, ticket back
#endif
    if (!last) return nkt;
    T::sum_partials(sr, (size_t)tile * G::PART4, (size_t)ntiles * G::PART4, gz, acc);
  }
  T::epilogue(p, m_blk, n_blk, acc);
  return nkt | (1 << 20);  // (bit 20: this block ran the epilogue — diagnostics, stamps.h)
}

// Launch geometry of one GEMM problem under its schedule (host-computed, passed by value).
// (Stream-K schedules — uniform and over the tap-window K maps — won conv launches in rounds
// 1-2 and lost every one to split-K after the tap windows and dual launches; the stream-K body
// also raised the dual kernels' register count, 120 -> 132 = 4 -> 3 waves per SIMD, and was
// removed in round 6: docs/DESIGN.md.)
struct SubGrid {
  int nblocks = 0;   // blocks (virtual ids 0..nblocks-1)
  int gx = 1, gy = 1, gz = 1;
  int kchunk = 0, mode = 0;  // split-K
  float4* slab = nullptr;
  int* tickets = nullptr;
#if DDL_STAMPS
  unsigned long long* stamps = nullptr;  // diagnostic build: per-block timestamps (stamps.h)
#endif
};

// virtual block vb -> (bx, by, bz): bx fastest, then by, then bz.  The hardware deals a launch's
// blocks round-robin over the 8 XCDs; XCD-contiguous renumberings (each XCD's L2 holding a band
// of the maps) measured +0.2 to +13 us/step and were removed (docs/DESIGN.md rounds 2 and 5)
DDL_DEV void split_coords(const SubGrid& g, int vb, int& bx, int& by, int& bz) {
  bx = vb % g.gx;
  const int t = vb / g.gx;
  by = t % g.gy;
  bz = t / g.gy;
}

// Split-K blocks keep the hardware's round-robin XCD placement (block b on XCD b % 8): with
// tap windows the per-tile cost depends on the position, and contiguous ranges would hand one
// XCD all the heavy centre tiles (docs/DESIGN.md).
template <int BM, int BN, int BK, int WM, int WN, class P, int V = 0>
DDL_DEV void run_sub(const P& p, const SubGrid& g, int vb, float* lds, int* flag) {
  int bx, by, bz;
  split_coords(g, vb, bx, by, bz);
#if DDL_STAMPS
  const Stamp st0 = stamp_now();
  unsigned long long mid[2] = {0, 0};
  const int nkt = splitk_body<BM, BN, BK, WM, WN, P, V>(p, g.kchunk, g.mode, g.slab, g.tickets,
                                                        bx, by, bz, g.gx, g.gy, g.gz, lds, flag,
                                                        mid);
  stamp_block(g.stamps, vb, st0, nkt, bx, by, bz, mid);
#else
  const int nkt = splitk_body<BM, BN, BK, WM, WN, P, V>(p, g.kchunk, g.mode, g.slab, g.tickets,
                                                        bx, by, bz, g.gx, g.gy, g.gz, lds, flag);
  (void)nkt;
#endif
}

// (No amdgpu_waves_per_eu occupancy hints: forcing 4 waves per SIMD on the 32x32x2 tiles
// measured slower on every driver — tighter schedules and small spills cost more than the
// extra wave hides; the 16x16x4 tile reaches 5 waves by its register budget instead.)
template <int BM, int BN, int BK, int WM, int WN, class P, int V = 0>
__global__ void __launch_bounds__(WM * WN * 64)
gemm_f32_kernel(P p, int kchunk, int mode, float4* __restrict__ slab, int* __restrict__ tickets
#if DDL_STAMPS
                , unsigned long long* stamps
#endif
) {
  using T = GemmTile<BM, BN, BK, WM, WN, P, V>;
  // staging images; the last-arriver flag reuses the first word (arrive() runs after the main
  // loop, whose last LDS reads have retired) — one array (guide §5 trap 4a), and no extra 16 B
  // that would push an 8 / 16 KB LDS-DMA block past an occupancy step
  __shared__ float4 lds4[T::LDS_F4 > 0 ? T::LDS_F4 : 1];
  const int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
#if DDL_STAMPS
  const Stamp st0 = stamp_now();
  unsigned long long mid[2] = {0, 0};
#else
  unsigned long long* mid = nullptr;
#endif
  const int nkt = splitk_body<BM, BN, BK, WM, WN, P, V>(
      p, kchunk, mode, slab, tickets, bx, by, bz, gridDim.x, gridDim.y, gridDim.z,
      reinterpret_cast<float*>(lds4), reinterpret_cast<int*>(lds4), mid);
#if DDL_STAMPS
  stamp_block(stamps, blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z), st0, nkt,
              bx, by, bz, mid);
#else
  (void)nkt;
#endif
}

// (Blocks running several work items in turn — DDL_FWD_ITEMS — measured 5.7-18 us/step slower on
// the conv forwards and were removed in round 6: docs/DESIGN.md.)

// K split inside ONE workgroup, for the skinny GEMMs (the fc layers at M = batch): KW waves each
// run the one-wave 32x32 tile over 1/KW of the K range (own LDS staging image, no barriers),
// then the KW accumulators are summed through LDS in wave order (deterministic) and the fused
// epilogue runs in the same launch — no partial slab in HBM and no reduce launch, where the
// split-K form of the same tile needs a partial round trip plus a dependent kernel boundary.
// One K-wave tile (bx, by) by the KW waves of this workgroup; wave w stages through the L
// float4 at lds4 + w * L (L >= the tile's LDS_F4, >= 1024 floats for the reduction image).
template <int BK, int KW, class P>
DDL_DEV void kwave_body(const P& p, int bx, int by, float4* lds4, int L) {
  using T = GemmTile<32, 32, BK, 1, 1, P>;
  static_assert(KW == 4 || KW == 8 || KW == 16, "4, 8 or 16 waves");
  // (wave-uniform by construction; readfirstlane tells the compiler, so the LDS-DMA main loop
  // gets its image address in an SGPR)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int m_blk = bx * 32, n_blk = by * 32;
  float* mine = reinterpret_cast<float*>(lds4 + wave * L);
  f32x16 acc[1][1];
  if constexpr (T::KM) {
    const typename T::Win w = p.kwin(m_blk, min(p.M, m_blk + 32));
    const int kv = p.kvlen(w);
    const int kc = ((kv + KW - 1) / KW + BK - 1) / BK * BK;
    const int kb = wave * kc;
    T::mainloop(p, m_blk, n_blk, kb, min(kv, kb + kc), mine, acc, w);
  } else {
    const int kc = ((p.K + KW - 1) / KW + BK - 1) / BK * BK;
    const int kb = wave * kc;
    T::mainloop(p, m_blk, n_blk, kb, min(p.K, kb + kc), mine, acc);
  }
  __syncthreads();  // every wave is past its staging reads: the images become the sum buffer
  float* red = reinterpret_cast<float*>(lds4);
#pragma unroll
  for (int q = 0; q < 16; ++q) red[(wave * 16 + q) * 64 + lane] = acc[0][0][q];
  __syncthreads();
  if (wave < 4) {  // wave g finishes row group g (accumulator registers 4g..4g+3) of every lane
    const int g = wave;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    for (int ww = 0; ww < KW; ++ww)
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] += red[(ww * 16 + 4 * g + j) * 64 + lane];
    const int n = n_blk + (lane & 31);
    const int m0 = m_blk + 8 * g + 4 * (lane >> 5);
    if constexpr (HasEpiT<P>::value) {  // row-wise (GemmTile::epilogue): whole wave active here
      const int qi = lane & 3;
      const float4 t = quad_transpose(v[0], v[1], v[2], v[3], qi);
      if (n - qi < p.N && m0 + qi < p.M) p.epi_t(m0 + qi, n - qi, t);
    } else {
      if (n < p.N && m0 < p.M) p.epi(m0, n, f32x4{v[0], v[1], v[2], v[3]});
    }
  }
}

template <int BK, int KW, class P>
__global__ void __launch_bounds__(KW * 64) gemm_kwave_kernel(P p) {
  using T = GemmTile<32, 32, BK, 1, 1, P>;
  // per wave: its staging image (none on the direct-fragment loop) and its 16x64-float
  // reduction image
  constexpr int LW = T::LDS_F4 > 256 ? T::LDS_F4 : 256;
  __shared__ float4 lds4[KW * LW];
  kwave_body<BK, KW, P>(p, blockIdx.x, blockIdx.y, lds4, LW);
}

// Packed dual launch for the fc backward (KW-wave workgroups): blocks [0, nA) run problem A —
// the data gradient, M = batch — as K-wave tiles (no partial slab, no reduce launch); blocks
// [nA, nA + nB) run KW independent one-wave 32x32 tiles of problem B — the weight gradient,
// K = batch, unsplit — one per wave; the rest run the auxiliary work (fc3 weight gradient /
// optimizer tail), one index per wave.  Replaces the one-wave dual launch + A's wide reduce.
template <int KW, class PA, class PB, class AUX>
__global__ void __launch_bounds__(KW * 64)
gemm_pack_kernel(PA pa, int nA, int gxA, PB pb, int nB, int gxB, int ntB, AUX ut) {
  using TA = GemmTile<32, 32, 32, 1, 1, PA>;
  using TB = GemmTile<32, 32, 32, 1, 1, PB>;
  constexpr int L0 = TA::LDS_F4 > TB::LDS_F4 ? TA::LDS_F4 : TB::LDS_F4;
  constexpr int L = L0 > 256 ? L0 : 256;
  __shared__ float4 lds4[KW * L];
  const int b = blockIdx.x, wave = threadIdx.x >> 6;
  if (b < nA) {
    kwave_body<32, KW, PA>(pa, b % gxA, b / gxA, lds4, L);
  } else if (b < nA + nB) {
    const int t = (b - nA) * KW + wave;
    if (t >= ntB) return;
    const int m_blk = (t % gxB) * 32, n_blk = (t / gxB) * 32;
    f32x16 acc[1][1];
    TB::mainloop(pb, m_blk, n_blk, 0, pb.K, reinterpret_cast<float*>(lds4 + wave * L), acc);
    TB::epilogue(pb, m_blk, n_blk, acc);
  } else {
    const int i = (b - nA - nB) * KW + wave;
    if (i < ut.nblk) ut.run(i);
  }
}

template <int KW, class PA, class PB, class AUX>
inline void launch_gemm_pack_w(const PA& pa, const PB& pb, const AUX& ut, hipStream_t stream) {
  const int gxA = (pa.M + 31) / 32, nA = gxA * ((pa.N + 31) / 32);
  const int gxB = (pb.M + 31) / 32, ntB = gxB * ((pb.N + 31) / 32);
  const int nB = (ntB + KW - 1) / KW, nX = (ut.nblk + KW - 1) / KW;
  if (nA + nB + nX > 0)
    DDL_LAUNCH((gemm_pack_kernel<KW, PA, PB, AUX>), dim3(nA + nB + nX), dim3(KW * 64), 0,
                       stream, pa, nA, gxA, pb, nB, gxB, ntB, ut);
}

inline int kwave_waves(int splits);

template <class PA, class PB, class AUX>
inline void launch_gemm_pack(const PA& pa, int splits_a, const PB& pb, const AUX& ut,
                             hipStream_t stream) {
  switch (kwave_waves(splits_a)) {
    case 4: launch_gemm_pack_w<4>(pa, pb, ut, stream); break;
    case 8: launch_gemm_pack_w<8>(pa, pb, ut, stream); break;
    default: launch_gemm_pack_w<16>(pa, pb, ut, stream);
  }
}

// waves per workgroup of the K-wave launch for a requested split factor
inline int kwave_waves(int splits) { return splits <= 4 ? 4 : (splits <= 8 ? 8 : 16); }

template <int BK, class P>
inline void launch_gemm_kwave(const P& p, int splits, hipStream_t stream) {
  if (p.M <= 0 || p.N <= 0) return;
  const dim3 grid((p.M + 31) / 32, (p.N + 31) / 32);
  switch (kwave_waves(splits)) {
    case 4: DDL_LAUNCH((gemm_kwave_kernel<BK, 4, P>), grid, dim3(256), 0, stream, p); break;
    case 8: DDL_LAUNCH((gemm_kwave_kernel<BK, 8, P>), grid, dim3(512), 0, stream, p); break;
    default:
      DDL_LAUNCH((gemm_kwave_kernel<BK, 16, P>), grid, dim3(1024), 0, stream, p);
  }
}

template <int BM_, int BN_, int BK_, int WM_, int WN_, int V_ = 0>
struct TileCfg {
  static constexpr int BM = BM_, BN = BN_, BK = BK_, WM = WM_, WN = WN_, V = V_;
  static constexpr int NT = WM * WN * 64;
};

// Auxiliary work riding in a dual launch: `nblk` extra one-wave blocks before (first_) or after
// the GEMM blocks, each running aux.run(block index).  The optimizer tail (tail.h) is one;
// head.h's fc3 weight gradient another.
struct TailAux {
  UpdTail t;
  int nblk = 0;
  int first_ = 0;
  TailAux() = default;
  explicit TailAux(const UpdTail& u) : t(u), nblk(u.nblocks), first_(u.first) {}
  DDL_DEV void run(int b) const { tail_body(t, b); }
};

// An aux type that needs the block's LDS staging array (AUX::LDS_F4 > 0: its GEMM tiles) is
// called as run(b, lds); the dual launch sizes its LDS for it.
template <class A, class = void>
struct AuxLds : std::integral_constant<int, 0> {};
template <class A>
struct AuxLds<A, std::void_t<decltype(A::LDS_F4)>> : std::integral_constant<int, A::LDS_F4> {};
template <class A>
DDL_DEV void run_aux(const A& ut, int b, float* lds) {
  if constexpr (AuxLds<A>::value > 0) ut.run(b, lds);
  else ut.run(b);
}

// Two independent GEMM problems in one launch: blocks [0, ga.nblocks) run problem A, the
// rest problem B.  Both must use one-wave blocks.  An optional optimizer tail (tail.h) takes
// ut.nblocks more blocks, after the GEMM blocks (ut.first = 0, measured faster: the update
// fills CUs as GEMM blocks retire) or before them (a multiple of 8 so the GEMMs' XCD-major
// numbering holds).  The tail path must stay under the GEMM paths' VGPR count: at 8 float4
// per lane it raised the conv4 dual from 113 to 149 VGPRs (3 -> 2 waves/SIMD, +9 us).
template <class CA, class PA, class CB, class PB, class AUX>
__global__ void __launch_bounds__(64)
gemm_dual_kernel(PA pa, SubGrid ga, PB pb, SubGrid gb, AUX ut, int bfirst) {
  static_assert(CA::NT == 64 && CB::NT == 64, "dual launch needs one-wave blocks");
  using TA = GemmTile<CA::BM, CA::BN, CA::BK, CA::WM, CA::WN, PA, CA::V>;
  using TB = GemmTile<CB::BM, CB::BN, CB::BK, CB::WM, CB::WN, PB, CB::V>;
  constexpr int L0 = TA::LDS_F4 > TB::LDS_F4 ? TA::LDS_F4 : TB::LDS_F4;
  constexpr int L1 = L0 > AuxLds<AUX>::value ? L0 : AuxLds<AUX>::value;
  constexpr int L = L1 > 0 ? L1 : 1;
  __shared__ float4 lds4[L];  // (the last-arriver flag in the first word: gemm_f32_kernel)
  float* lds = reinterpret_cast<float*>(lds4);
  int* flag = reinterpret_cast<int*>(lds4);
  const int gemm_blocks = ga.nblocks + gb.nblocks;
  int b = blockIdx.x;
  if (ut.first_) {
    if (b < ut.nblk) {
      run_aux(ut, b, lds);
      return;
    }
    b -= ut.nblk;
  } else if (b >= gemm_blocks) {
    run_aux(ut, b - gemm_blocks, lds);
    return;
  }
  // bfirst 1: problem B's blocks are dispatched first (longest-first ordering shortens the
  // launch's tail when B's blocks run longer); 0: A's first.  (Interleaving the two problems'
  // blocks measured slower for every layer: the blocks of one problem running together share
  // their operands in L2.)
  const bool is_a = bfirst ? (b >= gb.nblocks) : (b < ga.nblocks);
  const int ia = bfirst ? b - gb.nblocks : b;
  const int ib = bfirst ? b : b - ga.nblocks;
  if (is_a)
    run_sub<CA::BM, CA::BN, CA::BK, CA::WM, CA::WN, PA, CA::V>(pa, ga, ia, lds, flag);
  else
    run_sub<CB::BM, CB::BN, CB::BK, CB::WM, CB::WN, PB, CB::V>(pb, gb, ib, lds, flag);
}

// Output rows m0 .. m0 + 3 and column n of float4 element e of a mode-2 partial slab (the tile /
// wave / fragment / lane order the GEMM tiles store their partials in).
template <int BM, int BN, int WM, int WN>
DDL_DEV void wide_elem_coords(int e, int gx, int& m0, int& n) {
  using G = TileGeo<BM, BN, WM, WN>;
  const int tile = e / G::PART4;
  int r = e % G::PART4;
  constexpr int WPART = G::FRAGS * 4 * 64;
  const int wave = r / WPART;
  r %= WPART;
  const int fg = r / 64, lane = r % 64;
  const int frag = fg / 4, g = fg % 4;
  const int i = frag / G::TN, j = frag % G::TN;
  const int wm = wave / WN, wn = wave % WN;
  const int bx = tile % gx, by = tile / gx;
  m0 = bx * BM + wm * G::WTM + i * 32 + 8 * g + 4 * (lane >> 5);
  n = by * BN + wn * G::WTN + j * 32 + (lane & 31);
}

// Wide split-K reduce (mode 2): RL lanes cooperate on one float4 output element; `gid` is the
// global thread index (any block size that is a multiple of RL).
template <int BM, int BN, int WM, int WN, int RL, class P>
DDL_DEV void wide_reduce_body(const P& p, const float4* __restrict__ slab, int S, int gx,
                              int ntiles, int gid) {
  using G = TileGeo<BM, BN, WM, WN>;
  const int elem = gid / RL;
  const int sub = gid % RL;
  const int nelem = ntiles * G::PART4;
  const bool valid = elem < nelem;
  const int e = valid ? elem : 0;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  const size_t zstride = (size_t)ntiles * G::PART4;
  for (int z = sub; z < S; z += RL) {
    const float4 t = slab[z * zstride + e];
    s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
  }
  s.x = group_sum<RL>(s.x);  // (no lane has left yet: every lane of the wave is active)
  s.y = group_sum<RL>(s.y);
  s.z = group_sum<RL>(s.z);
  s.w = group_sum<RL>(s.w);
  if (!valid || sub != 0) return;
  int m0, n;
  wide_elem_coords<BM, BN, WM, WN>(e, gx, m0, n);
  if (n < p.N && m0 < p.M) p.epi(m0, n, f32x4{s.x, s.y, s.z, s.w});
}

template <int BM, int BN, int WM, int WN, int RL, class P>
__global__ void __launch_bounds__(256)
splitk_wide_reduce(P p, const float4* __restrict__ slab, int S, int gx, int ntiles) {
  wide_reduce_body<BM, BN, WM, WN, RL, P>(p, slab, S, gx, ntiles, blockIdx.x * 256 + threadIdx.x);
}

// The step's last launch at W = 1: the wide reduce of conv1's weight gradient (blocks
// [0, nrb); its policy's epilogue applies the optimizer to the elements it just summed, see
// layers.h WgradAdam) followed by the optimizer tail of every other range of the last
// segment (conv2: its gradients are final one launch earlier), four one-wave tail blocks per
// 256-thread block.  Replaces reduce -> stand-alone Adam launch (one dependent boundary).
template <int BM, int BN, int WM, int WN, int RL, class P>
__global__ void __launch_bounds__(256)
splitk_wide_reduce_tail(P p, const float4* __restrict__ slab, int S, int gx, int ntiles, int nrb,
                        UpdTail t) {
  if ((int)blockIdx.x < nrb) {
    wide_reduce_body<BM, BN, WM, WN, RL, P>(p, slab, S, gx, ntiles, blockIdx.x * 256 + threadIdx.x);
    return;
  }
  const int tb = ((int)blockIdx.x - nrb) * 4 + (int)(threadIdx.x >> 6);
  if (tb < t.nblocks) tail_body(t, tb);
}

// The wide reduce of one mode-2 split-K problem (R, tile geometry RBM x RBN / RWM x RWN) and
// an independent one-wave GEMM problem G in ONE launch: G's blocks, then nrb reduce blocks
// (64 threads each).  Saves a dependent kernel boundary at the end of the
// backward, where conv2's weight-gradient reduce and conv1's weight-gradient GEMM are
// independent (both need only what conv2's dual launch wrote).
template <int RBM, int RBN, int RWM, int RWN, int RL, class PR, class CG, class PG>
__global__ void __launch_bounds__(64)
reduce_gemm_kernel(PR pr, const float4* __restrict__ rslab, int S, int rgx, int rntiles, int nrb,
                   PG pg, SubGrid gg) {
  static_assert(CG::NT == 64, "one-wave GEMM blocks");
  using TG = GemmTile<CG::BM, CG::BN, CG::BK, CG::WM, CG::WN, PG, CG::V>;
  __shared__ float4 lds4[TG::LDS_F4 + 1];
  // GEMM blocks first (the longer pole: dispatched first), the reduce fills in behind them
  const int b = blockIdx.x;
  if (b >= gg.nblocks) {
    wide_reduce_body<RBM, RBN, RWM, RWN, RL, PR>(pr, rslab, S, rgx, rntiles,
                                                 (b - gg.nblocks) * 64 + threadIdx.x);
    return;
  }
  run_sub<CG::BM, CG::BN, CG::BK, CG::WM, CG::WN, PG, CG::V>(
      pg, gg, b, reinterpret_cast<float*>(lds4), reinterpret_cast<int*>(lds4 + TG::LDS_F4));
}

template <int BK>
inline int splitk_kchunk(int K, int splits) {
  if (splits <= 1) return K;
  const int per = (K + splits - 1) / splits;
  const int kc = ((per + BK - 1) / BK) * BK;
  return kc < BK ? BK : kc;
}

template <int BK>
inline int splitk_z(int K, int splits) {
  if (splits <= 1) return 1;
  const int kc = splitk_kchunk<BK>(K, splits);
  const int z = (K + kc - 1) / kc;
  return z < 1 ? 1 : z;
}

// float4 partial-slab elements a launch needs
template <int BM, int BN, int BK, int WM, int WN>
inline size_t splitk_slab_f4(int M, int N, int K, int splits) {
  const int z = splitk_z<BK>(K, splits);
  if (z <= 1) return 0;
  const size_t tiles = (size_t)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  return (size_t)z * tiles * TileGeo<BM, BN, WM, WN>::PART4;
}

// float4 partial-slab elements a launch needs
template <int BM, int BN, int BK, int WM, int WN>
inline size_t gemm_slab_f4(int M, int N, int K, int splits) {
  return splitk_slab_f4<BM, BN, BK, WM, WN>(M, N, K, splits);
}

// Schedule of one launch: split-K with `splits`: z > wide_thr uses mode 2 (separate wide reduce),
// else mode 1 (last arriver).
template <int BM, int BN, int BK, class P>
inline SubGrid plan_gemm(const P& p, int splits, int wide_thr, const SplitScratch& sc) {
  SubGrid g;
  g.slab = reinterpret_cast<float4*>(sc.slab);
  g.tickets = sc.tickets;
  if (p.M <= 0 || p.N <= 0) return g;
  g.gx = (p.M + BM - 1) / BM;
  g.gy = (p.N + BN - 1) / BN;
  g.gz = splitk_z<BK>(p.K, splits);
  g.kchunk = g.gz > 1 ? splitk_kchunk<BK>(p.K, splits) : p.K;
  g.mode = g.gz == 1 ? 0 : (g.gz > wide_thr ? 2 : 1);
  if (g.mode == 1 && (long long)g.gx * g.gy > sc.max_tiles) g.mode = 2;  // ticket capacity
  g.nblocks = g.gx * g.gy * g.gz;
  return g;
}

// The separate reduce of a mode-2 split-K launch (no-op otherwise).
template <int BM, int BN, int BK, int WM, int WN, class P>
inline void launch_reduce(const P& p, const SubGrid& g, hipStream_t stream) {
  if (g.mode != 2 || g.nblocks == 0) return;
  using G = TileGeo<BM, BN, WM, WN>;
  const int ntiles = g.gx * g.gy, z = g.gz;
  const size_t nelem = (size_t)ntiles * G::PART4;
  const float4* s4 = g.slab;
  if (z > 32) {
    const size_t th = nelem * 64;
    DDL_LAUNCH((splitk_wide_reduce<BM, BN, WM, WN, 64, P>), dim3((th + 255) / 256),
                       dim3(256), 0, stream, p, s4, z, g.gx, ntiles);
  } else if (z > 4) {
    const size_t th = nelem * 16;
    DDL_LAUNCH((splitk_wide_reduce<BM, BN, WM, WN, 16, P>), dim3((th + 255) / 256),
                       dim3(256), 0, stream, p, s4, z, g.gx, ntiles);
  } else {
    const size_t th = nelem * 4;
    DDL_LAUNCH((splitk_wide_reduce<BM, BN, WM, WN, 4, P>), dim3((th + 255) / 256),
                       dim3(256), 0, stream, p, s4, z, g.gx, ntiles);
  }
}

// launch_reduce with an optimizer tail riding behind it (splitk_wide_reduce_tail).  false
// (nothing launched) unless g is a pending mode-2 split-K reduce.
template <int BM, int BN, int BK, int WM, int WN, class P>
inline bool launch_reduce_tail(const P& p, const SubGrid& g, const UpdTail& t,
                               hipStream_t stream) {
  if (g.mode != 2 || g.nblocks == 0) return false;
  using G = TileGeo<BM, BN, WM, WN>;
  const int ntiles = g.gx * g.gy, z = g.gz;
  const size_t nelem = (size_t)ntiles * G::PART4;
  const int ntb = (t.nblocks + 3) / 4;
#define DDL_RT(RL)                                                                              \
  {                                                                                           \
    const int nrb = (int)((nelem * RL + 255) / 256);                                          \
    DDL_LAUNCH((splitk_wide_reduce_tail<BM, BN, WM, WN, RL, P>), dim3(nrb + ntb), dim3(256), 0, \
               stream, p, g.slab, z, g.gx, ntiles, nrb, t);                                   \
  }
  if (z > 32) DDL_RT(64) else if (z > 4) DDL_RT(16) else DDL_RT(4)
#undef DDL_RT
  return true;
}

template <int BM, int BN, int BK, int WM, int WN, int V = 0, class P>
inline void launch_gemm(const P& p, int splits, int wide_thr, const SplitScratch& sc,
                        hipStream_t stream, SubGrid* defer = nullptr) {
  const SubGrid g = plan_gemm<BM, BN, BK>(p, splits, wide_thr, sc);
  if (defer) *defer = g;
  if (g.nblocks == 0) return;
#if DDL_STAMPS
  unsigned long long* const stamps = stamp_slot(g.nblocks, 2, g.gx, g.gy, g.gz);
  DDL_LAUNCH((gemm_f32_kernel<BM, BN, BK, WM, WN, P, V>), dim3(g.gx, g.gy, g.gz),
                     dim3(WM * WN * 64), 0, stream, p, g.kchunk, g.mode, g.slab, g.tickets,
                     stamps);
#else
  DDL_LAUNCH((gemm_f32_kernel<BM, BN, BK, WM, WN, P, V>), dim3(g.gx, g.gy, g.gz),
             dim3(WM * WN * 64), 0, stream, p, g.kchunk, g.mode, g.slab, g.tickets);
#endif
  if (defer && g.mode == 2) return;  // the caller runs (or fuses) the wide reduce
  launch_reduce<BM, BN, BK, WM, WN, P>(p, g, stream);
}

// Launch R's pending wide reduce (SubGrid gr of a mode-2 split-K launch, tile config CR) fused
// with GEMM problem G (config CG, its own schedule/scratch); G's own mode-2 reduce follows.
// Returns false (nothing launched) when R has no pending wide reduce.
// defer_g: G's own reduce is left to the caller (its SubGrid is returned there).
template <class CR, class PR, class CG, class PG>
inline bool launch_reduce_with_gemm(const PR& pr, const SubGrid& gr, const PG& pg, int sg,
                                    int wide_g, const SplitScratch& scg, hipStream_t stream,
                                    SubGrid* defer_g = nullptr) {
  if (gr.mode != 2 || gr.nblocks == 0) return false;
  const SubGrid gg = plan_gemm<CG::BM, CG::BN, CG::BK>(pg, sg, wide_g, scg);
  if (gg.nblocks == 0) return false;
  using G = TileGeo<CR::BM, CR::BN, CR::WM, CR::WN>;
  const int ntiles = gr.gx * gr.gy, z = gr.gz;
  const size_t nelem = (size_t)ntiles * G::PART4;
  const float4* s4 = gr.slab;
#define DDL_RG(RL)                                                                            \
  {                                                                                         \
    const int nrb = (int)((nelem * RL + 63) / 64);                                          \
    DDL_LAUNCH((reduce_gemm_kernel<CR::BM, CR::BN, CR::WM, CR::WN, RL, PR, CG, PG>),  \
                       dim3(nrb + gg.nblocks), dim3(64), 0, stream, pr, s4, z, gr.gx, ntiles, nrb, \
                       pg, gg);                                                             \
  }
  if (z > 32) DDL_RG(64) else if (z > 4) DDL_RG(16) else DDL_RG(4)
#undef DDL_RG
  if (defer_g) *defer_g = gg;
  else launch_reduce<CG::BM, CG::BN, CG::BK, CG::WM, CG::WN, PG>(pg, gg, stream);
  return true;
}

// Problems A and B (one-wave tile configs CA / CB) in one launch, each with its own schedule
// and its own scratch (slab + tickets); mode-2 reduces follow on the same stream.
template <class CA, class PA, class CB, class PB, class AUX = TailAux>
inline void launch_gemm_dual(const PA& pa, int sa, const SplitScratch& sca, int wide_a,
                             const PB& pb, int sb, const SplitScratch& scb, int wide_b,
                             hipStream_t stream, const AUX& ut = AUX(),
                             SubGrid* defer_b = nullptr, int bfirst = 0) {
  SubGrid ga = plan_gemm<CA::BM, CA::BN, CA::BK>(pa, sa, wide_a, sca);
  SubGrid gb = plan_gemm<CB::BM, CB::BN, CB::BK>(pb, sb, wide_b, scb);
#if DDL_STAMPS
  ga.stamps = stamp_slot(ga.nblocks, 0, ga.gx, ga.gy, ga.gz);
  gb.stamps = stamp_slot(gb.nblocks, 1, gb.gx, gb.gy, gb.gz);
#endif
  const int n = ut.nblk + ga.nblocks + gb.nblocks;
  if (n > 0)
    DDL_LAUNCH((gemm_dual_kernel<CA, PA, CB, PB, AUX>), dim3(n), dim3(64), 0, stream, pa,
                       ga, pb, gb, ut, bfirst);
  launch_reduce<CA::BM, CA::BN, CA::BK, CA::WM, CA::WN, PA>(pa, ga, stream);
  if (defer_b) *defer_b = gb;  // the caller launches B's reduce (launch_reduce_with_gemm)
  else launch_reduce<CB::BM, CB::BN, CB::BK, CB::WM, CB::WN, PB>(pb, gb, stream);
}

}  // namespace ddl
