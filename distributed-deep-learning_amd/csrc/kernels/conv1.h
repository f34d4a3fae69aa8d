// conv1 weight gradient (Conv2DBackpropFilter + bias gradient of conv1, SURVEY.md §2.6 B10/B8
// for layer 1) as a direct kernel over LDS-staged image bands, with a deterministic two-level
// in-launch reduction, optionally sharing its launch with conv2's pending weight-gradient
// split-K reduce (gemm.h wide_reduce_body).
//
// Through the GEMM engine it is M = 26 (25 taps + the ones row of db), N = 32, K = B*784
// pixels split ~800 ways: every K tile re-gathers image taps with range-checked scalar loads
// (~29 VALU per MFMA in the launch it shares, profiles/r3_pmc.md) and the 800 partials need a
// wide reduce launch of their own.  Here workgroup (image b, band h) stages the band's 18 input
// rows once; wave w runs 49 v_mfma_f32_32x32x2_f32 over 98 of the band's 392 pixels with
// A[tap][pixel] = one ds_read (tap offset per lane), A[25][pixel] = 1, B[pixel][co] = d1
// (128 contiguous bytes per pixel); the four wave partials add in LDS in a fixed order.  The
// 2B block partials are reduced in the same launch: the last arriver of each group of 8 blocks
// sums its group in index order, the last group sums the group partials in index order (sc1
// write-through partials + arrival tickets, as gemm.h's last-arriver split-K), so the result
// does not depend on arrival order.
#pragma once
#include "gemm.h"
#include "layers.h"

namespace ddl {

constexpr int kC1wGroup = 8;       // block partials per first-level group
// staged image row pitch: a half-wave's ds_read_b32 reads one pixel at the 25 tap offsets
// ky * pitch + kx; pitch 37 (5 mod 32) puts the five tap rows in disjoint bank ranges
// (pitch 32: 5-way conflicts)
constexpr int kC1wPitch = 37;
constexpr int kC1wLdsBand = 18 * kC1wPitch + 2;  // (+2: keeps the partials 16-B aligned)

// optional optimizer on conv1's weight / bias as the final reduce writes them (the W = 1 tail
// path: the last segment's update needs no launch of its own); on = 0: gradients only
struct C1Adam {
  float *w_w = nullptr, *w_m = nullptr, *w_v = nullptr;  // weight [800] spans
  float *b_w = nullptr, *b_m = nullptr, *b_v = nullptr;  // bias [32] spans
  float lr_t = 0.f, c1 = 0.f, c2 = 0.f, eps = 0.f, scale = 1.f;
  int on = 0;
};
constexpr int kC1wElems = 26 * 32; // dW_aug[26][32] (row 25: db)

// scratch floats: 2B block partials + group partials (tickets: ngroups + 1 words, zero)
DDL_HD int c1w_groups(int B) { return (2 * B + kC1wGroup - 1) / kC1wGroup; }
DDL_HD size_t c1w_scratch_floats(int B) {
  return (size_t)(2 * B + c1w_groups(B)) * kC1wElems;
}

// the direct kernel's preconditions: scratch for the partials and tickets, 32-bit buffer
// offsets into d1 [B, 28, 28, 32]
inline bool conv1_wgrad_direct_ok(int B, size_t slab_floats, int max_tickets) {
  return B > 0 && c1w_scratch_floats(B) <= slab_floats && c1w_groups(B) + 1 <= max_tickets &&
         (uint64_t)B * 784u * 32u * 4u < (1ull << 31);
}

DDL_DEV bool c1w_arrive(int* ticket, int count, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int prev = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == count - 1;
    if (last) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  const bool last = *flag != 0;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  __syncthreads();
  return last;
}

// sum `n` partials of kC1wElems floats (index order) from `src` into `dst` (or into gw / gb
// when gw is given), 256 threads, sc1 loads (written write-through by other workgroups).  Every
// thread's loads of a chunk of U partials are issued before any is summed (one memory latency
// per chunk, not one per partial); the sum itself runs in index order.
constexpr int kC1wEPT = (kC1wElems + 255) / 256;  // elements per thread (4)
template <int U>
DDL_DEV void c1w_accum(brsrc_t part, int src, int n, float (&s)[kC1wEPT]) {
  constexpr int EPT = kC1wEPT;
#pragma unroll
  for (int j = 0; j < EPT; ++j) s[j] = 0.f;
  for (int i0 = 0; i0 < n; i0 += U) {
    float v[EPT][U];
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const int e = (int)threadIdx.x + 256 * j;
#pragma unroll
      for (int i = 0; i < U; ++i)
        v[j][i] = bload1_sc1(part, (i0 + i < n && e < kC1wElems)
                                       ? ((src + i0 + i) * kC1wElems + e) * 4 : kOOB);
    }
#pragma unroll
    for (int j = 0; j < EPT; ++j)
#pragma unroll
      for (int i = 0; i < U; ++i)
        if (i0 + i < n) s[j] += v[j][i];
  }
}

template <int U>
DDL_DEV void c1w_sum(brsrc_t part, int src, int n, brsrc_t out, int dst, float* gw, float* gb,
                     const C1Adam* ad = nullptr) {
  constexpr int EPT = kC1wEPT;
  float s[EPT];
  c1w_accum<U>(part, src, n, s);
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    const int e = (int)threadIdx.x + 256 * j;
    if (e >= kC1wElems) continue;
    if (gw) {
      const bool wrow = e < 25 * 32;
      const int i = wrow ? e : e - 25 * 32;
      (wrow ? gw : gb)[i] = s[j];
      if (ad && ad->on) {
        float* pw = wrow ? ad->w_w : ad->b_w;
        float* pm = wrow ? ad->w_m : ad->b_m;
        float* pv = wrow ? ad->w_v : ad->b_v;
        float W = pw[i], M = pm[i], V = pv[i];
        adam1(W, s[j] * ad->scale, M, V, ad->lr_t, ad->c1, ad->c2, ad->eps);
        pw[i] = W; pm[i] = M; pv[i] = V;
      }
    } else {
      bstore1_sc1(out, (dst * kC1wElems + e) * 4, s[j]);
    }
  }
}

// conv1 wgrad of (image b, band h) + the two-level reduce; `blk` = 2b + h
DDL_DEV void conv1_wgrad_block(const float* __restrict__ x, const float* __restrict__ d1, int B,
                               int blk, float* __restrict__ gw, float* __restrict__ gb,
                               float* __restrict__ part, int* __restrict__ tickets, float* lds,
                               int* flag, const C1Adam& ad) {
  const int b = blk >> 1, h = blk & 1;
  float* T = lds;                   // [18][kC1wPitch] image band
  float* R = lds + kC1wLdsBand;     // [4 waves][1024] wave partials
  const int y0 = 14 * h - 2;
  const float* img = x + (size_t)b * 784;
  for (int e = threadIdx.x; e < 18 * kC1wPitch; e += 256) {
    const int iy = y0 + e / kC1wPitch, ix = e % kC1wPitch - 2;
    T[e] = ((unsigned)iy < 28u && (unsigned)ix < 28u) ? img[iy * 28 + ix] : 0.f;
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int col = lane & 31, hk = lane >> 5;
  // this wave's 98 pixels of the band, two per MFMA (pixel 98w + 2s + hk); B operand
  // d1[b, 14h + py, px, col] prefetched whole (49 loads in flight)
  const brsrc_t dr = make_rsrc(d1, (uint32_t)B * 784u * 32u * 4u);
  const int pbase = (b * 784 + 14 * h * 28) * 32;
  float bv[49];
#pragma unroll
  for (int s = 0; s < 49; ++s) bv[s] = bload1(dr, (pbase + (98 * wave + 2 * s + hk) * 32 + col) * 4);
  // A operand row `col` = tap (ky, kx), row 25 = ones (db), rows 26..31 = 0
  const int toff = col < 25 ? (col / 5) * kC1wPitch + col % 5 : 0;
  const float arow = col == 25 ? 1.f : 0.f;
  __syncthreads();
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
  for (int s = 0; s < 49; ++s) {
    const int p = 98 * wave + 2 * s + hk;
    const int py = p / 28, px = p - py * 28;
    const float t = T[py * kC1wPitch + px + toff];
    acc = mfma32x32x2(col < 25 ? t : arow, bv[s], acc);
  }
  // wave partials -> LDS [wave][row 8g + 4hk + r][col]; block sum in a fixed order
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int r = 0; r < 4; ++r) R[wave * 1024 + (8 * g + 4 * hk + r) * 32 + col] = acc[4 * g + r];
  __syncthreads();
  const brsrc_t pr = make_rsrc(part, (uint32_t)c1w_scratch_floats(B) * 4u);
  for (int e = threadIdx.x; e < kC1wElems; e += 256) {
    const float s = (R[e] + R[1024 + e]) + (R[2048 + e] + R[3072 + e]);
    bstore1_sc1(pr, (blk * kC1wElems + e) * 4, s);
  }
  const int nblk = 2 * B, ng = c1w_groups(B);
  const int grp = blk / kC1wGroup;
  const int gcount = min(kC1wGroup, nblk - grp * kC1wGroup);
  if (!c1w_arrive(&tickets[grp], gcount, flag)) return;
  c1w_sum<kC1wGroup>(pr, grp * kC1wGroup, gcount, pr, nblk + grp, nullptr, nullptr);
  if (!c1w_arrive(&tickets[ng], ng, flag)) return;
  c1w_sum<32>(pr, nblk, ng, pr, 0, gw, gb, &ad);  // B <= 128: one chunk
}

// [2B conv1 wgrad blocks] then [conv2 wgrad wide reduce blocks (nrb, 256 threads, RL lanes per
// float4)]
template <int BM, int BN, int WM, int WN, int RL, class PR>
__global__ void __launch_bounds__(256)
conv1_wgrad_kernel(PR pr, const float4* __restrict__ rslab, int S, int rgx, int rntiles,
                   const float* __restrict__ x, const float* __restrict__ d1, int B,
                   float* __restrict__ gw, float* __restrict__ gb, float* __restrict__ part,
                   int* __restrict__ tickets, C1Adam ad) {
  __shared__ float lds[kC1wLdsBand + 4 * 1024];
  __shared__ int flag;
  // conv1's blocks first: their MFMA pass + two reduce levels are the launch's critical path,
  // the independent reduce blocks fill the CUs behind them
  const int nc = 2 * B;
  if ((int)blockIdx.x < nc) {
    conv1_wgrad_block(x, d1, B, (int)blockIdx.x, gw, gb, part, tickets, lds, &flag, ad);
    return;
  }
  wide_reduce_body<BM, BN, WM, WN, RL, PR>(pr, rslab, S, rgx, rntiles,
                                           ((int)blockIdx.x - nc) * 256 + threadIdx.x);
}

// Launch conv1's weight gradient, fused with problem R's pending mode-2 reduce when `gr` has one
// (tile config CR).  `part` / `tickets`: scratch (c1w_scratch_floats(B) floats, zeroed tickets).
template <class CR, class PR>
inline void launch_conv1_wgrad(const PR& pr, const SubGrid& gr, const float* x, const float* d1,
                               int B, float* gw, float* gb, float* part, int* tickets,
                               hipStream_t st, const C1Adam& ad = C1Adam()) {
  const bool red = gr.mode == 2 && gr.nblocks > 0;
  using G = TileGeo<CR::BM, CR::BN, CR::WM, CR::WN>;
  const int ntiles = gr.gx * gr.gy, z = gr.gz;
  const size_t nelem = red ? (size_t)ntiles * G::PART4 : 0;
#define DDL_C1W(RL)                                                                           \
  {                                                                                         \
    const int nrb = (int)((nelem * RL + 255) / 256);                                        \
    DDL_LAUNCH((conv1_wgrad_kernel<CR::BM, CR::BN, CR::WM, CR::WN, RL, PR>),                \
               dim3(nrb + 2 * B), dim3(256), 0, st, pr, gr.slab, z, gr.gx, ntiles, x, d1,      \
               B, gw, gb, part, tickets, ad);                                               \
  }
  if (z > 32) DDL_C1W(64) else if (z > 4) DDL_C1W(16) else DDL_C1W(4)
#undef DDL_C1W
}

// (Round 5's opt-in fused last bucket — the W > 1 xGMI exchange of conv1 + conv2 inside this
// launch — stalled intermittently with several ranks on one card, cause not established, and
// was removed in round 6: docs/DESIGN.md.  The replicated bucket runs xgmi.hip's
// xgmi_repl_kernel.)

}  // namespace ddl
