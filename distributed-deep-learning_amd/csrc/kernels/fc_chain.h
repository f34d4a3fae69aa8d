// The fully connected half of the step as ONE persistent launch:
// fc1 forward -> fc2 forward -> classifier head -> fc2 data / weight gradient, fc3 weight
// gradient -> fc1 data gradient (+ conv4 pool backward scatter) / weight gradient
// (reference ops: mnist_sync/model/model.py:67-92).
//
// At batch 100 these six stages are latency-bound (M = 100 rows: 4 row tiles) and were six
// dependent launches (~52 us, 17 % of the step for 4.5 % of its FLOPs): every boundary paid a
// drain and a fill.  Here the stages are ITEMS of one work queue.  A workgroup (8 waves) takes
// the next item id from a global counter (one returning atomic: the guide's cheapest cross-CU
// primitive); item ids are ordered so that every dependency points to LOWER ids, and an item
// waits (bounded poll) only for per-row-block / per-column-block completion counters of
// earlier stages.  The lowest unfinished item therefore always has its inputs: whatever the
// dispatch order or residency, the queue drains (no grid barrier, no co-residency assumption).
//
// Hand-off (MI355X guide §6 G16, first row of the sc1 table): a producer stores the handed-off
// activations / gradients write-through (sc1), every wave drains vmcnt(0), the workgroup
// barrier, then ONE relaxed agent-scope add on the stage counter; the consumer polls the counter
// from one lane, joins a workgroup barrier, and reads every handed-off byte with sc1 loads.
// Outputs consumed only by LATER launches (the weight gradients, the conv4 data gradient) are
// plain stores.  The last workgroup to leave resets the counters for the next launch.
//
// Items (B = 100: row tiles mi = 0..3):
//   A fc1 fwd    tile (mi, nj<32)  K-wave over 8 waves           -> h1    cnt_h1[mi] += 1
//   B fc2 fwd    tile (mi, nj<16)  needs cnt_h1[mi] == 32         -> h2    cnt_h2[mi] += 1
//   C head       rows of mi        needs cnt_h2[mi] == 16         -> dlog, loss, dpre2
//                                                                         cnt_hd[mi] = 1
//   D fc2 dgrad  tile (mi, nj<32)  needs cnt_hd[mi]               -> dpre1 cnt_d1r[mi], cnt_d1c[nj]
//   E fc2 wgrad  8 tiles of [1025 x 512], K = B: needs every head -> dW2, db2
//   F fc3 wgrad  8 rows of [513 x 10]:            needs every head -> dW3, db3
//   G fc1 dgrad  tile (mi, nj<32)  needs cnt_d1r[mi] == 32        -> d4 (pool scatter)
//   H fc1 wgrad  8 tiles of [1025 x 1024] column nj: cnt_d1c[nj] == 4 -> dW1, db1
#pragma once
#include "gemm.h"
#include "head.h"
#include "layers.h"

namespace ddl {

constexpr int kFcRowTiles = 4;     // ceil(100 / 32): the chain is built for batch <= 128
constexpr int kFcWaves = 8;        // waves per workgroup (the K-wave stages split K over them)

// counter block (ints, zero between launches)
enum FcCtr {
  FC_HEAD = 0, FC_DONE = 1, FC_ERR = 2,
  FC_H1 = 8, FC_H2 = 12, FC_HD = 16, FC_D1R = 20, FC_D1C = 24,  // + row / column index
  FC_NCTR = 24 + 32
};

struct FcChain {
  FcFwd<true, false, true> f1;         // p4 -> h1 (sc1 stores)
  FcFwd<false, true, true> f2;         // h1 -> h2 (sc1 loads and stores)
  FcDgradActT<true, true> d2;          // dpre2 W2^T, fc1 act. backward -> dpre1
  FcWgradT<true> w2;                   // [h1;1]^T dpre2 -> dW2, db2
  FcDgradPool<2, 256, true> d1;        // dpre1 W1^T -> d4 through conv4's pool codes
  FcWgradT<true> w1;                   // [p4;1]^T dpre1 -> dW1, db1
  // head (fc3 + softmax cross-entropy)
  const float* w3;
  const float* b3;
  const int64_t* labels;
  float* dlog;
  float* loss;
  float* dpre2;
  float* gw3;
  float* gb3;
  float inv_batch;
  uint32_t thr24;
  float inv_keep;
  int B;
  int* ctr;
  long long timeout_ticks;
  long long* stamps;                   // diagnostics (null: off): per item dequeue / ready / end
                                       // / block / 4 item-specific, 8 per item
};

// item ranges
constexpr int kFcA = kFcRowTiles * 32, kFcB = kFcRowTiles * 16, kFcC = kFcRowTiles;
constexpr int kFcD = kFcRowTiles * 32;
constexpr int kFcE = (33 * 16 + kFcWaves - 1) / kFcWaves;   // 528 one-wave tiles
constexpr int kFcF = (HK + 1 + kFcWaves - 1) / kFcWaves;    // 513 rows
constexpr int kFcG = kFcRowTiles * 32;
constexpr int kFcHg = (33 + kFcWaves - 1) / kFcWaves;       // m-tile groups per column
constexpr int kFcH = 32 * kFcHg;
constexpr int kFcOffB = kFcA, kFcOffC = kFcOffB + kFcB, kFcOffD = kFcOffC + kFcC;
constexpr int kFcOffE = kFcOffD + kFcD, kFcOffF = kFcOffE + kFcE, kFcOffG = kFcOffF + kFcF;
constexpr int kFcOffH = kFcOffG + kFcG, kFcItems = kFcOffH + kFcH;

DDL_DEV int fc_ctr_load(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// lane 0 of wave 0 waits until ctr[i] >= target (bounded: a timeout records FC_ERR and lets
// the item run on whatever is there, so a bug shows as a wrong result, never as a hang)
#ifndef DDL_FC_SLEEP
#define DDL_FC_SLEEP 32
#endif
DDL_DEV void fc_wait(const FcChain& a, int i, int target, long long deadline, int it) {
  if (threadIdx.x == 0) {
    while (fc_ctr_load(a.ctr + i) < target) {
      if (wall_clock64() > deadline) {
        __hip_atomic_store(a.ctr + FC_ERR, 1 + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(DDL_FC_SLEEP);
    }
    if (a.stamps) a.stamps[it * 8 + 1] = wall_clock64();
  }
  __syncthreads();
}

// publish: every wave's stores are complete (vmcnt(0)) before the workgroup barrier, then one add
DDL_DEV void fc_publish(const FcChain& a, int i0, int i1 = -1) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(a.ctr + i0, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (i1 >= 0) __hip_atomic_fetch_add(a.ctr + i1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// classifier head of up to 32 samples (row tile mi), one wave per sample, 4 per wave.  W3 is
// staged once per item into LDS transposed ([HC][HK]) so lane l owns h2 columns l + 64k
// (coalesced h2 reads / dpre2 stores, conflict-free LDS reads); the 4 rows' h2 loads are all in
// flight before the first row's math.  Logits (+ butterfly), softmax cross entropy, dlogits =
// (softmax - onehot) / B, and dpre2 = (dlogits W3^T) with fc2's dropout backward — every
// handed-off buffer read / written sc1.  Every access goes through a buffer descriptor: with
// plain pointers the compiler emitted flat loads / stores, each waited for on its own
// (vmcnt(0) + lgkmcnt(0)), and the item ran 22-40 us.
DDL_DEV void fc_head(const FcChain& a, int mi, float* w3t, long long* st) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int kT = kFcWaves * 64;
  static_assert((HK * HC) % kT == 0, "W3 staging: whole rounds");
  const brsrc_t w3r = make_rsrc(a.w3, HK * HC * 4u), b3r = make_rsrc(a.b3, HC * 4u);
  const brsrc_t h2r = make_rsrc(a.f2.out, (uint32_t)a.B * HK * 4u);
  const brsrc_t dpr = make_rsrc(a.dpre2, (uint32_t)a.B * HK * 4u);
  const brsrc_t dlr = make_rsrc(a.dlog, (uint32_t)a.B * HC * 4u);
  const brsrc_t lsr = make_rsrc(a.loss, (uint32_t)a.B * 4u);
  const brsrc_t lbr = make_rsrc(a.labels, (uint32_t)a.B * 8u);
  const int row0 = mi * 32 + wave * 4;
#pragma unroll
  for (int r = 0; r < HK * HC / kT; ++r) {
    const int j = r * kT + threadIdx.x, i = j / HC, c = j - i * HC;
    w3t[c * HK + i] = bload1(w3r, j * 4);
  }
  // fc2's dropout key (layer 2), as FcFwd / head_fused_kernel derive it
  const uint32_t key =
      a.thr24 ? ddl_mix32((a.f2.seed ? *a.f2.seed : a.f2.seed_v) + 2u * 0x9E3779B9u) : 0u;
  __syncthreads();
  if (st && threadIdx.x == 0) st[4] = wall_clock64();
  float b3v[HC];
#pragma unroll
  for (int c = 0; c < HC; ++c) b3v[c] = bload1(b3r, c * 4);
  float hv[HK / 64], hn[HK / 64];
#pragma unroll
  for (int k = 0; k < HK / 64; ++k) hn[k] = bload1_sc1(h2r, (row0 * HK + k * 64 + lane) * 4);
  for (int s = 0; s < 4; ++s) {
    const int row = row0 + s;
    if (row >= a.B) break;
#pragma unroll
    for (int k = 0; k < HK / 64; ++k) hv[k] = hn[k];
    if (s + 1 < 4) {  // (rows past B read 0 through the range check)
#pragma unroll
      for (int k = 0; k < HK / 64; ++k)
        hn[k] = bload1_sc1(h2r, ((row + 1) * HK + k * 64 + lane) * 4);
    }
    float lg[HC];
#pragma unroll
    for (int c = 0; c < HC; ++c) {
      float v = 0.f;
#pragma unroll
      for (int k = 0; k < HK / 64; ++k) v = fmaf(hv[k], w3t[c * HK + k * 64 + lane], v);
      lg[c] = v;
    }
#pragma unroll
    for (int c = 0; c < HC; ++c) lg[c] = wave_sum(lg[c]) + b3v[c];
    float mx = lg[0];
#pragma unroll
    for (int c = 1; c < HC; ++c) mx = lg[c] > mx ? lg[c] : mx;
    float se = 0.f;
#pragma unroll
    for (int c = 0; c < HC; ++c) se += __expf(lg[c] - mx);
    const int lab = bload1i(lbr, row * 8);  // int64 labels: low word
    const float inv_se = 1.f / se;
    float dl[HC];
#pragma unroll
    for (int c = 0; c < HC; ++c)
      dl[c] = (__expf(lg[c] - mx) * inv_se - (c == lab ? 1.f : 0.f)) * a.inv_batch;
    if (lane == 0) {
      float ll = 0.f;
#pragma unroll
      for (int c = 0; c < HC; ++c)
        if (c == lab) ll = lg[c];
      bstore1(lsr, row * 4, (mx + __logf(se)) - ll);
    }
    if (lane < HC) {
      float v = 0.f;
#pragma unroll
      for (int c = 0; c < HC; ++c)
        if (c == lane) v = dl[c];
      bstore1_sc1(dlr, (row * HC + lane) * 4, v);
    }
#pragma unroll
    for (int k = 0; k < HK / 64; ++k) {
      const int i = k * 64 + lane;
      float g = 0.f;
#pragma unroll
      for (int c = 0; c < HC; ++c) g = fmaf(dl[c], w3t[c * HK + i], g);
      const int idx = row * HK + i;
      if (a.thr24) g = ddl_keep(key, (uint32_t)idx, a.thr24) ? g * a.inv_keep : 0.f;
      bstore1_sc1(dpr, idx * 4, g);
    }
    if (st && threadIdx.x == 0 && s < 3) st[5 + s] = wall_clock64();
  }
}

// fc3 weight gradient row i (head.h head_wgrad_row with sc1 reads of h2 / dlog), all of a
// lane's loads in flight at once (B <= 128: two samples per lane)
DDL_DEV void fc_head_wgrad_row(const FcChain& a, int i) {
  const int lane = threadIdx.x & 63;
  const brsrc_t h2r = make_rsrc(a.f2.out, (uint32_t)a.B * HK * 4u);
  const brsrc_t dlr = make_rsrc(a.dlog, (uint32_t)a.B * HC * 4u);
  float hv[2], dv[2][HC];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int b = lane + 64 * q;
    hv[q] = i < HK ? bload1_sc1(h2r, (b * HK + i) * 4) : (b < a.B ? 1.f : 0.f);
#pragma unroll
    for (int c = 0; c < HC; ++c) dv[q][c] = bload1_sc1(dlr, (b * HC + c) * 4);
  }
  float acc[HC];
#pragma unroll
  for (int c = 0; c < HC; ++c) acc[c] = fmaf(hv[1], dv[1][c], hv[0] * dv[0][c]);
#pragma unroll
  for (int c = 0; c < HC; ++c) acc[c] = wave_sum(acc[c]);
  if (lane < HC) {
    float v = 0.f;
#pragma unroll
    for (int c = 0; c < HC; ++c)
      if (c == lane) v = acc[c];
    if (i < HK) bstore1(make_rsrc(a.gw3, HK * HC * 4u), (i * HC + lane) * 4, v);
    else bstore1(make_rsrc(a.gb3, HC * 4u), lane * 4, v);
  }
}

// one one-wave 32x32 tile of a weight-gradient problem per wave
template <class P>
DDL_DEV void fc_wave_tile(const P& p, int t, int ntiles, int gx, float4* lds4, int L) {
  using T = GemmTile<32, 32, 32, 1, 1, P>;
  if (t >= ntiles) return;
  const int wave = threadIdx.x >> 6;
  const int m_blk = (t % gx) * 32, n_blk = (t / gx) * 32;
  f32x16 acc[1][1];
  T::mainloop(p, m_blk, n_blk, 0, p.K, reinterpret_cast<float*>(lds4 + wave * L), acc);
  T::epilogue(p, m_blk, n_blk, acc);
}

// Item bodies: inlined (default) the kernel takes 256 VGPRs with a few spills; as calls
// (DDL_FC_NOINLINE=1) 216 VGPRs but 448 B of call-frame scratch per lane.
#ifndef DDL_FC_NOINLINE
#define DDL_FC_NOINLINE 0
#endif
#if DDL_FC_NOINLINE
#define DDL_FC_ITEM __device__ __attribute__((noinline))
#else
#define DDL_FC_ITEM DDL_DEV
#endif
template <class P>
DDL_FC_ITEM void fc_item_kwave(const P& p, int mi, int nj, float4* lds4, int L) {
  kwave_body<32, kFcWaves>(p, mi, nj, lds4, L);
}
DDL_FC_ITEM void fc_item_head(const FcChain& a, int mi, float* w3t, long long* st) {
  fc_head(a, mi, w3t, st);
}
DDL_FC_ITEM void fc_item_head_wgrad(const FcChain& a, int i) {
  if (i <= HK) fc_head_wgrad_row(a, i);
}
template <class P>
DDL_FC_ITEM void fc_item_tile(const P& p, int t, int ntiles, int gx, float4* lds4, int L) {
  fc_wave_tile(p, t, ntiles, gx, lds4, L);
}

template <int L>
__global__ void __launch_bounds__(kFcWaves * 64) fc_chain_kernel(FcChain a) {
  static_assert(kFcWaves * L * 4 >= HK * HC, "the head stages W3 in the staging images");
  __shared__ float4 lds4[kFcWaves * L + 1];  // staging / reduction images + the item word
  int* item_s = reinterpret_cast<int*>(lds4 + kFcWaves * L);
  const long long deadline = wall_clock64() + a.timeout_ticks;
  for (;;) {
    if (threadIdx.x == 0)
      *item_s = __hip_atomic_fetch_add(a.ctr + FC_HEAD, 1, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int it = *item_s;
    __syncthreads();  // (the word is rewritten by the next dequeue)
    if (it >= kFcItems) break;
    const int wave = threadIdx.x >> 6;
    if (a.stamps && threadIdx.x == 0) {
      a.stamps[it * 8 + 0] = wall_clock64();
      a.stamps[it * 8 + 3] = blockIdx.x;
    }
    if (it < kFcOffB) {                      // A: fc1 forward
      const int mi = it % kFcRowTiles, nj = it / kFcRowTiles;
      fc_item_kwave(a.f1, mi, nj, lds4, L);
      fc_publish(a, FC_H1 + mi);
    } else if (it < kFcOffC) {               // B: fc2 forward
      const int j = it - kFcOffB, mi = j % kFcRowTiles, nj = j / kFcRowTiles;
      fc_wait(a, FC_H1 + mi, 32, deadline, it);
      fc_item_kwave(a.f2, mi, nj, lds4, L);
      fc_publish(a, FC_H2 + mi);
    } else if (it < kFcOffD) {               // C: head
      const int mi = it - kFcOffC;
      fc_wait(a, FC_H2 + mi, 16, deadline, it);
      fc_item_head(a, mi, reinterpret_cast<float*>(lds4), a.stamps ? a.stamps + it * 8 : nullptr);
      fc_publish(a, FC_HD + mi);
    } else if (it < kFcOffE) {               // D: fc2 data gradient (+ fc1 act. backward)
      const int j = it - kFcOffD, mi = j % kFcRowTiles, nj = j / kFcRowTiles;
      fc_wait(a, FC_HD + mi, 1, deadline, it);
      fc_item_kwave(a.d2, mi, nj, lds4, L);
      fc_publish(a, FC_D1R + mi, FC_D1C + nj);
    } else if (it < kFcOffF) {               // E: fc2 weight gradient
      for (int mi = 0; mi < kFcRowTiles; ++mi) fc_wait(a, FC_HD + mi, 1, deadline, it);
      fc_item_tile(a.w2, (it - kFcOffE) * kFcWaves + wave, 33 * 16, 33, lds4, L);
    } else if (it < kFcOffG) {               // F: fc3 weight gradient
      for (int mi = 0; mi < kFcRowTiles; ++mi) fc_wait(a, FC_HD + mi, 1, deadline, it);
      fc_item_head_wgrad(a, (it - kFcOffF) * kFcWaves + wave);
    } else if (it < kFcOffH) {               // G: fc1 data gradient -> d4
      const int j = it - kFcOffG, mi = j % kFcRowTiles, nj = j / kFcRowTiles;
      fc_wait(a, FC_D1R + mi, 32, deadline, it);
      fc_item_kwave(a.d1, mi, nj, lds4, L);
    } else {                                 // H: fc1 weight gradient, column nj
      const int j = it - kFcOffH, nj = j / kFcHg, g = j % kFcHg;
      fc_wait(a, FC_D1C + nj, kFcRowTiles, deadline, it);
      const int mt = g * kFcWaves + wave;     // m tile 0..32 of column nj
      if (mt < 33) fc_item_tile(a.w1, nj * 33 + mt, 33 * 32, 33, lds4, L);
    }
    __syncthreads();  // the staging images are reused by the next item
    if (a.stamps && threadIdx.x == 0) a.stamps[it * 8 + 2] = wall_clock64();
  }
  // the last workgroup out re-arms every counter for the next launch (all others have taken
  // their final item id: they added to DONE after it)
  if (threadIdx.x == 0) {
    const int d = __hip_atomic_fetch_add(a.ctr + FC_DONE, 1, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    if (d == (int)gridDim.x - 1) {
      for (int i = 0; i < FC_NCTR; ++i)
        if (i != FC_ERR)
          __hip_atomic_store(a.ctr + i, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace ddl
