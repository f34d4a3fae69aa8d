// Classifier head: fc3 (512->10) + softmax cross-entropy (model.py:85-92) and its backward.
//
// fc3 is too skinny (N = 10) for MFMA tiles to pay, so it is two small VALU kernels:
//   head_fwd : one 4-wave workgroup per sample: logits, loss, dlogits = (softmax - onehot)/B
//              (SoftmaxCrossEntropyWithLogits + Mean fwd/bwd),
//              or in eval mode the correct-prediction count (F22).
//   head_bwd : dW3_aug[513,10] = [h2;1]^T dlogits and dh2 = dlogits W3^T, with the fc2
//              dropout backward fused (mask regenerated from the seed, nothing stored).
//   head_fused: head_fwd + the dh2 part of head_bwd per sample (one launch in training; the
//              fc3 weight gradient then rides in the next dual launch, head.h HeadWgradAux).
#include <stdexcept>

#include "common.h"
#include "api.h"
#include "head.h"

namespace ddl {

// Logits of sample `row` by a whole 256-thread workgroup: wave v sums columns [128v, 128v+128)
// (2 per lane), a shuffle tree per wave, then the four wave partials through LDS in a fixed order.
// Four waves per sample instead of one: at batch 100 the head is latency-bound (100 waves on a
// 256-CU chip), so shorter per-wave chains beat fewer launches.  Every thread returns all HC
// logits.  Shared by head_fwd and head_fused so their arithmetic is identical (bitwise).
DDL_DEV void head_logits_hv(const float (&hv)[2], const float* __restrict__ w,
                            const float* __restrict__ bias, float (&part)[4][HC],
                            float (&acc)[HC]) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int c = 0; c < HC; ++c) acc[c] = 0.f;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int k = wave * 128 + t * 64 + lane;
    const float* wr = w + k * HC;
#pragma unroll
    for (int c = 0; c < HC; ++c) acc[c] = fmaf(hv[t], wr[c], acc[c]);
  }
#pragma unroll
  for (int c = 0; c < HC; ++c) {
    const float v = wave_sum(acc[c]);
    if (lane == 0) part[wave][c] = v;
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < HC; ++c)
    acc[c] = ((part[0][c] + part[1][c]) + (part[2][c] + part[3][c])) + bias[c];
}
// the same with the thread's two W3 rows and fc3's bias already in registers (bitwise equal)
DDL_DEV void head_logits_regs(const float (&hv)[2], const float (&wv)[2][HC], const float (&bb)[HC],
                              float (&part)[4][HC], float (&acc)[HC]) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int c = 0; c < HC; ++c) acc[c] = 0.f;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int c = 0; c < HC; ++c) acc[c] = fmaf(hv[t], wv[t][c], acc[c]);
#pragma unroll
  for (int c = 0; c < HC; ++c) {
    const float v = wave_sum(acc[c]);
    if (lane == 0) part[wave][c] = v;
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < HC; ++c)
    acc[c] = ((part[0][c] + part[1][c]) + (part[2][c] + part[3][c])) + bb[c];
}
// thread (wave, lane) holds h2 columns k = wave*128 + t*64 + lane, t = 0, 1
DDL_DEV void head_logits(const float* __restrict__ hr, const float* __restrict__ w,
                         const float* __restrict__ bias, float (&part)[4][HC],
                         float (&acc)[HC]) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const float hv[2] = {hr[wave * 128 + lane], hr[wave * 128 + 64 + lane]};
  head_logits_hv(hv, w, bias, part, acc);
}

__global__ void __launch_bounds__(256)
head_fwd_kernel(const float* __restrict__ h2, const float* __restrict__ w,
                const float* __restrict__ bias, const int64_t* __restrict__ labels, int B,
                float inv_batch, float* __restrict__ dlog, float* __restrict__ loss,
                int* __restrict__ correct) {
  __shared__ float part[4][HC];
  const int row = blockIdx.x;
  if (row >= B) return;
  float acc[HC];
  head_logits(h2 + (size_t)row * HK, w, bias, part, acc);
  float mx = acc[0];
  int arg = 0;
#pragma unroll
  for (int c = 1; c < HC; ++c)
    if (acc[c] > mx) { mx = acc[c]; arg = c; }
  float se = 0.f;
#pragma unroll
  for (int c = 0; c < HC; ++c) se += __expf(acc[c] - mx);
  const int lab = (int)labels[row];
  if (threadIdx.x == 0) {
    float ll = 0.f;
#pragma unroll
    for (int c = 0; c < HC; ++c)
      if (c == lab) ll = acc[c];
    if (loss) loss[row] = (mx + __logf(se)) - ll;
    if (correct && arg == lab) atomicAdd(correct, 1);
  }
  if (dlog && threadIdx.x < HC) {
    float lc = 0.f;
#pragma unroll
    for (int c = 0; c < HC; ++c)
      if (c == (int)threadIdx.x) lc = acc[c];
    const float p = __expf(lc - mx) / se;
    dlog[(size_t)row * HC + threadIdx.x] = (p - ((int)threadIdx.x == lab ? 1.f : 0.f)) * inv_batch;
  }
}

__global__ void __launch_bounds__(256)
head_bwd_kernel(const float* __restrict__ h2, const float* __restrict__ w,
                const float* __restrict__ dlog, int B, int wblocks, const uint32_t* __restrict__ seed,
                uint32_t seed_v,
                uint32_t thr24, float inv_keep, float* __restrict__ gw, float* __restrict__ gb,
                float* __restrict__ dpre2) {
  if ((int)blockIdx.x < wblocks) {
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i <= HK) head_wgrad_row(h2, dlog, B, i, gw, gb);
    return;
  }
  const int idx = (blockIdx.x - wblocks) * 256 + threadIdx.x;
  if (idx >= B * HK) return;
  const int b = idx / HK, i = idx % HK;
  float g = 0.f;
#pragma unroll
  for (int c = 0; c < HC; ++c) g = fmaf(dlog[(size_t)b * HC + c], w[i * HC + c], g);
  if (thr24) {
    const uint32_t key = ddl_mix32((seed ? *seed : seed_v) + 2u * 0x9E3779B9u);
    g = ddl_keep(key, (uint32_t)idx, thr24) ? g * inv_keep : 0.f;
  }
  dpre2[idx] = g;
}

__global__ void __launch_bounds__(256)
head_fused_kernel(const float* __restrict__ h2, const float* __restrict__ w,
                  const float* __restrict__ bias, const int64_t* __restrict__ labels, int B,
                  float inv_batch, const uint32_t* __restrict__ seed, uint32_t seed_v,
                  uint32_t thr24, float inv_keep, float* __restrict__ dlog,
                  float* __restrict__ loss, float* __restrict__ dpre2) {
  __shared__ float part[4][HC];
  const int row = blockIdx.x;
  if (row >= B) return;
  // fc2's dropout key (layer 2) is also the dh2 mask key below
  const uint32_t key = thr24 ? ddl_mix32((seed ? *seed : seed_v) + 2u * 0x9E3779B9u) : 0u;
  float acc[HC];
  // every operand up front, as head_fused_fc2_kernel: this thread's two h2 columns k = wave*128
  // + t*64 + lane, their W3 rows (the logits AND the two dh2 columns below), fc3's bias, the
  // label — one load round instead of a second W3 round after the softmax
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float hv[2], wv[2][HC], bb[HC];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int k = wave * 128 + t * 64 + lane;
    hv[t] = h2[(size_t)row * HK + k];
#pragma unroll
    for (int c = 0; c < HC; ++c) wv[t][c] = w[k * HC + c];
  }
#pragma unroll
  for (int c = 0; c < HC; ++c) bb[c] = bias[c];
  const int lab = (int)labels[row];
  head_logits_regs(hv, wv, bb, part, acc);
  float mx = acc[0];
#pragma unroll
  for (int c = 1; c < HC; ++c) mx = acc[c] > mx ? acc[c] : mx;
  float se = 0.f;
#pragma unroll
  for (int c = 0; c < HC; ++c) se += __expf(acc[c] - mx);
  // dlogits of this sample in every thread (same arithmetic as head_fwd_kernel's per-lane form)
  float dl[HC];
#pragma unroll
  for (int c = 0; c < HC; ++c) dl[c] = (__expf(acc[c] - mx) / se - (c == lab ? 1.f : 0.f)) * inv_batch;
  if (threadIdx.x == 0) {
    float ll = 0.f;
#pragma unroll
    for (int c = 0; c < HC; ++c)
      if (c == lab) ll = acc[c];
    loss[row] = (mx + __logf(se)) - ll;
  }
  if (threadIdx.x < HC) {
    float v = 0.f;
#pragma unroll
    for (int c = 0; c < HC; ++c)
      if (c == (int)threadIdx.x) v = dl[c];
    dlog[(size_t)row * HC + threadIdx.x] = v;
  }
  // dh2 = dlogits W3^T with fc2's dropout backward (mask regenerated from the seed), 2 columns
  // per thread, from the W3 rows already in registers (the same fmaf chain per element as the
  // earlier form that reloaded W3 after the softmax: 0.2596-0.2603 -> 0.2592-0.2597 ms/step, 5
  // alternating same-box rounds, profiles/r6_ab_head_regs.log)
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int k = wave * 128 + t * 64 + lane;
    float g = 0.f;
#pragma unroll
    for (int c = 0; c < HC; ++c) g = fmaf(dl[c], wv[t][c], g);
    const int idx = row * HK + k;
    if (thr24) g = ddl_keep(key, (uint32_t)idx, thr24) ? g * inv_keep : 0.f;
    dpre2[idx] = g;
  }
}

// One output element of a mode-2 split-K reduce, summed in exactly the order of gemm.h
// wide_reduce_body with RL lanes (lane j: z = j, j + RL, ... from 0; then common.h group_sum's
// DPP stages, which form the balanced pairwise tree over the RL lane sums in lane order).
// S <= 32.  All loads are issued before the adds.
template <int RL>
DDL_DEV float wide_sum(const float* __restrict__ slab, size_t zstride, size_t off, int S) {
  float l[RL];
#pragma unroll
  for (int j = 0; j < RL; ++j) l[j] = 0.f;
  float v[32];
#pragma unroll
  for (int z = 0; z < 32; ++z) v[z] = z < S ? slab[(size_t)z * zstride + off] : 0.f;
#pragma unroll
  for (int z = 0; z < 32; ++z)
    if (z < S) l[z % RL] += v[z];
  if constexpr (RL == 16) {
    float q[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = (l[4 * i] + l[4 * i + 1]) + (l[4 * i + 2] + l[4 * i + 3]);
    return (q[0] + q[1]) + (q[2] + q[3]);
  } else {
    return (l[0] + l[1]) + (l[2] + l[3]);
  }
}

// head_fused with fc2's forward finished here: thread (wave, lane) sums the S split-K partials
// of its two h2 columns k = wave*128 + t*64 + lane (one-wave 32x32 tiles: partial image
// [z][tile][g][lane] float4, element (row r, col c) of a tile at g = r / 8, lane = c + 32 *
// ((r % 8) / 4), component r % 4; gemm.h store_partial) in z order, adds b2, applies fc2's
// dropout (layer key 2, the dh2 mask key) and stores h2 for fc3's weight gradient — fc2's
// wide-reduce launch (4.7 us) folded into the head's.
__global__ void __launch_bounds__(256)
head_fused_fc2_kernel(const float* __restrict__ slab, int S, int gx, int ntiles,
                      const float* __restrict__ b2, float* __restrict__ h2,
                      const float* __restrict__ w, const float* __restrict__ bias,
                      const int64_t* __restrict__ labels, int B, float inv_batch,
                      const uint32_t* __restrict__ seed, uint32_t seed_v, uint32_t thr24,
                      float inv_keep, float* __restrict__ dlog, float* __restrict__ loss,
                      float* __restrict__ dpre2) {
  __shared__ float part[4][HC];
  const int row = blockIdx.x;
  if (row >= B) return;
  const uint32_t key = thr24 ? ddl_mix32((seed ? *seed : seed_v) + 2u * 0x9E3779B9u) : 0u;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // every operand that does not depend on the partial sums is loaded up front, so the kernel's
  // dependent chain is one round of partial loads instead of four load rounds: this thread's two
  // W3 rows (the logits AND its two dh2 columns below), fc2's bias, fc3's bias, the label
  float wv[2][HC], b2v[2], bb[HC];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int k = wave * 128 + t * 64 + lane;
#pragma unroll
    for (int c = 0; c < HC; ++c) wv[t][c] = w[k * HC + c];
    b2v[t] = b2[k];
  }
#pragma unroll
  for (int c = 0; c < HC; ++c) bb[c] = bias[c];
  const int lab = (int)labels[row];
  const int bx = row >> 5, r = row & 31;
  const int fg = r >> 3, comp = r & 3, half = (r & 7) >> 2;
  const size_t zstride = (size_t)ntiles * 256 * 4;  // floats per split (PART4 = 256 float4)
  float hv[2];
  size_t off[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int k = wave * 128 + t * 64 + lane;
    const int tile = (k >> 5) * gx + bx;
    off[t] = ((size_t)tile * 256 + fg * 64 + (k & 31) + 32 * half) * 4 + comp;
    hv[t] = 0.f;
  }
  // the wide reduce's exact summation order (gemm.h wide_reduce_body + common.h group_sum, RL
  // lanes per element: lane j sums z = j, j + RL, ... from 0, then the DPP tree over the RL
  // lanes is the balanced pairwise tree in lane order), so h2 is bit-identical to the
  // separate reduce launch; every partial load is issued before the adds
  // (S > 32 is not deferred: engine_ops_fc.hip)
#pragma unroll
  for (int t = 0; t < 2; ++t)
    hv[t] = S > 4 ? wide_sum<16>(slab, zstride, off[t], S) : wide_sum<4>(slab, zstride, off[t], S);
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int k = wave * 128 + t * 64 + lane;
    const uint32_t idx = (uint32_t)(row * HK + k);
    float val = hv[t] + b2v[t];  // FcFwd<false>: no ReLU
    if (thr24) val = ddl_keep(key, idx, thr24) ? val * inv_keep : 0.f;
    h2[idx] = val;
    hv[t] = val;
  }
  float acc[HC];
  head_logits_regs(hv, wv, bb, part, acc);
  float mx = acc[0];
#pragma unroll
  for (int c = 1; c < HC; ++c) mx = acc[c] > mx ? acc[c] : mx;
  float se = 0.f;
#pragma unroll
  for (int c = 0; c < HC; ++c) se += __expf(acc[c] - mx);
  float dl[HC];
#pragma unroll
  for (int c = 0; c < HC; ++c) dl[c] = (__expf(acc[c] - mx) / se - (c == lab ? 1.f : 0.f)) * inv_batch;
  if (threadIdx.x == 0) {
    float ll = 0.f;
#pragma unroll
    for (int c = 0; c < HC; ++c)
      if (c == lab) ll = acc[c];
    loss[row] = (mx + __logf(se)) - ll;
  }
  if (threadIdx.x < HC) {
    float v = 0.f;
#pragma unroll
    for (int c = 0; c < HC; ++c)
      if (c == (int)threadIdx.x) v = dl[c];
    dlog[(size_t)row * HC + threadIdx.x] = v;
  }
  // dh2 of this thread's two columns from the W3 rows already in registers (the same fmaf chain
  // per element as head_fused_kernel's loop over i)
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int k = wave * 128 + t * 64 + lane;
    float g = 0.f;
#pragma unroll
    for (int c = 0; c < HC; ++c) g = fmaf(dl[c], wv[t][c], g);
    const int idx = row * HK + k;
    if (thr24) g = ddl_keep(key, (uint32_t)idx, thr24) ? g * inv_keep : 0.f;
    dpre2[idx] = g;
  }
}

void launch_head_fused_fc2(const float* slab, int S, int gx, int ntiles, const float* b2,
                           float* h2, const float* w, const float* bias, const int64_t* labels,
                           int B, const uint32_t* seed, uint32_t seed_v, uint32_t thr24,
                           float inv_keep, float* dlog, float* loss, float* dpre2,
                           hipStream_t st) {
  if (gx * 32 < B || ntiles != gx * (HK / 32))
    throw std::invalid_argument("head_fused_fc2: fc2 partial tiles do not cover [B, 512]");
  DDL_LAUNCH(head_fused_fc2_kernel, dim3(B), dim3(256), 0, st, slab, S, gx, ntiles, b2, h2, w,
             bias, labels, B, 1.f / (float)B, seed, seed_v, thr24, inv_keep, dlog, loss, dpre2);
}

void launch_head_fused(const float* h2, const float* w, const float* bias, const int64_t* labels,
                       int B, const uint32_t* seed, uint32_t seed_v, uint32_t thr24,
                       float inv_keep, float* dlog, float* loss, float* dpre2, hipStream_t st) {
  DDL_LAUNCH(head_fused_kernel, dim3(B), dim3(256), 0, st, h2, w, bias, labels, B,
             1.f / (float)B, seed, seed_v, thr24, inv_keep, dlog, loss, dpre2);
}

void launch_head_wgrad(const float* h2, const float* dlog, int B, float* gw, float* gb,
                       hipStream_t st) {
  const int wblocks = (HK + 1 + 3) / 4;
  DDL_LAUNCH(head_bwd_kernel, dim3(wblocks), dim3(256), 0, st, h2, nullptr, dlog, B,
                     wblocks, nullptr, 0u, 0u, 1.f, gw, gb, nullptr);
}

void launch_head_fwd(const float* h2, const float* w, const float* bias, const int64_t* labels,
                     int B, float* dlog, float* loss, int* correct, hipStream_t st) {
  DDL_LAUNCH(head_fwd_kernel, dim3(B), dim3(256), 0, st, h2, w, bias, labels, B,
                     1.f / (float)B, dlog, loss, correct);
}

void launch_head_bwd(const float* h2, const float* w, const float* dlog, int B,
                     const uint32_t* seed, uint32_t seed_v, uint32_t thr24, float inv_keep,
                     float* gw, float* gb,
                     float* dpre2, hipStream_t st) {
  const int wblocks = (HK + 1 + 3) / 4;  // one wave per dW_aug row
  const int dblocks = (B * HK + 255) / 256;
  DDL_LAUNCH(head_bwd_kernel, dim3(wblocks + dblocks), dim3(256), 0, st, h2, w, dlog, B,
                     wblocks, seed, seed_v, thr24, inv_keep, gw, gb, dpre2);
}

}  // namespace ddl
