// The CNN step engine: every forward / backward kernel launch of one worker step.
//
// Reference step: sess.run(grads) on the TF runtime, 14 host round trips
// to push, 14 to pull.  Here a step is ~20 GEMM-engine launches + 2 head kernels, all
// buffers preallocated (graph-capturable: no malloc, no sync).  The backward is split
// into 4 segments so the host can push a segment's gradients on a side stream while the
// next segment computes (SURVEY.md §5.8 bucket plan); inside a segment the weight-gradient
// GEMM runs on a second stream concurrently with the data-gradient GEMM that feeds the
// next segment (fork/join events, captured as parallel graph branches).
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "api.h"
#include "layers.h"
#include "engine_decl.h"

namespace ddl {

Engine::Engine() {
  // {tile config, split-K} per op: whole-step coordinate-descent tune
  // (scripts/step_tune.py over the scripts/op_bench.py per-op sweep) on one MI355X, batch 100,
  // single-stream backward with dual dgrad+wgrad launches: fwd+bwd 367 us (was 449 us)
  // (round 2, after the halo layout and the batch-minor weight-gradient enumeration: conv2
  // weight gradient on the basic BK 32 loop instead of the pipelined BK 16 one, 342.8 ->
  // 336.5 us, profiles/r2_runner_tune_halo.log)
  // fc1 forward on the K-wave launch (8 waves per workgroup, LDS reduction, no reduce launch):
  // 313.4 -> 310.6 us (profiles/r2_runner_tune_kwave.log); fc1 data gradient as the K-wave
  // half of one packed launch with its weight gradient (gemm_pack_kernel, 4 waves), instead
  // of the one-wave dual launch + wide reduce: 308.7 -> 304.4 us (profiles/r2_runner_tune_pack.log)
  // (round 3, after the direct conv1 kernels: fc2 data gradient on the K-wave half of a packed
  // launch with its weight gradient, like fc1's: 292.8 -> 291.5 us, profiles/r3_runner_tune.log)
  // (round 5, scripts/sched_ab.py on one MI355X, 5 alternating rounds of 300 steps: conv4
  // weight gradient and conv2 data gradient on the 16x16x4 MFMA tile (config 14), conv4 weight
  // gradient split 8: 295.3 -> 293.0 us, profiles/r5_sched_ab_mf16.log; then conv3 weight
  // gradient on config 14 too: 293.5 -> 292.7 us, profiles/r5_sched_ab_conv3w.log — conv2's
  // weight gradient on it loses 6 us)
  // (round 6: fc1's and fc2's forwards on the 16-row K-wave launch, 8 waves — fc2 then writes h2
  // itself and the head reads it instead of fc2's split-K partials: 260.7-261.0 -> 259.1-259.4
  // us/step, 4 interleaved rounds, profiles/r6_sched_ab_kw16.log)
  static const int defc[OP_COUNT] = {3, 3, 3, 3, CFG_KW16, CFG_KW16, CFG_KWAVE, 5, CFG_KWAVE, 5,
                                     3, CFG_MF16, 3, CFG_MF16, CFG_MF16, 3, 3};
  // (re-tuned in the real step with scripts/sched_ab.py after the compact 52-row conv3
  // enumeration and the wgrad row decode: conv3 forward split 4 + in-launch reduce instead of
  // stream-K 3072 workers, 372.4 -> 369.5 us; conv4 weight gradient split 4 instead of 8,
  // 370.5 -> 368.0 us; conv4 data gradient 2560 stream-K workers and conv3 weight gradient
  // split 12, 365.2 -> 362.3 us)
  // (round 2, with the tap-skipping K maps of conv3/conv4: conv4 data gradient split-K 4 with
  // a separate reduce instead of stream-K over the full K, 322.2 -> 313.3 us,
  // profiles/r2_runner_tune_kmap.log)
  // (round 3, conv forwards on the LDS-DMA main loop: conv2 / conv3 / conv4 forward split-K
  // 3 / 3 / 6 instead of 2 / 4 / 8, 302.5 -> 299.0 us fwd+bwd, scripts/sched_ab.py
  // --splits-variants, profiles/r3_sched_ab_ldsdma.log)
  // (round 6, after the row-wise data-gradient epilogues made the last arriver cheap: conv4's
  // data gradient split-K 5 with the in-launch reduce instead of 4 + the separate wide reduce,
  // conv3's split-K 5 instead of 8, and the conv3 dual dispatching its weight-gradient blocks
  // first (api.h dual_bfirst): 279.2 -> 267.7 us/step, scripts/sched_ab.py,
  // profiles/r6_sched_ab_grid.log; then conv2's weight gradient split-K 48 instead of 32 and
  // conv4's 6 instead of 8: 267.2 -> 264.8, profiles/r6_sched_ab_wgrad.log; conv4's forward
  // split-K 5 instead of 6 once the last arriver sums its partials in one batched round per 4:
  // 264.4 -> 262.9, profiles/r6_runner_tune.log, r6_sched_ab_zb.log)
  static const int defs[OP_COUNT] = {1, 3, 3, 5, 8, 8, 4, 1, 4, 1, 5, 6, 5, 12, 4, 48, 1024};
  // split-K reduce in-launch (last arriver) for these ops, separate wide-reduce kernel otherwise
  static const bool inl[OP_COUNT] = {0, 1, 1, 1, 0, 0, 1, 0, 0, 0, 1, 1, 1, 1, 1, 0, 0};
  memcpy(cfg, defc, sizeof(defc));
  memcpy(eval_cfg, defc, sizeof(defc));
  // eval forward at 10k-row chunks (scripts/eval_sweep.py, after the compact conv3 rows):
  // conv2-4 on 4-wave 64x64 blocks, full test-set eval 6.76 -> 6.66 ms (106 TF); round 2:
  // conv3 on the eval-only 128x128 block (2x2 waves of 64x64), 6.62 -> 6.53 ms (108 TF) —
  // the larger eval tiles (9-12) gain at most 1.4 %, so the eval is bound by the main loop,
  // not by tile shape (profiles/r2_eval_sweep_big_tiles.log)
  // round 3 (scripts/eval_sweep.py on the current build, profiles/r3_eval_sweep.log): the
  // one-wave 64x64 tile (4 fragments per wave, no LDS sharing between waves) for conv2-4,
  // full test-set eval 5.04 -> 4.64 ms
  eval_cfg[OP_CONV2_FWD] = 0;
  eval_cfg[OP_CONV3_FWD] = 0;
  eval_cfg[OP_CONV4_FWD] = 0;
  memcpy(splits, defs, sizeof(defs));
  for (int op = 0; op < OP_COUNT; ++op) wide[op] = inl[op] ? (1 << 20) : 1;
}

Engine::~Engine() {
  if (ev_fork) (void)hipEventDestroy(ev_fork);
  if (ev_join) (void)hipEventDestroy(ev_join);
  if (side) (void)hipStreamDestroy(side);
}

void Engine::init_streams() {
  if (side) return;
  (void)hipStreamCreateWithFlags(&side, hipStreamNonBlocking);
  (void)hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming);
  (void)hipEventCreateWithFlags(&ev_join, hipEventDisableTiming);
}

void Engine::op_shape(int op, int B, int* M, int* N, int* K) {
  int m = 0, n = 0, k = 0;
  switch (op) {
    case OP_CONV1_FWD: m = ConvFwd<28, 1, 32>::rows(B); n = 32; k = 25; break;
    case OP_CONV2_FWD: m = ConvFwd<14, 32, 64>::rows(B); n = 64; k = 800; break;
    case OP_CONV3_FWD: m = ConvFwd<7, 64, 128>::rows(B); n = 128; k = 1600; break;
    case OP_CONV4_FWD: m = ConvFwd<4, 128, 256>::rows(B); n = 256; k = 3200; break;
    case OP_FC1_FWD: m = B; n = 1024; k = 1024; break;
    case OP_FC2_FWD: m = B; n = 512; k = 1024; break;
    case OP_FC2_DGRAD: m = B; n = 1024; k = 512; break;
    case OP_FC2_WGRAD: m = 1025; n = 512; k = B; break;
    case OP_FC1_DGRAD: m = B; n = 1024; k = 1024; break;
    case OP_FC1_WGRAD: m = 1025; n = 1024; k = B; break;
    case OP_CONV4_DGRAD: m = B * 16; n = 128; k = 6400; break;
    case OP_CONV4_WGRAD: m = 3201; n = 256; k = WgradConv4::k_of(B); break;
    case OP_CONV3_DGRAD: m = B * 49; n = 64; k = 3200; break;
    case OP_CONV3_WGRAD: m = 1601; n = 128; k = WgradConv3::k_of(B); break;
    case OP_CONV2_DGRAD: m = B * 196; n = 32; k = 1600; break;
    case OP_CONV2_WGRAD: m = 801; n = 64; k = WgradConv2::k_of(B); break;
    case OP_CONV1_WGRAD: m = 26; n = 32; k = WgradConv1::padded_k(B); break;
    default: break;
  }
  *M = m; *N = n; *K = k;
}

#define TILE_0 64, 64, 32, 1, 1
#define TILE_1 128, 64, 32, 2, 1
#define TILE_2 64, 32, 32, 1, 1
#define TILE_3 32, 32, 32, 1, 1
#define TILE_4 32, 64, 32, 1, 1
#define TILE_5 32, 32, 16, 1, 1   // software-pipelined main loop (gemm.h GemmTile::PIPE)
#define TILE_6 64, 64, 32, 2, 2   // 4 waves of 32x32 sharing one LDS-staged 64x64 block tile
#define TILE_7 64, 32, 32, 2, 1   // 2 waves of 32x32 along M
#define TILE_8 32, 64, 32, 1, 2   // 2 waves of 32x32 along N

static size_t slab_need(int c, int M, int N, int K, int s) {
  switch (c) {
    // reduces in LDS; an op without a K-wave instantiation falls back to the 32x32 split-K
    // launch with the same split factor (engine_impl.h launch_cfg), so size for that
    case CFG_KWAVE: return gemm_slab_f4<TILE_3>(M, N, K, s);
    case CFG_MF16: return gemm_slab_f4<TILE_3>(M, N, K, s);  // same 32x32 partial layout
    case CFG_KW16: return gemm_slab_f4<TILE_3>(M, N, K, s);  // (fallback: 32x32 split-K)
    case 0: return gemm_slab_f4<TILE_0>(M, N, K, s);
    case 1: return gemm_slab_f4<TILE_1>(M, N, K, s);
    case 2: return gemm_slab_f4<TILE_2>(M, N, K, s);
    case 3: return gemm_slab_f4<TILE_3>(M, N, K, s);
    case 4: return gemm_slab_f4<TILE_4>(M, N, K, s);
    case 5: return gemm_slab_f4<TILE_5>(M, N, K, s);
    case 6: return gemm_slab_f4<TILE_6>(M, N, K, s);
    case 7: return gemm_slab_f4<TILE_7>(M, N, K, s);
    default: return gemm_slab_f4<TILE_8>(M, N, K, s);
  }
}

size_t Engine::slab_floats_needed(int B) const {
  size_t mx = 0;
  for (int op = 0; op < OP_COUNT; ++op) {
    int M, N, K;
    op_shape(op, B, &M, &N, &K);
    const size_t f = 4 * slab_need(cfg[op], M, N, K, splits[op]);
    if (f > mx) mx = f;
  }
  return mx;
}

static size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

// floats per image: p1..p3 and d4..d2 with the 2-pixel zero halo (layers.h kHalo)
static const size_t kActPer[] = {18 * 18 * 32, 11 * 11 * 64, 8 * 8 * 128, 1024, 1024, 512, 16, 1,
                                 512, 1024, 8 * 8 * 256, 11 * 11 * 128, 18 * 18 * 64, 25088};
static const size_t kCodePer[] = {6272, 3136, 2048, 1024};

size_t Engine::workspace_bytes() const {
  const size_t B = (size_t)max_batch;
  size_t f = 0;
  for (size_t p : kActPer) f += al256(4 * B * p);
  f += 2 * al256(4 * slab_floats);
  for (size_t c : kCodePer) f += al256(B * c);
  f += 256;                          // correct counter
  f += 2 * al256(4 * kMaxTickets);   // split-K arrival tickets (two streams)
  return f;
}

void Engine::bind_workspace(void* base) {
  const size_t B = (size_t)max_batch;
  char* p = (char*)base;
  auto take = [&](size_t bytes) { char* r = p; p += al256(bytes); return r; };
  float** acts[] = {&p1, &p2, &p3, &p4, &h1, &h2, &dlog, &loss,
                    &dpre2fc, &dpre1fc, &d4, &d3, &d2, &d1};
  for (int i = 0; i < 14; ++i) *acts[i] = (float*)take(4 * B * kActPer[i]);
  for (int s = 0; s < 2; ++s) {
    scratch[s].slab = take(4 * slab_floats);
    scratch[s].slab_f4 = slab_floats / 4;
  }
  uint8_t** codes[] = {&c1, &c2, &c3, &c4};
  for (int i = 0; i < 4; ++i) *codes[i] = (uint8_t*)take(B * kCodePer[i]);
  correct = (int*)take(256);
  for (int s = 0; s < 2; ++s) {
    scratch[s].tickets = (int*)take(4 * kMaxTickets);
    scratch[s].max_tiles = kMaxTickets;
  }
}

void Engine::run_op(int op, const float* x, int B, const uint32_t* seed, bool train,
                    hipStream_t st, int si) {
  if (op == OP_CONV1_FWD && conv1_direct) {
    launch_conv1_fwd(x, P[0], P[1], p1, train ? c1 : nullptr, B, st);
    return;
  }
  // (the dual path fuses it with conv2's weight-gradient reduce: engine_impl.h dual_then_b)
  if (op == OP_CONV1_WGRAD && conv1_wgrad_direct &&
      conv1_wgrad_fits(B, slab_floats, scratch[si].max_tiles)) {
    launch_conv1_wgrad_only(x, d1, B, G[0], G[1], static_cast<float*>(scratch[si].slab),
                            scratch[si].tickets, st);
    return;
  }
  switch (op) {
#define DDL_RUN(OPC) \
  case OPC: run_op_inst<OPC>(*this, x, B, seed, train, st, si); break;
    DDL_RUN(OP_CONV1_FWD) DDL_RUN(OP_CONV2_FWD) DDL_RUN(OP_CONV3_FWD) DDL_RUN(OP_CONV4_FWD)
    DDL_RUN(OP_FC1_FWD) DDL_RUN(OP_FC2_FWD) DDL_RUN(OP_FC2_DGRAD) DDL_RUN(OP_FC2_WGRAD)
    DDL_RUN(OP_FC1_DGRAD) DDL_RUN(OP_FC1_WGRAD) DDL_RUN(OP_CONV4_DGRAD) DDL_RUN(OP_CONV4_WGRAD)
    DDL_RUN(OP_CONV3_DGRAD) DDL_RUN(OP_CONV3_WGRAD) DDL_RUN(OP_CONV2_DGRAD)
    DDL_RUN(OP_CONV2_WGRAD) DDL_RUN(OP_CONV1_WGRAD)
#undef DDL_RUN
    default: break;
  }
}

// a push / ready-flag tail (tail.h kinds 1, 2) with no launch to ride in
__global__ void __launch_bounds__(64) push_tail_kernel(UpdTail t) { tail_body(t, blockIdx.x); }

void Engine::flush_tail(hipStream_t st) {
  if (tail.kind != 0) {
    if (tail.nblocks > 0)
      hipLaunchKernelGGL(push_tail_kernel, dim3(tail.nblocks), dim3(64), 0, st, tail);
    tail = UpdTail();
    return;
  }
  for (int i = 0; i < tail.npieces; ++i) {
    const UpdPiece& p = tail.p[i];
    launch_adam_c(p.w, p.g, p.m, p.v, p.n, p.lr_t, tail.c1, tail.c2, tail.eps, tail.scale, st);
  }
  tail = UpdTail();
}

void Engine::flush_fc_wgrad(const float* x, int B, const uint32_t* seed, hipStream_t st) {
  const int pend = fc_wgrad_pending;
  fc_wgrad_pending = 0;
  if (pend & 1) run_op(OP_FC2_WGRAD, x, B, seed, true, st, 0);
  if (pend & 2) run_op(OP_FC1_WGRAD, x, B, seed, true, st, 0);
}

void Engine::flush_head_wgrad(int B, hipStream_t st) {
  if (!head_wgrad_pending) return;
  launch_head_wgrad(h2, dlog, B, G[12], G[13], st);
  head_wgrad_pending = 0;
}

void Engine::forward(const float* x, int B, const uint32_t* seed, bool train, hipStream_t st,
                     bool defer_fc2) {
  fc2_slab = nullptr;  // (a deferred fc2 reduce nobody took: this forward rewrites h2 anyway)
  fc_wgrad_pending = 0;  // (likewise: their inputs are about to be rewritten)
  for (int op = OP_CONV1_FWD; op < OP_FC2_FWD; ++op) run_op(op, x, B, seed, train, st, 0);
  if (!(train && defer_fc2 && fc2_in_head && !concurrent && run_fc2_deferred(*this, x, B, seed, st)))
    run_op(OP_FC2_FWD, x, B, seed, train, st, 0);
}

void Engine::flush_fc2(const uint32_t* seed, int B, hipStream_t st) {
  if (fc2_slab) run_fc2_reduce(*this, seed, B, st);
}

// The side stream waits for everything enqueued on `st` so far.
void Engine::fork(hipStream_t st) {
  (void)hipEventRecord(ev_fork, st);
  (void)hipStreamWaitEvent(side, ev_fork, 0);
}

// `st` waits for everything enqueued on the side stream so far.
void Engine::join(hipStream_t st) {
  (void)hipEventRecord(ev_join, side);
  (void)hipStreamWaitEvent(st, ev_join, 0);
}

void Engine::wgrad(int op, const float* x, int B, const uint32_t* seed, hipStream_t st) {
  fork(st);
  run_op(op, x, B, seed, true, side, 1);
}

void Engine::backward_segment(int s, const float* x, const int64_t* labels, int B,
                              const uint32_t* seed, hipStream_t st) {
  if (concurrent && side) {  // weight gradients on the side stream (fork/join per segment)
    flush_tail(st);
    flush_fc2(seed, B, st);
    switch (s) {
      case 0:
        launch_head_fwd(h2, P[12], P[13], labels, B, dlog, loss, nullptr, st);
        launch_head_bwd(h2, P[12], dlog, B, seed, seed_value, thr24, inv_keep, G[12], G[13],
                        dpre2fc, st);
        wgrad(OP_FC2_WGRAD, x, B, seed, st);
        run_op(OP_FC2_DGRAD, x, B, seed, true, st, 0);
        wgrad(OP_FC1_WGRAD, x, B, seed, st);
        run_op(OP_FC1_DGRAD, x, B, seed, true, st, 0);
        break;
      case 1:
        wgrad(OP_CONV4_WGRAD, x, B, seed, st);
        run_op(OP_CONV4_DGRAD, x, B, seed, true, st, 0);
        break;
      case 2:
        wgrad(OP_CONV3_WGRAD, x, B, seed, st);
        run_op(OP_CONV3_DGRAD, x, B, seed, true, st, 0);
        break;
      case 3:
        wgrad(OP_CONV2_WGRAD, x, B, seed, st);
        run_op(OP_CONV2_DGRAD, x, B, seed, true, st, 0);
        wgrad(OP_CONV1_WGRAD, x, B, seed, st);
        break;
      default: break;
    }
    join(st);
    return;
  }
  // single stream: each layer's dgrad + wgrad as one dual launch
  switch (s) {
    case 0:
      // one head launch (per-sample fwd + dlogits + dh2); fc3's dW/db ride in the fc2 dual.
      // With fc2's reduce deferred the head also finishes fc2 (h2 = its reduce + epilogue).
      if (fc2_slab) {
        launch_head_fused_fc2(fc2_slab, fc2_S, fc2_gx, fc2_ntiles, P[11], h2, P[12], P[13],
                              labels, B, seed, seed_value, thr24, inv_keep, dlog, loss,
                              dpre2fc, st);
        fc2_slab = nullptr;
      } else {
        launch_head_fused(h2, P[12], P[13], labels, B, seed, seed_value, thr24, inv_keep, dlog,
                          loss, dpre2fc, st);
      }
      head_wgrad_pending = 1;
      run_dual_inst<OP_FC2_DGRAD, OP_FC2_WGRAD>(*this, x, B, seed, st);
      flush_head_wgrad(B, st);
      run_dual_inst<OP_FC1_DGRAD, OP_FC1_WGRAD>(*this, x, B, seed, st);
      break;
    case 1:
      run_dual_inst<OP_CONV4_DGRAD, OP_CONV4_WGRAD>(*this, x, B, seed, st);
      flush_fc_wgrad(x, B, seed, st);  // (a conv4 pair that ran back to back took none of them)
      break;
    case 2: run_dual_inst<OP_CONV3_DGRAD, OP_CONV3_WGRAD>(*this, x, B, seed, st); break;
    case 3:
      run_dual_then_inst<OP_CONV2_DGRAD, OP_CONV2_WGRAD, OP_CONV1_WGRAD>(*this, x, B, seed, st);
      break;
    default: break;
  }
}

void Engine::eval_count(const float* x, const int64_t* labels, int B, hipStream_t st) {
  forward(x, B, nullptr, false, st);  // (flushes a pending fc2 reduce of a training forward)
  launch_head_fwd(h2, P[12], P[13], labels, B, nullptr, nullptr, correct, st);
}

}  // namespace ddl
