// Host-side launch API of the gfx950 kernels (raw device pointers + hipStream_t; no torch).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "runtime/session.h"
#include "scratch.h"
#include "tail.h"

namespace ddl {

class ShmMailbox;

// ---- optimizer (optim.hip) -------------------------------------------------------------------
void launch_adam(float* w, const float* g, float* m, float* v, int64_t n, float lr_t, float b1,
                 float b2, float eps, float scale, hipStream_t st);
// same with c1 = 1 - beta1, c2 = 1 - beta2 precomputed (bit-identical to launch_adam)
void launch_adam_c(float* w, const float* g, float* m, float* v, int64_t n, float lr_t, float c1,
                   float c2, float eps, float scale, hipStream_t st, int max_grid = 2048);
void launch_momentum(float* w, const float* g, float* m, int64_t n, float lr, float mu,
                     float scale, hipStream_t st);
void launch_scale(float* p, int64_t n, float a, hipStream_t st);

// ---- conv1 forward as a direct LDS-staged kernel (conv1.hip) --------------------------------
// x [B,784], w [25,32], bias [32] -> pooled p1 [B,18,18,32] (halo layout) + codes [B,14,14,32]
void launch_conv1_fwd(const float* x, const float* w, const float* bias, float* out,
                      uint8_t* code, int B, hipStream_t st);
// conv1's weight / bias gradient, direct kernel with in-launch reduce (conv1.h); part /
// tickets: c1w_scratch_floats(B) floats and c1w_groups(B) + 1 zeroed ints of scratch
void launch_conv1_wgrad_only(const float* x, const float* d1, int B, float* gw, float* gb,
                             float* part, int* tickets, hipStream_t st);
bool conv1_wgrad_fits(int B, size_t slab_floats, int max_tickets);

// ---- classifier head (head.hip) --------------------------------------------------------------
void launch_head_fwd(const float* h2, const float* w, const float* bias, const int64_t* labels,
                     int B, float* dlog, float* loss, int* correct, hipStream_t st);
// fused head: logits, loss, dlogits and dh2 (with fc2's dropout backward) per sample; fc3's
// weight gradient is left to launch_head_wgrad or the next dual launch (head.h)
void launch_head_fused(const float* h2, const float* w, const float* bias, const int64_t* labels,
                       int B, const uint32_t* seed, uint32_t seed_v, uint32_t thr24,
                       float inv_keep, float* dlog, float* loss, float* dpre2, hipStream_t st);
void launch_head_wgrad(const float* h2, const float* dlog, int B, float* gw, float* gb,
                       hipStream_t st);
// launch_head_fused that first finishes fc2's forward: h2 = dropout(sum of the S split-K
// partials of fc2's one-wave 32x32 tiles + b2) per sample, stored for fc3's weight gradient
void launch_head_fused_fc2(const float* slab, int S, int gx, int ntiles, const float* b2,
                           float* h2, const float* w, const float* bias, const int64_t* labels,
                           int B, const uint32_t* seed, uint32_t seed_v, uint32_t thr24,
                           float inv_keep, float* dlog, float* loss, float* dpre2,
                           hipStream_t st);
void launch_head_bwd(const float* h2, const float* w, const float* dlog, int B,
                     const uint32_t* seed, uint32_t seed_v, uint32_t thr24, float inv_keep,
                     float* gw, float* gb, float* dpre2, hipStream_t st);

// ---- diagnostics (diag.hip) -------------------------------------------------------------------
void launch_mfma_peak(float* out, int blocks, int iters, hipStream_t st, int kind = 0);
void launch_gemm_nomem(float* out, int M, int N, int K, int splits, void* slab, int* tickets,
                       hipStream_t st);

// ---- the CNN step engine (engine.hip) --------------------------------------------------------
// GEMM-shaped ops, in SURVEY.md §2.6 order.  Index into Engine::splits / Engine::cfg.
enum Op {
  OP_CONV1_FWD = 0, OP_CONV2_FWD, OP_CONV3_FWD, OP_CONV4_FWD, OP_FC1_FWD, OP_FC2_FWD,
  OP_FC2_DGRAD, OP_FC2_WGRAD, OP_FC1_DGRAD, OP_FC1_WGRAD,
  OP_CONV4_DGRAD, OP_CONV4_WGRAD, OP_CONV3_DGRAD, OP_CONV3_WGRAD,
  OP_CONV2_DGRAD, OP_CONV2_WGRAD, OP_CONV1_WGRAD,
  OP_COUNT
};

// Block-tile configurations selectable per op at run time (gemm.h template args
// <BM, BN, BK=32, WM, WN>): 0 = 64x64 (1 wave 64x64), 1 = 128x64 (2 waves 64x64),
// 2 = 64x32 (1 wave), 3 = 32x32 (1 wave), 4 = 32x64 (1 wave),
// 5 = 32x32 with BK = 16 and the software-pipelined main loop (1 wave),
// 6 = 64x64 (4 waves of 32x32), 7 = 64x32 (2 waves of 32x32), 8 = 32x64 (2 waves of 32x32):
// multi-wave blocks share each staged operand tile between waves (half the L1/L2 bytes per
// MFMA of one-wave 32x32 blocks at 64x64), at one barrier per K tile.
constexpr int NUM_TILE_CFGS = 9;
// Eval-only large-M configs (conv forward ops at 10k-row test-set chunks; no split-K, so only
// instantiated for those ops): 9 = 128x128 (2x2 waves of 64x64), 10 = 128x64 (2x2 waves of
// 64x32), 11 = 256x64 (4x1 waves of 64x64), 12 = 128x128 (4x1 waves of 32x128).
constexpr int NUM_EVAL_TILE_CFGS = 13;
// training-only: 32x32 one-wave tiles with the K range split over the waves of ONE workgroup
// (gemm.h gemm_kwave_kernel; `splits` picks 4 / 8 / 16 waves); fc layers only
constexpr int CFG_KWAVE = 13;
// training-only: the one-wave 32x32x32 tile on v_mfma_f32_16x16x4_f32 with LDS-DMA staging
// (gemm.h GemmTile::mainloop_dma16); conv2-4 forward / data gradient / weight gradient only
// (other ops fall back to config 3)
constexpr int CFG_MF16 = 14;
// training-only: the K-wave launch on 16-row tiles (kwave16.h gemm_kw16_kernel; `splits` picks 4 /
// 8 / 16 waves); the fc forwards only (other ops fall back to config 3)
constexpr int CFG_KW16 = 15;
// (configs 16-20 — one-wave multi-fragment LDS-DMA tiles and the 32x32 ring tiles — were
// measured in round 5, never won a launch and were removed: docs/DESIGN.md)

struct Engine {
  const float* P[14] = {};   // parameter tensors v0..v13 (any flat layout)
  float* G[14] = {};         // gradient tensors v0..v13
  int max_batch = 0;         // activation buffers sized for this batch
  int train_batch = 0;       // slab sized for this batch with the current splits/cfgs
  int splits[OP_COUNT];
  int cfg[OP_COUNT];
  int eval_cfg[OP_COUNT];    // tile configs of the no-split eval forward (train = false)
  int wide_thr = 1;          // default split count above which the separate wide reduce is used
  int wide[OP_COUNT];        // per op: z > wide[op] -> separate wide reduce (mode 2), else the
                             // in-launch last-arriver reduction (mode 1)
  uint32_t thr24 = 0;        // dropout threshold (train)
  uint32_t seed_value = 0;   // dropout seed used when a step is given no device seed word
  float inv_keep = 1.f;
  // weight-gradient GEMMs on a second stream.  Off by default: a cross-queue event wait costs
  // tens of microseconds of GPU idle on MI355X/ROCm (step timelines), more than the overlap
  // gains; dgrad/wgrad concurrency comes from fused dual-problem launches instead.
  bool concurrent = false;
  bool dual = true;          // single stream: dgrad + wgrad of a layer in one launch
  // bit op: that dual launch dispatches its second problem first.  conv2's (weight gradient
  // split 32 ways, the longer pole) measured 0.3663 -> 0.3650 ms/step; conv4's / conv3's worse
  // (their data gradients are the longer poles; conv4's stream-K loses its XCD-major numbering).
  int dual_bfirst = (1 << OP_CONV2_DGRAD) | (1 << OP_CONV3_DGRAD);
  int dual_order(int op) const { return (dual_bfirst >> op) & 1; }

  // workspace carve-out
  float *p1 = nullptr, *p2 = nullptr, *p3 = nullptr, *p4 = nullptr, *h1 = nullptr, *h2 = nullptr;
  float *dlog = nullptr, *loss = nullptr, *dpre2fc = nullptr, *dpre1fc = nullptr;
  float *d4 = nullptr, *d3 = nullptr, *d2 = nullptr, *d1 = nullptr;
  uint8_t *c1 = nullptr, *c2 = nullptr, *c3 = nullptr, *c4 = nullptr;
  int* correct = nullptr;
  size_t slab_floats = 0;
  SplitScratch scratch[2];   // [0] main stream, [1] weight-gradient stream
  static constexpr int kMaxTickets = 8192;

  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // optimizer tail (tail.h) for the next dual launch; consumed (and cleared) by it, or by
  // flush_tail() as a launch of its own when no dual launch takes it
  UpdTail tail;
  // the LAST segment's update (W = 1 tail path): conv1's part applied by its weight-gradient
  // reduce epilogue, the rest as tail blocks of that launch (engine_impl.h dual_then_b).
  // Cleared when taken; the runner launches it as before when it is still pending.
  UpdTail final_upd;
  // eval forward: conv2 on the tap-skipping K map (DDL_EVAL_KMAP2=0: the image-major GEMM)
  bool eval_kmap2 = [] {
    const char* e = getenv("DDL_EVAL_KMAP2");
    return !e || e[0] != '0';
  }();
  // conv1 forward on the direct LDS-staged kernel (conv1.hip) instead of the GEMM engine's
  // gather-bound K = 25 launch.  DDL_CONV1_DIRECT=0: the GEMM path
  bool conv1_direct = [] {
    const char* e = getenv("DDL_CONV1_DIRECT");
    return !e || e[0] != '0';
  }();
  // conv1's weight gradient on the direct kernel with its in-launch reduce (conv1.h), riding
  // with conv2's weight-gradient reduce, instead of the GEMM launch + wide reduce launch.
  // DDL_CONV1_WGRAD_DIRECT=0: the GEMM path
  bool conv1_wgrad_direct = [] {
    const char* e = getenv("DDL_CONV1_WGRAD_DIRECT");
    return !e || e[0] != '0';
  }();
  // fc3 weight gradient still to compute (fused head kernel ran): taken by the fc2 dual launch
  int head_wgrad_pending = 0;
  // the fc backward's packed launches leave the fc weight gradients (bit 0: fc2, bit 1: fc1) to
  // the conv4 dual launch (engine_impl.h FcWgradAux); false: they stay in the packs
  bool fc_wgrad_defer = true;
  int fc_wgrad_pending = 0;
  // fc2 forward's split-K partials whose reduce + epilogue the head kernel runs (the step's
  // forward with defer_fc2, one-wave 32x32 split-K in mode 2): one launch fewer per step.
  // DDL_FC2_REDUCE_IN_HEAD=0 keeps the separate reduce launch.
  bool fc2_in_head = [] {
    const char* e = getenv("DDL_FC2_REDUCE_IN_HEAD");
    return !e || e[0] != '0';
  }();
  const float* fc2_slab = nullptr;  // pending partials (null: h2 is final)
  int fc2_S = 0, fc2_gx = 0, fc2_ntiles = 0;

  Engine();
  ~Engine();
  void init_streams();
  // M, N, K of op `op` at batch B (used for slab sizing and by tests)
  static void op_shape(int op, int B, int* M, int* N, int* K);
  size_t slab_floats_needed(int B) const;
  size_t workspace_bytes() const;
  void bind_workspace(void* base);

  // forward through fc2 (train: dropout on, configured split-K; eval: no dropout, no split).
  // defer_fc2: the caller runs backward_segment(0) next, so fc2's wide reduce may be left to
  // the head kernel (fc2_in_head); otherwise h2 is final when forward returns
  void forward(const float* x, int B, const uint32_t* seed, bool train, hipStream_t st,
               bool defer_fc2 = false);
  // launch fc2's pending reduce on its own (no-op when none is pending)
  void flush_fc2(const uint32_t* seed, int B, hipStream_t st);
  // backward segment s (0: head+fc, 1: conv4, 2: conv3, 3: conv2+conv1); weight-gradient
  // GEMMs fork onto the side stream and join back at the end of the segment
  void backward_segment(int s, const float* x, const int64_t* labels, int B,
                        const uint32_t* seed, hipStream_t st);
  // eval: forward(train=false) + correct-count accumulation into *correct
  void eval_count(const float* x, const int64_t* labels, int B, hipStream_t st);
  // run a single GEMM op on `st` with scratch `si` (tests / tuning)
  void run_op(int op, const float* x, int B, const uint32_t* seed, bool train, hipStream_t st,
              int si = 0);
  // launch a pending optimizer tail on its own (no-op when none is pending)
  void flush_tail(hipStream_t st);
  void flush_head_wgrad(int B, hipStream_t st);
  // launch pending fc weight gradients on their own (no-op when none are pending)
  void flush_fc_wgrad(const float* x, int B, const uint32_t* seed, hipStream_t st);

 private:
  void fork(hipStream_t st);
  void join(hipStream_t st);
  void wgrad(int op, const float* x, int B, const uint32_t* seed, hipStream_t st);
};

// ---- native synchronous step runner (runner.hip) -------------------------------------------
struct RunnerRange {
  int64_t lo, hi;       // plan-buffer element range [lo, hi)
  int64_t state_off;    // offset of the range's optimizer state in the unit's m / v
};
struct RunnerUnit {
  // AR: all-reduce + update on replicated state (the last bucket); XGMI_REPL: its xGMI form
  enum Kind { LOCAL = 0, RS = 1, REDUCE = 2, XGMI = 3, AR = 4, XGMI_REPL = 5 };
  int seg = 0;          // backward segment after which the unit's gradients are complete
  int kind = LOCAL;
  int host = 0;         // REDUCE: rank that owns the PS
  int ps = 0;           // index into the per-step lr_t table (RS: this rank's PS)
  std::vector<RunnerRange> ranges;
  float* m = nullptr;   // optimizer state base of the owning PS (null where not hosted)
  float* v = nullptr;
  float* shard = nullptr;  // RS: 1/W chunk buffer
  int bucket = -1;         // XGMI: bucket index of the runner's PeerExchange
};

// ---- parameter-server exchange over xGMI peer memory (xgmi.hip) ------------------------------
constexpr int kXgmiMaxPeers = 16;
// flat plans: one bucket per backward segment (<= 8); tensor-granular plans: one OWNER bucket per
// (PS, segment) exchange unit (<= 8 PS x 4 segments)
constexpr int kXgmiMaxBuckets = 32;
constexpr int kXgmiMaxRuns = 8;   // plan-buffer ranges of one owner bucket
#ifndef DDL_XGMI_MAX_SLICES
#define DDL_XGMI_MAX_SLICES 512
#endif
constexpr int kXgmiMaxSlices = DDL_XGMI_MAX_SLICES;
struct XgmiTable {               // every rank's IPC-mapped buffers, indexed by rank
  float* params[kXgmiMaxPeers];
  float* inbox[kXgmiMaxPeers];
  uint32_t* flags[kXgmiMaxPeers];
};
struct XgmiLaunch {              // one bucket's kernel arguments
  int world, rank, bucket, nbuckets, final_wait, opt;
  uint32_t epoch;
  int64_t lo, c, inbox_off, slice;
  int nslices[kXgmiMaxBuckets];
  const float* grads;
  float* m;
  float* v;
  float lr_t, c1, c2, eps, lr, mu, scale, coef;
  int* err;
  long long timeout_ticks;
  int check;                     // DDL_XGMI_CHECK: per-(bucket, source, slice) inbox checksums
  int repl_bucket;               // the replicated bucket (-1: none)
  int owners[kXgmiMaxBuckets];   // -1: chunk r of the bucket on rank r; >= 0: single owner rank
  // the READY gate ahead of this kernel on the comm stream timed out (host word, or null): the
  // segment's gradients may be incomplete, so the kernel publishes nothing (no pushes, no
  // ARRIVE / DONE words); the peers then time out too and every host raises
  const int* gate_err;
  // owner buckets: the launched bucket's runs (plan-buffer range, element offset in the owner
  // PS's optimizer state, offset in the bucket's concatenation, slice size, first slice)
  int owner, nruns;
  int64_t run_lo[kXgmiMaxRuns], run_n[kXgmiMaxRuns], run_soff[kXgmiMaxRuns];
  int64_t run_voff[kXgmiMaxRuns], run_slice[kXgmiMaxRuns];
  int run_sl0[kXgmiMaxRuns + 1];
  int64_t rslot;                 // the replicated bucket's inbox slot stride (floats)
};
// One bucket of a PeerExchange.  owner < 0: a single plan-buffer range split into W equal chunks,
// chunk r owned by rank r (the flat plan: reduce-scatter form).  owner >= 0: one PS's exchange
// unit of a tensor-granular plan (reference none / contiguous / greedy, lpt; or a flat plan with
// fewer PS than ranks) — every rank pushes the whole unit to its owner, which sums, updates with
// that PS's optimizer state (run r at state_offs[r]) and pushes the parameters to every rank.
struct XgmiBucketSpec {
  std::vector<std::pair<int64_t, int64_t>> runs;
  std::vector<int64_t> state_offs;
  int owner = -1;
};
struct XgmiUpdate {              // owner-side update of one bucket chunk
  int opt = 0;                   // 0 Adam (TF1), 1 momentum, 2 self-test (w := summed g)
  float* m = nullptr;            // optimizer state of this rank's chunk of the bucket
  float* v = nullptr;
  float lr_t = 0.f, c1 = 0.1f, c2 = 0.001f, eps = 1e-8f, lr = 0.f, mu = 0.9f;
  float scale = 1.f, coef = 1.f;
};

// The xGMI self-test's stale-L2 probe (xgmi.hip): every XCD reads every line of `a` (want null:
// warms the eight L2s) or counts into out[0] the elements that differ from `want`
void launch_xcd_sweep(const float* a, const float* want, int64_t n, int* out, hipStream_t st);

class PeerExchange {
 public:
  // buckets: [lo, hi) ranges of the flat plan buffer, each divisible by 4 * world; rank r owns
  // chunk r of every bucket.  Allocates the inbox (one slot per source rank) and the flags.
  // repl_bucket >= 0: that bucket is exchanged all-to-all and updated on every rank with
  // replicated optimizer state (xgmi_repl_kernel), instead of by its chunk owners
  PeerExchange(float* params, const float* grads, int64_t total, int world, int rank,
               const std::vector<std::pair<int64_t, int64_t>>& buckets, int max_slices,
               int repl_bucket = -1);
  // general form: equal-chunk and owner buckets (XgmiBucketSpec)
  PeerExchange(float* params, const float* grads, int64_t total, int world, int rank,
               const std::vector<XgmiBucketSpec>& buckets, int max_slices, int repl_bucket = -1);
  ~PeerExchange();
  std::string handle() const;                         // this rank's IPC handles, as bytes
  void open(const std::vector<std::string>& handles);  // every rank's, in rank order
  // the fused push / owner update / pull of one bucket at step `epoch` (same on all ranks)
  // gated: the launch sits behind the runner's READY gate on the comm stream (checks its error
  // word before publishing anything)
  void launch(int bucket, uint32_t epoch, const XgmiUpdate& u, bool final_wait, hipStream_t st,
              bool gated = false);
  int error() const;             // nonzero once a wait timed out (1 arrive, 2 done)
  // the runner's READY-gate error word, checked by every bucket kernel before it publishes
  void set_gate_error(const int* w) { gate_err_ = w; }
  // unmap the peers' buffers and free this rank's (after the device has drained); idempotent
  void close();
  double timeout_s() const { return timeout_s_; }
  int num_buckets() const { return (int)bk_.size(); }
  int nslices(int b) const { return bk_[b].nslice; }
  int64_t chunk(int b) const { return bk_[b].c; }
  int owner(int b) const { return bk_[b].owner; }
  int world() const { return world_; }
  int repl_bucket() const { return repl_; }
  bool check_mode() const { return check_; }

 private:
  struct Bucket {
    int64_t lo, c, inbox_off, slice;
    int64_t slot = 0;  // the replicated bucket: floats per (parity, source) inbox slot
    int nslice;
    int owner = -1;
    std::vector<int64_t> run_lo, run_n, run_soff, run_voff, run_slice;
    std::vector<int> run_sl0;
  };
  void init(const std::vector<XgmiBucketSpec>& buckets, int max_slices);
  void fill(int bucket, uint32_t epoch, const XgmiUpdate& u, bool final_wait, bool gated,
            XgmiLaunch& a) const;
  int repl_ = -1;
  bool check_ = false;
  float* params_;
  const float* grads_;
  int64_t total_;
  int world_, rank_;
  std::vector<Bucket> bk_;
  float* inbox_ = nullptr;
  int64_t inbox_elems_ = 0;
  uint32_t* flags_ = nullptr;
  size_t flag_bytes_ = 0;
  int* err_ = nullptr;
  const int* gate_err_ = nullptr;
  double timeout_s_ = 60.0;
  XgmiTable table_{};
  void* opened_[kXgmiMaxPeers][3] = {};
  bool opened_ok_ = false;
};

// ---- asynchronous PS over xGMI peer memory (xgmi_async.hip) ----------------------------------
constexpr int kAsyncMaxPs = 64;
constexpr int kAsyncMaxSlices = 512;
// a rank's uncached device flags: its DONE words as a worker (dense over all PS' slices)
constexpr int kAsyncDense = kAsyncMaxPs * kAsyncMaxSlices;
constexpr size_t kAsyncFlagWords = (size_t)kAsyncDense;
struct AsyncShard {              // one PS's contiguous range of the flat buffer
  int64_t lo, n, slice, inbox_off;
  int host, nslice;
  int slice0;                    // its first slice in the dense numbering of all PS' slices
};
struct AsyncTable {
  float* params[kXgmiMaxPeers];  // every rank's worker parameter buffer (IPC-mapped)
  float* inbox[kXgmiMaxPeers];
  uint32_t* flags[kXgmiMaxPeers];
  uint32_t* done;                // DONE[worker][ps][slice] in host memory shared by all ranks
  uint32_t* posted;              // the arrival board POSTED[ps][worker][slice], same segment
  // this rank's gradient buffer: with `elide` set, a push to a PS this rank hosts itself only
  // posts its words, and the apply of this worker's push reads the gradient here instead of an
  // inbox copy (the worker overwrites it only after its pull gate, i.e. after that apply)
  const float* grads;
  int elide;
  AsyncShard shard[kAsyncMaxPs];
};

class AsyncPeer {
 public:
  AsyncPeer(float* params, const float* grads, int64_t total, int world, int rank,
            const std::vector<std::pair<int64_t, int64_t>>& ps_ranges,
            const std::vector<int>& ps_host, int max_slices);
  ~AsyncPeer();
  std::string handle() const;
  void open(const std::vector<std::string>& handles);
  void close();  // unmap peers, free buffers and the shm board (after a device drain); idempotent
  // worker: every PS shard of the gradient (x coef) into its host's inbox slot, round `epoch`
  void push_all(uint32_t epoch, float coef, hipStream_t st);
  // the same for the listed PS only (one launch); with_gate: plus the pull gate of round
  // `epoch` as the launch's last block (the round's last push, async_runner.hip)
  void push_set(const std::vector<int>& ps, uint32_t epoch, float coef, hipStream_t st,
                bool with_gate = false);
  // the same push as tail blocks of another launch (tail.h kind 1, one block per arrival
  // slice); false when the set does not fit a tail (more than kTailPieces shards)
  bool push_tail(const std::vector<int>& ps, uint32_t epoch, UpdTail& out) const;
  // the DONE counters and the arrival board: a POSIX shm segment (created by one rank,
  // attached by the others) registered with HIP, so every GPU stores into them and every host
  // polls them directly
  void attach_done(const std::string& name, bool create);
  // PS host: has `worker` posted round `epoch` of PS `ps`?  next_slice: the caller's scan
  // position (the first slice not yet seen posted; 0 for a new round)
  bool posted(int ps, int worker, uint32_t epoch, int& next_slice) const;
  // worker host: wait until every PS has stored round `epoch`'s parameters here (false on
  // timeout or a recorded kernel error)
  bool wait_done(uint32_t epoch, double timeout_s);
  // the same wait as one wave on stream `st` (the GPU-side pull gate, async_runner.hip)
  void gate(uint32_t epoch, hipStream_t st);
  // PS host: apply worker `worker`'s round-`epoch` push to PS `ps` (private copy ps_params,
  // optimizer state in u) and store the new shard into that worker's parameter buffer
  void apply(int ps, int worker, uint32_t epoch, const XgmiUpdate& u, float* ps_params,
             hipStream_t st);
  int error() const;
  int num_ps() const { return nps_; }
  // PS p's range of the parameter / gradient buffers and its host
  void shard(int p, int64_t& lo, int64_t& n, int& host) const;
  float* params() const { return params_; }
  const float* grads() const { return grads_; }

 private:
  void upload_table();           // table_ -> table_dev_ (set-up only: open, attach_done)
  float* params_;
  const float* grads_;
  int world_, rank_, nps_ = 0;
  AsyncTable table_;
  AsyncTable* table_dev_ = nullptr;  // the kernels' copy
  float* inbox_ = nullptr;
  int64_t inbox_elems_ = 0;
  uint32_t* flags_ = nullptr;
  int* err_ = nullptr;
  double timeout_s_ = 60.0;
  void* opened_[kXgmiMaxPeers][3] = {};
  bool opened_ok_ = false;
  uint32_t* done_host_ = nullptr;
  uint32_t* posted_host_ = nullptr;
  size_t done_bytes_ = 0;
  std::string done_name_;
  bool done_owner_ = false;
};

struct AsyncPsState {            // one hosted PS as the service thread sees it
  int ps;
  float* params;                 // the PS's private parameter copy
  float* m;
  float* v;
  int64_t t;                     // its step counter (advanced once per arrival)
};

class AsyncService {
 public:
  AsyncService(AsyncPeer* peer, int world, int device, const std::vector<AsyncPsState>& ps,
               int opt, float lr, float b1, float b2, float eps, float mu, float scale,
               uint32_t epoch0, bool provenance);
  ~AsyncService();
  void start(int64_t expected);  // serve `expected` pushes on a native thread
  void join();                   // rethrows the thread's error, if any
  // checkpoint hook: no apply is issued between pause() and resume(), and every issued one has
  // completed when pause() returns (the PS state is one consistent step); same caller thread
  void pause();
  void resume();
  int64_t t(int ps) const;
  int64_t served() const;
  // (worker, ps, worker round, PS step) per apply, in service order
  const std::vector<std::array<int64_t, 4>>& provenance() const { return prov_; }
  // the thread scans the board and launches each apply
  const char* mode() const { return "host"; }

 private:
  void run();
  void serve(AsyncPsState& st, int worker);
  AsyncPeer* peer_;
  int world_, device_;
  std::vector<AsyncPsState> ps_;
  int opt_;
  float lr_, b1_, b2_, eps_, mu_, scale_;
  bool keep_prov_;
  std::vector<uint32_t> epoch_;
  std::vector<std::array<int64_t, 4>> prov_;
  std::atomic<int64_t> served_{0};
  int64_t expected_ = 0;
  hipStream_t stream_ = nullptr;
  std::thread th_;
  std::string error_;
  mutable std::mutex pause_mu_;  // held by the service thread while it issues an apply
};

// Native asynchronous worker step over the xGMI data plane (async_runner.hip): wait for the
// previous round's parameters (host), forward, backward with each PS's gradient push launched
// after the segment that completes its range (the push posts itself on the arrival board).
class AsyncRunner {
 public:
  static constexpr int kSegments = 4;
  // seg_of_ps[p]: backward segment after which PS p's range is complete; epoch0: the round
  // already completed (the set-up self-test)
  AsyncRunner(Engine* eng, AsyncPeer* peer, int world, int rank, int device,
              const std::vector<int>& seg_of_ps, uint32_t epoch0);
  void step(const float* x, const int64_t* labels, int B, uint32_t seed, hipStream_t st,
            double timeout_s);
  // the last round's parameters are back
  void finish(double timeout_s);
  uint32_t epoch() const { return epoch_; }
  // pushes as tail blocks of the next segment's launch (default) or push kernels of their own
  void set_use_tail(bool on) { use_tail_ = on; }
  // the pull as a GPU-side gate before the next forward (default) or a host wait
  void set_gate(bool on) { gate_ = on; }
  // In-line applies (one worker, every PS hosted by it, Adam): each push is applied on the
  // compute stream as Adam tail blocks of the next segment's launch — the last segment's inside
  // conv1's weight-gradient launch — with the PS's m / v and its own step counter t, in push
  // order.  A sole pusher's push order IS the arrival order, so no board claim, apply kernel,
  // DONE word or gate is needed; the PS's private parameter copy is not touched per step (it
  // equals the worker's buffer: inline_sync_ps() writes it back for checkpoints).  `ps` gives
  // every PS's m, v and t (its params pointer: the private copy).
  void set_inline(const std::vector<AsyncPsState>& ps, float lr, float b1, float b2, float eps,
                  float scale, bool provenance);
  bool inline_on() const { return inline_; }
  int64_t inline_t(int ps) const;
  void inline_sync_ps(hipStream_t st);  // worker buffer -> every PS's private copy
  // (worker, ps, round, t) per in-line apply, when provenance was asked for
  const std::vector<std::array<int64_t, 4>>& inline_provenance() const { return prov_; }

 private:
  void wait_round(double timeout_s);
  void check_round(uint32_t e, double timeout_s);
  void step_inline(const float* x, const int64_t* labels, int B, hipStream_t st);
  UpdTail inline_tail(int seg, int f4_per_block);
  bool inline_ = false, keep_prov_ = false;
  std::vector<AsyncPsState> ips_;  // by PS id
  float lr_ = 0.f, b1_ = 0.f, b2_ = 0.f, eps_ = 0.f, scale_ = 1.f;
  std::vector<float> lr_t_;        // this round's TF1 Adam step size per PS
  std::vector<std::array<int64_t, 4>> prov_;
  hipStream_t last_st_ = nullptr;
  bool stepped_ = false;
  bool use_tail_ = true;
  bool gate_ = true;
  uint32_t gated_ = 0;  // the round the last step's gate waits for (0: none)
  hipStream_t safe_stream_ = nullptr;  // the compute stream whose priority was checked
  bool safe_checked_ = false, safe_ = false;
  Engine* eng_;
  AsyncPeer* peer_;
  int world_, rank_, device_;
  uint32_t epoch_, epoch0_;
  std::vector<int> seg_ps_[kSegments];
};

// Asynchronous PS over point-to-point RCCL in exclusive sessions (rccl_async.hip): one
// communicator, one comm stream and one comm thread per process; a (worker, PS) round trip
// runs only while its initiator holds both processes' session locks.
class RcclAsync {
 public:
  RcclAsync(float* params, float* grads, int world, int rank, int device,
            const std::vector<std::pair<int64_t, int64_t>>& ps_ranges,
            const std::vector<int>& hosts, const std::vector<AsyncPsState>& hosted, int opt,
            double lr, double b1, double b2, float eps, float mu, bool self_sessions);
  ~RcclAsync();
  void init_comm(const char id[128]);               // collective over all ranks
  void attach_shm(const std::string& job, bool create);  // session locks (rank 0 creates)
  void open_boxes(bool own);                        // own: create mine; else attach the others
  void start(int64_t expected_served, bool provenance);
  void push_pull(hipStream_t compute);              // this worker's round (blocks the caller)
  void join();
  void pause();
  void resume();
  int64_t t(int ps) const;
  // a hosted PS's step counter before start() (resume: the checkpoint's t, restored after the
  // object was built — Adam's bias correction continues instead of restarting at t = 1)
  void set_t(int ps, int64_t t);
  int64_t served() const { return served_.load(); }
  // (worker, ps, that worker's round at this PS, PS step) per applied push
  const std::vector<std::array<int64_t, 4>>& provenance() const { return prov_; }

 private:
  void loop();
  bool push_one(int p);
  void serve(int worker, int p);
  void apply(int p, int worker, const float* g);
  AsyncPsState* state_of(int p);
  float* w_;
  float* g_;
  int world_, rank_, device_;
  std::vector<std::pair<int64_t, int64_t>> ranges_;
  std::vector<int> hosts_;
  std::vector<AsyncPsState> ps_;
  int opt_;
  float lr_, b1_, b2_, eps_, mu_;
  double lrd_, b1d_, b2d_;
  bool self_;
  void* comm_ = nullptr;
  hipStream_t cs_ = nullptr;
  hipEvent_t ev_ = nullptr;
  float* gbuf_ = nullptr;
  SessionLocks locks_;  // runtime/session.h (CPU-stress-tested protocol)
  std::string box_name_;
  std::unique_ptr<ShmMailbox> mine_;
  std::unique_ptr<ShmMailbox> boxes_[kXgmiMaxPeers];
  std::vector<int64_t> count_;
  bool keep_prov_ = false;
  std::vector<std::array<int64_t, 4>> prov_;
  std::atomic<int64_t> served_{0};
  int64_t expected_ = 0;
  std::thread th_;
  std::mutex qmu_;               // round queue / stop / error
  std::mutex pause_mu_;
  std::condition_variable cv_;
  std::vector<int> pending_;
  bool waited_ = false;
  bool stop_ = false;
  std::string error_;
};

class SyncRunner {
 public:
  static constexpr int kSegments = 4;
  SyncRunner(Engine* eng, float* params, float* grads, int world, int rank);
  ~SyncRunner();
  static void unique_id(char out[128]);
  // "" when torch's librccl and every entry point the runner uses resolve, else the reason
  static std::string probe();
  // collective over all ranks; W = 1 only with `force` (1-rank communicator: the collective
  // units then run as RCCL copies — the on-device test of the exchange path on one GPU)
  void init_comm(const char id[128], bool force = false);
  bool has_comm() const { return comm_ != nullptr; }
  void set_units(const std::vector<RunnerUnit>& units);
  void set_optimizer(int kind, float lr, float b1, float b2, float eps, float mu);
  void set_scale(float grad_scale, float coef) { grad_scale_ = grad_scale; coef_ = coef; }
  // one synchronous training step on stream `st`; lr_t indexed by RunnerUnit::ps
  void step(const float* x, const int64_t* labels, int B, uint32_t seed, const float* lr_t,
            hipStream_t st);
  bool selftest(std::string* why);
  void set_local_on_main(bool on) { local_on_main_ = on; }
  // collective units of the LAST backward segment on the compute stream (no event hop on the
  // step's critical path; RCCL still orders them after the comm stream's earlier units)
  void set_last_on_main(bool on) { last_on_main_ = on; }
  std::string async_error();  // "" while the communicator is healthy (RCCL and xGMI)
  // XGMI units exchange through this (owned by the caller; outlives the runner's use)
  PeerExchange* peer() const { return peer_; }
  void set_peer(PeerExchange* p) {
    peer_ = p;
    if (p) p->set_gate_error(ready_err_dev());  // (device memory: read by every bucket wave)
  }
  int* ready_err_dev() const { return ready_ ? reinterpret_cast<int*>(ready_ + kSegments) : nullptr; }
  // one full exchange of every bucket with w := sum over ranks of g (no optimizer) at the
  // next epoch; the caller fills g, checks w
  void peer_selftest_step(hipStream_t st);
  void abort();               // ncclCommAbort: unblocks this rank's pending collectives
  // orderly ncclCommDestroy (call on every rank at the same point), then release()
  void close();
  hipStream_t comm_stream() const { return cs_; }

 private:
  void issue(const RunnerUnit& u, const float* lr_t, hipStream_t st);
  // all REDUCE units of one segment: one RCCL group of reduces, the hosted updates, one
  // group of broadcasts (instead of two groups per unit)
  void issue_reduce_group(const std::vector<const RunnerUnit*>& us, const float* lr_t,
                          hipStream_t st);
  void update(float* w, const float* g, float* m, float* v, int64_t n, float lr_t,
              hipStream_t st);
  void issue_xgmi(const RunnerUnit& u, const float* lr_t, bool final_wait, hipStream_t st,
                  bool gated = false);
  int last_xgmi_ = -1;     // index of the step's last XGMI unit (carries the final wait)
  void release();          // destroy the comm stream, events and flags (idempotent)
  bool closed_ = false;
  Engine* eng_;
  float* w_;
  float* g_;
  int world_, rank_;
  void* comm_ = nullptr;  // ncclComm_t
  PeerExchange* peer_ = nullptr;
  uint32_t epoch_ = 0;     // xGMI flag epoch: one per step, identical on every rank
  hipStream_t cs_ = nullptr;
  hipEvent_t seg_ev_[kSegments] = {};
  hipEvent_t seg_ev_dev_[kSegments] = {};  // device-scope release (xGMI-only segments)
  bool seg_xgmi_only_[kSegments] = {};
  // segments with exchange units on the comm stream (xGMI or RCCL) hand their gradients over
  // by a READY flag (tail.h kind 2) instead of an event: 0 never, 1 every segment but the
  // first, 2 every segment (default: forced xGMI rehearsal 0.3156 / 0.3164 / 0.3058 ms/step,
  // scripts/ready_ab.py)
  int ready_flags_ = 2;
  bool seg_offstream_[kSegments] = {};     // the segment has units on the comm stream
  int seg_launches_[kSegments] = {};       // kernel launches of the segment in the last step
  // seg events recorded by the segment's own kernel packets (DDL_EXT_EVENT, default on)
  bool ext_event_ = true;
  hipEvent_t done_ev_ = nullptr;
  bool gate_safe(hipStream_t st);  // `st` is not a high-priority stream (runner.hip)
  hipStream_t gate_checked_stream_ = nullptr;
  bool gate_checked_ = false, gate_checked_ok_ = false;
  uint32_t* ready_ = nullptr;     // READY[segment] (uncached device memory, tail.h kind 2)
  int* ready_err_ = nullptr;      // a READY gate timed out (host memory)
  double gate_timeout_s_ = 20.0;  // DDL_XGMI_TIMEOUT_S
  uint32_t ready_epoch_ = 0;      // one per step
  std::vector<RunnerUnit> units_;
  int opt_ = 0;
  float lr_ = 1e-4f, b1_ = 0.9f, b2_ = 0.999f, eps_ = 1e-8f, mu_ = 0.9f;
  float grad_scale_ = 1.f, coef_ = 1.f;
  bool local_on_main_ = true;
  bool last_on_main_ = true;
  struct Piece {
    RunnerRange r;
    int ps;
    float* m;
    float* v;
  };
  bool all_local_ = false;
  std::vector<Piece> merged_;  // coalesced LOCAL update ranges (all_local_)
  // all_local_: the same ranges coalesced per backward segment; segment s's update rides as
  // an optimizer tail (tail.h) in segment s+1's dual launch when every piece is 16-B vector
  // shaped (tail_ok_), the last segment's is launched after the backward
  std::vector<Piece> seg_pieces_[kSegments];
  bool tail_ok_ = false;
  bool use_tail_ = true;
  bool final_in_reduce_ = [] {
    const char* e = getenv("DDL_FINAL_IN_REDUCE");
    return !e || e[0] != '0';
  }();
  void set_tail(int seg, const float* lr_t, int f4_per_block = 0);

 public:
  void set_ready_flags(int mode) { ready_flags_ = mode; }
  void set_use_tail(bool on) { use_tail_ = on; }
  // the last segment's update inside conv1's weight-gradient launch (tail path only): with the
  // direct conv1 kernel conv2's Adam runs in its weight-gradient reduce epilogue and conv1's in
  // the final reduce level (engine_impl.h final_split_conv12): 0.2988 -> 0.2973 ms/step; with
  // the GEMM conv1 path as tail blocks of the wide reduce (measured neutral).
  // DDL_FINAL_IN_REDUCE=0: the stand-alone Adam launch
  void set_final_in_reduce(bool on) { final_in_reduce_ = on; }
  // tail placement (1: before the GEMM blocks) and float4 per tail block (tuning)
  void set_tail_cfg(int first, int f4_per_block) {
    tail_first_ = first;
    tail_f4_ = std::max(1, f4_per_block / kTailF4PerBlock) * kTailF4PerBlock;
  }

 private:
  // measured (scripts/tail_probe.py, one MI355X): after the GEMM blocks, 512 float4 per
  // block: 373 us/step vs 381 without the tail; before the GEMM blocks 375-378
  int tail_first_ = 0;
  int tail_f4_ = kTailF4Default;
};

}  // namespace ddl
