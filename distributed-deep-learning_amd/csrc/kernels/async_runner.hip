// Native asynchronous worker step (SURVEY.md §3.2 worker loop + §3.4 async PS, over the xGMI
// peer-memory data plane of xgmi_async.hip).
//
// Reference worker round (mnist_async_sharding/worker.py:80-95): sess.run(grads), then one
// MPI Send per tensor to its PS, then a blocking Recv per tensor of the parameters that PS
// sends back.  Here one C++ call per step:
//
//   1. the PREVIOUS round's parameters must be in this worker's buffer before the forward that
//      reads them — the reference's blocking pull.  Default: a GPU-side gate, one wave enqueued
//      on the compute stream after the round's last push, polling the round's DONE words; the
//      forward behind it starts as soon as the last apply lands, with no host in between (the
//      host wait + launch cost ~22 us of idle GPU per step, profiles/r4_async_host_latency.txt).
//      The host only checks, bounded, the round before (failure detection).  set_gate(false):
//      the host waits for the round itself before enqueuing the forward.
//      Why the gate cannot deadlock: it blocks the compute stream's hardware queue until every
//      PS has applied this worker's round.  Those applies run on other processes' queues or on
//      this process's service stream, created with HIGH priority — HIP pools hardware queues
//      per priority, so that stream never shares the gated queue as long as the compute stream
//      is not high priority itself (checked once per stream; a high-priority compute stream gets
//      the host wait instead) — and each apply waits for nothing on the GPU (the service issues
//      it after seeing the push posted).  No wait in the chain sits behind the gate, and the
//      gate is bounded (error word, no hang);
//   2. forward, then the four backward segments; segment s's PS shards are pushed by tail blocks
//      of segment s+1's first launch (tail.h kind 1; the last segment's by a push kernel), each
//      block posting its slice on the arrival board in host memory once its payload is
//      acknowledged: no push kernels on the compute stream, no completion events (whose
//      system-scope release cost ~4.6 us of idle compute stream per push), no host thread
//      between a push and its PS host's service.
//
// In-line applies (set_inline; one worker hosting every PS, Adam — the W = 1 default): the
// push / apply / gate chain above costs ~13 us per step on the critical path after the last
// segment (push launch, host scan, apply launch, DONE, gate) against ~3.5 us for an in-line
// Adam (docs/DESIGN.md round 5).  A sole pusher's pushes reach each PS in the order it issues
// them, so applying segment s's shards as Adam tail blocks of segment s+1's first launch (the
// last segment's inside conv1's weight-gradient launch, engine_impl.h dual_then_b) IS the
// arrival-order apply: the same per-PS Adam step (its own counter t, one step per push), the
// same staleness (none, with one worker), and stream order instead of DONE words.
//
// The PS side: each host's AsyncService scans the board in host memory and issues one apply
// per completed push (Adam on the PS's private copy, the new shard stored into the worker's
// buffer, DONE words in the worker's device flags and in shared host memory).  Staleness stays
// one round per worker.
#include <stdlib.h>

#include <cmath>
#include <stdexcept>
#include <string>

#include "api.h"
#include "common.h"
#include "trace.h"

namespace ddl {

AsyncRunner::AsyncRunner(Engine* eng, AsyncPeer* peer, int world, int rank, int device,
                         const std::vector<int>& seg_of_ps, uint32_t epoch0)
    : eng_(eng), peer_(peer), world_(world), rank_(rank), device_(device), epoch_(epoch0),
      epoch0_(epoch0) {
  const int P = peer->num_ps();
  if ((int)seg_of_ps.size() != P) throw std::invalid_argument("async runner: one segment per PS");
  // (A/B switches: DDL_ASYNC_GATE=0 waits for the round on the host, DDL_ASYNC_TAIL=0 pushes
  // with kernels of their own instead of tail blocks)
  if (const char* g = getenv("DDL_ASYNC_GATE")) gate_ = g[0] != '0';
  if (const char* t = getenv("DDL_ASYNC_TAIL")) use_tail_ = t[0] != '0';
  for (int p = 0; p < P; ++p) {
    if (seg_of_ps[p] < 0 || seg_of_ps[p] >= kSegments)
      throw std::invalid_argument("async runner: PS segment out of range");
    seg_ps_[seg_of_ps[p]].push_back(p);
  }
}

void AsyncRunner::wait_round(double timeout_s) {
  if (epoch_ == epoch0_) return;  // no round in flight yet
  TraceRange r("ddl.async.worker.pull_wait");
  if (!peer_->wait_done(epoch_, timeout_s))
    throw std::runtime_error("async runner: round " + std::to_string(epoch_) +
                             " did not come back (kernel error code " +
                             std::to_string(peer_->error()) + ")");
}

void AsyncRunner::check_round(uint32_t e, double timeout_s) {
  TraceRange r("ddl.async.worker.pull_check");
  if (!peer_->wait_done(e, timeout_s))
    throw std::runtime_error("async runner: round " + std::to_string(e) +
                             " did not come back (kernel error code " +
                             std::to_string(peer_->error()) + ")");
}

void AsyncRunner::set_inline(const std::vector<AsyncPsState>& ps, float lr, float b1, float b2,
                             float eps, float scale, bool provenance) {
  const int P = peer_->num_ps();
  if (world_ != 1) throw std::invalid_argument("async runner: in-line applies need one worker");
  if ((int)ps.size() != P) throw std::invalid_argument("async runner: in-line applies need every PS");
  auto a16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  std::vector<AsyncPsState> by(P, AsyncPsState{-1, nullptr, nullptr, nullptr, 0});
  for (const auto& s : ps) {
    if (s.ps < 0 || s.ps >= P || by[s.ps].ps >= 0 || !s.params || !s.m || !s.v)
      throw std::invalid_argument("async runner: in-line PS state (one per PS, Adam m and v)");
    int64_t lo = 0, n = 0;
    int host = -1;
    peer_->shard(s.ps, lo, n, host);
    if (host != rank_) throw std::invalid_argument("async runner: in-line PS hosted elsewhere");
    if (n % 4 || !a16(peer_->params() + lo) || !a16(peer_->grads() + lo) || !a16(s.m) ||
        !a16(s.v))
      throw std::invalid_argument("async runner: in-line PS buffers must be 16-B aligned");
    by[s.ps] = s;
  }
  ips_ = by;
  lr_ = lr;
  b1_ = b1;
  b2_ = b2;
  eps_ = eps;
  scale_ = scale;
  keep_prov_ = provenance;
  prov_.clear();
  lr_t_.assign(P, 0.f);
  inline_ = true;
}

int64_t AsyncRunner::inline_t(int ps) const {
  if (!inline_ || ps < 0 || ps >= (int)ips_.size())
    throw std::invalid_argument("async runner: no in-line PS " + std::to_string(ps));
  return ips_[ps].t;
}

void AsyncRunner::inline_sync_ps(hipStream_t st) {
  if (!inline_) return;
  for (size_t p = 0; p < ips_.size(); ++p) {
    int64_t lo = 0, n = 0;
    int host = -1;
    peer_->shard((int)p, lo, n, host);
    const hipError_t e = hipMemcpyAsync(ips_[p].params, peer_->params() + lo,
                                        (size_t)n * sizeof(float), hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess)
      throw std::runtime_error(std::string("async runner: PS copy: ") + hipGetErrorString(e));
  }
}

// Segment `seg`'s PS shards as one Adam tail (tail.h kind 0); empty if they do not fit one
UpdTail AsyncRunner::inline_tail(int seg, int f4_per_block) {
  UpdTail t;
  if ((int)seg_ps_[seg].size() > kTailPieces) return t;
  t.first = 0;
  t.f4_per_block = f4_per_block;
  t.c1 = 1.f - b1_;
  t.c2 = 1.f - b2_;
  t.eps = eps_;
  t.scale = scale_;
  int blk = 0;
  for (int p : seg_ps_[seg]) {
    int64_t lo = 0, n = 0;
    int host = -1;
    peer_->shard(p, lo, n, host);
    UpdPiece& q = t.p[t.npieces++];
    q.w = peer_->params() + lo;
    q.g = peer_->grads() + lo;
    q.m = ips_[p].m;
    q.v = ips_[p].v;
    q.n = n;
    q.lr_t = lr_t_[p];
    q.blk0 = blk;
    blk += (int)((n / 4 + f4_per_block - 1) / f4_per_block);
  }
  t.nblocks = (blk + 7) & ~7;
  return t;
}

void AsyncRunner::step_inline(const float* x, const int64_t* labels, int B, hipStream_t st) {
  ++epoch_;
  // one Adam step of each PS's own counter per push (TF1: lr_t = lr sqrt(1 - b2^t) / (1 - b1^t))
  for (size_t p = 0; p < ips_.size(); ++p) {
    const int64_t t = ++ips_[p].t;
    lr_t_[p] = (float)((double)lr_ * std::sqrt(1.0 - std::pow((double)b2_, (double)t)) /
                       (1.0 - std::pow((double)b1_, (double)t)));
    if (keep_prov_) prov_.push_back({(int64_t)rank_, (int64_t)p, (int64_t)epoch_, t});
  }
  {
    TraceRange r("ddl.fwd");
    eng_->forward(x, B, nullptr, true, st, /*defer_fc2=*/true);
  }
  auto apply_now = [&](int seg) {  // a segment whose shards do not fit one tail
    for (int p : seg_ps_[seg]) {
      int64_t lo = 0, n = 0;
      int host = -1;
      peer_->shard(p, lo, n, host);
      launch_adam_c(peer_->params() + lo, peer_->grads() + lo, ips_[p].m, ips_[p].v, n,
                    lr_t_[p], 1.f - b1_, 1.f - b2_, eps_, scale_, st);
    }
  };
  for (int s = 0; s < kSegments; ++s) {
    TraceRange r("ddl.bwd");
    if (s > 0 && !seg_ps_[s - 1].empty()) {
      UpdTail t = inline_tail(s - 1, kTailF4Default);
      if (t.npieces) eng_->tail = t;
      else apply_now(s - 1);
    }
    if (s == kSegments - 1 && !seg_ps_[s].empty()) {
      // one pass per tail block: on the step's critical path the update wants width
      UpdTail t = inline_tail(s, kTailF4PerBlock);
      if (t.npieces) eng_->final_upd = t;
    }
    eng_->backward_segment(s, x, labels, B, nullptr, st);
    eng_->flush_tail(st);
  }
  if (!seg_ps_[kSegments - 1].empty() &&
      (eng_->final_upd.npieces > 0 || (int)seg_ps_[kSegments - 1].size() > kTailPieces)) {
    eng_->final_upd = UpdTail();  // not taken by conv1's launch: a launch of its own
    apply_now(kSegments - 1);
  }
}

void AsyncRunner::step(const float* x, const int64_t* labels, int B, uint32_t seed,
                       hipStream_t st, double timeout_s) {
  TraceRange step_range("ddl.async.step");
  if (inline_) {
    eng_->seed_value = seed;
    last_st_ = st;
    stepped_ = true;
    step_inline(x, labels, B, st);
    return;
  }
  // (1) the previous round's parameters are in place before the forward: the gate enqueued at
  // the end of the previous step (the host checks the round before that: it ran before the
  // previous forward, so in steady state this returns at once), or a host wait
  if (gated_ != 0) {
    if (gated_ - 1 != epoch0_) check_round(gated_ - 1, timeout_s);
  } else {
    wait_round(timeout_s);
  }
  ++epoch_;
  eng_->seed_value = seed;
  {
    TraceRange r("ddl.fwd");
    eng_->forward(x, B, nullptr, true, st, /*defer_fc2=*/true);  // backward_segment(0) follows
  }
  // the gate may only sit on a stream that is not high priority (queried once per stream: a
  // runtime call at the end of the step would sit in the window where this process's service
  // thread launches the round's last apply)
  if (!safe_checked_ || st != safe_stream_) {
    int lo = 0, hi = 0, pr = 0;  // (the null stream is a normal-priority stream)
    safe_ = hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess &&
            (st == nullptr || hipStreamGetPriority(st, &pr) == hipSuccess) && hi != lo &&
            pr != hi;
    safe_stream_ = st;
    safe_checked_ = true;
  }
  const bool gate = gate_ && safe_;
  int last = kSegments - 1;
  while (last > 0 && seg_ps_[last].empty()) --last;
  gated_ = 0;
  for (int s = 0; s < kSegments; ++s) {
    {
      TraceRange r("ddl.bwd");
      eng_->backward_segment(s, x, labels, B, nullptr, st);  // (takes a pending push tail)
    }
    if (seg_ps_[s].empty()) continue;
    // (2) this segment's shards to their hosts, posted on the board: as tail blocks of the
    // next segment's first launch (flush_tail launches them alone if it takes none), the last
    // segment's by a push kernel
    TraceRange r("ddl.async.worker.push");
    UpdTail t;
    if (use_tail_ && s + 1 < kSegments && peer_->push_tail(seg_ps_[s], epoch_, t)) {
      eng_->flush_tail(st);
      eng_->tail = t;
    } else {
      eng_->flush_tail(st);
      // the round's last push carries the pull gate as its launch's last block
      const bool with_gate = gate && s == last;
      peer_->push_set(seg_ps_[s], epoch_, 1.f, st, with_gate);
      if (with_gate) gated_ = epoch_;
    }
  }
  eng_->flush_tail(st);
  if (gate && gated_ == 0) {  // (the last push rode as tail blocks: a gate launch of its own)
    peer_->gate(epoch_, st);
    gated_ = epoch_;
  }
}

void AsyncRunner::finish(double timeout_s) {
  if (inline_) {  // the round's applies are on the compute stream
    if (stepped_) {
      const hipError_t e = hipStreamSynchronize(last_st_);
      if (e != hipSuccess)
        throw std::runtime_error(std::string("async runner: finish: ") + hipGetErrorString(e));
    }
    return;
  }
  wait_round(timeout_s);
}

}  // namespace ddl
