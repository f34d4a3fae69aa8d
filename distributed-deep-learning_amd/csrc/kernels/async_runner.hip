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
// The PS side: each host's AsyncService scans the board in host memory and issues one apply
// per completed push (Adam on the PS's private copy, the new shard stored into the worker's
// buffer, DONE words in the worker's device flags and in shared host memory).  Staleness stays
// one round per worker.
#include <stdlib.h>

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

void AsyncRunner::step(const float* x, const int64_t* labels, int B, uint32_t seed,
                       hipStream_t st, double timeout_s) {
  TraceRange step_range("ddl.async.step");
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

void AsyncRunner::finish(double timeout_s) { wait_round(timeout_s); }

}  // namespace ddl
