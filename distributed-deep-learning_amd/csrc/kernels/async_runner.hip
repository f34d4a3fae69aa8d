// Native asynchronous worker step (SURVEY.md §3.2 worker loop + §3.4 async PS, over the xGMI
// peer-memory data plane of xgmi_async.hip).
//
// Reference worker round (mnist_async_sharding/worker.py:80-95): sess.run(grads), then one
// MPI Send per tensor to its PS, then a blocking Recv per tensor of the parameters that PS
// sends back.  Here one C++ call per step:
//
//   1. wait (host, GIL released) until every PS has stored the PREVIOUS round's parameters
//      into this worker's buffer — the reference's blocking pull, moved to just before the
//      forward that reads them, so the Python loop never blocks between enqueues;
//   2. forward, then the four backward segments; after segment s, one push kernel stores the
//      gradient shards of every PS whose range is complete after s into their hosts' inboxes
//      (the fc shards leave while the conv backward still computes).  The push launch carries
//      its own completion event (hipExtLaunchKernelGGL stop event, common.h DDL_LAUNCH);
//   3. a poster thread waits for each push event and then posts the (worker, ps) tokens into
//      the PS hosts' arrival mailboxes (the MPI.ANY_SOURCE order) — no Python, no GIL.
//
// The PS side is unchanged: each host's AsyncService pops tokens in arrival order and issues
// one apply per token (Adam on the PS's private copy, the new shard stored into the worker's
// buffer, DONE in shared host memory).  As in the rest of the async protocol NO kernel waits
// for another kernel (xgmi_async.hip explains the hardware-queue deadlock that rules it out):
// a token is posted only after its push has completed, and the only wait for remote work is
// the host wait of step 1.  Staleness stays one round per worker.
#include <chrono>
#include <thread>
#include <stdexcept>
#include <string>

#include "api.h"
#include "common.h"
#include "runtime/mailbox.h"
#include "trace.h"

namespace ddl {

#define A_CHECK(x)                                                                          \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess)                                                                   \
      throw std::runtime_error(std::string("async runner: ") + #x + ": " + hipGetErrorString(e_)); \
  } while (0)

AsyncRunner::AsyncRunner(Engine* eng, AsyncPeer* peer, int world, int rank, int device,
                         const std::vector<int>& seg_of_ps, const std::vector<int>& hosts,
                         const std::vector<std::string>& boxes, uint32_t epoch0)
    : eng_(eng), peer_(peer), world_(world), rank_(rank), device_(device), epoch_(epoch0),
      epoch0_(epoch0) {
  const int P = peer->num_ps();
  if ((int)seg_of_ps.size() != P || (int)hosts.size() != P)
    throw std::invalid_argument("async runner: one segment and one host per PS");
  if ((int)boxes.size() != world) throw std::invalid_argument("async runner: one box per rank");
  for (int p = 0; p < P; ++p) {
    if (seg_of_ps[p] < 0 || seg_of_ps[p] >= kSegments)
      throw std::invalid_argument("async runner: PS segment out of range");
    if (hosts[p] < 0 || hosts[p] >= world || boxes[hosts[p]].empty())
      throw std::invalid_argument("async runner: PS host without a mailbox");
    seg_ps_[seg_of_ps[p]].push_back(p);
  }
  hosts_ = hosts;
  for (int r = 0; r < world; ++r)
    if (!boxes[r].empty()) boxes_[r] = std::make_unique<ShmMailbox>(boxes[r], 2, false);
  for (int s = 0; s < kSegments; ++s)
    A_CHECK(hipEventCreateWithFlags(&ev_[s], hipEventDisableTiming));
  posts_ = std::make_unique<PostQueue<Posting>>([this](const Posting& j) { wait_push(j); },
                                                [this](const Posting& j) { post_tokens(j); });
}

AsyncRunner::~AsyncRunner() {
  posts_.reset();  // joins the poster before the events go
  for (auto& e : ev_)
    if (e) (void)hipEventDestroy(e);
}

// Poster thread: the push kernel of a job has completed.  A query loop, not
// hipEventSynchronize: the token post is on the round trip of every async step, and a
// blocking event wait adds its wake-up latency to it.
void AsyncRunner::wait_push(const Posting& job) {
  thread_local int dev = -1;
  if (dev != device_) {
    A_CHECK(hipSetDevice(device_));
    dev = device_;
  }
  TraceRange r("ddl.async.worker.push_wait");
  for (int spins = 0;; ++spins) {
    const hipError_t e = hipEventQuery(job.ev);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) A_CHECK(e);
    if (spins > 64) std::this_thread::yield();
  }
}

void AsyncRunner::post_tokens(const Posting& job) {
  for (int p : job.ps) {
    const int64_t token = ((int64_t)rank_ << 20) | p;  // parallel/mailbox.py encode()
    if (!boxes_[hosts_[p]]->push(token, 600.0))
      throw std::runtime_error("arrival mailbox of rank " + std::to_string(hosts_[p]) +
                               " full for 600 s");
  }
}

void AsyncRunner::wait_round(double timeout_s) {
  if (epoch_ == epoch0_) return;  // no round in flight yet
  TraceRange r("ddl.async.worker.pull_wait");
  if (!peer_->wait_done(epoch_, timeout_s)) {
    const std::string pe = posts_->error();
    throw std::runtime_error("async runner: round " + std::to_string(epoch_) +
                             " did not come back (kernel error code " +
                             std::to_string(peer_->error()) + ")" +
                             (pe.empty() ? "" : "; poster: " + pe));
  }
}

void AsyncRunner::step(const float* x, const int64_t* labels, int B, uint32_t seed,
                       hipStream_t st, double timeout_s) {
  TraceRange step_range("ddl.async.step");
  if (const std::string pe = posts_->error(); !pe.empty())
    throw std::runtime_error("async runner poster: " + pe);
  // (1) the previous round's parameters are in place (this also means every token of it was
  // posted, so the segment events are free to record again)
  wait_round(timeout_s);
  ++epoch_;
  eng_->seed_value = seed;
  {
    TraceRange r("ddl.fwd");
    eng_->forward(x, B, nullptr, true, st);
  }
  for (int s = 0; s < kSegments; ++s) {
    {
      TraceRange r("ddl.bwd");
      eng_->backward_segment(s, x, labels, B, nullptr, st);
    }
    if (seg_ps_[s].empty()) continue;
    // (2) this segment's shards to their hosts; the push kernel records ev_[s] itself
    {
      TraceRange r("ddl.async.worker.push");
      StopEventScope bind(ev_[s]);
      peer_->push_set(seg_ps_[s], epoch_, 1.f, st);
    }
    posts_->push({ev_[s], seg_ps_[s]});
  }
  eng_->flush_tail(st);  // (no tails are set on this path; keeps the engine state clean)
}

void AsyncRunner::finish(double timeout_s) {
  wait_round(timeout_s);
  posts_->finish();
}

}  // namespace ddl
