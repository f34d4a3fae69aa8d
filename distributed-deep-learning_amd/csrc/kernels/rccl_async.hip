// Asynchronous parameter server over point-to-point RCCL, issued natively (SURVEY.md §5.8
// async row).
//
// Reference (mnist_async_sharding/worker.py:30-37,88-94; parameter_server.py:94-111): a worker
// Sends its gradient shard to each PS and blocks in Recv for the parameters; the PS Recvs from
// ANY_SOURCE, applies Adam and Sends the parameters back to that worker.
//
// RCCL has no wildcard receive, and an RCCL p2p kernel BLOCKS its hardware queue until the
// peer posts the matching op.  HIP multiplexes a process's streams onto GPU_MAX_HW_QUEUES (4)
// hardware queues, so p2p kernels of several (worker, PS) conversations issued concurrently —
// the round-2 Python path: W(W-1) pair groups, driven from a worker thread and a service thread
// at once — can each end up queued behind another conversation's blocked kernel, in a cycle
// across processes.  This design makes every p2p op part of an EXCLUSIVE SESSION:
//
//   * one RCCL communicator and ONE comm stream per process, and ONE native comm thread that
//     issues every RCCL op of the process (no two threads ever interleave ops on it);
//   * a session = one (worker a, PS p on host h) round trip: a: group{send(g_p, h),
//     recv(w_p, h)};  h: recv(g, a) -> Adam on its private copy of p -> send(w_p, a).  Before
//     it starts, the initiator a holds BOTH per-process session locks L_a and L_h (words in a
//     POSIX shm segment, all-or-nothing try-lock, so no hold-and-wait and no lock cycle), then
//     posts (a, p) to h's session mailbox; h's comm thread serves its mailbox whenever it is not
//     itself in a session (it cannot be: L_h is held for this one);
//   * each side synchronises its comm stream at the end of its part, and a releases the locks
//     only after its recv completed (h's send is then past its last transfer).
// So at any time a process's comm stream holds only the ops of its single current session, and
// the partner's comm stream only the matching ops: every p2p kernel's peer is either running or
// queued behind compute kernels, which never wait for anything — whatever the stream-to-hardware
// -queue mapping, no cycle of blocked kernels exists.  The price is serialisation (one session
// per process at a time, a host round trip each): this is the RCCL fallback next to the xGMI
// async exchange (xgmi_async.hip), which needs no p2p kernels at all.
//
// Semantics are the reference's with its race removed: one Adam step per received push, the
// PS's own step counter, whole-shard updates (no per-tag mixing), at most
// one round in flight per worker (staleness bound).  A hosted PS's own worker is served in the
// comm thread directly (no session).  `self_sessions` (1-rank rehearsal) runs that local
// exchange as send/recv to itself too, so the p2p path runs on one GPU, bit-equal to local.
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <chrono>
#include <cmath>
#include <stdexcept>
#include <string>
#include <algorithm>
#include <thread>

#include "api.h"
#include "rccl_api.h"
#include "runtime/mailbox.h"
#include "trace.h"

namespace ddl {

static ncclComm_t comm_of(void* c) { return reinterpret_cast<ncclComm_t>(c); }

RcclAsync::RcclAsync(float* params, float* grads, int world, int rank, int device,
                     const std::vector<std::pair<int64_t, int64_t>>& ps_ranges,
                     const std::vector<int>& hosts, const std::vector<AsyncPsState>& hosted,
                     int opt, double lr, double b1, double b2, float eps, float mu,
                     bool self_sessions)
    : w_(params), g_(grads), world_(world), rank_(rank), device_(device), ranges_(ps_ranges),
      hosts_(hosts), ps_(hosted), opt_(opt), lr_((float)lr), b1_((float)b1), b2_((float)b2),
      eps_(eps), mu_(mu), lrd_(lr), b1d_(b1), b2d_(b2), self_(self_sessions) {
  if (world < 1 || world > kXgmiMaxPeers) throw std::invalid_argument("rccl async: world");
  if (ranges_.size() != hosts_.size() || ranges_.empty())
    throw std::invalid_argument("rccl async: one host per PS range");
  for (const auto& s : ps_) {
    if (s.ps < 0 || s.ps >= (int)ranges_.size() || hosts_[s.ps] != rank_)
      throw std::invalid_argument("rccl async: hosted PS state of a PS this rank does not host");
    if (!s.params || !s.m || (opt == 0 && !s.v)) throw std::invalid_argument("rccl async: PS state");
  }
  HIP_CHECK(hipSetDevice(device_));
  HIP_CHECK(hipStreamCreateWithFlags(&cs_, hipStreamNonBlocking));
  HIP_CHECK(hipEventCreateWithFlags(&ev_, hipEventDisableTiming));
  int64_t mx = 0;
  for (const auto& s : ps_) mx = std::max(mx, ranges_[s.ps].second - ranges_[s.ps].first);
  if (mx > 0) HIP_CHECK(hipMalloc(&gbuf_, mx * sizeof(float)));
  count_.assign((size_t)world * ranges_.size(), 0);
}

RcclAsync::~RcclAsync() {
  {
    std::lock_guard<std::mutex> g(qmu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (th_.joinable()) th_.join();
  if (comm_) (void)rccl().CommDestroy(comm_of(comm_));
  if (gbuf_) (void)hipFree(gbuf_);
  if (ev_) (void)hipEventDestroy(ev_);
  if (cs_) (void)hipStreamDestroy(cs_);
}

void RcclAsync::init_comm(const char id_bytes[128]) {
  ncclUniqueId id;
  memcpy(&id, id_bytes, 128);
  ncclComm_t c;
  HIP_CHECK(hipSetDevice(device_));
  RCCL_CHECK(rccl().CommInitRank(&c, world_, id, rank_));
  comm_ = c;
}

void RcclAsync::attach_shm(const std::string& job, bool create) {
  locks_.attach("/" + job + "_rlock", kXgmiMaxPeers, create);
  // session mailboxes: every rank owns one (created by its owner before the job's barrier)
  box_name_ = "/" + job + "_rsess_";
}

void RcclAsync::open_boxes(bool own) {
  if (own) mine_ = std::make_unique<ShmMailbox>(box_name_ + std::to_string(rank_), 4096, true);
  else
    for (int r = 0; r < world_; ++r)
      if (r != rank_) boxes_[r] = std::make_unique<ShmMailbox>(box_name_ + std::to_string(r), 2, false);
}

AsyncPsState* RcclAsync::state_of(int p) {
  for (auto& s : ps_)
    if (s.ps == p) return &s;
  throw std::runtime_error("rccl async: PS " + std::to_string(p) + " not hosted here");
}

// One Adam (or momentum) step of hosted PS p from gradient g, on the comm stream.
void RcclAsync::apply(int p, int worker, const float* g) {
  AsyncPsState* st = state_of(p);
  const int64_t n = ranges_[p].second - ranges_[p].first;
  const int64_t t = __atomic_add_fetch(&st->t, 1, __ATOMIC_ACQ_REL);
  if (opt_ == 0) {
    // TF1 Adam's lr_t in double, as ops/adam.py adam_coeffs (the same bits as the sync path)
    const float lr_t = (float)(lrd_ * std::sqrt(1.0 - std::pow(b2d_, (double)t)) /
                               (1.0 - std::pow(b1d_, (double)t)));
    launch_adam(st->params, g, st->m, st->v, n, lr_t, b1_, b2_, eps_, 1.f, cs_);
  } else {
    launch_momentum(st->params, g, st->m, n, lr_, mu_, 1.f, cs_);
  }
  const int64_t k = ++count_[(size_t)worker * ranges_.size() + p];
  if (keep_prov_) prov_.push_back({(int64_t)worker, (int64_t)p, k, t});
}

// PS side of a session with worker a (who holds both session locks)
void RcclAsync::serve(int a, int p) {
  TraceRange r("ddl.async.rccl.serve");
  AsyncPsState* st = state_of(p);
  const int64_t n = ranges_[p].second - ranges_[p].first;
  std::lock_guard<std::mutex> hold(pause_mu_);
  RCCL_CHECK(rccl().GroupStart());
  RCCL_CHECK(rccl().Recv(gbuf_, (size_t)n, ncclFloat32, a, comm_of(comm_), cs_));
  RCCL_CHECK(rccl().GroupEnd());
  apply(p, a, gbuf_);
  RCCL_CHECK(rccl().GroupStart());
  RCCL_CHECK(rccl().Send(st->params, (size_t)n, ncclFloat32, a, comm_of(comm_), cs_));
  RCCL_CHECK(rccl().GroupEnd());
  HIP_CHECK(hipStreamSynchronize(cs_));
  served_.fetch_add(1);
}

// Worker side of this rank's push of PS p; false when the host is busy (try again later).
bool RcclAsync::push_one(int p) {
  const int h = hosts_[p];
  const int64_t lo = ranges_[p].first, n = ranges_[p].second - lo;
  if (h == rank_ && !self_) {  // own PS: no session
    std::lock_guard<std::mutex> hold(pause_mu_);
    AsyncPsState* st = state_of(p);
    apply(p, rank_, g_ + lo);
    HIP_CHECK(hipMemcpyAsync(w_ + lo, st->params, n * sizeof(float), hipMemcpyDeviceToDevice, cs_));
    HIP_CHECK(hipStreamSynchronize(cs_));
    return true;
  }
  if (h == rank_) {  // 1-rank rehearsal: the same exchange as send/recv to itself
    std::lock_guard<std::mutex> hold(pause_mu_);
    AsyncPsState* st = state_of(p);
    RCCL_CHECK(rccl().GroupStart());
    RCCL_CHECK(rccl().Send(g_ + lo, (size_t)n, ncclFloat32, rank_, comm_of(comm_), cs_));
    RCCL_CHECK(rccl().Recv(gbuf_, (size_t)n, ncclFloat32, rank_, comm_of(comm_), cs_));
    RCCL_CHECK(rccl().GroupEnd());
    apply(p, rank_, gbuf_);
    RCCL_CHECK(rccl().GroupStart());
    RCCL_CHECK(rccl().Send(st->params, (size_t)n, ncclFloat32, rank_, comm_of(comm_), cs_));
    RCCL_CHECK(rccl().Recv(w_ + lo, (size_t)n, ncclFloat32, rank_, comm_of(comm_), cs_));
    RCCL_CHECK(rccl().GroupEnd());
    HIP_CHECK(hipStreamSynchronize(cs_));
    return true;
  }
  if (!locks_.try_lock_pair(rank_, h)) return false;
  TraceRange r("ddl.async.rccl.push");
  try {
    if (!boxes_[h]->push(((int64_t)rank_ << 20) | p, 600.0))
      throw std::runtime_error("session mailbox of rank " + std::to_string(h) + " full");
    RCCL_CHECK(rccl().GroupStart());
    RCCL_CHECK(rccl().Send(g_ + lo, (size_t)n, ncclFloat32, h, comm_of(comm_), cs_));
    RCCL_CHECK(rccl().Recv(w_ + lo, (size_t)n, ncclFloat32, h, comm_of(comm_), cs_));
    RCCL_CHECK(rccl().GroupEnd());
    HIP_CHECK(hipStreamSynchronize(cs_));
  } catch (...) {
    locks_.unlock_pair(rank_, h);
    throw;
  }
  locks_.unlock_pair(rank_, h);
  return true;
}

void RcclAsync::start(int64_t expected_served, bool provenance) {
  if (th_.joinable()) throw std::runtime_error("rccl async: already started");
  if (!comm_) throw std::runtime_error("rccl async: init_comm() first");
  expected_ = expected_served;
  keep_prov_ = provenance;
  th_ = std::thread([this] { loop(); });
}

void RcclAsync::loop() {
  try {
    HIP_CHECK(hipSetDevice(device_));
    for (;;) {
      bool progressed = false;
      if (mine_) {  // incoming session requests first: a waiting worker holds two locks
        const int64_t v = mine_->pop(0.0);
        if (v >= 0) {
          serve((int)(v >> 20), (int)(v & ((1 << 20) - 1)));
          continue;
        }
      }
      std::vector<int> todo;
      {
        std::lock_guard<std::mutex> g(qmu_);
        if (stop_ && pending_.empty() && served_.load() >= expected_) return;
        todo = pending_;
        if (!todo.empty() && !waited_) {
          HIP_CHECK(hipStreamWaitEvent(cs_, ev_, 0));  // this round's gradients are complete
          waited_ = true;
        }
      }
      for (int p : todo) {
        if (!push_one(p)) continue;
        progressed = true;
        std::lock_guard<std::mutex> g(qmu_);
        pending_.erase(std::find(pending_.begin(), pending_.end(), p));
        if (pending_.empty()) cv_.notify_all();
        break;  // back to serving incoming requests between sessions
      }
      if (!progressed) std::this_thread::sleep_for(std::chrono::microseconds(5));
    }
  } catch (const std::exception& e) {
    std::lock_guard<std::mutex> g(qmu_);
    error_ = e.what();
    pending_.clear();
    cv_.notify_all();
  }
}

void RcclAsync::push_pull(hipStream_t compute) {
  TraceRange r("ddl.async.rccl.push_pull");
  HIP_CHECK(hipEventRecord(ev_, compute));
  std::unique_lock<std::mutex> g(qmu_);
  if (!error_.empty()) throw std::runtime_error("rccl async: " + error_);
  for (int p = 0; p < (int)ranges_.size(); ++p) pending_.push_back(p);
  waited_ = false;
  cv_.wait(g, [this] { return pending_.empty(); });
  if (!error_.empty()) throw std::runtime_error("rccl async: " + error_);
}

void RcclAsync::join() {
  {
    std::lock_guard<std::mutex> g(qmu_);
    stop_ = true;
  }
  if (th_.joinable()) th_.join();
  if (!error_.empty()) throw std::runtime_error("rccl async: " + error_);
}

void RcclAsync::pause() {
  pause_mu_.lock();
  const hipError_t e = hipStreamSynchronize(cs_);
  if (e != hipSuccess) {
    pause_mu_.unlock();
    throw std::runtime_error(std::string("rccl async: pause: ") + hipGetErrorString(e));
  }
}

void RcclAsync::resume() { pause_mu_.unlock(); }

void RcclAsync::set_t(int p, int64_t t) {
  if (th_.joinable()) throw std::runtime_error("rccl async: set_t after start()");
  if (t < 0) throw std::invalid_argument("rccl async: negative step counter");
  __atomic_store_n(&state_of(p)->t, t, __ATOMIC_RELEASE);
}

int64_t RcclAsync::t(int p) const {
  for (const auto& s : ps_)
    if (s.ps == p) return __atomic_load_n(&s.t, __ATOMIC_ACQUIRE);
  throw std::invalid_argument("rccl async: PS not hosted here");
}

}  // namespace ddl
