// Native synchronous training-step runner: forward, the four backward segments, and the
// per-unit gradient exchange + PS update, all enqueued from C++ (one Python call per step).
//
// Reference behaviour (SURVEY.md §2.7 sync data plane; mnist_sync_sharding/worker.py:95-120,
// parameter_server.py:108-126): every worker pushes its gradients to the owning PS, the PS
// applies Adam once per global step and every worker pulls the new parameters.  Here:
//
//  * a unit = a set of plan-buffer ranges whose gradients are complete after backward segment
//    `seg`; the comm stream waits on that segment's event, so the exchange of the fc layers
//    runs while the conv backward is still computing (bucketed overlap);
//  * kind LOCAL  : this rank owns the PS of the ranges (W = 1, or co-located) -> fused Adam;
//  * kind RS     : flat plan with one PS per GPU: ncclReduceScatter -> fused Adam on this
//                  rank's 1/W chunk -> in-place ncclAllGather (ring-optimal on xGMI);
//  * kind REDUCE : tensor-granular plans: ncclReduce(dst=host) -> Adam at the host ->
//                  ncclBroadcast(src=host), ranges of a unit grouped in one RCCL group.
//
// The communicator is our own RCCL comm (torch's librccl instance, id exchanged through
// torch.distributed), so the per-step host cost is a few launches instead of one Python
// ProcessGroup call per collective — the Python exchange was host-bound (step timeline:
// 20-45 us GPU idle at every segment boundary).

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "api.h"
#include "common.h"
#include "rccl_api.h"
#include "trace.h"

namespace ddl {

static ncclComm_t as_comm(void* c) { return reinterpret_cast<ncclComm_t>(c); }

// One wave on the comm stream ahead of segment s's exchange units: returns once the compute
// stream has started segment s+1 (READY[s] >= epoch, stored by that launch's first tail block,
// tail.h kind 2), i.e. once every launch of segment s has completed — a kernel boundary writes
// the producer's dirty L2 lines back, so the gradients are in memory for this GPU's exchange
// kernels and for a peer's P2P reads alike.  The comm stream has a priority of its own, so this wait
// never shares a hardware queue with the kernel that releases it.  Bounded (error word).
// On a timeout it also raises the device copy of the error (err_dev, uncached device memory),
// which the gated xGMI bucket kernels behind it read — a host-memory word read by every wave of
// a 512-block bucket kernel was ~2,000 PCIe reads per launch: the forced xGMI rehearsal ran
// 0.49 instead of 0.30 ms/step, the GEMMs beside it ~7x slower.
__global__ void __launch_bounds__(64) ready_gate_kernel(const uint32_t* flag, uint32_t epoch,
                                                        int* err, int* err_dev,
                                                        long long timeout_ticks) {
  if (threadIdx.x != 0) return;
  const long long deadline = wall_clock64() + timeout_ticks;
  // a long sleep between polls (~0.5 us): the first segment's gate of the next step is issued
  // while that step's forward runs, and a tight poll slowed the forward GEMMs by ~20 %
  for (int it = 0;
       (int32_t)(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0;
       ++it) {
    if ((it & 15) == 15 && wall_clock64() > deadline) {
      __hip_atomic_store(err_dev, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __builtin_amdgcn_s_sleep(16);
  }
}

SyncRunner::SyncRunner(Engine* eng, float* params, float* grads, int world, int rank)
    : eng_(eng), w_(params), g_(grads), world_(world), rank_(rank) {
  int lo = 0, hi = 0;
  HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  // collectives + optimizer on a high-priority stream so they are not starved by the GEMMs
  // (DDL_COMM_PRIORITY=low: the least priority instead — also a pool of its own, so the READY
  // gate's argument holds; A/B for ranks sharing a card)
  const char* cp = getenv("DDL_COMM_PRIORITY");
  HIP_CHECK(hipStreamCreateWithPriority(&cs_, hipStreamNonBlocking,
                                        cp && cp[0] == 'l' ? lo : hi));
  // The segment events hand gradients written by this device's GEMMs to RCCL kernels on this
  // device.  On the 1-rank rehearsal (W = 1, every collective a local copy) a device-scope
  // release suffices and removed a ~7 us gap per backward segment (forced 1-rank timeline).
  // With W > 1, RCCL's P2P transports may read these buffers from a peer GPU, and the relaxed
  // fence has not been validated there, so W > 1 keeps the system-scope fence.  The
  // end-of-exchange event keeps the system scope: it orders the next forward after collectives
  // that received peer data, and it is recorded on the comm stream, off the compute stream's
  // critical path.
  const bool sysfence = world_ > 1;
  const unsigned ev_flags =
      hipEventDisableTiming | (sysfence ? 0u : (unsigned)hipEventDisableSystemFence);
  for (int s = 0; s < kSegments; ++s) {
    HIP_CHECK(hipEventCreateWithFlags(&seg_ev_[s], ev_flags));
    // xGMI units: the consumer of the segment's gradients is our own kernel on this device
    // (peers never read them: the exchange pushes), so a device-scope release is exact at
    // any world size
    HIP_CHECK(hipEventCreateWithFlags(&seg_ev_dev_[s],
                                      hipEventDisableTiming | hipEventDisableSystemFence));
  }
  HIP_CHECK(hipEventCreateWithFlags(&done_ev_, hipEventDisableTiming));
  // READY[s] words, then the device copy of the gate's error word
  HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&ready_),
                                  (kSegments + 1) * sizeof(uint32_t), hipDeviceMallocUncached));
  HIP_CHECK(hipMemset(ready_, 0, (kSegments + 1) * sizeof(uint32_t)));
  HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&ready_err_), 64, hipHostMallocDefault));
  memset(ready_err_, 0, 64);
  HIP_CHECK(hipDeviceSynchronize());
  const char* xe = getenv("DDL_EXT_EVENT");
  ext_event_ = xe ? xe[0] == '1' : true;
  // the READY gate is bounded like the xGMI waits (the same setting and default)
  const char* to = getenv("DDL_XGMI_TIMEOUT_S");
  gate_timeout_s_ = to ? atof(to) : 20.0;
}

SyncRunner::~SyncRunner() {
  if (comm_) (void)rccl().CommDestroy(as_comm(comm_));
  comm_ = nullptr;
  release();
}

// Every HIP object the runner owns: the comm stream (a hardware queue of its own priority), the
// events, the READY flags.  Idempotent; after it the runner refuses to step.
void SyncRunner::release() {
  if (cs_) (void)hipStreamSynchronize(cs_);
  if (peer_) peer_->set_gate_error(nullptr);
  for (int s = 0; s < kSegments; ++s) {
    if (seg_ev_[s]) (void)hipEventDestroy(seg_ev_[s]);
    if (seg_ev_dev_[s]) (void)hipEventDestroy(seg_ev_dev_[s]);
    seg_ev_[s] = seg_ev_dev_[s] = nullptr;
  }
  if (done_ev_) (void)hipEventDestroy(done_ev_);
  done_ev_ = nullptr;
  if (ready_) (void)hipFree(ready_);
  ready_ = nullptr;
  if (ready_err_) (void)hipHostFree(ready_err_);
  ready_err_ = nullptr;
  if (cs_) (void)hipStreamDestroy(cs_);
  cs_ = nullptr;
  closed_ = true;
}

void SyncRunner::unique_id(char out[128]) {
  ncclUniqueId id;
  RCCL_CHECK(rccl().GetUniqueId(&id));
  static_assert(sizeof(id) == 128, "ncclUniqueId size");
  memcpy(out, &id, 128);
}

std::string SyncRunner::probe() {
  try {
    (void)rccl();
  } catch (const std::exception& e) {
    return e.what();
  }
  return std::string();
}

void SyncRunner::init_comm(const char id_bytes[128], bool force) {
  if (world_ <= 1 && !force) return;
  ncclUniqueId id;
  memcpy(&id, id_bytes, 128);
  ncclComm_t c;
  RCCL_CHECK(rccl().CommInitRank(&c, world_, id, rank_));
  comm_ = c;
}

void SyncRunner::set_units(const std::vector<RunnerUnit>& units) {
  for (const auto& u : units) {
    if (u.seg < 0 || u.seg >= kSegments) throw std::invalid_argument("unit segment out of range");
    const bool xg = u.kind == RunnerUnit::XGMI || u.kind == RunnerUnit::XGMI_REPL;
    if (u.kind != RunnerUnit::LOCAL && !xg && !comm_)
      throw std::invalid_argument("collective unit without an RCCL communicator");
    if (u.kind == RunnerUnit::AR && u.ranges.size() != 1)
      throw std::invalid_argument("all-reduce unit needs exactly one range");
    if (u.kind == RunnerUnit::RS && (u.ranges.size() != 1 || !u.shard))
      throw std::invalid_argument("RS unit needs exactly one range and a shard buffer");
    if (u.kind == RunnerUnit::RS && (u.ranges[0].hi - u.ranges[0].lo) % world_ != 0)
      throw std::invalid_argument("RS unit range not divisible by the world size");
    if (xg) {
      if (!peer_) throw std::invalid_argument("xGMI unit without a PeerExchange");
      if (u.bucket < 0 || u.bucket >= peer_->num_buckets())
        throw std::invalid_argument("xGMI unit bucket out of range");
      if ((u.kind == RunnerUnit::XGMI_REPL) != (u.bucket == peer_->repl_bucket()))
        throw std::invalid_argument("xGMI unit kind does not match the exchange's replicated bucket");
      // the replicated kernel has no DONE words (the final wait cannot see it) and reuses its
      // parity slots on the next-but-one step: only the compute stream's program order after
      // the last backward segment makes both safe
      if (u.kind == RunnerUnit::XGMI_REPL && u.seg != kSegments - 1)
        throw std::invalid_argument("the replicated xGMI bucket must be the last segment's");
      // (an owner bucket's optimizer state exists only on its owner rank)
      const bool owns = peer_->owner(u.bucket) < 0 || peer_->owner(u.bucket) == rank_;
      if (owns && opt_ == 0 && !u.v) throw std::invalid_argument("xGMI unit without Adam state");
      if (peer_->owner(u.bucket) >= 0 && peer_->owner(u.bucket) != u.host)
        throw std::invalid_argument("xGMI owner bucket hosted on another rank than its unit");
    }
  }
  units_ = units;
  // segments whose off-stream units are all xGMI take the device-scope event
  for (int sg = 0; sg < kSegments; ++sg) {
    bool any = false, only = true;
    for (const auto& u : units_)
      if (u.seg == sg && !(u.kind == RunnerUnit::LOCAL && local_on_main_)) {
        any = true;
        only &= u.kind == RunnerUnit::XGMI || u.kind == RunnerUnit::XGMI_REPL;
      }
    seg_xgmi_only_[sg] = any && only;
    seg_offstream_[sg] = any;
  }
  // the step's last xGMI unit also waits until every owner's parameters have landed here
  last_xgmi_ = -1;
  for (size_t i = 0; i < units_.size(); ++i)
    if ((units_[i].kind == RunnerUnit::XGMI || units_[i].kind == RunnerUnit::XGMI_REPL) &&
        (last_xgmi_ < 0 || units_[i].seg >= units_[last_xgmi_].seg))
      last_xgmi_ = (int)i;
  // W = 1 (every unit LOCAL): one stream.  Ranges adjacent in both the parameter buffer and
  // the PS state merge; per segment they become the optimizer tail of the next segment's dual
  // launch (tail.h), else all of them one coalesced launch at the end of the step.  Same
  // result either way: no backward GEMM reads a tensor after its update.
  merged_.clear();
  for (auto& sp : seg_pieces_) sp.clear();
  tail_ok_ = false;
  all_local_ = true;
  for (const auto& u : units_) all_local_ &= (u.kind == RunnerUnit::LOCAL);
  if (!all_local_) return;
  auto coalesce = [](std::vector<Piece>& v) {
    std::sort(v.begin(), v.end(), [](const Piece& a, const Piece& b) { return a.r.lo < b.r.lo; });
    std::vector<Piece> out;
    for (const auto& p : v) {
      if (!out.empty()) {
        Piece& q = out.back();
        if (q.r.hi == p.r.lo && q.ps == p.ps && q.m == p.m && q.v == p.v &&
            q.r.state_off + (q.r.hi - q.r.lo) == p.r.state_off) {
          q.r.hi = p.r.hi;
          continue;
        }
      }
      out.push_back(p);
    }
    v.swap(out);
  };
  for (const auto& u : units_)
    for (const auto& r : u.ranges) {
      merged_.push_back({r, u.ps, u.m, u.v});
      seg_pieces_[u.seg].push_back({r, u.ps, u.m, u.v});
    }
  coalesce(merged_);
  tail_ok_ = true;
  auto a16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  for (auto& sp : seg_pieces_) {
    coalesce(sp);
    tail_ok_ &= sp.size() <= (size_t)kTailPieces;
    for (const auto& p : sp)
      tail_ok_ &= p.v && (p.r.hi - p.r.lo) % 4 == 0 && a16(w_ + p.r.lo) && a16(g_ + p.r.lo) &&
                  a16(p.m + p.r.state_off) && a16(p.v + p.r.state_off);
  }
}

// Segment `seg`'s Adam as the optimizer tail of the engine's next dual launch.
void SyncRunner::set_tail(int seg, const float* lr_t, int f4_per_block) {
  UpdTail t;
  t.first = tail_first_;
  t.f4_per_block = f4_per_block > 0 ? f4_per_block : tail_f4_;
  t.c1 = 1.f - b1_;
  t.c2 = 1.f - b2_;
  t.eps = eps_;
  t.scale = grad_scale_;
  int blk = 0;
  for (const auto& p : seg_pieces_[seg]) {
    UpdPiece& q = t.p[t.npieces++];
    q.w = w_ + p.r.lo;
    q.g = g_ + p.r.lo;
    q.m = p.m + p.r.state_off;
    q.v = p.v + p.r.state_off;
    q.n = p.r.hi - p.r.lo;
    q.lr_t = lr_t[p.ps];
    q.blk0 = blk;
    blk += (int)((q.n / 4 + t.f4_per_block - 1) / t.f4_per_block);
  }
  t.nblocks = (blk + 7) & ~7;
  eng_->tail = t;
}

void SyncRunner::set_optimizer(int kind, float lr, float b1, float b2, float eps, float mu) {
  if (kind != 0 && kind != 1) throw std::invalid_argument("native runner: adam or momentum");
  opt_ = kind; lr_ = lr; b1_ = b1; b2_ = b2; eps_ = eps; mu_ = mu;
}

// An update on the comm stream overlaps the backward's dual launches: fewer workgroups leave
// the slots those free to the duals (as the xGMI bucket kernels' cap, native_exchange.py).
// Forced RCCL rehearsal, 300-step bench: 2048 / 512 / 256 / 128 / 64 workgroups: 0.2762-0.2771 /
// 0.2745-0.2755 / 0.2723-0.2741 / 0.2717-0.2718 / 0.2752-0.2756 ms/step
// (profiles/r6_comm_adam_grid.log)
#ifndef DDL_COMM_ADAM_GRID
#define DDL_COMM_ADAM_GRID 128
#endif
void SyncRunner::update(float* w, const float* g, float* m, float* v, int64_t n, float lr_t,
                        hipStream_t st) {
  if (opt_ == 0)
    launch_adam_c(w, g, m, v, n, lr_t, 1.f - b1_, 1.f - b2_, eps_, grad_scale_, st,
                  st == cs_ ? DDL_COMM_ADAM_GRID : 2048);
  else launch_momentum(w, g, m, n, lr_, mu_, grad_scale_, st);
}

void SyncRunner::issue(const RunnerUnit& u, const float* lr_t, hipStream_t st) {
  if (u.kind == RunnerUnit::REDUCE) {
    issue_reduce_group({&u}, lr_t, st);
    return;
  }
  if (coef_ != 1.f)
    for (const auto& r : u.ranges) launch_scale(g_ + r.lo, r.hi - r.lo, coef_, st);
  const float lt = lr_t[u.ps];
  switch (u.kind) {
    case RunnerUnit::LOCAL:
      for (const auto& r : u.ranges)
        update(w_ + r.lo, g_ + r.lo, u.m + r.state_off, u.v ? u.v + r.state_off : nullptr,
               r.hi - r.lo, lt, st);
      break;
    case RunnerUnit::RS: {
      const auto& r = u.ranges[0];
      const int64_t c = (r.hi - r.lo) / world_;
      float* mine = w_ + r.lo + rank_ * c;
      RCCL_CHECK(rccl().ReduceScatter(g_ + r.lo, u.shard, (size_t)c, ncclFloat32, ncclSum,
                                   as_comm(comm_), st));
      update(mine, u.shard, u.m + r.state_off, u.v ? u.v + r.state_off : nullptr, c, lt, st);
      RCCL_CHECK(rccl().AllGather(mine, w_ + r.lo, (size_t)c, ncclFloat32, as_comm(comm_), st));
    } break;
    case RunnerUnit::AR: {
      // the step's last bucket, replicated: ONE all-reduce, then every rank runs the update on
      // its replicated optimizer state (one collective instead of reduce-scatter + all-gather
      // on the exposed end of the step)
      const auto& r = u.ranges[0];
      const int64_t n = r.hi - r.lo;
      RCCL_CHECK(rccl().AllReduce(g_ + r.lo, g_ + r.lo, (size_t)n, ncclFloat32, ncclSum,
                                  as_comm(comm_), st));
      update(w_ + r.lo, g_ + r.lo, u.m + r.state_off, u.v ? u.v + r.state_off : nullptr, n, lt, st);
    } break;
    default:
      throw std::invalid_argument("unknown unit kind");
  }
}

// Tensor-granular plans put the units of one backward segment on different hosts (e.g. at
// W = 8 contiguous: conv4 weight on PS 6, its bias on PS 7).  Grouping every reduce of the
// segment lets RCCL run them as one launch with the roots' transfers concurrent on
// different xGMI links, then every broadcast likewise: 2 collective launches per segment
// instead of 2 per unit (each launch costs ~10-20 us of latency on an 8-GPU ring).
void SyncRunner::issue_reduce_group(const std::vector<const RunnerUnit*>& us, const float* lr_t,
                                    hipStream_t st) {
  for (const RunnerUnit* u : us)
    if (coef_ != 1.f)
      for (const auto& r : u->ranges) launch_scale(g_ + r.lo, r.hi - r.lo, coef_, st);
  RCCL_CHECK(rccl().GroupStart());
  for (const RunnerUnit* u : us)
    for (const auto& r : u->ranges)
      RCCL_CHECK(rccl().Reduce(g_ + r.lo, g_ + r.lo, (size_t)(r.hi - r.lo), ncclFloat32, ncclSum,
                               u->host, as_comm(comm_), st));
  RCCL_CHECK(rccl().GroupEnd());
  for (const RunnerUnit* u : us)
    if (rank_ == u->host)
      for (const auto& r : u->ranges)
        update(w_ + r.lo, g_ + r.lo, u->m + r.state_off, u->v ? u->v + r.state_off : nullptr,
               r.hi - r.lo, lr_t[u->ps], st);
  RCCL_CHECK(rccl().GroupStart());
  for (const RunnerUnit* u : us)
    for (const auto& r : u->ranges)
      RCCL_CHECK(rccl().Broadcast(w_ + r.lo, w_ + r.lo, (size_t)(r.hi - r.lo), ncclFloat32,
                                  u->host, as_comm(comm_), st));
  RCCL_CHECK(rccl().GroupEnd());
}

static const char* const kBwdRange[SyncRunner::kSegments] = {
    "ddl.bwd.seg0(head+fc)", "ddl.bwd.seg1(conv4)", "ddl.bwd.seg2(conv3)",
    "ddl.bwd.seg3(conv2+conv1)"};
static const char* const kExRange[SyncRunner::kSegments] = {
    "ddl.exchange.seg0", "ddl.exchange.seg1", "ddl.exchange.seg2", "ddl.exchange.seg3"};

void SyncRunner::step(const float* x, const int64_t* labels, int B, uint32_t seed_value,
                      const float* lr_t, hipStream_t st) {
  if (closed_) throw std::runtime_error("sync runner: step() after close()");
  TraceRange step_range("ddl.step");
  eng_->seed_value = seed_value;  // dropout seed by kernel argument: no seed-upload kernel
  const uint32_t* seed = nullptr;
  // Cross-queue dependencies (event record -> stream wait) cost tens of microseconds of GPU
  // idle each on this stack (measured), so LOCAL updates go straight onto the compute
  // stream in order; only units with collectives use the comm stream, which then overlaps
  // the remaining backward segments.
  {
    TraceRange r("ddl.fwd");
    eng_->forward(x, B, seed, true, st, /*defer_fc2=*/true);  // backward_segment(0) follows
  }
  if (all_local_ && local_on_main_ && use_tail_ && tail_ok_ && opt_ == 0 && coef_ == 1.f) {
    // segment s-1's update rides in segment s's dual launch (flushed as a launch of its own
    // if the segment had no dual launch to take it); the last segment's follows the backward
    for (int s = 0; s < kSegments; ++s) {
      TraceRange r(kBwdRange[s]);
      if (s > 0 && !seg_pieces_[s - 1].empty()) set_tail(s - 1, lr_t);
      // the last segment's own update rides in its final launch when the engine can take it
      // (conv1's weight-gradient reduce: engine_impl.h dual_then_b)
      if (s == kSegments - 1 && final_in_reduce_ && !seg_pieces_[s].empty()) {
        // one pass per tail block (2 float4 per lane): on the step's critical path the update
        // wants width, not the long blocks that hide beside a dual launch's GEMM blocks
        const UpdTail keep = eng_->tail;
        set_tail(s, lr_t, kTailF4PerBlock);
        eng_->final_upd = eng_->tail;
        eng_->tail = keep;
      }
      eng_->backward_segment(s, x, labels, B, seed, st);
      eng_->flush_tail(st);
    }
    if (eng_->final_upd.npieces == 0 && final_in_reduce_ && !seg_pieces_[kSegments - 1].empty())
      return;  // taken by the last launch
    eng_->final_upd = UpdTail();
    TraceRange r("ddl.update.last_segment");
    for (const auto& p : seg_pieces_[kSegments - 1])
      update(w_ + p.r.lo, g_ + p.r.lo, p.m + p.r.state_off, p.v + p.r.state_off,
             p.r.hi - p.r.lo, lr_t[p.ps], st);
    return;
  }
  if (all_local_ && local_on_main_) {
    for (int s = 0; s < kSegments; ++s) {
      TraceRange r(kBwdRange[s]);
      eng_->backward_segment(s, x, labels, B, seed, st);
    }
    TraceRange r("ddl.update");
    if (coef_ != 1.f)
      for (const auto& p : merged_) launch_scale(g_ + p.r.lo, p.r.hi - p.r.lo, coef_, st);
    for (const auto& p : merged_)
      update(w_ + p.r.lo, g_ + p.r.lo, p.m + p.r.state_off, p.v ? p.v + p.r.state_off : nullptr,
             p.r.hi - p.r.lo, lr_t[p.ps], st);
    return;
  }
  // The last segment's gradients complete with the backward, so nothing is left to overlap
  // its exchange with: its collectives go in order on the compute stream (no event record /
  // stream wait between the final backward launch, the exchange and the next forward).
  bool comm_used = false;
  if (__atomic_load_n(ready_err_, __ATOMIC_ACQUIRE))
    throw std::runtime_error("sync runner: a READY gate timed out (a segment never completed)");
  ++ready_epoch_;
  if (last_xgmi_ >= 0) {
    if (const int e = peer_->error())
      throw std::runtime_error("xGMI exchange timed out waiting for a peer (code " +
                               std::to_string(e) + ")");
    ++epoch_;
  }
  std::vector<const RunnerUnit*> reduces;
  for (int s = 0; s < kSegments; ++s) {
    const bool on_main = last_on_main_ && s == kSegments - 1;
    hipEvent_t ev = seg_xgmi_only_[s] ? seg_ev_dev_[s] : seg_ev_[s];
    // xGMI-only segment followed by another: the hand-off to the comm stream is a READY flag
    // stored by the next segment's first launch (tail.h kind 2) and a one-wave gate ahead of the
    // bucket kernels on the comm stream — no event record / stream wait (each left ~5 us of
    // idle compute stream: profiles/r4_step_timeline_forced_xgmi.txt).  The comm stream has
    // high priority, so the gate never shares a hardware queue with the kernel it waits for;
    // and it is bounded (error 5).
    const bool flag = ready_flags_ > (s == 0 ? 1 : 0) && !on_main && seg_offstream_[s] &&
                      s + 1 < kSegments && gate_safe(st);
    // otherwise the comm stream waits for this segment's gradients by an event: bound to the
    // segment's kernel launches themselves (the wait below is issued after the last one) rather
    // than a marker packet behind them
    const bool bind = ext_event_ && !on_main && seg_offstream_[s] && !flag;
    // bound to the segment's LAST launch (its count is learned from the previous step; a
    // wrong or unknown count falls back to a marker record below, which supersedes the binding)
    bool marker = !bind;
    {
      TraceRange r(kBwdRange[s]);
      StopEventScope scope(bind ? ev : nullptr, seg_launches_[s] > 0 ? seg_launches_[s] - 1
                                                                      : 1 << 30);
      eng_->backward_segment(s, x, labels, B, seed, st);
      if (bind) {
        const int n = scope.launches();
        if (scope.bound() != n - 1) marker = true;
        seg_launches_[s] = n;
      }
    }
    TraceRange ex_range(kExRange[s]);
    hipStream_t xs = on_main ? st : cs_;
    bool waited = on_main;
    reduces.clear();
    for (size_t i = 0; i < units_.size(); ++i) {
      const auto& u = units_[i];
      if (u.seg != s) continue;
      if (u.kind == RunnerUnit::LOCAL && local_on_main_) {
        issue(u, lr_t, st);
        continue;
      }
      if (!waited) {
        if (flag) {
          eng_->flush_tail(st);  // (no update tail is pending at W > 1; keep the slot free)
          UpdTail t;
          t.kind = 2;
          t.epoch = ready_epoch_;
          t.npieces = 1;
          t.p[0].arrive = ready_ + s;
          t.nblocks = 8;
          t.first = 1;
          eng_->tail = t;
          hipLaunchKernelGGL(ready_gate_kernel, dim3(1), dim3(64), 0, cs_, ready_ + s,
                             ready_epoch_, ready_err_, ready_err_dev(),
                             (long long)(gate_timeout_s_ * 1e8));
          DDL_CHECK_LAUNCH();
        } else {
          if (marker) HIP_CHECK(hipEventRecord(ev, st));
          HIP_CHECK(hipStreamWaitEvent(cs_, ev, 0));
        }
        waited = true;
      }
      if (u.kind == RunnerUnit::XGMI || u.kind == RunnerUnit::XGMI_REPL) {
        // the final wait orders the next forward after every owner's pushes; only if it runs
        // on the comm stream does the compute stream need the end-of-exchange event
        const bool fin = (int)i == last_xgmi_;
        comm_used |= fin && !on_main;
        issue_xgmi(u, lr_t, fin, xs, flag);
        continue;
      }
      comm_used |= !on_main;
      if (u.kind == RunnerUnit::REDUCE) reduces.push_back(&u);
      else issue(u, lr_t, xs);
    }
    if (!reduces.empty()) issue_reduce_group(reduces, lr_t, xs);
  }
  eng_->flush_tail(st);  // a READY flag no launch took (none in the tuned schedules)
  if (comm_used) {
    TraceRange r("ddl.exchange.join");
    // the next step's forward reads the updated parameters
    HIP_CHECK(hipEventRecord(done_ev_, cs_));
    HIP_CHECK(hipStreamWaitEvent(st, done_ev_, 0));
  }
}

// The READY gate waits on the comm stream for a kernel of `st`: only safe when `st` cannot share
// a hardware queue with the comm stream, i.e. when its priority differs from the comm stream's
// (HIP pools hardware queues per priority; the comm stream is the greatest priority, or the
// least with DDL_COMM_PRIORITY=low).  Otherwise the segment falls back to the event hand-off.
bool SyncRunner::gate_safe(hipStream_t st) {
  if (gate_checked_ && st == gate_checked_stream_) return gate_checked_ok_;
  int lo = 0, hi = 0, p = 0, cp = 0;  // (the null stream is a normal-priority stream)
  gate_checked_ok_ = hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess &&
                     (st == nullptr || hipStreamGetPriority(st, &p) == hipSuccess) &&
                     hipStreamGetPriority(cs_, &cp) == hipSuccess && hi != lo && p != cp;
  gate_checked_stream_ = st;
  gate_checked_ = true;
  return gate_checked_ok_;
}

void SyncRunner::issue_xgmi(const RunnerUnit& u, const float* lr_t, bool final_wait,
                            hipStream_t st, bool gated) {
  XgmiUpdate up;
  const auto& r = u.ranges[0];
  up.opt = opt_;
  // an owner bucket addresses its runs' state offsets itself (PeerExchange bucket spec)
  const bool own = peer_->owner(u.bucket) >= 0;
  up.m = u.m ? u.m + (own ? 0 : r.state_off) : nullptr;
  up.v = u.v ? u.v + (own ? 0 : r.state_off) : nullptr;
  up.lr_t = lr_t[u.ps];
  up.c1 = 1.f - b1_;
  up.c2 = 1.f - b2_;
  up.eps = eps_;
  up.lr = lr_;
  up.mu = mu_;
  up.scale = grad_scale_;
  up.coef = coef_;
  peer_->launch(u.bucket, epoch_, up, final_wait, st, gated);
}

void SyncRunner::peer_selftest_step(hipStream_t st) {
  if (!peer_) throw std::runtime_error("no PeerExchange");
  ++epoch_;
  XgmiUpdate up;
  up.opt = 2;
  const int nb = peer_->num_buckets();
  for (int b = 0; b < nb; ++b) peer_->launch(b, epoch_, up, b == nb - 1, st);
}

// Failure detection: RCCL reports remote-peer / network failures
// asynchronously; the trainer polls this between steps and the watchdog aborts the comm (so
// blocked collectives on this rank return and the job can be torn down) on a hang.
std::string SyncRunner::async_error() {
  if (peer_ && peer_->error())
    return "xGMI exchange timed out waiting for a peer (code " + std::to_string(peer_->error()) +
           ")";
  if (!comm_) return std::string();
  ncclResult_t st = ncclSuccess;
  RCCL_CHECK(rccl().CommGetAsyncError(as_comm(comm_), &st));
  if (st == ncclSuccess || st == ncclInProgress) return std::string();
  return rccl().GetErrorString(st);
}

// Orderly teardown: every rank calls this at the same point of its program (after a barrier),
// so a communicator finalisation that synchronises with the peers cannot hang on a rank that
// has not reached it yet; afterwards the destructor has nothing collective left to do.
void SyncRunner::close() {
  if (comm_) {
    HIP_CHECK(hipStreamSynchronize(cs_));
    (void)rccl().CommDestroy(as_comm(comm_));
    comm_ = nullptr;
  }
  // and every stream / event / flag with it: a closed runner holds no hardware queue (the
  // one-card W = 4 rehearsal kept four processes' released runners' queues until GC)
  release();
}

void SyncRunner::abort() {
  if (!comm_) return;
  (void)rccl().CommAbort(as_comm(comm_));
  comm_ = nullptr;
}

// Collective sanity check used before trusting the native path on a multi-GPU job: the RS
// and REDUCE patterns on a known pattern, compared on the host.
bool SyncRunner::selftest(std::string* why) {
  if (!comm_) return world_ <= 1;
  const int64_t c = 1031, n = c * world_;
  float *buf = nullptr, *shard = nullptr;
  HIP_CHECK(hipMalloc(&buf, n * sizeof(float)));
  HIP_CHECK(hipMalloc(&shard, c * sizeof(float)));
  std::vector<float> h(n), out(n);
  auto val = [&](int r, int64_t i) { return (float)((r + 1) * ((i % 13) + 1)); };
  for (int64_t i = 0; i < n; ++i) h[i] = val(rank_, i);
  bool ok = true;
  try {
    HIP_CHECK(hipMemcpy(buf, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
    // RS then AG of the reduced chunk: every element = sum_r val(r, i)
    RCCL_CHECK(rccl().ReduceScatter(buf, shard, (size_t)c, ncclFloat32, ncclSum, as_comm(comm_), cs_));
    RCCL_CHECK(rccl().AllGather(shard, buf, (size_t)c, ncclFloat32, as_comm(comm_), cs_));
    HIP_CHECK(hipStreamSynchronize(cs_));
    HIP_CHECK(hipMemcpy(out.data(), buf, n * sizeof(float), hipMemcpyDeviceToHost));
    const float rs = (float)(world_ * (world_ + 1) / 2);
    for (int64_t i = 0; i < n && ok; ++i)
      if (out[i] != rs * (float)((i % 13) + 1)) {
        ok = false;
        if (why) *why = "reduce_scatter/all_gather mismatch at " + std::to_string(i);
      }
    // REDUCE to the last rank, then BROADCAST from it
    const int root = world_ - 1;
    HIP_CHECK(hipMemcpy(buf, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
    RCCL_CHECK(rccl().GroupStart());
    RCCL_CHECK(rccl().Reduce(buf, buf, (size_t)n, ncclFloat32, ncclSum, root, as_comm(comm_), cs_));
    RCCL_CHECK(rccl().GroupEnd());
    RCCL_CHECK(rccl().GroupStart());
    RCCL_CHECK(rccl().Broadcast(buf, buf, (size_t)n, ncclFloat32, root, as_comm(comm_), cs_));
    RCCL_CHECK(rccl().GroupEnd());
    HIP_CHECK(hipStreamSynchronize(cs_));
    HIP_CHECK(hipMemcpy(out.data(), buf, n * sizeof(float), hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < n && ok; ++i)
      if (out[i] != rs * (float)((i % 13) + 1)) {
        ok = false;
        if (why) *why = "reduce/broadcast mismatch at " + std::to_string(i);
      }
  } catch (const std::exception& e) {
    ok = false;
    if (why) *why = e.what();
  }
  (void)hipFree(buf);
  (void)hipFree(shard);
  return ok;
}

}  // namespace ddl
