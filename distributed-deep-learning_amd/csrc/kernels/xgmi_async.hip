// Asynchronous parameter server over xGMI peer memory (SURVEY.md §2.3 async PS, §7.3 hard
// part 1).
//
// Reference behaviour (mnist_async_sharding/worker.py:30-37,88-94; parameter_server.py:94-111):
// every worker Sends each gradient tensor to its PS and blocks in Recv for the parameters; the
// PS Recvs from ANY_SOURCE, applies Adam per arrival (its own step counter) and Sends the
// parameters back to whoever sent.  Staleness is at most one step per worker.
//
// A worker round:
//   push      (worker stream, after the backward segment that completes the listed PS ranges;
//             tail blocks of the next segment's launch, async_runner.hip) those PS shards of the
//             gradient -> each PS host's inbox slot [ps][worker] (system write-through stores);
//             per workgroup, once its payload is acknowledged, POSTED[ps][worker][slice] = e on
//             the ARRIVAL BOARD in host memory
//   serve     (PS host) a native service thread scans the host board and launches one apply
//             per (worker, ps) whose every slice is posted, in the order it observes them (the
//             reference's MPI.ANY_SOURCE order; AsyncService::run).  (Round 5's on-GPU pop —
//             claim kernels polling a device copy of the board — measured equal at W = 1 and
//             1.3-1.7x slower with several ranks on one card, and was removed in round 6:
//             docs/DESIGN.md.)
//   apply     (PS host, its PS stream) Adam on the PS's private parameter copy (one step of its
//             counter t per arrival, atomic per shard: the reference's per-tag mixing race Q3
//             cannot happen), store the new shard into the WORKER's parameter buffer, then
//             DONE[ps][slice] = e in the worker's device flags (its GPU-side pull gate) and
//             DONE[worker][ps][slice] = e in host memory (its host's bounded check)
//   wait      (worker) a one-wave gate on its compute stream polls DONE[ps][slice] >= e
//             before the next forward (async_runner.hip; the host wait of set_gate(false) and
//             of the Python push_pull path polls the host copy)
// Board and DONE words live in one POSIX shm segment registered with HIP by every rank (one
// node: the xGMI hive).  The board replaced a token mailbox fed by a poster thread that waited
// for each push's completion EVENT: a kernel with a completion signal ends with a system-scope
// release (an L2 write-back) and left a ~4.6 us hole on the compute stream after every push,
// plus two host hand-offs (poster -> mailbox -> service) on the critical path of the last push
// (docs/DESIGN.md, round 4 async timeline).
// The hardware-queue argument (why no wait here can deadlock).  The only kernel wait is the
// worker's pull gate (compute stream), which waits for applies.  HIP maps a process's streams
// onto hardware queues pooled PER PRIORITY; the PS stream is HIGH priority and the compute
// stream is not (async_runner.hip checks it and falls back to a host wait), so no apply is ever
// queued behind a gate.  An apply waits for nothing (the host launches it once the push is on
// the board), so every chain ends at a kernel that waits for nothing.  The one remaining hazard
// is time slicing of oversubscribed hardware queues (several ranks on one card): a waiter then
// spins until the queue holding what it waits for is mapped in again (milliseconds), which
// parallel/comm.py share_gpu_queue_cap avoids with one hardware queue per process.  Every wait
// is bounded: the gate records an error word instead of hanging.
#include <fcntl.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>

#include <cmath>

#include "api.h"
#include "trace.h"
#include "common.h"

namespace ddl {

namespace {

DDL_DEV void drain_vm() { drain_vmem(); }

DDL_DEV bool wait_ge(const uint32_t* f, uint32_t target, long long deadline, int* err, int code) {
  // the error word lives in host memory (a PCIe round trip per load): look at it, and at the
  // clock, only every 32nd poll, so a flag that lands is seen within one poll of local memory
  for (int it = 0; (int32_t)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - target) < 0; ++it) {
    if ((it & 31) == 31) {
      if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) return false;
      if (wall_clock64() > deadline) {
        __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return false;
      }
    }
    __builtin_amdgcn_s_sleep(2);
  }
  return true;
}
// The flag that publishes a workgroup's payload.  Every payload store is a system-scope
// (sc0|sc1) write-through store, and every storing wave drains vmcnt(0) before the workgroup
// barrier that precedes the flag store: a write-through store is counted complete only once the
// memory side (local HBM, or the peer over xGMI, or host memory) has acknowledged it, so the
// payload is globally visible before the flag is issued — no L2 write-back is needed (the CDNA
// guide's G16 write-through hand-off, at system scope).  A full system release at each flag (L2
// write-back + wait) writes back every dirty line of the XCD's L2 — the GEMMs' output included —
// and measured 3.2 -> 5.4 ms/step on the two-ranks-on-one-GPU rehearsal (round 2).
DDL_DEV void flag_store(uint32_t* f, uint32_t v) {
  __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// completion words DONE[worker][ps][slice] in the shared host segment, then the arrival board
// POSTED[ps][worker][slice].  Every word has ONE writer and is only stored, never
// read-modify-written (atomics through IPC / host mappings are not safe to combine)
DDL_DEV int done_word(int w, int p, int j) { return (w * kAsyncMaxPs + p) * kAsyncMaxSlices + j; }
__host__ __device__ inline size_t posted_word(int p, int w, int j) {
  return ((size_t)p * kXgmiMaxPeers + w) * kAsyncMaxSlices + j;
}
// the same completion words in the WORKER's uncached device flags, densely numbered over all PS'
// slices (AsyncShard::slice0): what its GPU-side pull gate polls (a GPU polling the host-memory
// copy measured ~25 us late: the registered host segment is not guaranteed to bypass the GPU's
// L2 for a system-scope load)
DDL_DEV int done_dev_idx(const AsyncShard& S, int j) { return S.slice0 + j; }

struct PushArgs {
  int world, rank, nps;
  uint32_t epoch;
  int first_blk[kAsyncMaxPs + 1];  // block range of entry i: [first_blk[i], first_blk[i+1])
  int ps[kAsyncMaxPs];             // subset: the PS id of entry i (else entry i is PS i)
  int subset;
  const float* grads;
  float coef;
  // the pull gate as the launch's last block (async_runner.hip: the round's last push)
  int gate, gate_total;
  int* err;
  long long timeout_ticks;
};

DDL_DEV void gate_body(const AsyncTable& T, int rank, int total, uint32_t epoch, int* err,
                       long long timeout_ticks);

// The table (3 KB: 64 shard descriptors) is read from device memory, not passed by value: a
// 3 KB kernel-argument block made every push / apply launch cost ~6-12 us of host time.
__global__ void __launch_bounds__(256) async_push_kernel(const AsyncTable* __restrict__ Tp,
                                                         PushArgs a) {
  const AsyncTable& T = *Tp;
  const int blk = blockIdx.x, tid = threadIdx.x;
  if (a.gate && blk == (int)gridDim.x - 1) {  // dispatched after every push block of the launch
    if (tid < 64) gate_body(T, a.rank, a.gate_total, a.epoch, a.err, a.timeout_ticks);
    return;
  }
  int e = 0;
  while (e + 1 < a.nps && blk >= a.first_blk[e + 1]) ++e;
  const int p = a.subset ? a.ps[e] : e;
  const AsyncShard& S = T.shard[p];
  const int j = blk - a.first_blk[e];
  const int64_t s0 = (int64_t)j * S.slice;
  const int64_t s1 = s0 + S.slice < S.n ? s0 + S.slice : S.n;
  const int n4 = s0 < s1 ? (int)((s1 - s0) >> 2) : 0;
  const float4* src = reinterpret_cast<const float4*>(a.grads + S.lo + s0);
  const brsrc_t dst = make_rsrc(T.inbox[S.host] + S.inbox_off + (int64_t)a.rank * S.n + s0,
                                (uint32_t)n4 * 16u);
  const bool local = T.elide && S.host == a.rank;  // the apply reads T.grads itself
  for (int i = local ? n4 : tid; i < n4; i += 256) {
    float4 x = src[i];
    if (a.coef != 1.f) { x.x *= a.coef; x.y *= a.coef; x.z *= a.coef; x.w *= a.coef; }
    bstore4_sys(dst, i * 16, x);
  }
  drain_vm();
  __syncthreads();
  if (tid == 0) {
    __hip_atomic_store(T.posted + posted_word(p, a.rank, j), a.epoch, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

struct ApplyArgs {
  int me, ps, worker;
  uint32_t epoch;
  float* ps_params;  // the PS's private parameter copy of its shard [n]
  float* m;
  float* v;
  int opt;
  float lr_t, c1, c2, eps, lr, mu, scale;
};

// Slice j of one apply.  No arrival poll: the apply runs only after every slice of the push was
// seen posted by the host service, and a push block
// posts only after its payload stores were acknowledged (the inbox loads below are
// system-coherent, so they see that payload).
DDL_DEV void apply_body(const AsyncTable& T, const ApplyArgs& a, int j) {
  const AsyncShard& S = T.shard[a.ps];
  const int tid = threadIdx.x;
  const int64_t s0 = (int64_t)j * S.slice;
  const int64_t s1 = s0 + S.slice < S.n ? s0 + S.slice : S.n;
  const int n4 = s0 < s1 ? (int)((s1 - s0) >> 2) : 0;
  const float* src = T.elide && a.worker == a.me
                        ? T.grads + S.lo + s0  // this rank's own push: no inbox copy
                        : T.inbox[a.me] + S.inbox_off + (int64_t)a.worker * S.n + s0;
  const brsrc_t in = make_rsrc(src, (uint32_t)n4 * 16u);
  const brsrc_t out = make_rsrc(T.params[a.worker] + S.lo + s0, (uint32_t)n4 * 16u);
  float4* w4 = reinterpret_cast<float4*>(a.ps_params + s0);
  float4* m4 = reinterpret_cast<float4*>(a.m + s0);
  float4* v4 = a.v ? reinterpret_cast<float4*>(a.v + s0) : nullptr;
  for (int i = tid; i < n4; i += 256) {
    const float4 g = bload4_sys(in, i * 16);
    float4 w = w4[i];
    if (a.opt == 0) {
      float4 M = m4[i], V = v4[i];
      adam1(w.x, g.x * a.scale, M.x, V.x, a.lr_t, a.c1, a.c2, a.eps);
      adam1(w.y, g.y * a.scale, M.y, V.y, a.lr_t, a.c1, a.c2, a.eps);
      adam1(w.z, g.z * a.scale, M.z, V.z, a.lr_t, a.c1, a.c2, a.eps);
      adam1(w.w, g.w * a.scale, M.w, V.w, a.lr_t, a.c1, a.c2, a.eps);
      m4[i] = M; v4[i] = V;
    } else if (a.opt == 1) {
      float4 M = m4[i];
      momentum1(w.x, g.x, M.x, a.lr, a.mu, a.scale);
      momentum1(w.y, g.y, M.y, a.lr, a.mu, a.scale);
      momentum1(w.z, g.z, M.z, a.lr, a.mu, a.scale);
      momentum1(w.w, g.w, M.w, a.lr, a.mu, a.scale);
      m4[i] = M;
    } else {  // self-test: the PS shard := the pushed gradient
      w = g;
    }
    w4[i] = w;
    bstore4_sys(out, i * 16, w);
  }
  drain_vm();
  __syncthreads();
  if (tid == 0) {
    flag_store(T.flags[a.worker] + done_dev_idx(S, j), a.epoch);  // the worker's gate
    flag_store(T.done + done_word(a.worker, a.ps, j), a.epoch);       // the worker's host
  }
}

__global__ void __launch_bounds__(256) async_apply_kernel(const AsyncTable* __restrict__ Tp,
                                                          ApplyArgs a) {
  apply_body(*Tp, a, blockIdx.x);
}

// The worker's pull as a GPU-side gate (async_runner.hip): one wave on the compute stream,
// enqueued after the round's last push and before the next forward, polls this worker's DONE
// words of round `epoch` (every PS, every slice; the device copy in its own flags) and ends
// when all have landed; the forward
// behind it starts with no host round trip.  Bounded like every wait here: on timeout it records
// error code 4 and ends (the host's lagged check raises).  Why this wait cannot deadlock is in
// async_runner.hip (the applies it waits for run on other processes' queues or on this
// process's high-priority service queue, never behind it).
struct GateArgs {
  int total;  // slices of all PS (the dense DONE words 0 .. total-1)
  uint32_t epoch;
  int* err;
  long long timeout_ticks;
  int rank;
};

// Each sweep issues eight independent loads per lane before comparing (one round of latency for
// 512 words, instead of one per word), and skips the leading batches already seen complete
// (the early segments' PS finish first).
DDL_DEV void gate_body(const AsyncTable& T, int rank, int total, uint32_t epoch, int* err,
                       long long timeout_ticks) {
  const long long deadline = wall_clock64() + timeout_ticks;
  const uint32_t* done = T.flags[rank];
  const int lane = threadIdx.x & 63;
  int start = 0;  // wave-uniform: batches below it are complete
  for (int it = 0;; ++it) {
    bool all = true;
    for (int k0 = start; k0 < total; k0 += 512) {
      uint32_t v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + u * 64 + lane;
        v[u] = k < total ? __hip_atomic_load(done + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                         : epoch;
      }
      bool ok = true;
#pragma unroll
      for (int u = 0; u < 8; ++u) ok &= (int32_t)(v[u] - epoch) >= 0;
      const bool batch = __all(ok);
      if (batch && k0 == start) start += 512;
      all &= batch;
    }
    if (all) return;
    if ((it & 31) == 31) {
      if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) return;
      if (wall_clock64() > deadline) {
        if (lane == 0) __hip_atomic_store(err, 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
      }
    }
    // a tight poll for the first ~64 sweeps (the W = 1 wait for the last apply is a few us),
    // then ~0.45 us apart: a gate waiting for another rank's applies must not load the memory
    // system under that rank's GEMMs (one-card W = 2)
    if (it < 64) __builtin_amdgcn_s_sleep(2);
    else __builtin_amdgcn_s_sleep(16);
  }
}

__global__ void __launch_bounds__(64) async_gate_kernel(const AsyncTable* __restrict__ Tp,
                                                        GateArgs a) {
  gate_body(*Tp, a.rank, a.total, a.epoch, a.err, a.timeout_ticks);
}

#define X_CHECK(x)                                                                        \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess)                                                                 \
      throw std::runtime_error(std::string("xgmi-async: ") + #x + ": " + hipGetErrorString(e_)); \
  } while (0)

struct HandleBlob {
  hipIpcMemHandle_t params, inbox, flags;
  int64_t params_off;
  int32_t world, rank;
};

}  // namespace

AsyncPeer::AsyncPeer(float* params, const float* grads, int64_t total, int world, int rank,
                     const std::vector<std::pair<int64_t, int64_t>>& ps_ranges,
                     const std::vector<int>& ps_host, int max_slices)
    : params_(params), grads_(grads), world_(world), rank_(rank) {
  if (world < 1 || world > kXgmiMaxPeers) throw std::invalid_argument("async xgmi: world");
  if (rank < 0 || rank >= world) throw std::invalid_argument("async xgmi: rank");
  if (ps_ranges.empty() || (int)ps_ranges.size() > kAsyncMaxPs ||
      ps_ranges.size() != ps_host.size())
    throw std::invalid_argument("async xgmi: 1..64 PS, one host each");
  if (max_slices < 1 || max_slices > kAsyncMaxSlices)
    throw std::invalid_argument("async xgmi: max_slices");
  if (reinterpret_cast<uintptr_t>(params) % 16 || reinterpret_cast<uintptr_t>(grads) % 16)
    throw std::invalid_argument("async xgmi: buffers must be 16-B aligned");
  memset(&table_, 0, sizeof(table_));
  nps_ = (int)ps_ranges.size();
  int64_t inbox = 0;
  for (int p = 0; p < nps_; ++p) {
    AsyncShard& S = table_.shard[p];
    S.lo = ps_ranges[p].first;
    S.n = ps_ranges[p].second - ps_ranges[p].first;
    S.host = ps_host[p];
    if (S.lo < 0 || S.n <= 0 || S.lo + S.n > total || S.n % 4 || S.lo % 4)
      throw std::invalid_argument("async xgmi: PS range must be a 4-aligned slice of the buffer");
    if (S.host < 0 || S.host >= world) throw std::invalid_argument("async xgmi: PS host");
    // >= 2048 elements (8 KB) per workgroup, at most max_slices workgroups: a 1.6 M-element
    // shard spreads over 512 workgroups (64 left the apply at ~2 TB/s, 41.6 us for the whole
    // model at W = 1, profiles/r4_step_timeline_async_xgmi_w1.txt)
    int64_t ns = (S.n + 2047) / 2048;
    if (ns > max_slices) ns = max_slices;
    S.slice = ((S.n + ns - 1) / ns + 3) & ~(int64_t)3;
    S.nslice = (int)((S.n + S.slice - 1) / S.slice);
    S.slice0 = p == 0 ? 0 : table_.shard[p - 1].slice0 + table_.shard[p - 1].nslice;
    if (S.n * 4 * world > 0x7fffffffLL) throw std::invalid_argument("async xgmi: shard too large");
  }
  // inbox of a host: one [W][n] slot block per hosted PS, in PS order (every rank computes
  // every host's layout identically, so pushes know where to write)
  std::vector<int64_t> off(world, 0);
  for (int p = 0; p < nps_; ++p) {
    AsyncShard& S = table_.shard[p];
    S.inbox_off = off[S.host];
    off[S.host] += S.n * world;
  }
  inbox = off[rank];
  inbox_elems_ = inbox > 0 ? inbox : 4;
  X_CHECK(hipMalloc(&inbox_, inbox_elems_ * sizeof(float)));
  X_CHECK(hipMemset(inbox_, 0, inbox_elems_ * sizeof(float)));
  const size_t flag_bytes = kAsyncFlagWords * sizeof(uint32_t);  // DONE, then POSTED[worker]
  X_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&flags_), flag_bytes,
                                hipDeviceMallocUncached));
  X_CHECK(hipMemset(flags_, 0, flag_bytes));
  X_CHECK(hipHostMalloc(reinterpret_cast<void**>(&err_), 64, hipHostMallocDefault));
  memset(err_, 0, 64);
  X_CHECK(hipMalloc(reinterpret_cast<void**>(&table_dev_), sizeof(AsyncTable)));
  X_CHECK(hipDeviceSynchronize());
  const char* t = getenv("DDL_XGMI_TIMEOUT_S");
  timeout_s_ = t ? atof(t) : 60.0;
  const char* el = getenv("DDL_ASYNC_ELIDE_LOCAL");
  table_.grads = grads;
  table_.elide = el ? atoi(el) != 0 : 1;
}

AsyncPeer::~AsyncPeer() { close(); }

void AsyncPeer::close() {
  if (inbox_ || flags_ || opened_ok_) (void)hipDeviceSynchronize();
  for (int q = 0; q < world_; ++q) {
    if (q == rank_) continue;
    for (void*& p : opened_[q]) {
      if (p) (void)hipIpcCloseMemHandle(p);
      p = nullptr;
    }
  }
  opened_ok_ = false;
  if (inbox_) (void)hipFree(inbox_);
  if (flags_) (void)hipFree(flags_);
  if (err_) (void)hipHostFree(err_);
  if (table_dev_) (void)hipFree(table_dev_);
  inbox_ = nullptr;
  flags_ = nullptr;
  err_ = nullptr;
  table_dev_ = nullptr;
  if (done_host_) {
    (void)hipHostUnregister(done_host_);
    munmap(done_host_, done_bytes_);
    if (done_owner_) shm_unlink(done_name_.c_str());
  }
  done_host_ = nullptr;
  posted_host_ = nullptr;
}

std::string AsyncPeer::handle() const {
  HandleBlob h;
  memset(&h, 0, sizeof(h));
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  X_CHECK(hipMemGetAddressRange(&base, &size, const_cast<float*>(params_)));
  X_CHECK(hipIpcGetMemHandle(&h.params, base));
  h.params_off = reinterpret_cast<const char*>(params_) - reinterpret_cast<const char*>(base);
  X_CHECK(hipIpcGetMemHandle(&h.inbox, inbox_));
  X_CHECK(hipIpcGetMemHandle(&h.flags, flags_));
  h.world = world_;
  h.rank = rank_;
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void AsyncPeer::open(const std::vector<std::string>& handles) {
  if ((int)handles.size() != world_) throw std::invalid_argument("async xgmi: one handle per rank");
  for (int q = 0; q < world_; ++q) {
    if (handles[q].size() != sizeof(HandleBlob)) throw std::invalid_argument("async xgmi: handle");
    HandleBlob h;
    memcpy(&h, handles[q].data(), sizeof(h));
    if (h.world != world_ || h.rank != q) throw std::invalid_argument("async xgmi: handle rank");
    if (q == rank_) {
      table_.params[q] = params_;
      table_.inbox[q] = inbox_;
      table_.flags[q] = flags_;
      continue;
    }
    void *p = nullptr, *ib = nullptr, *fl = nullptr;
    X_CHECK(hipIpcOpenMemHandle(&p, h.params, hipIpcMemLazyEnablePeerAccess));
    opened_[q][0] = p;
    X_CHECK(hipIpcOpenMemHandle(&ib, h.inbox, hipIpcMemLazyEnablePeerAccess));
    opened_[q][1] = ib;
    X_CHECK(hipIpcOpenMemHandle(&fl, h.flags, hipIpcMemLazyEnablePeerAccess));
    opened_[q][2] = fl;
    table_.params[q] = reinterpret_cast<float*>(reinterpret_cast<char*>(p) + h.params_off);
    table_.inbox[q] = reinterpret_cast<float*>(ib);
    table_.flags[q] = reinterpret_cast<uint32_t*>(fl);
  }
  upload_table();
  opened_ok_ = true;
}

void AsyncPeer::shard(int p, int64_t& lo, int64_t& n, int& host) const {
  if (p < 0 || p >= nps_) throw std::invalid_argument("async xgmi: PS id");
  lo = table_.shard[p].lo;
  n = table_.shard[p].n;
  host = table_.shard[p].host;
}

void AsyncPeer::upload_table() {
  X_CHECK(hipMemcpy(table_dev_, &table_, sizeof(AsyncTable), hipMemcpyHostToDevice));
}

void AsyncPeer::push_all(uint32_t epoch, float coef, hipStream_t st) {
  if (!opened_ok_ || !table_.posted)
    throw std::runtime_error("async xgmi: open(), attach_done() first");
  PushArgs a;
  memset(&a, 0, sizeof(a));
  a.world = world_;
  a.rank = rank_;
  a.nps = nps_;
  a.epoch = epoch;
  int blk = 0;
  for (int p = 0; p < nps_; ++p) {
    a.first_blk[p] = blk;
    blk += table_.shard[p].nslice;
  }
  a.first_blk[nps_] = blk;
  a.grads = grads_;
  a.coef = coef;
  if (coef != 1.f && table_.elide)
    throw std::invalid_argument("async xgmi: a scaled push needs DDL_ASYNC_ELIDE_LOCAL=0");
  hipLaunchKernelGGL(async_push_kernel, dim3(blk), dim3(256), 0, st, table_dev_, a);
  DDL_CHECK_LAUNCH();
}

void AsyncPeer::push_set(const std::vector<int>& ps, uint32_t epoch, float coef, hipStream_t st,
                         bool with_gate) {
  if (!opened_ok_ || !table_.posted)
    throw std::runtime_error("async xgmi: open(), attach_done() first");
  if (ps.empty()) return;
  if ((int)ps.size() > kAsyncMaxPs) throw std::invalid_argument("async xgmi: PS list");
  PushArgs a;
  memset(&a, 0, sizeof(a));
  a.world = world_;
  a.rank = rank_;
  a.nps = (int)ps.size();
  a.epoch = epoch;
  int blk = 0;
  for (size_t i = 0; i < ps.size(); ++i) {
    if (ps[i] < 0 || ps[i] >= nps_) throw std::invalid_argument("async xgmi: PS id");
    a.ps[i] = ps[i];
    a.first_blk[i] = blk;
    blk += table_.shard[ps[i]].nslice;
  }
  a.first_blk[ps.size()] = blk;
  a.grads = grads_;
  a.coef = coef;
  if (coef != 1.f && table_.elide)
    throw std::invalid_argument("async xgmi: a scaled push needs DDL_ASYNC_ELIDE_LOCAL=0");
  a.subset = 1;
  if (with_gate) {  // one more block: the pull gate of round `epoch`
    if (!table_.done) throw std::runtime_error("async xgmi: attach_done() first");
    a.gate = 1;
    a.gate_total = table_.shard[nps_ - 1].slice0 + table_.shard[nps_ - 1].nslice;
    a.err = err_;
    a.timeout_ticks = (long long)(timeout_s_ * 1e8);
    ++blk;
  }
  hipLaunchKernelGGL(async_push_kernel, dim3(blk), dim3(256), 0, st, table_dev_, a);
  DDL_CHECK_LAUNCH();
}

bool AsyncPeer::push_tail(const std::vector<int>& ps, uint32_t epoch, UpdTail& out) const {
  if (!opened_ok_ || !table_.posted)
    throw std::runtime_error("async xgmi: open(), attach_done() first");
  if (ps.empty() || (int)ps.size() > kTailPieces) return false;
  UpdTail t;
  t.kind = 1;
  t.epoch = epoch;
  int blk = 0;
  for (int p : ps) {
    if (p < 0 || p >= nps_) throw std::invalid_argument("async xgmi: PS id");
    const AsyncShard& S = table_.shard[p];
    UpdPiece& q = t.p[t.npieces++];
    q.g = grads_ + S.lo;
    // a shard this rank hosts itself: post only (the apply reads the gradient in place)
    q.w = table_.elide && S.host == rank_ ? nullptr
                                          : table_.inbox[S.host] + S.inbox_off + (int64_t)rank_ * S.n;
    q.n = S.n;
    q.posted = table_.posted + posted_word(p, rank_, 0);
    q.slice4 = (int)(S.slice / 4);
    q.nslice = S.nslice;
    q.blk0 = blk;
    blk += S.nslice;
  }
  t.nblocks = (blk + 7) & ~7;  // the GEMM blocks' XCD mapping (tail.h)
  out = t;
  return true;
}

void AsyncPeer::attach_done(const std::string& name, bool create) {
  // DONE[worker][ps][slice] for every rank, then the board POSTED[ps][worker][slice]
  const size_t done_words = (size_t)world_ * kAsyncMaxPs * kAsyncMaxSlices;
  const size_t bytes =
      (done_words + (size_t)kAsyncMaxPs * kXgmiMaxPeers * kAsyncMaxSlices) * sizeof(uint32_t);
  int fd = -1;
  if (create) {
    shm_unlink(name.c_str());  // stale segment of a crashed job
    fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd >= 0 && ftruncate(fd, (off_t)bytes) != 0) {
      ::close(fd);
      fd = -1;
    }
  } else {
    fd = shm_open(name.c_str(), O_RDWR, 0600);
  }
  if (fd < 0) throw std::runtime_error("async xgmi: shm_open failed: " + name);
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (p == MAP_FAILED) throw std::runtime_error("async xgmi: mmap failed: " + name);
  if (create) memset(p, 0, bytes);
  X_CHECK(hipHostRegister(p, bytes, hipHostRegisterMapped));
  void* dp = nullptr;
  X_CHECK(hipHostGetDevicePointer(&dp, p, 0));
  done_host_ = reinterpret_cast<uint32_t*>(p);
  posted_host_ = done_host_ + done_words;
  done_bytes_ = bytes;
  done_name_ = name;
  done_owner_ = create;
  table_.done = reinterpret_cast<uint32_t*>(dp);
  table_.posted = table_.done + done_words;
  upload_table();
}

bool AsyncPeer::posted(int ps, int worker, uint32_t epoch, int& next_slice) const {
  const int n = table_.shard[ps].nslice;
  while (next_slice < n) {
    const uint32_t v = __atomic_load_n(posted_host_ + posted_word(ps, worker, next_slice),
                                       __ATOMIC_ACQUIRE);
    if ((int32_t)(v - epoch) < 0) return false;
    ++next_slice;
  }
  return true;
}

bool AsyncPeer::wait_done(uint32_t epoch, double timeout_s) {
  if (!done_host_) throw std::runtime_error("async xgmi: attach_done() first");
  const auto t0 = std::chrono::steady_clock::now();
  // the words complete roughly in PS order and never go back: resume the scan where the last
  // poll stopped instead of re-reading every completed word (up to 64 x 512 of them)
  int p = 0, j = 0;
  for (int spins = 0;; ++spins) {
    while (p < nps_) {
      const uint32_t v = __atomic_load_n(
          done_host_ + ((size_t)rank_ * kAsyncMaxPs + p) * kAsyncMaxSlices + j, __ATOMIC_ACQUIRE);
      if ((int32_t)(v - epoch) < 0) break;
      if (++j == table_.shard[p].nslice) {
        j = 0;
        ++p;
      }
    }
    if (p == nps_) return true;
    if (error()) return false;
    if (spins > 256) {
      // (the worker's pull is on the step's critical path: yield for ~2 ms before sleeping —
      // a short sleep_for costs ~50 us of timer slack per wake-up)
      if ((spins & 255) == 0 &&
          std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
        return false;
      if (spins < 20000) std::this_thread::yield();
      else std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }
}

void AsyncPeer::apply(int ps, int worker, uint32_t epoch, const XgmiUpdate& u, float* ps_params,
                      hipStream_t st) {
  if (!opened_ok_ || !table_.done) throw std::runtime_error("async xgmi: open(), attach_done() first");
  if (ps < 0 || ps >= nps_ || table_.shard[ps].host != rank_)
    throw std::invalid_argument("async xgmi: apply on a PS this rank does not host");
  if (worker < 0 || worker >= world_) throw std::invalid_argument("async xgmi: worker");
  if (u.opt != 2 && !u.m) throw std::invalid_argument("async xgmi: optimizer state missing");
  if (u.opt == 0 && !u.v) throw std::invalid_argument("async xgmi: Adam needs v");
  ApplyArgs a;
  memset(&a, 0, sizeof(a));
  a.me = rank_;
  a.ps = ps;
  a.worker = worker;
  a.epoch = epoch;
  a.ps_params = ps_params;
  a.m = u.m;
  a.v = u.v;
  a.opt = u.opt;
  a.lr_t = u.lr_t;
  a.c1 = u.c1;
  a.c2 = u.c2;
  a.eps = u.eps;
  a.lr = u.lr;
  a.mu = u.mu;
  a.scale = u.scale;
  hipLaunchKernelGGL(async_apply_kernel, dim3(table_.shard[ps].nslice), dim3(256), 0, st,
                     table_dev_, a);
  DDL_CHECK_LAUNCH();
}

void AsyncPeer::gate(uint32_t epoch, hipStream_t st) {
  if (!opened_ok_ || !table_.done) throw std::runtime_error("async xgmi: open(), attach_done() first");
  GateArgs a;
  a.total = table_.shard[nps_ - 1].slice0 + table_.shard[nps_ - 1].nslice;
  a.epoch = epoch;
  a.err = err_;
  a.timeout_ticks = (long long)(timeout_s_ * 1e8);
  a.rank = rank_;
  hipLaunchKernelGGL(async_gate_kernel, dim3(1), dim3(64), 0, st, table_dev_, a);
  DDL_CHECK_LAUNCH();
}

int AsyncPeer::error() const { return err_ ? __atomic_load_n(err_, __ATOMIC_ACQUIRE) : 0; }

// ---- the PS service loop in C++ -------------------------------------------------------------------
// Scans the arrival board of this host's PS and enqueues one apply per completed push on one PS
// stream; no Python, no GIL, no hand-off thread on the critical path of any worker's round.
AsyncService::AsyncService(AsyncPeer* peer, int world, int device,
                           const std::vector<AsyncPsState>& ps, int opt, float lr, float b1,
                           float b2, float eps, float mu, float scale, uint32_t epoch0,
                           bool provenance)
    : peer_(peer), world_(world), device_(device), ps_(ps), opt_(opt), lr_(lr), b1_(b1),
      b2_(b2), eps_(eps), mu_(mu), scale_(scale), keep_prov_(provenance) {
  if (world < 1 || world > kXgmiMaxPeers) throw std::invalid_argument("async service: world");
  for (const auto& s : ps)
    if (s.ps < 0 || s.ps >= peer->num_ps() || !s.params || !s.m || (opt == 0 && !s.v))
      throw std::invalid_argument("async service: PS state");
  epoch_.assign((size_t)world * kAsyncMaxPs, epoch0);
  if ((int)ps.size() > kAsyncMaxPs) throw std::invalid_argument("async service: too many PS");
}

AsyncService::~AsyncService() {
  if (th_.joinable()) th_.join();
  if (stream_) {
    (void)hipStreamSynchronize(stream_);
    (void)hipStreamDestroy(stream_);
  }
}

void AsyncService::start(int64_t expected) {
  if (th_.joinable()) throw std::runtime_error("async service already running");
  X_CHECK(hipSetDevice(device_));
  // HIGH priority: HIP pools hardware queues per priority, so the applies never share a queue
  // with the compute stream, where the worker's GPU-side pull gate may be waiting for them
  // (async_runner.hip)
  // (DDL_ASYNC_PS_PRIORITY=low: the least priority instead — also a pool of its own, so the
  // deadlock argument holds; the dispatcher then prefers the compute stream's waves over the
  // overlapped applies)
  int lo = 0, hi = 0;
  X_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  const char* pp = getenv("DDL_ASYNC_PS_PRIORITY");
  const int prio = pp && std::string(pp) == "low" ? lo : hi;
  if (!stream_) X_CHECK(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, prio));
  expected_ = expected;
  th_ = std::thread([this] { run(); });
}

void AsyncService::serve(AsyncPsState& st, int w) {
  TraceRange apply_range("ddl.async.ps.apply");
  const int p = st.ps;
  std::lock_guard<std::mutex> hold(pause_mu_);  // pause(): no apply while a snapshot is taken
  const uint32_t e = ++epoch_[(size_t)w * kAsyncMaxPs + p];
  // one apply_gradients of this PS per arrival
  const int64_t t = __atomic_add_fetch(&st.t, 1, __ATOMIC_ACQ_REL);
  XgmiUpdate u;
  u.opt = opt_;
  u.m = st.m;
  u.v = st.v;
  // TF1 Adam: lr_t = lr * sqrt(1 - beta2^t) / (1 - beta1^t) (ops/adam.py adam_coeffs)
  u.lr_t = (float)((double)lr_ * std::sqrt(1.0 - std::pow((double)b2_, (double)t)) /
                   (1.0 - std::pow((double)b1_, (double)t)));
  u.c1 = 1.f - b1_;
  u.c2 = 1.f - b2_;
  u.eps = eps_;
  u.lr = lr_;
  u.mu = mu_;
  u.scale = scale_;
  peer_->apply(p, w, e, u, st.params, stream_);
  if (keep_prov_) prov_.push_back({(int64_t)w, (int64_t)p, (int64_t)e, t});
  served_.fetch_add(1);
}

void AsyncService::run() {
  try {
    X_CHECK(hipSetDevice(device_));
    const int np = (int)ps_.size();
    const int pairs = np * world_;
    // per (hosted PS, worker): the first slice of the next round not yet seen posted
    std::vector<int> seen((size_t)pairs, 0);
    int start = 0;  // round-robin: the scan resumes after the pair served last
    int64_t k = 0;
    auto idle_since = std::chrono::steady_clock::now();
    TraceRange wait_range("ddl.async.ps.wait_arrival");
    for (int spins = 0; k < expected_;) {
      int hit = -1;
      for (int i = 0; i < pairs && hit < 0; ++i) {
        const int q = (start + i) % pairs;
        AsyncPsState& st = ps_[q / world_];
        const int w = q % world_;
        const uint32_t next = epoch_[(size_t)w * kAsyncMaxPs + st.ps] + 1;
        if (peer_->posted(st.ps, w, next, seen[q])) hit = q;
      }
      if (hit >= 0) {
        serve(ps_[hit / world_], hit % world_);
        seen[hit] = 0;
        start = hit + 1;
        ++k;
        spins = 0;
        idle_since = std::chrono::steady_clock::now();
        if (const int err = peer_->error())
          throw std::runtime_error("async PS: kernel wait timed out (code " +
                                   std::to_string(err) + ")");
        continue;
      }
      if (peer_->error())
        throw std::runtime_error("async PS: kernel wait timed out (code " +
                                 std::to_string(peer_->error()) + ")");
      // an arrival is on some worker's critical path: yield (not sleep) for ~2 ms first
      if (++spins < 20000) {
        if (spins > 64) std::this_thread::yield();
      } else {
        std::this_thread::sleep_for(std::chrono::microseconds(20));
      }
      if ((spins & 255) == 0 &&
          std::chrono::duration<double>(std::chrono::steady_clock::now() - idle_since).count() >
              600.0)
        throw std::runtime_error("async PS: no arrival within 600 s");
    }
    X_CHECK(hipStreamSynchronize(stream_));
  } catch (const std::exception& ex) {
    error_ = ex.what();
  }
}

void AsyncService::join() {
  if (th_.joinable()) th_.join();
  if (!error_.empty()) throw std::runtime_error(error_);
}

void AsyncService::pause() {
  pause_mu_.lock();
  if (stream_) {
    const hipError_t e = hipStreamSynchronize(stream_);
    if (e != hipSuccess) {
      pause_mu_.unlock();
      throw std::runtime_error(std::string("async service: pause: ") + hipGetErrorString(e));
    }
  }
}

void AsyncService::resume() {
  pause_mu_.unlock();
}

int64_t AsyncService::t(int ps) const {
  for (size_t i = 0; i < ps_.size(); ++i)  // lock-free: also read while paused
    if (ps_[i].ps == ps)
      return __atomic_load_n(&ps_[i].t, __ATOMIC_ACQUIRE);
  throw std::invalid_argument("async service: PS not hosted here");
}

int64_t AsyncService::served() const {
  return served_.load();
}

}  // namespace ddl

