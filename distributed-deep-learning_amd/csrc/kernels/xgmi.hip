// Parameter-server exchange over xGMI peer memory: one kernel per gradient bucket does the
// whole synchronous PS round trip of SURVEY.md §2.7 for the byte-equal flat plan — push the
// gradient chunks to their owners, sum at the owner, Adam on the owner's shard, push the new
// parameters back to every worker — with remote stores into IPC-mapped peer buffers instead
// of RCCL's reduce-scatter + all-gather (two collective launches, a ring pass each).
//
// Reference behaviour being replaced: every worker Sends each gradient tensor to the owning
// PS, the PS sums the W arrivals with NumPy and runs ApplyAdam, then Sends the parameters back
// (mnist_sync_sharding/worker.py:30-37,88-94; parameter_server.py:76-82,108-126).
//
// Why a kernel of our own (MI355X): the 8 GPUs of a node are a full xGMI mesh (7 links per GPU),
// so the owner of chunk r can receive its W-1 gradient pieces on W-1 different links at once,
// and a store to a peer's HBM is posted (no round trip).  One launch per bucket with a few dozen
// workgroups leaves the CUs to the backward GEMMs it overlaps with; all traffic is writes.
//
// Protocol (per bucket b, step epoch e; workgroup j owns slice j of every rank's chunk):
//   phase 1  for every owner r != me: store grads[b][chunk r][slice j] -> inbox_r[b][me][slice j]
//            (write-through, system scope), drain, then ARRIVE_r[b][me][j] = e
//   phase 2  wait ARRIVE_me[b][q][j] >= e for every peer q; sum the W contributions in rank order
//            (deterministic), optimizer update of my chunk's slice, store the new parameters to
//            EVERY rank's parameter buffer (self included, write-through), drain, DONE_q[b][me][j] = e
//   final    (the step's last bucket, on the compute stream) wait DONE_me[b'][q][*] >= e for every
//            bucket, rank and slice: when the kernel ends, every parameter of this step has
//            landed and the next forward (a later kernel: L2 invalidated at its start) reads them.
// Buffer reuse is safe by construction: a rank overwrites an inbox slot (step e+1 backward) only
// after its step e+1 forward, i.e. after the final wait saw every owner's DONE of step e, which
// each owner sets after reading that slot; an owner writes a peer's parameters of bucket b only
// after that peer's ARRIVE for b, i.e. after its backward segment b, the last reader of them.
// Flags live in uncached device memory, each has ONE writer and is only stored (never
// read-modify-written) and polled, all with system-scope atomic loads/stores; payload
// stores carry sc0|sc1 (system write-through) and every storing wave drains (vmcnt(0)) before
// the workgroup barrier that precedes the flag store.  Every wait is bounded: on timeout the
// kernel records an error word in host memory and runs to completion (no GPU hang); the host
// raises at the next step.
#include <stdlib.h>
#include <string.h>

#include <stdexcept>
#include <string>

#include "api.h"
#include "common.h"
#include "xgmi_dev.h"

namespace ddl {

namespace {

constexpr unsigned kSys = 1u | 16u;  // buffer-op cache policy: sc0 | sc1 = system coherent

DDL_DEV void st4_sys(brsrc_t r, int byte_off, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(
      __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v), r, byte_off, 0,
      kSys);
}
DDL_DEV float4 ld4_sys(brsrc_t r, int byte_off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, kSys);
  return *reinterpret_cast<float4*>(&v);
}
DDL_DEV void drain_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// the flag protocol's device side lives in xgmi_dev.h
DDL_DEV void flag_store(uint32_t* f, uint32_t v) { xg_flag_store(f, v); }
DDL_DEV int arrive_idx(int b, int src, int j) { return xg_arrive_idx(b, src, j); }
DDL_DEV int done_idx(int b, int src, int j) { return xg_done_idx(b, src, j); }
DDL_DEV bool wait_ge(const uint32_t* f, uint32_t target, long long deadline, int* err, int code) {
  return xg_wait_ge(f, target, deadline, err, code);
}

// The READY gate ahead of this kernel timed out (its gradients may be incomplete): publish
// nothing, record error 6 (the peers' waits then time out as well and every host raises).
DDL_DEV bool gate_failed(const XgmiLaunch& a) {
  if (!a.gate_err || __hip_atomic_load(a.gate_err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0)
    return false;
  if (threadIdx.x == 0) __hip_atomic_store(a.err, 6, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return true;
}

DDL_DEV float4 scale4(float4 x, float a) {
  x.x *= a; x.y *= a; x.z *= a; x.w *= a;
  return x;
}

// ---- debug checksums (DDL_XGMI_CHECK=1, the sync analogue of async --check-provenance) ------
// The pusher of slice j of bucket b stores, next to its ARRIVE word at the owner, the wrapping
// sum of the 32-bit patterns of exactly the floats it pushed; the owner recomputes that sum over
// what it reads from its inbox before it uses the slice and records error code 3 (and skips the
// update) on a mismatch — a stale or torn inbox read is caught where it happens, per (bucket,
// source, step), instead of as a parameter divergence steps later.
// The replicated bucket's checksum words carry the step parity like its inbox slots: a peer may
// publish step e+1's checksum (its parity-(e+1) slot) while this rank still checks step e's —
// with one word per (bucket, source, slice) the check of step e read step e+1's sum (error 3
// in the W = 8 one-card test, where ranks drift a whole step apart).  Owner buckets need no
// parity: a pusher writes an owner's inbox again only after that owner's DONE, i.e. after its
// check.
DDL_DEV int ck_idx(int b, int src, int j, int par = 0) {
  return (2 + par) * kXgmiMaxBuckets * kXgmiMaxPeers * kXgmiMaxSlices + arrive_idx(b, src, j);
}

DDL_DEV uint32_t bits4(float4 v) {
  return __float_as_uint(v.x) + __float_as_uint(v.y) + __float_as_uint(v.z) + __float_as_uint(v.w);
}
// sum over the 256 threads of the workgroup (every thread gets it); red: 4 words of LDS
DDL_DEV uint32_t block_sum(uint32_t v, uint32_t* red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const uint32_t t = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return t;
}

// owner-side check of one source's piece [n4 float4 at byte offset off of `in`]: false (error
// code 3 recorded) when it differs from the checksum the source published
DDL_DEV bool check_piece(brsrc_t in, int off, int n4, const uint32_t* ck, int* err,
                         uint32_t* red) {
  uint32_t c = 0;
  for (int i = threadIdx.x; i < n4; i += 256) c += bits4(ld4_sys(in, off + i * 16));
  const uint32_t got = block_sum(c, red);
  const uint32_t want = __hip_atomic_load(ck, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (got == want) return true;
  if (threadIdx.x == 0) __hip_atomic_store(err, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return false;
}

// The final wait of a step (xgmi_dev.h xg_final_wait) over every thread of the launch.
DDL_DEV void final_wait(const XgmiLaunch& a, const uint32_t* myflags, int W, long long deadline) {
  xg_final_wait(a, a.epoch, myflags, W, deadline, blockIdx.x * 256 + threadIdx.x,
                gridDim.x * 256);
}

// The owner-side optimizer update of one float4 (TF1 Adam, momentum, or the self-test's
// w := g), shared by the owner kernel and the replicated kernel so both give the same bits.
DDL_DEV void update4(const XgmiLaunch& a, float4& w, float4 g, float4* m4, float4* v4, int i) {
  if (a.opt == 0) {  // TF1 Adam (optim.hip form)
    float4 M = m4[i], V = v4[i];
    adam1(w.x, g.x * a.scale, M.x, V.x, a.lr_t, a.c1, a.c2, a.eps);
    adam1(w.y, g.y * a.scale, M.y, V.y, a.lr_t, a.c1, a.c2, a.eps);
    adam1(w.z, g.z * a.scale, M.z, V.z, a.lr_t, a.c1, a.c2, a.eps);
    adam1(w.w, g.w * a.scale, M.w, V.w, a.lr_t, a.c1, a.c2, a.eps);
    m4[i] = M; v4[i] = V;
  } else if (a.opt == 1) {  // momentum SGD (optim.hip momentum_kernel form)
    float4 M = m4[i];
    momentum1(w.x, g.x, M.x, a.lr, a.mu, a.scale);
    momentum1(w.y, g.y, M.y, a.lr, a.mu, a.scale);
    momentum1(w.z, g.z, M.z, a.lr, a.mu, a.scale);
    momentum1(w.w, g.w, M.w, a.lr, a.mu, a.scale);
    m4[i] = M;
  } else {  // self-test: parameters := the summed gradient
    w = g;
  }
}

// WT = world size when instantiated for it (loops over ranks fully unrolled: all of an
// element's remote loads / stores are in flight together), 0 = any world size.
template <int WT>
__global__ void __launch_bounds__(256) xgmi_ps_kernel(XgmiTable T, XgmiLaunch a) {
  if (gate_failed(a)) return;
  constexpr int NQ = WT ? WT : kXgmiMaxPeers;
  const int j = blockIdx.x, tid = threadIdx.x;
  const int W = WT ? WT : a.world, me = a.rank, b = a.bucket;
  const long long deadline = wall_clock64() + a.timeout_ticks;
  const int64_t s0 = (int64_t)j * a.slice;
  const int64_t s1 = s0 + a.slice < a.c ? s0 + a.slice : a.c;
  const int n4 = s0 < s1 ? (int)((s1 - s0) >> 2) : 0;
  uint32_t* myflags = T.flags[me];
  __shared__ uint32_t red[4];
  __shared__ int arrived;

  // ---- phase 1: push my gradient pieces to their owners.  Per element index every owner's
  // load is issued before the first store; workgroup j starts at a different owner so the
  // W-1 links carry traffic at once.
  uint32_t cs[NQ - 1];
#pragma unroll
  for (int k = 0; k < NQ - 1; ++k) cs[k] = 0;
  for (int i = tid; i < n4; i += 256) {
    float4 x[NQ - 1];
#pragma unroll
    for (int k = 0; k < NQ - 1; ++k) {
      if (k < W - 1) {
        const int r = (me + 1 + (k + j) % (W - 1)) % W;
        x[k] = reinterpret_cast<const float4*>(a.grads + a.lo + r * a.c + s0)[i];
      }
    }
#pragma unroll
    for (int k = 0; k < NQ - 1; ++k) {
      if (k < W - 1) {
        const int r = (me + 1 + (k + j) % (W - 1)) % W;
        const brsrc_t dst = make_rsrc(T.inbox[r] + a.inbox_off + (int64_t)me * a.c + s0,
                                      (uint32_t)n4 * 16u);
        const float4 v = a.coef != 1.f ? scale4(x[k], a.coef) : x[k];
        st4_sys(dst, i * 16, v);
        if (a.check) cs[k] += bits4(v);
      }
    }
  }
  if (a.check) {  // publish each owner's checksum before the ARRIVE word (same drain covers it)
#pragma unroll
    for (int k = 0; k < NQ - 1; ++k) {
      if (k < W - 1) {
        const uint32_t t = block_sum(cs[k], red);
        const int r = (me + 1 + (k + j) % (W - 1)) % W;
        if (tid == 0)
          __hip_atomic_store(T.flags[r] + ck_idx(b, me, j), t, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
  drain_vm();
  __syncthreads();
  if (tid < W && tid != me) flag_store(T.flags[tid] + arrive_idx(b, me, j), a.epoch);

  // ---- phase 2: every peer's piece of my slice has arrived (one parallel poll).  If any wait
  // failed (timeout, or another workgroup's recorded error) the slice is NOT updated: summing a
  // stale inbox would advance m / v and push wrong parameters into every replica.  DONE is still
  // stored, so the peers do not wait out their own timeouts; the host raises on the error word.
  if (tid == 0) arrived = 1;
  __syncthreads();
  if (tid < W && tid != me &&
      !wait_ge(myflags + arrive_idx(b, tid, j), a.epoch, deadline, a.err, 1))
    arrived = 0;  // benign race: every writer stores 0
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // keep the loads below the poll

  const brsrc_t inbox = make_rsrc(T.inbox[me] + a.inbox_off, (uint32_t)(W * a.c * 4));
  if (a.check && arrived) {
    bool ok = true;
    for (int q = 0; q < W; ++q)
      if (q != me)
        ok &= check_piece(inbox, (int)(((int64_t)q * a.c + s0) * 4), n4,
                          myflags + ck_idx(b, q, j), a.err, red);
    if (!ok && tid == 0) arrived = 0;
    __syncthreads();
  }
  const int n4u = arrived ? n4 : 0;

  const float4* own = reinterpret_cast<const float4*>(a.grads + a.lo + me * a.c + s0);
  float4* m4 = reinterpret_cast<float4*>(a.m + s0);
  float4* v4 = a.v ? reinterpret_cast<float4*>(a.v + s0) : nullptr;
  float4* w4 = reinterpret_cast<float4*>(T.params[me] + a.lo + me * a.c + s0);
  for (int i = tid; i < n4u; i += 256) {
    float4 x[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      if (q < W)
        x[q] = q == me ? (a.coef != 1.f ? scale4(own[i], a.coef) : own[i])
                       : ld4_sys(inbox, (int)(((int64_t)q * a.c + s0) * 4) + i * 16);
    float4 w = w4[i];
    float4 g = f4zero();
#pragma unroll
    for (int q = 0; q < NQ; ++q)  // rank order: the same sum on every run and every rank count
      if (q < W) { g.x += x[q].x; g.y += x[q].y; g.z += x[q].z; g.w += x[q].w; }
    update4(a, w, g, m4, v4, i);
    // every rank's copy, this one included: write-through, so a later kernel of any rank
    // (other XCD, other GPU) reads it from memory even while this kernel is still running
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      if (k < W) {
        const int q = (me + k + j) % W;
        const brsrc_t dst = make_rsrc(T.params[q] + a.lo + me * a.c + s0, (uint32_t)n4 * 16u);
        st4_sys(dst, i * 16, w);
      }
    }
  }
  drain_vm();
  __syncthreads();
  if (tid < W) flag_store(T.flags[tid] + done_idx(b, me, j), a.epoch);

  // ---- final wait: every bucket's new parameters from every owner have landed here
  if (a.final_wait) final_wait(a, myflags, W, deadline);
}

// The step's LAST bucket, replicated: nothing overlaps its exchange — it is
// complete only after the final backward launch — so instead of push chunk -> owner update ->
// push parameters -> DONE (two cross-GPU hops on the critical path), every rank pushes the
// WHOLE bucket gradient to every peer (W-1 links at once, 208 KB each for conv1+conv2), sums the
// W contributions in rank order and runs the update itself on replicated optimizer state, then
// stores only its own parameters.  One hop.  The inbox has two parity slots per source: a peer
// writes slot (e+1)&1 of step e+1 while this rank may still read slot e&1; it can write slot e&1
// again only at step e+2, after its final wait of step e+1 saw this rank's DONE of every owner
// bucket at e+1 — issued after this rank's step-e+1 forward, i.e. after this kernel of step e.
// This needs the replicated bucket to be the one the last backward segment completes (conv1 +
// conv2, launched on the compute stream): parallel/native_exchange.py last_segment_bucket.
template <int WT>
__global__ void __launch_bounds__(256) xgmi_repl_kernel(XgmiTable T, XgmiLaunch a) {
  if (gate_failed(a)) return;
  constexpr int NQ = WT ? WT : kXgmiMaxPeers;
  const int j = blockIdx.x, tid = threadIdx.x;
  const int W = WT ? WT : a.world, me = a.rank, b = a.bucket;
  const long long deadline = wall_clock64() + a.timeout_ticks;
  const int64_t n = a.c;  // replicated: the whole bucket
  const int64_t s0 = (int64_t)j * a.slice;
  const int64_t s1 = s0 + a.slice < n ? s0 + a.slice : n;
  const int n4 = s0 < s1 ? (int)((s1 - s0) >> 2) : 0;
  const int par = (int)(a.epoch & 1u);
  uint32_t* myflags = T.flags[me];
  __shared__ uint32_t red[4];
  __shared__ int arrived;
  const float4* own = reinterpret_cast<const float4*>(a.grads + a.lo + s0);
  // slot (par, src) of rank r's replicated inbox, this slice
  auto slot = [&](int r, int src) {
    return make_rsrc(T.inbox[r] + a.inbox_off + ((int64_t)par * W + src) * a.rslot + s0,
                     (uint32_t)n4 * 16u);
  };

  // ---- phase 1: my whole slice to every peer
  uint32_t cs = 0;
  for (int i = tid; i < n4; i += 256) {
    float4 x = own[i];
    if (a.coef != 1.f) x = scale4(x, a.coef);
    if (a.check) cs += bits4(x);
#pragma unroll
    for (int k = 0; k < NQ - 1; ++k)
      if (k < W - 1) st4_sys(slot((me + 1 + (k + j) % (W - 1)) % W, me), i * 16, x);
  }
  if (a.check) {
    const uint32_t t = block_sum(cs, red);
    if (tid < W && tid != me)
      __hip_atomic_store(T.flags[tid] + ck_idx(b, me, j, par), t, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
  drain_vm();
  __syncthreads();
  if (tid < W && tid != me) flag_store(T.flags[tid] + arrive_idx(b, me, j), a.epoch);

  // ---- phase 2: all peers' slices are here (failed wait: no update, as in xgmi_ps_kernel)
  if (tid == 0) arrived = 1;
  __syncthreads();
  if (tid < W && tid != me &&
      !wait_ge(myflags + arrive_idx(b, tid, j), a.epoch, deadline, a.err, 1))
    arrived = 0;
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  if (a.check && arrived) {
    bool ok = true;
    for (int q = 0; q < W; ++q)
      if (q != me)
        ok &= check_piece(slot(me, q), 0, n4, myflags + ck_idx(b, q, j, par), a.err, red);
    if (!ok && tid == 0) arrived = 0;
    __syncthreads();
  }
  const int n4u = arrived ? n4 : 0;
  float4* m4 = reinterpret_cast<float4*>(a.m + s0);
  float4* v4 = a.v ? reinterpret_cast<float4*>(a.v + s0) : nullptr;
  float4* w4 = reinterpret_cast<float4*>(T.params[me] + a.lo + s0);
  for (int i = tid; i < n4u; i += 256) {
    float4 x[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      if (q < W)
        x[q] = q == me ? (a.coef != 1.f ? scale4(own[i], a.coef) : own[i])
                       : ld4_sys(slot(me, q), i * 16);
    float4 g = f4zero();
#pragma unroll
    for (int q = 0; q < NQ; ++q)  // rank order, as the owner kernel: identical bits
      if (q < W) { g.x += x[q].x; g.y += x[q].y; g.z += x[q].z; g.w += x[q].w; }
    float4 w = w4[i];
    update4(a, w, g, m4, v4, i);
    w4[i] = w;  // this rank's copy only (the next forward is a later kernel of this stream)
  }
  if (a.final_wait) final_wait(a, myflags, W, deadline);
}

// One OWNER bucket: a tensor-granular plan's exchange unit — the ranges of
// one PS's tensors that backward segment s completes — with a single owner, the rank hosting
// that PS (reference: every worker Sends the PS's tensors to it, the PS sums the W arrivals,
// applies Adam and Sends the parameters back, mnist_sync/parameter_server.py:52-69,
// mnist_sync_sharding/parameter_server.py:108-126).  Workgroup j owns slice j of the unit; a
// slice lies inside one run (plan-buffer range), so its gradient, parameters and optimizer state
// are each one contiguous span.
//   every rank but the owner: push my slice to the owner's inbox slot [me], drain, ARRIVE = e;
//   the owner: wait for every peer's ARRIVE, sum the W contributions in rank order, update with
//   the PS's state, store the parameters to EVERY rank (write-through), drain, DONE_q[owner] = e.
// A non-owner's workgroups end after their push (unless they carry the step's final wait), so an
// unbalanced plan (contiguous at W = 8: PS 7 owns 59 % of the bytes) loads only its owner's CUs
// and links.  Same flags, bounds, error words and reuse argument as xgmi_ps_kernel: a rank
// rewrites the owner's inbox slot only after its next forward, i.e. after its final wait saw the
// owner's DONE, which the owner sets after reading that slot.
template <int WT>
__global__ void __launch_bounds__(256) xgmi_owner_kernel(XgmiTable T, XgmiLaunch a) {
  if (gate_failed(a)) return;
  constexpr int NQ = WT ? WT : kXgmiMaxPeers;
  const int j = blockIdx.x, tid = threadIdx.x;
  const int W = WT ? WT : a.world, me = a.rank, b = a.bucket, own = a.owner;
  const long long deadline = wall_clock64() + a.timeout_ticks;
  int r = 0;
#pragma unroll
  for (int k = 1; k < kXgmiMaxRuns; ++k)
    if (k < a.nruns && j >= a.run_sl0[k]) r = k;
  const int64_t s0 = (int64_t)(j - a.run_sl0[r]) * a.run_slice[r];
  const int64_t s1 = s0 + a.run_slice[r] < a.run_n[r] ? s0 + a.run_slice[r] : a.run_n[r];
  const int n4 = s0 < s1 ? (int)((s1 - s0) >> 2) : 0;
  const int64_t lo = a.run_lo[r] + s0;    // plan-buffer offset of the slice
  const int64_t vo = a.run_voff[r] + s0;  // its offset in the unit's inbox slot
  uint32_t* myflags = T.flags[me];
  __shared__ uint32_t red[4];
  __shared__ int arrived;
  const float4* mine = reinterpret_cast<const float4*>(a.grads + lo);

  if (me != own) {
    const brsrc_t dst = make_rsrc(T.inbox[own] + a.inbox_off + (int64_t)me * a.c + vo,
                                  (uint32_t)n4 * 16u);
    uint32_t cs = 0;
    for (int i = tid; i < n4; i += 256) {
      const float4 x = mine[i];
      const float4 v = a.coef != 1.f ? scale4(x, a.coef) : x;
      st4_sys(dst, i * 16, v);
      if (a.check) cs += bits4(v);
    }
    if (a.check) {  // the slice's checksum at the owner, before the ARRIVE word (same drain)
      const uint32_t t = block_sum(cs, red);
      if (tid == 0)
        __hip_atomic_store(T.flags[own] + ck_idx(b, me, j), t, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
    drain_vm();
    __syncthreads();
    if (tid == 0) flag_store(T.flags[own] + arrive_idx(b, me, j), a.epoch);
    if (a.final_wait) final_wait(a, myflags, W, deadline);
    return;
  }

  if (tid == 0) arrived = 1;
  __syncthreads();
  if (tid < W && tid != me &&
      !wait_ge(myflags + arrive_idx(b, tid, j), a.epoch, deadline, a.err, 1))
    arrived = 0;  // (no update on a failed wait: see xgmi_ps_kernel)
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  const brsrc_t inbox = make_rsrc(T.inbox[me] + a.inbox_off, (uint32_t)(W * a.c * 4));
  if (a.check && arrived) {  // every pusher's slice against its published checksum
    bool ok = true;
    for (int q = 0; q < W; ++q)
      if (q != me)
        ok &= check_piece(inbox, (int)(((int64_t)q * a.c + vo) * 4), n4,
                          myflags + ck_idx(b, q, j), a.err, red);
    if (!ok && tid == 0) arrived = 0;
    __syncthreads();
  }
  const int n4u = arrived ? n4 : 0;
  float4* m4 = a.m ? reinterpret_cast<float4*>(a.m + a.run_soff[r] + s0) : nullptr;
  float4* v4 = a.v ? reinterpret_cast<float4*>(a.v + a.run_soff[r] + s0) : nullptr;
  float4* w4 = reinterpret_cast<float4*>(T.params[me] + lo);
  for (int i = tid; i < n4u; i += 256) {
    float4 x[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      if (q < W)
        x[q] = q == me ? (a.coef != 1.f ? scale4(mine[i], a.coef) : mine[i])
                       : ld4_sys(inbox, (int)(((int64_t)q * a.c + vo) * 4) + i * 16);
    float4 w = w4[i];
    float4 g = f4zero();
#pragma unroll
    for (int q = 0; q < NQ; ++q)  // rank order, as the RCCL reduce and xgmi_ps_kernel
      if (q < W) { g.x += x[q].x; g.y += x[q].y; g.z += x[q].z; g.w += x[q].w; }
    update4(a, w, g, m4, v4, i);
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      if (k < W) {
        const int q = (me + k + j) % W;
        st4_sys(make_rsrc(T.params[q] + lo, (uint32_t)n4 * 16u), i * 16, w);
      }
    }
  }
  drain_vm();
  __syncthreads();
  if (tid < W) flag_store(T.flags[tid] + done_idx(b, me, j), a.epoch);
  if (a.final_wait) final_wait(a, myflags, W, deadline);
}

#define X_CHECK(x)                                                                        \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess)                                                                 \
      throw std::runtime_error(std::string("xgmi: ") + #x + ": " + hipGetErrorString(e_)); \
  } while (0)

struct HandleBlob {  // what one rank publishes (exchanged as bytes over the default group)
  hipIpcMemHandle_t params, inbox, flags;
  int64_t params_off;
  int32_t world, rank;
};

}  // namespace

static std::vector<XgmiBucketSpec> equal_specs(
    const std::vector<std::pair<int64_t, int64_t>>& buckets) {
  std::vector<XgmiBucketSpec> v;
  for (const auto& b : buckets) {
    XgmiBucketSpec s;
    s.runs.push_back(b);
    v.push_back(s);
  }
  return v;
}

PeerExchange::PeerExchange(float* params, const float* grads, int64_t total, int world, int rank,
                           const std::vector<std::pair<int64_t, int64_t>>& buckets, int max_slices,
                           int repl_bucket)
    : PeerExchange(params, grads, total, world, rank, equal_specs(buckets), max_slices,
                   repl_bucket) {}

PeerExchange::PeerExchange(float* params, const float* grads, int64_t total, int world, int rank,
                           const std::vector<XgmiBucketSpec>& buckets, int max_slices,
                           int repl_bucket)
    : params_(params), grads_(grads), total_(total), world_(world), rank_(rank),
      repl_(repl_bucket) {
  if (world < 1 || world > kXgmiMaxPeers) throw std::invalid_argument("xgmi: world out of range");
  if (rank < 0 || rank >= world) throw std::invalid_argument("xgmi: rank out of range");
  if (buckets.empty() || (int)buckets.size() > kXgmiMaxBuckets)
    throw std::invalid_argument("xgmi: 1..32 buckets");
  if (max_slices < 1 || max_slices > kXgmiMaxSlices)
    throw std::invalid_argument("xgmi: max_slices out of range");
  if (reinterpret_cast<uintptr_t>(params) % 16 || reinterpret_cast<uintptr_t>(grads) % 16)
    throw std::invalid_argument("xgmi: buffers must be 16-B aligned");
  if (repl_bucket >= (int)buckets.size()) throw std::invalid_argument("xgmi: replicated bucket");
  init(buckets, max_slices);
}

void PeerExchange::init(const std::vector<XgmiBucketSpec>& buckets, int max_slices) {
  const int world = world_;
  int64_t inbox = 0;
  for (size_t bi = 0; bi < buckets.size(); ++bi) {
    const XgmiBucketSpec& sp = buckets[bi];
    const bool repl = (int)bi == repl_;
    Bucket B;
    B.owner = sp.owner;
    B.inbox_off = inbox;
    if (sp.owner >= 0) {
      // owner bucket: the runs concatenated; each run sliced on its own (a slice never crosses
      // a run), >= 1024 elements per slice, at most max_slices slices over the whole unit
      if (sp.owner >= world) throw std::invalid_argument("xgmi: bucket owner out of range");
      if (repl) throw std::invalid_argument("xgmi: an owner bucket cannot be replicated");
      if (sp.runs.empty() || (int)sp.runs.size() > kXgmiMaxRuns ||
          sp.state_offs.size() != sp.runs.size())
        throw std::invalid_argument("xgmi: owner bucket needs 1..8 runs with state offsets");
      int64_t n = 0;
      for (size_t r = 0; r < sp.runs.size(); ++r) {
        const int64_t lo = sp.runs[r].first, hi = sp.runs[r].second;
        if (lo < 0 || hi > total_ || hi <= lo || (hi - lo) % 4 || lo % 4 || sp.state_offs[r] % 4)
          throw std::invalid_argument("xgmi: owner-bucket run out of range or not 16-B shaped");
        n += hi - lo;
      }
      int64_t ns = (n + 1023) / 1024;
      if (ns > max_slices) ns = max_slices;
      if (ns < (int64_t)sp.runs.size()) ns = (int64_t)sp.runs.size();
      const int64_t per = ((n + ns - 1) / ns + 3) & ~(int64_t)3;
      int sl = 0;
      int64_t voff = 0;
      for (size_t r = 0; r < sp.runs.size(); ++r) {
        const int64_t rn = sp.runs[r].second - sp.runs[r].first;
        B.run_lo.push_back(sp.runs[r].first);
        B.run_n.push_back(rn);
        B.run_soff.push_back(sp.state_offs[r]);
        B.run_voff.push_back(voff);
        B.run_slice.push_back(per);
        B.run_sl0.push_back(sl);
        sl += (int)((rn + per - 1) / per);
        voff += rn;
      }
      B.run_sl0.push_back(sl);
      if (sl > kXgmiMaxSlices) throw std::invalid_argument("xgmi: owner bucket has too many slices");
      B.lo = sp.runs[0].first;
      B.c = n;
      B.slice = per;
      B.nslice = sl;
      if (n * 4 * world > 0x7fffffffLL) throw std::invalid_argument("xgmi: bucket too large");
      inbox += n * world;
      bk_.push_back(B);
      continue;
    }
    if (sp.runs.size() != 1) throw std::invalid_argument("xgmi: equal-chunk bucket needs one range");
    const int64_t lo = sp.runs[0].first, hi = sp.runs[0].second;
    if (lo < 0 || hi > total_ || hi <= lo) throw std::invalid_argument("xgmi: bucket out of range");
    if ((hi - lo) % (repl ? 4 : 4 * world))
      throw std::invalid_argument("xgmi: bucket not divisible by 4W (replicated: by 4)");
    B.lo = lo;
    // owner buckets: this rank's chunk; the replicated bucket: all of it
    B.c = repl ? hi - lo : (hi - lo) / world;
    // >= 1024 elements (4 KB) per workgroup slice, at most max_slices workgroups
    int64_t ns = (B.c + 1023) / 1024;
    if (ns > max_slices) ns = max_slices;
    if (ns < 1) ns = 1;
    B.slice = ((B.c + ns - 1) / ns + 3) & ~(int64_t)3;
    B.nslice = (int)((B.c + B.slice - 1) / B.slice);
    B.slot = B.c;
    if (B.slot * 4 * world * (repl ? 2 : 1) > 0x7fffffffLL)
      throw std::invalid_argument("xgmi: bucket too large");
    inbox += B.slot * world * (repl ? 2 : 1);  // replicated: two parity slots per source
    bk_.push_back(B);
  }
  inbox_elems_ = inbox;
  X_CHECK(hipMalloc(&inbox_, inbox_elems_ * sizeof(float)));
  X_CHECK(hipMemset(inbox_, 0, inbox_elems_ * sizeof(float)));
  // ARRIVE, DONE and (check mode) checksum words, the replicated bucket's in two parities
  flag_bytes_ = 4ull * kXgmiMaxBuckets * kXgmiMaxPeers * kXgmiMaxSlices * sizeof(uint32_t);
  X_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&flags_), flag_bytes_,
                                hipDeviceMallocUncached));
  X_CHECK(hipMemset(flags_, 0, flag_bytes_));
  X_CHECK(hipHostMalloc(reinterpret_cast<void**>(&err_), 64, hipHostMallocDefault));
  memset(err_, 0, 64);
  X_CHECK(hipDeviceSynchronize());
  const char* t = getenv("DDL_XGMI_TIMEOUT_S");
  timeout_s_ = t ? atof(t) : 20.0;  // a healthy wait takes microseconds
  const char* ck = getenv("DDL_XGMI_CHECK");
  check_ = ck && ck[0] == '1';
}

PeerExchange::~PeerExchange() { close(); }

void PeerExchange::close() {
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
  inbox_ = nullptr;
  flags_ = nullptr;
  err_ = nullptr;
}

std::string PeerExchange::handle() const {
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

void PeerExchange::open(const std::vector<std::string>& handles) {
  if ((int)handles.size() != world_) throw std::invalid_argument("xgmi: need one handle per rank");
  for (int q = 0; q < world_; ++q) {
    if (handles[q].size() != sizeof(HandleBlob)) throw std::invalid_argument("xgmi: bad handle");
    HandleBlob h;
    memcpy(&h, handles[q].data(), sizeof(h));
    if (h.world != world_ || h.rank != q) throw std::invalid_argument("xgmi: handle rank mismatch");
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
  opened_ok_ = true;
}

void PeerExchange::fill(int bucket, uint32_t epoch, const XgmiUpdate& u, bool final_wait,
                        bool gated, XgmiLaunch& a) const {
  if (!opened_ok_) throw std::runtime_error("xgmi: open() the peer handles first");
  if (bucket < 0 || bucket >= (int)bk_.size()) throw std::invalid_argument("xgmi: bucket index");
  const Bucket& B = bk_[bucket];
  const bool owns = B.owner < 0 || B.owner == rank_;  // runs the update of (part of) the bucket
  if (owns && u.opt != 2 && !u.m) throw std::invalid_argument("xgmi: optimizer state missing");
  if (owns && u.opt == 0 && !u.v) throw std::invalid_argument("xgmi: Adam needs v");
  memset(&a, 0, sizeof(a));
  a.world = world_;
  a.rank = rank_;
  a.bucket = bucket;
  a.nbuckets = (int)bk_.size();
  a.final_wait = final_wait ? 1 : 0;
  a.epoch = epoch;
  a.lo = B.lo;
  a.c = B.c;
  a.inbox_off = B.inbox_off;
  a.slice = B.slice;
  a.rslot = B.slot;
  for (size_t i = 0; i < bk_.size(); ++i) a.nslices[i] = bk_[i].nslice;
  a.grads = grads_;
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
  a.coef = u.coef;
  a.err = err_;
  a.timeout_ticks = (long long)(timeout_s_ * 1e8);  // wall_clock64: 100 MHz
  a.check = check_ ? 1 : 0;
  a.repl_bucket = repl_;
  a.gate_err = gated ? gate_err_ : nullptr;
  for (size_t i = 0; i < bk_.size(); ++i) a.owners[i] = bk_[i].owner;
  for (int i = (int)bk_.size(); i < kXgmiMaxBuckets; ++i) a.owners[i] = -1;
  if (B.owner >= 0) {
    a.owner = B.owner;
    a.nruns = (int)B.run_lo.size();
    for (int r = 0; r < a.nruns; ++r) {
      a.run_lo[r] = B.run_lo[r];
      a.run_n[r] = B.run_n[r];
      a.run_soff[r] = B.run_soff[r];
      a.run_voff[r] = B.run_voff[r];
      a.run_slice[r] = B.run_slice[r];
      a.run_sl0[r] = B.run_sl0[r];
    }
    a.run_sl0[a.nruns] = B.run_sl0[a.nruns];
  }
}

void PeerExchange::launch(int bucket, uint32_t epoch, const XgmiUpdate& u, bool final_wait,
                          hipStream_t st, bool gated) {
  XgmiLaunch a;
  fill(bucket, epoch, u, final_wait, gated, a);
  const Bucket& B = bk_[bucket];
  if (B.owner >= 0) {
    switch (world_) {
#define X_CASE(N) \
  case N: DDL_LAUNCH(xgmi_owner_kernel<N>, dim3(B.nslice), dim3(256), 0, st, table_, a); break;
      X_CASE(1) X_CASE(2) X_CASE(3) X_CASE(4) X_CASE(5) X_CASE(6) X_CASE(7) X_CASE(8)
#undef X_CASE
      default: DDL_LAUNCH(xgmi_owner_kernel<0>, dim3(B.nslice), dim3(256), 0, st, table_, a);
    }
    DDL_CHECK_LAUNCH();
    return;
  }
  if (bucket == repl_) {
    switch (world_) {
#define X_CASE(N) \
  case N: DDL_LAUNCH(xgmi_repl_kernel<N>, dim3(B.nslice), dim3(256), 0, st, table_, a); break;
      X_CASE(2) X_CASE(3) X_CASE(4) X_CASE(5) X_CASE(6) X_CASE(7) X_CASE(8)
#undef X_CASE
      default: DDL_LAUNCH(xgmi_repl_kernel<0>, dim3(B.nslice), dim3(256), 0, st, table_, a);
    }
    DDL_CHECK_LAUNCH();
    return;
  }
  switch (world_) {
#define X_CASE(N) \
  case N: DDL_LAUNCH(xgmi_ps_kernel<N>, dim3(B.nslice), dim3(256), 0, st, table_, a); break;
    X_CASE(2) X_CASE(3) X_CASE(4) X_CASE(5) X_CASE(6) X_CASE(7) X_CASE(8)
#undef X_CASE
    default: DDL_LAUNCH(xgmi_ps_kernel<0>, dim3(B.nslice), dim3(256), 0, st, table_, a);
  }
  DDL_CHECK_LAUNCH();
}

int PeerExchange::error() const {
  return err_ ? __atomic_load_n(err_, __ATOMIC_ACQUIRE) : 0;
}

// ---- the stale-L2 probe of the xGMI self-test (native_exchange.py) ----------------------------
// A peer's parameter stores reach this GPU's HBM over xGMI without touching its eight per-XCD
// L2s, so a line that some XCD cached BEFORE the exchange could be read back stale by the next
// kernel unless that kernel's start acquire invalidates it (the protocol's assumption, header
// comment above).  The probe makes the hazard reachable on purpose: the sweep is launched with 8
// blocks per 16 KB chunk, block b on XCD b % 8 (the hardware's round-robin dispatch), so before
// the exchange every XCD reads — and caches, with ordinary loads — every line of the buffer, and
// after it every XCD compares every line with the expected values.  want == null: warm only.
__global__ void __launch_bounds__(256) xcd_sweep_kernel(const float4* __restrict__ a,
                                                        const float4* __restrict__ want,
                                                        int64_t n4, int* __restrict__ out) {
  const int64_t chunk = blockIdx.x >> 3;
  const int64_t lo = chunk * 1024, hi = lo + 1024 < n4 ? lo + 1024 : n4;
  int bad = 0;
  float acc = 0.f;
  for (int64_t i = lo + threadIdx.x; i < hi; i += 256) {
    const float4 v = a[i];
    if (want) {
      const float4 w = want[i];
      bad += (v.x != w.x) + (v.y != w.y) + (v.z != w.z) + (v.w != w.w);
    } else {
      acc += v.x + v.y + v.z + v.w;
    }
  }
  if (bad) atomicAdd(out, bad);
  if (!want && acc == 1.2345e-30f) atomicAdd(out + 1, 1);  // keeps the warm loads alive
}

void launch_xcd_sweep(const float* a, const float* want, int64_t n, int* out, hipStream_t st) {
  if (n % 4 || reinterpret_cast<uintptr_t>(a) % 16 || (want && reinterpret_cast<uintptr_t>(want) % 16))
    throw std::invalid_argument("xcd sweep: 16-B aligned float4 buffers");
  const int64_t n4 = n / 4, chunks = (n4 + 1023) / 1024;
  if (chunks <= 0) return;
  DDL_LAUNCH(xcd_sweep_kernel, dim3((unsigned)(chunks * 8)), dim3(256), 0, st,
             reinterpret_cast<const float4*>(a), reinterpret_cast<const float4*>(want), n4, out);
}

}  // namespace ddl
