// Device side of the xGMI peer-memory flag protocol (xgmi.hip header comment): flag stores,
// bounded waits and the final DONE wait of the bucket kernels.
#pragma once
#include "api.h"
#include "common.h"

namespace ddl {

// The flag that publishes a workgroup's payload.  Every payload store is a system-scope
// (sc0|sc1) write-through store, and every storing wave drains vmcnt(0) before the workgroup
// barrier that precedes the flag store: a write-through store is counted complete only once the
// memory side (local HBM, or the peer over xGMI, or host memory) has acknowledged it, so the
// payload is globally visible before the flag is issued — no L2 write-back is needed (the CDNA
// guide's G16 write-through hand-off, at system scope).  A full system release at each flag (L2
// write-back + wait) writes back every dirty line of the XCD's L2 — the GEMMs' output included —
// and measured 3.2 -> 5.4 ms/step on the two-ranks-on-one-GPU rehearsal (round 2).

DDL_DEV uint32_t xg_flag_load(const uint32_t* f) {
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
DDL_DEV void xg_flag_store(uint32_t* f, uint32_t v) {
  __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

DDL_HD int xg_arrive_idx(int b, int src, int j) {
  return (b * kXgmiMaxPeers + src) * kXgmiMaxSlices + j;
}
// one completion word per (bucket, owner, slice), written only by that owner's workgroup: every
// flag has a single writer and is only ever stored (no read-modify-write: atomics through an
// IPC mapping are performed in whichever XCD L2 the writer's mapping caches them in, so counters
// bumped by several writers can lose updates); the final wait polls them all in parallel
DDL_HD int xg_done_idx(int b, int src, int j) {
  return kXgmiMaxBuckets * kXgmiMaxPeers * kXgmiMaxSlices + xg_arrive_idx(b, src, j);
}

// Bounded wait until *f >= target (wrap-safe).  false on timeout or when another workgroup
// already reported an error (then the caller just runs to the end).
DDL_DEV bool xg_wait_ge(const uint32_t* f, uint32_t target, long long deadline, int* err, int code) {
  // the error word lives in host memory (a PCIe round trip per load): look at it, and at the
  // clock, only every 32nd poll, so a flag that lands is seen within one poll of local memory
  for (int it = 0; (int32_t)(xg_flag_load(f) - target) < 0; ++it) {
    if ((it & 31) == 31) {
      if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) return false;
      if (wall_clock64() > deadline) {
        __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return false;
      }
    }
    // tight for the first ~64 polls (a peer's flag normally lands within a few us), then
    // ~0.45 us apart: waiting waves that poll hard slow the GEMMs running beside them
    // (docs/DESIGN.md round 5, one-card async)
    if (it < 64) __builtin_amdgcn_s_sleep(2);
    else __builtin_amdgcn_s_sleep(16);
  }
  return true;
}

// The final wait of a step: every (bucket, owner, slice) DONE word of the step, except the
// replicated bucket's (it has none), spread over threads [t0, t0 + nt) of the launch (thread t
// polls words t - t0, t - t0 + nt, ...) and polled at once.  An owner bucket's DONE words come
// from its one owner, an equal-chunk bucket's from every rank.
DDL_DEV void xg_final_wait(const XgmiLaunch& a, uint32_t epoch, const uint32_t* myflags, int W,
                           long long deadline, int t, int nt) {
  auto words = [&](int bb) {
    return bb == a.repl_bucket ? 0 : (a.owners[bb] >= 0 ? 1 : W) * a.nslices[bb];
  };
  int total = 0;
  for (int bb = 0; bb < a.nbuckets; ++bb) total += words(bb);
  for (int k = t; k < total; k += nt) {
    int bb = 0, x = k;
    for (;;) {
      const int nb = words(bb);
      if (x < nb) break;
      x -= nb;
      ++bb;
    }
    const int q = x / a.nslices[bb], jj = x - q * a.nslices[bb];
    xg_wait_ge(myflags + xg_done_idx(bb, a.owners[bb] >= 0 ? a.owners[bb] : q, jj), epoch,
               deadline, a.err, 2);
  }
}

}  // namespace ddl
