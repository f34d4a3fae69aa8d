// Host-side concurrency of the asynchronous RCCL PS runtime, CPU-buildable so it can be
// stress-tested under AddressSanitizer / UBSan without a GPU (tests/test_sanitizers_cpu.py,
// csrc/runtime/tests/session_stress.cpp):
//
//  * SessionLocks — the exclusive-session protocol of the RCCL async data plane
//    (kernels/rccl_async.hip): one lock word per process in a POSIX shm segment; an
//    initiator takes BOTH its own and its partner's word with an all-or-nothing try-lock
//    (no hold-and-wait, so no lock cycle can form), releases both after the session.
// (The xGMI async step's poster thread and its FIFO were removed in round 4: pushes post
// themselves on an arrival board in host memory, kernels/xgmi_async.hip.)
#pragma once
#include <cstdint>
#include <string>

namespace ddl {

class SessionLocks {
 public:
  SessionLocks() = default;
  ~SessionLocks();
  SessionLocks(const SessionLocks&) = delete;
  SessionLocks& operator=(const SessionLocks&) = delete;
  // the job's segment of `max_ranks` lock words (one cache line each); rank 0 creates it
  void attach(const std::string& name, int max_ranks, bool create);
  // take the words of `me` and `h` (ascending rank order), both or neither
  bool try_lock_pair(int me, int h);
  void unlock_pair(int me, int h);
  // the tag a rank writes into a word it holds (rank + 1; 0 = free)
  uint64_t holder(int r) const;

 private:
  uint64_t* word(int r) const { return words_ + (size_t)r * 8; }
  uint64_t* words_ = nullptr;
  size_t bytes_ = 0;
  int max_ = 0;
  bool owner_ = false;
  std::string name_;
};

}  // namespace ddl
