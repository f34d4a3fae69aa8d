// Lock-free bounded MPMC arrival queue in POSIX shared memory (async PS control plane).
//
// Replaces the reference's MPI.ANY_SOURCE receive (mnist_async_sharding/parameter_server.py:
// 99-100): workers post (worker, ps) tokens, the PS service thread pops them in arrival
// order and then talks to that worker over a dedicated RCCL pair communicator.
// Algorithm: Vyukov bounded queue (per-slot sequence numbers), address-free atomics.
#pragma once
#include <atomic>
#include <cstddef>
#include <cstdint>
#include <string>

namespace ddl {

class ShmMailbox {
 public:
  ShmMailbox(const std::string& name, int64_t capacity, bool create);
  ~ShmMailbox();
  ShmMailbox(const ShmMailbox&) = delete;
  ShmMailbox& operator=(const ShmMailbox&) = delete;

  bool push(int64_t value, double timeout_s);  // false on timeout (queue full)
  int64_t pop(double timeout_s);               // -1 on timeout
  int64_t size() const;
  int64_t capacity() const { return (int64_t)(mask_ + 1); }
  void unlink();

 private:
  struct Slot {
    std::atomic<uint64_t> seq;
    int64_t value;
  };
  struct Header {
    uint64_t magic;
    uint64_t cap;
    alignas(64) std::atomic<uint64_t> head;
    alignas(64) std::atomic<uint64_t> tail;
  };
  std::string name_;
  void* base_ = nullptr;
  size_t bytes_ = 0;
  Header* hdr_ = nullptr;
  Slot* slots_ = nullptr;
  uint64_t mask_ = 0;
  bool owner_ = false;
};

}  // namespace ddl
