#include "mailbox.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <new>
#include <stdexcept>
#include <thread>

namespace ddl {

static constexpr uint64_t kMagic = 0x44444c4d424f5831ull;  // "DDLMBOX1"

ShmMailbox::ShmMailbox(const std::string& name, int64_t capacity, bool create)
    : name_(name), owner_(create) {
  uint64_t cap = 2;
  while ((int64_t)cap < capacity) cap <<= 1;
  bytes_ = sizeof(Header) + cap * sizeof(Slot);
  int fd = -1;
  if (create) {
    shm_unlink(name.c_str());  // stale segment from a crashed job
    fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("shm_open(create) failed: " + name);
    if (ftruncate(fd, (off_t)bytes_) != 0) {
      close(fd);
      throw std::runtime_error("ftruncate failed: " + name);
    }
  } else {
    for (int tries = 0; tries < 2000 && fd < 0; ++tries) {
      fd = shm_open(name.c_str(), O_RDWR, 0600);
      if (fd < 0) std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
    if (fd < 0) throw std::runtime_error("shm_open(attach) failed: " + name);
    struct stat st;
    if (fstat(fd, &st) != 0 || (size_t)st.st_size < sizeof(Header)) {
      close(fd);
      throw std::runtime_error("mailbox segment too small: " + name);
    }
    bytes_ = (size_t)st.st_size;
  }
  base_ = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (base_ == MAP_FAILED) throw std::runtime_error("mmap failed: " + name);
  hdr_ = reinterpret_cast<Header*>(base_);
  slots_ = reinterpret_cast<Slot*>(reinterpret_cast<char*>(base_) + sizeof(Header));
  if (create) {
    new (hdr_) Header();
    hdr_->cap = cap;
    hdr_->head.store(0, std::memory_order_relaxed);
    hdr_->tail.store(0, std::memory_order_relaxed);
    for (uint64_t i = 0; i < cap; ++i) {
      new (&slots_[i]) Slot();
      slots_[i].seq.store(i, std::memory_order_relaxed);
      slots_[i].value = 0;
    }
    std::atomic_thread_fence(std::memory_order_release);
    hdr_->magic = kMagic;
  } else {
    for (int tries = 0; tries < 2000 && hdr_->magic != kMagic; ++tries)
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
    if (hdr_->magic != kMagic) throw std::runtime_error("mailbox not initialised: " + name);
    std::atomic_thread_fence(std::memory_order_acquire);
  }
  mask_ = hdr_->cap - 1;
}

ShmMailbox::~ShmMailbox() {
  if (base_ && base_ != MAP_FAILED) munmap(base_, bytes_);
}

void ShmMailbox::unlink() { shm_unlink(name_.c_str()); }

// The arrival queue is on the round trip of every async step (worker post -> PS service pop),
// so an idle waiter stays on the CPU for a while before it sleeps: a sleep_for of a few
// microseconds lasts ~50-80 us on Linux (timer slack), which the round trip would pay whenever
// a token arrives just after the waiter dozed off.  Spin, then yield for ~2 ms, then sleep.
static inline void backoff(int& spins) {
  if (spins < 64) {
    ++spins;
  } else if (spins < 64 + 20000) {
    ++spins;
    std::this_thread::yield();
  } else {
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

bool ShmMailbox::push(int64_t value, double timeout_s) {
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  int spins = 0;
  uint64_t pos = hdr_->tail.load(std::memory_order_relaxed);
  for (;;) {
    Slot& s = slots_[pos & mask_];
    const uint64_t seq = s.seq.load(std::memory_order_acquire);
    const int64_t dif = (int64_t)seq - (int64_t)pos;
    if (dif == 0) {
      if (hdr_->tail.compare_exchange_weak(pos, pos + 1, std::memory_order_relaxed)) {
        s.value = value;
        s.seq.store(pos + 1, std::memory_order_release);
        return true;
      }
    } else if (dif < 0) {  // full
      if (std::chrono::steady_clock::now() > deadline) return false;
      backoff(spins);
      pos = hdr_->tail.load(std::memory_order_relaxed);
    } else {
      pos = hdr_->tail.load(std::memory_order_relaxed);
    }
  }
}

int64_t ShmMailbox::pop(double timeout_s) {
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  int spins = 0;
  uint64_t pos = hdr_->head.load(std::memory_order_relaxed);
  for (;;) {
    Slot& s = slots_[pos & mask_];
    const uint64_t seq = s.seq.load(std::memory_order_acquire);
    const int64_t dif = (int64_t)seq - (int64_t)(pos + 1);
    if (dif == 0) {
      if (hdr_->head.compare_exchange_weak(pos, pos + 1, std::memory_order_relaxed)) {
        const int64_t v = s.value;
        s.seq.store(pos + mask_ + 1, std::memory_order_release);
        return v;
      }
    } else if (dif < 0) {  // empty
      if (std::chrono::steady_clock::now() > deadline) return -1;
      backoff(spins);
      pos = hdr_->head.load(std::memory_order_relaxed);
    } else {
      pos = hdr_->head.load(std::memory_order_relaxed);
    }
  }
}

int64_t ShmMailbox::size() const {
  const uint64_t t = hdr_->tail.load(std::memory_order_acquire);
  const uint64_t h = hdr_->head.load(std::memory_order_acquire);
  return (int64_t)(t - h);
}

}  // namespace ddl
