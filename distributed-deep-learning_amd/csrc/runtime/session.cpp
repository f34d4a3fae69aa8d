// SessionLocks (session.h): the RCCL async plane's all-or-nothing pair lock on POSIX shm.
#include "session.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>

namespace ddl {

SessionLocks::~SessionLocks() {
  if (words_) {
    munmap(words_, bytes_);
    if (owner_) shm_unlink(name_.c_str());
  }
}

void SessionLocks::attach(const std::string& name, int max_ranks, bool create) {
  if (words_) throw std::runtime_error("session locks: already attached");
  if (max_ranks < 1) throw std::invalid_argument("session locks: max_ranks");
  name_ = name;
  max_ = max_ranks;
  bytes_ = (size_t)max_ranks * 64;  // one cache line per rank's word
  int fd;
  if (create) {
    shm_unlink(name_.c_str());
    fd = shm_open(name_.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd >= 0 && ftruncate(fd, (off_t)bytes_) != 0) {
      close(fd);
      fd = -1;
    }
  } else {
    fd = shm_open(name_.c_str(), O_RDWR, 0600);
  }
  if (fd < 0) throw std::runtime_error("session locks: shm_open failed: " + name_);
  void* p = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) throw std::runtime_error("session locks: mmap failed: " + name_);
  if (create) memset(p, 0, bytes_);
  words_ = reinterpret_cast<uint64_t*>(p);
  owner_ = create;
}

bool SessionLocks::try_lock_pair(int me, int h) {
  if (me < 0 || me >= max_ || h < 0 || h >= max_) throw std::out_of_range("session locks: rank");
  const uint64_t tag = (uint64_t)me + 1;
  const int lo = std::min(me, h), hi = std::max(me, h);
  uint64_t z = 0;
  if (!__atomic_compare_exchange_n(word(lo), &z, tag, false, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED))
    return false;
  z = 0;
  if (lo != hi &&
      !__atomic_compare_exchange_n(word(hi), &z, tag, false, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED)) {
    __atomic_store_n(word(lo), 0, __ATOMIC_RELEASE);  // all or nothing: no hold-and-wait
    return false;
  }
  return true;
}

void SessionLocks::unlock_pair(int me, int h) {
  __atomic_store_n(word(std::max(me, h)), 0, __ATOMIC_RELEASE);
  __atomic_store_n(word(std::min(me, h)), 0, __ATOMIC_RELEASE);
}

uint64_t SessionLocks::holder(int r) const { return __atomic_load_n(word(r), __ATOMIC_ACQUIRE); }

}  // namespace ddl
