// Host stress test of the async PS runtimes' concurrency (runtime/session.h), built with
// -fsanitize=address,undefined by tests/test_sanitizers_cpu.py.
//
// Exclusive sessions (kernels/rccl_async.hip protocol) between P forked processes: each runs
//    the RcclAsync comm-thread loop shape — serve a pending request from its own mailbox first,
//    else try to open a session to a random peer (all-or-nothing pair lock), post the request
//    into the peer's mailbox and wait for the peer's acknowledgement, then release both locks.
//    The serving side checks that BOTH lock words hold the initiator's tag for the whole
//    session.  Checks: every session is served exactly once by the right peer (per-pair counts),
//    the lock invariant never breaks, and nobody waits past a deadline (a lock cycle or a lost
//    request would show up as a timeout).
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <new>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../mailbox.h"
#include "../session.h"

namespace {

constexpr int kMaxP = 16;
struct Shared {                       // MAP_SHARED | MAP_ANONYMOUS, inherited by the children
  std::atomic<uint64_t> ack[kMaxP];   // sessions of initiator a acknowledged so far
  std::atomic<int64_t> served[kMaxP][kMaxP];   // [initiator][server]
  std::atomic<int64_t> started[kMaxP][kMaxP];  // [initiator][server]
  std::atomic<int64_t> violations;
};

double secs_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

int child(int r, int P, int N, const std::string& tag, Shared* sh) {
  ddl::SessionLocks locks;
  locks.attach("/" + tag + "_lock", P, false);
  std::vector<std::unique_ptr<ddl::ShmMailbox>> boxes(P);
  for (int q = 0; q < P; ++q)
    boxes[q] = std::make_unique<ddl::ShmMailbox>(tag + "_box" + std::to_string(q), 8, false);
  std::mt19937 rng(1234 + r);
  int done = 0;
  uint64_t mine = 0;
  while (done < N) {
    // (a) serve: an initiator holding both words waits for us
    const int64_t v = boxes[r]->pop(0.0);
    if (v >= 0) {
      const int a = (int)v;
      if (a < 0 || a >= P || a == r || locks.holder(a) != (uint64_t)a + 1 ||
          locks.holder(r) != (uint64_t)a + 1)
        sh->violations.fetch_add(1);
      sh->served[a][r].fetch_add(1);
      for (volatile int k = 0; k < (int)(rng() % 200); ++k) {
      }
      if (locks.holder(a) != (uint64_t)a + 1 || locks.holder(r) != (uint64_t)a + 1)
        sh->violations.fetch_add(1);  // nobody stole a word mid-session
      sh->ack[a].fetch_add(1, std::memory_order_release);
      continue;
    }
    if (done >= N) break;
    // (b) initiate a session with a random peer
    int h = (int)(rng() % (P - 1));
    if (h >= r) ++h;
    if (!locks.try_lock_pair(r, h)) {
      std::this_thread::yield();
      continue;
    }
    sh->started[r][h].fetch_add(1);
    if (!boxes[h]->push(r, 10.0)) return 4;
    const auto t0 = std::chrono::steady_clock::now();
    while (sh->ack[r].load(std::memory_order_acquire) == mine) {
      if (secs_since(t0) > 20.0) return 5;  // deadlock or lost request
      std::this_thread::yield();
    }
    ++mine;
    locks.unlock_pair(r, h);
    ++done;
  }
  // keep serving until every peer is done (their sessions may still target us)
  const auto t1 = std::chrono::steady_clock::now();
  for (;;) {
    int64_t want = 0, got = 0;
    for (int a = 0; a < P; ++a) {
      want += sh->started[a][r].load();
      got += sh->served[a][r].load();
    }
    int64_t all_done = 0;
    for (int a = 0; a < P; ++a) all_done += (int64_t)sh->ack[a].load();
    const int64_t v = boxes[r]->pop(0.001);
    if (v >= 0) {
      const int a = (int)v;
      if (locks.holder(a) != (uint64_t)a + 1 || locks.holder(r) != (uint64_t)a + 1)
        sh->violations.fetch_add(1);
      sh->served[a][r].fetch_add(1);
      sh->ack[a].fetch_add(1, std::memory_order_release);
      continue;
    }
    if (all_done >= (int64_t)P * N && want == got) return 0;
    if (secs_since(t1) > 60.0) return 6;
  }
}

}  // namespace

int main(int argc, char** argv) {
  const int P = argc > 1 ? atoi(argv[1]) : 8;
  const int N = argc > 2 ? atoi(argv[2]) : 2000;
  if (P < 2 || P > kMaxP) return 2;
  const std::string tag = "ddl_sess_" + std::to_string(getpid());
  auto* sh = static_cast<Shared*>(mmap(nullptr, sizeof(Shared), PROT_READ | PROT_WRITE,
                                       MAP_SHARED | MAP_ANONYMOUS, -1, 0));
  if (sh == MAP_FAILED) return 2;
  new (sh) Shared();
  ddl::SessionLocks locks;
  locks.attach("/" + tag + "_lock", P, true);
  std::vector<std::unique_ptr<ddl::ShmMailbox>> boxes;
  for (int q = 0; q < P; ++q)
    boxes.push_back(std::make_unique<ddl::ShmMailbox>(tag + "_box" + std::to_string(q), 8, true));
  std::vector<pid_t> kids;
  for (int r = 0; r < P; ++r) {
    const pid_t pid = fork();
    if (pid == 0) _exit(child(r, P, N, tag, sh));
    kids.push_back(pid);
  }
  int bad = 0;
  for (pid_t k : kids) {
    int st = 0;
    waitpid(k, &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) {
      printf("child exit %d\n", WIFEXITED(st) ? WEXITSTATUS(st) : -1);
      ++bad;
    }
  }
  int64_t total = 0;
  for (int a = 0; a < P; ++a)
    for (int h = 0; h < P; ++h) {
      if (sh->served[a][h].load() != sh->started[a][h].load()) ++bad;
      total += sh->served[a][h].load();
    }
  if (sh->violations.load() != 0) {
    printf("lock violations %lld\n", (long long)sh->violations.load());
    ++bad;
  }
  for (auto& b : boxes) b->unlink();
  if (bad || total != (int64_t)P * N) {
    printf("FAIL sessions %lld of %lld\n", (long long)total, (long long)P * N);
    return 1;
  }
  printf("OK %lld sessions, %d processes\n", (long long)total, P);
  return 0;
}
