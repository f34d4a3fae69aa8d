// Host stress test of the shm mailbox (built with -fsanitize=address,undefined by
// tests/test_sanitizers_cpu.py; SURVEY.md §5.2 "sanitizer builds for the C++ comm layer").
//
// P forked producer processes push N tokens each (producer << 32 | seq) through a small ring
// (forcing full-queue back-pressure); C consumer threads in the parent pop concurrently.
// Checks: every token arrives exactly once, and each consumer sees each producer's tokens in
// increasing order (per-producer FIFO through the MPMC ring).
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../mailbox.h"

int main(int argc, char** argv) {
  const int P = argc > 1 ? atoi(argv[1]) : 4;
  const int C = argc > 2 ? atoi(argv[2]) : 3;
  const int N = argc > 3 ? atoi(argv[3]) : 20000;
  const std::string name = "ddl_stress_" + std::to_string(getpid());
  ddl::ShmMailbox box(name, 64, /*create=*/true);

  std::vector<pid_t> kids;
  for (int p = 0; p < P; ++p) {
    pid_t pid = fork();
    if (pid == 0) {
      ddl::ShmMailbox prod(name, 64, /*create=*/false);
      for (int i = 0; i < N; ++i)
        if (!prod.push(((int64_t)p << 32) | i, 30.0)) _exit(3);
      _exit(0);
    }
    kids.push_back(pid);
  }

  std::vector<std::vector<uint8_t>> seen(P, std::vector<uint8_t>(N, 0));
  std::mutex mu;
  std::atomic<int64_t> got{0};
  std::atomic<bool> bad{false};
  const int64_t total = (int64_t)P * N;
  auto consume = [&]() {
    std::vector<int> last(P, -1);
    while (got.load() < total && !bad.load()) {
      const int64_t v = box.pop(0.05);
      if (v < 0) continue;
      const int p = (int)(v >> 32), i = (int)(v & 0xffffffff);
      if (p < 0 || p >= P || i < 0 || i >= N || i <= last[p]) { bad = true; break; }
      last[p] = i;
      {
        std::lock_guard<std::mutex> g(mu);
        if (seen[p][i]) { bad = true; break; }
        seen[p][i] = 1;
      }
      got.fetch_add(1);
    }
  };
  std::vector<std::thread> th;
  for (int c = 0; c < C; ++c) th.emplace_back(consume);
  for (auto& t : th) t.join();
  int rc = 0;
  for (pid_t k : kids) {
    int st = 0;
    waitpid(k, &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) rc = 1;
  }
  box.unlink();
  if (bad.load() || rc || got.load() != total || box.size() != 0) {
    fprintf(stderr, "FAIL bad=%d rc=%d got=%lld/%lld\n", (int)bad.load(), rc,
            (long long)got.load(), (long long)total);
    return 1;
  }
  printf("OK %lld tokens, %d producers, %d consumers\n", (long long)total, P, C);
  return 0;
}
