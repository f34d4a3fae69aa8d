// Host-side concurrency pieces of the asynchronous PS runtimes, CPU-buildable so they can be
// stress-tested under AddressSanitizer / UBSan without a GPU (tests/test_sanitizers_cpu.py,
// csrc/runtime/tests/session_stress.cpp):
//
//  * SessionLocks — the exclusive-session protocol of the RCCL async data plane
//    (kernels/rccl_async.hip): one lock word per process in a POSIX shm segment; an
//    initiator takes BOTH its own and its partner's word with an all-or-nothing try-lock
//    (no hold-and-wait, so no lock cycle can form), releases both after the session.
//  * PostQueue — the worker-side hand-off of the native async step (kernels/async_runner.hip):
//    the step thread enqueues (completion, tokens) jobs, one poster thread waits for each
//    job's completion and posts its tokens in order; finish() waits until every job is posted,
//    and an error on the poster thread fails every later call instead of hanging it.
#pragma once
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>

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

// One poster thread draining jobs in FIFO order.  J is the job type; `wait` blocks until a
// job's work has completed, `post` publishes it (both run on the poster thread; an exception
// from either is recorded and fails every later push() / finish()).
template <class J>
class PostQueue {
 public:
  using Fn = std::function<void(const J&)>;
  PostQueue(Fn wait, Fn post) : wait_(std::move(wait)), post_(std::move(post)) {
    th_ = std::thread([this] { loop(); });
  }
  ~PostQueue() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
  }
  PostQueue(const PostQueue&) = delete;
  PostQueue& operator=(const PostQueue&) = delete;

  void push(J job) {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!error_.empty()) throw std::runtime_error("poster: " + error_);
      q_.push_back(std::move(job));
      ++inflight_;
    }
    cv_.notify_all();
  }
  // every pushed job has been posted (rethrows the poster's error)
  void finish() {
    std::unique_lock<std::mutex> g(mu_);
    cv_.wait(g, [this] { return inflight_ == 0; });
    if (!error_.empty()) throw std::runtime_error("poster: " + error_);
  }
  std::string error() const {
    std::lock_guard<std::mutex> g(mu_);
    return error_;
  }
  int inflight() const {
    std::lock_guard<std::mutex> g(mu_);
    return inflight_;
  }

 private:
  void loop() {
    try {
      for (;;) {
        J job;
        {
          std::unique_lock<std::mutex> g(mu_);
          cv_.wait(g, [this] { return stop_ || !q_.empty(); });
          if (q_.empty()) return;  // stop_
          job = q_.front();
          q_.pop_front();
        }
        wait_(job);
        post_(job);
        {
          std::lock_guard<std::mutex> g(mu_);
          --inflight_;
        }
        cv_.notify_all();
      }
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> g(mu_);
      error_ = e.what();
      inflight_ = 0;
      q_.clear();
      cv_.notify_all();
    }
  }
  Fn wait_, post_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<J> q_;
  int inflight_ = 0;
  bool stop_ = false;
  std::string error_;
  std::thread th_;
};

}  // namespace ddl
