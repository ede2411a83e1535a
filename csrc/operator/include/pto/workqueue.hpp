// Rate-limited work queue with client-go semantics
// (k8s.io/client-go/util/workqueue: queue.go, delaying_queue.go, default_rate_limiters.go):
//
// * a key is never handed to two workers at once (dirty / processing sets);
// * a key added while being processed is re-queued when done() is called;
// * add_after() delays; add_rate_limited() delays by the DefaultControllerRateLimiter:
//   max(per-item exponential 5 ms * 2^n capped at 1000 s, token bucket 10 qps / 100 burst);
// * forget() resets the per-item backoff; num_requeues() reports it.
#pragma once

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <deque>
#include <map>
#include <mutex>
#include <queue>
#include <set>
#include <string>
#include <vector>

namespace pto {

class RateLimitedQueue {
 public:
  using clock = std::chrono::steady_clock;

  RateLimitedQueue(double base_delay_s = 0.005, double max_delay_s = 1000.0, double qps = 10.0,
                   int burst = 100)
      : base_(base_delay_s), max_(max_delay_s), qps_(qps), burst_(burst), tokens_(burst),
        last_(clock::now()) {}

  void add(const std::string& key) {
    std::lock_guard<std::mutex> g(mu_);
    add_locked(key);
  }

  void add_after(const std::string& key, double delay_s) {
    std::lock_guard<std::mutex> g(mu_);
    if (shutdown_) return;
    if (delay_s <= 0) {
      add_locked(key);
      return;
    }
    auto when = clock::now() + std::chrono::duration_cast<clock::duration>(std::chrono::duration<double>(delay_s));
    waiting_.push({when, seq_++, key});
    cv_.notify_all();
  }

  // Delay the next processing of key by the rate limiter and re-queue it.
  void add_rate_limited(const std::string& key) { add_after(key, when(key)); }

  double when(const std::string& key) {
    std::lock_guard<std::mutex> g(mu_);
    int n = failures_[key]++;
    double exp = base_ * std::pow(2.0, (double)n);
    if (exp > max_) exp = max_;
    // token bucket reservation
    auto now = clock::now();
    double elapsed = std::chrono::duration<double>(now - last_).count();
    last_ = now;
    tokens_ = std::min<double>(burst_, tokens_ + elapsed * qps_);
    tokens_ -= 1.0;
    double bucket = tokens_ >= 0 ? 0.0 : -tokens_ / qps_;
    return std::max(exp, bucket);
  }

  void forget(const std::string& key) {
    std::lock_guard<std::mutex> g(mu_);
    failures_.erase(key);
  }

  int num_requeues(const std::string& key) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = failures_.find(key);
    return it == failures_.end() ? 0 : it->second;
  }

  // Blocks until a key is available (or timeout_s elapses when >= 0, or shutdown).
  bool get(std::string* key, double timeout_s = -1.0) {
    std::unique_lock<std::mutex> lk(mu_);
    auto deadline = timeout_s >= 0
                        ? clock::now() + std::chrono::duration_cast<clock::duration>(
                                             std::chrono::duration<double>(timeout_s))
                        : clock::time_point::max();
    while (true) {
      promote_due_locked();
      if (!queue_.empty()) break;
      if (shutdown_) return false;
      auto wake = deadline;
      if (!waiting_.empty()) wake = std::min(wake, waiting_.top().when);
      if (wake == clock::time_point::max()) {
        cv_.wait(lk);
      } else {
        // Sleep on a system_clock deadline: libstdc++ maps steady_clock waits to
        // pthread_cond_clockwait, which ThreadSanitizer (gcc 11) does not intercept and
        // misreports as a double lock.  Every wake re-checks the steady-clock state.
        auto sys_wake = std::chrono::system_clock::now() +
                        std::chrono::duration_cast<std::chrono::system_clock::duration>(wake - clock::now());
        cv_.wait_until(lk, sys_wake);
        if (clock::now() >= deadline) {
          promote_due_locked();
          if (queue_.empty()) return false;
          break;
        }
      }
    }
    *key = queue_.front();
    queue_.pop_front();
    processing_.insert(*key);
    dirty_.erase(*key);
    return true;
  }

  void done(const std::string& key) {
    std::lock_guard<std::mutex> g(mu_);
    processing_.erase(key);
    if (dirty_.count(key)) {
      queue_.push_back(key);
      cv_.notify_one();
    }
  }

  int len() {
    std::lock_guard<std::mutex> g(mu_);
    return (int)queue_.size();
  }

  void shutdown() {
    std::lock_guard<std::mutex> g(mu_);
    shutdown_ = true;
    cv_.notify_all();
  }
  bool shutting_down() {
    std::lock_guard<std::mutex> g(mu_);
    return shutdown_;
  }

 private:
  struct Waiting {
    clock::time_point when;
    uint64_t seq;
    std::string key;
    bool operator>(const Waiting& o) const { return when != o.when ? when > o.when : seq > o.seq; }
  };
  void add_locked(const std::string& key) {
    if (shutdown_) return;
    if (dirty_.count(key)) return;
    dirty_.insert(key);
    if (processing_.count(key)) return;
    queue_.push_back(key);
    cv_.notify_one();
  }
  void promote_due_locked() {
    auto now = clock::now();
    while (!waiting_.empty() && waiting_.top().when <= now) {
      std::string k = waiting_.top().key;
      waiting_.pop();
      add_locked(k);
    }
  }

  double base_, max_, qps_;
  int burst_;
  double tokens_;
  clock::time_point last_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::string> queue_;
  std::set<std::string> dirty_, processing_;
  std::map<std::string, int> failures_;
  std::priority_queue<Waiting, std::vector<Waiting>, std::greater<Waiting>> waiting_;
  uint64_t seq_ = 0;
  bool shutdown_ = false;
};

}  // namespace pto
