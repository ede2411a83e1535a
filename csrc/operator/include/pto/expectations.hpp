// Controller expectations (k8s.io/kubernetes/pkg/controller/controller_utils.go:182-292):
// a TTL cache of "creations/deletions I have issued but not yet observed" per key.
// satisfied() is true when a key has no record, its record is fulfilled, or the
// record is older than the TTL (5 min) -- so a lost watch event cannot wedge a job.
#pragma once

#include <chrono>
#include <map>
#include <mutex>
#include <string>

namespace pto {

class Expectations {
 public:
  explicit Expectations(double ttl_s = 300.0) : ttl_s_(ttl_s) {}

  // ExpectCreations / ExpectDeletions *set* the record (SetExpectations semantics).
  void expect_creations(const std::string& key, int n) { set(key, n, 0); }
  void expect_deletions(const std::string& key, int n) { set(key, 0, n); }
  void creation_observed(const std::string& key) { lower(key, 1, 0); }
  void deletion_observed(const std::string& key) { lower(key, 0, 1); }
  void raise(const std::string& key, int add, int del) { lower(key, -add, -del); }
  bool satisfied(const std::string& key) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = recs_.find(key);
    if (it == recs_.end()) return true;
    if (it->second.add <= 0 && it->second.del <= 0) return true;
    double age = std::chrono::duration<double>(clock::now() - it->second.ts).count();
    return age > ttl_s_;
  }
  void remove(const std::string& key) {
    std::lock_guard<std::mutex> g(mu_);
    recs_.erase(key);
  }

 private:
  using clock = std::chrono::steady_clock;
  struct Rec {
    long add = 0, del = 0;
    clock::time_point ts;
  };
  void set(const std::string& key, int add, int del) {
    std::lock_guard<std::mutex> g(mu_);
    recs_[key] = Rec{add, del, clock::now()};
  }
  void lower(const std::string& key, int add, int del) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = recs_.find(key);
    if (it == recs_.end()) return;
    it->second.add -= add;
    it->second.del -= del;
  }
  double ttl_s_;
  std::mutex mu_;
  std::map<std::string, Rec> recs_;
};

}  // namespace pto
