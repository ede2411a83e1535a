// Prometheus metrics with the reference's names (text exposition format 0.0.4):
//   pytorch_operator_jobs_created_total     (pkg/controller.v1/pytorch/job.go:27-32)
//   pytorch_operator_jobs_deleted_total     (controller.go:67-70)
//   pytorch_operator_jobs_successful_total  (status.go:47-60)
//   pytorch_operator_jobs_failed_total
//   pytorch_operator_jobs_restarted_total
//   pytorch_operator_is_leader              (cmd/pytorch-operator.v1/app/server.go:58-61)
// plus operator-internal latency counters (sync count / seconds, reconcile errors).
#pragma once

#include <atomic>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace pto {

class Metrics {
 public:
  static Metrics& instance();

  void inc(const std::string& name, double v = 1.0);
  void set(const std::string& name, double v);
  double get(const std::string& name) const;
  void observe_sync(double seconds);
  std::string exposition() const;

 private:
  Metrics();
  struct M {
    std::string help, type;
    double value = 0;
  };
  mutable std::mutex mu_;
  std::vector<std::string> order_;
  std::map<std::string, M> m_;
  std::vector<double> sync_buckets_ = {0.001, 0.005, 0.01, 0.05, 0.1, 0.5, 1, 5};
  std::vector<uint64_t> sync_counts_;
  double sync_sum_ = 0;
  uint64_t sync_n_ = 0;
};

}  // namespace pto
