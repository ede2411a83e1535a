#include "pto/metrics.hpp"

#include <cstdio>

namespace pto {

Metrics& Metrics::instance() {
  static Metrics m;
  return m;
}

Metrics::Metrics() : sync_counts_(sync_buckets_.size(), 0) {
  auto add = [&](const char* n, const char* help, const char* type) {
    order_.push_back(n);
    m_[n] = M{help, type, 0};
  };
  add("pytorch_operator_jobs_created_total", "Counts number of PyTorch jobs created", "counter");
  add("pytorch_operator_jobs_deleted_total", "Counts number of PyTorch jobs deleted", "counter");
  add("pytorch_operator_jobs_successful_total", "Counts number of PyTorch jobs successful", "counter");
  add("pytorch_operator_jobs_failed_total", "Counts number of PyTorch jobs failed", "counter");
  add("pytorch_operator_jobs_restarted_total", "Counts number of PyTorch jobs restarted", "counter");
  add("pytorch_operator_is_leader", "Is this client the leader of this pytorch-operator client set?", "gauge");
  add("pytorch_operator_reconcile_errors_total", "Number of failed job syncs (requeued rate-limited)", "counter");
  add("pytorch_operator_api_requests_total", "Kubernetes API requests issued by the controller", "counter");
}

void Metrics::inc(const std::string& name, double v) {
  std::lock_guard<std::mutex> g(mu_);
  m_[name].value += v;
}

void Metrics::set(const std::string& name, double v) {
  std::lock_guard<std::mutex> g(mu_);
  m_[name].value = v;
}

double Metrics::get(const std::string& name) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = m_.find(name);
  return it == m_.end() ? 0 : it->second.value;
}

void Metrics::observe_sync(double s) {
  std::lock_guard<std::mutex> g(mu_);
  for (size_t i = 0; i < sync_buckets_.size(); ++i)
    if (s <= sync_buckets_[i]) sync_counts_[i]++;
  sync_sum_ += s;
  sync_n_++;
}

std::string Metrics::exposition() const {
  std::lock_guard<std::mutex> g(mu_);
  std::string out;
  char buf[256];
  for (const auto& n : order_) {
    const M& m = m_.at(n);
    out += "# HELP " + n + " " + m.help + "\n# TYPE " + n + " " + m.type + "\n";
    std::snprintf(buf, sizeof buf, "%s %.17g\n", n.c_str(), m.value);
    out += buf;
  }
  const char* h = "pytorch_operator_sync_duration_seconds";
  out += std::string("# HELP ") + h + " Duration of one job sync (syncPyTorchJob)\n# TYPE " + h + " histogram\n";
  for (size_t i = 0; i < sync_buckets_.size(); ++i) {
    std::snprintf(buf, sizeof buf, "%s_bucket{le=\"%g\"} %llu\n", h, sync_buckets_[i],
                  (unsigned long long)sync_counts_[i]);
    out += buf;
  }
  std::snprintf(buf, sizeof buf, "%s_bucket{le=\"+Inf\"} %llu\n%s_sum %.9g\n%s_count %llu\n", h,
                (unsigned long long)sync_n_, h, sync_sum_, h, (unsigned long long)sync_n_);
  out += buf;
  return out;
}

}  // namespace pto
