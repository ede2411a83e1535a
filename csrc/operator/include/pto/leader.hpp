// Leader election on a coordination.k8s.io/v1 Lease (reference: client-go
// leaderelection with an EndpointsLock "pytorch-operator" in the operator's
// namespace, cmd/pytorch-operator.v1/app/server.go:125-171; Endpoints locks are
// deprecated upstream, the Lease keeps the same timings and semantics):
//   lease 15 s, renew deadline 5 s, retry period 3 s; identity "<hostname>_<uuid>";
//   on start -> is_leader=1 + run; on loss -> is_leader=0 + on_stopped (the
//   reference calls log.Fatalf there, i.e. the process exits and restarts).
#pragma once

#include <atomic>
#include <functional>
#include <string>

#include "pto/kube.hpp"

namespace pto {

struct LeaderElectionConfig {
  std::string ns = "default";
  std::string name = "pytorch-operator";
  std::string identity;
  double lease_s = 15.0, renew_deadline_s = 5.0, retry_s = 3.0;
};

class LeaderElector {
 public:
  LeaderElector(KubeClient* client, LeaderElectionConfig cfg);
  // Blocks: acquire, then call on_started_leading (in a thread) and keep renewing.
  // Returns when leadership is lost (after on_stopped_leading) or *stop is set.
  void run(const std::function<void()>& on_started_leading,
           const std::function<void()>& on_stopped_leading, const std::atomic<bool>* stop);
  bool try_acquire_or_renew();
  bool is_leader() const { return leader_.load(); }

 private:
  KubeClient* client_;
  LeaderElectionConfig cfg_;
  std::atomic<bool> leader_{false};
};

std::string make_identity();

}  // namespace pto
