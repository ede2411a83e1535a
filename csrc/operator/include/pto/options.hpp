// Operator command-line flags (reference: cmd/pytorch-operator.v1/app/options/options.go:24-84),
// parsed with Go `flag` package rules: -flag / --flag, -flag=value / -flag value, bare
// booleans.  glog flags passed by the reference Deployment (-alsologtostderr, -v=1,
// manifests/deployment.yaml:17-21, Dockerfile:18) are accepted and ignored.
#pragma once

#include <string>
#include <vector>

namespace pto {

struct ServerOption {
  std::string kubeconfig;
  std::string master_url;
  int threadiness = 1;
  bool print_version = false;
  bool json_log_format = true;
  bool enable_gang_scheduling = false;
  std::string gang_scheduler_name = "volcano";
  std::string gang_podgroup_api = "kube-batch";  // --gang-podgroup-api kube-batch|volcano (extension)
  std::string namespace_;  // "" = all namespaces (v1.NamespaceAll)
  int monitoring_port = 8443;
  double resync_period_s = 12 * 3600.0;  // --resyc-period (sic)
  std::string init_container_image = "alpine:3.10";
  int qps = 5;
  int burst = 10;
  // extensions
  bool leader_elect = true;
  // leader-election timings (client-go LeaderElectionConfig; reference hardcodes 15s/5s/3s)
  double lease_duration_s = 15.0, renew_deadline_s = 5.0, retry_period_s = 3.0;
  bool inject_rccl_env = false;
  bool xgmi_pod_topology = false;
  std::vector<std::pair<std::string, std::string>> rccl_env;  // --rccl-env KEY=VALUE (repeatable)
  bool rccl_env_set = false;
  std::string init_container_template_file = "/etc/config/initContainer.yaml";
  std::string log_level = "info";
};

// Returns "" on success, else an error message (unknown flag / bad value).
std::string parse_flags(int argc, char** argv, ServerOption* opt);
// Go time.ParseDuration subset: "12h", "30m", "1h30m", "45s", "500ms", "2.5s".
bool parse_duration(const std::string& s, double* seconds);
std::string usage();

}  // namespace pto
