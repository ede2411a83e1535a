// Kubernetes REST client for the operator (the reference's clientsets:
// pkg/client/clientset/versioned + client-go kubernetes.Interface + the kube-batch
// client, cmd/pytorch-operator.v1/app/server.go:176-199).
//
// Config resolution follows clientcmd.BuildConfigFromFlags(--master, --kubeconfig)
// with KUBECONFIG overriding the flag (server.go:85-89) and in-cluster service
// account fallback.  Requests are throttled client-side by a token bucket
// (--qps 5 / --burst 10 by default, options.go:82-83).
#pragma once

#include <chrono>
#include <memory>
#include <mutex>
#include <optional>
#include <string>
#include <vector>

#include "pto/http.hpp"
#include "pto/json.hpp"

namespace pto {

// kubeconfig users[].user.exec credential plugin (client.authentication.k8s.io).
struct ExecPlugin {
  std::string command;
  std::vector<std::string> args;
  std::vector<std::pair<std::string, std::string>> env;
  std::string api_version = "client.authentication.k8s.io/v1";
};

struct KubeConfig {
  std::string server;  // https://host:port
  std::string token;
  TlsConfig tls;
  std::string ns = "default";  // current-context namespace
  std::optional<ExecPlugin> exec;
};

// Runs an exec plugin and applies its ExecCredential (token and/or client certificate)
// to `kc`.  false + *error on failure.
bool run_exec_plugin(const ExecPlugin& plugin, KubeConfig* kc, std::string* error);

// --master/--kubeconfig/KUBECONFIG/in-cluster.  Returns nullopt + error on failure.
std::optional<KubeConfig> load_kube_config(const std::string& master_url, const std::string& kubeconfig,
                                           std::string* error);

struct ApiError {
  int code = 0;  // HTTP status; 0 = transport error
  std::string message;
  bool not_found() const { return code == 404; }
  bool conflict() const { return code == 409; }
  bool gone() const { return code == 410; }
  bool timeout() const { return code == 504 || code == 408; }
  bool already_exists() const { return code == 409; }
};

// Resource coordinates: group "" = core /api/v1.
struct Resource {
  std::string group, version, plural;
  bool namespaced = true;
  std::string path(const std::string& ns, const std::string& name = "", const std::string& sub = "") const;
};

extern const Resource kPods, kServices, kEvents, kEndpoints, kLeases, kPyTorchJobs, kPodGroups, kCRDs;
extern const Resource kVolcanoPodGroups;  // --gang-podgroup-api volcano

class KubeClient {
 public:
  KubeClient(const KubeConfig& cfg, double qps = 5.0, int burst = 10);

  std::optional<Json> get(const Resource& r, const std::string& ns, const std::string& name, ApiError* err);
  // LIST; returns the List object (items + metadata.resourceVersion).
  std::optional<Json> list(const Resource& r, const std::string& ns, const std::string& label_selector,
                           ApiError* err);
  std::optional<Json> create(const Resource& r, const std::string& ns, const Json& obj, ApiError* err);
  std::optional<Json> update(const Resource& r, const std::string& ns, const Json& obj, ApiError* err);
  std::optional<Json> update_status(const Resource& r, const std::string& ns, const Json& obj, ApiError* err);
  std::optional<Json> patch_merge(const Resource& r, const std::string& ns, const std::string& name,
                                  const Json& patch, ApiError* err);
  bool del(const Resource& r, const std::string& ns, const std::string& name, ApiError* err);
  // WATCH from resource_version; on_event(type, object) returns false to stop.  Returns
  // when the stream ends; *err set on failure (410 => caller relists).
  void watch(const Resource& r, const std::string& ns, const std::string& label_selector,
             const std::string& resource_version, const std::function<bool(const std::string&, const Json&)>& on_event,
             const std::atomic<bool>* stop, double timeout_s, ApiError* err);

  const KubeConfig& config() const { return cfg_; }

 private:
  std::optional<Json> call(const std::string& method, const std::string& path, const std::string& body,
                           ApiError* err, const std::string& ctype = "application/json");
  void throttle();

  KubeConfig cfg_;
  Url url_;
  std::unique_ptr<HttpClient> http_;
  double qps_;
  int burst_;
  double tokens_;
  std::chrono::steady_clock::time_point last_;
  std::mutex mu_;
};

}  // namespace pto
