// The PyTorchJob reconcile core as a pure function.
//
// reconcile() takes one job plus the pods/services it owns and returns the
// actions the controller must apply (pod/service creates + deletes, PodGroup
// sync, job deletion, status update, events, requeues, metric increments).
// It performs no I/O, so every behaviour of the reference controller is unit
// testable table-driven (tests/test_operator_reconcile.py ports the Go tests).
//
// Parity map (jiaqianjing/pytorch-operator pkg/controller.v1/pytorch):
//   reconcile                  controller.go:336-492 (reconcilePyTorchJobs)
//   backoff / active deadline  controller.go:391-453, 520-568
//   pod reconcile + creation   pod.go:49-232, 283-298
//   cluster-spec env           pod.go:234-281
//   init container             util.go:49-87, pkg/common/config/config.go:9-34
//   services                   service.go:36-153
//   status / conditions        status.go:63-146
//   clean-pod policy / TTL     job.go:153-211
//   job added (Created / invalid spec -> Failed)  job.go:35-111
#pragma once

#include <optional>
#include <string>
#include <vector>

#include "pto/api.hpp"
#include "pto/json.hpp"

namespace pto {

extern const char* const kDefaultInitContainerTemplate;

struct ControllerConfig {
  bool enable_gang_scheduling = false;
  std::string gang_scheduler_name = "volcano";
  // PodGroup API the gang PodGroup is created in: "kube-batch" (reference parity:
  // scheduling.incubator.k8s.io/v1alpha1, tf-operator jobcontroller.go:224-278) or "volcano"
  // (scheduling.volcano.sh/v1beta1, what Volcano >= 1.0 reads)
  std::string gang_podgroup_api = "kube-batch";
  std::string init_container_image = "alpine:3.10";
  std::string init_container_template = kDefaultInitContainerTemplate;
  // MI355X extensions (all off by default = reference behaviour):
  // inject LOCAL_RANK (=0: one GPU per pod) and the env below into every "pytorch"
  // container that does not already set them.  The default set holds only what the
  // IPC path needs; tuning variables (e.g. NCCL_MIN_NCHANNELS, NCCL_PROTO) are added
  // with --rccl-env KEY=VALUE once measured on the target node (docs/xgmi_pods.md).
  bool inject_rccl_env = false;
  std::vector<std::pair<std::string, std::string>> rccl_env = {
      {"HSA_ENABLE_IPC_MODE_LEGACY", "0"},  // dmabuf IPC (what current amdgpu drivers support)
  };
  // One node, one GPU per pod, peer memory over xGMI (docs/xgmi_pods.md): for replicas
  // that request amd.com/gpu, share the node's PID namespace (dmabuf IPC import reads the
  // exporter's /proc/<pid>/fd/<fd>), its IPC namespace and /dev/shm (RCCL SHM transport),
  // give RCCL the node identity (NCCL_HOSTID <- spec.nodeName: pods otherwise hash as
  // different hosts and fall back to the network transport) and co-locate the job's pods
  // on one node (required pod affinity on kubernetes.io/hostname).
  bool xgmi_pod_topology = false;
};

struct Event {
  std::string type;     // Normal | Warning
  std::string reason;
  std::string message;
  std::string kind = "PyTorchJob";  // involved object kind
  std::string name;                 // involved object name
};

struct ObjectRef {
  std::string ns, name;
  std::string replica_type;  // pods: pytorch-replica-type label (log field), "" for services
};

struct MetricDeltas {
  int created = 0, deleted = 0, successful = 0, failed = 0, restarted = 0;
};

struct ReconcileInput {
  Json job;                       // defaulted PyTorchJob
  std::vector<Json> pods;         // pods owned by (claimed for) the job
  std::vector<Json> services;     // services owned by the job
  int64_t now = 0;                // unix ms
  int requeues = 0;               // workqueue NumRequeues(key)
  bool podgroup_exists = false;   // gang scheduling: PodGroup already present
};

struct ReconcileResult {
  std::vector<Json> create_pods;          // full manifests, in creation order
  std::vector<std::string> create_pod_expectation_keys;  // parallel to create_pods
  std::vector<ObjectRef> delete_pods;
  std::vector<Json> create_services;
  std::vector<std::string> create_service_expectation_keys;
  std::vector<ObjectRef> delete_services;
  std::optional<Json> create_podgroup;    // gang scheduling
  bool delete_podgroup = false;
  bool delete_job = false;                // TTL expired
  bool status_changed = false;
  Json status;                            // new .status (always filled)
  std::vector<Event> events;
  std::vector<double> requeue_after_s;    // WorkQueue.AddAfter
  bool requeue_rate_limited = false;      // WorkQueue.AddRateLimited
  MetricDeltas metrics;
  std::string error;                      // non-empty: sync failed, requeue rate-limited
};

ReconcileResult reconcile(const ReconcileInput& in, const ControllerConfig& cfg);

// addPyTorchJob: validate, default, add the Created condition.
struct JobAddedResult {
  bool valid = true;
  std::string error;   // validation error message
  Json status;         // status to write (Created, or Failed/InvalidPyTorchJobSpec)
  std::vector<Event> events;
  MetricDeltas metrics;
};
JobAddedResult on_job_added(const Json& job, int64_t now);

// Requeue delay when activeDeadlineSeconds changes on update (job.go:133-149); <0: none.
double deadline_requeue_on_update(const Json& old_job, const Json& cur_job, int64_t now);

// Building blocks, exposed for tests.
Json build_pod(const Json& job, const std::string& rtype, int index, const ControllerConfig& cfg,
               std::vector<Event>* events, std::string* error);
Json build_service(const Json& job, const std::string& rtype, int index, std::string* error);
std::string set_cluster_spec(Json& pod_template, const Json& job, int32_t total, int index,
                             const std::string& rtype);
std::vector<Json> init_containers(const ControllerConfig& cfg, const std::string& master_addr,
                                  std::string* error);
std::vector<Json> filter_by_replica_type(const std::vector<Json>& objs, const std::string& rt_lower);
std::vector<std::vector<Json>> slices_by_index(const std::vector<Json>& objs, int replicas);
bool past_backoff_limit(const Json& job, const std::vector<Json>& pods);
bool past_active_deadline(const Json& job, int64_t now);
Json update_status_single_json(const Json& job, const std::string& rtype, int replicas, bool restart,
                               int64_t now);

}  // namespace pto
