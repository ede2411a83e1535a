// kubeflow.org/v1 PyTorchJob API: constants, defaulting, validation, naming and
// status/condition helpers.
//
// Parity map (jiaqianjing/pytorch-operator):
//   constants          pkg/apis/pytorch/v1/constants.go:21-34, register.go:23-44
//   set_defaults       pkg/apis/pytorch/v1/defaults.go:36-106
//   validate_spec      pkg/apis/pytorch/validation/validation.go:23-77
//   labels / names     tf-operator/pkg/common/jobcontroller/jobcontroller.go:138-222, util.go:24-57
//   conditions         pkg/controller.v1/pytorch/status.go:149-272
//   exit codes         tf-operator/pkg/util/train/train_util.go:18-53
//
// A job is handled as a JSON document (`Json`): the controller reads and writes
// the fields it reasons about and preserves everything else byte-for-byte.
#pragma once

#include <cstdint>
#include <optional>
#include <string>
#include <vector>

#include "pto/json.hpp"

namespace pto {

// ---------------------------------------------------------------- constants
inline constexpr const char* kGroupName = "kubeflow.org";
inline constexpr const char* kGroupVersion = "v1";
inline constexpr const char* kApiVersion = "kubeflow.org/v1";
inline constexpr const char* kKind = "PyTorchJob";
inline constexpr const char* kPlural = "pytorchjobs";
inline constexpr const char* kSingular = "pytorchjob";
inline constexpr const char* kCRDName = "pytorchjobs.kubeflow.org";
inline constexpr const char* kEnvKubeflowNamespace = "KUBEFLOW_NAMESPACE";
inline constexpr const char* kDefaultPortName = "pytorchjob-port";
inline constexpr const char* kDefaultContainerName = "pytorch";
inline constexpr int kDefaultPort = 23456;
inline constexpr const char* kDefaultRestartPolicy = "OnFailure";
inline constexpr const char* kControllerName = "pytorch-operator";

inline constexpr const char* kReplicaMaster = "Master";
inline constexpr const char* kReplicaWorker = "Worker";

// label keys (pkg/controller.v1/pytorch/controller.go:51-59, jobcontroller.go:138-147)
inline constexpr const char* kLabelGroupName = "group-name";
inline constexpr const char* kLabelJobName = "job-name";
inline constexpr const char* kLabelPyTorchJobName = "pytorch-job-name";  // deprecated
inline constexpr const char* kLabelControllerName = "controller-name";
inline constexpr const char* kLabelReplicaType = "pytorch-replica-type";
inline constexpr const char* kLabelReplicaIndex = "pytorch-replica-index";
inline constexpr const char* kLabelJobRole = "job-role";
inline constexpr const char* kGangPodGroupAnnotation = "scheduling.k8s.io/group-name";

// condition types (kubeflow/common api/v1 types.go)
inline constexpr const char* kJobCreated = "Created";
inline constexpr const char* kJobRunning = "Running";
inline constexpr const char* kJobRestarting = "Restarting";
inline constexpr const char* kJobSucceeded = "Succeeded";
inline constexpr const char* kJobFailed = "Failed";

// condition reasons (pkg/controller.v1/pytorch/status.go:34-45, job.go)
inline constexpr const char* kReasonCreated = "PyTorchJobCreated";
inline constexpr const char* kReasonSucceeded = "PyTorchJobSucceeded";
inline constexpr const char* kReasonRunning = "PyTorchJobRunning";
inline constexpr const char* kReasonFailed = "PyTorchJobFailed";
inline constexpr const char* kReasonRestarting = "PyTorchJobRestarting";
inline constexpr const char* kReasonInvalidSpec = "InvalidPyTorchJobSpec";

// event reasons (pod.go:36-45, pod_control.go, service_control.go)
inline constexpr const char* kReasonPodTemplateRestartPolicy = "SettedPodTemplateRestartPolicy";
inline constexpr const char* kReasonExitedWithCode = "ExitedWithCode";
inline constexpr const char* kReasonPodTemplateSchedulerName = "SettedPodTemplateSchedulerName";

// clean pod policies / restart policies
inline constexpr const char* kCleanPodPolicyAll = "All";
inline constexpr const char* kCleanPodPolicyRunning = "Running";
inline constexpr const char* kCleanPodPolicyNone = "None";
inline constexpr const char* kRestartAlways = "Always";
inline constexpr const char* kRestartOnFailure = "OnFailure";
inline constexpr const char* kRestartNever = "Never";
inline constexpr const char* kRestartExitCode = "ExitCode";

// ---------------------------------------------------------------- time
int64_t now_ms();
std::string format_time(int64_t unix_ms);            // RFC 3339, second precision ("...Z")
std::optional<int64_t> parse_time(const std::string&);  // RFC 3339 -> unix ms

// ---------------------------------------------------------------- strings
std::string to_lower(std::string s);
bool iequals(const std::string& a, const std::string& b);

// ---------------------------------------------------------------- job accessors
std::string job_name(const Json& obj);
std::string job_namespace(const Json& obj);
std::string job_uid(const Json& obj);
std::string job_key(const Json& obj);  // "<ns>/<name>"
bool split_key(const std::string& key, std::string* ns, std::string* name);

// The replica types present in spec.pytorchReplicaSpecs, Master first.
std::vector<std::string> replica_types(const Json& job);
const Json* replica_spec(const Json& job, const std::string& rtype);
int32_t replicas_of(const Json& job, const std::string& rtype);  // 1 when unset
int32_t total_replicas(const Json& job);
std::string restart_policy_of(const Json& job, const std::string& rtype);
bool contains_master_spec(const Json& job);
// Port named pytorchjob-port of the "pytorch" container of rtype (util.go:34-47).
std::optional<int32_t> port_of(const Json& job, const std::string& rtype);

// ---------------------------------------------------------------- defaults / validation
void set_defaults(Json& job);
// "" when valid, else the reference's error message verbatim.
std::string validate_spec(const Json& spec);

// ---------------------------------------------------------------- naming
Json gen_labels(const std::string& job_name);  // group-name, job-name, pytorch-job-name, controller-name
std::string gen_general_name(const std::string& job_name, const std::string& rtype_lower,
                             const std::string& index);
Json gen_owner_reference(const Json& job);
std::string gen_expectation_pods_key(const std::string& job_key, const std::string& rtype);
std::string gen_expectation_services_key(const std::string& job_key, const std::string& rtype);
std::string gen_pod_group_name(const std::string& job_name);

// ---------------------------------------------------------------- status / conditions
struct ReplicaStatus {
  int32_t active = 0, succeeded = 0, failed = 0;
};
struct JobCondition {
  std::string type, status, reason, message, last_update_time, last_transition_time;
};
struct JobStatus {
  std::vector<JobCondition> conditions;
  std::vector<std::pair<std::string, ReplicaStatus>> replica_statuses;  // ordered by type
  std::optional<std::string> start_time, completion_time, last_reconcile_time;

  ReplicaStatus* replica(const std::string& rtype);
  ReplicaStatus& ensure_replica(const std::string& rtype);
  static JobStatus from_json(const Json& j);
  Json to_json() const;
  bool operator==(const JobStatus& o) const;
};

JobCondition new_condition(const std::string& type, const std::string& reason,
                           const std::string& message, int64_t now);
bool has_condition(const JobStatus& s, const std::string& type);
bool is_succeeded(const JobStatus& s);
bool is_failed(const JobStatus& s);
void set_condition(JobStatus& s, JobCondition c);
std::vector<JobCondition> filter_out_condition(const std::vector<JobCondition>& conds,
                                               const std::string& type);

// ---------------------------------------------------------------- pods
std::string pod_phase(const Json& pod);
bool is_pod_active(const Json& pod);  // not Succeeded/Failed and not being deleted
bool is_retryable_exit_code(int32_t code);

}  // namespace pto
