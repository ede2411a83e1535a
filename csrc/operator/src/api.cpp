#include "pto/api.hpp"

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cstdio>
#include <ctime>
#include <cerrno>

namespace pto {

// ---------------------------------------------------------------- time
int64_t now_ms() {
  using namespace std::chrono;
  return duration_cast<milliseconds>(system_clock::now().time_since_epoch()).count();
}

std::string format_time(int64_t unix_ms) {
  time_t t = (time_t)(unix_ms / 1000);
  struct tm tmv;
  gmtime_r(&t, &tmv);
  char buf[32];
  std::strftime(buf, sizeof buf, "%Y-%m-%dT%H:%M:%SZ", &tmv);
  return buf;
}

std::optional<int64_t> parse_time(const std::string& s) {
  int Y, M, D, h, m;
  double sec;
  char tail[16] = {0};
  if (std::sscanf(s.c_str(), "%4d-%2d-%2dT%2d:%2d:%lf%15s", &Y, &M, &D, &h, &m, &sec, tail) < 6)
    return std::nullopt;
  struct tm tmv = {};
  tmv.tm_year = Y - 1900;
  tmv.tm_mon = M - 1;
  tmv.tm_mday = D;
  tmv.tm_hour = h;
  tmv.tm_min = m;
  tmv.tm_sec = 0;
  int64_t base = (int64_t)timegm(&tmv) * 1000 + (int64_t)(sec * 1000.0 + 0.5);
  // numeric offset: +HH:MM / -HH:MM ("Z" or empty = UTC)
  std::string tz(tail);
  if (!tz.empty() && (tz[0] == '+' || tz[0] == '-')) {
    int oh = 0, om = 0;
    if (std::sscanf(tz.c_str() + 1, "%2d:%2d", &oh, &om) >= 1) {
      int64_t off = ((int64_t)oh * 60 + om) * 60 * 1000;
      base += tz[0] == '+' ? -off : off;
    }
  }
  return base;
}

// ---------------------------------------------------------------- strings
std::string to_lower(std::string s) {
  for (auto& c : s) c = (char)std::tolower((unsigned char)c);
  return s;
}
bool iequals(const std::string& a, const std::string& b) { return to_lower(a) == to_lower(b); }

// ---------------------------------------------------------------- accessors
std::string job_name(const Json& obj) {
  const Json* md = obj.get("metadata");
  return md ? md->str_or("name") : "";
}
std::string job_namespace(const Json& obj) {
  const Json* md = obj.get("metadata");
  std::string ns = md ? md->str_or("namespace") : "";
  return ns;
}
std::string job_uid(const Json& obj) {
  const Json* md = obj.get("metadata");
  return md ? md->str_or("uid") : "";
}
std::string job_key(const Json& obj) {
  std::string ns = job_namespace(obj);
  return ns.empty() ? job_name(obj) : ns + "/" + job_name(obj);
}
bool split_key(const std::string& key, std::string* ns, std::string* name) {
  auto pos = key.find('/');
  if (pos == std::string::npos) {
    *ns = "";
    *name = key;
    return !key.empty();
  }
  if (key.find('/', pos + 1) != std::string::npos) return false;
  *ns = key.substr(0, pos);
  *name = key.substr(pos + 1);
  return true;
}

static const Json* replica_specs(const Json& job) { return job.path({"spec", "pytorchReplicaSpecs"}); }

std::vector<std::string> replica_types(const Json& job) {
  std::vector<std::string> out;
  const Json* rs = replica_specs(job);
  if (!rs || !rs->is_object()) return out;
  for (const auto& kv : rs->as_object()) out.push_back(kv.first);
  // deterministic order: Master, Worker, then anything else alphabetically
  std::stable_sort(out.begin(), out.end(), [](const std::string& a, const std::string& b) {
    auto rank = [](const std::string& t) { return t == kReplicaMaster ? 0 : t == kReplicaWorker ? 1 : 2; };
    if (rank(a) != rank(b)) return rank(a) < rank(b);
    return a < b;
  });
  return out;
}

const Json* replica_spec(const Json& job, const std::string& rtype) {
  const Json* rs = replica_specs(job);
  return rs ? rs->get(rtype) : nullptr;
}

int32_t replicas_of(const Json& job, const std::string& rtype) {
  const Json* s = replica_spec(job, rtype);
  if (!s) return 0;
  return (int32_t)s->int_or("replicas", 1);
}

int32_t total_replicas(const Json& job) {
  int32_t n = 0;
  for (const auto& t : replica_types(job)) n += replicas_of(job, t);
  return n;
}

std::string restart_policy_of(const Json& job, const std::string& rtype) {
  const Json* s = replica_spec(job, rtype);
  return s ? s->str_or("restartPolicy") : "";
}

bool contains_master_spec(const Json& job) { return replica_spec(job, kReplicaMaster) != nullptr; }

std::optional<int32_t> port_of(const Json& job, const std::string& rtype) {
  const Json* s = replica_spec(job, rtype);
  if (!s) return std::nullopt;
  const Json* containers = s->path({"template", "spec", "containers"});
  if (!containers || !containers->is_array()) return std::nullopt;
  for (const auto& c : containers->as_array()) {
    if (c.str_or("name") != kDefaultContainerName) continue;
    const Json* ports = c.get("ports");
    if (!ports || !ports->is_array()) continue;
    for (const auto& p : ports->as_array())
      if (p.str_or("name") == kDefaultPortName) return (int32_t)p.int_or("containerPort", -1);
  }
  return std::nullopt;
}

// ---------------------------------------------------------------- defaults
static void set_default_port(Json& pod_spec) {
  Json* containers = pod_spec.get("containers");
  if (!containers || !containers->is_array() || containers->size() == 0) return;
  size_t index = 0;
  for (size_t i = 0; i < containers->size(); ++i) {
    if ((*containers)[i].str_or("name") == kDefaultContainerName) {
      index = i;
      break;
    }
  }
  Json& c = (*containers)[index];
  Json* ports = c.get("ports");
  if (ports && ports->is_array()) {
    for (const auto& p : ports->as_array())
      if (p.str_or("name") == kDefaultPortName) return;
  }
  Json port = Json::object();
  port["name"] = kDefaultPortName;
  port["containerPort"] = kDefaultPort;
  c["ports"].push_back(port);
}

static void set_type_name_to_camel_case(Json& specs, const std::string& typ) {
  std::string found;
  for (auto& kv : specs.as_object()) {
    if (iequals(kv.first, typ) && kv.first != typ) {
      found = kv.first;
      break;
    }
  }
  if (found.empty()) return;
  Json v = *specs.get(found);
  specs.erase(found);
  specs[typ] = v;
}

void set_defaults(Json& job) {
  Json& spec = job["spec"];
  if (!spec.is_object()) spec = Json::object();
  const Json* cpp = spec.get("cleanPodPolicy");
  if (!cpp || cpp->is_null()) spec["cleanPodPolicy"] = kCleanPodPolicyNone;
  Json* specs = spec.get("pytorchReplicaSpecs");
  if (!specs || !specs->is_object()) return;
  set_type_name_to_camel_case(*specs, kReplicaMaster);
  set_type_name_to_camel_case(*specs, kReplicaWorker);
  for (auto& kv : specs->as_object()) {
    Json& rs = kv.second;
    if (!rs.is_object()) continue;
    const Json* r = rs.get("replicas");
    if (!r || r->is_null()) rs["replicas"] = 1;
    if (rs.str_or("restartPolicy").empty()) rs["restartPolicy"] = kDefaultRestartPolicy;
    if (kv.first == kReplicaMaster) {
      Json* podspec = rs.path({"template", "spec"});
      if (podspec) set_default_port(*podspec);
    }
  }
}

// ---------------------------------------------------------------- validation
std::string validate_spec(const Json& spec) {
  const Json* specs = spec.get("pytorchReplicaSpecs");
  if (!specs || !specs->is_object()) return "PyTorchJobSpec is not valid";
  bool master_exists = false;
  for (const auto& kv : specs->as_object()) {
    const std::string& rtype = kv.first;
    const Json& value = kv.second;
    const Json* containers = value.is_object() ? value.path({"template", "spec", "containers"}) : nullptr;
    if (value.is_null() || !containers || !containers->is_array() || containers->size() == 0)
      return "PyTorchJobSpec is not valid: containers definition expected in " + rtype;
    if (rtype != kReplicaMaster && rtype != kReplicaWorker)
      return "PyTorchReplicaType is " + rtype + " but must be one of [Master Worker]";
    bool default_container_present = false;
    for (const auto& c : containers->as_array()) {
      if (c.str_or("image").empty())
        return "PyTorchJobSpec is not valid: Image is undefined in the container of " + rtype;
      if (c.str_or("name") == kDefaultContainerName) default_container_present = true;
    }
    if (!default_container_present)
      return std::string("PyTorchJobSpec is not valid: There is no container named ") +
             kDefaultContainerName + " in " + rtype;
    if (rtype == kReplicaMaster) {
      master_exists = true;
      const Json* r = value.get("replicas");
      if (r && r->is_number() && r->as_int() != 1)
        return "PyTorchJobSpec is not valid: There must be only 1 master replica";
    }
  }
  if (!master_exists) return "PyTorchJobSpec is not valid: Master ReplicaSpec must be present";
  return "";
}

// ---------------------------------------------------------------- naming
static std::string replace_slash(std::string s) {
  std::replace(s.begin(), s.end(), '/', '-');
  return s;
}

Json gen_labels(const std::string& name) {
  Json l = Json::object();
  l[kLabelGroupName] = kGroupName;
  l[kLabelJobName] = replace_slash(name);
  l[kLabelPyTorchJobName] = replace_slash(name);
  l[kLabelControllerName] = kControllerName;
  return l;
}

std::string gen_general_name(const std::string& name, const std::string& rt, const std::string& index) {
  return replace_slash(name + "-" + rt + "-" + index);
}

Json gen_owner_reference(const Json& job) {
  Json r = Json::object();
  r["apiVersion"] = kApiVersion;
  r["kind"] = kKind;
  r["name"] = job_name(job);
  r["uid"] = job_uid(job);
  r["controller"] = true;
  r["blockOwnerDeletion"] = true;
  return r;
}

std::string gen_expectation_pods_key(const std::string& key, const std::string& rtype) {
  return key + "/" + to_lower(rtype) + "/pods";
}
std::string gen_expectation_services_key(const std::string& key, const std::string& rtype) {
  return key + "/" + to_lower(rtype) + "/services";
}
std::string gen_pod_group_name(const std::string& name) { return name; }

// ---------------------------------------------------------------- status
ReplicaStatus* JobStatus::replica(const std::string& rtype) {
  for (auto& kv : replica_statuses)
    if (kv.first == rtype) return &kv.second;
  return nullptr;
}
ReplicaStatus& JobStatus::ensure_replica(const std::string& rtype) {
  if (ReplicaStatus* r = replica(rtype)) return *r;
  replica_statuses.emplace_back(rtype, ReplicaStatus{});
  return replica_statuses.back().second;
}

JobStatus JobStatus::from_json(const Json& j) {
  JobStatus s;
  if (!j.is_object()) return s;
  if (const Json* cs = j.get("conditions"); cs && cs->is_array()) {
    for (const auto& c : cs->as_array()) {
      JobCondition jc;
      jc.type = c.str_or("type");
      jc.status = c.str_or("status");
      jc.reason = c.str_or("reason");
      jc.message = c.str_or("message");
      jc.last_update_time = c.str_or("lastUpdateTime");
      jc.last_transition_time = c.str_or("lastTransitionTime");
      s.conditions.push_back(jc);
    }
  }
  if (const Json* rs = j.get("replicaStatuses"); rs && rs->is_object()) {
    for (const auto& kv : rs->as_object()) {
      ReplicaStatus r;
      r.active = (int32_t)kv.second.int_or("active", 0);
      r.succeeded = (int32_t)kv.second.int_or("succeeded", 0);
      r.failed = (int32_t)kv.second.int_or("failed", 0);
      s.replica_statuses.emplace_back(kv.first, r);
    }
  }
  auto opt = [&](const char* k) -> std::optional<std::string> {
    const Json* v = j.get(k);
    if (v && v->is_string()) return v->as_string();
    return std::nullopt;
  };
  s.start_time = opt("startTime");
  s.completion_time = opt("completionTime");
  s.last_reconcile_time = opt("lastReconcileTime");
  return s;
}

Json JobStatus::to_json() const {
  Json j = Json::object();
  Json conds = Json::array();
  for (const auto& c : conditions) {
    Json o = Json::object();
    o["type"] = c.type;
    o["status"] = c.status;
    if (!c.reason.empty()) o["reason"] = c.reason;
    if (!c.message.empty()) o["message"] = c.message;
    o["lastUpdateTime"] = c.last_update_time;
    o["lastTransitionTime"] = c.last_transition_time;
    conds.push_back(o);
  }
  j["conditions"] = conds;
  Json rs = Json::object();
  for (const auto& kv : replica_statuses) {
    Json o = Json::object();  // omitempty, like the Go type
    if (kv.second.active) o["active"] = kv.second.active;
    if (kv.second.succeeded) o["succeeded"] = kv.second.succeeded;
    if (kv.second.failed) o["failed"] = kv.second.failed;
    rs[kv.first] = o;
  }
  j["replicaStatuses"] = rs;
  if (start_time) j["startTime"] = *start_time;
  if (completion_time) j["completionTime"] = *completion_time;
  if (last_reconcile_time) j["lastReconcileTime"] = *last_reconcile_time;
  return j;
}

bool JobStatus::operator==(const JobStatus& o) const { return to_json() == o.to_json(); }

JobCondition new_condition(const std::string& type, const std::string& reason,
                           const std::string& message, int64_t now) {
  JobCondition c;
  c.type = type;
  c.status = "True";
  c.reason = reason;
  c.message = message;
  c.last_update_time = format_time(now);
  c.last_transition_time = format_time(now);
  return c;
}

bool has_condition(const JobStatus& s, const std::string& type) {
  for (const auto& c : s.conditions)
    if (c.type == type && c.status == "True") return true;
  return false;
}
bool is_succeeded(const JobStatus& s) { return has_condition(s, kJobSucceeded); }
bool is_failed(const JobStatus& s) { return has_condition(s, kJobFailed); }

std::vector<JobCondition> filter_out_condition(const std::vector<JobCondition>& conds,
                                               const std::string& type) {
  std::vector<JobCondition> out;
  for (auto c : conds) {
    if (type == kJobRestarting && c.type == kJobRunning) continue;
    if (type == kJobRunning && c.type == kJobRestarting) continue;
    if (c.type == type) continue;
    if ((type == kJobFailed || type == kJobSucceeded) && c.type == kJobRunning) c.status = "False";
    out.push_back(c);
  }
  return out;
}

void set_condition(JobStatus& s, JobCondition c) {
  if (is_failed(s) || is_succeeded(s)) return;
  const JobCondition* cur = nullptr;
  for (const auto& x : s.conditions)
    if (x.type == c.type) {
      cur = &x;
      break;
    }
  if (cur && cur->status == c.status && cur->reason == c.reason) return;
  if (cur && cur->status == c.status) c.last_transition_time = cur->last_transition_time;
  auto conds = filter_out_condition(s.conditions, c.type);
  conds.push_back(c);
  s.conditions = std::move(conds);
}

// ---------------------------------------------------------------- pods
std::string pod_phase(const Json& pod) {
  const Json* st = pod.get("status");
  return st ? st->str_or("phase") : "";
}

bool is_pod_active(const Json& pod) {
  std::string ph = pod_phase(pod);
  const Json* del = pod.path({"metadata", "deletionTimestamp"});
  return ph != "Succeeded" && ph != "Failed" && (!del || del->is_null());
}

bool is_retryable_exit_code(int32_t code) {
  if (code == 1 || code == 2 || code == 126 || code == 127 || code == 128 || code == 139) return false;
  if (code == 130 || code == 137 || code == 143) return true;
  if (code == 138) return true;  // SIGUSR1: user-defined retryable failure
  return false;
}

}  // namespace pto
