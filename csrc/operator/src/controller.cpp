#include "pto/controller.hpp"

#include <chrono>
#include <map>

#include "pto/log.hpp"
#include "pto/metrics.hpp"

namespace pto {

namespace {
double mono() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

std::string sel_from(const Json& labels) {
  std::string s;
  for (const auto& kv : labels.as_object()) {
    if (!s.empty()) s += ",";
    s += kv.first + "=" + kv.second.as_string();
  }
  return s;
}

bool labels_match(const Json& obj, const Json& selector) {
  const Json* l = obj.path({"metadata", "labels"});
  for (const auto& kv : selector.as_object()) {
    const Json* v = l ? l->get(kv.first) : nullptr;
    if (!v || !v->is_string() || v->as_string() != kv.second.as_string()) return false;
  }
  return true;
}

const Json* controller_ref(const Json& obj) {
  const Json* refs = obj.path({"metadata", "ownerReferences"});
  if (!refs || !refs->is_array()) return nullptr;
  for (const auto& r : refs->as_array())
    if (r.bool_or("controller", false)) return &r;
  return nullptr;
}

std::string meta_str(const Json& obj, const char* k) {
  const Json* md = obj.get("metadata");
  return md ? md->str_or(k) : "";
}

bool being_deleted(const Json& obj) {
  const Json* d = obj.path({"metadata", "deletionTimestamp"});
  return d && !d->is_null();
}
}  // namespace

// ------------------------------------------------------------------ events
EventSink::EventSink(KubeClient* c) : client_(c) { th_ = std::thread([this] { loop(); }); }

EventSink::~EventSink() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (th_.joinable()) th_.join();
}

void EventSink::record(const Json& involved, const Event& e) {
  static std::atomic<uint64_t> seq{0};
  Json ev = Json::object();
  ev["apiVersion"] = "v1";
  ev["kind"] = "Event";
  Json md = Json::object();
  std::string name = meta_str(involved, "name");
  char suffix[32];
  std::snprintf(suffix, sizeof suffix, ".%llx%04llx", (unsigned long long)now_ms(),
                (unsigned long long)(seq++ & 0xffff));
  md["name"] = name + suffix;
  md["namespace"] = meta_str(involved, "namespace");
  ev["metadata"] = md;
  Json io = Json::object();
  io["kind"] = involved.str_or("kind", e.kind);
  io["apiVersion"] = involved.str_or("apiVersion", kApiVersion);
  io["namespace"] = meta_str(involved, "namespace");
  io["name"] = name;
  io["uid"] = meta_str(involved, "uid");
  ev["involvedObject"] = io;
  ev["reason"] = e.reason;
  ev["message"] = e.message;
  ev["type"] = e.type;
  Json src = Json::object();
  src["component"] = kControllerName;
  ev["source"] = src;
  ev["firstTimestamp"] = format_time(now_ms());
  ev["lastTimestamp"] = format_time(now_ms());
  ev["count"] = 1;
  PTO_LOG(LogLevel::Info, fields_for_job(meta_str(involved, "namespace"), name),
          "Event(%s): type: '%s' reason: '%s' %s", name.c_str(), e.type.c_str(), e.reason.c_str(),
          e.message.c_str());
  {
    std::lock_guard<std::mutex> g(mu_);
    if (q_.size() > 4096) q_.pop_front();  // bounded: events are best effort
    q_.push_back(ev);
  }
  cv_.notify_one();
}

void EventSink::flush(double timeout_s) {
  double end = mono() + timeout_s;
  while (mono() < end) {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (q_.empty() && inflight_ == 0) return;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
}

// Posts events on its own thread.  Repeats are aggregated like client-go's EventCorrelator
// (vendor/k8s.io/client-go/tools/record/events_cache.go): an event with the same involved
// object, type, reason and message as one posted less than kEventDedupS ago is a PATCH of
// that Event's count and lastTimestamp, not a new object -- a crash-looping job does not
// flood the namespace.  The cache is owned by this thread (no locking) and bounded.
void EventSink::loop() {
  constexpr double kEventDedupS = 600.0;
  constexpr size_t kCacheMax = 4096;
  struct Seen {
    std::string name, ns;
    long long count;
    double last;
  };
  std::map<std::string, Seen> seen;
  while (true) {
    Json ev;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
      // on shutdown the queue is dropped (main() already gave flush() its bounded drain):
      // posting a backlog through the client's 5-qps limiter could hold the exit for tens
      // of seconds under job churn, like a broadcaster that outlives its process
      if (stop_ || q_.empty()) return;
      ev = q_.front();
      q_.pop_front();
      inflight_++;
    }
    const Json* io = ev.get("involvedObject");
    const std::string ns = meta_str(ev, "namespace");
    const std::string key = ns + "\x1f" + (io ? io->str_or("uid") + "\x1f" + io->str_or("name") : "") + "\x1f" +
                            ev.str_or("type") + "\x1f" + ev.str_or("reason") + "\x1f" + ev.str_or("message");
    const double now = mono();
    ApiError err;
    bool done = false;
    auto it = seen.find(key);
    if (it != seen.end() && now - it->second.last < kEventDedupS) {
      Json patch = Json::object();
      patch["count"] = it->second.count + 1;
      patch["lastTimestamp"] = ev.str_or("lastTimestamp");
      if (client_->patch_merge(kEvents, it->second.ns, it->second.name, patch, &err)) {
        it->second.count++;
        it->second.last = now;
        done = true;
      }
    }
    if (!done) {
      if (seen.size() >= kCacheMax) {  // drop the stalest entry
        auto oldest = seen.begin();
        for (auto j = seen.begin(); j != seen.end(); ++j)
          if (j->second.last < oldest->second.last) oldest = j;
        seen.erase(oldest);
      }
      ApiError e2;
      if (client_->create(kEvents, ns, ev, &e2)) seen[key] = Seen{meta_str(ev, "name"), ns, 1, now};
    }
    std::lock_guard<std::mutex> g(mu_);
    inflight_--;
  }
}

// ------------------------------------------------------------------ controller
PyTorchController::PyTorchController(KubeClient* core, KubeClient* jobs, ControllerOptions opts)
    : client_(core), jclient_(jobs ? jobs : core), o_(std::move(opts)), events_(core) {
  Informer::Handlers jh{[this](const Json& o) { add_job(o); },
                        [this](const Json& a, const Json& b) { update_job(a, b); },
                        [this](const Json& o) { delete_job(o); }};
  jobs_ = std::make_unique<Informer>(jclient_, kPyTorchJobs, o_.watch_namespace, "", o_.job_resync_s, jh);
  Informer::Handlers ph{[this](const Json& o) { add_pod(o); },
                        [this](const Json& a, const Json& b) { update_pod(a, b); },
                        [this](const Json& o) { delete_pod(o); }};
  const std::string sel = std::string(kLabelGroupName) + "=" + kGroupName;
  pods_ = std::make_unique<Informer>(client_, kPods, o_.watch_namespace, sel, o_.resync_s, ph);
  Informer::Handlers sh{[this](const Json& o) { add_service(o); },
                        [this](const Json&, const Json&) {},  // UpdateService: no-op (reference)
                        [this](const Json& o) { delete_service(o); }};
  services_ = std::make_unique<Informer>(client_, kServices, o_.watch_namespace, sel, o_.resync_s, sh);
}

PyTorchController::~PyTorchController() {
  queue_.shutdown();
  if (jobs_) jobs_->stop();
  if (pods_) pods_->stop();
  if (services_) services_->stop();
}

void PyTorchController::start_informers() {
  jobs_->start();
  pods_->start();
  services_->start();
}

bool PyTorchController::wait_for_cache_sync(double timeout_s) {
  return jobs_->wait_for_sync(timeout_s) && pods_->wait_for_sync(timeout_s) &&
         services_->wait_for_sync(timeout_s);
}

void PyTorchController::enqueue(const Json& job) { queue_.add(job_key(job)); }

// ---- job handlers (job.go:35-150)
void PyTorchController::add_job(const Json& obj) {
  JobAddedResult r = on_job_added(obj, now_ms());
  for (const auto& e : r.events) events_.record(obj, e);
  if (!r.valid) {
    PTO_LOG(LogLevel::Error, fields_for_job(job_namespace(obj), job_name(obj)),
            "Failed to convert the PyTorchJob: %s", r.error.c_str());
    // Log the failure to conditions: write the Failed status through the raw REST path.
    const Json* st = obj.get("status");
    JobStatus cur = JobStatus::from_json(st ? *st : Json());
    if (!is_failed(cur)) {
      Json job = obj;
      job["status"] = r.status;
      ApiError err;
      if (auto out = jclient_->update_status(kPyTorchJobs, job_namespace(obj), job, &err)) jobs_->update_cache(*out);
      else LOG_ERROR("Could not update the PyTorchJob: %s", err.message.c_str());
    }
    return;
  }
  Json job = obj;
  job["status"] = r.status;  // Created condition on the cached copy; persisted by the first sync
  jobs_->update_cache(job);
  PTO_LOG(LogLevel::Info, fields_for_job(job_namespace(obj), job_name(obj), job_uid(obj)),
          "PyTorchJob %s is created.", job_name(obj).c_str());
  enqueue(job);
  Metrics::instance().inc("pytorch_operator_jobs_created_total", r.metrics.created);
}

void PyTorchController::update_job(const Json& old_obj, const Json& cur) {
  enqueue(cur);
  double d = deadline_requeue_on_update(old_obj, cur, now_ms());
  if (d >= 0) {
    LOG_INFO("job ActiveDeadlineSeconds updated, will rsync after %.0f seconds", d);
    queue_.add_after(job_key(cur), d);
  }
}

void PyTorchController::delete_job(const Json& obj) { enqueue(obj); }

// ---- pod / service handlers (tf-operator jobcontroller/pod.go, service.go)
std::optional<Json> PyTorchController::resolve_controller_ref(const Json& obj) {
  const Json* ref = controller_ref(obj);
  if (!ref || ref->str_or("kind") != kKind) return std::nullopt;
  auto job = jobs_->get(meta_str(obj, "namespace"), ref->str_or("name"));
  if (!job || job_uid(*job) != ref->str_or("uid")) return std::nullopt;
  return job;
}

static std::string rtype_label(const Json& obj) {
  const Json* v = obj.path({"metadata", "labels", kLabelReplicaType});
  return v && v->is_string() ? v->as_string() : "";
}

void PyTorchController::add_pod(const Json& pod) {
  if (being_deleted(pod)) {
    delete_pod(pod);
    return;
  }
  auto job = resolve_controller_ref(pod);
  if (!job) return;  // orphans are adopted by the next sync of a matching job
  std::string rt = rtype_label(pod);
  if (rt.empty()) return;
  exp_.creation_observed(gen_expectation_pods_key(job_key(*job), rt));
  enqueue(*job);
}

void PyTorchController::update_pod(const Json& old_pod, const Json& cur) {
  if (meta_str(old_pod, "resourceVersion") == meta_str(cur, "resourceVersion") &&
      !meta_str(cur, "resourceVersion").empty())
    return;  // periodic resync: nothing changed
  const Json* oref = controller_ref(old_pod);
  const Json* cref = controller_ref(cur);
  bool changed = (oref == nullptr) != (cref == nullptr) ||
                 (oref && cref && oref->str_or("uid") != cref->str_or("uid"));
  if (changed && oref) {
    if (auto j = resolve_controller_ref(old_pod)) enqueue(*j);
  }
  if (auto j = resolve_controller_ref(cur)) enqueue(*j);
}

void PyTorchController::delete_pod(const Json& pod) {
  auto job = resolve_controller_ref(pod);
  if (!job) return;
  std::string rt = rtype_label(pod);
  if (rt.empty()) return;
  exp_.deletion_observed(gen_expectation_pods_key(job_key(*job), rt));
  enqueue(*job);
}

void PyTorchController::add_service(const Json& svc) {
  auto job = resolve_controller_ref(svc);
  if (!job) return;
  std::string rt = rtype_label(svc);
  if (rt.empty()) return;
  exp_.creation_observed(gen_expectation_services_key(job_key(*job), rt));
  enqueue(*job);
}

void PyTorchController::delete_service(const Json& svc) {
  // Reference: no-op (Q11).  Enqueueing the owner lets a deleted headless master
  // service be recreated; it changes nothing else observable.
  if (auto job = resolve_controller_ref(svc)) enqueue(*job);
}

// ---- claim / adopt / release (ControllerRefManager)
std::vector<Json> PyTorchController::claim(const Json& job, Informer* inf, const Resource& res) {
  std::vector<Json> out;
  const Json selector = gen_labels(job_name(job));
  const std::string uid = job_uid(job);
  const std::string ns = job_namespace(job);
  bool can_adopt_checked = false, can_adopt = false;
  for (auto obj : inf->list(ns)) {
    const Json* ref = controller_ref(obj);
    bool match = labels_match(obj, selector);
    if (ref) {
      if (ref->str_or("uid") != uid) continue;  // owned by someone else
      if (match) {
        out.push_back(obj);
        continue;
      }
      if (being_deleted(job)) continue;
      // release: drop our controller reference
      Json refs = Json::array();
      for (const auto& r : obj.path({"metadata", "ownerReferences"})->as_array())
        if (r.str_or("uid") != uid) refs.push_back(r);
      Json patch = Json::object();
      patch["metadata"]["ownerReferences"] = refs;
      ApiError err;
      client_->patch_merge(res, ns, meta_str(obj, "name"), patch, &err);
      continue;
    }
    if (!match || being_deleted(job) || being_deleted(obj)) continue;
    // orphan with matching labels: adopt after re-checking the job is not being deleted
    if (!can_adopt_checked) {
      ApiError err;
      auto fresh = jclient_->get(kPyTorchJobs, ns, job_name(job), &err);
      can_adopt = fresh && job_uid(*fresh) == uid && !being_deleted(*fresh);
      can_adopt_checked = true;
    }
    if (!can_adopt) continue;
    Json refs = obj.path({"metadata", "ownerReferences"}) ? *obj.path({"metadata", "ownerReferences"})
                                                           : Json::array();
    if (!refs.is_array()) refs = Json::array();
    refs.push_back(gen_owner_reference(job));
    Json patch = Json::object();
    patch["metadata"]["ownerReferences"] = refs;
    ApiError err;
    if (auto adopted = client_->patch_merge(res, ns, meta_str(obj, "name"), patch, &err)) out.push_back(*adopted);
  }
  return out;
}

// (Q6) OR across replica types and pods/services, like the reference.
bool PyTorchController::satisfied_expectations(const Json& job) {
  const std::string key = job_key(job);
  bool satisfied = false;
  for (const auto& rt : replica_types(job)) {
    satisfied = satisfied || exp_.satisfied(gen_expectation_pods_key(key, rt));
    satisfied = satisfied || exp_.satisfied(gen_expectation_services_key(key, rt));
  }
  return satisfied;
}

std::string PyTorchController::write_status(Json& job, const Json& status) {
  Json upd = job;
  upd["status"] = status;
  ApiError err;
  auto out = jclient_->update_status(kPyTorchJobs, job_namespace(job), upd, &err);
  if (!out) return "update status: " + err.message;
  jobs_->update_cache(*out);
  job = *out;
  return "";
}

std::string PyTorchController::apply(Json& job, ReconcileResult& r) {
  const std::string key = job_key(job);
  const std::string ns = job_namespace(job);
  auto& M = Metrics::instance();
  for (const auto& e : r.events) events_.record(job, e);
  ApiError err;
  if (r.create_podgroup) {
    if (!client_->create(podgroups(), ns, *r.create_podgroup, &err) && !err.already_exists())
      LOG_WARN("Sync PodGroup %s: %s", job_name(job).c_str(), err.message.c_str());
  }
  if (r.delete_podgroup) {
    ApiError e2;
    if (client_->get(podgroups(), ns, gen_pod_group_name(job_name(job)), &e2)) {
      if (client_->del(podgroups(), ns, gen_pod_group_name(job_name(job)), &e2))
        events_.record(job, {"Normal", "SuccessfulDeletePodGroup", "Deleted PodGroup: " + job_name(job)});
      else
        events_.record(job, {"Warning", "FailedDeletePodGroup", "Error deleting: " + e2.message});
    }
  }
  for (const auto& d : r.delete_pods) {
    ApiError e2;
    if (!client_->del(kPods, d.ns, d.name, &e2) && !e2.not_found()) {
      events_.record(job, {"Warning", "FailedDeletePod", "Error deleting: " + e2.message});
      return "unable to delete pods: " + e2.message;
    }
    if (!e2.not_found()) {
      events_.record(job, {"Normal", "SuccessfulDeletePod", "Deleted pod: " + d.name});
      PTO_LOG(LogLevel::Info, fields_for_pod(d.ns, job_name(job), job_uid(job), d.replica_type, d.name),
              "Deleted pod %s", d.name.c_str());
    }
  }
  // expectations: count creations per key, then set once (k8s ReplicaSet style)
  std::map<std::string, int> want;
  for (const auto& k : r.create_pod_expectation_keys) want[k]++;
  for (const auto& k : r.create_service_expectation_keys) want[k]++;
  for (const auto& kv : want) exp_.expect_creations(kv.first, kv.second);
  for (size_t i = 0; i < r.create_pods.size(); ++i) {
    ApiError e2;
    const std::string pname = meta_str(r.create_pods[i], "name");
    if (!client_->create(kPods, ns, r.create_pods[i], &e2)) {
      if (e2.timeout()) continue;  // created but initialisation timed out: the informer will see it
      exp_.creation_observed(r.create_pod_expectation_keys[i]);
      events_.record(job, {"Warning", "FailedCreatePod", "Error creating: " + e2.message});
      if (e2.already_exists()) continue;  // stale cache: the informer will deliver it
      return "create pod " + pname + ": " + e2.message;
    }
    events_.record(job, {"Normal", "SuccessfulCreatePod", "Created pod: " + pname});
    {
      const Json* lb = r.create_pods[i].path({"metadata", "labels"});
      PTO_LOG(LogLevel::Info,
              fields_for_pod(ns, job_name(job), job_uid(job), lb ? lb->str_or(kLabelReplicaType) : "", pname),
              "Created pod %s", pname.c_str());
    }
  }
  for (size_t i = 0; i < r.create_services.size(); ++i) {
    ApiError e2;
    const std::string sname = meta_str(r.create_services[i], "name");
    if (!client_->create(kServices, ns, r.create_services[i], &e2)) {
      if (e2.timeout()) continue;
      exp_.creation_observed(r.create_service_expectation_keys[i]);
      events_.record(job, {"Warning", "FailedCreateService", "Error creating: " + e2.message});
      if (e2.already_exists()) continue;
      return "unable to create services: " + e2.message;
    }
    events_.record(job, {"Normal", "SuccessfulCreateService", "Created service: " + sname});
  }
  for (const auto& d : r.delete_services) {
    ApiError e2;
    if (!client_->del(kServices, d.ns, d.name, &e2) && !e2.not_found()) {
      events_.record(job, {"Warning", "FailedDeleteService", "Error deleting: " + e2.message});
      return "unable to delete service: " + e2.message;
    }
    if (!e2.not_found()) events_.record(job, {"Normal", "SuccessfulDeleteService", "Deleted service: " + d.name});
  }
  if (!r.error.empty()) return r.error;
  if (r.delete_job) {
    ApiError e2;
    if (!jclient_->del(kPyTorchJobs, ns, job_name(job), &e2) && !e2.not_found())
      return "Cleanup PyTorchJob error: " + e2.message;
  }
  if (r.status_changed && !r.delete_job) {
    std::string e = write_status(job, r.status);
    if (!e.empty()) return e;
  }
  // a job's Succeeded / Failed / Restarting transition is counted once it is persisted: a status
  // write that loses a resourceVersion race requeues the key, and the retry (which still sees the
  // old status in the cache) would otherwise count the same transition again.  Failed and
  // restarted move together, as status.go:128-129 increments them
  M.inc("pytorch_operator_jobs_successful_total", r.metrics.successful);
  M.inc("pytorch_operator_jobs_failed_total", r.metrics.failed);
  M.inc("pytorch_operator_jobs_restarted_total", r.metrics.restarted);
  for (double d : r.requeue_after_s) queue_.add_after(key, d);
  if (r.requeue_rate_limited) queue_.add_rate_limited(key);
  return "";
}

bool PyTorchController::sync(const std::string& key) {
  const double t0 = mono();
  std::string ns, name;
  if (!split_key(key, &ns, &name) || ns.empty() || name.empty()) {
    LOG_ERROR("invalid job key %s: either namespace or name is missing", key.c_str());
    return true;
  }
  auto shared = jobs_->get(ns, name);
  if (!shared) {
    PTO_LOG(LogLevel::Info, fields_for_key(key), "PyTorchJob has been deleted: %s", key.c_str());
    Metrics::instance().inc("pytorch_operator_jobs_deleted_total");
    return true;
  }
  Json job = *shared;
  const bool needs_sync = satisfied_expectations(job);
  std::string err;
  if (needs_sync && !being_deleted(job)) {
    const Json* spec = job.get("spec");
    std::string verr = spec && spec->is_object() ? validate_spec(*spec) : "PyTorchJobSpec is not valid";
    if (!verr.empty()) {
      add_job(job);  // invalid spec: surfaces as Failed/InvalidPyTorchJobSpec
    } else {
      set_defaults(job);
      const Json orig_status = job.get("status") ? *job.get("status") : Json();
      JobStatus s = JobStatus::from_json(orig_status);
      if (!has_condition(s, kJobCreated) && !is_succeeded(s) && !is_failed(s) && s.conditions.empty()) {
        set_condition(s, new_condition(kJobCreated, kReasonCreated, "PyTorchJob " + name + " is created.", now_ms()));
        job["status"] = s.to_json();
      }
      ReconcileInput in;
      in.job = job;
      in.pods = claim(job, pods_.get(), kPods);
      in.services = claim(job, services_.get(), kServices);
      in.now = now_ms();
      in.requeues = queue_.num_requeues(key);
      if (o_.cfg.enable_gang_scheduling) {
        ApiError e2;
        in.podgroup_exists = client_->get(podgroups(), ns, gen_pod_group_name(name), &e2).has_value();
      }
      PTO_LOG(LogLevel::Info, fields_for_job(ns, name, job_uid(job)), "Reconcile PyTorchJobs %s", name.c_str());
      ReconcileResult r = reconcile(in, o_.cfg);
      // persist a Created condition added above even when reconcile saw no other change
      if (!(JobStatus::from_json(orig_status) == JobStatus::from_json(r.status))) r.status_changed = true;
      err = apply(job, r);
    }
  }
  const double dt = mono() - t0;
  Metrics::instance().observe_sync(dt);
  PTO_LOG(LogLevel::Info, fields_for_key(key), "Finished syncing job \"%s\" (%.3fms)", key.c_str(), dt * 1e3);
  if (!err.empty()) {
    PTO_LOG(LogLevel::Warn, fields_for_key(key), "sync error: %s", err.c_str());
    Metrics::instance().inc("pytorch_operator_reconcile_errors_total");
    return false;
  }
  return true;
}

void PyTorchController::run(const std::atomic<bool>* stop) {
  LOG_INFO("Starting PyTorchJob controller");
  LOG_INFO("Waiting for informer caches to sync");
  while (!wait_for_cache_sync(1.0)) {
    if (stop->load()) return;
  }
  LOG_INFO("Starting %d workers", o_.threadiness);
  std::vector<std::thread> workers;
  for (int i = 0; i < std::max(1, o_.threadiness); ++i) {
    workers.emplace_back([this, stop] {
      while (!stop->load()) {
        std::string key;
        if (!queue_.get(&key, 0.25)) {
          if (queue_.shutting_down()) return;
          continue;
        }
        bool forget = false;
        try {
          forget = sync(key);
        } catch (const std::exception& e) {
          LOG_ERROR("sync %s threw: %s", key.c_str(), e.what());
        }
        if (forget) queue_.forget(key);
        else queue_.add_rate_limited(key);
        queue_.done(key);
      }
    });
  }
  for (auto& w : workers) w.join();
  LOG_INFO("Shutting down workers");
}

}  // namespace pto
