// PyTorchJob controller: informers + rate-limited work queue + expectations around
// the pure reconcile() core, applying its actions through the Kubernetes API.
//
// Parity map (jiaqianjing/pytorch-operator):
//   construction / Run / workers      pkg/controller.v1/pytorch/controller.go:104-285
//   syncPyTorchJob                    controller.go:290-332 (+ satisfiedExpectations :497-516)
//   job handlers                      job.go:35-150
//   pod / service handlers            tf-operator/pkg/common/jobcontroller/pod.go:20-160, service.go:17-66
//   claim / adopt / release           tf-operator/.../pod.go:165-196, k8s controller_ref_manager.go
//   pod / service / podgroup control  tf-operator/pkg/control/*.go, jobcontroller.go:224-278
//   events                            record.EventRecorder (async sink here)
#pragma once

#include <atomic>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "pto/expectations.hpp"
#include "pto/informer.hpp"
#include "pto/kube.hpp"
#include "pto/reconcile.hpp"
#include "pto/workqueue.hpp"

namespace pto {

struct ControllerOptions {
  std::string watch_namespace;     // "" = all namespaces (--namespace)
  int threadiness = 1;             // --threadiness
  double job_resync_s = 30.0;      // unstructured job informer resync (informer.go:24)
  double resync_s = 12 * 3600.0;   // --resyc-period (pods/services)
  ControllerConfig cfg;
};

class EventSink {
 public:
  explicit EventSink(KubeClient* c);
  ~EventSink();
  void record(const Json& involved, const Event& e);
  void flush(double timeout_s);

 private:
  void loop();
  KubeClient* client_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Json> q_;
  bool stop_ = false;
  int inflight_ = 0;
  std::thread th_;
};

class PyTorchController {
 public:
  // `core` serves pods/services/events/podgroups, `jobs` the PyTorchJob resource: two
  // clients with independent rate limiters, like the reference's kubeClientSet and
  // pytorchJobClientSet (app/server.go:createClientSets).  jobs may equal core.
  PyTorchController(KubeClient* core, KubeClient* jobs, ControllerOptions opts);
  ~PyTorchController();

  void start_informers();
  bool wait_for_cache_sync(double timeout_s);
  // Blocks until *stop becomes true (workers: threadiness threads).
  void run(const std::atomic<bool>* stop);
  // One sync of key; returns true when the key should be forgotten.
  bool sync(const std::string& key);
  RateLimitedQueue& queue() { return queue_; }
  EventSink& events() { return events_; }

 private:
  void enqueue(const Json& job);
  // the PodGroup resource of the configured gang API (--gang-podgroup-api)
  const Resource& podgroups() const {
    return o_.cfg.gang_podgroup_api == "volcano" ? kVolcanoPodGroups : kPodGroups;
  }
  void add_job(const Json& obj);
  void update_job(const Json& old_obj, const Json& cur);
  void delete_job(const Json& obj);
  void add_pod(const Json& pod);
  void update_pod(const Json& old_pod, const Json& cur);
  void delete_pod(const Json& pod);
  void add_service(const Json& svc);
  void delete_service(const Json& svc);
  std::optional<Json> resolve_controller_ref(const Json& obj);
  std::vector<Json> claim(const Json& job, Informer* inf, const Resource& res);
  bool satisfied_expectations(const Json& job);
  std::string apply(Json& job, ReconcileResult& r);
  std::string write_status(Json& job, const Json& status);

  KubeClient* client_;
  KubeClient* jclient_;
  ControllerOptions o_;
  Expectations exp_;
  RateLimitedQueue queue_;
  EventSink events_;
  std::unique_ptr<Informer> jobs_, pods_, services_;
};

}  // namespace pto
