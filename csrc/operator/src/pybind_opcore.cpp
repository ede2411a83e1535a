// Python binding of the operator core (JSON in / JSON out), used by the test
// suite (tests/test_operator_*.py ports the reference's Go unit tests) and by
// the Python tooling (SDK validation, local cluster emulator).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "pto/api.hpp"
#include "pto/expectations.hpp"
#include "pto/reconcile.hpp"
#include "pto/workqueue.hpp"
#include "pto/yaml_lite.hpp"

namespace py = pybind11;
using namespace pto;

static Json J(const std::string& s) { return Json::parse(s); }

static ControllerConfig cfg_from(const std::string& s) {
  ControllerConfig c;
  if (s.empty()) return c;
  Json j = J(s);
  c.enable_gang_scheduling = j.bool_or("enableGangScheduling", false);
  c.gang_scheduler_name = j.str_or("gangSchedulerName", c.gang_scheduler_name);
  c.gang_podgroup_api = j.str_or("gangPodgroupApi", c.gang_podgroup_api);
  c.init_container_image = j.str_or("initContainerImage", c.init_container_image);
  c.init_container_template = j.str_or("initContainerTemplate", c.init_container_template);
  c.inject_rccl_env = j.bool_or("injectRcclEnv", false);
  c.xgmi_pod_topology = j.bool_or("xgmiPodTopology", false);
  if (const Json* re = j.get("rcclEnv"))
    if (re->is_object()) {
      c.rccl_env.clear();
      for (const auto& kv : re->as_object()) c.rccl_env.emplace_back(kv.first, kv.second.as_string());
    }
  return c;
}

static Json events_json(const std::vector<Event>& evs) {
  Json a = Json::array();
  for (const auto& e : evs) {
    Json o = Json::object();
    o["type"] = e.type;
    o["reason"] = e.reason;
    o["message"] = e.message;
    o["kind"] = e.kind;
    o["name"] = e.name;
    a.push_back(o);
  }
  return a;
}

static Json metrics_json(const MetricDeltas& m) {
  Json o = Json::object();
  o["created"] = m.created;
  o["deleted"] = m.deleted;
  o["successful"] = m.successful;
  o["failed"] = m.failed;
  o["restarted"] = m.restarted;
  return o;
}

static std::string py_reconcile(const std::string& job, const std::string& pods,
                                const std::string& services, int64_t now, int requeues,
                                const std::string& cfg, bool podgroup_exists) {
  ReconcileInput in;
  in.job = J(job);
  const Json pj = J(pods), sj = J(services);  // keep alive: range-for over a temporary's member dangles
  for (const auto& p : pj.as_array()) in.pods.push_back(p);
  for (const auto& s : sj.as_array()) in.services.push_back(s);
  in.now = now;
  in.requeues = requeues;
  in.podgroup_exists = podgroup_exists;
  ReconcileResult r = reconcile(in, cfg_from(cfg));
  Json o = Json::object();
  Json cp = Json::array();
  for (auto& p : r.create_pods) cp.push_back(p);
  o["createPods"] = cp;
  Json cpk = Json::array();
  for (auto& k : r.create_pod_expectation_keys) cpk.push_back(k);
  o["createPodExpectationKeys"] = cpk;
  Json dp = Json::array();
  for (auto& d : r.delete_pods) dp.push_back(d.ns + "/" + d.name);
  o["deletePods"] = dp;
  Json cs = Json::array();
  for (auto& s : r.create_services) cs.push_back(s);
  o["createServices"] = cs;
  Json ds = Json::array();
  for (auto& d : r.delete_services) ds.push_back(d.ns + "/" + d.name);
  o["deleteServices"] = ds;
  o["createPodGroup"] = r.create_podgroup ? *r.create_podgroup : Json();
  o["deletePodGroup"] = r.delete_podgroup;
  o["deleteJob"] = r.delete_job;
  o["statusChanged"] = r.status_changed;
  o["status"] = r.status;
  o["events"] = events_json(r.events);
  Json ra = Json::array();
  for (double d : r.requeue_after_s) ra.push_back(d);
  o["requeueAfter"] = ra;
  o["requeueRateLimited"] = r.requeue_rate_limited;
  o["metrics"] = metrics_json(r.metrics);
  o["error"] = r.error;
  return o.dump();
}

static std::string py_on_job_added(const std::string& job, int64_t now) {
  JobAddedResult r = on_job_added(J(job), now);
  Json o = Json::object();
  o["valid"] = r.valid;
  o["error"] = r.error;
  o["status"] = r.status;
  o["events"] = events_json(r.events);
  o["metrics"] = metrics_json(r.metrics);
  return o.dump();
}

PYBIND11_MODULE(_opcore, m) {
  m.doc() = "PyTorchJob operator core (C++): defaults, validation, reconcile";
  m.attr("API_VERSION") = kApiVersion;
  m.attr("KIND") = kKind;
  m.attr("PLURAL") = kPlural;
  m.attr("DEFAULT_PORT") = kDefaultPort;
  m.attr("DEFAULT_INIT_CONTAINER_TEMPLATE") = kDefaultInitContainerTemplate;
  m.def("set_defaults", [](const std::string& job) {
    Json j = J(job);
    set_defaults(j);
    return j.dump();
  });
  m.def("validate_spec", [](const std::string& spec) { return validate_spec(J(spec)); });
  m.def("reconcile", &py_reconcile, py::arg("job"), py::arg("pods") = "[]",
        py::arg("services") = "[]", py::arg("now") = 0, py::arg("requeues") = 0,
        py::arg("config") = "", py::arg("podgroup_exists") = false);
  m.def("on_job_added", &py_on_job_added, py::arg("job"), py::arg("now") = 0);
  m.def("deadline_requeue_on_update", [](const std::string& old, const std::string& cur, int64_t now) {
    return deadline_requeue_on_update(J(old), J(cur), now);
  });
  m.def("gen_labels", [](const std::string& n) { return gen_labels(n).dump(); });
  m.def("gen_general_name", &gen_general_name);
  m.def("gen_owner_reference", [](const std::string& job) { return gen_owner_reference(J(job)).dump(); });
  m.def("gen_expectation_pods_key", &gen_expectation_pods_key);
  m.def("gen_expectation_services_key", &gen_expectation_services_key);
  m.def("is_retryable_exit_code", &is_retryable_exit_code);
  m.def("build_pod", [](const std::string& job, const std::string& rtype, int index, const std::string& cfg) {
    std::vector<Event> evs;
    std::string err;
    Json p = build_pod(J(job), rtype, index, cfg_from(cfg), &evs, &err);
    if (!err.empty()) throw std::runtime_error(err);
    return p.dump();
  }, py::arg("job"), py::arg("rtype"), py::arg("index"), py::arg("config") = "");
  m.def("init_containers", [](const std::string& master_addr, const std::string& cfg) {
    std::string err;
    auto v = init_containers(cfg_from(cfg), master_addr, &err);
    if (!err.empty()) throw std::runtime_error(err);
    Json a = Json::array();
    for (auto& c : v) a.push_back(c);
    return a.dump();
  }, py::arg("master_addr"), py::arg("config") = "");
  m.def("past_backoff_limit", [](const std::string& job, const std::string& pods) {
    std::vector<Json> ps;
    const Json pj = J(pods);
    for (const auto& p : pj.as_array()) ps.push_back(p);
    return past_backoff_limit(J(job), ps);
  });
  m.def("update_status_single", [](const std::string& job, const std::string& rtype, int replicas,
                                   bool restart, int64_t now) {
    return update_status_single_json(J(job), rtype, replicas, restart, now).dump();
  });
  m.def("yaml_to_json", [](const std::string& y) { return yaml_parse(y).dump(); });
  m.def("json_roundtrip", [](const std::string& s) { return J(s).dump(); });
  m.def("format_time", &format_time);
  m.def("parse_time", [](const std::string& s) {
    auto v = parse_time(s);
    if (!v) throw std::runtime_error("bad time");
    return *v;
  });

  py::class_<Expectations>(m, "Expectations")
      .def(py::init<double>(), py::arg("ttl_s") = 300.0)
      .def("expect_creations", &Expectations::expect_creations)
      .def("expect_deletions", &Expectations::expect_deletions)
      .def("creation_observed", &Expectations::creation_observed)
      .def("deletion_observed", &Expectations::deletion_observed)
      .def("satisfied", &Expectations::satisfied)
      .def("delete", &Expectations::remove);

  py::class_<RateLimitedQueue>(m, "WorkQueue")
      .def(py::init<double, double, double, int>(), py::arg("base_delay_s") = 0.005,
           py::arg("max_delay_s") = 1000.0, py::arg("qps") = 10.0, py::arg("burst") = 100)
      .def("add", &RateLimitedQueue::add)
      .def("add_after", &RateLimitedQueue::add_after)
      .def("add_rate_limited", &RateLimitedQueue::add_rate_limited)
      .def("forget", &RateLimitedQueue::forget)
      .def("num_requeues", &RateLimitedQueue::num_requeues)
      .def("get", [](RateLimitedQueue& q, double timeout_s) {
        std::string key;
        bool ok;
        {
          py::gil_scoped_release rel;
          ok = q.get(&key, timeout_s);
        }
        if (!ok) return py::object(py::none());
        return py::object(py::str(key));
      }, py::arg("timeout_s") = -1.0)
      .def("done", &RateLimitedQueue::done)
      .def("len", &RateLimitedQueue::len)
      .def("shutdown", &RateLimitedQueue::shutdown)
      .def("when", &RateLimitedQueue::when);
}
