// C++ unit tests for the operator runtime (run by tests/test_operator_native.py; also
// built with -fsanitize=address,undefined / thread there).
#include <atomic>
#include <chrono>
#include <cstdio>
#include <functional>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "pto/util.hpp"
#include "pto/api.hpp"
#include "pto/expectations.hpp"
#include "pto/http.hpp"
#include "pto/json.hpp"
#include "pto/metrics.hpp"
#include "pto/options.hpp"
#include "pto/reconcile.hpp"
#include "pto/workqueue.hpp"
#include "pto/yaml_lite.hpp"

using namespace pto;

static int g_fail = 0, g_pass = 0;
#define CHECK(cond)                                                         \
  do {                                                                      \
    if (cond) {                                                             \
      ++g_pass;                                                             \
    } else {                                                                \
      ++g_fail;                                                             \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
    }                                                                       \
  } while (0)

static void test_json() {
  Json j = Json::parse(R"({"a":[1,2,{"b":"c\né"}],"d":-1.5e3,"e":true,"f":null,"g":9007199254740993})");
  CHECK(j["a"][2]["b"].as_string() == "c\n\xc3\xa9");
  CHECK(j["d"].as_double() == -1500.0);
  CHECK(j["g"].as_int() == 9007199254740993LL);
  CHECK(Json::parse(j.dump()) == j);
  Json o = Json::object();
  Json* first = &o["x"];
  for (int i = 0; i < 100; ++i) o["k" + std::to_string(i)] = i;
  *first = "still-valid";  // deque storage: inserting keeps member pointers valid
  CHECK(o["x"].as_string() == "still-valid");
  bool threw = false;
  try {
    Json::parse("{\"a\":}");
  } catch (const JsonError&) {
    threw = true;
  }
  CHECK(threw);
  Json t = Json::parse(R"({"a":{"b":1,"c":2},"d":3})");
  json_merge_patch(t, Json::parse(R"({"a":{"b":null,"e":5},"d":[1]})"));
  CHECK(t == Json::parse(R"({"a":{"c":2,"e":5},"d":[1]})"));
}

static void test_yaml() {
  Json y = yaml_parse(R"(
apiVersion: kubeflow.org/v1
kind: PyTorchJob
metadata:
  name: pytorch-dist-mnist-gloo   # comment
spec:
  pytorchReplicaSpecs:
    Master:
      replicas: 1
      restartPolicy: OnFailure
      template:
        spec:
          containers:
            - name: pytorch
              image: "img:1.0"
              args: ["--backend", "gloo"]
              resources:
                limits:
                  amd.com/gpu: 1
)");
  CHECK(y["metadata"]["name"].as_string() == "pytorch-dist-mnist-gloo");
  const Json& c = y["spec"]["pytorchReplicaSpecs"]["Master"]["template"]["spec"]["containers"][0];
  CHECK(c.str_or("image") == "img:1.0");
  CHECK(c.path({"args"})->size() == 2);
  CHECK(c.path({"resources", "limits", "amd.com/gpu"})->as_int() == 1);
}

static void test_options() {
  double s = 0;
  CHECK(parse_duration("12h", &s) && s == 43200);
  CHECK(parse_duration("1h30m", &s) && s == 5400);
  CHECK(parse_duration("500ms", &s) && s == 0.5);
  CHECK(!parse_duration("abc", &s));
  ServerOption o;
  const char* argv[] = {"pytorch-operator", "-alsologtostderr", "-v=1", "--monitoring-port=9000",
                        "--resyc-period", "30m", "--json-log-format=false", "--threadiness", "4"};
  CHECK(parse_flags(9, (char**)argv, &o) == "");
  CHECK(o.monitoring_port == 9000 && o.resync_period_s == 1800 && !o.json_log_format && o.threadiness == 4);
  const char* bad[] = {"x", "--nope"};
  CHECK(parse_flags(2, (char**)bad, &o).find("not defined") != std::string::npos);
}

static void test_workqueue_concurrency() {
  // a key is never processed by two workers at once, and every add is eventually processed
  RateLimitedQueue q;
  std::atomic<int> processed{0}, concurrent_violation{0};
  std::mutex m;
  std::set<std::string> in_flight;
  std::atomic<bool> stop{false};
  std::vector<std::thread> ws;
  for (int w = 0; w < 4; ++w) {
    ws.emplace_back([&] {
      std::string k;
      while (!stop.load()) {
        if (!q.get(&k, 0.05)) continue;
        {
          std::lock_guard<std::mutex> g(m);
          if (!in_flight.insert(k).second) concurrent_violation++;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(200));
        {
          std::lock_guard<std::mutex> g(m);
          in_flight.erase(k);
        }
        processed++;
        q.done(k);
      }
    });
  }
  for (int i = 0; i < 2000; ++i) q.add("job-" + std::to_string(i % 7));
  auto t0 = std::chrono::steady_clock::now();
  while (q.len() > 0 && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(5))
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  stop = true;
  for (auto& w : ws) w.join();
  CHECK(concurrent_violation.load() == 0);
  CHECK(processed.load() >= 7);
  q.shutdown();
  std::string k;
  CHECK(!q.get(&k, 0.01));
}

static void test_http_loopback() {
  HttpServer srv("127.0.0.1", 0, [](const std::string& m, const std::string& p, const std::string& body) {
    HttpServer::Reply r;
    r.body = m + " " + p + " " + body;
    return r;
  });
  std::string err;
  CHECK(srv.start(&err));
  Url u;
  CHECK(Url::parse("http://127.0.0.1:" + std::to_string(srv.port()), &u));
  HttpClient c(u);
  HttpResponse r = c.request("POST", "/x?y=1", "{\"a\":1}");
  CHECK(r.status == 200);
  CHECK(r.body == "POST /x?y=1 {\"a\":1}");
  srv.stop();
  Url v;
  CHECK(Url::parse("https://10.0.0.1:6443/base/", &v) && v.port == 6443 && v.base_path == "/base");
}

static void test_metrics() {
  Metrics::instance().inc("pytorch_operator_jobs_created_total");
  std::string e = Metrics::instance().exposition();
  CHECK(e.find("# TYPE pytorch_operator_jobs_created_total counter") != std::string::npos);
  CHECK(e.find("pytorch_operator_is_leader") != std::string::npos);
}

static void test_reconcile_smoke() {
  Json job = Json::parse(R"({"metadata":{"name":"j","namespace":"ns","uid":"u"},"spec":{"pytorchReplicaSpecs":{
    "Master":{"template":{"spec":{"containers":[{"name":"pytorch","image":"i"}]}}},
    "Worker":{"replicas":2,"template":{"spec":{"containers":[{"name":"pytorch","image":"i"}]}}}}}})");
  set_defaults(job);
  ReconcileInput in;
  in.job = job;
  in.now = 1700000000000LL;
  ControllerConfig cfg;
  ReconcileResult r = reconcile(in, cfg);
  CHECK(r.error.empty());
  CHECK(r.create_pods.size() == 3);
  CHECK(r.create_services.size() == 1);
  CHECK(r.status_changed);
  CHECK(r.status.path({"startTime"}) != nullptr);
}

// pkg/util/util_test.go:5-11 (TestRandString) + Pformat
static void test_util() {
  CHECK(rand_string(4).size() == 4);
  CHECK(rand_string(0).empty());
  const std::string r = rand_string(64);
  bool ok = true;
  for (char c : r) ok = ok && ((c >= '0' && c <= '9') || (c >= 'a' && c <= 'z'));
  CHECK(ok);
  CHECK(rand_string(16) != rand_string(16));
  CHECK(pformat(Json("plain")) == "plain");
  const Json o = Json::parse(R"({"a":1,"b":[true,null]})");
  CHECK(pformat(o) == o.dump(2));
  CHECK(Json::parse(pformat(o)).dump() == o.dump());
}

int main() {
  test_util();
  test_json();
  test_yaml();
  test_options();
  test_workqueue_concurrency();
  test_http_loopback();
  test_metrics();
  test_reconcile_smoke();
  std::printf("%d passed, %d failed\n", g_pass, g_fail);
  return g_fail == 0 ? 0 : 1;
}
