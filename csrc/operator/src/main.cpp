// pytorch-operator: the PyTorchJob operator binary.
// Reference: cmd/pytorch-operator.v1/main.go + app/server.go (Run, createClientSets,
// checkCRDExists, leader election) and tf-operator/pkg/util/signals.
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <thread>
#include <unistd.h>

#include "pto/api.hpp"
#include "pto/controller.hpp"
#include "pto/http.hpp"
#include "pto/kube.hpp"
#include "pto/leader.hpp"
#include "pto/log.hpp"
#include "pto/metrics.hpp"
#include "pto/options.hpp"

using namespace pto;

namespace {
std::atomic<bool> g_stop{false};
std::atomic<int> g_signals{0};

void on_signal(int) {
  // first signal: graceful stop; second: exit(1) (tf-operator/pkg/util/signals/signal.go:29-43)
  if (g_signals.fetch_add(1) >= 1) _exit(1);
  g_stop.store(true);
}

constexpr const char* kVersion = "v0.1.0-alpha";  // tf-operator/pkg/version/version.go:22
constexpr const char* kAppVersion = "0.3.0+git";  // version/version.go (repo root)

void print_version() {
  std::printf("API Version: %s\n", kGroupVersion);
  std::printf("Version: %s\n", kVersion);
  std::printf("Git SHA: %s\n", "Not provided.");
  std::printf("Go Version: n/a (C++17, %s %d.%d)\n", "g++", __GNUC__, __GNUC_MINOR__);
  std::printf("Go OS/Arch: linux/amd64\n");
}

LogLevel level_from(const std::string& s) {
  if (s == "debug") return LogLevel::Debug;
  if (s == "warning" || s == "warn") return LogLevel::Warn;
  if (s == "error") return LogLevel::Error;
  return LogLevel::Info;
}
}  // namespace

int main(int argc, char** argv) {
  ServerOption opt;
  std::string perr = parse_flags(argc, argv, &opt);
  if (perr == "help") {
    std::fputs(usage().c_str(), stderr);
    return 0;
  }
  if (!perr.empty()) {
    std::fprintf(stderr, "%s\n%s", perr.c_str(), usage().c_str());
    return 2;
  }
  log_configure(opt.json_log_format, level_from(opt.log_level));
  if (opt.print_version) {
    print_version();
    return 0;
  }

  // /metrics (promhttp equivalent) + /healthz
  HttpServer monitor("", opt.monitoring_port, [](const std::string& m, const std::string& path, const std::string&) {
    HttpServer::Reply r;
    if (path == "/metrics" || path.rfind("/metrics?", 0) == 0) {
      r.content_type = "text/plain; version=0.0.4; charset=utf-8";
      r.body = Metrics::instance().exposition();
    } else if (path == "/healthz") {
      r.body = "ok\n";
    } else {
      r.status = 404;
      r.body = "404 page not found\n";
    }
    return r;
  });
  LOG_INFO("Setting up client for monitoring on port: %d", opt.monitoring_port);
  std::string merr;
  if (!monitor.start(&merr)) LOG_ERROR("Monitoring endpoint setup failure: %s", merr.c_str());

  const char* kns = std::getenv(kEnvKubeflowNamespace);
  std::string lock_ns = kns && *kns ? kns : "default";
  if (!(kns && *kns)) LOG_INFO("EnvKubeflowNamespace not set, use default namespace");
  LOG_INFO("API Version: %s Version: %s", kGroupVersion, kVersion);
  (void)kAppVersion;

  struct sigaction sa{};
  sa.sa_handler = on_signal;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGINT, &sa, nullptr);
  sigaction(SIGTERM, &sa, nullptr);

  if (const char* kc = std::getenv("KUBECONFIG"); kc && *kc) opt.kubeconfig = kc;
  std::string cerr;
  auto kcfg = load_kube_config(opt.master_url, opt.kubeconfig, &cerr);
  if (!kcfg) {
    LOG_ERROR("Error building kubeconfig: %s", cerr.c_str());
    return 1;
  }
  KubeClient client(*kcfg, opt.qps, opt.burst);       // pods / services / events / podgroups
  KubeClient job_client(*kcfg, opt.qps, opt.burst);   // pytorchjobs (own rate limiter)
  KubeClient lease_client(*kcfg, opt.qps, opt.burst); // leader election

  // checkCRDExists (server.go:201-213): a NotFound on LIST means the CRD is missing.
  {
    ApiError err;
    if (!job_client.list(kPyTorchJobs, opt.namespace_, "", &err)) {
      LOG_ERROR("list pytorchjobs: %s", err.message.c_str());
      if (err.not_found()) {
        LOG_INFO("CRD doesn't exist. Exiting");
        return 1;
      }
    }
  }

  ControllerOptions co;
  co.watch_namespace = opt.namespace_;
  co.threadiness = opt.threadiness;
  co.resync_s = opt.resync_period_s;
  co.cfg.enable_gang_scheduling = opt.enable_gang_scheduling;
  co.cfg.gang_scheduler_name = opt.gang_scheduler_name;
  co.cfg.gang_podgroup_api = opt.gang_podgroup_api;
  co.cfg.init_container_image = opt.init_container_image;
  co.cfg.inject_rccl_env = opt.inject_rccl_env;
  co.cfg.xgmi_pod_topology = opt.xgmi_pod_topology;
  if (opt.rccl_env_set) co.cfg.rccl_env = opt.rccl_env;
  {
    std::ifstream f(opt.init_container_template_file);
    if (f) {
      std::stringstream ss;
      ss << f.rdbuf();
      co.cfg.init_container_template = ss.str();
      LOG_INFO("Using init container template from %s", opt.init_container_template_file.c_str());
    } else {
      LOG_INFO("Using default init container template");
    }
  }
  PyTorchController tc(&client, &job_client, co);
  tc.start_informers();

  auto run = [&] { tc.run(&g_stop); };
  if (opt.leader_elect) {
    LeaderElectionConfig lc;
    lc.ns = lock_ns;
    lc.lease_s = opt.lease_duration_s;
    lc.renew_deadline_s = opt.renew_deadline_s;
    lc.retry_s = opt.retry_period_s;
    LeaderElector le(&lease_client, lc);
    le.run(run, [] {
      LOG_ERROR("leader election lost");
      std::fflush(stderr);
      _exit(1);  // log.Fatalf in the reference: the Deployment restarts us
    }, &g_stop);
  } else {
    Metrics::instance().set("pytorch_operator_is_leader", 1);
    run();
  }
  tc.events().flush(2.0);
  monitor.stop();
  LOG_INFO("pytorch-operator stopped");
  return 0;
}
