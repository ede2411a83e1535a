#include "pto/options.hpp"

#include <cstdlib>
#include <fstream>
#include <functional>
#include <map>

namespace pto {

bool parse_duration(const std::string& s, double* seconds) {
  if (s.empty()) return false;
  double total = 0;
  size_t i = 0;
  bool any = false;
  while (i < s.size()) {
    size_t j = i;
    while (j < s.size() && (std::isdigit((unsigned char)s[j]) || s[j] == '.')) ++j;
    if (j == i) return false;
    double v = std::atof(s.substr(i, j - i).c_str());
    size_t k = j;
    while (k < s.size() && std::isalpha((unsigned char)s[k])) ++k;
    std::string unit = s.substr(j, k - j);
    double mul;
    if (unit == "h") mul = 3600;
    else if (unit == "m") mul = 60;
    else if (unit == "s") mul = 1;
    else if (unit == "ms") mul = 1e-3;
    else if (unit == "us" || unit == "µs") mul = 1e-6;
    else if (unit == "ns") mul = 1e-9;
    else if (unit.empty() && v == 0) mul = 0;
    else return false;
    total += v * mul;
    any = true;
    i = k;
  }
  *seconds = total;
  return any;
}

namespace {
bool parse_bool(const std::string& v, bool* out) {
  if (v == "1" || v == "t" || v == "T" || v == "true" || v == "TRUE" || v == "True") return *out = true, true;
  if (v == "0" || v == "f" || v == "F" || v == "false" || v == "FALSE" || v == "False") return *out = false, true;
  return false;
}
}  // namespace

std::string usage() {
  return "Usage of pytorch-operator:\n"
         "  -kubeconfig string        The path of kubeconfig file\n"
         "  -master string            The url of the Kubernetes API server, will overrides any value in kubeconfig\n"
         "  -namespace string         The namespace to monitor pytorch jobs (default: all namespaces)\n"
         "  -threadiness int          How many threads to process the main logic (default 1)\n"
         "  -version                  Show version and quit\n"
         "  -json-log-format          Set true to use json style log format (default true)\n"
         "  -enable-gang-scheduling   Set true to enable gang scheduling\n"
         "  -gang-scheduler-name      The scheduler to gang-schedule jobs (default \"volcano\")\n"
         "  -gang-podgroup-api        PodGroup API of gang scheduling: kube-batch (scheduling.incubator.k8s.io/\n"
         "                            v1alpha1, default) or volcano (scheduling.volcano.sh/v1beta1)\n"
         "  -monitoring-port int      Endpoint port for displaying monitoring metrics (default 8443)\n"
         "  -resyc-period duration    Resync interval of the operator (default 12h0m0s)\n"
         "  -init-container-image     The image of the injected init container (default \"alpine:3.10\")\n"
         "  -qps int                  Maximum QPS to the master from this client (default 5)\n"
         "  -burst int                Maximum burst for throttle (default 10)\n"
         "  -leader-elect             Run leader election on a Lease (default true)\n"
         "  -leader-elect-lease-duration duration   (default 15s)\n"
         "  -leader-elect-renew-deadline duration   (default 5s)\n"
         "  -leader-elect-retry-period duration     (default 3s)\n"
         "  -inject-rccl-env          Inject LOCAL_RANK and the RCCL env set into pytorch containers\n"
         "  -rccl-env KEY=VALUE       Replace the injected RCCL env set (repeatable; default\n"
         "                            HSA_ENABLE_IPC_MODE_LEGACY=0)\n"
         "  -rccl-env-file path       As -rccl-env, one KEY=VALUE per line (# comments): the\n"
         "                            measured set tools/rccl_tune.py --env-out writes\n"
         "  -xgmi-pod-topology        GPU pods: hostPID/hostIPC, NCCL_HOSTID=<node>, one-node affinity\n"
         "  -init-container-template-file  (default /etc/config/initContainer.yaml)\n"
         "  -log-level string         debug|info|warning|error (default info)\n";
}

std::string parse_flags(int argc, char** argv, ServerOption* o) {
  using Setter = std::function<std::string(const std::string&)>;
  struct Flag {
    bool is_bool;
    Setter set;
  };
  auto str = [](std::string* dst) { return Flag{false, [dst](const std::string& v) { *dst = v; return std::string(); }}; };
  auto integer = [](int* dst) {
    return Flag{false, [dst](const std::string& v) {
                  char* e = nullptr;
                  long x = std::strtol(v.c_str(), &e, 10);
                  if (!e || *e) return std::string("invalid integer value \"") + v + "\"";
                  *dst = (int)x;
                  return std::string();
                }};
  };
  auto boolean = [](bool* dst) {
    return Flag{true, [dst](const std::string& v) {
                  if (!parse_bool(v, dst)) return std::string("invalid boolean value \"") + v + "\"";
                  return std::string();
                }};
  };
  auto duration = [](double* dst) {
    return Flag{false, [dst](const std::string& v) {
                  if (!parse_duration(v, dst)) return std::string("invalid duration \"") + v + "\"";
                  return std::string();
                }};
  };
  auto ignore_bool = Flag{true, [](const std::string&) { return std::string(); }};
  auto ignore_val = Flag{false, [](const std::string&) { return std::string(); }};
  std::map<std::string, Flag> flags = {
      {"kubeconfig", str(&o->kubeconfig)},
      {"master", str(&o->master_url)},
      {"namespace", str(&o->namespace_)},
      {"threadiness", integer(&o->threadiness)},
      {"version", boolean(&o->print_version)},
      {"json-log-format", boolean(&o->json_log_format)},
      {"enable-gang-scheduling", boolean(&o->enable_gang_scheduling)},
      {"gang-scheduler-name", str(&o->gang_scheduler_name)},
      {"gang-podgroup-api", Flag{false, [o](const std::string& v) {
         if (v != "kube-batch" && v != "volcano")
           return std::string("--gang-podgroup-api must be kube-batch or volcano, got \"") + v + "\"";
         o->gang_podgroup_api = v;
         return std::string();
       }}},
      {"monitoring-port", integer(&o->monitoring_port)},
      {"resyc-period", Flag{false, [o](const std::string& v) {
         if (!parse_duration(v, &o->resync_period_s)) return std::string("invalid duration \"") + v + "\"";
         return std::string();
       }}},
      {"init-container-image", str(&o->init_container_image)},
      {"qps", integer(&o->qps)},
      {"burst", integer(&o->burst)},
      {"leader-elect", boolean(&o->leader_elect)},
      {"leader-elect-lease-duration", duration(&o->lease_duration_s)},
      {"leader-elect-renew-deadline", duration(&o->renew_deadline_s)},
      {"leader-elect-retry-period", duration(&o->retry_period_s)},
      {"inject-rccl-env", boolean(&o->inject_rccl_env)},
      {"xgmi-pod-topology", boolean(&o->xgmi_pod_topology)},
      {"rccl-env", Flag{false, [o](const std::string& v) {
         auto eq = v.find('=');
         if (eq == std::string::npos || eq == 0) return std::string("expected KEY=VALUE, got \"") + v + "\"";
         o->rccl_env.emplace_back(v.substr(0, eq), v.substr(eq + 1));
         o->rccl_env_set = true;
         return std::string();
       }}},
      {"rccl-env-file", Flag{false, [o](const std::string& path) {
         std::ifstream f(path);
         if (!f) return std::string("cannot read \"") + path + "\"";
         std::string line;
         int n = 0, pairs = 0;
         while (std::getline(f, line)) {
           ++n;
           const auto b = line.find_first_not_of(" \t\r");
           if (b == std::string::npos || line[b] == '#') continue;
           const auto e = line.find_last_not_of(" \t\r");
           const std::string kv = line.substr(b, e - b + 1);
           const auto eq = kv.find('=');
           if (eq == std::string::npos || eq == 0)
             return path + ":" + std::to_string(n) + ": expected KEY=VALUE, got \"" + kv + "\"";
           o->rccl_env.emplace_back(kv.substr(0, eq), kv.substr(eq + 1));
           ++pairs;
         }
         // an empty (or comments-only) file would replace the default injected set with
         // nothing and silently drop HSA_ENABLE_IPC_MODE_LEGACY=0 from every pod
         if (pairs == 0) return path + ": no KEY=VALUE lines";
         o->rccl_env_set = true;
         return std::string();
       }}},
      {"init-container-template-file", str(&o->init_container_template_file)},
      {"log-level", str(&o->log_level)},
      // glog flags accepted for compatibility with the reference Deployment
      {"alsologtostderr", ignore_bool},
      {"logtostderr", ignore_bool},
      {"v", ignore_val},
      {"stderrthreshold", ignore_val},
      {"log_dir", ignore_val},
      {"vmodule", ignore_val},
      {"log_backtrace_at", ignore_val},
  };
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--") break;
    if (a.size() < 2 || a[0] != '-') return "unexpected argument: " + a;
    std::string body = a.substr(a[1] == '-' ? 2 : 1);
    if (body == "h" || body == "help") return "help";
    std::string name = body, value;
    bool has_value = false;
    auto eq = body.find('=');
    if (eq != std::string::npos) {
      name = body.substr(0, eq);
      value = body.substr(eq + 1);
      has_value = true;
    }
    auto it = flags.find(name);
    if (it == flags.end()) return "flag provided but not defined: -" + name;
    if (it->second.is_bool) {
      std::string err = it->second.set(has_value ? value : "true");
      if (!err.empty()) return err + " for -" + name;
      continue;
    }
    if (!has_value) {
      if (i + 1 >= argc) return "flag needs an argument: -" + name;
      value = argv[++i];
    }
    std::string err = it->second.set(value);
    if (!err.empty()) return err + " for -" + name;
  }
  return "";
}

}  // namespace pto
