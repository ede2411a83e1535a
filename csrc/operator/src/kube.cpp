#include "pto/kube.hpp"

#include <poll.h>
#include <algorithm>
#include <cerrno>
#include <signal.h>
#include <spawn.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <thread>

#include "pto/log.hpp"
#include "pto/metrics.hpp"
#include "pto/yaml_lite.hpp"

namespace pto {

const Resource kPods{"", "v1", "pods"};
const Resource kServices{"", "v1", "services"};
const Resource kEvents{"", "v1", "events"};
const Resource kEndpoints{"", "v1", "endpoints"};
const Resource kLeases{"coordination.k8s.io", "v1", "leases"};
const Resource kPyTorchJobs{"kubeflow.org", "v1", "pytorchjobs"};
const Resource kPodGroups{"scheduling.incubator.k8s.io", "v1alpha1", "podgroups"};
const Resource kVolcanoPodGroups{"scheduling.volcano.sh", "v1beta1", "podgroups"};
const Resource kCRDs{"apiextensions.k8s.io", "v1", "customresourcedefinitions", false};

std::string Resource::path(const std::string& ns, const std::string& name, const std::string& sub) const {
  std::string p = group.empty() ? "/api/" + version : "/apis/" + group + "/" + version;
  if (namespaced && !ns.empty()) p += "/namespaces/" + ns;
  p += "/" + plural;
  if (!name.empty()) p += "/" + name;
  if (!sub.empty()) p += "/" + sub;
  return p;
}

static std::string read_file(const std::string& path, bool* ok) {
  std::ifstream f(path, std::ios::binary);
  *ok = (bool)f;
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

// Entry `name` of a kubeconfig list (doc[key]); a pointer into doc, never a temporary.
static const Json* named(const Json& doc, const char* key, const std::string& name) {
  const Json* list = doc.get(key);
  if (!list || !list->is_array()) return nullptr;
  for (const auto& e : list->as_array())
    if (e.str_or("name") == name) return &e;
  return nullptr;
}

extern "C" char** environ;

// client-go's exec credential flow: run the plugin with KUBERNETES_EXEC_INFO in its
// environment, parse the ExecCredential it prints.  argv is passed as-is (no shell).
bool run_exec_plugin(const ExecPlugin& plugin, KubeConfig* kc, std::string* error) {
  std::vector<std::string> envs;
  for (char** e = environ; e && *e; ++e) envs.emplace_back(*e);
  for (const auto& kv : plugin.env) envs.push_back(kv.first + "=" + kv.second);
  envs.push_back("KUBERNETES_EXEC_INFO={\"apiVersion\":\"" + plugin.api_version +
                 "\",\"kind\":\"ExecCredential\",\"spec\":{\"interactive\":false}}");
  std::vector<char*> envp;
  for (auto& e : envs) envp.push_back(e.data());
  envp.push_back(nullptr);
  std::vector<std::string> args{plugin.command};
  args.insert(args.end(), plugin.args.begin(), plugin.args.end());
  std::vector<char*> argv;
  for (auto& a : args) argv.push_back(a.data());
  argv.push_back(nullptr);
  int out[2];
  if (pipe(out) != 0) {
    *error = "exec plugin: pipe failed";
    return false;
  }
  posix_spawn_file_actions_t fa;
  posix_spawn_file_actions_init(&fa);
  posix_spawn_file_actions_adddup2(&fa, out[1], STDOUT_FILENO);
  posix_spawn_file_actions_addclose(&fa, out[0]);
  pid_t pid = 0;
  const int rc = posix_spawnp(&pid, plugin.command.c_str(), &fa, nullptr, argv.data(), envp.data());
  posix_spawn_file_actions_destroy(&fa);
  close(out[1]);
  if (rc != 0) {
    close(out[0]);
    *error = "exec plugin " + plugin.command + ": " + std::strerror(rc);
    return false;
  }
  std::string text;
  char buf[4096];
  struct pollfd p{out[0], POLLIN, 0};
  // one deadline for output AND exit (client-go's exec credential timeout is 60 s too);
  // PTO_EXEC_PLUGIN_TIMEOUT_S overrides it (tests)
  long timeout_s = 60;
  if (const char* t = std::getenv("PTO_EXEC_PLUGIN_TIMEOUT_S")) timeout_s = std::max(1L, std::atol(t));
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(timeout_s);
  while (std::chrono::steady_clock::now() < deadline) {
    if (::poll(&p, 1, 200) <= 0) continue;
    const ssize_t n = ::read(out[0], buf, sizeof buf);
    if (n <= 0) break;
    text.append(buf, (size_t)n);
  }
  close(out[0]);
  // reap without blocking past the deadline: a plugin that hangs (with or without its stdout
  // open) is killed, so a reconcile worker refreshing credentials never blocks forever
  int status = 0;
  bool exited = false;
  while (true) {
    const pid_t w = waitpid(pid, &status, WNOHANG);
    if (w == pid || (w < 0 && errno != EINTR)) {
      exited = w == pid;
      break;
    }
    if (std::chrono::steady_clock::now() >= deadline) break;
    ::poll(nullptr, 0, 20);
  }
  if (!exited) {
    ::kill(pid, SIGKILL);
    while (waitpid(pid, &status, 0) < 0 && errno == EINTR) {
    }
    *error = "exec plugin " + plugin.command + " timed out after " + std::to_string(timeout_s) + " s (killed)";
    return false;
  }
  if (!WIFEXITED(status) || WEXITSTATUS(status) != 0) {
    *error = "exec plugin " + plugin.command + " failed (status " + std::to_string(status) + ")";
    return false;
  }
  try {
    Json cred = Json::parse(text);
    if (cred.str_or("kind") != "ExecCredential") {
      *error = "exec plugin " + plugin.command + " did not print an ExecCredential";
      return false;
    }
    const Json* st = cred.get("status");
    if (!st) {
      *error = "exec plugin " + plugin.command + ": ExecCredential without status";
      return false;
    }
    if (!st->str_or("token").empty()) kc->token = st->str_or("token");
    if (!st->str_or("clientCertificateData").empty() && !st->str_or("clientKeyData").empty()) {
      kc->tls.cert_data = st->str_or("clientCertificateData");
      kc->tls.key_data = st->str_or("clientKeyData");
      kc->tls.cert_file.clear();
      kc->tls.key_file.clear();
    }
  } catch (const std::exception& e) {
    *error = std::string("exec plugin output: ") + e.what();
    return false;
  }
  return true;
}

std::optional<KubeConfig> load_kube_config(const std::string& master_url, const std::string& kubeconfig,
                                           std::string* error) {
  KubeConfig kc;
  if (!kubeconfig.empty()) {
    bool ok = false;
    std::string text = read_file(kubeconfig, &ok);
    if (!ok) {
      *error = "cannot read kubeconfig " + kubeconfig;
      return std::nullopt;
    }
    Json doc;
    try {
      doc = text.find_first_not_of(" \t\r\n") != std::string::npos && text[text.find_first_not_of(" \t\r\n")] == '{'
                ? Json::parse(text)
                : yaml_parse(text);
    } catch (const std::exception& e) {
      *error = std::string("kubeconfig parse error: ") + e.what();
      return std::nullopt;
    }
    std::string ctx_name = doc.str_or("current-context");
    const Json* ctx = named(doc, "contexts", ctx_name);
    const Json* ctxv = ctx ? ctx->get("context") : nullptr;
    std::string cluster_name = ctxv ? ctxv->str_or("cluster") : "";
    std::string user_name = ctxv ? ctxv->str_or("user") : "";
    if (ctxv && !ctxv->str_or("namespace").empty()) kc.ns = ctxv->str_or("namespace");
    const Json* cl = named(doc, "clusters", cluster_name);
    if (!cl && doc.get("clusters") && doc.get("clusters")->size() > 0) cl = &doc.get("clusters")->as_array()[0];
    const Json* clv = cl ? cl->get("cluster") : nullptr;
    if (clv) {
      kc.server = clv->str_or("server");
      kc.tls.ca_file = clv->str_or("certificate-authority");
      if (!clv->str_or("certificate-authority-data").empty())
        kc.tls.ca_data = base64_decode(clv->str_or("certificate-authority-data"));
      kc.tls.insecure_skip_verify = clv->bool_or("insecure-skip-tls-verify", false);
      kc.tls.server_name = clv->str_or("tls-server-name");
    }
    const Json* us = named(doc, "users", user_name);
    const Json* usv = us ? us->get("user") : nullptr;
    if (usv) {
      kc.token = usv->str_or("token");
      if (!usv->str_or("tokenFile").empty()) {
        bool tok_ok;
        kc.token = read_file(usv->str_or("tokenFile"), &tok_ok);
      }
      kc.tls.cert_file = usv->str_or("client-certificate");
      kc.tls.key_file = usv->str_or("client-key");
      if (!usv->str_or("client-certificate-data").empty())
        kc.tls.cert_data = base64_decode(usv->str_or("client-certificate-data"));
      if (!usv->str_or("client-key-data").empty())
        kc.tls.key_data = base64_decode(usv->str_or("client-key-data"));
      if (const Json* ex = usv->get("exec")) {
        ExecPlugin pl;
        pl.command = ex->str_or("command");
        if (!ex->str_or("apiVersion").empty()) pl.api_version = ex->str_or("apiVersion");
        if (const Json* a = ex->get("args"))
          if (a->is_array())
            for (const auto& v : a->as_array()) pl.args.push_back(v.is_string() ? v.as_string() : v.dump());
        if (const Json* en = ex->get("env"))
          if (en->is_array())
            for (const auto& v : en->as_array()) pl.env.emplace_back(v.str_or("name"), v.str_or("value"));
        if (pl.command.empty()) {
          *error = "kubeconfig exec plugin without a command";
          return std::nullopt;
        }
        if (!run_exec_plugin(pl, &kc, error)) return std::nullopt;
        kc.exec = pl;
      }
      if (usv->get("auth-provider")) {
        *error = "kubeconfig auth-provider plugins are not supported (removed from client-go); use an exec plugin";
        return std::nullopt;
      }
    }
  } else if (master_url.empty()) {
    // in-cluster config
    const char* host = std::getenv("KUBERNETES_SERVICE_HOST");
    const char* port = std::getenv("KUBERNETES_SERVICE_PORT");
    if (!host || !port) {
      *error = "no --kubeconfig/--master given and not running in a cluster";
      return std::nullopt;
    }
    kc.server = std::string("https://") + host + ":" + port;
    bool ok;
    kc.token = read_file("/var/run/secrets/kubernetes.io/serviceaccount/token", &ok);
    kc.tls.ca_file = "/var/run/secrets/kubernetes.io/serviceaccount/ca.crt";
    std::string ns = read_file("/var/run/secrets/kubernetes.io/serviceaccount/namespace", &ok);
    if (ok && !ns.empty()) kc.ns = ns;
  }
  if (!master_url.empty()) kc.server = master_url;
  while (!kc.token.empty() && (kc.token.back() == '\n' || kc.token.back() == '\r')) kc.token.pop_back();
  if (kc.server.empty()) {
    *error = "no API server address";
    return std::nullopt;
  }
  return kc;
}

KubeClient::KubeClient(const KubeConfig& cfg, double qps, int burst)
    : cfg_(cfg), qps_(qps), burst_(burst), tokens_(burst), last_(std::chrono::steady_clock::now()) {
  if (!Url::parse(cfg.server, &url_)) url_ = Url{};
  http_ = std::make_unique<HttpClient>(url_, cfg.tls, cfg.token, 30.0);
}

void KubeClient::throttle() {
  if (qps_ <= 0) return;
  double wait = 0;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto now = std::chrono::steady_clock::now();
    double el = std::chrono::duration<double>(now - last_).count();
    last_ = now;
    tokens_ = std::min<double>(burst_, tokens_ + el * qps_);
    tokens_ -= 1.0;
    if (tokens_ < 0) wait = -tokens_ / qps_;
  }
  if (wait > 0) std::this_thread::sleep_for(std::chrono::duration<double>(wait));
}

std::optional<Json> KubeClient::call(const std::string& method, const std::string& path,
                                     const std::string& body, ApiError* err, const std::string& ctype) {
  throttle();
  Metrics::instance().inc("pytorch_operator_api_requests_total");
  HttpResponse r = http_->request(method, path, body, ctype);
  if (r.status == 401 && cfg_.exec) {
    // an expired exec-plugin credential: refresh once and retry (client-go does the same)
    std::string perr;
    KubeConfig fresh = cfg_;
    if (run_exec_plugin(*cfg_.exec, &fresh, &perr)) {
      http_->set_bearer_token(fresh.token);
      Metrics::instance().inc("pytorch_operator_api_requests_total");
      r = http_->request(method, path, body, ctype);
    } else {
      LOG_WARN("exec credential refresh failed: %s", perr.c_str());
    }
  }
  if (r.status == 0) {
    if (err) *err = ApiError{0, r.error};
    return std::nullopt;
  }
  if (r.status < 200 || r.status >= 300) {
    std::string msg = r.body;
    try {
      Json j = Json::parse(r.body);
      msg = j.str_or("message", r.body);
    } catch (...) {
    }
    if (err) *err = ApiError{r.status, msg};
    return std::nullopt;
  }
  if (r.body.empty()) return Json::object();
  try {
    return Json::parse(r.body);
  } catch (const std::exception& e) {
    if (err) *err = ApiError{r.status, std::string("bad JSON from server: ") + e.what()};
    return std::nullopt;
  }
}

std::optional<Json> KubeClient::get(const Resource& r, const std::string& ns, const std::string& name,
                                    ApiError* err) {
  return call("GET", r.path(ns, name), "", err);
}

std::optional<Json> KubeClient::list(const Resource& r, const std::string& ns, const std::string& sel,
                                     ApiError* err) {
  std::string p = r.path(ns);
  if (!sel.empty()) p += "?labelSelector=" + url_encode(sel);
  return call("GET", p, "", err);
}

std::optional<Json> KubeClient::create(const Resource& r, const std::string& ns, const Json& obj, ApiError* err) {
  return call("POST", r.path(ns), obj.dump(), err);
}

std::optional<Json> KubeClient::update(const Resource& r, const std::string& ns, const Json& obj, ApiError* err) {
  const Json* md = obj.get("metadata");
  return call("PUT", r.path(ns, md ? md->str_or("name") : ""), obj.dump(), err);
}

std::optional<Json> KubeClient::update_status(const Resource& r, const std::string& ns, const Json& obj,
                                              ApiError* err) {
  const Json* md = obj.get("metadata");
  return call("PUT", r.path(ns, md ? md->str_or("name") : "", "status"), obj.dump(), err);
}

std::optional<Json> KubeClient::patch_merge(const Resource& r, const std::string& ns, const std::string& name,
                                            const Json& patch, ApiError* err) {
  return call("PATCH", r.path(ns, name), patch.dump(), err, "application/merge-patch+json");
}

bool KubeClient::del(const Resource& r, const std::string& ns, const std::string& name, ApiError* err) {
  Json opts = Json::object();
  opts["kind"] = "DeleteOptions";
  opts["apiVersion"] = "v1";
  opts["propagationPolicy"] = "Background";
  return call("DELETE", r.path(ns, name), opts.dump(), err).has_value();
}

void KubeClient::watch(const Resource& r, const std::string& ns, const std::string& sel,
                       const std::string& rv, const std::function<bool(const std::string&, const Json&)>& on_event,
                       const std::atomic<bool>* stop, double timeout_s, ApiError* err) {
  std::string p = r.path(ns) + "?watch=true&allowWatchBookmarks=true&timeoutSeconds=" +
                  std::to_string((int)timeout_s);
  if (!rv.empty()) p += "&resourceVersion=" + url_encode(rv);
  if (!sel.empty()) p += "&labelSelector=" + url_encode(sel);
  std::string transport_err;
  int code = http_->stream_lines(
      p,
      [&](const std::string& line) {
        Json ev;
        try {
          ev = Json::parse(line);
        } catch (...) {
          return true;
        }
        std::string type = ev.str_or("type");
        const Json* obj = ev.get("object");
        if (type == "ERROR") {
          int c = obj ? (int)obj->int_or("code", 500) : 500;
          if (err) *err = ApiError{c, obj ? obj->str_or("message") : "watch error"};
          return false;
        }
        return on_event(type, obj ? *obj : Json());
      },
      stop, timeout_s + 30.0, &transport_err);
  if (code == 0 && err && err->code == 0) *err = ApiError{0, transport_err};
  else if (code != 200 && code != 0 && err && err->code == 0) *err = ApiError{code, "watch failed"};
}

}  // namespace pto
