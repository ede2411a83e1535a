#include "pto/leader.hpp"

#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <fstream>
#include <random>
#include <thread>

#include "pto/api.hpp"
#include "pto/log.hpp"
#include "pto/metrics.hpp"

namespace pto {

std::string make_identity() {
  char host[256] = {0};
  gethostname(host, sizeof host - 1);
  std::random_device rd;
  std::mt19937_64 g(rd());
  uint64_t a = g(), b = g();
  char uuid[40];
  std::snprintf(uuid, sizeof uuid, "%08x-%04x-4%03x-%04x-%012llx", (unsigned)(a >> 32), (unsigned)(a >> 16) & 0xffff,
                (unsigned)a & 0xfff, (unsigned)((b >> 48) & 0x3fff) | 0x8000,
                (unsigned long long)(b & 0xffffffffffffULL));
  return std::string(host) + "_" + uuid;
}

static std::string micro_time(int64_t ms) {
  // RFC 3339 with microseconds (MicroTime), as Lease fields require
  std::string s = format_time(ms);
  char buf[16];
  std::snprintf(buf, sizeof buf, ".%06d", (int)((ms % 1000) * 1000));
  return s.substr(0, s.size() - 1) + buf + "Z";
}

LeaderElector::LeaderElector(KubeClient* client, LeaderElectionConfig cfg)
    : client_(client), cfg_(std::move(cfg)) {
  if (cfg_.identity.empty()) cfg_.identity = make_identity();
}

bool LeaderElector::try_acquire_or_renew() {
  const int64_t now = now_ms();
  ApiError err;
  auto cur = client_->get(kLeases, cfg_.ns, cfg_.name, &err);
  Json spec = Json::object();
  spec["holderIdentity"] = cfg_.identity;
  spec["leaseDurationSeconds"] = (int64_t)cfg_.lease_s;
  spec["renewTime"] = micro_time(now);
  if (!cur) {
    if (!err.not_found()) return false;
    Json lease = Json::object();
    lease["apiVersion"] = "coordination.k8s.io/v1";
    lease["kind"] = "Lease";
    lease["metadata"]["name"] = cfg_.name;
    lease["metadata"]["namespace"] = cfg_.ns;
    spec["acquireTime"] = micro_time(now);
    spec["leaseTransitions"] = 0;
    lease["spec"] = spec;
    ApiError e2;
    return client_->create(kLeases, cfg_.ns, lease, &e2).has_value();
  }
  const Json* cs = cur->get("spec");
  std::string holder = cs ? cs->str_or("holderIdentity") : "";
  int64_t transitions = cs ? cs->int_or("leaseTransitions", 0) : 0;
  if (!holder.empty() && holder != cfg_.identity) {
    auto renew = cs ? parse_time(cs->str_or("renewTime")) : std::nullopt;
    int64_t dur = cs ? cs->int_or("leaseDurationSeconds", (int64_t)cfg_.lease_s) : (int64_t)cfg_.lease_s;
    if (renew && now < *renew + dur * 1000) return false;  // held and not expired
    spec["acquireTime"] = micro_time(now);
    spec["leaseTransitions"] = transitions + 1;
  } else {
    spec["acquireTime"] = cs && cs->get("acquireTime") ? *cs->get("acquireTime") : Json(micro_time(now));
    spec["leaseTransitions"] = transitions;
  }
  Json upd = *cur;  // keeps metadata.resourceVersion: optimistic concurrency
  upd["spec"] = spec;
  ApiError e2;
  return client_->update(kLeases, cfg_.ns, upd, &e2).has_value();
}

void LeaderElector::run(const std::function<void()>& on_started, const std::function<void()>& on_stopped,
                        const std::atomic<bool>* stop) {
  using clk = std::chrono::steady_clock;
  LOG_INFO("attempting to acquire leader lease %s/%s...", cfg_.ns.c_str(), cfg_.name.c_str());
  while (!stop->load()) {
    if (try_acquire_or_renew()) break;
    std::this_thread::sleep_for(std::chrono::duration<double>(cfg_.retry_s));
  }
  if (stop->load()) return;
  LOG_INFO("successfully acquired lease %s/%s as %s", cfg_.ns.c_str(), cfg_.name.c_str(), cfg_.identity.c_str());
  leader_.store(true);
  Metrics::instance().set("pytorch_operator_is_leader", 1);
  std::thread worker(on_started);
  auto last_renew = clk::now();
  while (!stop->load()) {
    std::this_thread::sleep_for(std::chrono::duration<double>(std::min(cfg_.retry_s, cfg_.renew_deadline_s / 2)));
    if (try_acquire_or_renew()) {
      last_renew = clk::now();
    } else if (std::chrono::duration<double>(clk::now() - last_renew).count() > cfg_.renew_deadline_s) {
      leader_.store(false);
      Metrics::instance().set("pytorch_operator_is_leader", 0);
      LOG_ERROR("leader election lost");
      on_stopped();
      break;
    }
  }
  worker.join();
}

}  // namespace pto
