#include "pto/informer.hpp"

#include <chrono>

#include "pto/log.hpp"

namespace pto {

using clk = std::chrono::steady_clock;

Informer::Informer(KubeClient* client, Resource res, std::string ns, std::string sel, double resync_s,
                   Handlers h)
    : client_(client), res_(std::move(res)), ns_(std::move(ns)), selector_(std::move(sel)),
      resync_s_(resync_s), h_(std::move(h)) {}

Informer::~Informer() { stop(); }

void Informer::start() { th_ = std::thread([this] { run(); }); }

void Informer::stop() {
  stop_.store(true);
  if (th_.joinable()) th_.join();
}

bool Informer::wait_for_sync(double timeout_s) const {
  auto end = clk::now() + std::chrono::duration_cast<clk::duration>(std::chrono::duration<double>(timeout_s));
  while (!synced_.load()) {
    if (clk::now() > end || stop_.load()) return false;
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
  return true;
}

std::string Informer::key_of(const Json& obj) {
  const Json* md = obj.get("metadata");
  if (!md) return "";
  std::string ns = md->str_or("namespace");
  return ns.empty() ? md->str_or("name") : ns + "/" + md->str_or("name");
}

std::string Informer::rv_of(const Json& obj) const {
  const Json* md = obj.get("metadata");
  return md ? md->str_or("resourceVersion") : "";
}

std::optional<Json> Informer::get(const std::string& ns, const std::string& name) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = store_.find(ns.empty() ? name : ns + "/" + name);
  if (it == store_.end()) return std::nullopt;
  return it->second;
}

std::vector<Json> Informer::list(const std::string& ns) const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<Json> out;
  for (const auto& kv : store_) {
    if (!ns.empty()) {
      const Json* md = kv.second.get("metadata");
      if (!md || md->str_or("namespace") != ns) continue;
    }
    out.push_back(kv.second);
  }
  return out;
}

void Informer::update_cache(const Json& obj) {
  std::lock_guard<std::mutex> g(mu_);
  store_[key_of(obj)] = obj;
}

bool Informer::relist() {
  ApiError err;
  auto lst = client_->list(res_, ns_, selector_, &err);
  if (!lst) {
    LOG_WARN("list %s failed (%d): %s", res_.plural.c_str(), err.code, err.message.c_str());
    return false;
  }
  std::map<std::string, Json> fresh;
  if (const Json* items = lst->get("items"); items && items->is_array()) {
    for (auto item : items->as_array()) {
      // list items carry no kind/apiVersion; restore them for handlers
      if (!item.get("kind") && lst->get("kind")) {
        std::string k = lst->str_or("kind");
        if (k.size() > 4 && k.compare(k.size() - 4, 4, "List") == 0) item["kind"] = k.substr(0, k.size() - 4);
        item["apiVersion"] = lst->str_or("apiVersion");
      }
      fresh[key_of(item)] = item;
    }
  }
  std::vector<std::pair<int, std::pair<Json, Json>>> events;  // 0 add, 1 update, 2 delete
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : fresh) {
      auto it = store_.find(kv.first);
      if (it == store_.end()) events.push_back({0, {Json(), kv.second}});
      else if (rv_of(it->second) != rv_of(kv.second)) events.push_back({1, {it->second, kv.second}});
    }
    for (auto& kv : store_)
      if (!fresh.count(kv.first)) events.push_back({2, {kv.second, Json()}});
    store_ = std::move(fresh);
    const Json* md = lst->get("metadata");
    last_rv_ = md ? md->str_or("resourceVersion") : "";
  }
  for (auto& e : events) {
    if (e.first == 0 && h_.on_add) h_.on_add(e.second.second);
    if (e.first == 1 && h_.on_update) h_.on_update(e.second.first, e.second.second);
    if (e.first == 2 && h_.on_delete) h_.on_delete(e.second.first);
  }
  return true;
}

void Informer::run() {
  auto next_resync = clk::now() + std::chrono::duration_cast<clk::duration>(std::chrono::duration<double>(resync_s_));
  double backoff = 0.2;
  while (!stop_.load()) {
    if (!relist()) {
      std::this_thread::sleep_for(std::chrono::duration<double>(backoff));
      backoff = std::min(backoff * 2, 5.0);
      continue;
    }
    backoff = 0.2;
    synced_.store(true);
    // watch until error / timeout, resyncing periodically from the local store
    while (!stop_.load()) {
      ApiError err;
      std::string rv;
      {
        std::lock_guard<std::mutex> g(mu_);
        rv = last_rv_;
      }
      double until_resync = std::chrono::duration<double>(next_resync - clk::now()).count();
      double wtimeout = std::max(1.0, std::min(60.0, until_resync));
      client_->watch(
          res_, ns_, selector_, rv,
          [&](const std::string& type, const Json& obj) {
            std::string key = key_of(obj);
            std::string orv = rv_of(obj);
            if (type == "BOOKMARK") {
              std::lock_guard<std::mutex> g(mu_);
              last_rv_ = orv;
              return !stop_.load();
            }
            Json old;
            bool had = false;
            {
              std::lock_guard<std::mutex> g(mu_);
              auto it = store_.find(key);
              if (it != store_.end()) {
                old = it->second;
                had = true;
              }
              if (type == "DELETED") store_.erase(key);
              else store_[key] = obj;
              if (!orv.empty()) last_rv_ = orv;
            }
            if (type == "ADDED" || (type == "MODIFIED" && !had)) {
              if (had && h_.on_update) h_.on_update(old, obj);
              else if (h_.on_add) h_.on_add(obj);
            } else if (type == "MODIFIED") {
              if (h_.on_update) h_.on_update(old, obj);
            } else if (type == "DELETED") {
              if (h_.on_delete) h_.on_delete(had ? old : obj);
            }
            return !stop_.load() && clk::now() < next_resync;
          },
          &stop_, wtimeout, &err);
      if (stop_.load()) return;
      if (clk::now() >= next_resync) {
        next_resync = clk::now() + std::chrono::duration_cast<clk::duration>(std::chrono::duration<double>(resync_s_));
        if (h_.on_update) {
          for (const auto& o : list()) h_.on_update(o, o);
        }
      }
      if (err.gone()) break;  // resourceVersion too old: relist
      if (err.code != 0 || !err.message.empty()) {
        LOG_DEBUG("watch %s ended (%d): %s", res_.plural.c_str(), err.code, err.message.c_str());
        if (err.code != 0 && err.code != 200) break;
        std::this_thread::sleep_for(std::chrono::milliseconds(200));
        break;
      }
    }
  }
}

}  // namespace pto
