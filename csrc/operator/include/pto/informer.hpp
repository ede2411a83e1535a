// Shared-informer equivalent (client-go tools/cache): LIST then WATCH from the
// list's resourceVersion, keep a local store keyed "<ns>/<name>", dispatch
// add/update/delete callbacks, re-LIST on 410 Gone or stream errors, and fire
// a periodic resync (update(obj, obj) for every cached object).
//
// The PyTorchJob informer in the reference is an *unstructured* informer
// (pkg/common/util/v1/unstructured/informer.go:25-63, resync 30 s): objects stay
// raw JSON and are parsed / validated lazily -- this store works the same way.
#pragma once

#include <atomic>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "pto/json.hpp"
#include "pto/kube.hpp"

namespace pto {

class Informer {
 public:
  struct Handlers {
    std::function<void(const Json&)> on_add;
    std::function<void(const Json& old_obj, const Json& new_obj)> on_update;
    std::function<void(const Json&)> on_delete;
  };

  Informer(KubeClient* client, Resource res, std::string ns, std::string label_selector,
           double resync_s, Handlers h);
  ~Informer();

  void start();
  void stop();
  bool has_synced() const { return synced_.load(); }
  bool wait_for_sync(double timeout_s) const;

  std::optional<Json> get(const std::string& ns, const std::string& name) const;
  std::vector<Json> list(const std::string& ns = "") const;  // "" = all namespaces
  // Replace a cached object locally (e.g. status written by the controller itself).
  void update_cache(const Json& obj);

  static std::string key_of(const Json& obj);

 private:
  void run();
  bool relist();
  std::string rv_of(const Json& obj) const;

  KubeClient* client_;
  Resource res_;
  std::string ns_, selector_;
  double resync_s_;
  Handlers h_;
  mutable std::mutex mu_;
  std::map<std::string, Json> store_;
  std::string last_rv_;
  std::atomic<bool> synced_{false}, stop_{false};
  std::thread th_;
};

}  // namespace pto
