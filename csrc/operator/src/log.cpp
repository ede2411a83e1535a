#include "pto/log.hpp"

#include <atomic>
#include <cctype>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <sys/time.h>
#include <ctime>

#include "pto/json.hpp"

namespace pto {

namespace {
// read on every log call from any thread, written by log_configure: atomics, so a late
// reconfiguration is never a data race (the output mutex only serialises the writes)
std::atomic<bool> g_json{true};
std::atomic<int> g_min{(int)LogLevel::Info};
std::mutex g_mu;

const char* level_name(LogLevel l) {
  switch (l) {
    case LogLevel::Debug: return "debug";
    case LogLevel::Info: return "info";
    case LogLevel::Warn: return "warning";
    default: return "error";
  }
}

std::string timestamp() {
  struct timeval tv;
  gettimeofday(&tv, nullptr);
  struct tm tmv;
  gmtime_r(&tv.tv_sec, &tmv);
  char buf[64];
  std::strftime(buf, sizeof buf, "%Y-%m-%dT%H:%M:%S", &tmv);
  char out[80];
  std::snprintf(out, sizeof out, "%s.%06ldZ", buf, (long)tv.tv_usec);
  return out;
}
}  // namespace

void log_configure(bool json, LogLevel min_level) {
  g_json.store(json, std::memory_order_relaxed);
  g_min.store((int)min_level, std::memory_order_relaxed);
}

void log_msg(LogLevel lvl, const LogFields& fields, const char* file, int line, const char* fmt, ...) {
  if ((int)lvl < g_min.load(std::memory_order_relaxed)) return;
  char buf[4096];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  const char* base = std::strrchr(file, '/');
  base = base ? base + 1 : file;
  std::string loc = std::string(base) + ":" + std::to_string(line);
  std::string out;
  if (g_json.load(std::memory_order_relaxed)) {
    Json o = Json::object();
    o["filename"] = loc;
    for (const auto& kv : fields) o[kv.first] = kv.second;
    o["level"] = level_name(lvl);
    o["msg"] = std::string(buf);
    o["time"] = timestamp();
    out = o.dump();
  } else {
    out = timestamp() + " " + level_name(lvl) + " " + loc + " " + buf;
    for (const auto& kv : fields) out += " " + kv.first + "=" + kv.second;
  }
  std::lock_guard<std::mutex> g(g_mu);
  std::fprintf(stderr, "%s\n", out.c_str());
  std::fflush(stderr);
}

LogFields fields_for_job(const std::string& ns, const std::string& name, const std::string& uid) {
  LogFields f{{"job", ns + "." + name}};
  if (!uid.empty()) f.push_back({"uid", uid});
  return f;
}

LogFields fields_for_replica(const std::string& ns, const std::string& name, const std::string& uid,
                             const std::string& rtype) {
  LogFields f = fields_for_job(ns, name, uid);
  std::string rt = rtype;
  for (auto& ch : rt) ch = (char)std::tolower((unsigned char)ch);
  f.push_back({"replica-type", rt});
  return f;
}

LogFields fields_for_pod(const std::string& ns, const std::string& job, const std::string& uid,
                         const std::string& rtype, const std::string& pod) {
  LogFields f = fields_for_replica(ns, job, uid, rtype);
  f.push_back({"pod", ns + "." + pod});
  return f;
}

LogFields fields_for_key(const std::string& key) {
  std::string k = key;
  auto p = k.find('/');
  if (p != std::string::npos) k[p] = '.';
  return {{"job", k}};
}

}  // namespace pto
