#include "pto/log.hpp"

#include <cstdio>
#include <cstring>
#include <mutex>
#include <sys/time.h>
#include <ctime>

#include "pto/json.hpp"

namespace pto {

namespace {
bool g_json = true;
LogLevel g_min = LogLevel::Info;
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
  std::lock_guard<std::mutex> g(g_mu);
  g_json = json;
  g_min = min_level;
}

void log_msg(LogLevel lvl, const LogFields& fields, const char* file, int line, const char* fmt, ...) {
  if ((int)lvl < (int)g_min) return;
  char buf[4096];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  const char* base = std::strrchr(file, '/');
  base = base ? base + 1 : file;
  std::string loc = std::string(base) + ":" + std::to_string(line);
  std::string out;
  if (g_json) {
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

LogFields fields_for_key(const std::string& key) {
  std::string k = key;
  auto p = k.find('/');
  if (p != std::string::npos) k[p] = '.';
  return {{"job", k}};
}

}  // namespace pto
