// Structured logger: JSON lines (default, like the reference's logrus JSONFormatter,
// cmd/pytorch-operator.v1/main.go:55-58) or plain text.  Fields follow
// tf-operator/pkg/logger/logger.go:26-80: job=<ns>.<name>, uid, replica-type, pod.
#pragma once

#include <cstdarg>
#include <string>
#include <utility>
#include <vector>

namespace pto {

enum class LogLevel { Debug = 0, Info = 1, Warn = 2, Error = 3 };

void log_configure(bool json, LogLevel min_level);
using LogFields = std::vector<std::pair<std::string, std::string>>;
void log_msg(LogLevel lvl, const LogFields& fields, const char* file, int line, const char* fmt, ...)
    __attribute__((format(printf, 5, 6)));

LogFields fields_for_job(const std::string& ns, const std::string& name, const std::string& uid = "");
// LoggerForReplica / LoggerForPod (tf-operator/pkg/logger/logger.go:26-56): + replica-type
// (lower-case), + pod=<ns>.<pod name>
LogFields fields_for_replica(const std::string& ns, const std::string& name, const std::string& uid,
                             const std::string& rtype);
LogFields fields_for_pod(const std::string& ns, const std::string& job, const std::string& uid,
                         const std::string& rtype, const std::string& pod);
LogFields fields_for_key(const std::string& key);

#define PTO_LOG(lvl, fields, ...) ::pto::log_msg(lvl, fields, __FILE__, __LINE__, __VA_ARGS__)
#define LOG_INFO(...) PTO_LOG(::pto::LogLevel::Info, {}, __VA_ARGS__)
#define LOG_WARN(...) PTO_LOG(::pto::LogLevel::Warn, {}, __VA_ARGS__)
#define LOG_ERROR(...) PTO_LOG(::pto::LogLevel::Error, {}, __VA_ARGS__)
#define LOG_DEBUG(...) PTO_LOG(::pto::LogLevel::Debug, {}, __VA_ARGS__)

}  // namespace pto
