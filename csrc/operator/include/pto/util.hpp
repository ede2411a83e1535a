// Misc helpers of the reference's pkg/util (pkg/util/util.go:33-74): Pformat pretty-prints
// any JSON value (strings pass through verbatim) for logs and e2e diagnostics; RandString
// makes a random lowercase-alphanumeric (DNS-1035 character set) suffix for test job names.
#pragma once

#include <random>
#include <string>

#include "pto/json.hpp"

namespace pto {

inline std::string pformat(const Json& v) {
  if (v.is_string()) return v.as_string();
  return v.dump(2);
}

// Thread-safe: one generator per thread, seeded from the OS entropy source.
inline std::string rand_string(int n) {
  static const char kLetters[] = "0123456789abcdefghijklmnopqrstuvwxyz";
  thread_local std::mt19937_64 gen{std::random_device{}()};
  std::uniform_int_distribution<int> pick(0, 35);
  std::string s(n > 0 ? n : 0, '0');
  for (auto& c : s) c = kLetters[pick(gen)];
  return s;
}

}  // namespace pto
