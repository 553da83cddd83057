// Host-side view of ops/routing.py's override string for the few kernel choices made in C++ (launch geometry and
// test hooks): DLLM_ROUTE="key=value,..." is the framework's ONE knob variable; Python validates the keys (every key used
// here has a DEFAULTS entry there), this reads integer values.  Parsed again only when the string changes.
#pragma once
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>

namespace dllm {

inline int route_int(const char* key, int dflt) {
  static std::mutex mu;
  static std::string raw_seen = "\x01";
  static std::unordered_map<std::string, int> vals;
  const char* e = std::getenv("DLLM_ROUTE");
  const std::string raw = e ? e : "";
  std::lock_guard<std::mutex> lk(mu);
  if (raw != raw_seen) {
    raw_seen = raw;
    vals.clear();
    size_t i = 0;
    while (i < raw.size()) {
      size_t j = raw.find(',', i);
      if (j == std::string::npos) j = raw.size();
      const std::string item = raw.substr(i, j - i);
      const size_t eq = item.find('=');
      if (eq != std::string::npos) {
        std::string k = item.substr(0, eq), v = item.substr(eq + 1);
        while (!k.empty() && k.front() == ' ') k.erase(k.begin());
        while (!k.empty() && k.back() == ' ') k.pop_back();
        vals[k] = std::atoi(v.c_str());
      }
      i = j + 1;
    }
  }
  auto it = vals.find(key);
  return it == vals.end() ? dflt : it->second;
}

}  // namespace dllm
