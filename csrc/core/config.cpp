// Config table: defaults -> RT_<NAME> env -> configure().
#include "ogkm/config.hpp"

#include <algorithm>
#include <cctype>
#include <cstdlib>

namespace ogkm {

namespace {
struct KnobDesc {
  const char* name;
  int64_t Config::*field;
  const char* doc;
};
const std::vector<KnobDesc>& knobs() {
  static const std::vector<KnobDesc> k = {
#define OGKM_DESC(name, def, doc) {#name, &Config::name, doc},
      OGKM_CONFIG_KNOBS(OGKM_DESC)
#undef OGKM_DESC
  };
  return k;
}
}  // namespace

bool Config::set(const std::string& name, int64_t v) {
  for (auto& k : knobs())
    if (name == k.name) {
      this->*k.field = v;
      return true;
    }
  return false;
}

bool Config::get(const std::string& name, int64_t* v) const {
  for (auto& k : knobs())
    if (name == k.name) {
      *v = this->*k.field;
      return true;
    }
  return false;
}

void Config::load_env() {
  for (auto& k : knobs()) {
    std::string env = "RT_";
    for (const char* p = k.name; *p; ++p) env += (char)toupper(*p);
    if (const char* e = getenv(env.c_str())) this->*k.field = strtoll(e, nullptr, 0);
  }
}

std::vector<std::string> Config::names() const {
  std::vector<std::string> n;
  for (auto& k : knobs()) n.push_back(k.name);
  return n;
}

std::string Config::doc(const std::string& name) const {
  for (auto& k : knobs())
    if (name == k.name) return k.doc;
  return "";
}

Config& config() {
  static Config* c = [] {
    auto* x = new Config();
    x->load_env();
    return x;
  }();
  return *c;
}

std::mutex& config_mutex() {
  static std::mutex m;
  return m;
}

}  // namespace ogkm
