#include "config/resolver.h"

#include <algorithm>

extern char** environ;

namespace hola::config {

Resolver::Resolver(std::vector<Source> sources) : sources_(std::move(sources)) {
  std::stable_sort(sources_.begin(), sources_.end(),
                   [](const Source& a, const Source& b) { return a.ordinal > b.ordinal; });
}

bool Resolver::lookup(const std::string& key, std::string* value, std::string* source) const {
  for (const Source& s : sources_) {
    auto it = s.values.find(key);
    if (it != s.values.end()) {
      *value = it->second;
      if (source) *source = s.name;
      return true;
    }
  }
  return false;
}

std::string Resolver::project_stage() const {
  std::string v;
  if (lookup("org.apache.deltaspike.ProjectStage", &v, nullptr) && !v.empty()) return v;
  return "Production";
}

Resolved Resolver::resolve(const std::string& key, const std::string& def) const {
  Resolved r;
  std::string v, src;
  std::string staged = key + "." + project_stage();
  if (lookup(staged, &v, &src) && !v.empty()) {
    r.found = true;
    r.value = v;
    r.key = staged;
    r.source = src;
    return r;
  }
  if (lookup(key, &v, &src) && !v.empty()) {
    r.found = true;
    r.value = v;
    r.key = key;
    r.source = src;
    return r;
  }
  r.value = def;
  r.key = key;
  r.source = "default";
  return r;
}

std::map<std::string, std::string> parse_java_options(const std::string& s) {
  std::vector<std::string> toks;
  std::string cur;
  bool in_tok = false;
  char quote = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (quote) {
      if (c == quote) quote = 0;
      else if (c == '\\' && quote == '"' && i + 1 < s.size()) cur.push_back(s[++i]);
      else cur.push_back(c);
      continue;
    }
    if (c == '\'' || c == '"') {
      quote = c;
      in_tok = true;
      continue;
    }
    if (c == ' ' || c == '\t' || c == '\n') {
      if (in_tok) toks.push_back(cur);
      cur.clear();
      in_tok = false;
      continue;
    }
    if (c == '\\' && i + 1 < s.size()) {
      cur.push_back(s[++i]);
      in_tok = true;
      continue;
    }
    cur.push_back(c);
    in_tok = true;
  }
  if (in_tok) toks.push_back(cur);
  std::map<std::string, std::string> out;
  for (const std::string& t : toks) {
    if (t.size() < 3 || t[0] != '-' || t[1] != 'D') continue;
    size_t eq = t.find('=');
    if (eq == std::string::npos) out[t.substr(2)] = "";  // -Dflag => "" (as the JVM does)
    else out[t.substr(2, eq - 2)] = t.substr(eq + 1);
  }
  return out;
}

std::map<std::string, std::string> environment_map() {
  std::map<std::string, std::string> m;
  for (char** e = environ; e && *e; ++e) {
    std::string kv(*e);
    size_t eq = kv.find('=');
    if (eq == std::string::npos) continue;
    m[kv.substr(0, eq)] = kv.substr(eq + 1);
  }
  return m;
}

}  // namespace hola::config
