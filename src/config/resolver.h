// Layered configuration resolver — the DeltaSpike ConfigResolver role.
//
// Sources by ordinal, highest first ([lib-default] DeltaSpike 1.6 ordinals):
//   400 system properties   (-Dkey=value on the command line or inside $JAVA_OPTIONS)
//   300 environment          (exact key name)
//   200 JNDI                 (never populated: there is no JNDI outside a Java EE container)
//   100 deltaspike props     (--deltaspike-properties, the META-INF/apache-deltaspike.properties role)
//     0 ConfigFile           (the `-Dconf=<file>` Java properties file, Configuration.java:10-49)
// then the caller's default. Lookups are project-stage aware like TypedResolver
// (`hello.Production` before `hello`); empty values fall back to the default.
#pragma once
#include <map>
#include <string>
#include <vector>

namespace hola::config {

struct Source {
  std::string name;
  int ordinal = 0;
  std::map<std::string, std::string> values;
};

struct Resolved {
  bool found = false;  // false => default used
  std::string value;
  std::string key;     // the key that matched (may carry the project-stage suffix)
  std::string source;  // source name, or "default"
};

class Resolver {
 public:
  // Sources may be given in any order; they are consulted by descending ordinal.
  explicit Resolver(std::vector<Source> sources);
  // Raw lookup: first source with a non-null value, no defaulting.
  bool lookup(const std::string& key, std::string* value, std::string* source) const;
  // DeltaSpike TypedResolver semantics (project stage aware, empty -> default).
  Resolved resolve(const std::string& key, const std::string& def) const;
  std::string project_stage() const;
  const std::vector<Source>& sources() const { return sources_; }

 private:
  std::vector<Source> sources_;
};

// Parses `-Dkey=value` tokens from a JAVA_OPTIONS-style string (shell-like quoting).
std::map<std::string, std::string> parse_java_options(const std::string& s);
// Snapshot of environ.
std::map<std::string, std::string> environment_map();

}  // namespace hola::config
