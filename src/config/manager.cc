#include "config/manager.h"

#include <cstdlib>

#include "config/properties.h"
#include "core/log.h"

namespace hola::config {

Manager::Manager(ManagerOptions o) : o_(std::move(o)) {
  auto it = o_.sysprops.find("conf");
  if (it != o_.sysprops.end()) conf_path_ = it->second;
}

Manager::~Manager() { stop(); }

std::shared_ptr<Snapshot> Manager::build(const FileWatcher::Contents& files) {
  auto s = std::make_shared<Snapshot>();
  s->generation = ++gen_;
  s->conf_path = conf_path_;
  std::vector<Source> sources;
  sources.push_back({"SystemProperties", 400, o_.sysprops});
  sources.push_back({"EnvironmentProperties", 300, o_.env});
  sources.push_back({"JNDI", 200, {}});
  if (!o_.deltaspike_properties.empty()) {
    Source ds{"PropertyFileConfig[" + o_.deltaspike_properties + "]", 100, {}};
    auto f = files.find(o_.deltaspike_properties);
    if (f != files.end() && f->second) {
      PropertiesResult pr = parse_properties(*f->second);
      if (pr.ok) ds.values = pr.map;
      // DeltaSpike property-file sources may override their own ordinal [lib-default].
      auto o = ds.values.find("deltaspike_ordinal");
      if (o != ds.values.end()) {
        char* end = nullptr;
        long v = strtol(o->second.c_str(), &end, 10);
        if (end && *end == '\0' && !o->second.empty()) ds.ordinal = int(v);
      }
    }
    sources.push_back(std::move(ds));
  }
  Source cf{"ConfigFile", 0, {}};  // Configuration.java:40-48
  if (!conf_path_.empty()) {
    auto f = files.find(conf_path_);
    if (f != files.end() && f->second) {
      PropertiesResult pr = parse_properties(*f->second);
      if (pr.ok) {
        cf.values = pr.map;
        s->conf_loaded = true;
      } else {
        s->conf_error = pr.error;  // swallowed like Configuration.java:34-36, but logged
      }
    }
  }
  sources.push_back(std::move(cf));
  s->resolver = std::make_shared<Resolver>(std::move(sources));

  // Hystrix properties: the Archaius classpath file, overridden by system properties.
  if (!o_.hystrix_config.empty()) {
    auto f = files.find(o_.hystrix_config);
    if (f != files.end() && f->second) {
      PropertiesResult pr = parse_properties(*f->second);
      for (auto& [k, v] : pr.map)
        if (k.rfind("hystrix.", 0) == 0) s->hystrix[k] = v;
    }
  }
  for (auto& [k, v] : o_.sysprops)
    if (k.rfind("hystrix.", 0) == 0) s->hystrix[k] = v;
  return s;
}

void Manager::start(Listener l) {
  listener_ = std::move(l);
  std::vector<std::string> paths;
  if (!conf_path_.empty()) paths.push_back(conf_path_);
  if (!o_.deltaspike_properties.empty()) paths.push_back(o_.deltaspike_properties);
  if (!o_.hystrix_config.empty()) paths.push_back(o_.hystrix_config);
  watcher_ = std::make_unique<FileWatcher>(paths, o_.poll_ms, [this](const FileWatcher::Contents& c) {
    auto s = build(c);
    if (!s->conf_error.empty()) LOG_WARN("config file %s: %s", s->conf_path.c_str(), s->conf_error.c_str());
    {
      std::lock_guard<std::mutex> g(mu_);
      cur_ = s;
    }
    if (listener_) listener_(*s);
  });
  auto s = build(watcher_->initial());
  if (!s->conf_error.empty()) LOG_WARN("config file %s: %s", s->conf_path.c_str(), s->conf_error.c_str());
  {
    std::lock_guard<std::mutex> g(mu_);
    cur_ = s;
  }
  if (listener_) listener_(*s);
  watcher_->start();
}

void Manager::stop() {
  if (watcher_) watcher_->stop();
}

std::shared_ptr<const Snapshot> Manager::current() const {
  std::lock_guard<std::mutex> g(mu_);
  return cur_;
}

}  // namespace hola::config
