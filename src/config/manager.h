// Owns the configuration sources and publishes a fresh Resolver whenever a watched file
// changes. Fixed sources (system properties, environment) are captured once at start — as in
// the JVM, neither can change at runtime; the file-backed sources are re-read by the
// FileWatcher thread.
#pragma once
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>

#include "config/resolver.h"
#include "config/watcher.h"

namespace hola::config {

struct ManagerOptions {
  std::map<std::string, std::string> sysprops;  // -D... (argv + $JAVA_OPTIONS)
  std::map<std::string, std::string> env;
  std::string deltaspike_properties;  // optional file, ordinal 100
  std::string hystrix_config;         // Archaius config.properties role (config.properties:16-19)
  int poll_ms = 1000;
};

struct Snapshot {
  uint64_t generation = 0;
  std::shared_ptr<const Resolver> resolver;
  std::string conf_path;        // value of system property `conf` ("" if unset)
  bool conf_loaded = false;     // file present and parsed
  std::string conf_error;       // parse error (file then contributes nothing)
  std::map<std::string, std::string> hystrix;  // merged hystrix.* properties
};

class Manager {
 public:
  using Listener = std::function<void(const Snapshot&)>;
  explicit Manager(ManagerOptions o);
  ~Manager();
  // Builds the initial snapshot and starts watching; the listener runs once synchronously
  // here and then on the watcher thread after every change.
  void start(Listener l);
  void stop();
  std::shared_ptr<const Snapshot> current() const;
  uint64_t reloads() const { return watcher_ ? watcher_->reloads() : 0; }

 private:
  std::shared_ptr<Snapshot> build(const FileWatcher::Contents& files);
  ManagerOptions o_;
  std::string conf_path_;
  std::unique_ptr<FileWatcher> watcher_;
  Listener listener_;
  mutable std::mutex mu_;
  std::shared_ptr<const Snapshot> cur_;
  uint64_t gen_ = 0;
};

}  // namespace hola::config
