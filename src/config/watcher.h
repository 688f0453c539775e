// Config-file hot reload without per-request I/O.
//
// The reference re-opens and re-parses the `-Dconf` file on every request
// (Configuration.java:27-29), so edits show up on the next request. Here one background
// thread watches the *parent directories* with inotify (a Kubernetes ConfigMap update
// atomically swaps the `..data` symlink, which a watch on the file itself would miss) and
// re-checks file contents every `poll_ms` as a fallback; listeners are called only when the
// bytes actually change.
#pragma once
#include <atomic>
#include <functional>
#include <map>
#include <mutex>
#include <optional>
#include <string>
#include <thread>
#include <vector>

namespace hola::config {

// Reads a whole file; nullopt when it cannot be opened.
std::optional<std::string> read_file(const std::string& path);

class FileWatcher {
 public:
  using Contents = std::map<std::string, std::optional<std::string>>;
  FileWatcher(std::vector<std::string> paths, int poll_ms,
              std::function<void(const Contents&)> on_change);
  ~FileWatcher();
  // Reads the files once (initial state, no callback) and starts the thread.
  void start();
  void stop();
  const Contents& initial() const { return initial_; }
  uint64_t reloads() const { return reloads_.load(); }

 private:
  void run();
  bool check();  // true if contents changed (callback invoked)
  void add_watches();
  std::vector<std::string> paths_;
  int poll_ms_;
  std::function<void(const Contents&)> on_change_;
  Contents last_, initial_;
  int ifd_ = -1, stopfd_ = -1;
  std::map<int, std::string> wds_;
  std::thread th_;
  std::atomic<bool> running_{false};
  std::atomic<uint64_t> reloads_{0};
};

}  // namespace hola::config
