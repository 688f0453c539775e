#include "config/watcher.h"

#include <fcntl.h>
#include <limits.h>
#include <poll.h>
#include <sys/eventfd.h>
#include <sys/inotify.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>

#include "core/log.h"

namespace hola::config {

std::optional<std::string> read_file(const std::string& path) {
  // O_NONBLOCK: opening a FIFO must not block the watcher; only regular files are read.
  int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC | O_NONBLOCK);
  if (fd < 0) return std::nullopt;
  struct stat st;
  if (fstat(fd, &st) != 0 || !S_ISREG(st.st_mode)) {
    ::close(fd);
    return std::nullopt;
  }
  std::string s;
  char buf[8192];
  for (;;) {
    ssize_t n = ::read(fd, buf, sizeof buf);
    if (n < 0) {
      if (errno == EINTR) continue;
      ::close(fd);
      return std::nullopt;
    }
    if (n == 0) break;
    s.append(buf, size_t(n));
    if (s.size() > (4u << 20)) {  // config files are tiny; refuse /dev/zero-style inputs
      ::close(fd);
      return std::nullopt;
    }
  }
  ::close(fd);  // (the reference leaks this descriptor on every request: Configuration.java:29)
  return s;
}

namespace {
std::string parent_dir(const std::string& p) {
  size_t s = p.rfind('/');
  if (s == std::string::npos) return ".";
  if (s == 0) return "/";
  return p.substr(0, s);
}
}  // namespace

FileWatcher::FileWatcher(std::vector<std::string> paths, int poll_ms,
                         std::function<void(const Contents&)> on_change)
    : paths_(std::move(paths)), poll_ms_(poll_ms), on_change_(std::move(on_change)) {
  for (const auto& p : paths_) last_[p] = read_file(p);
  initial_ = last_;
}

FileWatcher::~FileWatcher() { stop(); }

void FileWatcher::add_watches() {
  const uint32_t mask = IN_CREATE | IN_MODIFY | IN_MOVED_TO | IN_MOVED_FROM | IN_DELETE |
                        IN_CLOSE_WRITE | IN_ATTRIB | IN_DELETE_SELF | IN_MOVE_SELF;
  for (auto& [wd, dir] : wds_) inotify_rm_watch(ifd_, wd);
  wds_.clear();
  std::vector<std::string> dirs;
  for (const auto& p : paths_) {
    dirs.push_back(parent_dir(p));
    // Follow a symlinked file to its real directory as well (e.g. ConfigMap ..data/...).
    char real[PATH_MAX];
    if (realpath(p.c_str(), real)) dirs.push_back(parent_dir(real));
  }
  for (const auto& d : dirs) {
    bool dup = false;
    for (auto& [wd, dir] : wds_) dup |= dir == d;
    if (dup) continue;
    int wd = inotify_add_watch(ifd_, d.c_str(), mask);
    if (wd >= 0) wds_[wd] = d;
  }
}

void FileWatcher::start() {
  if (paths_.empty() || running_.exchange(true)) return;
  ifd_ = inotify_init1(IN_NONBLOCK | IN_CLOEXEC);
  stopfd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  if (ifd_ >= 0) add_watches();
  else LOG_WARN("inotify unavailable (%s); config reload falls back to polling", strerror(errno));
  th_ = std::thread([this] { run(); });
}

void FileWatcher::stop() {
  if (!running_.exchange(false)) return;
  uint64_t one = 1;
  ssize_t r = ::write(stopfd_, &one, sizeof one);
  (void)r;
  if (th_.joinable()) th_.join();
  if (ifd_ >= 0) ::close(ifd_);
  if (stopfd_ >= 0) ::close(stopfd_);
  ifd_ = stopfd_ = -1;
}

bool FileWatcher::check() {
  Contents now;
  bool changed = false;
  for (const auto& p : paths_) {
    now[p] = read_file(p);
    if (now[p] != last_[p]) changed = true;
  }
  if (!changed) return false;
  last_ = now;
  reloads_.fetch_add(1);
  on_change_(last_);
  return true;
}

void FileWatcher::run() {
  char buf[16 * 1024] __attribute__((aligned(alignof(inotify_event))));
  while (running_.load()) {
    pollfd fds[2] = {{stopfd_, POLLIN, 0}, {ifd_, POLLIN, 0}};
    int n = ::poll(fds, ifd_ >= 0 ? 2 : 1, poll_ms_);
    if (!running_.load()) break;
    if (n > 0 && ifd_ >= 0 && (fds[1].revents & POLLIN)) {
      bool rewatch = false;
      ssize_t len;
      while ((len = ::read(ifd_, buf, sizeof buf)) > 0) {
        for (char* p = buf; p < buf + len;) {
          auto* ev = reinterpret_cast<inotify_event*>(p);
          if (ev->mask & (IN_DELETE_SELF | IN_MOVE_SELF | IN_IGNORED)) rewatch = true;
          p += sizeof(inotify_event) + ev->len;
        }
      }
      // Coalesce bursts (editors and ConfigMap swaps produce several events).
      ::usleep(5000);
      while (::read(ifd_, buf, sizeof buf) > 0) {
      }
      if (rewatch) add_watches();
      if (check()) add_watches();  // symlink targets may have moved
      continue;
    }
    check();  // periodic fallback (also covers filesystems without inotify)
  }
}

}  // namespace hola::config
