// fpstack PID — one call stack per thread of a running process, by frame-pointer walk.
//
// A diagnostic for a process that is alive but not progressing (a replica that outlives its
// grace period): each thread is stopped briefly with PTRACE_SEIZE + PTRACE_INTERRUPT, its
// registers read, and its RBP chain walked through /proc/PID/mem (the native code is built
// with frame pointers; libc has none, so the stack above rsp is also scanned for return
// addresses into the other mappings). The box has no gdb or perf.
// Output: one line per thread, `tid name state pc frame...`, addresses as `module+offset`,
// ready for `addr2line -f -C -e <module>`.
//
//   g++ -O2 -std=c++20 bench/probes/fpstack.cc -o /tmp/fpstack && /tmp/fpstack PID
#include <dirent.h>
#include <fcntl.h>
#include <signal.h>
#include <sys/ptrace.h>
#include <sys/user.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cerrno>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

namespace {

struct Map {
  uintptr_t lo, hi, off;
  std::string path;
};

std::vector<Map> read_maps(int pid) {
  std::vector<Map> out;
  std::ifstream f("/proc/" + std::to_string(pid) + "/maps");
  for (std::string line; std::getline(f, line);) {
    std::istringstream s(line);
    std::string range, perms, off, dev, inode, path;
    s >> range >> perms >> off >> dev >> inode;
    std::getline(s >> std::ws, path);
    if (perms.size() < 3 || perms[2] != 'x') continue;
    const size_t dash = range.find('-');
    out.push_back({std::stoull(range.substr(0, dash), nullptr, 16), std::stoull(range.substr(dash + 1), nullptr, 16),
                   std::stoull(off, nullptr, 16), path});
  }
  return out;
}

std::string where(const std::vector<Map>& maps, uintptr_t pc) {
  for (const Map& m : maps)
    if (pc >= m.lo && pc < m.hi) {
      char b[64];
      snprintf(b, sizeof b, "+0x%lx", (unsigned long)(pc - m.lo + m.off));
      const size_t slash = m.path.rfind('/');
      return (slash == std::string::npos ? m.path : m.path.substr(slash + 1)) + b;
    }
  char b[32];
  snprintf(b, sizeof b, "0x%lx", (unsigned long)pc);
  return b;
}

std::string slurp(const std::string& p) {
  std::ifstream f(p);
  std::string s;
  std::getline(f, s, '\0');
  while (!s.empty() && (s.back() == '\n' || s.back() == ' ')) s.pop_back();
  return s;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 2) {
    fprintf(stderr, "usage: fpstack PID\n");
    return 2;
  }
  const int pid = atoi(argv[1]);
  const auto maps = read_maps(pid);
  const int mem = open(("/proc/" + std::to_string(pid) + "/mem").c_str(), O_RDONLY);
  if (mem < 0) {
    perror("open mem");
    return 1;
  }
  DIR* d = opendir(("/proc/" + std::to_string(pid) + "/task").c_str());
  if (!d) {
    perror("opendir");
    return 1;
  }
  std::vector<int> tids;
  while (dirent* e = readdir(d))
    if (e->d_name[0] != '.') tids.push_back(atoi(e->d_name));
  closedir(d);
  for (int tid : tids) {
    const std::string base = "/proc/" + std::to_string(pid) + "/task/" + std::to_string(tid);
    const std::string stat = slurp(base + "/stat");
    const size_t lp = stat.find('('), rp = stat.rfind(')');
    const std::string name = lp != std::string::npos && rp != std::string::npos ? stat.substr(lp + 1, rp - lp - 1) : "?";
    const char state = rp != std::string::npos && rp + 2 < stat.size() ? stat[rp + 2] : '?';
    printf("%d %s %c", tid, name.c_str(), state);
    if (ptrace(PTRACE_SEIZE, tid, 0, 0) != 0) {
      printf(" (seize: %s)\n", strerror(errno));
      continue;
    }
    ptrace(PTRACE_INTERRUPT, tid, 0, 0);
    int st = 0;
    if (waitpid(tid, &st, __WALL) == tid) {
      user_regs_struct r{};
      if (ptrace(PTRACE_GETREGS, tid, 0, &r) == 0) {
        printf(" pc=%s", where(maps, uintptr_t(r.rip)).c_str());
        // a libc leaf (syscall wrapper) keeps no frame: its return address is at rsp
        uintptr_t ret = 0;
        if (pread(mem, &ret, sizeof ret, off_t(r.rsp)) == sizeof ret) printf(" [rsp]=%s", where(maps, ret).c_str());
        // libc keeps no frame pointers, so a thread waiting in libc has no usable chain: scan
        // the stack above rsp for words that point into other executable mappings (the
        // nearest are the return addresses of its callers; a scan can also find stale ones)
        {
          uintptr_t words[512];
          const ssize_t got = pread(mem, words, sizeof words, off_t(r.rsp));
          int shown = 0;
          printf(" scan:");
          for (ssize_t k = 0; k < got / ssize_t(sizeof(uintptr_t)) && shown < 6; ++k) {
            const std::string w = where(maps, words[k]);
            if (w.rfind("0x", 0) == 0 || w.rfind("libc.so", 0) == 0) continue;
            printf(" %s", w.c_str());
            ++shown;
          }
          printf(" |");
        }
        uintptr_t fp = uintptr_t(r.rbp);
        for (int k = 0; k < 24 && fp; ++k) {
          uintptr_t fr[2];
          if (pread(mem, fr, sizeof fr, off_t(fp)) != sizeof fr || fr[1] == 0) break;
          printf(" %s", where(maps, fr[1]).c_str());
          if (fr[0] <= fp) break;
          fp = fr[0];
        }
      }
    }
    ptrace(PTRACE_DETACH, tid, 0, 0);
    printf("\n");
  }
  return 0;
}
