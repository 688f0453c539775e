#include "core/affinity.h"

#include <pthread.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cerrno>
#include <cstdint>

#include <cstdio>
#include <cstdlib>
#include <fstream>

namespace hola {

bool parse_cpu_list(const std::string& s, std::vector<int>* out) {
  out->clear();
  size_t i = 0;
  while (i < s.size()) {
    size_t j = s.find(',', i);
    if (j == std::string::npos) j = s.size();
    std::string tok = s.substr(i, j - i);
    i = j + 1;
    if (tok.empty()) continue;
    size_t dash = tok.find('-');
    char* end = nullptr;
    long a = strtol(tok.c_str(), &end, 10);
    if (end == tok.c_str() || a < 0) return false;
    long b = a;
    if (dash != std::string::npos) {
      b = strtol(tok.c_str() + dash + 1, &end, 10);
      if (*end || b < a) return false;
    } else if (*end) {
      return false;
    }
    for (long c = a; c <= b; ++c) out->push_back(int(c));
  }
  return true;
}

std::string format_cpu_list(const std::vector<int>& cpus) {
  std::string r;
  size_t i = 0;
  while (i < cpus.size()) {
    size_t j = i;
    while (j + 1 < cpus.size() && cpus[j + 1] == cpus[j] + 1) ++j;
    if (!r.empty()) r += ",";
    r += std::to_string(cpus[i]);
    if (j > i) r += "-" + std::to_string(cpus[j]);
    i = j + 1;
  }
  return r;
}

std::vector<int> allowed_cpus() {
  cpu_set_t set;
  CPU_ZERO(&set);
  std::vector<int> r;
  if (sched_getaffinity(0, sizeof set, &set) != 0) return r;
  for (int c = 0; c < CPU_SETSIZE; ++c)
    if (CPU_ISSET(c, &set)) r.push_back(c);
  return r;
}

bool pin_current_thread(int cpu) {
  cpu_set_t set;
  CPU_ZERO(&set);
  CPU_SET(cpu, &set);
  return pthread_setaffinity_np(pthread_self(), sizeof set, &set) == 0;
}

namespace {
struct SchedAttr {  // struct sched_attr, SCHED_ATTR_SIZE_VER1
  uint32_t size;
  uint32_t sched_policy;
  uint64_t sched_flags;
  int32_t sched_nice;
  uint32_t sched_priority;
  uint64_t sched_runtime;
  uint64_t sched_deadline;
  uint64_t sched_period;
  uint32_t sched_util_min;
  uint32_t sched_util_max;
};
}  // namespace

long current_thread_slice_us() {
  SchedAttr a{};
  if (syscall(SYS_sched_getattr, 0, &a, unsigned(sizeof a), 0u) != 0) return 0;
  return long(a.sched_runtime / 1000);
}

long set_current_thread_slice_us(int us) {
  SchedAttr a{};
  if (syscall(SYS_sched_getattr, 0, &a, unsigned(sizeof a), 0u) != 0) return -errno;
  if (a.sched_policy != SCHED_OTHER && a.sched_policy != SCHED_BATCH) return -EINVAL;
  a.size = sizeof a;
  a.sched_flags = 0;
  a.sched_runtime = uint64_t(us) * 1000;  // the kernel clamps it to [0.1 ms, 100 ms]
  if (syscall(SYS_sched_setattr, 0, &a, 0u) != 0) return -errno;
  return current_thread_slice_us();
}

int l3_domain_of(int cpu) {
  // Read once for every possible CPU (thread-safe static init); lookups are then lock-free.
  static const std::vector<int> table = [] {
    std::vector<int> v;
    for (int c = 0; c < CPU_SETSIZE; ++c) {
      std::ifstream f("/sys/devices/system/cpu/cpu" + std::to_string(c) + "/cache/index3/id");
      if (!f) {
        if (c > 0 && v.size() == size_t(c)) {
          std::ifstream online("/sys/devices/system/cpu/cpu" + std::to_string(c));
          if (!online) break;  // past the last CPU
        }
        v.push_back(-1);
        continue;
      }
      int id = -1;
      if (!(f >> id)) id = -1;
      v.push_back(id);
    }
    return v;
  }();
  return (cpu >= 0 && size_t(cpu) < table.size()) ? table[size_t(cpu)] : -1;
}

int core_of(int cpu) {
  static const std::vector<int> table = [] {
    std::vector<int> v;
    for (int c = 0; c < CPU_SETSIZE; ++c) {
      std::ifstream f("/sys/devices/system/cpu/cpu" + std::to_string(c) + "/topology/thread_siblings_list");
      if (!f) {
        std::ifstream online("/sys/devices/system/cpu/cpu" + std::to_string(c));
        if (!online) break;  // past the last CPU
        v.push_back(-1);
        continue;
      }
      std::string line;
      std::vector<int> sib;
      if (std::getline(f, line) && parse_cpu_list(line, &sib) && !sib.empty()) {
        int lo = sib[0];
        for (int x : sib) lo = x < lo ? x : lo;
        v.push_back(lo);
      } else {
        v.push_back(-1);
      }
    }
    return v;
  }();
  return (cpu >= 0 && size_t(cpu) < table.size()) ? table[size_t(cpu)] : -1;
}

int sibling_of(int cpu) {
  std::ifstream f("/sys/devices/system/cpu/cpu" + std::to_string(cpu) + "/topology/thread_siblings_list");
  std::string line;
  std::vector<int> sib;
  if (f && std::getline(f, line) && parse_cpu_list(line, &sib))
    for (int x : sib)
      if (x != cpu) return x;
  return cpu;
}

int package_of(int cpu) {
  static const std::vector<int> table = [] {
    std::vector<int> v;
    for (int c = 0; c < CPU_SETSIZE; ++c) {
      std::ifstream f("/sys/devices/system/cpu/cpu" + std::to_string(c) + "/topology/physical_package_id");
      if (!f) {
        std::ifstream online("/sys/devices/system/cpu/cpu" + std::to_string(c));
        if (!online) break;  // past the last CPU
        v.push_back(-1);
        continue;
      }
      int id = -1;
      if (!(f >> id)) id = -1;
      v.push_back(id);
    }
    return v;
  }();
  return (cpu >= 0 && size_t(cpu) < table.size()) ? table[size_t(cpu)] : -1;
}

namespace {
// "QUOTA PERIOD" (cpu.max's format) as CPUs; 0 for "max" or anything unreadable.
double parse_cpu_max(const std::string& q, const std::string& p) {
  if (q.empty() || q == "max") return 0;
  const double qv = atof(q.c_str()), pv = atof(p.c_str());
  return pv > 0 && qv > 0 ? qv / pv : 0;
}
}  // namespace

double cgroup_cpu_quota() {
  double quota = 0;
  {
    std::ifstream f("/sys/fs/cgroup/cpu.max");
    std::string q, p;
    if (f >> q >> p) quota = parse_cpu_max(q, p);
  }
  // HOLA_CGROUP_CPU_MAX (cpu.max's format) stands in for the pod's own cgroup where the
  // container runtime cannot write one: the local manifest executor sets it from limits.cpu
  // and enforces it from user space (hola_amd/kube/kubelet.py, CpuBandwidth). Nested quotas
  // bound each other, so the lower one counts.
  if (const char* e = getenv("HOLA_CGROUP_CPU_MAX")) {
    std::string s(e);
    const size_t sp = s.find(' ');
    const double pod = parse_cpu_max(s.substr(0, sp), sp == std::string::npos ? "100000" : s.substr(sp + 1));
    if (pod > 0 && (quota == 0 || pod < quota)) quota = pod;
  }
  return quota;
}

}  // namespace hola
