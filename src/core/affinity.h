// CPU pinning helpers: one event loop per pinned host core.
#pragma once
#include <string>
#include <vector>

namespace hola {

// Parses a Linux cpu-list ("0-3,8,10-11"); false on syntax error.
bool parse_cpu_list(const std::string& s, std::vector<int>* out);
std::string format_cpu_list(const std::vector<int>& cpus);
// CPUs in this process' affinity mask.
std::vector<int> allowed_cpus();
// Pins the calling thread to one CPU; false on failure (e.g. CPU not in the cgroup).
bool pin_current_thread(int cpu);
// Asks the scheduler for a `us`-microsecond time slice for the calling thread (EEVDF custom
// slice: sched_attr::sched_runtime of a SCHED_OTHER task, Linux 6.12+; an unprivileged thread
// may set its own). A shorter slice gives the thread earlier virtual deadlines, so it wins
// the CPU back sooner from a task that preempted it. Returns the slice the kernel reports
// afterwards in microseconds (0 when it does not support custom slices), -errno on failure.
long set_current_thread_slice_us(int us);
// The calling thread's current slice in microseconds as sched_getattr reports it (0 unknown).
long current_thread_slice_us();
// L3 cache domain (a CCD on EPYC) of a CPU from sysfs; -1 when unknown. Cached.
int l3_domain_of(int cpu);
// Physical core of a CPU: the lowest CPU id among its SMT siblings (sysfs
// thread_siblings_list); -1 when unknown. Cached.
int core_of(int cpu);
// The other SMT thread of `cpu`'s physical core (the first sibling that is not `cpu`), or
// `cpu` itself when it has none.
int sibling_of(int cpu);
// Socket (physical package) of a CPU from sysfs; -1 when unknown. Cached.
int package_of(int cpu);
// CPU quota from cgroup v2 cpu.max (e.g. 16.0 for "1600000 100000"); 0 when unlimited.
double cgroup_cpu_quota();

}  // namespace hola
