// Hardware counters of a thread's own user-space work: instructions and cycles, counted by the
// PMU for the thread that opened them (perf_event_open, user space only: allowed for one's own
// threads at perf_event_paranoid <= 2; a container whose seccomp profile refuses the call
// simply has no counters). Counting costs nothing on the counted thread; a read is one
// read(2) from any thread.
//
// The figure the CPU-time efficiency numbers cannot give at saturation:
// a server and its load generator that both run flat out spend the same CPU time per request
// by construction (their CPUs' wall time over one request count), while the instructions and
// cycles each spends in its own code are its own.
#pragma once
#include <atomic>
#include <cstdint>

namespace hola {

class ThreadCounters {
 public:
  ThreadCounters() = default;
  ~ThreadCounters();
  ThreadCounters(const ThreadCounters&) = delete;
  ThreadCounters& operator=(const ThreadCounters&) = delete;

  // Opens the counters for the calling thread; false (and no counters) when not permitted.
  bool open();
  bool is_open() const { return fd_.load(std::memory_order_acquire) >= 0; }
  // Totals since open(), scaled by the time the PMU actually counted them (when counters are
  // multiplexed with other users). False when closed or unreadable.
  bool read(uint64_t* instructions, uint64_t* cycles) const;

 private:
  // group leader (instructions): published by the opening thread, read by the metrics thread
  std::atomic<int> fd_{-1};
  int fd_cycles_ = -1;
};

}  // namespace hola
