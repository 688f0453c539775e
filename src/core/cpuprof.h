// Sampling CPU profiler for the server's own threads (`hola --cpu-profile FILE`).
//
// The GPU boxes have no perf and rocprofv3 sees no kernels here (the service dispatches none),
// so this is the host-side profile: each registered thread arms a timer on its own CPU-time
// clock (timer_create(CLOCK_THREAD_CPUTIME_ID) delivering SIGPROF to that thread), and the
// handler records a short call stack into a preallocated buffer by walking the frame-pointer
// chain from the interrupted context's RBP (the native code is built with
// -fno-omit-frame-pointer; every read is bounds-checked against the thread's stack). The walk
// is async-signal-safe: no unwinder, no loader lock, no allocation. Time spent inside a
// syscall is charged to the libc wrapper the thread returns to (send, recv, epoll_wait), so
// the profile also splits kernel time by call. At exit the samples and the executable
// mappings are written as text; `bench/cpuprof_report.py` symbolises them.
#pragma once
#include <cstdint>
#include <string>

namespace hola::cpuprof {

// Allocates the sample buffer and installs the SIGPROF handler; `hz` samples per second of
// each thread's CPU time. Returns false (and profiles nothing) on failure.
bool start(const std::string& path, int hz = 1000);
// Arms the calling thread's CPU-time timer (a no-op unless start() succeeded).
void register_thread();
// Disarms the calling thread's timer.
void unregister_thread();
// Disarms every timer and writes the profile file. Call once, after the threads have stopped.
bool write();

// ---- stacks of a thread that stopped answering (stall reports) ----
// The same frame-pointer walk, run on demand in the target thread by a real-time signal
// (40), whose handler only copies return addresses. Threads whose stacks may be captured call
// note_thread() once at start (it records their stack bounds, read by the walk).
constexpr int kMaxCaptureDepth = 32;
void note_thread();
// Installs the capture signal's handler (idempotent; false on failure).
bool enable_capture();
// Stack of the thread with kernel id `tid` in this process (innermost first), or 0 frames if it
// did not answer within timeout_ms (a thread stopped by ptrace, or blocking the signal). By
// tid, not pthread_t: a handle of a thread that has exited and been joined may not be used.
int capture(int tid, uintptr_t* pcs, int max, int timeout_ms = 200);
// The calling thread's kernel id.
int current_tid();
// " #0 hola+0x1234 #1 libc.so.6+0x5678 ..." from the current mappings.
std::string describe_pcs(const uintptr_t* pcs, int n);

}  // namespace hola::cpuprof
