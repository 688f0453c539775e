// Hystrix shard locks under contention, for the sanitizer builds.
//
// The per-thread shards of a Command are guarded by a test-and-set ShardLock released with a
// plain release store (src/resilience/hystrix.cc). This driver holds one shard's lock for a
// while, again and again, while eight "workers" run the request path (try_start, complete,
// circuit_open with a health snapshot refreshed on every call, so each refresh walks every
// shard and waits on the held one) and a reader takes snapshots (the /hystrix.stream and
// /metrics path). Under TSan any unsynchronised access is a report; under ASan a use after
// free; in every build the event totals must add up and nothing may deadlock.
//
// --per-thread runs the same with the per-thread bulkhead (Command::set_per_thread_bulkhead):
// the workers' shares and their borrowing from each other under the same pressure.
//
//   hola_hystrix_race [--iters N] [--per-thread]     exit 0 = consistent, 1 = counts wrong
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "core/clock.h"
#include "resilience/hystrix.h"

using hola::resilience::Command;
using hola::resilience::Event;
using hola::resilience::Settings;

int main(int argc, char** argv) {
  int iters = 20000;
  bool per_thread = false;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--iters") && i + 1 < argc) iters = atoi(argv[i + 1]);
    if (!strcmp(argv[i], "--per-thread")) per_thread = true;
  }
  Settings s;
  s.health_snapshot_ms = 0;          // every call refreshes the snapshot: walks all shards
  s.request_volume_threshold = 1 << 30;  // keep the breaker closed: every call is admitted
  s.pool_core_size = 1 << 20;
  if (per_thread) s.pool_core_size = 64;  // 4 slots per share: the workers borrow from each other
  Command cmd("aloha", "AlohaService", "AlohaService", s, hola::SystemClock::instance());
  cmd.set_per_thread_bulkhead(per_thread);

  constexpr int kWorkers = 8;
  std::atomic<bool> stop{false};
  std::atomic<int64_t> started{0}, holds{0};
  // the holder: shard 0's lock, held 200 us at a time; while held, it also reads the health
  // (its own refresh must skip nothing and not self-deadlock: it is a try-lock on health_mu_,
  // and the walk would wait on shard 0, so it reads the last snapshot instead)
  std::thread holder([&] {
    while (!stop.load(std::memory_order_relaxed)) {
      cmd.hold_shard_for_test(0, [&] {
        holds.fetch_add(1, std::memory_order_relaxed);
        std::this_thread::sleep_for(std::chrono::microseconds(200));
      });
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  });
  std::thread reader([&] {
    int64_t last = 0;
    while (!stop.load(std::memory_order_relaxed)) {
      auto snap = cmd.snapshot();
      const int64_t done = snap.cumulative[size_t(Event::kSuccess)] + snap.cumulative[size_t(Event::kFailure)];
      if (done < last) {
        fprintf(stderr, "cumulative count went backwards: %lld < %lld\n", (long long)done, (long long)last);
        std::exit(1);
      }
      last = done;
      std::this_thread::sleep_for(std::chrono::microseconds(300));
    }
  });
  std::vector<std::thread> workers;
  for (int w = 0; w < kWorkers; ++w)
    workers.emplace_back([&, w] {
      for (int i = 0; i < iters; ++i) {
        if (cmd.try_start() != Command::Admit::kRun) continue;
        started.fetch_add(1, std::memory_order_relaxed);
        const bool ok = (i + w) % 4 != 0;
        cmd.complete(ok ? Event::kSuccess : Event::kFailure, 1, !ok, 2);
        (void)cmd.circuit_open();
      }
    });
  for (auto& t : workers) t.join();
  stop.store(true);
  holder.join();
  reader.join();

  auto snap = cmd.snapshot();
  const int64_t ok = snap.cumulative[size_t(Event::kSuccess)], bad = snap.cumulative[size_t(Event::kFailure)];
  printf("{\"started\":%lld,\"success\":%lld,\"failure\":%lld,\"holds\":%lld,\"active\":%lld}\n",
         (long long)started.load(), (long long)ok, (long long)bad, (long long)holds.load(),
         (long long)snap.pool_active);
  if (ok + bad != started.load() || snap.pool_active != 0 || holds.load() == 0) return 1;
  return 0;
}
