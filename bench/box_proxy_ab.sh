#!/bin/bash
# Box session: hola_rrproxy before/after the event-loop rewrite (edge-triggered sessions,
# L3 accept steering, busy-polling), interleaved, in the mirrored proxy core plan; plus the
# client-side round-robin reference point.
set -o pipefail
OUT=${1:-gpurun_out/proxy_ab}
mkdir -p "$OUT"
S="python -m hola_amd.parallel.scaling --replicas 1,4 --lb proxy --duration 6 --warmup 2 --busy-poll-us 20"
for i in 1 2; do
  timeout -k 10 120 $S --proxy-exe build/ab/old_rrproxy --proxy-busy-poll-us 0 --out "$OUT/old_$i.json" > "$OUT/old_$i.log" 2>&1 &&
  timeout -k 10 120 $S --out "$OUT/new_$i.json" > "$OUT/new_$i.log" 2>&1 || exit 1
done
timeout -k 10 120 $S --proxy-busy-poll-us 0 --out "$OUT/new_nobp.json" > "$OUT/new_nobp.log" 2>&1 &&
timeout -k 10 120 python -m hola_amd.parallel.scaling --replicas 1,4 --duration 6 --warmup 2 --busy-poll-us 20 --out "$OUT/client.json" > "$OUT/client.log" 2>&1
