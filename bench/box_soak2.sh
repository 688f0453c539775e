#!/bin/bash
# Box session: a 4-minute mixed-load soak with edge-triggered sockets (parked chaining calls,
# SSE subscribers, config reloads, fault-cycling fake aloha), then the two-hop chaining bench.
set -o pipefail
OUT=${1:-gpurun_out/soak2}
mkdir -p "$OUT"
timeout -k 10 330 python -u bench/soak.py --minutes 4 --sample-s 10 --out "$OUT/soak.json" > "$OUT/soak.log" 2>&1 &&
timeout -k 10 120 python bench/chain_bench.py --duration 10 --out "$OUT/chain_bench.json" > "$OUT/chain_bench.log" 2>&1
