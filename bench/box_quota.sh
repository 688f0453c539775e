#!/bin/bash
# Box session: does the 16-CPU CFS quota throttle the headline layout (16 busy threads plus
# the control plane)? Interleaved: default (8 server + 8 loadgen threads) vs 15 threads
# (8+7 and 7+8), with cgroup cpu.stat throttling deltas in every line; then the pipelined
# bench after the loadgen's in-place response parsing.
set -o pipefail
OUT=${1:-gpurun_out/quota}
mkdir -p "$OUT"
B="python bench.py --steps 15 --warmup 3"
for i in 1 2; do
  timeout -k 10 120 $B > "$OUT/c16_s8_$i.json" 2>> "$OUT/err.log" &&
  timeout -k 10 120 $B --cores 15 --server-threads 8 > "$OUT/c15_s8_$i.json" 2>> "$OUT/err.log" &&
  timeout -k 10 120 $B --cores 15 --server-threads 7 > "$OUT/c15_s7_$i.json" 2>> "$OUT/err.log" || exit 1
done
timeout -k 10 200 python bench.py --pipeline 16 --steps 15 --warmup 3 --reqs-per-conn 400000 > "$OUT/bench_p16.json" 2>> "$OUT/err.log"
