#!/bin/bash
# Box session: pipelined (depth 16) and default bench after the single-pass response parsing
# in the load generator and the per-batch Request in the server.
set -o pipefail
OUT=${1:-gpurun_out/pipe2}
mkdir -p "$OUT"
timeout -k 10 200 python bench.py --pipeline 16 --steps 15 --warmup 3 --reqs-per-conn 400000 > "$OUT/bench_p16_1.json" 2>> "$OUT/err.log" &&
timeout -k 10 300 python bench.py > "$OUT/bench_default.json" 2>> "$OUT/err.log" &&
timeout -k 10 200 python bench.py --pipeline 16 --steps 15 --warmup 3 --reqs-per-conn 400000 > "$OUT/bench_p16_2.json" 2>> "$OUT/err.log"
