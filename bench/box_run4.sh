#!/bin/bash
# Box session: open-loop latency curve, chaining two-hop benchmark, default bench.
set -o pipefail
OUT=${1:-gpurun_out/run}
mkdir -p "$OUT"
timeout -k 10 200 python bench/latency_curve.py --duration 8 --out "$OUT/latency_curve.json" > "$OUT/latency_curve.log" 2>&1 &&
timeout -k 10 120 python bench/chain_bench.py --duration 10 --out "$OUT/chain_bench.json" > "$OUT/chain_bench.log" 2>&1 &&
timeout -k 10 300 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench.err"
