#!/bin/bash
# Interleaved A/B of bench.py variants on the box: each variant runs REPS times, alternating.
# usage: bench/box_ab.sh OUT REPS "label|args" "label|args" ...
set -o pipefail
OUT=$1; REPS=$2; shift 2
mkdir -p "$OUT"
for rep in $(seq 1 "$REPS"); do
  for v in "$@"; do
    label=${v%%|*}; args=${v#*|}
    timeout -k 10 240 python bench.py --steps 15 --warmup 4 $args > "$OUT/${label}_${rep}.json" 2>> "$OUT/err.log" || exit 1
    python3 -c "import json,sys; d=json.load(open('$OUT/${label}_${rep}.json')); print('$label', $rep, d['value'], d['p50_ms'], d['p99_ms'], d['server_cpu_us_per_req'], d['loadgen_cpu_us_per_req'])" >> "$OUT/summary.txt"
  done
done
cat "$OUT/summary.txt"
