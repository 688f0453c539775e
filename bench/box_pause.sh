#!/bin/bash
# Box session: PAUSE backoff between empty busy polls, for SMT-paired layouts, plus
# BASELINE config 2 (1 connection) on two cores with siblings idle.
set -o pipefail
OUT=${1:-gpurun_out/pause}
mkdir -p "$OUT"
run() {  # name, extra args
  local name=$1; shift
  timeout -k 10 120 python bench.py --warmup 3 "$@" > "$OUT/$name.json" 2>> "$OUT/err.log"
}
for rep in 1 2; do
  for p in 0 16 64 256; do
    run "pair_p${p}_$rep" --cores 8 --smt pair --steps 15 --busy-poll-pause $p || exit 1
  done
done
run c1_off --connections 1 --cores 2 --smt off --server-threads 1 --steps 20 --reqs-per-conn 200000 &&
run c1_pair_p0 --connections 1 --cores 1 --smt pair --steps 20 --reqs-per-conn 200000 &&
run c1_pair_p64 --connections 1 --cores 1 --smt pair --steps 20 --reqs-per-conn 200000 --busy-poll-pause 64
