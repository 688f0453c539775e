#!/bin/bash
# Box session: BASELINE config 2 (1 connection) with the worker and its client on sibling SMT
# threads vs on two cores of one L3; busy-polling on/off in pair mode (config 3 shape).
set -o pipefail
OUT=${1:-gpurun_out/smt3}
mkdir -p "$OUT"
run() {  # name, extra args
  local name=$1; shift
  timeout -k 10 120 python bench.py --warmup 3 --profile-dir "$OUT/prof_$name" "$@" > "$OUT/$name.json" 2>> "$OUT/err.log"
}
for rep in 1 2; do
  run "c1_2cores_$rep" --connections 1 --cores 2 --steps 40 --reqs-per-conn 100000 &&
  run "c1_pair_$rep" --connections 1 --cores 1 --smt pair --steps 40 --reqs-per-conn 100000 &&
  run "pair_bp20_$rep" --cores 8 --smt pair --steps 15 &&
  run "pair_bp0_$rep" --cores 8 --smt pair --steps 15 --busy-poll-us 0 || exit 1
done
