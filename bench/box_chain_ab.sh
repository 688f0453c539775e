#!/bin/bash
# Box session: two-hop chaining (loadgen -> A -> B) before/after the per-worker timeout FIFO
# and call slots in A's aloha client, interleaved.
set -o pipefail
OUT=${1:-gpurun_out/chain_ab}
mkdir -p "$OUT"
for i in 1 2 3; do
  timeout -k 10 90 python bench/chain_bench.py --duration 8 --exe-a build/ab/old_hola --out "$OUT/old_$i.json" > /dev/null 2>> "$OUT/err.log" &&
  timeout -k 10 90 python bench/chain_bench.py --duration 8 --out "$OUT/new_$i.json" > /dev/null 2>> "$OUT/err.log" || exit 1
done
