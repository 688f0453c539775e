#!/bin/bash
# Box session: the SMT-pair layout the unconstrained 8-GPU node uses (`--smt auto` -> pair),
# rehearsed on the final tree: 2 ranks x 4 physical cores, cross-rank client-side
# round-robin, server stage profiles with the accept-steering counters; and 1 rank x 8.
set -o pipefail
OUT=${1:-gpurun_out/pair_check}
mkdir -p "$OUT"
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29581 bench.py --gpus 2 --cores 4 --smt pair --steps 15 --warmup 3 \
  --profile-dir "$OUT/prof_2rank" > "$OUT/2rank_pair.json" 2> "$OUT/err.log" &&
timeout -k 10 180 python bench.py --cores 8 --smt pair --steps 15 --warmup 3 \
  --profile-dir "$OUT/prof_1rank" > "$OUT/1rank_pair.json" 2>> "$OUT/err.log"
