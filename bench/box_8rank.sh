#!/bin/bash
# Box session: an 8-rank rehearsal of the driver's N=8 scaling run inside the 1-GPU box's
# 16-CPU slice (2 physical cores per rank, SMT pair): torchrun + gloo, 8 replicas, 512
# connections dealt round-robin over all replicas, per-replica steering counters.
set -o pipefail
OUT=${1:-gpurun_out/r8rank}
mkdir -p "$OUT"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29571 bench.py --gpus 8 --cores 2 --smt pair --steps 8 --warmup 2 --reqs-per-conn 4000 \
  --profile-dir "$OUT/prof" > "$OUT/8rank_pair.json" 2> "$OUT/err.log" &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29572 bench.py --gpus 4 --cores 4 --smt pair --steps 8 --warmup 2 --reqs-per-conn 8000 \
  > "$OUT/4rank_pair.json" 2>> "$OUT/err.log"
