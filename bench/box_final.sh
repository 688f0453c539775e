#!/bin/bash
# Box session: gpu-marked tests, a 2-rank SMT-pair rehearsal of the full-node layout with the
# current defaults (edge-triggered epoll, IPv6 loopback, PAUSE backoff), and the default bench.
set -o pipefail
OUT=${1:-gpurun_out/final}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --gpus 2 --cores 4 --smt pair --steps 15 --warmup 3 \
  --profile-dir "$OUT/prof_2rank" > "$OUT/2rank_pair.json" 2>> "$OUT/err.log" &&
timeout -k 10 300 python bench.py > "$OUT/bench_default.json" 2>> "$OUT/err.log"
