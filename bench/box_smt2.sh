#!/bin/bash
# Box session: SMT pair sensitivity to connections per pair, 2-rank cross-rank pairing, and
# the default bench (--smt auto must resolve to off under the 16-CPU quota).
set -o pipefail
OUT=${1:-gpurun_out/smt2}
mkdir -p "$OUT"
python -c 'import bench; print("gpu_slots", bench._gpu_slots())' > "$OUT/slots.txt" 2>&1
run() {  # name, extra args
  local name=$1; shift
  timeout -k 10 120 python bench.py --steps 15 --warmup 3 --profile-dir "$OUT/prof_$name" "$@" > "$OUT/$name.json" 2>> "$OUT/err.log"
}
run pair_c64 --cores 8 --smt pair &&
run pair_c32 --cores 8 --smt pair --connections 32 &&
run pair_c16 --cores 8 --smt pair --connections 16 &&
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --cores 4 --smt pair --steps 15 --warmup 3 \
  --profile-dir "$OUT/prof_2rank" > "$OUT/2rank_pair.json" 2>> "$OUT/err.log" &&
timeout -k 10 300 python bench.py > "$OUT/bench_default.json" 2>> "$OUT/err.log"
