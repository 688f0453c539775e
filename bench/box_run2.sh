#!/bin/bash
# Box session: default bench (steering on/off A/B, interleaved twice), multi-rank bench
# rehearsals at N=2 and N=4 over gloo (16-CPU box: 8 and 4 CPUs per rank), scaling curve.
set -o pipefail
OUT=${1:-gpurun_out/run}
mkdir -p "$OUT"
B="timeout -k 10 240 python bench.py --steps 20 --warmup 5"
$B > "$OUT/bench_a1.json" 2> "$OUT/err.log" &&
$B --profile-dir "$OUT/prof_a" > "$OUT/bench_profiled.json" 2>> "$OUT/err.log" &&
$B > "$OUT/bench_a2.json" 2>> "$OUT/err.log" &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 > "$OUT/bench_n2.log" 2>> "$OUT/err.log" &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 20 --warmup 5 > "$OUT/bench_n4.log" 2>> "$OUT/err.log" &&
timeout -k 10 300 python3 -m hola_amd scaling --replicas 1,2,4,8 --duration 8 --out "$OUT/scaling_client_rr.json" > "$OUT/scaling_client_rr.log" 2>&1 &&
timeout -k 10 300 python3 -m hola_amd scaling --replicas 1,2,4 --duration 8 --lb proxy --proxy-threads 4 --out "$OUT/scaling_proxy.json" > "$OUT/scaling_proxy.log" 2>&1
