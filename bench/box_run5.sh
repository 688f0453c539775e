#!/bin/bash
# Box session: gpu-marked tests, the default headline bench (with loopback TCP segment counts
# per request), and a short bench with the servers' per-stage profile.
set -o pipefail
OUT=${1:-gpurun_out/run}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 300 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench.err" &&
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --profile-dir "$OUT/prof" > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err"
