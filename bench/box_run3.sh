#!/bin/bash
# Box session: relocated-tree rebuild check, syscall cost probe, gpu tests, default bench.
set -o pipefail
OUT=${1:-gpurun_out/run}
mkdir -p "$OUT"
g++ -O2 -o /tmp/syscall_cost bench/probes/syscall_cost.cc && timeout -k 5 60 /tmp/syscall_cost > "$OUT/syscall_cost.json" &&
touch src/main.cc && timeout -k 10 300 python3 -c "
import time, sys
sys.path.insert(0, '.')
from hola_amd import native
t = time.time(); native.ensure_built('release'); print('rebuild_s', round(time.time() - t, 1))
" > "$OUT/rebuild.txt" 2>&1 &&
timeout -k 10 300 python -m pytest tests -x -q -m gpu > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 300 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench.err"
