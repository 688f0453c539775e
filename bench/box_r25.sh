#!/bin/bash
# Box session r25: driver-equivalent checks on the current tree (smoke(), gpu-marked tests)
# and the default bench (slot_cores default, IPv6 loopback, edge-triggered epoll).
set -o pipefail
OUT=${1:-gpurun_out/r25}
mkdir -p "$OUT"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 300 python bench.py > "$OUT/bench_default.json" 2>> "$OUT/err.log"
