#!/bin/bash
# Box session: the round-end checks on the current tree — smoke(), pytest -m gpu, the
# default bench (with replica RSS after the tracer-ring change), and `hola_amd info`.
set -o pipefail
OUT=${1:-gpurun_out/final2}
mkdir -p "$OUT"
python -m hola_amd info > "$OUT/info.txt" 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 300 python bench.py > "$OUT/bench_default.json" 2>> "$OUT/err.log"
