#!/bin/bash
# Box session: latency evidence on the current tree — BASELINE config 2 (1 connection, 1
# replica) and the open-loop (wrk2-style) latency curve; plus an io_uring availability probe.
set -o pipefail
OUT=${1:-gpurun_out/latency}
mkdir -p "$OUT"
python3 -c "
import ctypes, os
libc = ctypes.CDLL(None, use_errno=True)
p = ctypes.create_string_buffer(120)
r = libc.syscall(425, 8, p)
print('io_uring_setup:', r, os.strerror(ctypes.get_errno()) if r < 0 else 'ok')
" > "$OUT/io_uring_probe.txt" 2>&1
timeout -k 10 150 python bench.py --connections 1 --cores 2 --smt off --steps 15 --warmup 3 --reqs-per-conn 200000 \
  > "$OUT/config2_c1.json" 2>> "$OUT/err.log" &&
timeout -k 10 200 python bench/latency_curve.py --duration 6 --out "$OUT/latency_curve.json" > "$OUT/latency_curve.log" 2>&1
