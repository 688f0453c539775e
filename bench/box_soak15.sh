#!/bin/bash
# Box session: a 15-minute mixed-load soak on the final tree (closed-loop /api/hola, chaining
# against a fault-cycling fake aloha, /hystrix.stream subscribers, /metrics scrapes, config
# reloads), sampling RSS and FDs every 30 s.
set -o pipefail
OUT=${1:-gpurun_out/soak15}
mkdir -p "$OUT"
timeout -k 10 1050 python -u bench/soak.py --minutes 15 --sample-s 30 --out "$OUT/soak.json" > "$OUT/soak.log" 2>&1
