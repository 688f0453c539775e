#!/bin/bash
# Box session: IPv4 vs IPv6 loopback repeat (3 interleaved pairs) and the default bench.
set -o pipefail
OUT=${1:-gpurun_out/v6b}
mkdir -p "$OUT"
run() {  # name, extra args
  local name=$1; shift
  timeout -k 10 120 python bench.py --steps 15 --warmup 3 "$@" > "$OUT/$name.json" 2>> "$OUT/err.log"
}
for rep in 1 2 3; do
  run "v6_$rep" --host ::1 && run "v4_$rep" --host 127.0.0.1 || exit 1
done
timeout -k 10 300 python bench.py > "$OUT/bench_default.json" 2>> "$OUT/err.log"
