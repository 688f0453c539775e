#!/bin/bash
# Box session: edge- vs level-triggered epoll on both sides (3 interleaved pairs), headline layout.
set -o pipefail
OUT=${1:-gpurun_out/et}
mkdir -p "$OUT"
run() {  # name, extra args
  local name=$1; shift
  timeout -k 10 120 python bench.py --steps 15 --warmup 3 --profile-dir "$OUT/prof_$name" "$@" > "$OUT/$name.json" 2>> "$OUT/err.log"
}
for rep in 1 2 3; do
  run "et_$rep" && run "lt_$rep" --epoll-lt || exit 1
done
