#!/bin/bash
# Box session: pipelined closed loop (wrk pipeline.lua shape, TechEmpower plaintext depth 16)
# with the server stage profile, plus depth 1 with the same profile for comparison, and the
# micro-costs of the per-request user-space path.
set -o pipefail
OUT=${1:-gpurun_out/pipe}
mkdir -p "$OUT"
timeout -k 10 60 build/release/hola_micro > "$OUT/micro.json" 2>> "$OUT/err.log" &&
timeout -k 10 200 python bench.py --pipeline 16 --steps 15 --warmup 3 --reqs-per-conn 400000 > "$OUT/bench_p16.json" 2>> "$OUT/err.log" &&
timeout -k 10 200 python bench.py --pipeline 16 --steps 8 --warmup 2 --reqs-per-conn 400000 --profile-dir "$OUT/prof_p16" > "$OUT/bench_p16_prof.json" 2>> "$OUT/err.log" &&
timeout -k 10 200 python bench.py --steps 8 --warmup 2 --profile-dir "$OUT/prof_p1" > "$OUT/bench_p1_prof.json" 2>> "$OUT/err.log"
