#!/bin/bash
# Box session: io_uring vs edge-triggered epoll for one saturated loopback request/response
# server thread (bench/probes/uring_vs_epoll.cc), interleaved rounds.
set -o pipefail
OUT=${1:-gpurun_out/uring}
mkdir -p "$OUT" build/probes
g++ -O2 -std=c++20 -march=x86-64-v3 -o build/probes/uring_vs_epoll bench/probes/uring_vs_epoll.cc -lpthread &&
timeout -k 10 120 build/probes/uring_vs_epoll --server-cpu 16 --client-cpus 17,18,19 --connections 24 --seconds 3 --rounds 4 \
  > "$OUT/uring_vs_epoll.jsonl" 2> "$OUT/err.log" &&
timeout -k 10 120 build/probes/uring_vs_epoll --server-cpu 16 --client-cpus 17,18,19 --connections 3 --seconds 3 --rounds 3 \
  > "$OUT/uring_vs_epoll_c3.jsonl" 2>> "$OUT/err.log"
