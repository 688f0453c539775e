#!/bin/bash
# One measurement session on the MI355X box (called through gpurun). Every step has its own
# time limit and the steps are chained with && so the first failure ends the session.
set -o pipefail
OUT=${1:-gpurun_out/run}
mkdir -p "$OUT"
{ nproc; cat /sys/fs/cgroup/cpu.max; python3 -m hola_amd info; } > "$OUT/env.txt" 2>&1
timeout -k 10 300 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --profile-dir "$OUT/profile" > "$OUT/bench_profiled.json" 2>> "$OUT/bench_default.err" &&
timeout -k 10 200 python3 -c "
import json, sys
sys.path.insert(0, '.')
from hola_amd.server import HolaProcess
from hola_amd.parallel.loadgen import run_duration
from hola_amd.utils.cpu import plan_node, split_server_loadgen, format_cpu_list
cores = plan_node(1)[0]
srv, lg = split_server_loadgen(cores, len(cores) // 2)
res = {'cpu_map': {'server': format_cpu_list(srv), 'loadgen': format_cpu_list(lg)}}
with HolaProcess(env={'HOSTNAME': 'h'}, threads=len(srv), cpu_list=format_cpu_list(srv), port=18900, log_level='warn') as s:
    # BASELINE.json config 2 (1 connection, 30 s) and config 3 (64 connections, 30 s)
    res['config2_c1_30s'] = run_duration([('127.0.0.1', s.port)], 1, 1, 30.0, 2.0, cpu_list=format_cpu_list(lg[:1]))
    res['config3_c64_30s'] = run_duration([('127.0.0.1', s.port)], 64, len(lg), 30.0, 2.0, cpu_list=format_cpu_list(lg))
json.dump(res, open('$OUT/configs_2_3.json', 'w'), indent=1)
" > "$OUT/configs.log" 2>&1 &&
timeout -k 10 300 python3 -m hola_amd scaling --replicas 1,2,4,8 --duration 10 --out "$OUT/scaling_client_rr.json" > "$OUT/scaling_client_rr.log" 2>&1 &&
timeout -k 10 300 python3 -m hola_amd scaling --replicas 1,2,4,8 --duration 10 --lb proxy --proxy-threads 2 --out "$OUT/scaling_proxy.json" > "$OUT/scaling_proxy.log" 2>&1
