#!/bin/bash
# One gpurun session on the MI355X host. Replaces the per-session box_*.sh scripts.
#
#   gpurun -- 'bash bench/box_session.sh MODE OUT [ARGS...]'
#
# MODE
#   final              smoke(), pytest -m gpu, the default bench (the driver's round-end tiers)
#   bench ARGS...      one bench.py run with ARGS
#   repeat REPS [ARGS] the default bench REPS times (run-to-run spread)
#   instr label=BIN ... [--rounds N]   user-space instructions per request (bench/instr_ab.py)
#   ab REPS "label|args[|VAR=value]" ...   interleaved A/B of bench.py variants, REPS rounds; AB_SWAP=1 alternates the order
#   rehearsal [Ns]     the driver's own N>1 command line (default N = 2 4 8) inside the box's
#                      CPU slice, plus --profile-dir stage profiles for locality attribution
#   locality           N = 1, 2, 4, 8 in the box's slice, L3-grouped vs. plain connection dealing
#   scalemini [K] [NS] [PLAIN]  the miniature weak-scaling curve: K physical cores per replica at the
#                      8-slot node plan's places. bench.py's torchrun path at N = 1, 2, 4, 8 (node-plan
#                      dealing, then plain round-robin dealing), then hola_amd.parallel.scaling with
#                      client round-robin, reuseport and hola_rrproxy
#   pairmode           N = 1, 2, 4 with --smt pair (the 8-GPU node's per-replica layout shape)
#   latency            BASELINE config 2 (1 connection) and the open-loop latency curve
#   chain              two-hop chaining bench (loadgen -> hola A -> hola B)
#   tails              open-loop latency curves (auto x3, off x1) with per-point tail attribution
#   deployedab REPS [ARGS]  headline replica vs as-deployed (ZIPKIN_SERVER_URL as deployed /
#                      unset / native sink), interleaved (bench/deployed_ab.py)
#   chainwork          instructions per chained request (this tree, r5end, r4end) and user-cycles
#                      and CPU-time profiles of hola A
#   podshape [REPS] [ARGS]  the shipped pod shape's CPU per request, one thing varied at a time
#                      (bench/pod_shape.py), then the default bench
#   chainmodes REPS [ARGS]  bench.py's chain sub-run REPS times per variant with its attribution
#                      (bench/chain_modes.py; ARGS e.g. --variants lg0,lg20 --seconds 10)
#   chainab [REPS]     chaining with Feign BASIC logging on/off, this server vs. PREV_BIN
#   chainab2 [REPS]    chaining, this server vs. PREV_BIN (BASIC logging), order swapped each round
#   chainpipe [REPS]   chaining with --aloha-pipeline 8 vs. one request per connection
#   cpuprof            sampled CPU profiles (hola --cpu-profile) of the headline and of chaining
#   tracing            headline without a collector, with the native Zipkin sink (default 1000-span
#                      export budget, and unbounded), and with tracing off
#   soak MINUTES [ARGS] mixed-load soak sampling RSS and FDs (ARGS go to bench/soak.py)
#   busypoll [REPS]    the replica's busy-polling fixed / adaptive (auto) / off: saturated headline
#                      and server CPU at light load (open-loop curve)
#   uringchain         io_uring vs epoll on the chaining hop's four syscalls (bench/probes/uring_chain.cc)
#   kubesoak [MIN] [ARGS]  config 5 soak: back-to-back rollouts of the 8 pods under one continuous
#                      load (bench/kube_soak.py; ARGS e.g. --service proxy)
#   kube [ARGS]        BASELINE config 5: deploy/openshift applied by the local executor at real
#                      timings (8 pods, probes, rollouts under 512-connection load, SIGKILL,
#                      ConfigMap edit; ARGS go to bench/kube_rollout.py)
#
# Every GPU-box step runs under its own `timeout -k`, steps are chained with &&, and the
# script stops at the first failure (no retries).
set -o pipefail
MODE=${1:?mode}; OUT=${2:?out dir}; shift 2
mkdir -p "$OUT"
info() { python -m hola_amd info > "$OUT/info.txt" 2>&1 || true; }

case "$MODE" in
final)
  # the driver's round-end tiers, then the drain-hang trap: back-to-back
  # rollouts of the 8 pods with no shutdown delay under load; any termination that stalls
  # leaves its report in $OUT/kubesoak_nodelay/stalls/
  info
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 &&
  timeout -k 10 400 python bench.py > "$OUT/bench_default.json" 2>> "$OUT/err.log" &&
  timeout -k 10 420 python -u bench/kube_soak.py --minutes "${SOAK_MIN:-3}" --shutdown-delay-ms 0 \
    --out "$OUT/kubesoak_nodelay" > "$OUT/kubesoak_nodelay.json" 2> "$OUT/kubesoak_nodelay.log"
  ;;
bench)
  timeout -k 10 400 python bench.py "$@" > "$OUT/bench.json" 2>> "$OUT/err.log"
  ;;
instr)
  # user-space instructions per request of server binaries (bench/instr_ab.py: label=path ...)
  timeout -k 10 900 python -u bench/instr_ab.py "$OUT" "$@" > "$OUT/instr.log" 2>> "$OUT/err.log"
  ;;
uringchain)
  # the chaining hop's four syscalls per request: epoll vs one io_uring batch per loop pass
  g++ -O2 -std=c++20 -pthread bench/probes/uring_chain.cc -o /tmp/uring_chain &&
  timeout -k 10 200 /tmp/uring_chain --hop-cpu 8 --aloha-cpu 9 --client-cpus 10,11 --connections 64 \
    --rounds 6 --seconds 3 > "$OUT/uring_chain.jsonl" 2>> "$OUT/err.log"
  ;;
busypoll)
  # the replica's busy-polling: fixed 20 us (the headline), adaptive (auto) and off, under the
  # headline's saturation (interleaved benches), and the server CPU it costs at light load
  # (open-loop latency curve)
  REPS=${1:-3}
  for rep in $(seq 1 "$REPS"); do
    for v in fixed:20 auto:auto off:0; do
      label=${v%%:*}; bp=${v#*:}
      timeout -k 10 240 python bench.py --steps 12 --warmup 3 --c1-seconds 0 --deployed-seconds 0 \
        --server-busy-poll "$bp" > "$OUT/${label}_${rep}.json" 2>> "$OUT/err.log" || exit 1
      python3 -c "import json; d=json.load(open('$OUT/${label}_${rep}.json')); print('$label', $rep, d['value'], d['p50_ms'], d['p99_ms'], d['server_cpu_us_per_req'], d['host_load'][0]['siblings'])" \
        >> "$OUT/summary.txt"
    done
  done
  for v in fixed:20 auto:auto off:0; do
    label=${v%%:*}; bp=${v#*:}
    timeout -k 10 200 python bench/latency_curve.py --rates 50000,200000,1000000,2000000 --duration 4 \
      --busy-poll-us 20 --server-busy-poll "$bp" --out "$OUT/curve_${label}.json" > "$OUT/curve_${label}.log" 2>&1 || exit 1
  done
  cat "$OUT/summary.txt"
  ;;
kube)
  timeout -k 10 540 python -u bench/kube_rollout.py --out "$OUT/run" "$@" > "$OUT/kube.json" 2> "$OUT/kube.log"
  ;;
kubesoak)
  MIN=${1:-6}; shift || true
  timeout -k 10 $((MIN * 60 + 240)) python -u bench/kube_soak.py --minutes "$MIN" --out "$OUT/run" "$@" \
    > "$OUT/soak.json" 2> "$OUT/soak.log"
  ;;
repeat)
  # the default bench REPS times back to back: run-to-run spread of the headline on this host
  REPS=${1:-5}; shift
  for rep in $(seq 1 "$REPS"); do
    timeout -k 10 400 python bench.py "$@" > "$OUT/bench_$rep.json" 2>> "$OUT/err.log" || exit 1
  done
  ;;
ab)
  REPS=${1:?reps}; shift
  for rep in $(seq 1 "$REPS"); do
    # AB_SWAP=1: every other round runs the sides in reverse order (the first slot of a round
    # can be the slow one on this box: profiles/round4/03_chainab)
    sides=("$@")
    if [ "${AB_SWAP:-0}" = 1 ] && [ $((rep % 2)) = 0 ]; then
      sides=(); for ((k = $#; k >= 1; k--)); do sides+=("${!k}"); done
    fi
    for v in "${sides[@]}"; do
      # "label|bench args" or "label|bench args|VAR=value ..." (environment for that variant)
      label=${v%%|*}; rest=${v#*|}; args=${rest%%|*}; envs=""
      [ "$rest" != "$args" ] && envs=${rest#*|}
      env $envs timeout -k 10 240 python bench.py --steps 15 --warmup 4 $args > "$OUT/${label}_${rep}.json" \
        2>> "$OUT/err.log" || exit 1
      python3 -c "import json; d=json.load(open('$OUT/${label}_${rep}.json')); print('$label', $rep, d['value'], d['p50_ms'], d['p99_ms'], d['server_cpu_us_per_req'], d['loadgen_cpu_us_per_req'])" \
        >> "$OUT/summary.txt"
    done
  done
  cat "$OUT/summary.txt"
  ;;
rehearsal)
  NS=${*:-2 4 8}
  for n in $NS; do
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
      --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus "$n" --steps 8 --warmup 2 \
      --profile-dir "$OUT/prof_n$n" > "$OUT/n$n.json" 2> "$OUT/err_n$n.log" || exit $?
  done
  ;;
locality)
  # N>1 layouts inside the box's CPU slice: the planner's L3-grouped load generators vs. the
  # plain (i + rank) % N dealing from each rank's own cores, with stage profiles.
  for spec in "1|" "2|" "4|" "4|--plain-dealing" "8|" "8|--plain-dealing"; do
    n=${spec%%|*}; extra=${spec#*|}; tag=n$n${extra:+_plain}
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
      --master-addr 127.0.0.1 --master-port $((29700 + n)) bench.py --gpus "$n" --steps 8 --warmup 2 \
      --c1-seconds 0 --profile-dir "$OUT/prof_$tag" $extra > "$OUT/$tag.json" 2> "$OUT/err_$tag.log" || exit $?
  done
  ;;
scalemini)
  # K = physical cores per replica; NS = the replica counts (K x N x 2 CPUs must fit the quota)
  # PLAIN = the counts also run with --plain-dealing ("" = none); HARNESS_ONLY=1 skips bench.py
  K=${1:-1}; NS=${2:-"1 2 4 8"}; PLAIN=${3-"2 4 8"}
  specs=(); for n in $NS; do specs+=("$n|"); done; for n in $PLAIN; do specs+=("$n|--plain-dealing"); done
  [ "${HARNESS_ONLY:-0}" = 1 ] && specs=()
  for spec in "${specs[@]}"; do
    n=${spec%%|*}; extra=${spec#*|}; tag=n$n${extra:+_plain}
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
      --master-addr 127.0.0.1 --master-port $((29800 + n)) bench.py --gpus "$n" --gpu-slots 8 --slot-cores "$K" \
      --steps 10 --warmup 3 --c1-seconds 0 --deployed-seconds 0 --chain-seconds 0 --chain-shipped-seconds 0 \
      --alt-seconds 0 $extra > "$OUT/bench_$tag.json" 2> "$OUT/bench_err_$tag.log" || exit $?
  done
  for lb in ${LBS:-client reuseport proxy}; do
    ns=$(echo $NS | tr ' ' ,); [ "$lb" = proxy ] && ns=${PROXY_NS:-1,2,4}
    timeout -k 10 400 python -m hola_amd.parallel.scaling --slot-cores "$K" --slots 8 --replicas $ns --lb $lb \
      --duration 10 --warmup 2 --busy-poll-us 20 --server-busy-poll auto --busy-poll-pause 16 \
      --out "$OUT/scaling_$lb.json" > "$OUT/scaling_$lb.log" 2>&1 || exit $?
  done
  ;;
pairmode)
  # the 8-GPU node's layout shape (--smt pair: each server worker with its client thread on
  # one physical core) at N = 1, 2, 4 inside the box's 16-CPU quota
  for spec in "1|8" "2|4" "4|2"; do
    n=${spec%%|*}; cores=${spec#*|}
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
      --master-addr 127.0.0.1 --master-port $((29750 + n)) bench.py --gpus "$n" --cores "$cores" --smt pair \
      --steps 8 --warmup 2 --profile-dir "$OUT/prof_n$n" > "$OUT/pair_n$n.json" 2> "$OUT/err_n$n.log" || exit $?
  done
  ;;
latency)
  timeout -k 10 150 python bench.py --connections 1 --cores 2 --smt off --steps 15 --warmup 3 \
    --reqs-per-conn 200000 > "$OUT/config2_c1.json" 2>> "$OUT/err.log" &&
  timeout -k 10 200 python bench/latency_curve.py --duration 6 --out "$OUT/latency_curve.json" \
    > "$OUT/latency_curve.log" 2>&1
  ;;
chain)
  timeout -k 10 120 python bench/chain_bench.py --duration 10 --out "$OUT/chain.json" > "$OUT/chain.log" 2>&1
  ;;
tails)
  # open-loop curves of the shipped default (auto) three times and one
  # with busy-polling off, each point with its tail attribution (bench/latency_curve.py)
  info
  # what the scheduler lets an ordinary user do about other tasks on the job's CPUs
  { echo "rtprio limit: $(ulimit -r)"; echo "nice limit: $(ulimit -e)";
    echo "sched_rt_runtime_us: $(cat /proc/sys/kernel/sched_rt_runtime_us 2>/dev/null)";
    echo "base_slice_ns: $(cat /sys/kernel/debug/sched/base_slice_ns 2>/dev/null || echo n/a)";
    echo "kernel: $(uname -r)"; grep -h "^CONFIG_HZ=\|^CONFIG_PREEMPT" /boot/config-"$(uname -r)" 2>/dev/null;
    chrt -f 1 true 2>&1 && echo "SCHED_FIFO: allowed" || echo "SCHED_FIFO: refused";
    nice -n -5 true 2>&1 && echo "negative nice: allowed" || echo "negative nice: refused"; } > "$OUT/sched.txt" 2>&1
  # a name starting "off" runs the server without busy-polling; one ending "s" asks for a
  # ${SLICE:-100} us scheduler slice for the server's workers and the generator's threads
  for k in ${CURVES:-auto1 auto2 off auto3}; do
    bp=auto; [ "${k#off}" != "$k" ] && bp=0
    sl=0; [ "${k%s}" != "$k" ] && sl=${SLICE:-100}
    timeout -k 10 200 python bench/latency_curve.py --duration 6 --server-busy-poll "$bp" --sched-slice-us "$sl" \
      --out "$OUT/curve_$k.json" > "$OUT/curve_$k.log" 2>&1 || exit $?
  done
  ;;
deployedab)
  REPS=${1:-4}; shift || true
  timeout -k 10 1000 python -u bench/deployed_ab.py --reps "$REPS" --out "$OUT" "$@" > "$OUT/deployed_ab.log" 2>&1
  ;;
chainwork)
  # user-space instructions per chained request on hola A (this tree vs
  # round 5's end and round 4's end), then a user-cycles profile of A's workers (where the
  # remaining own-code cycles are) with the raw profile kept for address resolution
  info
  timeout -k 10 600 python -u bench/instr_ab.py "$OUT/instr" head=build/release/hola r5end=build/r5end/hola \
    ${SIDES:-r4end=build/r4end/hola} --chain --rounds "${ROUNDS:-3}" > "$OUT/instr.log" 2>&1 &&
  HOLA_CPUPROF_EVENT=user-cycles timeout -k 10 120 python bench/chain_bench.py --duration 8 \
    --cpu-profile "$OUT/chain_a_user.prof" --out "$OUT/chain_user.json" > "$OUT/chain_user.log" 2>&1 &&
  python bench/cpuprof_report.py "$OUT/chain_a_user.prof" --top 60 --json "$OUT/chain_user_report.json" \
    > "$OUT/chain_user_report.txt" 2>> "$OUT/err.log" &&
  HOLA_CPUPROF_EVENT=user-instructions timeout -k 10 120 python bench/chain_bench.py --duration 8 \
    --cpu-profile "$OUT/chain_a_instr.prof" --out "$OUT/chain_instr.json" > "$OUT/chain_instr.log" 2>&1 &&
  python bench/cpuprof_report.py "$OUT/chain_a_instr.prof" --top 80 --json "$OUT/chain_instr_report.json" \
    > "$OUT/chain_instr_report.txt" 2>> "$OUT/err.log" &&
  timeout -k 10 120 python bench/chain_bench.py --duration 8 --cpu-profile "$OUT/chain_a.prof" \
    --out "$OUT/chain.json" > "$OUT/chain.log" 2>&1 &&
  python bench/cpuprof_report.py "$OUT/chain_a.prof" --top 60 --json "$OUT/chain_report.json" \
    > "$OUT/chain_report.txt" 2>> "$OUT/err.log"
  ;;
podshape)
  # the pod shape (2 CPUs) vs 8 CPUs, one thing varied at a time, then the
  # default bench (its deployed_pod_* sub-run carries the same attribution)
  REPS=${1:-2}; shift || true
  info
  timeout -k 10 900 python -u bench/pod_shape.py --reps "$REPS" --out "$OUT" "$@" > "$OUT/pod_shape.log" 2>&1 &&
  timeout -k 10 420 python bench.py > "$OUT/bench_default.json" 2>> "$OUT/err.log"
  ;;
chainfinal)
  # instructions per chained request (this tree, round 5's and round 4's
  # servers), then bench.py's chain sub-run of each, interleaved with paired CIs, then the
  # default bench
  info
  timeout -k 10 600 python -u bench/instr_ab.py "$OUT/instr" head=build/release/hola r5end=build/r5end/hola \
    r4end=build/r4end/hola --chain --rounds "${ROUNDS:-3}" > "$OUT/instr.log" 2>&1 &&
  timeout -k 10 900 python -u bench/chain_modes.py --reps "${REPS:-6}" --seconds 10 \
    --variants lg0,lg0/r4end,lg0/r5end --out "$OUT/modes" > "$OUT/chain_modes.log" 2>&1 &&
  timeout -k 10 420 python bench.py > "$OUT/bench_default.json" 2>> "$OUT/err.log"
  ;;
chainmodes)
  REPS=${1:-10}; shift || true
  timeout -k 10 1000 python -u bench/chain_modes.py --reps "$REPS" --out "$OUT" "$@" > "$OUT/chain_modes.log" 2>&1
  ;;
chainab)
  # chaining with A's Feign BASIC logging on (the server default) and off, this tree's server
  # against PREV_BIN (a server built from an earlier commit), REPS interleaved rounds
  REPS=${1:-3}; PREV=${PREV_BIN:-build/prev/hola}
  for rep in $(seq 1 "$REPS"); do
    for v in "new_basic|basic|" "prev_basic|basic|$PREV" "new_none|none|"; do
      label=${v%%|*}; rest=${v#*|}; log=${rest%%|*}; exe=${rest#*|}
      timeout -k 10 120 python bench/chain_bench.py --duration 8 --feign-log "$log" ${exe:+--exe-a "$exe"} \
        --out "$OUT/${label}_${rep}.json" > "$OUT/${label}_${rep}.log" 2>&1 || exit 1
      python3 -c "import json; d=json.load(open('$OUT/${label}_${rep}.json')); print('$label', $rep, d['rps'], d['p50_ms'], d['p99_ms'], d['cpu_us_per_req']['A'], d['user_share']['A'])" \
        >> "$OUT/summary.txt"
    done
  done
  cat "$OUT/summary.txt"
  ;;
chainab2)
  # chaining, this server vs PREV_BIN, both with Feign BASIC logging, REPS rounds with the
  # order of the two sides swapped every round (an order effect would show as a difference
  # that flips with the order)
  REPS=${1:-6}; PREV=${PREV_BIN:-build/prev/hola}
  for rep in $(seq 1 "$REPS"); do
    if [ $((rep % 2)) -eq 1 ]; then order="new prev"; else order="prev new"; fi
    for v in $order; do
      exe=""; [ "$v" = prev ] && exe="$PREV"
      timeout -k 10 120 python bench/chain_bench.py --duration 8 --feign-log basic ${exe:+--exe-a "$exe"} \
        --out "$OUT/${v}_${rep}.json" > "$OUT/${v}_${rep}.log" 2>&1 || exit 1
      python3 -c "import json; d=json.load(open('$OUT/${v}_${rep}.json')); print('$v', $rep, d['rps'], d['p50_ms'], d['p99_ms'], d['cpu_us_per_req']['A'], d['user_share']['A'])" \
        >> "$OUT/summary.txt"
    done
  done
  cat "$OUT/summary.txt"
  ;;
chainpipe)
  # chaining with A's aloha calls pipelined (--aloha-pipeline 8) vs one request per connection
  # (the default), Feign BASIC logging on, REPS interleaved rounds
  REPS=${1:-3}
  for rep in $(seq 1 "$REPS"); do
    for pl in 1 8; do
      timeout -k 10 120 python bench/chain_bench.py --duration 8 --feign-log basic --aloha-pipeline $pl \
        --out "$OUT/pipe${pl}_${rep}.json" > "$OUT/pipe${pl}_${rep}.log" 2>&1 || exit 1
      python3 -c "import json; d=json.load(open('$OUT/pipe${pl}_${rep}.json')); print('pipe$pl', $rep, d['rps'], d['p50_ms'], d['p99_ms'], d['cpu_us_per_req']['A'], d['cpu_us_per_req']['B'], d['errors'], d['body_mismatch'])" \
        >> "$OUT/summary.txt"
    done
  done
  cat "$OUT/summary.txt"
  ;;
cpuprof)
  # sampled call stacks of the server's threads: the headline (1 replica, 64 connections) and
  # the chaining path with Feign BASIC logging, each symbolised on the box
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --c1-seconds 0 --cpu-profile-dir "$OUT/headline" \
    > "$OUT/headline.json" 2>> "$OUT/err.log" &&
  python bench/cpuprof_report.py "$OUT/headline/server_cpu_rank0.prof" --top 40 --json "$OUT/headline_report.json" \
    > "$OUT/headline_report.txt" 2>> "$OUT/err.log" &&
  python bench/cpuprof_report.py "$OUT/headline/loadgen_cpu_rank0.prof" --threads hola-lg --top 40 \
    --json "$OUT/loadgen_report.json" > "$OUT/loadgen_report.txt" 2>> "$OUT/err.log" &&
  timeout -k 10 120 python bench/chain_bench.py --duration 8 --feign-log basic --cpu-profile "$OUT/chain_a.prof" \
    --out "$OUT/chain.json" > "$OUT/chain.log" 2>&1 &&
  python bench/cpuprof_report.py "$OUT/chain_a.prof" --top 40 --json "$OUT/chain_report.json" \
    > "$OUT/chain_report.txt" 2>> "$OUT/err.log"
  ;;
tracing)
  timeout -k 10 300 python bench.py --steps 15 --warmup 3 --c1-seconds 0 > "$OUT/no_collector.json" 2>> "$OUT/err.log" &&
  timeout -k 10 300 python bench.py --steps 15 --warmup 3 --c1-seconds 0 --zipkin-sink > "$OUT/sink.json" 2>> "$OUT/err.log" &&
  timeout -k 10 300 python bench.py --steps 15 --warmup 3 --c1-seconds 0 --zipkin-sink --trace-queue 0 \
    > "$OUT/sink_unbounded.json" 2>> "$OUT/err.log" &&
  timeout -k 10 300 python bench.py --steps 15 --warmup 3 --c1-seconds 0 --no-tracing > "$OUT/tracing_off.json" 2>> "$OUT/err.log"
  ;;
soak)
  MIN=${1:-5}; shift || true
  timeout -k 10 $((MIN * 60 + 150)) python -u bench/soak.py --minutes "$MIN" --sample-s 30 "$@" \
    --out "$OUT/soak.json" > "$OUT/soak.log" 2>&1
  ;;
*)
  echo "unknown mode $MODE" >&2; exit 2
  ;;
esac
