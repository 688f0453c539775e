#!/bin/bash
# Box session: SMT A/B under the box's 16-CPU quota, interleaved.
#   c16     16 physical cores, siblings idle (the default bench layout)
#   c8      8 physical cores, siblings idle
#   c8pair  8 physical cores; worker on one SMT thread, its load-generator thread on the other
#   c8split 8 physical cores; each side uses both SMT threads of its own cores
set -o pipefail
OUT=${1:-gpurun_out/smt}
mkdir -p "$OUT"
run() {  # name, extra args
  local name=$1; shift
  timeout -k 10 120 python bench.py --steps 15 --warmup 3 --profile-dir "$OUT/prof_$name" "$@" > "$OUT/$name.json" 2>> "$OUT/err.log"
}
for rep in 1 2; do
  run "c16_$rep" &&
  run "c8_$rep" --cores 8 &&
  run "c8pair_$rep" --cores 8 --smt pair &&
  run "c8split_$rep" --cores 8 --smt split || exit 1
done
python - "$OUT" <<'PY' > "$OUT/summary.txt"
import json, glob, os, sys
out = sys.argv[1]
for f in sorted(glob.glob(os.path.join(out, "*.json"))):
    d = json.load(open(f))
    name = os.path.basename(f)[:-5]
    prof = json.load(open(os.path.join(out, "prof_" + name, "server_profile_rank0.json")))
    print(f"{name:12s} {d['value']:>12,.0f} req/s p50 {d['p50_ms']*1000:6.1f} us p99 {d['p99_ms']*1000:6.1f} us "
          f"srv {d['server_cpu_us_per_req']:.2f} us/req lg {d['loadgen_cpu_us_per_req']:.2f} us/req "
          f"send {prof['send']['mean']:.0f} ns steer {prof.get('steering')} map {d['config']['cpu_map']['rank0']}")
PY
cat "$OUT/summary.txt"
