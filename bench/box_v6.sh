#!/bin/bash
# Box session: netfilter state of the box's network namespace, and IPv4 vs IPv6 loopback
# for the headline layout (interleaved).
set -o pipefail
OUT=${1:-gpurun_out/v6}
mkdir -p "$OUT"
{
  for f in /proc/sys/net/netfilter/nf_conntrack_count /proc/sys/net/netfilter/nf_conntrack_max \
           /proc/net/ip_tables_names /proc/net/ip6_tables_names /proc/net/nf_conntrack; do
    echo "== $f"; head -c 2000 "$f" 2>&1 | head -5
  done
  echo "== modules"; grep -E "^(nf_|ip6?table|x_tables|nft|iptable|br_netfilter)" /proc/modules 2>&1 | cut -d' ' -f1-3
  echo "== uname"; uname -r
} > "$OUT/netfilter.txt" 2>&1
run() {  # name, extra args
  local name=$1; shift
  timeout -k 10 120 python bench.py --steps 15 --warmup 3 "$@" > "$OUT/$name.json" 2>> "$OUT/err.log"
}
for rep in 1 2; do
  run "v4_$rep" && run "v6_$rep" --host ::1 || exit 1
done
