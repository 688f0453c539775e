#!/bin/bash
# Box session: the driver's own N>1 command line, with no extra flags, at N = 2, 4 and 8
# inside the 1-GPU box's 16-CPU slice. bench.py must size cores per rank by itself here.
set -o pipefail
OUT=${1:-gpurun_out/driver_rehearsal}
mkdir -p "$OUT"
for n in 2 4 8; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 8 --warmup 2 \
    > "$OUT/n$n.json" 2> "$OUT/err_n$n.log" || exit $?
done
