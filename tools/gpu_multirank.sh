#!/bin/bash
# Rehearsal of bench.py's N > 1 paths on a one-GPU box: 2 ranks on the same GPU over gloo
# (RCCL needs one GPU per rank; the driver's 8-GPU run uses nccl).  usage: bash tools/gpu_multirank.sh <tag>
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-multirank}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export RSD_BENCH_BACKEND=gloo
for SH in frame band; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 40 --warmup 5 --cpu-baseline-seconds 0 --shard $SH \
    > "$OUT/bench_n2_$SH.json" 2> "$OUT/bench_n2_$SH.err" || exit $?
done
unset RSD_BENCH_BACKEND
timeout -k 10 180 python -u bench.py --cpu-baseline-seconds 0 --steps 200 --warmup 10 > "$OUT/bench_n1.json" 2> "$OUT/bench_n1.err"
