#!/bin/bash
# Rehearsal of bench.py's N > 1 paths on a one-GPU box: ranks sharing the GPU over gloo (RCCL
# needs one GPU per rank; the driver's 8-GPU run uses nccl).  Every sharding mode at 2 ranks on
# the default config, and the 4K band (halo) split at 2 and 3 ranks.
# usage: bash tools/gpu_multirank.sh <tag>
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-multirank}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export RSD_BENCH_BACKEND=gloo
for SH in frame band gather; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 4 --cpu-baseline-seconds 0 --shard $SH \
    > "$OUT/bench_n2_$SH.json" 2> "$OUT/bench_n2_$SH.err" || exit $?
done
for N in 2 3; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port 29534 bench.py --gpus $N --steps 6 --warmup 2 --frames-in-flight 1 --cpu-baseline-seconds 0 \
    --config emerald_4k_q > "$OUT/bench_n${N}_4k_band.json" 2> "$OUT/bench_n${N}_4k_band.err" || exit $?
done
