#!/bin/bash
# Frames in flight x HIP hardware queues per process (GPU_MAX_HW_QUEUES; HIP default 4).
# usage: bash tools/gpu_queues.sh <tag>
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-queues}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for Q in 4 8; do
  for F in 4 6 8; do
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 120 python -u bench.py --cpu-baseline-seconds 0 --steps 400 --warmup 20 --frames-in-flight $F > "$OUT/q${Q}_f$F.json" 2> "$OUT/q${Q}_f$F.err" || exit $?
    echo "Q=$Q F=$F $(python -c "import json;d=json.load(open('$OUT/q${Q}_f$F.json'));print(d['ms_per_step'])")" | tee -a "$OUT/summary.txt"
  done
done
