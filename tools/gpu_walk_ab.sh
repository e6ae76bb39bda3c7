#!/bin/bash
# SD-trace walk A/B with frames in flight (RSD_TRACE_WALK = default row split / quad / fused).
# usage: bash tools/gpu_walk_ab.sh <tag>
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-walk}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for WALK in split quad; do
  for F in 1 3 4; do
    RSD_TRACE_WALK=$WALK timeout -k 10 120 python -u bench.py --cpu-baseline-seconds 0 --steps 300 --warmup 10 --frames-in-flight $F > "$OUT/${WALK}_f$F.json" 2> "$OUT/${WALK}_f$F.err" || exit $?
    echo "walk=$WALK F=$F $(python -c "import json;d=json.load(open('$OUT/${WALK}_f$F.json'));print(d['ms_per_step'], d['sd_kernel_ms'])")" | tee -a "$OUT/summary.txt"
  done
done
