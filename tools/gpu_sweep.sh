#!/bin/bash
# Frames-in-flight x SD-trace persistent waves per CU sweep (bench.py defaults otherwise, no CPU
# baseline).  usage: bash tools/gpu_sweep.sh <tag> "<F values>" "<W values>"
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-sweep}
FS=${2:-"3 4 6"}
WS=${3:-"4 8 16"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for F in $FS; do
  for W in $WS; do
    RSD_TRACE_WAVES_PER_CU=$W timeout -k 10 120 python -u bench.py --cpu-baseline-seconds 0 --steps 400 --warmup 20 --frames-in-flight $F > "$OUT/f${F}_w${W}.json" 2> "$OUT/f${F}_w${W}.err" || exit $?
    echo "F=$F W=$W $(python -c "import json;d=json.load(open('$OUT/f${F}_w${W}.json'));print(d['ms_per_step'])")" | tee -a "$OUT/summary.txt"
  done
done
