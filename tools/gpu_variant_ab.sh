#!/bin/bash
# A/B of librsd build variants (librsd_<v>.so beside librsd.so, loaded via RSD_LIB_VARIANT):
# bench at 1 and 4 frames in flight.  usage: bash tools/gpu_variant_ab.sh <tag> "<variants>"
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-variant}
VS=${2:-"base"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for V in $VS; do
  for F in 1 4; do
    if [ "$V" = base ]; then unset RSD_LIB_VARIANT; else export RSD_LIB_VARIANT=$V; fi
    timeout -k 10 120 python -u bench.py --cpu-baseline-seconds 0 --steps 400 --warmup 20 --frames-in-flight $F > "$OUT/${V}_f$F.json" 2> "$OUT/${V}_f$F.err" || exit $?
    echo "V=$V F=$F $(python -c "import json;d=json.load(open('$OUT/${V}_f$F.json'));print(d['ms_per_step'], d['sequential']['ms_per_frame'])")" | tee -a "$OUT/summary.txt"
  done
done
