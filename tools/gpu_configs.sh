#!/bin/bash
# bench.py on every BASELINE GPU config (1 GPU), one and four frames in flight, no CPU baseline.
# usage: bash tools/gpu_configs.sh <tag>
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-configs}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for C in bistro_1080p_full emerald_4k_q bistro_4k_full_n16; do
  for F in 1 4; do
    timeout -k 10 240 python -u bench.py --config $C --cpu-baseline-seconds 0 --steps 60 --warmup 8 --frames-in-flight $F > "$OUT/${C}_f$F.json" 2> "$OUT/${C}_f$F.err" || exit $?
    echo "$C F=$F $(python -c "import json;d=json.load(open('$OUT/${C}_f$F.json'));print(d['ms_per_step'], d['ao_frames_per_s'], d['value'], d['sequential']['ms_per_frame'], d['sd_kernel_ms'])")" | tee -a "$OUT/summary.txt"
  done
done
