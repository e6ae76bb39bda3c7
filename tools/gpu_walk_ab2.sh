#!/bin/bash
# A/B of SD-trace walks on configs[1] (median timings; RSD_TRACE_WALK values given as args)
set -o pipefail
OUT=gpurun_out/${AB_OUT:-walk_ab2}
mkdir -p "$OUT"
for w in "$@"; do
  RSD_TRACE_WALK=$w timeout -k 10 120 python3 -u tools/trace_probe.py --quick > "$OUT/probe_$w.json" 2> "$OUT/probe_$w.err" || exit $?
  echo "$w $(cat $OUT/probe_$w.json)"
done
