#!/bin/bash
# Throughput frame of one config with and without an env setting, alternating (diagnostics, same box).
# usage: bash tools/ab_bench_cfg.sh <tag> <config> <reps> "<env>"
set -o pipefail
O=gpurun_out/$1; C=$2; R=$3; E=$4; mkdir -p $O
export TMPDIR=/tmp
for rep in $(seq 1 $R); do
  for e in RSD_AB_NONE=1 "$E"; do
    echo "$C $e $(env $e timeout -k 10 200 python3 -u bench.py --config $C --cpu-baseline-seconds 0 2>>$O/err.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["throughput"]["ms_per_frame"], d["sd_kernel_ms"], d["ao_span_ms"])')" >> $O/bench_cfg.txt || exit 1
  done
done
