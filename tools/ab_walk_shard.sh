#!/bin/bash
# Same-box A/B of the frames-in-flight schedule choices at configs[1] (diagnostics):
# default (row walk, HaloFrame at N = 1), quad walk (RSD_TRACE_WALK=quad), BandFrame (--shard frame).
set -o pipefail
O=gpurun_out/${1:-abws}; mkdir -p $O
for rep in 1 2; do
for v in row quad frame; do
  case $v in
    row) E=""; A="";; quad) E="RSD_TRACE_WALK=quad"; A="";; frame) E=""; A="--shard frame";;
  esac
  for st in 20 200; do
    env $E timeout -k 10 200 python -u bench.py --steps $st --warmup 5 --cpu-baseline-seconds 0 $A > $O/${v}_s${st}_$rep.json 2>$O/err_${v}.log || exit 1
  done
done; done
