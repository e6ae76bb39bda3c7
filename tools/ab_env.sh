#!/bin/bash
# Same-box A/B of environment settings (diagnostics): per-pass times (tools/pass_time.py) and the bench
# line at --steps 20 / 200 for each "NAME=VALUE[,NAME=VALUE]" variant ("-" = defaults), alternating.
# usage: bash tools/ab_env.sh <tag> <reps> <variant>...
set -o pipefail
O=gpurun_out/$1; R=$2; shift 2; mkdir -p $O
for rep in $(seq 1 $R); do
for v in "$@"; do
  if [ "$v" = "-" ]; then E=""; n=default; else E=$(echo "$v" | tr ',' ' '); n=$(echo "$v" | tr ',=' '__'); fi
  env $E timeout -k 10 120 python -u tools/pass_time.py > $O/pass_${n}_$rep.json 2>>$O/err.log || exit 1
  env $E timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 > $O/s20_${n}_$rep.json 2>>$O/err.log || exit 1
  env $E timeout -k 10 200 python -u bench.py --cpu-baseline-seconds 0 > $O/s200_${n}_$rep.json 2>>$O/err.log || exit 1
done; done
