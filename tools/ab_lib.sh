#!/bin/bash
# Same-box A/B of two librsd builds (diagnostics): librsd_<base>.so (RSD_LIB_VARIANT) against librsd.so,
# alternating: per-pass times (tools/pass_time.py) and the bench line at --steps 20 / 200.
# usage: bash tools/ab_lib.sh <tag> <base-variant> [config] [reps]
set -o pipefail
O=gpurun_out/$1; B=$2; C=${3:-suntemple_1080p_q}; R=${4:-2}; mkdir -p $O
for rep in $(seq 1 $R); do
for v in $B new; do
  if [ $v = new ]; then E="RSD_LIB_VARIANT="; else E="RSD_LIB_VARIANT=$v"; fi
  env $E timeout -k 10 120 python -u tools/pass_time.py $C > $O/pass_${v}_$rep.json 2>>$O/err.log || exit 1
  env $E timeout -k 10 200 python -u bench.py --config $C --steps 20 --warmup 5 --cpu-baseline-seconds 0 > $O/s20_${v}_$rep.json 2>>$O/err.log || exit 1
  env $E timeout -k 10 200 python -u bench.py --config $C --cpu-baseline-seconds 0 > $O/s200_${v}_$rep.json 2>>$O/err.log || exit 1
done; done
