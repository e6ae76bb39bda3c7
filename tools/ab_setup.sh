#!/bin/bash
# Same-box A/B of the SD trace between librsd_<base>.so (RSD_LIB_VARIANT) and librsd.so (diagnostics):
# tools/sd_time.py alternating, then a kernel trace per build split into setup / gap / walk
# (tools/trace_gaps.py).  usage: bash tools/ab_setup.sh <tag> <base-variant> [config] [reps]
set -o pipefail
O=gpurun_out/$1; B=$2; C=${3:-suntemple_1080p_q}; R=${4:-3}; mkdir -p $O
export TMPDIR=/tmp
for rep in $(seq 1 $R); do
for v in $B new; do
  if [ $v = new ]; then E="RSD_LIB_VARIANT="; else E="RSD_LIB_VARIANT=$v"; fi
  echo "$v $(env $E timeout -k 10 120 python3 -u tools/sd_time.py $C 2>>$O/err.log)" >> $O/sd_time.txt || exit 1
done; done
for v in $B new; do
  if [ $v = new ]; then export RSD_LIB_VARIANT=; else export RSD_LIB_VARIANT=$v; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$v -o run -- python3 -u tools/sd_time.py $C > $O/kt_$v.log 2>&1 || exit 1
  echo "$v $(python3 tools/trace_gaps.py $O/kt_$v)" >> $O/gaps.txt || exit 1
done
