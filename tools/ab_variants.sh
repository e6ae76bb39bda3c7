#!/bin/bash
# Same-box A/B of several librsd builds / env settings (diagnostics), alternating per repetition:
# per-pass times (tools/pass_time.py) and the driver-style bench line (--steps 20).
# A variant is "new" (librsd.so), a build name (librsd_<name>.so via RSD_LIB_VARIANT), or
# "<name>+KEY=VAL[+KEY=VAL...]" (that build with extra environment settings).
# usage: bash tools/ab_variants.sh <tag> <reps> <variant>...
set -o pipefail
O=gpurun_out/$1; R=$2; shift 2; mkdir -p $O
export TMPDIR=/tmp
for rep in $(seq 1 $R); do
for v in "$@"; do
  lib=${v%%+*}; extra=""; [ "$lib" != "$v" ] && extra=$(echo "${v#*+}" | tr '+' ' ')
  if [ "$lib" = new ]; then E="RSD_LIB_VARIANT="; else E="RSD_LIB_VARIANT=$lib"; fi
  tag=$(echo "$v" | tr '+=' '__')
  env $E $extra timeout -k 10 120 python -u tools/pass_time.py > $O/pass_${tag}_$rep.json 2>>$O/err.log || exit 1
  env $E $extra timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 > $O/s20_${tag}_$rep.json 2>>$O/err.log || exit 1
done; done
python3 tools/ab_summary.py $O > $O/summary.txt 2>&1 || true
