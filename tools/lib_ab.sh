#!/bin/bash
# Two librsd builds on one box: RSD_LIB_VARIANT=<base> (librsd_<base>.so) against librsd.so, alternating processes,
# each timing one config's SD trace with tools/env_ab.py (a no-op variable: both of its settings are the same build)
# usage: bash tools/lib_ab.sh <outdir> <base> <config> [env_ab args...]
set -o pipefail
O=$1; B=$2; C=$3; shift 3
mkdir -p $O
for rep in 1 2 3; do
  for v in $B new; do
    if [ $v = new ]; then unset RSD_LIB_VARIANT; else export RSD_LIB_VARIANT=$v; fi
    timeout -k 10 240 python tools/env_ab.py RSD_AB_NOOP a b $C --n 20 --reps 3 --clean-tiles "$@" > $O/${C}_${v}_$rep.json 2> $O/${C}_${v}_$rep.err || { unset RSD_LIB_VARIANT; tail -3 $O/${C}_${v}_$rep.err; exit 1; }
    unset RSD_LIB_VARIANT
    python3 -c "import json; d=json.loads(open('$O/${C}_${v}_$rep.json').read().strip().splitlines()[-1]); print('$C $v $rep', d['median_us'])"
  done
done
