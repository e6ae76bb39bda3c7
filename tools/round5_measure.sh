#!/bin/bash
# Round-5 measurement of one BASELINE config (tools/config_measure.sh) into gpurun_out/<tag>/<config>/, plus, for
# the default config, the pass-1 VALU PMC pass bench.py's pass1_roofline reads.  usage: bash tools/round5_measure.sh <tag> <config>...
set -u -o pipefail
TAG=$1
shift
export TMPDIR=/tmp
for CFG in "$@"; do
  bash tools/config_measure.sh "$TAG" "$CFG" 20 5 || exit 1
  if [ "$CFG" = suntemple_1080p_q ]; then
    timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace -d "gpurun_out/$TAG/pmc_valu" -o run --output-format csv -- \
      python3 bench.py --steps 10 --warmup 2 --cpu-baseline-seconds 0 --hit-order-record 0 > "gpurun_out/$TAG/pmc_valu.log" 2>&1 &&
    cp "$(find gpurun_out/$TAG/pmc_valu -name '*counter_collection.csv' -print -quit)" "gpurun_out/$TAG/pmc_sq_valu.csv" || exit 1
  fi
done
echo ok
