#!/bin/bash
# A/B of SD-trace variants on configs[1]: each argument is a comma-separated env list
# ("-" = defaults), e.g.  - RSD_TRACE_COOP=1 RSD_TRACE_WALK=split,RSD_TRACE_POOL=128
set -o pipefail
OUT=gpurun_out/${AB_OUT:-env_ab}
mkdir -p "$OUT"
i=0
for spec in "$@"; do
  i=$((i+1))
  envs=()
  [ "$spec" != "-" ] && IFS=',' read -ra envs <<< "$spec"
  env "${envs[@]}" timeout -k 10 120 python3 -u tools/trace_probe.py ${PROBE_ARGS:---quick} > "$OUT/probe_$i.json" 2> "$OUT/probe_$i.err" || exit $?
  echo "$spec $(cat $OUT/probe_$i.json)"
done
