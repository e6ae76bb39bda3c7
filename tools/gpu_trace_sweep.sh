#!/bin/bash
# SD-trace launch-shape sweep (tools/trace_probe.py --quick under env knobs); one process each
set -o pipefail
OUT=gpurun_out/${1:-sweep}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python -u tools/trace_probe.py --quick > "$OUT/$name.json" 2> "$OUT/$name.err" || return $?
  echo "$name $(cat $OUT/$name.json)"
}
run base &&
run pool128_w8 RSD_TRACE_POOL=128 &&
run pool128_w12 RSD_TRACE_POOL=128 RSD_TRACE_WAVES_PER_CU=12 &&
run pool128_w16 RSD_TRACE_POOL=128 RSD_TRACE_WAVES_PER_CU=16 &&
run pool128_w20 RSD_TRACE_POOL=128 RSD_TRACE_WAVES_PER_CU=20 &&
run w12 RSD_TRACE_WAVES_PER_CU=12 &&
run fused RSD_TRACE_WALK=fused &&
run fused_pool128_w16 RSD_TRACE_WALK=fused RSD_TRACE_POOL=128 RSD_TRACE_WAVES_PER_CU=16
