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
RSD_TRACE_PART=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 600 --timeout-method thread -k "sd_trace or full_frame or config1 or band" > "$OUT/pytest_part4.log" 2>&1 &&
run base &&
run part2 RSD_TRACE_PART=2 &&
run part4 RSD_TRACE_PART=4 &&
run part8 RSD_TRACE_PART=8 &&
run part16 RSD_TRACE_PART=16 &&
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d "$OUT/l2_base" -o run --output-format csv -- python3 tools/sd_time.py > "$OUT/l2_base.log" 2>&1 &&
RSD_TRACE_PART=4 timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d "$OUT/l2_part4" -o run --output-format csv -- python3 tools/sd_time.py > "$OUT/l2_part4.log" 2>&1
