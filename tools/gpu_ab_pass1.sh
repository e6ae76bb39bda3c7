#!/bin/bash
# pass-1 A/B: parity tests with the default (lean) kernel, then pass times and the driver's bench
# for the default and RSD_PASS1=generic, alternating.  usage: bash tools/gpu_ab_pass1.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-ab_pass1}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 &&
for k in 1 2; do
  timeout -k 10 120 python -u tools/pass_time.py > "$OUT/pass_time_lean_$k.json" 2>> "$OUT/err.log" &&
  RSD_PASS1=generic timeout -k 10 120 python -u tools/pass_time.py > "$OUT/pass_time_generic_$k.json" 2>> "$OUT/err.log" || exit 1
done &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 > "$OUT/bench20_lean.json" 2>> "$OUT/err.log" &&
RSD_PASS1=generic timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 > "$OUT/bench20_generic.json" 2>> "$OUT/err.log" &&
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --cpu-baseline-seconds 0 > "$OUT/bench200_lean.json" 2>> "$OUT/err.log" &&
RSD_PASS1=generic timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --cpu-baseline-seconds 0 > "$OUT/bench200_generic.json" 2>> "$OUT/err.log"
rc=$?
echo "exit $rc" > "$OUT/status"
exit $rc
