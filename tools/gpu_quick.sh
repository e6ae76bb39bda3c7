#!/bin/bash
# quick GPU iteration: selected GPU tests, per-pass times, the driver's bench command
# usage: bash tools/gpu_quick.sh <tag> "<pytest -k expr or test paths>"
set -o pipefail
OUT=gpurun_out/${1:-quick}
mkdir -p "$OUT"
export TMPDIR=/tmp
TESTS=${2:-tests/test_gpu_parity.py}
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 &&
timeout -k 10 120 python -u tools/pass_time.py > "$OUT/pass_time.json" 2> "$OUT/pass_time.err" &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline-seconds 0 > "$OUT/bench20.json" 2> "$OUT/bench20.err" &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 20 --cpu-baseline-seconds 0 > "$OUT/bench200.json" 2> "$OUT/bench200.err"
rc=$?
echo "exit $rc" > "$OUT/status"
exit $rc
