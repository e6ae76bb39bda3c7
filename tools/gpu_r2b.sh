#!/bin/bash
# round-2: hit-order + Use16Bit parity, full GPU suite, hit-order study
set -o pipefail
OUT=gpurun_out/${1:-r2b}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_hit_order.py -x -v --timeout 300 --timeout-method thread --durations=10 > "$OUT/pytest_hit_order.log" 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 1300 --timeout-method thread --durations=10 > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 300 python -u tools/hit_order_study.py > "$OUT/hit_order_study.json" 2> "$OUT/hit_order_study.err"
rc=$?
echo "exit $rc" > "$OUT/status"
exit $rc
