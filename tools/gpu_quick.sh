#!/bin/bash
# Parity + A/B timing after a kernel change: GPU tests, bench at 1 and 3 frames in flight,
# per-pass diagnostics.  usage: bash tools/gpu_quick.sh <tag>
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-quick}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 180 python -u bench.py --cpu-baseline-seconds 0 --steps 200 --warmup 10 --frames-in-flight 1 > "$OUT/bench_f1.json" 2> "$OUT/bench_f1.err" &&
timeout -k 10 180 python -u bench.py --cpu-baseline-seconds 0 --steps 200 --warmup 10 --frames-in-flight 3 > "$OUT/bench_f3.json" 2> "$OUT/bench_f3.err" &&
timeout -k 10 300 python -u tools/diag_sd.py > "$OUT/diag.log" 2>&1
rc=$?
echo "exit $rc" > "$OUT/status"
exit $rc
