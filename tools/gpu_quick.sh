#!/bin/bash
# Parity + A/B timing after a kernel change: GPU tests, bench at 1, 3 and 4 (default) frames in
# flight, per-pass diagnostics.  usage: bash tools/gpu_quick.sh <tag>
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-quick}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
for F in 1 3 4 6; do
  timeout -k 10 180 python -u bench.py --cpu-baseline-seconds 0 --steps 300 --warmup 10 --frames-in-flight $F > "$OUT/bench_f$F.json" 2> "$OUT/bench_f$F.err" || exit $?
done
rc=$?
echo "exit $rc" > "$OUT/status"
exit $rc
