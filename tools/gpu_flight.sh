#!/bin/bash
# Frames-in-flight A/B on the GPU box: GPU parity (incl. the concurrent-slot test), then the
# default bench at F = 1..4 frames in flight.  usage: bash tools/gpu_flight.sh <tag>
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-flight}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
for F in 1 2 3 4; do
  timeout -k 10 180 python -u bench.py --cpu-baseline-seconds 0 --steps 200 --warmup 10 --frames-in-flight $F > "$OUT/bench_f$F.json" 2> "$OUT/bench_f$F.err" || exit $?
done
echo ok > "$OUT/status"
