#!/bin/bash
# One GPU-box session: parity tests, diagnostic pass timings, bench, rocprof kernel stats.
# Every GPU step has its own time limit; steps are chained with && so the first failure ends it.
# usage (from the repo root, on the box): bash tools/gpu_check.sh <tag> [pytest-args...]
set -o pipefail
TAG=${1:-run}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "$@" > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 300 python -u tools/diag_sd.py > "$OUT/diag.log" 2>&1 &&
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --cpu-baseline-seconds 0 > "$OUT/bench_prof.log" 2>&1
rc=$?
echo "exit $rc" > "$OUT/status"
exit $rc
