#!/bin/bash
# Round-3 starting point on one MI355X: the driver's bench command twice, a kernel trace of the
# same command (timeline of the 4-frames-in-flight region), and the pass-1 PMC passes.
set -o pipefail
OUT=gpurun_out/${1:-r3a}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench20_1.json" 2> "$OUT/bench20_1.err" &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline-seconds 0 > "$OUT/bench20_2.json" 2> "$OUT/bench20_2.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 > "$OUT/bench_prof.log" 2>&1 &&
bash tools/pmc_pass1.sh "${1:-r3a}/pmc_pass1" pass1
rc=$?
echo "exit $rc" > "$OUT/status"
exit $rc
