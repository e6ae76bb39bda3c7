#!/bin/bash
# One BASELINE config measured as the driver runs the default one: the FETCH_SIZE and
# WRITE_SIZE rocprofv3 --pmc passes of a short bench (separate runs, MI355X_MICROARCH.md), the bench
# line with roofline.traffic from those passes and the CPU baseline, and the rocprofv3 kernel stats
# of the same bench command.  Each GPU step has its own time limit; the steps are chained with &&.
# usage: bash tools/config_measure.sh <tag> <config> [steps] [warmup]
set -u -o pipefail
TAG=$1
CFG=$2
STEPS=${3:-20}
WARM=${4:-5}
OUT=gpurun_out/$TAG/$CFG
mkdir -p "$OUT"
export TMPDIR=/tmp
SHORT="--config $CFG --steps 6 --warmup 2 --cpu-baseline-seconds 0 --hit-order-record 0"
pick() { find "$1" -name '*counter_collection.csv' -print -quit; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch" -o run --output-format csv -- \
    python3 bench.py $SHORT > "$OUT/pmc_fetch.log" 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write" -o run --output-format csv -- \
    python3 bench.py $SHORT > "$OUT/pmc_write.log" 2>&1 &&
cp "$(pick "$OUT/pmc_fetch")" "$OUT/pmc_fetch_size.csv" && cp "$(pick "$OUT/pmc_write")" "$OUT/pmc_write_size.csv" &&
timeout -k 10 600 python3 -u bench.py --config "$CFG" --steps "$STEPS" --warmup "$WARM" \
    --pmc-csv "$OUT/pmc_fetch_size.csv" "$OUT/pmc_write_size.csv" > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 bench.py --config "$CFG" --steps "$STEPS" --warmup "$WARM" --cpu-baseline-seconds 0 --hit-order-record 0 \
    > "$OUT/prof.log" 2>&1 &&
cp "$(find "$OUT/prof" -name '*kernel_stats.csv' -print -quit)" "$OUT/kernel_stats.csv" &&
cp "$(find "$OUT/prof" -name '*kernel_trace.csv' -print -quit)" "$OUT/kernel_trace.csv"
