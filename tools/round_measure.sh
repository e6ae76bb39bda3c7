#!/bin/bash
# Round-end measurement on the GPU box: parity tests, the default bench line (with the CPU
# baseline), rocprofv3 kernel stats of the same bench, and the PMC passes bench.py reads its
# roofline traffic (FETCH_SIZE, WRITE_SIZE) and pass-1 VALU rate (SQ_INSTS_VALU) from.  Each GPU step has its own limit and
# the steps are chained with &&.  usage: bash tools/round_measure.sh <tag>
set -o pipefail
TAG=${1:-measure}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --cpu-baseline-seconds 0 > "$OUT/bench_prof.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline-seconds 0 > "$OUT/pmc_fetch.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline-seconds 0 > "$OUT/pmc_write.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace -d "$OUT/pmc_valu" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline-seconds 0 > "$OUT/pmc_valu.log" 2>&1 &&
timeout -k 10 300 python -u bench.py --camera-path orbit120 --config bistro_4k_full_n16 --steps 120 --warmup 8 --cpu-baseline-seconds 0 > "$OUT/bench_config5.json" 2> "$OUT/bench_config5.err"
rc=$?
echo "exit $rc" > "$OUT/status"
exit $rc
