#!/bin/bash
# round-2 check: new config tests, default bench line, config-5 camera-path bench
set -o pipefail
OUT=gpurun_out/${1:-r2a}
mkdir -p "$OUT"
export TMPDIR=/tmp
python -c "import bench, json; print(json.dumps(bench.host_cpus()))" > "$OUT/host.json" 2>&1
nproc >> "$OUT/host.json"
timeout -k 10 1500 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 1300 --timeout-method thread --durations=0 > "$OUT/pytest_configs.log" 2>&1 &&
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 600 python -u bench.py --config bistro_4k_full_n16 --steps 120 --warmup 8 --cpu-baseline-seconds 20 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err"
rc=$?
echo "exit $rc" > "$OUT/status"
exit $rc
