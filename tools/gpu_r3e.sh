#!/bin/bash
# pass-2 grid A/B: persistent (default), persistent without the waves-per-EU bound (librsd_p2nowpe.so),
# one workgroup per tile (RSD_P2_GRID=tiles); then parity tests and the driver's bench
set -o pipefail
OUT=gpurun_out/${1:-r3e}
mkdir -p "$OUT"
export TMPDIR=/tmp
for k in 1 2; do
  timeout -k 10 120 python -u tools/pass2_probe.py > "$OUT/p2_persist_$k.json" 2>> "$OUT/err.log" &&
  RSD_LIB_VARIANT=p2nowpe timeout -k 10 120 python -u tools/pass2_probe.py > "$OUT/p2_nowpe_$k.json" 2>> "$OUT/err.log" &&
  RSD_P2_GRID=tiles timeout -k 10 120 python -u tools/pass2_probe.py > "$OUT/p2_tiles_$k.json" 2>> "$OUT/err.log" || exit 1
done &&
timeout -k 10 120 python -u tools/pass_time.py > "$OUT/pass_time.json" 2>> "$OUT/err.log" &&
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_graph.py -m gpu -x -q --timeout 900 --timeout-method thread > "$OUT/pytest.log" 2>&1 &&
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 > "$OUT/bench20_persist_$k.json" 2>> "$OUT/err.log" &&
  RSD_P2_GRID=tiles timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 > "$OUT/bench20_tiles_$k.json" 2>> "$OUT/err.log" || exit 1
done
rc=$?
echo "exit $rc" > "$OUT/status"
exit $rc
