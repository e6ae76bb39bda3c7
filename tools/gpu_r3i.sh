#!/bin/bash
# pass-1 direction groups (RSD_PASS1_GROUP = 1 / 2 / 4): isolated pass times, then the driver's bench
# alternating, then 200-frame benches
set -o pipefail
OUT=gpurun_out/${1:-r3i}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "pass1 or frame or busy" --timeout 300 --timeout-method thread > "$OUT/pytest_g1.log" 2>&1 &&
RSD_PASS1_GROUP=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "pass1 or frame or busy" --timeout 300 --timeout-method thread > "$OUT/pytest_g2.log" 2>&1 &&
RSD_PASS1_GROUP=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "pass1 or frame or busy" --timeout 300 --timeout-method thread > "$OUT/pytest_g4.log" 2>&1 &&
for g in 1 2 4; do
  RSD_PASS1_GROUP=$g timeout -k 10 120 python -u tools/pass_time.py > "$OUT/pt_g$g.json" 2>> "$OUT/err.log" || exit 1
done &&
for k in 1 2 3; do
  for g in 1 2 4; do
    RSD_PASS1_GROUP=$g timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 > "$OUT/b20_g${g}_$k.json" 2>> "$OUT/err.log" || exit 1
  done
done &&
for g in 1 2 4; do
  RSD_PASS1_GROUP=$g timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --cpu-baseline-seconds 0 > "$OUT/b200_g$g.json" 2>> "$OUT/err.log" || exit 1
done
rc=$?
echo "exit $rc" > "$OUT/status"
exit $rc
