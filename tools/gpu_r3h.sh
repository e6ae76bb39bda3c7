#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r3h}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/flight_probe.py 20 12 0.05 > "$OUT/flight_20_idle50.json" 2>> "$OUT/err.log" &&
timeout -k 10 200 python -u tools/flight_probe.py 20 12 0 > "$OUT/flight_20_idle0.json" 2>> "$OUT/err.log" &&
timeout -k 10 200 python -u tools/flight_probe.py 200 4 0.05 > "$OUT/flight_200.json" 2>> "$OUT/err.log" &&
for k in 1 2 3 4; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 > "$OUT/bench20_$k.json" 2>> "$OUT/err.log" || exit 1
done
rc=$?
echo "exit $rc" > "$OUT/status"
exit $rc
