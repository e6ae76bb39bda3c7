#!/bin/bash
# pass-1 residency cap sweep (RSD_PASS1_WG_PER_CU) with the row walk in the throughput region
set -o pipefail
OUT=gpurun_out/${1:-r3g}
mkdir -p "$OUT"
export TMPDIR=/tmp
for k in 1 2; do
  for cap in 0 7 6 5 4; do
    RSD_PASS1_WG_PER_CU=$cap timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 > "$OUT/cap${cap}_$k.json" 2>> "$OUT/err.log" || exit 1
  done
done &&
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --cpu-baseline-seconds 0 > "$OUT/bench200_row.json" 2>> "$OUT/err.log" &&
RSD_TRACE_WALK=quad timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --cpu-baseline-seconds 0 > "$OUT/bench200_quad.json" 2>> "$OUT/err.log" &&
RSD_PASS1_WG_PER_CU=6 timeout -k 10 120 python -u tools/pass_time.py > "$OUT/pt_cap6.json" 2>> "$OUT/err.log" &&
timeout -k 10 120 python -u tools/pass_time.py > "$OUT/pt_cap0.json" 2>> "$OUT/err.log"
rc=$?
echo "exit $rc" > "$OUT/status"
exit $rc
