#!/bin/bash
# tiled SD layout A/B (librsd_sdtiled.so) + the frames-in-flight walk sweep (quad vs row, F = 2/3/4/6)
set -o pipefail
OUT=gpurun_out/${1:-r3f}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/ao_digest.py > "$OUT/digest_std.json" 2>> "$OUT/err.log" &&
RSD_LIB_VARIANT=sdtiled timeout -k 10 120 python -u tools/ao_digest.py > "$OUT/digest_tiled.json" 2>> "$OUT/err.log" &&
timeout -k 10 120 python -u tools/ao_digest.py emerald_4k_q > "$OUT/digest4k_std.json" 2>> "$OUT/err.log" &&
RSD_LIB_VARIANT=sdtiled timeout -k 10 120 python -u tools/ao_digest.py emerald_4k_q > "$OUT/digest4k_tiled.json" 2>> "$OUT/err.log" &&
for k in 1 2; do
  timeout -k 10 120 python -u tools/pass_time.py > "$OUT/pt_std_$k.json" 2>> "$OUT/err.log" &&
  RSD_LIB_VARIANT=sdtiled timeout -k 10 120 python -u tools/pass_time.py > "$OUT/pt_tiled_$k.json" 2>> "$OUT/err.log" &&
  timeout -k 10 120 python -u tools/pass_time.py bistro_1080p_full --frames 60 > "$OUT/pt3_std_$k.json" 2>> "$OUT/err.log" &&
  RSD_LIB_VARIANT=sdtiled timeout -k 10 120 python -u tools/pass_time.py bistro_1080p_full --frames 60 > "$OUT/pt3_tiled_$k.json" 2>> "$OUT/err.log" || exit 1
done &&
for F in 2 3 4 6; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 --frames-in-flight $F > "$OUT/walk_quad_F$F.json" 2>> "$OUT/err.log" &&
  RSD_TRACE_WALK=fused timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 --frames-in-flight $F > "$OUT/walk_row_F$F.json" 2>> "$OUT/err.log" || exit 1
done
rc=$?
echo "exit $rc" > "$OUT/status"
exit $rc
