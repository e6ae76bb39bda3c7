#!/bin/bash
# round 5: quad walk compiled for 5 waves per SIMD at K <= 8 (96 VGPRs): 16 vs 20 persistent waves per CU
set -o pipefail
O=gpurun_out/r5y; mkdir -p $O
for c in bistro_1080p_full emerald_4k_q; do
  timeout -k 10 240 python tools/env_ab.py RSD_TRACE_WAVES_PER_CU 16 20 $c --n 20 --reps 5 --clean-tiles > $O/wpc_$c.json 2> $O/wpc_$c.err || { tail -5 $O/wpc_$c.err; exit 1; }
  tail -1 $O/wpc_$c.json
done
