#!/bin/bash
# configs[1]: the fused row walk vs the hybrid launch (quad walk forced, hybrid on by default)
set -o pipefail
O=gpurun_out/r6r; mkdir -p $O
for qr in "8 4" "4 8" "2 8" "6 6"; do
  set -- $qr
  RSD_TRACE_WAVES_PER_CU=$1 RSD_TRACE_HYBRID_ROWWPC=$2 timeout -k 10 200 python tools/env_ab.py RSD_TRACE_WALK fused quad suntemple_1080p_q --n 30 --reps 5 --clean-tiles > $O/c1_$1_$2.json 2> $O/c1_$1_$2.err || exit 1
  tail -1 $O/c1_$1_$2.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c1 quad $1 row $2', d['median_us'], d['same_bits'])"
done
