#!/bin/bash
# round 5: hybrid walk (longest-first rays on the row walk on a side stream, the rest on the quad walk) A/Bs
set -o pipefail
O=gpurun_out/r6j; mkdir -p $O
run() {  # config quadWpc rowWpc
  RSD_TRACE_WAVES_PER_CU=$2 RSD_TRACE_HYBRID_ROWWPC=$3 timeout -k 10 300 python tools/env_ab.py RSD_TRACE_HYBRID off on $1 --n 20 --reps 3 --clean-tiles > $O/hy_$1_$2_$3.json 2> $O/hy_$1_$2_$3.err || { tail -3 $O/hy_$1_$2_$3.err; exit 1; }
  tail -1 $O/hy_$1_$2_$3.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 quad $2 row $3', d['median_us'], d['same_bits'])"
}
run emerald_4k_q 16 4
run emerald_4k_q 12 4
run emerald_4k_q 8 8
run bistro_1080p_full 16 4
run bistro_1080p_full 12 4
run bistro_4k_full_n16 16 4
run bistro_4k_full_n16 8 4
bash tools/gpu_r6i.sh || exit 1
