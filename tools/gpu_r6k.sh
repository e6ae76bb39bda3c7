#!/bin/bash
# round 5: hybrid walk occupancy sweep (quad waves / row waves per CU), configs[1] with the quad walk forced, benches
set -o pipefail
O=gpurun_out/r6k; mkdir -p $O
run() {  # config quadWpc rowWpc [walk]
  W=${4:+--walk $4}
  RSD_TRACE_WAVES_PER_CU=$2 RSD_TRACE_HYBRID_ROWWPC=$3 timeout -k 10 300 python tools/env_ab.py RSD_TRACE_HYBRID off on $1 --n 20 --reps 3 --clean-tiles $W > $O/hy_$1_$2_$3$4.json 2> $O/hy_$1_$2_$3$4.err || { tail -3 $O/hy_$1_$2_$3$4.err; exit 1; }
  tail -1 $O/hy_$1_$2_$3$4.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 quad $2 row $3 $4', d['median_us'], d['same_bits'])"
}
for qr in "8 8" "8 12" "12 8" "4 8" "4 12" "8 4"; do run emerald_4k_q $qr; done
for qr in "8 8" "12 8" "8 4" "12 4" "16 8"; do run bistro_1080p_full $qr; done
for qr in "8 8" "4 8" "12 4"; do run suntemple_1080p_q $qr quad; done
for h in off on; do
  RSD_TRACE_HYBRID=$h RSD_TRACE_WAVES_PER_CU=8 RSD_TRACE_HYBRID_ROWWPC=8 timeout -k 10 400 python bench.py --config emerald_4k_q --steps 20 --warmup 5 --cpu-baseline-seconds 0 --hit-order-record 0 > $O/bench_c3_$h.json 2> $O/bench_c3_$h.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/bench_c3_$h.json').read().strip().splitlines()[-1]); print('c3 hybrid $h', d['value'], d['ms_per_step'], d.get('sd_kernel_ms'))"
done
