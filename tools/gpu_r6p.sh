#!/bin/bash
# round 5: the hybrid walk with frames in flight too (RSD_TRACE_HYBRID=all) vs latency-only (default)
set -o pipefail
O=gpurun_out/r6p; mkdir -p $O
for c in bistro_1080p_full emerald_4k_q; do
  for h in default all default all; do
    if [ $h = all ]; then export RSD_TRACE_HYBRID=all; else unset RSD_TRACE_HYBRID; fi
    timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 5 --cpu-baseline-seconds 0 --hit-order-record 0 > $O/bench_${c}_$h.json 2> $O/bench_${c}_$h.err || exit 1
    unset RSD_TRACE_HYBRID
    python3 -c "import json; d=json.loads(open('$O/bench_${c}_$h.json').read().strip().splitlines()[-1]); print('$c $h', d['value'], d['ms_per_step'], d['throughput']['walk'])"
  done
done
