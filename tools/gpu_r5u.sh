#!/bin/bash
# round 5: the N = 2 / 4 / 8 band-split model (tools/scaling_model.py) with clean tiles and the native band frame's host issue
set -o pipefail
O=gpurun_out/r5u; mkdir -p $O
for c in suntemple_1080p_q emerald_4k_q bistro_4k_full_n16; do
  timeout -k 10 700 python -u tools/scaling_model.py $c --reps 11 > $O/scaling_$c.json 2> $O/scaling_$c.err || { tail -5 $O/scaling_$c.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/scaling_$c.json').read().strip().splitlines()[-1])
print('$c', d['sd_split'], d['one_gpu'])
for w,v in d['worlds'].items(): print(' ', w, v['max_rank_gpu_us'], v['max_rank_bytes'], v['predicted_latency_us'], v['predicted_speedup_latency'], v['host_issue_us_per_frame'], v['host_issue_native_us_per_frame'])"
done
