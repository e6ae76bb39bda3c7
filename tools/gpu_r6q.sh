#!/bin/bash
# round 5: the band-split model again for configs[3] / [1] after the hybrid walk
set -o pipefail
O=gpurun_out/r6q; mkdir -p $O
for c in emerald_4k_q suntemple_1080p_q; do
  timeout -k 10 700 python -u tools/scaling_model.py $c --reps 11 > $O/scaling_$c.json 2> $O/scaling_$c.err || { tail -5 $O/scaling_$c.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/scaling_$c.json').read().strip().splitlines()[-1])
print('$c', d['sd_split'], d['one_gpu'])
for w,v in d['worlds'].items(): print(' ', w, v['max_rank_gpu_us'], v['max_rank_bytes'], v['predicted_latency_us'], v['predicted_speedup_latency'], v['host_issue_us_per_frame'], v['host_issue_native_us_per_frame'])"
done
