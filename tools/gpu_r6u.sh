#!/bin/bash
set -o pipefail
O=gpurun_out/r6u2; mkdir -p $O
timeout -k 10 700 python -u tools/scaling_model.py suntemple_1080p_q --reps 11 > $O/scaling_suntemple_1080p_q.json 2> $O/scaling.err || { tail -5 $O/scaling.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/scaling_suntemple_1080p_q.json').read().strip().splitlines()[-1])
print(d['sd_split'], d['one_gpu'])
for w,v in d['worlds'].items(): print(' ', w, v['max_rank_gpu_us'], v['max_rank_bytes'], v['predicted_latency_us'], v['predicted_speedup_latency'], v['host_issue_us_per_frame'], v['host_issue_native_us_per_frame'])"
