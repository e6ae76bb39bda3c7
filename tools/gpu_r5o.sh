#!/bin/bash
# round 5: the quad walks' node fetch as two 16-B loads + quad transpose (RSD_TRACE_NODE_X4) A/B
set -o pipefail
O=gpurun_out/r5o; mkdir -p $O
for c in bistro_4k_full_n16 emerald_4k_q bistro_1080p_full; do
  timeout -k 10 240 python tools/env_ab.py RSD_TRACE_NODE_X4 off on $c --n 20 --reps 5 > $O/x4_$c.json 2> $O/x4_$c.err || exit 1
  tail -1 $O/x4_$c.json
done
timeout -k 10 200 python tools/env_ab.py RSD_TRACE_NODE_X4 off on suntemple_1080p_q --hit-order traversal --n 30 --reps 5 > $O/x4_ordered_c1.json 2> $O/x4_ordered.err || exit 1
tail -1 $O/x4_ordered_c1.json
