#!/bin/bash
# round 5: the quad walks' LDS stack sized to the tree (dynamic LDS): tree depths, waves-per-CU A/Bs, parity
set -o pipefail
O=gpurun_out/r5p; mkdir -p $O
timeout -k 10 300 python tools/tree_info.py suntemple_1080p_q bistro_1080p_full emerald_4k_q bistro_4k_full_n16 > $O/tree_info.txt 2>&1 || exit 1
cat $O/tree_info.txt
timeout -k 10 240 python tools/env_ab.py RSD_TRACE_WAVES_PER_CU 12 16 bistro_4k_full_n16 --n 20 --reps 5 > $O/wpc_c4.json 2> $O/wpc_c4.err || exit 1
tail -1 $O/wpc_c4.json
for c in emerald_4k_q bistro_1080p_full; do
  timeout -k 10 240 python tools/env_ab.py RSD_TRACE_WAVES_PER_CU 16 20 $c --n 20 --reps 5 > $O/wpc_$c.json 2> $O/wpc_$c.err || exit 1
  tail -1 $O/wpc_$c.json
done
timeout -k 10 200 python tools/env_ab.py RSD_TRACE_WAVES_PER_CU 8 16 suntemple_1080p_q --hit-order traversal --n 30 --reps 5 > $O/wpc_ordered_c1.json 2> $O/wpc_ordered.err || exit 1
tail -1 $O/wpc_ordered_c1.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_hit_order.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
tail -2 $O/pytest.log
