#!/bin/bash
set -o pipefail
O=gpurun_out/r6a
for c in bistro_4k_full_n16 emerald_4k_q bistro_1080p_full; do bash tools/lib_ab.sh $O base $c || exit 1; done
bash tools/lib_ab.sh $O base suntemple_1080p_q --hit-order traversal || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_hit_order.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
