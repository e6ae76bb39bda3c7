#!/bin/bash
# round 5: quantised nodes for the canonical quad walk (RSD_TRACE_QNODES) -- A/B and parity
set -o pipefail
O=gpurun_out/r5x; mkdir -p $O
for c in bistro_4k_full_n16 emerald_4k_q bistro_1080p_full; do
  timeout -k 10 240 python tools/env_ab.py RSD_TRACE_QNODES off on $c --n 20 --reps 5 --clean-tiles > $O/qn_$c.json 2> $O/qn_$c.err || { tail -5 $O/qn_$c.err; exit 1; }
  tail -1 $O/qn_$c.json
done
RSD_TRACE_QNODES=on RSD_TRACE_WALK=quad timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py tests/test_gpu_entry.py -x -q --timeout 600 --timeout-method thread > $O/pytest_qn.log 2>&1 || { tail -30 $O/pytest_qn.log; exit 1; }
tail -2 $O/pytest_qn.log
