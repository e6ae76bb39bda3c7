#!/bin/bash
# round 5: the wavefront traversal-order stream (RSD_HIT_ORDER_WAVEFRONT) -- parity and timing
set -o pipefail
O=gpurun_out/r6c; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_hit_order.py -x -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for h in wavefront traversal canonical; do
  timeout -k 10 200 python tools/env_ab.py RSD_AB_NOOP a b suntemple_1080p_q --hit-order $h --n 30 --reps 5 --clean-tiles > $O/t_$h.json 2> $O/t_$h.err || { tail -5 $O/t_$h.err; exit 1; }
  tail -1 $O/t_$h.json
done
timeout -k 10 200 python tools/env_ab.py RSD_AB_NOOP a b emerald_4k_q --hit-order wavefront --n 10 --reps 3 --clean-tiles > $O/t_wave_c3.json 2> $O/t_wave_c3.err || { tail -5 $O/t_wave_c3.err; exit 1; }
tail -1 $O/t_wave_c3.json
