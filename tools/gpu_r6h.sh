#!/bin/bash
# round 5: the quad walk tests the entry frontier itself (RSD_TRACE_ENTRY_DEFER) -- A/B and parity
set -o pipefail
O=gpurun_out/r6h; mkdir -p $O
for c in bistro_4k_full_n16 bistro_1080p_full emerald_4k_q; do
  timeout -k 10 240 python tools/env_ab.py RSD_TRACE_ENTRY_DEFER off on $c --n 20 --reps 5 --clean-tiles > $O/defer_$c.json 2> $O/defer_$c.err || { tail -5 $O/defer_$c.err; exit 1; }
  tail -1 $O/defer_$c.json
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py tests/test_gpu_entry.py tests/test_gpu_clean_tiles.py -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python bench.py --config bistro_4k_full_n16 --steps 20 --warmup 5 --cpu-baseline-seconds 0 --hit-order-record 0 > $O/bench_c4.json 2> $O/bench_c4.err || exit 1
python3 -c "import json; d=json.loads(open('$O/bench_c4.json').read().strip().splitlines()[-1]); print('c4', d['value'], d['ms_per_step'], d.get('sd_kernel_ms'))"
