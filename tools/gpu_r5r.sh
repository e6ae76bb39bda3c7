#!/bin/bash
# round 5: the consuming setup resets only interval words that are not at their reset values -- parity, bench
set -o pipefail
O=gpurun_out/r5r; mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_band_native.py tests/test_gpu_sharding.py tests/test_gpu_clean_tiles.py -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for c in bistro_1080p_full bistro_4k_full_n16 suntemple_1080p_q; do
  timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 5 > $O/bench_$c.json 2> $O/bench_$c.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/bench_$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'], d.get('sd_kernel_ms'))"
done
