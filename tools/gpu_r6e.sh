#!/bin/bash
# round 5: clean texels (a 64-texel DEFAULT mask per tile) -- parity, then the full-res benches
set -o pipefail
O=gpurun_out/r6e; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_clean_tiles.py tests/test_gpu_parity.py tests/test_gpu_band_native.py -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for c in bistro_4k_full_n16 bistro_1080p_full; do
  timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 5 --cpu-baseline-seconds 0 --hit-order-record 0 > $O/bench_$c.json 2> $O/bench_$c.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/bench_$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'], d.get('sd_kernel_ms'))"
  timeout -k 10 240 python tools/env_ab.py RSD_AB_NOOP a b $c --n 20 --reps 3 --clean-tiles > $O/static_$c.json 2> $O/static_$c.err || exit 1
  tail -1 $O/static_$c.json
done
