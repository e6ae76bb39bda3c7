#!/bin/bash
# round 5: clean tiles (rsd_sd_params.d_tile_state) -- parity tests, then bench on / off at the full-res configs
set -o pipefail
O=gpurun_out/r5q; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_clean_tiles.py -x -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for c in bistro_1080p_full bistro_4k_full_n16; do
  for ct in on off; do
    timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 5 --clean-tiles $ct > $O/bench_${c}_$ct.json 2> $O/bench_${c}_$ct.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/bench_${c}_$ct.json').read().strip().splitlines()[-1]); print('$c $ct', d['value'], d['ms_per_step'], d.get('sd_kernel_ms'), d['roofline']['achieved'])"
  done
done
