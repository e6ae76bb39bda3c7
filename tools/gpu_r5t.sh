#!/bin/bash
# round 5: tiles per SD-setup wave (RSD_SETUP_TILES) A/B, clean tiles on (the bench's maps); parity
set -o pipefail
O=gpurun_out/r5t; mkdir -p $O
for c in bistro_4k_full_n16 bistro_1080p_full emerald_4k_q suntemple_1080p_q; do
  for v in 4 8; do
    timeout -k 10 240 python tools/env_ab.py RSD_SETUP_TILES 1 $v $c --n 20 --reps 5 --clean-tiles > $O/st_${c}_$v.json 2> $O/st_${c}_$v.err || exit 1
    tail -1 $O/st_${c}_$v.json
  done
done
RSD_SETUP_TILES=8 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_clean_tiles.py tests/test_gpu_band_native.py -x -q --timeout 600 --timeout-method thread > $O/pytest_t8.log 2>&1 || { tail -30 $O/pytest_t8.log; exit 1; }
tail -2 $O/pytest_t8.log
for v in 1 8; do
  RSD_SETUP_TILES=$v timeout -k 10 400 python bench.py --config bistro_4k_full_n16 --steps 20 --warmup 5 --cpu-baseline-seconds 0 > $O/bench_c4_t$v.json 2> $O/bench_c4_t$v.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/bench_c4_t$v.json').read().strip().splitlines()[-1]); print('c4 T=$v', d['value'], d['ms_per_step'], d.get('sd_kernel_ms'))"
done
