#!/bin/bash
# round 5: hybrid walk default -- parity suites, then the configs[2] / [3] measurement
set -o pipefail
O=gpurun_out/r6l; mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests/test_gpu_hybrid.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py tests/test_gpu_band_native.py tests/test_gpu_clean_tiles.py tests/test_gpu_parity.py -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
rm -rf gpurun_out/r6m
bash tools/round5_measure.sh r6m bistro_1080p_full emerald_4k_q || exit 1
for c in bistro_1080p_full emerald_4k_q; do
  tail -1 gpurun_out/r6m/$c/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c', d['value'], d['ms_per_step'], d['sd_kernel_ms'], r['frac'], r['kernel'], r.get('traffic'))"
done
