#!/bin/bash
# round 5: the fused hybrid kernel (row-walk blocks + quad-walk blocks in one launch) -- sweep, parity
set -o pipefail
O=gpurun_out/r6n; mkdir -p $O
run() {  # config quadWpc rowWpc
  RSD_TRACE_WAVES_PER_CU=$2 RSD_TRACE_HYBRID_ROWWPC=$3 timeout -k 10 300 python tools/env_ab.py RSD_TRACE_HYBRID off on $1 --n 20 --reps 3 --clean-tiles > $O/hy_$1_$2_$3.json 2> $O/hy_$1_$2_$3.err || { tail -3 $O/hy_$1_$2_$3.err; exit 1; }
  tail -1 $O/hy_$1_$2_$3.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 quad $2 row $3', d['median_us'], d['same_bits'])"
}
for qr in "16 4" "8 4" "10 2" "6 6" "12 4" "8 8"; do run emerald_4k_q $qr; done
for qr in "16 4" "8 4" "6 6" "12 4" "8 8"; do run bistro_1080p_full $qr; done
timeout -k 10 1200 python -u -m pytest tests/test_gpu_hybrid.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py tests/test_gpu_band_native.py tests/test_gpu_parity.py -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
