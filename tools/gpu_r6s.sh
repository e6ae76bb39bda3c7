#!/bin/bash
# round 5: hybrid walk at configs[1] by default -- parity, then the default bench (+ PMC passes for its traffic)
set -o pipefail
O=gpurun_out/r6s; mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python tools/env_ab.py RSD_TRACE_HYBRID off on suntemple_1080p_q --n 30 --reps 5 --clean-tiles > $O/hy_c1.json 2> $O/hy_c1.err || exit 1
tail -1 $O/hy_c1.json
rm -rf gpurun_out/r6t
bash tools/round5_measure.sh r6t suntemple_1080p_q || exit 1
tail -1 gpurun_out/r6t/suntemple_1080p_q/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], d['sd_kernel_ms'], r['frac'], r['kernel'], r['traffic'], r.get('latency_frac'), d['latency']['walk'], d['hit_order_wavefront']['sd_kernel_ms'])"
