# round-5 batch m2: the traversal-order walk with the longest-first queue (parity + A/B against LPT off)
mkdir -p gpurun_out/r5m2
timeout -k 10 300 python -u -m pytest tests/test_gpu_hit_order.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r5m2/tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/env_ab.py RSD_TRACE_LPT off -0.1 --n 20 --reps 4 --hit-order traversal > gpurun_out/r5m2/lpt_ordered_c1.json 2>&1
