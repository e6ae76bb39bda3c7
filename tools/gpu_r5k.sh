# round-5 batch k: the quad walk with quad-distributed keys (K = 16: 115 VGPRs, K = 8: 96): parity, then waves per CU
mkdir -p gpurun_out/r5k
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_configs.py tests/test_gpu_entry.py tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r5k/tests.log 2>&1 || exit 1
timeout -k 10 300 python tools/env_ab.py RSD_TRACE_WAVES_PER_CU 12 16 bistro_4k_full_n16 --n 5 --reps 3 > gpurun_out/r5k/wpc_c4_16.json 2>&1 || exit 1
timeout -k 10 200 python tools/env_ab.py RSD_TRACE_WAVES_PER_CU 8 16 bistro_1080p_full --n 10 --reps 3 > gpurun_out/r5k/wpc_c2_16.json 2>&1 || exit 1
timeout -k 10 200 python tools/env_ab.py RSD_TRACE_WAVES_PER_CU 8 12 bistro_1080p_full --n 10 --reps 3 > gpurun_out/r5k/wpc_c2_12.json 2>&1 || exit 1
timeout -k 10 200 python tools/env_ab.py RSD_TRACE_WAVES_PER_CU 8 16 emerald_4k_q --n 10 --reps 3 --walk quad > gpurun_out/r5k/wpc_c3_16.json 2>&1
