# round-5 batch i: the quad walk with keys-only K-lists (151 / 113 VGPRs at K = 16 / 8): waves per CU
mkdir -p gpurun_out/r5i
timeout -k 10 300 python tools/env_ab.py RSD_TRACE_WAVES_PER_CU 8 12 bistro_4k_full_n16 --n 5 --reps 3 > gpurun_out/r5i/wpc_c4_12.json 2>&1 || exit 1
timeout -k 10 200 python tools/env_ab.py RSD_TRACE_WAVES_PER_CU 8 12 bistro_1080p_full --n 10 --reps 3 > gpurun_out/r5i/wpc_c2_12.json 2>&1 || exit 1
timeout -k 10 200 python tools/env_ab.py RSD_TRACE_WAVES_PER_CU 8 16 bistro_1080p_full --n 10 --reps 3 > gpurun_out/r5i/wpc_c2_16.json 2>&1 || exit 1
timeout -k 10 200 python tools/env_ab.py RSD_TRACE_WAVES_PER_CU 8 12 emerald_4k_q --n 10 --reps 3 --walk quad > gpurun_out/r5i/wpc_c3_12.json 2>&1 || exit 1
timeout -k 10 200 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_configs.py -q --timeout 300 --timeout-method thread > gpurun_out/r5i/tests.log 2>&1
