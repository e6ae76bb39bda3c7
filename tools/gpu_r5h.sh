# round-5 batch h: persistent waves per CU of the quad walk (full-res / 4K maps) and of the row walk
mkdir -p gpurun_out/r5h
timeout -k 10 200 python tools/env_ab.py RSD_TRACE_WAVES_PER_CU 8 12 bistro_1080p_full --n 10 --reps 3 > gpurun_out/r5h/wpc_c2_12.json 2>&1 || exit 1
timeout -k 10 200 python tools/env_ab.py RSD_TRACE_WAVES_PER_CU 8 16 bistro_1080p_full --n 10 --reps 3 > gpurun_out/r5h/wpc_c2_16.json 2>&1 || exit 1
timeout -k 10 200 python tools/env_ab.py RSD_TRACE_WAVES_PER_CU 8 12 emerald_4k_q --n 10 --reps 3 > gpurun_out/r5h/wpc_c3_12.json 2>&1 || exit 1
timeout -k 10 300 python tools/env_ab.py RSD_TRACE_WAVES_PER_CU 8 12 bistro_4k_full_n16 --n 5 --reps 3 > gpurun_out/r5h/wpc_c4_12.json 2>&1 || exit 1
timeout -k 10 200 python tools/env_ab.py RSD_TRACE_WAVES_PER_CU 8 12 --n 40 --reps 4 > gpurun_out/r5h/wpc_c1_12.json 2>&1
