# round-5 batch l: configs[1] walk choice with the new quad walk; the traversal-order walk's waves per CU
mkdir -p gpurun_out/r5l
timeout -k 10 200 python tools/env_ab.py RSD_TRACE_WALK fused quad --n 40 --reps 4 > gpurun_out/r5l/walk_c1.json 2>&1 || exit 1
timeout -k 10 200 python tools/env_ab.py RSD_TRACE_WAVES_PER_CU 8 16 --n 20 --reps 4 --hit-order traversal > gpurun_out/r5l/wpc_ordered_c1.json 2>&1 || exit 1
timeout -k 10 200 python tools/env_ab.py RSD_TRACE_WAVES_PER_CU 8 12 --n 20 --reps 4 --hit-order traversal > gpurun_out/r5l/wpc12_ordered_c1.json 2>&1
