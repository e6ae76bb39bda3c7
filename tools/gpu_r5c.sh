# round-5 measurement batch c: native band-frame host cost, HIP launch floor, walk choice at the 4K / full-res configs
mkdir -p gpurun_out/r5c
timeout -k 10 120 python -u -m pytest tests/test_gpu_kernels.py -k "refuses" -q --timeout 100 --timeout-method thread > gpurun_out/r5c/tests.log 2>&1 || exit 1
timeout -k 10 60 ./tools/_launch_floor > gpurun_out/r5c/launch_floor.json 2>&1 || exit 1
timeout -k 10 300 python tools/halo_host_profile.py > gpurun_out/r5c/host_profile.log 2>&1 || exit 1
timeout -k 10 200 python tools/env_ab.py RSD_TRACE_WALK quad fused bistro_1080p_full --n 10 --reps 3 > gpurun_out/r5c/walk_c2.json 2>&1 || exit 1
timeout -k 10 200 python tools/env_ab.py RSD_TRACE_WALK quad fused emerald_4k_q --n 10 --reps 3 > gpurun_out/r5c/walk_c3.json 2>&1 || exit 1
timeout -k 10 300 python tools/env_ab.py RSD_TRACE_WALK quad fused bistro_4k_full_n16 --n 5 --reps 3 > gpurun_out/r5c/walk_c4.json 2>&1 || exit 1
timeout -k 10 300 python tools/env_ab.py RSD_TRACE_SPREAD off on bistro_4k_full_n16 --n 5 --reps 3 > gpurun_out/r5c/spread_c4.json 2>&1 || exit 1
timeout -k 10 200 python tools/env_ab.py RSD_TRACE_SPREAD off on emerald_4k_q --n 10 --reps 3 --walk quad > gpurun_out/r5c/spread_c3.json 2>&1
