mkdir -p gpurun_out/r5b
timeout -k 10 900 python -u -m pytest tests/test_gpu_band_native.py tests/test_gpu_kernels.py tests/test_gpu_numerics.py -k "native or rccl or local_comm or raytraced or degenerate" -v --timeout 600 --timeout-method thread > gpurun_out/r5b/tests.log 2>&1
rc=$?; echo rc=$rc >> gpurun_out/r5b/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python tools/env_ab.py RSD_TRACE_SPREAD off on > gpurun_out/r5b/spread_c1.json 2>&1 || exit 1
timeout -k 10 200 python tools/env_ab.py RSD_TRACE_SPREAD off on bistro_1080p_full --n 10 --reps 4 > gpurun_out/r5b/spread_c2.json 2>&1 || exit 1
timeout -k 10 300 python tools/halo_host_profile.py > gpurun_out/r5b/host_profile.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config bistro_1080p_full --steps 10 --warmup 3 --cpu-baseline-seconds 0 --hit-order-record 0 > gpurun_out/r5b/bench_c2.json 2> gpurun_out/r5b/bench_c2.err
