# round-5 batch e: the native band frame after the count-publish / point-to-point AO changes
mkdir -p gpurun_out/r5e
timeout -k 10 600 python -u -m pytest tests/test_gpu_band_native.py tests/test_gpu_sharding.py -v --timeout 500 --timeout-method thread > gpurun_out/r5e/tests.log 2>&1
rc=$?; echo rc=$rc >> gpurun_out/r5e/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/halo_host_profile.py > gpurun_out/r5e/host_profile.log 2>&1
