# round-5 batch d: the whole GPU suite after the band-frame / quad-walk / Raytraced changes, then the host profile
mkdir -p gpurun_out/r5d
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r5d/pytest_gpu.log 2>&1
rc=$?; echo rc=$rc >> gpurun_out/r5d/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/halo_host_profile.py > gpurun_out/r5d/host_profile.log 2>&1
