set -o pipefail
mkdir -p gpurun_out/p1
export RSD_LIB_VARIANT=p
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/p1/pytest.log 2>&1 &&
unset RSD_LIB_VARIANT &&
bash tools/gpu_variant_ab.sh p1 "base p"
