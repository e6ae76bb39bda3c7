set -o pipefail
mkdir -p gpurun_out/x1
export RSD_LIB_VARIANT=x
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/x1/pytest.log 2>&1 &&
unset RSD_LIB_VARIANT &&
bash tools/gpu_variant_ab.sh x1 "base x"
