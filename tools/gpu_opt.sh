set -o pipefail
export TMPDIR=/tmp
TAG=${1:-opt}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 &&
timeout -k 10 120 python -u tools/sd_time.py > gpurun_out/$TAG/sd.log 2>&1 &&
RSD_RESOLVE_WAVES_PER_CU=16 timeout -k 10 120 python -u tools/sd_time.py >> gpurun_out/$TAG/sd.log 2>&1 &&
RSD_RESOLVE_WAVES_PER_CU=32 timeout -k 10 120 python -u tools/sd_time.py >> gpurun_out/$TAG/sd.log 2>&1 &&
timeout -k 10 300 python -u bench.py --cpu-baseline-seconds 0 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --cpu-baseline-seconds 0 > gpurun_out/$TAG/prof.log 2>&1
