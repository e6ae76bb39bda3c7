set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest exit $?" >> gpurun_out/pytest_gpu.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline-seconds 0 > gpurun_out/bench2.log 2>&1; echo "bench exit $?" >> gpurun_out/bench2.log
