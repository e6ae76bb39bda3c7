set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest exit $?" >> gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline-seconds 5 > gpurun_out/bench1.log 2>&1; echo "bench exit $?" >> gpurun_out/bench1.log
