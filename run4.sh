cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest exit $?" >> gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/diag_sd.py > gpurun_out/diag10.log 2>&1; echo "exit $?" >> gpurun_out/diag10.log
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-baseline-seconds 2 > gpurun_out/bench10.log 2>&1; echo "bench exit $?" >> gpurun_out/bench10.log
