cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/r6/pytest_gpu.log 2>&1; echo "pytest exit $?" >> gpurun_out/r6/pytest_gpu.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof -o run --output-format csv -- python3 bench.py --steps 100 --warmup 10 --cpu-baseline-seconds 0 > gpurun_out/r6/bench_prof.log 2>&1; echo "prof exit $?" >> gpurun_out/r6/bench_prof.log
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r6/pmc1 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --cpu-baseline-seconds 0 > gpurun_out/r6/pmc1.log 2>&1; echo "pmc1 exit $?" >> gpurun_out/r6/pmc1.log
