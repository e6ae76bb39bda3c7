cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r5; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/r5/pytest_gpu.log 2>&1; echo "pytest exit $?" >> gpurun_out/r5/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/r5/bench.log 2>&1; echo "bench exit $?" >> gpurun_out/r5/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof -o run --output-format csv -- python3 bench.py --steps 100 --warmup 10 --cpu-baseline-seconds 0 > gpurun_out/r5/bench_prof.log 2>&1; echo "prof exit $?" >> gpurun_out/r5/bench_prof.log
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r5/pmc1 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --cpu-baseline-seconds 0 > gpurun_out/r5/pmc1.log 2>&1; echo "pmc1 exit $?" >> gpurun_out/r5/pmc1.log
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r5/pmc2 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --cpu-baseline-seconds 0 > gpurun_out/r5/pmc2.log 2>&1; echo "pmc2 exit $?" >> gpurun_out/r5/pmc2.log
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/r5/bench_2rank_1gpu.log 2>&1; echo "torchrun exit $?" >> gpurun_out/r5/bench_2rank_1gpu.log
