# round-5 batch f: stale busy-tile flags test, the parity file, pass-1 memory counters
mkdir -p gpurun_out/r5f
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread > gpurun_out/r5f/tests.log 2>&1
rc=$?; echo rc=$rc >> gpurun_out/r5f/tests.log
[ $rc -le 1 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && bash tools/pmc_pass1_mem.sh r5f/pass1_mem pass1
