cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python tools/diag_sd.py > gpurun_out/diag3.log 2>&1; echo "exit $?" >> gpurun_out/diag3.log
