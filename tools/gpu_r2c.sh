#!/bin/bash
# round-2: contiguous-band / halo sharding on the GPU, then the gloo multi-rank bench rehearsal
set -o pipefail
OUT=gpurun_out/${1:-r2c}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharding.py -x -v --timeout 600 --timeout-method thread --durations=5 > "$OUT/pytest_sharding.log" 2>&1 &&
bash tools/gpu_multirank.sh ${1:-r2c}/multirank
rc=$?
echo "exit $rc" > "$OUT/status"
exit $rc
