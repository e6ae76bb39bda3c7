#!/bin/bash
# round-2: raster SD walk parity + timing
set -o pipefail
OUT=gpurun_out/${1:-r2d}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_raster.py -x -v --timeout 600 --timeout-method thread --durations=5 > "$OUT/pytest_raster.log" 2>&1 &&
RSD_TRACE_WALK=raster timeout -k 10 300 python -u tools/trace_probe.py > "$OUT/probe_raster.json" 2> "$OUT/probe_raster.err" &&
timeout -k 10 300 python -u tools/trace_probe.py --quick > "$OUT/probe_base.json" 2> "$OUT/probe_base.err" &&
RSD_TRACE_WALK=raster timeout -k 10 300 python -u tools/trace_probe.py bistro_1080p_full --quick > "$OUT/probe_raster_c3.json" 2> "$OUT/probe_raster_c3.err" &&
timeout -k 10 300 python -u tools/trace_probe.py bistro_1080p_full --quick > "$OUT/probe_base_c3.json" 2> "$OUT/probe_base_c3.err"
rc=$?
echo "exit $rc" > "$OUT/status"
exit $rc
