#!/bin/bash
# SD-trace change check: the GPU parity tests of every trace walk, then trace timings (configs[1], [2])
set -o pipefail
OUT=gpurun_out/${1:-trace_check}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_hit_order.py tests/test_gpu_raster.py tests/test_gpu_fullsize.py -x -q --timeout 900 --timeout-method thread > "$OUT/pytest.log" 2>&1 &&
timeout -k 10 120 python -u tools/trace_probe.py --quick > "$OUT/probe_c1.json" 2> "$OUT/probe_c1.err" &&
RSD_TRACE_WALK=quad timeout -k 10 120 python -u tools/trace_probe.py --quick > "$OUT/probe_c1_quad.json" 2> "$OUT/probe_c1_quad.err" &&
timeout -k 10 120 python -u tools/trace_probe.py bistro_1080p_full --quick > "$OUT/probe_c2.json" 2> "$OUT/probe_c2.err"
rc=$?
echo "exit $rc" > "$OUT/status"
tail -1 "$OUT/pytest.log"; cat "$OUT"/probe*.json
exit $rc
