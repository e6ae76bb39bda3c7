#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r3d}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/host_probe.py > "$OUT/host_probe.json" 2> "$OUT/err.log" &&
timeout -k 10 120 python -u tools/pass2_probe.py > "$OUT/pass2_probe.json" 2>> "$OUT/err.log" &&
for k in 1 2; do
  timeout -k 10 120 python -u tools/pass_time.py > "$OUT/pass_time_lean_$k.json" 2>> "$OUT/err.log" &&
  RSD_PASS1=generic timeout -k 10 120 python -u tools/pass_time.py > "$OUT/pass_time_generic_$k.json" 2>> "$OUT/err.log" || exit 1
done &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py "tests/test_gpu_fullsize.py::test_frame_graphs_equal_sequential" -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 &&
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 --graphs on > "$OUT/bench20_graphs_$k.json" 2>> "$OUT/err.log" &&
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 --graphs off > "$OUT/bench20_eager_$k.json" 2>> "$OUT/err.log" || exit 1
done &&
timeout -k 10 300 python -u tools/halo_plan.py bistro_4k_full_n16 > "$OUT/halo_plan_config4.json" 2>> "$OUT/err.log" &&
timeout -k 10 300 python -u tools/halo_plan.py emerald_4k_q --worlds 2,4,8 > "$OUT/halo_plan_config3.json" 2>> "$OUT/err.log" &&
timeout -k 10 300 python -u tools/halo_plan.py suntemple_1080p_q --worlds 2,4,8 > "$OUT/halo_plan_config1.json" 2>> "$OUT/err.log" &&
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharding.py -m gpu -x -q --timeout 600 --timeout-method thread > "$OUT/pytest_sharding.log" 2>&1
rc=$?
echo "exit $rc" > "$OUT/status"
exit $rc
