#!/bin/bash
# PMC passes over the SD trace alone (tools/sd_time.py: 21 row-walk traces of configs[1]) + phase clocks
set -o pipefail
OUT=gpurun_out/${1:-pmc_trace}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA --kernel-trace -d "$OUT/p1" -o run --output-format csv -- python3 tools/sd_time.py > "$OUT/p1.log" 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAVES SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS --kernel-trace -d "$OUT/p2" -o run --output-format csv -- python3 tools/sd_time.py > "$OUT/p2.log" 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_LATENCY_sum --kernel-trace -d "$OUT/p3" -o run --output-format csv -- python3 tools/sd_time.py > "$OUT/p3.log" 2>&1
rc=$?
echo "exit $rc" > "$OUT/status"
exit $rc
