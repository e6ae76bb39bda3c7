#!/bin/bash
# memory-path PMC passes over the SD trace (tools/sd_time.py: 21 traces of configs[1]); one pass
# per counter block, each under its own kill timer
set -o pipefail
OUT=gpurun_out/${1:-pmc_mem}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum --kernel-trace -d "$OUT/tcp" -o run --output-format csv -- python3 tools/sd_time.py > "$OUT/tcp.log" 2>&1
echo "tcp rc $?"
timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_TAG_STALL_sum --kernel-trace -d "$OUT/tcc" -o run --output-format csv -- python3 tools/sd_time.py > "$OUT/tcc.log" 2>&1
echo "tcc rc $?"
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CU_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_WAVE_CYCLES --kernel-trace -d "$OUT/sq" -o run --output-format csv -- python3 tools/sd_time.py > "$OUT/sq.log" 2>&1
echo "sq rc $?"
exit 0
