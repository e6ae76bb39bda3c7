#!/bin/bash
# Memory-path PMC passes over SVAO pass 1 alone (tools/pass_loop.py pass1 10 at configs[1], the product's fast
# numerics): vector L1 (TCP) hit traffic and the latency of its L2 requests, L2 (TCC) hits / misses and
# memory-side reads, texture-address (TA) and -data (TD) unit activity.  One pass per counter block under
# its own kill timer; names this rocprofv3 does not know are dropped (tools/pmc_filter.py).
# usage: bash tools/pmc_pass1_mem.sh <tag> [pass1|pass2|trace] [config]
# (the last pass is the instruction mix: VALU / SALU / LDS / SMEM instructions and the VALU / LDS issue cycles)
set -o pipefail
OUT=gpurun_out/${1:-pmc_pass1_mem}
WHAT=${2:-pass1}
CONFIG=${3:-suntemple_1080p_q}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
for ctr in "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" \
           "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum" \
           "TD_BUSY_avr TD_TD_BUSY_sum" \
           "TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"; do
  i=$((i+1))
  sel=$(python3 tools/pmc_filter.py "$OUT/counters_list.txt" $ctr)
  echo "pass $i: $sel" >> "$OUT/passes.txt"
  [ -z "$sel" ] && continue
  timeout -s KILL 90 rocprofv3 --pmc $sel --kernel-trace -d "$OUT/p$i" -o run --output-format csv -- python3 tools/pass_loop.py "$WHAT" 10 "$CONFIG" > "$OUT/p$i.log" 2>&1 || exit 1
done
echo ok
