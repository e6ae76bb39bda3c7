#!/bin/bash
# PMC passes over SVAO pass 1 alone (tools/pass_loop.py pass1: 10 launches at configs[1]): the
# issue-cycle split VERDICT r2 asks for (VALU / transcendental / f64 instruction counts, active
# VALU cycles, busy and wait cycles).  Counter names absent from this rocprofv3 are dropped
# (tools/pmc_filter.py over `rocprofv3 -L`).  usage: bash tools/pmc_pass1.sh [tag] [pass1|pass2|trace]
set -o pipefail
OUT=gpurun_out/${1:-pmc_pass1}
WHAT=${2:-pass1}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
for ctr in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 SQ_ACTIVE_INST_SCA" \
           "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32" \
           "SQ_INST_CYCLES_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_BRANCH SQ_INSTS_SENDMSG SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_MFMA_F32 SQ_WAIT_INST_LDS" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  sel=$(python3 tools/pmc_filter.py "$OUT/counters_list.txt" $ctr)
  echo "pass $i: $sel" >> "$OUT/passes.txt"
  [ -z "$sel" ] && continue
  timeout -s KILL 90 rocprofv3 --pmc $sel --kernel-trace -d "$OUT/p$i" -o run --output-format csv -- python3 tools/pass_loop.py "$WHAT" 10 > "$OUT/p$i.log" 2>&1 || exit 1
done
echo ok
