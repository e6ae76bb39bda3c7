set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
i=0
for ctr in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64" "FETCH_SIZE TA_BUSY_avr"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-trace -d gpurun_out/pmc/p$i -o run --output-format csv -- python3 tools/pass_loop.py pass1 10 > gpurun_out/pmc/p$i.log 2>&1 || exit 1
done
echo ok
