#!/bin/bash
# Memory-path PMC passes over one SVAO pass alone (tools/pass_loop.py <what> 10 at configs[1]): L2 hit /
# miss, L1->L2 requests and their latency, HBM read requests.  One pass per counter block, each under
# its own kill timer.  usage: bash tools/pmc_mem_pass.sh <tag> [pass1|pass2|trace] [lib variant]
set -o pipefail
OUT=gpurun_out/${1:-pmc_mem_pass}
WHAT=${2:-pass1}
[ -n "$3" ] && export RSD_LIB_VARIANT=$3
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum --kernel-trace -d "$OUT/tcp" -o run --output-format csv -- python3 tools/pass_loop.py "$WHAT" 10 > "$OUT/tcp.log" 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --kernel-trace -d "$OUT/tcc" -o run --output-format csv -- python3 tools/pass_loop.py "$WHAT" 10 > "$OUT/tcc.log" 2>&1
rc=$?
echo "exit $rc" > "$OUT/status"
exit $rc
