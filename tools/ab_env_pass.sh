#!/bin/bash
# Same-box A/B of env settings (diagnostics): per-pass times (tools/pass_time.py) and the bench line at
# --steps 200, alternating.  usage: bash tools/ab_env_pass.sh <tag> <reps> "<env>" "<env>" ...  ("-": none)
set -o pipefail
O=gpurun_out/$1; R=$2; shift 2; mkdir -p $O
export TMPDIR=/tmp
for rep in $(seq 1 $R); do
  i=0
  for cfg in "$@"; do
    i=$((i + 1)); [ "$cfg" = "-" ] && cfg="RSD_AB_NONE=1"
    echo "$cfg pass $(env $cfg timeout -k 10 120 python3 -u tools/pass_time.py 2>>$O/err.log)" >> $O/ab.txt || exit 1
    echo "$cfg s200 $(env $cfg timeout -k 10 200 python3 -u bench.py --cpu-baseline-seconds 0 2>>$O/err.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["throughput"]["ms_per_frame"], d["sd_kernel_ms"])')" >> $O/ab.txt || exit 1
  done
done
