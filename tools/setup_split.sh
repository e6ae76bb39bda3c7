#!/bin/bash
# SD-trace setup / walk split under env settings (diagnostics): a kernel trace of tools/sd_time.py per
# setting, split by tools/trace_gaps.py.  usage: bash tools/setup_split.sh <tag> "<env>" ...  ("-": none)
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i + 1)); [ "$cfg" = "-" ] && cfg="RSD_AB_NONE=1"
  env $cfg timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$i -o run -- python3 -u tools/sd_time.py ${SD_TIME_ARGS:-} > $O/kt_$i.log 2>&1 || exit 1
  echo "$cfg $(python3 tools/trace_gaps.py $O/kt_$i)" >> $O/split.txt || exit 1
done
