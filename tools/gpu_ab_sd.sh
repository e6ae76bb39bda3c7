#!/bin/bash
# A/B of SD-trace variants on configs[1]: tools/sd_time.py twice per variant (env per variant), then a
# rocprofv3 kernel split of the default.  usage: bash tools/gpu_ab_sd.sh <tag> "<env>" "<env>" ...
set -o pipefail
OUT=gpurun_out/${1:-ab}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in "$@"; do
  echo "== $cfg" >> "$OUT/sd_time.txt"
  env $cfg timeout -k 10 120 python3 -u tools/sd_time.py >> "$OUT/sd_time.txt" 2>&1 || exit 1
  env $cfg timeout -k 10 120 python3 -u tools/sd_time.py >> "$OUT/sd_time.txt" 2>&1 || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 -u tools/sd_time.py > "$OUT/prof.log" 2>&1
