#!/bin/bash
# per-kernel durations of the SD trace (configs[1]) under rocprofv3 --kernel-trace --stats
set -o pipefail
OUT=gpurun_out/${1:-kstats}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 -u tools/trace_probe.py --quick > "$OUT/probe.json" 2> "$OUT/probe.err"
rc=$?
cat "$OUT/probe.json"
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && cut -d, -f1-8 "$f" | head -20
exit $rc
