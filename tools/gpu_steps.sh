#!/usr/bin/env bash
# Run GPU steps in order inside one gpurun call, each under its own time limit; stop at the first
# step that ends by a fault, an abort, a signal or a time limit (exit 124 / 134 / 137 / 139 / > 128),
# go on after ordinary failures (a failed assertion: exit 1 / 2).
#
#   tools/gpu_steps.sh OUTDIR "SECONDS NAME COMMAND..." ["SECONDS NAME COMMAND..." ...]
#
# Each step's stdout + stderr goes to OUTDIR/NAME.log; OUTDIR/steps.txt records every exit status.
set -u
out=$1
shift
mkdir -p "$out"
export TMPDIR=/tmp
for step in "$@"; do
    read -r secs name cmd <<<"$step"
    echo "[$(date +%T)] $name: $cmd" | tee -a "$out/steps.txt"
    timeout -k 10 "$secs" bash -c "$cmd" >"$out/$name.log" 2>&1
    rc=$?
    echo "[$(date +%T)] $name rc=$rc" | tee -a "$out/steps.txt"
    tail -n 3 "$out/$name.log"
    if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ] || [ $rc -gt 128 ]; then
        echo "stopping: $name ended with $rc" | tee -a "$out/steps.txt"
        exit $rc
    fi
done
