#!/bin/bash
# rocprofv3 kernel stats of tools/pass_time.py in the round-2 tree (_ab/r2) and the working tree (same box).
set -o pipefail
O=gpurun_out/$1; mkdir -p $O; export TMPDIR=/tmp
(cd _ab/r2 && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d ../../$O/r2 -o run --output-format csv -- python3 tools/pass_time.py) > $O/r2.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/new -o run --output-format csv -- python3 tools/pass_time.py > $O/new.log 2>&1
