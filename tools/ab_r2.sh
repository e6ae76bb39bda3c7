#!/bin/bash
# Same-box comparison of the round-2 final tree (_ab/r2, built from a932cbf) with the working tree.
set -o pipefail
O=gpurun_out/$1; R=${2:-2}; mkdir -p $O
for rep in $(seq 1 $R); do
  (cd _ab/r2 && timeout -k 10 120 python -u tools/pass_time.py) > $O/pass_r2_$rep.json 2>>$O/err.log || exit 1
  timeout -k 10 120 python -u tools/pass_time.py > $O/pass_new_$rep.json 2>>$O/err.log || exit 1
  for st in 20 200; do
    (cd _ab/r2 && timeout -k 10 200 python -u bench.py --steps $st --warmup 5 --cpu-baseline-seconds 0) > $O/s${st}_r2_$rep.json 2>>$O/err.log || exit 1
    timeout -k 10 200 python -u bench.py --steps $st --warmup 5 --cpu-baseline-seconds 0 > $O/s${st}_new_$rep.json 2>>$O/err.log || exit 1
  done
done
