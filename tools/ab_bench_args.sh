#!/bin/bash
# Same-box A/B of bench.py argument sets (diagnostics), alternating per repetition; each argument set
# is one quoted string.  usage: bash tools/ab_bench_args.sh <tag> <reps> "<args>"...
set -o pipefail
O=gpurun_out/$1; R=$2; shift 2; mkdir -p $O
export TMPDIR=/tmp
for rep in $(seq 1 $R); do
k=0
for args in "$@"; do
  k=$((k+1))
  timeout -k 10 200 python -u bench.py $args --cpu-baseline-seconds 0 > $O/b${k}_$rep.json 2>>$O/err.log || exit 1
  echo "b$k: $args" > $O/b${k}.args
done; done
python3 - "$O" <<'EOF' > $O/summary.txt
import json, sys, glob, os
o = sys.argv[1]
for a in sorted(glob.glob(o + "/b*.args")):
    k = os.path.basename(a)[:-5]
    v = [json.loads(open(f).read().strip().splitlines()[-1]) for f in sorted(glob.glob(f"{o}/{k}_*.json"))]
    print(open(a).read().strip(), "ms_per_step", [x["ms_per_step"] for x in v], "sd_ms", [x["sd_kernel_ms"] for x in v])
EOF
