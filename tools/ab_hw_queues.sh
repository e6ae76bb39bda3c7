#!/bin/bash
# A/B: HIP hardware queues per process x frames in flight (bench.py --steps 20)
set -o pipefail
O=gpurun_out/r3s3g; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
for cfg in "4 4" "8 4" "8 6" "8 8"; do
  set -- $cfg
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 200 python -u bench.py --steps 20 --frames-in-flight $2 --cpu-baseline-seconds 0 > $O/q$1_f$2_$rep.json 2>>$O/err.log || exit 1
done; done
python3 - <<'PY' > $O/summary.txt
import json, glob, collections
r = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r3s3g/q*_f*_*.json")):
    k = f.split("/")[-1].rsplit("_", 1)[0]
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r[k].append((d["ms_per_step"], d["throughput"]["sd_kernel_ms_overlapped"]))
for k, v in r.items():
    print(k, "ms_per_step", [a for a, _ in v], "sd_overlapped", [b for _, b in v])
PY
