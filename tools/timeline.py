"""Kernel timeline of bench.py's throughput region from a rocprofv3 --kernel-trace CSV (diagnostics).

The throughput region is taken as the last `--frames` pass-1 launches and everything that starts
after the first of them.  Prints per kernel class: launches, mean duration, and how the region's
wall time splits by which classes are running (idle / pass 1 only / trace only / ...).
usage: python tools/timeline.py <run_kernel_trace.csv> [--frames N]"""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
frames = int(sys.argv[sys.argv.index("--frames") + 1]) if "--frames" in sys.argv else 200


def klass(name):
    if "svao_pass1" in name:
        return "p1"
    if "svao_pass2" in name:
        return "p2"
    if "sd_setup" in name:
        return "setup"
    if "sd_trace" in name or "sd_resolve" in name:
        return "walk"
    return "other"


rows = []
with open(path) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), klass(r["Kernel_Name"]), int(r["Queue_Id"])))
rows.sort()
p1 = [r for r in rows if r[2] == "p1"]
t0 = p1[-frames][0]
reg = [r for r in rows if r[0] >= t0]
t1 = max(r[1] for r in reg)
print(f"region: {len(reg)} kernels, {(t1 - t0) / 1e3:.1f} us, {(t1 - t0) / 1e3 / frames:.2f} us per frame")
dur = defaultdict(list)
for s, e, k, q in reg:
    dur[k].append((e - s) / 1e3)
for k, v in sorted(dur.items()):
    print(f"  {k:6s} n={len(v):4d} mean {sum(v) / len(v):7.2f} us  sum/frame {sum(v) / frames:7.2f} us")
# sweep: time by the set of running classes
ev = []
for s, e, k, q in reg:
    ev.append((s, 1, k))
    ev.append((e, -1, k))
ev.sort()
run = defaultdict(int)
acc = defaultdict(float)
last = t0
for t, d, k in ev:
    if t > last:
        key = "+".join(sorted(c for c, n in run.items() if n > 0)) or "idle"
        acc[key] += t - last
        last = t
    run[k] += d
tot = sum(acc.values())
print("time by running set (share of region):")
for key, v in sorted(acc.items(), key=lambda x: -x[1]):
    print(f"  {key:24s} {v / tot * 100:5.1f} %  {v / 1e3 / frames:6.2f} us/frame")
# concurrency of each class: mean number of instances running while any runs
for k in dur:
    busy = sum(v for key, v in acc.items() if k in key.split("+"))
    print(f"  {k}: running {busy / tot * 100:5.1f} % of the region")
