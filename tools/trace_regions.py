"""Per-region kernel timeline of a bench.py rocprofv3 --kernel-trace run (diagnostics): splits the
trace into the latency region (one frame in flight) and the throughput region (F frames in flight)
at the first pass-1 launch on a second queue/stream, then prints per-kernel mean durations, the
region span per frame, the GPU-busy fraction (union of kernel intervals) and the mean concurrency.
usage: python tools/trace_regions.py <run_kernel_trace.csv> [frames_per_region]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
K = int(sys.argv[2]) if len(sys.argv) > 2 else 50
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Stream_Id", r.get("Queue_Id")))
            for r in rows)
p1 = [e for e in ev if "svao_pass1" in e[2]]
# the last 2K pass-1 launches: K latency frames then K throughput frames (warm-ups come before each)
def short(n):
    for k in ("svao_pass1", "svao_pass2", "sd_setup", "sd_trace_row", "sd_trace_queue", "sd_trace_quad", "clear_intervals",
              "gbuffer", "elementwise", "fillBuffer", "copyBuffer"):
        if k in n:
            return k
    return n[:30]
def region(t0, t1, label, nfr):
    ks = [e for e in ev if e[0] >= t0 and e[1] <= t1]
    d = defaultdict(list)
    for s, e, n, q in ks:
        d[short(n)].append(e - s)
    iv = sorted((s, e) for s, e, _, _ in ks)
    busy, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    span = t1 - t0
    work = sum(e - s for s, e, _, _ in ks)
    print(f"== {label}: span/frame {span / nfr / 1e3:.1f} us, busy {busy / span:.3f}, mean concurrency when busy {work / max(busy, 1):.2f}")
    for k, v in sorted(d.items(), key=lambda x: -sum(x[1])):
        print(f"   {k:18s} n={len(v):4d} mean {sum(v) / len(v) / 1e3:8.1f} us  per frame {sum(v) / nfr / 1e3:8.1f} us")
lat = p1[-2 * K - (len(p1) - 2 * K) // 2:]  # approximate: use explicit split below
# split: throughput frames are the last K pass-1 launches; latency frames the K before the throughput warm-ups
n = len(p1)
thr = p1[n - K:]
warm = (n - 2 * K) // 2
latf = p1[n - 2 * K - warm:n - K - warm]
region(latf[0][0], thr[0][0] - 1, "latency", K)  # includes the throughput warm-ups' tail; see below
region(latf[0][0], latf[-1][0], "latency (first to last pass-1 start)", K - 1)
region(thr[0][0], max(e[1] for e in ev), "throughput", K)
