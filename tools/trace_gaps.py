#!/usr/bin/env python3
"""Setup / walk durations and the gaps between consecutive kernels of back-to-back SD traces, from a
rocprofv3 kernel trace (diagnostics: how much of rsd_sd_trace's event-to-event time is kernel time).

    rocprofv3 --kernel-trace -d DIR -o run --output-format csv -- python3 tools/sd_time.py
    python tools/trace_gaps.py DIR"""
import csv
import json
import statistics
import sys
from pathlib import Path

path = next(Path(sys.argv[1]).rglob("*kernel_trace.csv"))
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
ks = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
setup = [(s, e) for n, s, e in ks if "sd_setup_kernel" in n]
# the two-pass setup (sd_classify_kernel + sd_live_kernel): one setup span from the classify start to the live end
cls = [(s, e) for n, s, e in ks if "sd_classify_kernel" in n]
live = [(s, e) for n, s, e in ks if "sd_live_kernel" in n]
if cls:
    setup = []
    for s0, e0 in cls:
        nl = next(((s, e) for s, e in live if s >= e0), None)
        if nl:
            setup.append((s0, nl[1]))
    lk = [(e - s) / 1e3 for s, e in live][2:]
    ck = [(e - s) / 1e3 for s, e in cls][2:]
    print(json.dumps({"classify_us": round(statistics.median(ck), 2), "live_us": round(statistics.median(lk), 2)}))
walk = [(n, s, e) for n, s, e in ks if "sd_trace_row_kernel" in n or "sd_trace_queue_kernel" in n or
        "sd_trace_hybrid_kernel" in n]
pairs = []
for s0, e0 in setup:
    nxt = next(((n, s, e) for n, s, e in walk if s >= e0), None)
    if nxt:
        pairs.append((e0 - s0, nxt[1] - e0, nxt[2] - nxt[1], nxt[2] - s0))
pairs = pairs[2:]  # skip the first traces (cold caches, code-object load)
med = lambda i: round(statistics.median(p[i] for p in pairs) / 1e3, 2)  # noqa: E731
print(json.dumps({"traces": len(pairs), "setup_us": med(0), "gap_setup_to_walk_us": med(1), "walk_us": med(2),
                  "setup_start_to_walk_end_us": med(3)}))
