"""Summarise an A/B directory written by tools/ab_lib.sh: pass times and bench numbers per variant."""
import json
import sys
from collections import defaultdict
from pathlib import Path

d = Path(sys.argv[1])
rows = defaultdict(lambda: defaultdict(list))
for f in sorted(d.glob("*.json")):
    kind, var = f.stem.split("_")[0], "_".join(f.stem.split("_")[1:-1])
    j = json.loads(f.read_text())
    if kind == "pass":
        for k in ("pass1_us", "sd_trace_us", "pass2_us", "ao_span_us"):
            if k in j:
                rows[var][k].append(j[k])
    else:
        rows[var][kind + "_ms_per_step"].append(j["ms_per_step"])
        rows[var][kind + "_sd_kernel_ms"].append(j["sd_kernel_ms"])
for var, r in rows.items():
    print(var, {k: v for k, v in r.items()})
