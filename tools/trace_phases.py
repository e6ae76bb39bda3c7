#!/usr/bin/env python3
"""Where a row step of the SD walk spends its time (diagnostics): the instrumented walk's phase clocks
per row step -- fetch wait, box tests + child sort, triangle tests, merge + push, LDS pool -- in
microseconds (s_memtime calibrated against s_memrealtime in the same launch).  The instrumented walk
waits on every load (its fetch phase is the full load latency) and keeps the 256-entry pool.

usage: python tools/trace_phases.py [config] [--reps 5]"""
import json
import os
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
if os.environ.get("RSD_TRACE_PHASES") != "1":  # re-run with the phase print on (a child, before any GPU use)
    env = dict(os.environ, RSD_TRACE_PHASES="1")
    p = subprocess.run([sys.executable, __file__] + sys.argv[1:], env=env, capture_output=True, text=True)
    lines = [ln for ln in p.stderr.splitlines() if "row walk phase clocks" in ln]
    if p.returncode or not lines:
        sys.stderr.write(p.stderr[-3000:])
        sys.exit(p.returncode or 1)
    info = json.loads(p.stdout.strip().splitlines()[-1])
    keys = ["fetch", "step", "resolve", "steps", "loops", "mem", "compute", "pool", "box", "tri", "merge"]
    tot = {k: 0 for k in keys}
    for ln in lines:
        vals = [int(x) for x in re.findall(r"\d+", ln.split("clocks:")[1])]
        for k, v in zip(keys, vals):
            tot[k] += v
    mhz, steps = info["shader_clock_mhz"], tot["steps"]
    per = {k: round(tot[k] / steps / mhz, 3) for k in ("mem", "box", "tri", "merge", "pool")}
    print(json.dumps({"config": info["config"], "traces": len(lines), "row_steps": steps,
                      "max_steps_per_ray": info["max_steps"], "shader_clock_mhz": round(mhz, 1),
                      "us_per_row_step": per,
                      "note": "instrumented walk (waits on every load); mem = fetch wait, box = box tests + child "
                              "sort, tri = triangle tests, merge = hit merge + push"}))
    sys.exit(0)

sys.path[:0] = [str(ROOT), str(ROOT / "ray-traced-stochastic-depth-map_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rsd.frame import CONFIGS, FrameConfig, Renderer  # noqa: E402
from rsd.scenes import make_scene  # noqa: E402

name = next((a for a in sys.argv[1:] if not a.startswith("--") and a in CONFIGS), "suntemple_1080p_q")
reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 5
kw, sc = CONFIGS[name]
r = Renderer(make_scene(sc), FrameConfig(**kw))
r.gbuffer()
mhz, mx = [], 0
for _ in range(reps):
    r.clear_intervals()
    r.pass1()
    c = r.sd_trace(counters=True)
    mhz.append(c.shader_clock_mhz)
    mx = max(mx, int(c.max_steps_per_ray))
torch.cuda.synchronize()
print(json.dumps({"config": name, "shader_clock_mhz": float(np.mean(mhz)), "max_steps": mx}))
