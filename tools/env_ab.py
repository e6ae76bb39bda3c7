"""Same-process A/B of an SD-trace environment switch (diagnostics, GPU box): the trace of one frame's
intervals (pass 1 once, the maps kept: no consume) timed with HIP events over `n` back-to-back launches,
alternating the settings for `reps` rounds; the SD maps of every setting must be the same bits.
usage: python tools/env_ab.py VAR value_a value_b [config] [--n 40] [--reps 6] [--walk fused|quad]"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ray-traced-stochastic-depth-map_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rsd.frame import CONFIGS, FrameConfig, Renderer  # noqa: E402
from rsd.scenes import make_scene  # noqa: E402


def arg(flag, default):
    return sys.argv[sys.argv.index(flag) + 1] if flag in sys.argv else default


pos = [a for i, a in enumerate(sys.argv[1:], 1) if not a.startswith("--") and not sys.argv[i - 1].startswith("--")]
var, vals = pos[0], pos[1:3]
name = pos[3] if len(pos) > 3 else "suntemple_1080p_q"
n, reps = int(arg("--n", "40")), int(arg("--reps", "6"))
if "--walk" in sys.argv:
    os.environ["RSD_TRACE_WALK"] = arg("--walk", "fused")
kw, sc = CONFIGS[name]
r = Renderer(make_scene(sc), FrameConfig(**kw))
r.gbuffer()
r.clear_intervals()
r.pass1()
torch.cuda.synchronize()


def run(v):
    os.environ[var] = v
    r.sd_trace()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        r.sd_trace()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


times = {v: [] for v in vals}
maps = {}
for _ in range(reps):
    for v in vals:
        times[v].append(run(v))
        maps[v] = r.sd.cpu().numpy().view(np.uint32).copy()
same = all(np.array_equal(maps[vals[0]], maps[v]) for v in vals[1:])
print(json.dumps({"config": name, "var": var, "walk": os.environ.get("RSD_TRACE_WALK", "default"), "n": n,
                  "us": {v: [round(t, 2) for t in ts] for v, ts in times.items()},
                  "median_us": {v: round(float(np.median(ts)), 2) for v, ts in times.items()}, "same_bits": same}))
