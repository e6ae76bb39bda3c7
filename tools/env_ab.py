"""Same-process A/B of an SD-trace environment switch (diagnostics, GPU box): the trace of one frame's
intervals (pass 1 once, the maps kept: no consume) timed with HIP events over `n` back-to-back launches,
alternating the settings for `reps` rounds; the SD maps of every setting must be the same bits.
usage: python tools/env_ab.py VAR value_a value_b [config] [--n 40] [--reps 6] [--walk fused|quad]
       [--what trace|pass1|pass2] (pass1 / pass2: that pass alone, its outputs compared the same way)
       [--hit-order canonical|traversal|wavefront] [--clean-tiles] (Renderer.keep_clean_tiles: the bench's SD maps)"""
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
if arg("--hit-order", "canonical") in ("traversal", "wavefront"):  # the DXR-like any-hit streams
    from rsd import abi
    kw = dict(kw, hit_order=abi.HIT_ORDER_TRAVERSAL if arg("--hit-order", "") == "traversal" else abi.HIT_ORDER_WAVEFRONT)
r = Renderer(make_scene(sc), FrameConfig(**kw))
if "--clean-tiles" in sys.argv:
    r.keep_clean_tiles()
r.gbuffer()
r.clear_intervals()
r.pass1()
torch.cuda.synchronize()


what = arg("--what", "trace")
if what == "pass2":
    r.sd_trace()
call = {"trace": r.sd_trace, "pass1": r.pass1, "pass2": r.pass2}[what]
out_of = {"trace": lambda: r.sd, "pass1": lambda: r.ray_minmax, "pass2": lambda: r.ao}[what]


def run(v):
    os.environ[var] = v
    call()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        call()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


times = {v: [] for v in vals}
maps = {}
for _ in range(reps):
    for v in vals:
        times[v].append(run(v))
        maps[v] = out_of().cpu().numpy().view(np.uint8).copy()
same = all(np.array_equal(maps[vals[0]], maps[v]) for v in vals[1:])
print(json.dumps({"config": name, "what": what, "var": var, "walk": os.environ.get("RSD_TRACE_WALK", "default"), "n": n,
                  "us": {v: [round(t, 2) for t in ts] for v, ts in times.items()},
                  "median_us": {v: round(float(np.median(ts)), 2) for v, ts in times.items()}, "same_bits": same}))
