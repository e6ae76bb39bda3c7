"""Per-pass GPU time of one AO frame (diagnostics): pass 1, SD trace, pass 2 of a BASELINE config,
each the median of 7 batches of 40 back-to-back launches (HIP events).  Pass 2 re-runs on the
same stencil / SD map (it rewrites the AO image in place: timing only).
usage: python tools/pass_time.py [config]"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ray-traced-stochastic-depth-map_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rsd.frame import CONFIGS, FrameConfig, Renderer  # noqa: E402
from rsd.scenes import make_scene  # noqa: E402


def timeit(fn, n=40, batches=7):
    fn()
    torch.cuda.synchronize()
    res = []
    for _ in range(batches):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            fn()
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) / n * 1e3)
    return float(np.median(res))


name = next((a for a in sys.argv[1:] if not a.startswith("--")), "suntemple_1080p_q")
kw, sc = CONFIGS[name]
r = Renderer(make_scene(sc), FrameConfig(**kw))
r.gbuffer()
r.frame()
torch.cuda.synchronize()
out = {"config": name, "pass1_us": timeit(r.pass1), "pass2_us": timeit(r.pass2)}
iv = r.ray_minmax.clone()
r.clear_intervals()
r.pass1()
out["sd_trace_us"] = timeit(lambda: r.sd_trace())
print(json.dumps(out))
