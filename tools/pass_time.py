"""Per-pass GPU time of one AO frame (diagnostics): pass 1, SD trace, pass 2 of a BASELINE config,
each the median over 200 sequential frames of HIP events around the pass (clear -> pass 1 ->
trace -> pass 2 per frame, so pass 2 always consumes the busy-tile flags of its own pass 1).
usage: python tools/pass_time.py [config] [--frames N]"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ray-traced-stochastic-depth-map_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rsd.frame import CONFIGS, FrameConfig, Renderer  # noqa: E402
from rsd.scenes import make_scene  # noqa: E402
from rsd.timing import TimingEvent  # noqa: E402

name = next((a for a in sys.argv[1:] if not a.startswith("--")), "suntemple_1080p_q")
frames = int(sys.argv[sys.argv.index("--frames") + 1]) if "--frames" in sys.argv else 200
kw, sc = CONFIGS[name]
r = Renderer(make_scene(sc), FrameConfig(**kw))
r.gbuffer()
for _ in range(5):
    r.frame()
torch.cuda.synchronize()
ev = [[TimingEvent() for _ in range(4)] for _ in range(frames)]  # fence-free (rsd/timing.py)
for e in ev:
    r.clear_intervals()
    e[0].record()
    r.pass1()
    e[1].record()
    r.sd_trace()
    e[2].record()
    r.pass2()
    e[3].record()
torch.cuda.synchronize()
t = np.array([[e[i].elapsed_time(e[i + 1]) * 1e3 for i in range(3)] for e in ev])
med = np.median(t, axis=0)
print(json.dumps({"config": name, "frames": frames, "pass1_us": round(float(med[0]), 2),
                  "sd_trace_us": round(float(med[1]), 2), "pass2_us": round(float(med[2]), 2),
                  "ao_span_us": round(float(np.median(t.sum(axis=1))), 2)}))
