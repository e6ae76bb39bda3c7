"""Launch one pass of a BASELINE config back to back (for rocprofv3 --pmc passes over a single
kernel): python tools/pass_loop.py {pass1|pass2|trace|frame} [n] [config]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ray-traced-stochastic-depth-map_amd")]
import torch  # noqa: E402

from rsd.frame import CONFIGS, FrameConfig, Renderer  # noqa: E402
from rsd.scenes import make_scene  # noqa: E402

what = sys.argv[1] if len(sys.argv) > 1 else "pass1"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
name = sys.argv[3] if len(sys.argv) > 3 else "suntemple_1080p_q"
kw, sc = CONFIGS[name]
r = Renderer(make_scene(sc), FrameConfig(**kw))
r.gbuffer()
r.frame()
torch.cuda.synchronize()
for _ in range(n):
    if what == "pass1":
        r.pass1()
    elif what == "pass2":
        r.pass2()
    elif what == "trace":
        r.clear_intervals()
        r.pass1()
        r.sd_trace()
    else:
        r.frame()
torch.cuda.synchronize()
print("ok", what, n, name)
