"""Run one pass of the 1080p/4 frame in a loop (for rocprofv3 --pmc passes on the GPU box).
usage: python tools/pass_loop.py pass1|pass2|sd|frame [iterations]"""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ray-traced-stochastic-depth-map_amd")]
import torch  # noqa: E402
from rsd.frame import CONFIGS, FrameConfig, Renderer  # noqa: E402
from rsd.scenes import make_scene  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "pass1"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
kw, sc = CONFIGS["suntemple_1080p_q"]
r = Renderer(make_scene(sc), FrameConfig(**kw))
r.gbuffer()
r.frame()
torch.cuda.synchronize()
fn = {"pass1": r.pass1, "pass2": r.pass2, "sd": r.sd_trace, "frame": r.frame}[which]
for _ in range(n):
    fn()
torch.cuda.synchronize()
print("done", which, n)
