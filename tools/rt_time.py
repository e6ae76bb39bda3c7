"""Time the Raytraced secondary mode (pass 1 + ray-traced pass 2) at a BASELINE config."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ray-traced-stochastic-depth-map_amd")]
import torch  # noqa: E402
from rsd import abi  # noqa: E402
from rsd.frame import CONFIGS, FrameConfig, Renderer  # noqa: E402
from rsd.scenes import make_scene  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "suntemple_1080p_q"
kw, sc = CONFIGS[name]
cfg = FrameConfig(**kw)
cfg.secondary = abi.DEPTH_RAYTRACED
r = Renderer(make_scene(sc), cfg)
r.gbuffer()
r.frame()
torch.cuda.synchronize()


def timeit(fn, n=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


print(name, "raytraced frame ms", round(timeit(r.frame), 4), "pass1 ms", round(timeit(r.pass1), 4),
      "pass2_raytraced ms", round(timeit(r.pass2_raytraced), 4))
