"""Time one rsd_sd_trace of a BASELINE config (diagnostics; env vars select the walk).
usage: python tools/sd_time.py [config] [--clean-tiles]"""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ray-traced-stochastic-depth-map_amd")]
import torch
from rsd.frame import CONFIGS, FrameConfig, Renderer
from rsd.scenes import make_scene

name = next((a for a in sys.argv[1:] if not a.startswith("--")), "suntemple_1080p_q")
kw, sc = CONFIGS[name]
r = Renderer(make_scene(sc), FrameConfig(**kw))
if "--clean-tiles" in sys.argv:  # the bench's SD maps (Renderer.keep_clean_tiles)
    r.keep_clean_tiles()
r.gbuffer()
r.clear_intervals()
r.pass1()
r.sd_trace()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(20):
    r.sd_trace()
e.record()
torch.cuda.synchronize()
print(name, "sd_trace ms", round(s.elapsed_time(e) / 20, 4))
