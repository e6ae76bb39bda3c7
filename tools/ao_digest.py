"""SHA-256 of one frame's AO, stencil and interval maps (A/B builds must agree bit for bit):
python tools/ao_digest.py [config]"""
import hashlib
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ray-traced-stochastic-depth-map_amd")]
import torch  # noqa: E402

from rsd.frame import CONFIGS, FrameConfig, Renderer  # noqa: E402
from rsd.scenes import make_scene  # noqa: E402

name = next((a for a in sys.argv[1:] if not a.startswith("--")), "suntemple_1080p_q")
kw, sc = CONFIGS[name]
r = Renderer(make_scene(sc), FrameConfig(**kw))
r.gbuffer()
r.clear_intervals()
r.pass1()
torch.cuda.synchronize()
iv = r.ray_minmax.clone()
r.sd_trace()
r.pass2()
torch.cuda.synchronize()
h = lambda t: hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest()[:16]  # noqa: E731
print(json.dumps({"config": name, "ao": h(r.ao), "stencil": h(r.stencil), "intervals": h(iv)}))
