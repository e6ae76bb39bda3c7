"""How much of pass 2 is the launch over tiles with no stencilled pixel?  (diagnostics, GPU box)
Times pass 2 of a BASELINE config as rendered, then with the stencil zeroed (every workgroup only
loads its tile's stencil and exits), and reports the fraction of 16x16 tiles that have work.
usage: python tools/pass2_empty_probe.py [config]"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ray-traced-stochastic-depth-map_amd"), str(ROOT / "tools")]
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
st = r.stencil.cpu().numpy()
H, W = st.shape[:2]
t = 16
tiles = st[: H - H % t, : W - W % t].reshape(H // t, t, W // t, t, -1)
busy = float((tiles != 0).any(axis=(1, 3, 4)).mean())
out = {"config": name, "pass2_us": timeit(r.pass2), "busy_tile_frac": round(busy, 4),
       "stencil_pixel_frac": round(float((st != 0).any(axis=-1).mean() if st.ndim == 3 else (st != 0).mean()), 4)}
r.stencil.zero_()
out["pass2_empty_us"] = timeit(r.pass2)
print(json.dumps(out))
