"""Per-step time split of the row walk (instrumented build, RSD_TRACE_PHASES=1 prints it): all live
rays of configs[1] vs small subsets of them.  Diagnostics (GPU box)."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ray-traced-stochastic-depth-map_amd")]
os.environ["RSD_TRACE_PHASES"] = "1"
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rsd.frame import CONFIGS, FrameConfig, Renderer  # noqa: E402
from rsd.scenes import make_scene  # noqa: E402

kw, sc = CONFIGS["suntemple_1080p_q"]
r = Renderer(make_scene(sc), FrameConfig(**kw))
r.gbuffer()
r.clear_intervals()
r.pass1()
torch.cuda.synchronize()
full = r.ray_minmax.clone()
live = (full[1] != 0).flatten().nonzero().flatten()
rng = np.random.default_rng(1)
for k in (live.numel(), 4096, 256, 1):
    sel = live[torch.from_numpy(rng.choice(live.numel(), k, replace=False)).to(live.device)]
    r.ray_minmax.copy_(full)
    mask = torch.ones(r.sd_h * r.sd_w, dtype=torch.bool, device=full.device)
    mask[sel] = False
    r.ray_min.view(-1)[mask] = 0x7F7FFFFF
    r.ray_max.view(-1)[mask] = 0
    torch.cuda.synchronize()
    print("rays", k, flush=True)
    c = r.sd_trace(counters=True)
    torch.cuda.synchronize()
    print(" steps max", c.max_steps_per_ray, "nodes", c.nodes_visited, "leaves", c.leaves_visited, flush=True)
