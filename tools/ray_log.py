"""Which live SD rays make the row walk long?  (diagnostics, GPU box)

One instrumented trace of a BASELINE config (fused row walk) with RSD_TRACE_RAYLOG: librsd writes
per live ray {texel, steps, nodes, leaves, keys found, clocks, TMax - TMin, TMin}.  Prints the clock
distribution and, per clock band, the mean steps / nodes / leaves / keys / interval length.
usage: python tools/ray_log.py [config] > ray_log.json"""
import json
import os
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ray-traced-stochastic-depth-map_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rsd.frame import CONFIGS, FrameConfig, Renderer  # noqa: E402
from rsd.scenes import make_scene  # noqa: E402


def main():
    name = next((a for a in sys.argv[1:] if not a.startswith("--")), "suntemple_1080p_q")
    kw, sc = CONFIGS[name]
    r = Renderer(make_scene(sc), FrameConfig(**kw))
    r.gbuffer()
    r.clear_intervals()
    r.pass1()
    path = os.path.join(tempfile.gettempdir(), "rsd_raylog.bin")
    os.environ["RSD_TRACE_RAYLOG"] = path
    c = r.sd_trace(counters=True)
    torch.cuda.synchronize()
    del os.environ["RSD_TRACE_RAYLOG"]
    lg = np.fromfile(path, np.uint32).reshape(-1, 8)
    lg = lg[lg[:, 1] > 0]  # slots a ray was walked in
    steps, nodes, leaves, found, clk = (lg[:, k].astype(np.float64) for k in (1, 2, 3, 4, 5))
    length, tmin = lg[:, 6].view(np.float32).astype(np.float64), lg[:, 7].view(np.float32).astype(np.float64)
    out = {"config": name, "walk": int(c.walk), "rays_logged": int(len(lg)),
           "clocks": {f"p{q}": float(np.percentile(clk, q)) for q in (50, 90, 99, 99.9, 100)}}
    order = np.argsort(clk)
    bands = {"all": order, "top1%": order[-max(1, len(order) // 100):], "top5%": order[-max(1, len(order) // 20):],
             "bottom50%": order[: len(order) // 2]}
    for b, idx in bands.items():
        out[b] = {"rays": int(len(idx)), "clocks": float(clk[idx].mean()), "steps": float(steps[idx].mean()),
                  "nodes": float(nodes[idx].mean()), "leaves": float(leaves[idx].mean()),
                  "keys": float(found[idx].mean()), "len": float(length[idx].mean()),
                  "len_rel": float((length[idx] / tmin[idx]).mean())}
    out["corr_clocks"] = {k: float(np.corrcoef(clk, v)[0, 1]) for k, v in
                          (("steps", steps), ("nodes", nodes), ("leaves", leaves), ("keys", found), ("len", length))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
