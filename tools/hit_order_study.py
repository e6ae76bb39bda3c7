"""How far is the canonical any-hit order from a DXR-like traversal order?  

For BASELINE configs[1] and configs[2] (GPU box): the same frame traced with
RSD_HIT_ORDER_CANONICAL and RSD_HIT_ORDER_TRAVERSAL (Default reservoir, the headline setting),
then pass 2 on each SD map.  Reports the SD-map differences over the live texels and the AO
difference over the visible region against SURVEY 8(c)'s image tolerance (mean |dAO| <= 1/255,
|dAO| <= 2/255 on >= 99.5 % of the pixels), plus the same for KBuffer (whose N nearest hits do
not depend on the order unless MAX_COUNT truncates the stream).
usage: python tools/hit_order_study.py [--order traversal|wavefront] > profiles/roundN/hit_order_study.json
(--order wavefront: RSD_HIT_ORDER_WAVEFRONT, round 5, instead of the depth-first order)"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ray-traced-stochastic-depth-map_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rsd.frame import CONFIGS, FrameConfig, Renderer  # noqa: E402
from rsd.scenes import make_scene  # noqa: E402


def frame(scene, kw, impl, order):
    r = Renderer(scene, FrameConfig(**kw, implementation=impl, hit_order=order))
    r.gbuffer()
    r.frame()
    g = r.numpy()
    r.close()
    return g, r.cfg


def main():
    order = 2 if "wavefront" in sys.argv else 1
    out = {"tolerance": {"ao_mae_max": 1 / 255, "ao_abs_le_2_over_255_min_frac": 0.995},
           "order": {1: "traversal (depth-first)", 2: "wavefront"}[order]}
    for config in ("suntemple_1080p_q", "bistro_1080p_full"):
        kw, name = CONFIGS[config]
        scene = make_scene(name)
        for impl, iname in ((0, "Default"), (3, "KBuffer")):
            a, cfg = frame(scene, kw, impl, 0)
            b, _ = frame(scene, kw, impl, order)
            live = a["ray_max"] != 0
            da, db = a["sd"].view(np.uint32), b["sd"].view(np.uint32)
            texel_diff = (da != db).any(axis=-1).any(axis=0)  # [sdH, sdW]
            sample_diff = np.abs(a["sd"] - b["sd"])[:, live]
            g = cfg.guard_band
            vis = (slice(g, cfg.fb_h - g), slice(g, cfg.fb_w - g))
            dao = np.abs(a["ao"][vis].astype(np.int32) - b["ao"][vis].astype(np.int32))
            out[f"{config}/{iname}"] = {
                "live_texels": int(live.sum()),
                "live_texels_differing": int(texel_diff[live].sum()),
                "live_texels_differing_frac": round(float(texel_diff[live].mean()), 5),
                "sd_sample_mean_abs_diff": float(sample_diff.mean()),
                "ao_mae_255": round(float(dao.mean()), 5),
                "ao_frac_within_2_255": round(float((dao <= 2).mean()), 6),
                "ao_max_abs_255": int(dao.max()),
                "within_tolerance": bool(dao.mean() <= 1.0 and (dao <= 2).mean() >= 0.995),
            }
            torch.cuda.empty_cache()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
