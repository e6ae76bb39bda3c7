"""Segment entry grid A/B (diagnostics, GPU box): the same frame traced with the entry grid on and
off (RSD_TRACE_ENTRY=off walks every ray from the root), for the row walk (one frame in flight)
and the quad walk (RSD_SD_THROUGHPUT).  Checks the SD maps are bit-identical, reports the
median trace time (7 batches of 40 launches, HIP events) and the traversal counters.
usage: python tools/entry_ab.py [config ...] > entry_ab.json"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ray-traced-stochastic-depth-map_amd")]
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


def main():
    names = [a for a in sys.argv[1:] if not a.startswith("--")] or ["suntemple_1080p_q"]
    out = {}
    for name in names:
        kw, sc = CONFIGS[name]
        r = Renderer(make_scene(sc), FrameConfig(**kw))
        r.gbuffer()
        r.clear_intervals()
        r.pass1()
        torch.cuda.synchronize()
        res = {"entry_cells": int(r.gscene.info.entry_cells), "build_ms": round(r.gscene.info.build_ms, 1)}
        maps = {}
        for mode in ("on", "off"):
            os.environ["RSD_TRACE_ENTRY"] = mode
            for walk, thr in (("row", False), ("quad", True)):
                c = r.sd_trace(counters=True, throughput=thr)
                torch.cuda.synchronize()
                maps[(mode, walk)] = r.sd.clone()
                act = max(int(c.rays_active), 1)
                res[f"{walk}_{mode}"] = {
                    "us": round(timeit(lambda: r.sd_trace(throughput=thr)), 2),
                    "rays_active": int(c.rays_active),
                    "nodes_per_active_ray": round(c.nodes_visited / act, 2),
                    "tris_per_active_ray": round(c.tris_tested / act, 2),
                    "max_steps_per_ray": int(c.max_steps_per_ray),
                    "leaves_per_active_ray": round(c.leaves_visited / act, 2),
                    "mean_ray_clocks": round(c.sum_ray_clocks / act, 1),
                    "max_ray_clocks": int(c.max_ray_clocks),
                    "walk": int(c.walk),
                }
        os.environ.pop("RSD_TRACE_ENTRY")
        ref = maps[("off", "row")].view(torch.int32)
        res["bit_identical"] = all(bool(torch.equal(m.view(torch.int32), ref)) for m in maps.values())
        out[name] = res
        r.close()
        torch.cuda.empty_cache()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
