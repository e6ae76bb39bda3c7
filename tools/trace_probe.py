"""Where does the SD trace's time go?  (diagnostics, GPU box)

configs[1] frame: pass 1 gives ~22 K live SD rays.  The trace is timed (HIP events, 20 launches)
with only a subset of the live texels kept live (the others' intervals emptied), from K = 0 (the
launch chain alone) over single rays to all of them -- separating the per-ray dependent chain from
contention between rays.  usage: python tools/trace_probe.py [config] > probe.json"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ray-traced-stochastic-depth-map_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rsd.frame import CONFIGS, FrameConfig, Renderer  # noqa: E402
from rsd.scenes import make_scene  # noqa: E402


def timeit(fn, n=40, batches=7):
    """median over `batches` of the mean launch time of n back-to-back calls (us)"""
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
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    name = args[0] if args else "suntemple_1080p_q"
    kw, sc = CONFIGS[name]
    r = Renderer(make_scene(sc), FrameConfig(**kw))
    r.gbuffer()
    r.clear_intervals()
    r.pass1()
    torch.cuda.synchronize()
    full = r.ray_minmax.clone()
    live = (full[1] != 0).flatten().nonzero().flatten()
    out = {"config": name, "live_texels": int(live.numel())}
    rng = np.random.default_rng(1)

    def keep(idx, throughput=False):
        r.ray_minmax.copy_(full)
        mask = torch.ones(r.sd_h * r.sd_w, dtype=torch.bool, device=full.device)
        mask[idx] = False
        r.ray_min.view(-1)[mask] = 0x7F7FFFFF
        r.ray_max.view(-1)[mask] = 0
        return timeit(lambda: r.sd_trace(throughput=throughput))

    out["all_us"] = keep(live)
    out["none_us"] = keep(live[:0])
    if "--tail" in sys.argv:  # drop the rays with the longest intervals: is the launch tail-bound?
        lo = full[0].flatten()[live].view(torch.float32)
        hi = full[1].flatten()[live].view(torch.float32)
        order = torch.argsort(hi - lo, descending=True)
        for frac in (0.001, 0.01, 0.05, 0.2):
            k = int(live.numel() * frac)
            out[f"drop_longest_{frac}"] = keep(live[order[k:]])
            out[f"drop_random_{frac}"] = keep(live[torch.randperm(live.numel(), device=live.device)[k:]])
        # rows of the queue in dequeue order: the longest rays first vs last (queue order = tile order)
    if "--counters" in sys.argv:  # instrumented trace: per-ray chain statistics (s_memtime cycles)
        def cnt(idx):
            keep(idx)
            c = r.sd_trace(counters=True)
            return {k: int(getattr(c, k)) for k, _ in c._fields_}
        out["counters_all"] = cnt(live)
        for k in (16, 2048):
            sel = live[torch.from_numpy(rng.choice(live.numel(), k, replace=False)).to(live.device)]
            out[f"counters_{k}"] = cnt(sel)
    if "--quick" in sys.argv:
        print(json.dumps(out))
        return
    out["all_quad_us"] = keep(live, throughput=True)
    subsets = {}
    for k in (1, 16, 256, 2048, 8192):
        sel = live[torch.from_numpy(rng.choice(live.numel(), k, replace=False)).to(live.device)]
        subsets[k] = keep(sel)
    out["subset_us"] = subsets
    # single rays: the per-ray dependent chain on an otherwise idle machine
    singles = []
    for i in rng.choice(live.numel(), 48, replace=False):
        singles.append(keep(live[int(i):int(i) + 1]))
    out["single_ray_us"] = {"min": min(singles), "median": float(np.median(singles)), "max": max(singles)}
    # the slowest single rays: rank texels by their traversal steps (instrumented trace, one at a time
    # is too slow) -- use the 256 texels with the largest TMax - TMin
    r.ray_minmax.copy_(full)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
