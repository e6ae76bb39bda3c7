"""Diagnostics only (not a benchmark): the throughput cost of each pass with 4 frames in flight,
measured by dropping one pass from every frame (its results are then wrong).  GPU box."""
import sys
import time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ray-traced-stochastic-depth-map_amd")]
import torch
from rsd.frame import CONFIGS, FrameConfig, Renderer
from rsd.scenes import make_scene
from rsd.shard import BandFrame

kw, sc = CONFIGS["suntemple_1080p_q"]
r = Renderer(make_scene(sc), FrameConfig(**kw))
r.gbuffer()
F = 4
slots = [r] + [r.frame_slot() for _ in range(F - 1)]
streams = [torch.cuda.Stream() for _ in range(F)]
for st in streams:
    st.wait_stream(torch.cuda.current_stream())


def run(label, drop=()):
    saved = {}
    for s in slots:
        for name in drop:
            saved[(id(s), name)] = getattr(s, name)
            setattr(s, name, lambda *a, **k: None)
    frames = [BandFrame(s, throughput=True) for s in slots]
    for i in range(40):
        with torch.cuda.stream(streams[i % F]):
            frames[i % F].frame()
    torch.cuda.synchronize()
    n = 400
    t0 = time.perf_counter()
    for i in range(n):
        with torch.cuda.stream(streams[i % F]):
            frames[i % F].frame()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n * 1e6
    for s in slots:
        for name in drop:
            setattr(s, name, saved[(id(s), name)])
    print(f"{label:28s} {dt:7.1f} us/frame", flush=True)


run("full frame")
run("without pass2", ("pass2",))
run("without sd_trace", ("sd_trace",))
run("without pass1", ("pass1",))
run("pass1 only", ("pass2", "sd_trace"))
