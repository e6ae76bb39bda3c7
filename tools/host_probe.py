"""Diagnostics: is the frames-in-flight loop host-bound?  Times the host's launch loop alone
(no sync) against the wall time of the same frames (GPU box)."""
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
frames = [BandFrame(s, throughput=True) for s in slots]
sts = [torch.cuda.Stream() for _ in range(F)]
for s in sts:
    s.wait_stream(torch.cuda.current_stream())


def loop(n):
    for i in range(n):
        with torch.cuda.stream(sts[i % F]):
            frames[i % F].frame()


loop(40)
torch.cuda.synchronize()
for n in (400, 2000):
    t0 = time.perf_counter()
    loop(n)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"n={n}: host launch loop {(t1 - t0) / n * 1e6:.1f} us/frame, wall {(t2 - t0) / n * 1e6:.1f} us/frame",
          flush=True)
