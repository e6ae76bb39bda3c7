"""Diagnostics: frame throughput of different stream schedules for frames in flight (GPU box).
  S1 slot streams, slot 0 on torch's current stream (bench.py up to now)
  S2 slot streams, all fresh
  S3 pipeline: front (clear + pass 1) on NP 'pass-1 streams' (frame i -> i % NP), back (trace +
     pass 2) on NC 'chain streams' (frame i -> i % NC), ordered by events; slot i % F buffers;
     optionally the chain streams at high and the pass-1 streams at low stream priority."""
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
torch.cuda.synchronize()
MAXF = 8
bufs = [r] + [r.frame_slot() for _ in range(MAXF - 1)]


def timed(label, step, n=400, warm=40):
    for i in range(warm):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(warm, warm + n):
        step(i)
    torch.cuda.synchronize()
    print(f"{label:44s} {(time.perf_counter() - t0) / n * 1e6:7.1f} us/frame", flush=True)


def slot_sched(F, first_current):
    frames = [BandFrame(b, throughput=True) for b in bufs[:F]]
    sts = ([torch.cuda.current_stream()] if first_current else []) + \
          [torch.cuda.Stream() for _ in range(F - (1 if first_current else 0))]
    for s in sts:
        s.wait_stream(torch.cuda.current_stream())

    def step(i):
        with torch.cuda.stream(sts[i % F]):
            frames[i % F].frame()
    return step


def pipe_sched(F, NP, NC, prio=False):
    frames = [BandFrame(b, throughput=True) for b in bufs[:F]]
    lo, hi = torch.cuda.Stream.priority_range() if prio else (0, 0)
    P = [torch.cuda.Stream(priority=lo) for _ in range(NP)]   # pass 1: low priority
    C = [torch.cuda.Stream(priority=hi) for _ in range(NC)]   # trace + pass 2 chain: high
    for s in P + C:
        s.wait_stream(torch.cuda.current_stream())
    done = [None] * F

    def step(i):
        k = i % F
        p, c = P[i % NP], C[i % NC]
        with torch.cuda.stream(p):
            if done[k] is not None:
                p.wait_event(done[k])
            frames[k].front()
            e = torch.cuda.Event()
            e.record(p)
        with torch.cuda.stream(c):
            c.wait_event(e)
            frames[k].back()
            d = torch.cuda.Event()
            d.record(c)
            done[k] = d
    return step


print("priority range (low, high):", torch.cuda.Stream.priority_range(), flush=True)
timed("S2 F=4 slot streams, fresh", slot_sched(4, False))
for F, NP, NC in ((4, 1, 3), (6, 1, 3), (4, 2, 2), (6, 2, 2), (8, 2, 2), (6, 1, 2)):
    timed(f"S3 F={F} pipeline NP={NP} NC={NC} chain high prio", pipe_sched(F, NP, NC, prio=True))
