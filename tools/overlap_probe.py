"""Which kernel slows pass 1 down when frames overlap?  Pass 1 of slot A runs on stream A
while stream B runs one kind of work of slot B repeatedly; pass 1's time is read from events on
stream A (GPU box; diagnostics only)."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ray-traced-stochastic-depth-map_amd")]
import torch
from rsd.frame import CONFIGS, FrameConfig, Renderer
from rsd.scenes import make_scene

kw, sc = CONFIGS["suntemple_1080p_q"]
a = Renderer(make_scene(sc), FrameConfig(**kw))
a.gbuffer()
b = a.frame_slot()
b.clear_intervals(); b.pass1(); b.sd_trace(); b.pass2()
torch.cuda.synchronize()
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()


def chain_trace():
    b.sd_trace()


def chain_pass2():
    b.pass2()


def run(label, work, reps_b=6, n=10):
    ts = []
    for _ in range(n):
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if work is not None:
            with torch.cuda.stream(sb):
                for _ in range(reps_b):
                    work()
        with torch.cuda.stream(sa):
            s.record()
            a.clear_intervals()
            a.pass1()
            e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    print(f"{label:28s} pass1 median {ts[len(ts) // 2] * 1e3:7.1f} us  min {ts[0] * 1e3:7.1f} us", flush=True)


def b_pass1():
    b.clear_intervals()
    b.pass1()


run("alone", None)
run("with B sd_trace", chain_trace)
run("with B sd_trace quad", lambda: b.sd_trace(throughput=True))
run("with B pass2", chain_pass2)
run("with B pass1", b_pass1, reps_b=1)
