"""Run-to-run spread of the frames-in-flight region (diagnostics): bench.py's throughput loop (F slots
on F streams, K frames) repeated R times on one box, each repetition timed like bench.py (sync ->
wall -> sync) with a HIP event at the end of every frame, so a slow repetition shows whether it was
slow throughout (clock) or stalled somewhere (a gap).  usage: python tools/flight_probe.py [K] [R] [idle_s]"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ray-traced-stochastic-depth-map_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rsd.frame import CONFIGS, FrameConfig, Renderer  # noqa: E402
from rsd.scenes import make_scene  # noqa: E402
from rsd.shard import BandFrame  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
R = int(sys.argv[2]) if len(sys.argv) > 2 else 12
IDLE = float(sys.argv[3]) if len(sys.argv) > 3 else 0.05  # seconds of GPU idle between repetitions
kw, sc = CONFIGS["suntemple_1080p_q"]
r = Renderer(make_scene(sc), FrameConfig(**kw))
r.gbuffer()
F = 4
slots = [BandFrame(r, throughput=True)] + [BandFrame(r.frame_slot(), throughput=True) for _ in range(F - 1)]
streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(F - 1)]
for s in streams[1:]:
    s.wait_stream(streams[0])


def loop(n, evs=None):
    for i in range(n):
        with torch.cuda.stream(streams[i % F]):
            slots[i % F].frame()
            if evs is not None:
                evs[i].record()


loop(5)
torch.cuda.synchronize()
reps = []
for _ in range(R):
    start = torch.cuda.Event(enable_timing=True)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(K)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    start.record()
    loop(K, evs)
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ends = sorted(start.elapsed_time(e) for e in evs)
    gaps = np.diff([0.0] + ends)
    reps.append({"us_per_frame": round(wall / K * 1e6, 1), "issue_us": round(t_issue * 1e6, 1),
                 "gpu_span_us": round(ends[-1] * 1e3, 1), "first_end_us": round(ends[0] * 1e3, 1),
                 "max_gap_us": round(float(gaps.max()) * 1e3, 1)})
    time.sleep(IDLE)
w = np.array([x["us_per_frame"] for x in reps])
print(json.dumps({"K": K, "R": R, "idle_s": IDLE, "us_per_frame": {"min": float(w.min()), "median": float(np.median(w)),
                                                   "max": float(w.max())}, "reps": reps}))
