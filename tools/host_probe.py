"""Host-side cost of issuing frames (diagnostics): how long the Python + librsd host path takes to
enqueue the frames-in-flight loop of bench.py, per frame and per ABI call, against the GPU time per
frame.  If issuing a frame costs about as much host time as the GPU spends on it, the GPU starves.
usage: python tools/host_probe.py [config] [--frames N]

svao_frame_python_only is the same ctypes call with a description librsd rejects at once: the Python +
ctypes + current-stream part of svao_frame; the rest is librsd's host code and the HIP runtime's launch
path (tools/launch_floor.hip measures the runtime alone).  svao_frame issues 5 launches (interval clear,
pass 1, SD setup, walk, pass 2), svao_frame_cleared 4 (the previous trace consumed the intervals, the
bench's steady state)."""
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

name = next((a for a in sys.argv[1:] if not a.startswith("--")), "suntemple_1080p_q")
frames = int(sys.argv[sys.argv.index("--frames") + 1]) if "--frames" in sys.argv else 20
kw, sc = CONFIGS[name]
r = Renderer(make_scene(sc), FrameConfig(**kw))
r.gbuffer()
F = 4
slots = [BandFrame(r, throughput=True)] + [BandFrame(r.frame_slot(), throughput=True) for _ in range(F - 1)]
streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(F - 1)]
for s in streams[1:]:
    s.wait_stream(streams[0])


def loop(n):
    for i in range(n):
        with torch.cuda.stream(streams[i % F]):
            slots[i % F].frame()


loop(8)
torch.cuda.synchronize()
out = {"config": name, "frames": frames}
for n in (frames, 10 * frames):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loop(n)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out[f"issue_us_per_frame_{n}"] = round((t1 - t0) / n * 1e6, 1)
    out[f"wall_us_per_frame_{n}"] = round((t2 - t0) / n * 1e6, 1)
# per-call host cost (the GPU queue kept short: synchronize between batches)
from rsd import abi  # noqa: E402
import ctypes as C  # noqa: E402

null_desc = abi.FrameDesc()  # cam == NULL: rsd_svao_frame returns at its first check (no HIP call)
calls = {"svao_frame": lambda: r.svao_frame(throughput=True),
         "svao_frame_cleared": lambda: r.svao_frame(intervals_clear=True, throughput=True),
         # the host path around the C++ work: Python + ctypes marshalling + torch's current stream
         "svao_frame_python_only": lambda: abi.lib().rsd_svao_frame(C.byref(null_desc), 0, None, r.stream),
         "current_stream": lambda: r.stream, "frame_desc": r._frame_desc,
         "pass1": r.pass1,
         "sd_trace": lambda: r.sd_trace(throughput=True), "pass2": r.pass2,
         "stream_ctx": lambda: torch.cuda.stream(streams[1]).__enter__(), "event_record": lambda: torch.cuda.Event().record()}
for k, fn in calls.items():
    ts = []
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            fn()
        ts.append((time.perf_counter() - t0) / 10 * 1e6)
    torch.cuda.set_stream(streams[0])
    out[f"host_us_{k}"] = round(float(np.median(ts)), 1)
torch.cuda.synchronize()
print(json.dumps(out))
