#!/usr/bin/env python3
"""Predicted per-rank frame time of the N > 1 band split (rsd/shard.py HaloFrame) from measurements
on ONE GPU (a model the driver's 8-GPU run can be judged against).

For a config and N in --worlds, on the real frame (fast numerics, the product default):

  * per rank k of HaloFrame's first (equal-groups) split: the GPU time of its pass 1
    (rsd_svao_pass1_rows), its SD trace given the 1-GPU interval union (its round-robin SD tiles,
    rsd_sd_trace_band_ex, or with --sd-split rows the rows under its band, rsd_sd_trace_rows) and its
    pass 2 given the 1-GPU SD map (rsd_svao_pass2_rows), each the median of --reps runs between
    fence-free HIP events, one launch in flight;
  * the bytes it sends per frame (sparse interval triples to the bands it touches, the depths it
    returns, its AO band), as tools/halo_plan.py computes them;
  * the host time of HaloFrame.front() + back() for that rank with the collectives stubbed out (the
    Python + torch + librsd issue cost of one frame; the results of those frames are not used).

Model (stated assumptions, checked by the driver's run): one frame in flight,
  T(N) = max_k (pass1_k + trace_k + pass2_k) + 4 x L_coll + max_k bytes_k / B_link
with L_coll = 12 us per small collective / point-to-point round (--coll-us) and B_link = 50 GB/s
per xGMI peer link (--link-gbs); with F frames in flight the GPU part overlaps across frames as at
N = 1 (factor --overlap = ms_per_step(F = 4) / one-frame GPU time, measured at N = 1 here), and the
frame rate is bounded by max(overlapped GPU time, host issue time).
Round 5: the product's clean SD tiles are on (Renderer.keep_clean_tiles; --no-clean-tiles: off), and the host issue
is also measured for the native band frame (rsd_band_frame over the null communicator, librsd's own accounting:
front + back minus the wait for the counts), the N > 1 path bench.py runs.
Round 6: the throughput region too: the 1-GPU ms_per_step (F frames in flight) and, per world, the
slowest rank's time per frame in flight measured alone on this GPU -> predicted_ms_per_step_us.
usage: python tools/scaling_model.py [config] [--worlds 2,4,8] [--reps 15] [--pose i] [--sd-split auto|tiles|rows]
       [--frames-in-flight 4]"""
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ray-traced-stochastic-depth-map_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from rsd.frame import CONFIGS, DEFAULT_CAMERA_PATH, FrameConfig, Renderer, camera_path  # noqa: E402
from rsd.scenes import make_scene  # noqa: E402
from rsd.shard import FLT_MAX_BITS, HaloFrame, NativeComm, NativeHaloFrame  # noqa: E402
from rsd.timing import TimingEvent  # noqa: E402


def arg(flag, default):
    return sys.argv[sys.argv.index(flag) + 1] if flag in sys.argv else default


name = next((a for a in sys.argv[1:] if not a.startswith("--") and a in CONFIGS), "suntemple_1080p_q")
worlds = [int(x) for x in arg("--worlds", "2,4,8").split(",")]
reps = int(arg("--reps", "15"))
pose = int(arg("--pose", "0"))
coll_us, link_gbs = float(arg("--coll-us", "12")), float(arg("--link-gbs", "50"))
sd_split = arg("--sd-split", "auto")  # HaloFrame's SD trace split: auto (its default), tiles or rows
kw, sc = CONFIGS[name]
r = Renderer(make_scene(sc), FrameConfig(**kw))
if "--no-clean-tiles" not in sys.argv:
    r.keep_clean_tiles()
poses = camera_path(DEFAULT_CAMERA_PATH.get(name, "static"))
if poses:
    r.set_pose(*poses[pose % len(poses)])
r.gbuffer()
N = r.cfg.sd_samples


def timed(fn, prep=None):
    ts = []
    for _ in range(reps):
        if prep:
            prep()
        a, b = TimingEvent(), TimingEvent()
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


# the 1-GPU frame: interval union, stencil, SD map
for _ in range(3):
    r.frame()
r.clear_intervals()
r.pass1()
torch.cuda.synchronize()
union = r.ray_minmax.clone()
r.sd_trace()
torch.cuda.synchronize()
sd_full = r.sd.clone()
one = {"pass1_us": timed(r.pass1, r.clear_intervals),
       "trace_us": timed(lambda: r.sd_trace(), lambda: r.ray_minmax.copy_(union)),
       "pass2_us": timed(r.pass2, lambda: (r.clear_intervals(), r.pass1()))}
one["gpu_us"] = one["pass1_us"] + one["trace_us"] + one["pass2_us"]


def one_gpu_throughput(F=4, n=60):
    """bench.py's N = 1 throughput region: rsd_svao_frame on F frame slots / streams, time per frame."""
    slots = []
    for j in range(F):
        rr = r if j == 0 else r.frame_slot()
        st = torch.cuda.current_stream() if j == 0 else torch.cuda.Stream()
        slots.append((rr, st))
    torch.cuda.synchronize()
    for rnd in (2 * F, n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(rnd):
            rr, st = slots[i % F]
            with torch.cuda.stream(st):
                rr.frame()
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


one["ms_per_step_us"] = round(one_gpu_throughput(int(arg("--frames-in-flight", "4"))), 1)
overlap = float(arg("--overlap", "0") or 0) or None

dist.get_backend = lambda pg=None: "gloo"  # plans only: no process group


class NoComm:
    """Collectives stubbed out: host issue cost only (frame results unused)."""
    nccl = False

    def all_gather(self, out, inp):
        out[0].copy_(inp.view(out[0].shape))

    def exchange(self, sends, recvs):
        pass


out = {"config": name, "sd_split": HaloFrame(r, 0, 2, rebalance=False, sd_split=sd_split).sd_split, "pose": pose,
       "reps": reps, "one_gpu": {k: round(v, 2) for k, v in one.items()},
       "assumptions": {"coll_us": coll_us, "link_gbs": link_gbs, "collectives_per_frame": 4}, "worlds": {}}
for world in worlds:
    plans = [HaloFrame(r, k, world, rebalance=False, sd_split=sd_split) for k in range(world)]
    ranks = []
    touched = []
    for k, p in enumerate(plans):
        r.clear_intervals()
        r.pass1_rows(p.px_rows[k])
        m = (r.ray_minmax[0] != FLT_MAX_BITS) | (r.ray_minmax[1] != 0)
        touched.append([sum(int(m[lo:hi].sum()) for lo, hi in p.owned_sd_rows(j)) if j != k else 0
                        for j in range(world)])
    for k, p in enumerate(plans):
        t1 = timed(lambda: r.pass1_rows(p.px_rows[k]), r.clear_intervals)
        r.sd.copy_(sd_full)
        r.invalidate_sd_tiles()
        t2 = timed(p.trace, lambda: r.ray_minmax.copy_(union))  # its SD tiles (or rows)
        r.sd.copy_(sd_full)
        r.invalidate_sd_tiles()
        t3 = timed(lambda: r.pass2_rows(p.px_rows[k]), lambda: (r.clear_intervals(), r.pass1()))
        iv = 12 * sum(touched[k])
        sdb = 4 * N * sum(touched[j][k] for j in range(world))
        ao = p.ao_max * r.ao[0].numel() * r.ao.element_size()
        ranks.append({"pass1_us": round(t1, 2), "trace_us": round(t2, 2), "pass2_us": round(t3, 2),
                      "gpu_us": round(t1 + t2 + t3, 2), "bytes": iv + sdb + ao,
                      "px_rows": p.px_rows[k], "sd_split": p.sd_split})
    # host issue of one rank's frame (rank 0 and the middle rank), collectives stubbed
    host = []
    for k in sorted({0, world // 2}):
        f = HaloFrame(r, k, world, rebalance=False, comm=NoComm(), sd_split=sd_split)
        for _ in range(3):
            f.front()
            f.back()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 20
        for _ in range(n):
            f.front()
            f.back()
        host.append((time.perf_counter() - t0) / n * 1e6)
        torch.cuda.synchronize()
    # the native band frame of the same ranks (bench.py's N > 1 path): librsd's host issue per frame, the time
    # its front() / back() calls spent minus their wait for the count matrix
    native = []
    for k in sorted({0, world // 2}):
        c = NativeComm.null(k, world)
        f = NativeHaloFrame(r, c, rebalance=False, sd_split=sd_split)
        for _ in range(23):
            f.front()
            f.back()
        torch.cuda.synchronize()
        st = f.stats()
        native.append((st.host_front_ns + st.host_back_ns - st.host_wait_ns) / st.frames * 1e-3)
        f.close()
        c.close()
    # round 6: the throughput region (bench.py's ms_per_step at N > 1), per rank ALONE on this GPU --
    # rank k's native band frame over the null communicator (its pass 1 rows, compaction, the trace of its share,
    # pass 2 of its rows; no exchange), F frame slots on F streams with back() lagging F - 1 fronts as bench.py
    # issues them; the slowest rank's time per frame bounds ms_per_step from below, and the exchange bytes over
    # one xGMI link (overlapped with the other frames' compute) from the side
    F = int(arg("--frames-in-flight", "4"))
    slowest = max(range(world), key=lambda k: ranks[k]["gpu_us"])
    thr = {}
    for k in sorted({0, world // 2, slowest}):
        c = NativeComm.null(k, world)
        slots = []
        for j in range(F):
            rr = r.frame_slot()
            st = torch.cuda.Stream()
            st.wait_stream(torch.cuda.current_stream())
            slots.append((rr, st, NativeHaloFrame(rr, c, throughput=True, rebalance=False, sd_split=sd_split)))
        torch.cuda.synchronize()

        def run(n):  # bench.py's native N > 1 loop: explicit streams, no torch stream contexts
            pending = []
            for i in range(n):
                rr, st, f = slots[i % F]
                f.front(stream=st.cuda_stream)
                pending.append(i)
                if len(pending) > F - 1:
                    j = pending.pop(0)
                    slots[j % F][2].back(stream=slots[j % F][1].cuda_stream)
            while pending:
                j = pending.pop(0)
                slots[j % F][2].back(stream=slots[j % F][1].cuda_stream)

        run(2 * F)
        torch.cuda.synchronize()
        n = 60
        t0 = time.perf_counter()
        run(n)
        torch.cuda.synchronize()
        thr[k] = (time.perf_counter() - t0) / n * 1e6
        for _, _, f in slots:
            f.close()
        c.close()
    r.invalidate_sd_tiles()
    gpu = max(x["gpu_us"] for x in ranks)
    xfer = max(x["bytes"] for x in ranks) / (link_gbs * 1e3)  # bytes / (GB/s) in us
    lat = gpu + 4 * coll_us + xfer
    out["worlds"][str(world)] = {
        "ranks": ranks, "max_rank_gpu_us": round(gpu, 2), "max_rank_bytes": max(x["bytes"] for x in ranks),
        "host_issue_us_per_frame": round(max(host), 1),
        "host_issue_native_us_per_frame": round(max(native), 1),
        "predicted_latency_us": round(lat, 1),
        "predicted_speedup_latency": round((one["gpu_us"]) / lat, 2),
        "rank_alone_us_per_frame_in_flight": {str(k): round(v, 1) for k, v in thr.items()},
        "predicted_ms_per_step_us": round(max(max(thr.values()), xfer), 1),
        "throughput_note": f"frames in flight (F = {F}): max(the slowest measured rank's time per frame alone on one "
                           "GPU -- its band frame over the null communicator, bench.py's lag schedule --, the "
                           "largest rank's exchange bytes / link bandwidth); collective latencies overlap the other "
                           "frames in flight",
        "note": "latency = max-rank GPU time + 4 collective latencies + max-rank bytes / link bandwidth; with "
                "frames in flight the frame interval is bounded below by the host issue (Python HaloFrame: "
                "host_issue_us_per_frame; the native band frame bench.py runs: host_issue_native_us_per_frame)"}
print(json.dumps(out))
