"""Bytes of the sparse band split (rsd/shard.py HaloFrame) per rank and frame, computed from a real
frame on ONE GPU: for each rank of a B-way split, pass 1 of its rows alone (rsd_svao_pass1_rows) gives
exactly the SD texels it touches, hence what it sends (12 B per touched texel of another band) and
what it gets back (4 N B per texel); the dense round-2 halo (whole candidate rows) and the SD map
are printed beside it.  usage: python tools/halo_plan.py [config] [--pose i] [--worlds 2,4,8]"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ray-traced-stochastic-depth-map_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from rsd.frame import CONFIGS, DEFAULT_CAMERA_PATH, FrameConfig, Renderer, camera_path  # noqa: E402
from rsd.scenes import make_scene  # noqa: E402
from rsd.shard import FLT_MAX_BITS, HaloFrame  # noqa: E402

name = next((a for a in sys.argv[1:] if not a.startswith("--") and a in CONFIGS), "bistro_4k_full_n16")
pose = int(sys.argv[sys.argv.index("--pose") + 1]) if "--pose" in sys.argv else 0
worlds = [int(x) for x in (sys.argv[sys.argv.index("--worlds") + 1] if "--worlds" in sys.argv else "2,4,8").split(",")]
kw, sc = CONFIGS[name]
r = Renderer(make_scene(sc), FrameConfig(**kw))
poses = camera_path(DEFAULT_CAMERA_PATH.get(name, "static"))
if poses:
    r.set_pose(*poses[pose % len(poses)])
r.gbuffer()
N = r.cfg.sd_samples
sd_map_bytes = r.sd.numel() * r.sd.element_size()
dist.get_backend = lambda pg=None: "gloo"  # plans only: no process group
out = {"config": name, "pose": pose, "sd_map_bytes": sd_map_bytes, "sd_map": [r.sd_w, r.sd_h], "N": N, "worlds": {}}
for world in worlds:
    plans = [HaloFrame(r, k, world) for k in range(world)]
    touched = []  # touched[k][j]: texels of band j touched by rank k's pass 1
    for k, p in enumerate(plans):
        r.clear_intervals()
        r.pass1_rows(p.px_rows[k])
        m = (r.ray_minmax[0] != FLT_MAX_BITS) | (r.ray_minmax[1] != 0)
        touched.append([sum(int(m[lo:hi].sum()) for lo, hi in p.owned_sd_rows(j)) if j != k else 0
                        for j in range(world)])
    torch.cuda.synchronize()
    ranks = []
    for k, p in enumerate(plans):
        iv = 12 * sum(touched[k])                                  # (index, rayMin, rayMax) to band j
        sd = 4 * N * sum(touched[j][k] for j in range(world))       # depths returned to the requesters
        ao = p.ao_max * r.ao[0].numel() * r.ao.element_size()
        dense = p.dense_bytes_per_frame()
        ranks.append({"intervals": iv, "sd": sd, "ao": ao, "sparse_total": iv + sd + ao,
                      "dense_intervals": dense["intervals"], "dense_sd": dense["sd"],
                      "dense_total": dense["intervals"] + dense["sd"] + dense["ao"]})
    worst = max(x["sparse_total"] for x in ranks)
    out["worlds"][str(world)] = {"ranks": ranks, "max_rank_sparse_bytes": worst,
                                 "max_rank_sparse_frac_of_sd_map": round(worst / sd_map_bytes, 4),
                                 "max_rank_dense_bytes": max(x["dense_total"] for x in ranks),
                                 "max_rank_dense_frac_of_sd_map": round(max(x["dense_total"] for x in ranks)
                                                                        / sd_map_bytes, 4),
                                 "all_ranks_sparse_bytes": sum(x["sparse_total"] for x in ranks)}
print(json.dumps(out))
