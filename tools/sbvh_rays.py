"""Live SD ray segments of a BASELINE config, computed on the CPU (oracle G-buffer -> pass 1 -> initRayDesc),
for the spatial-split BVH study (tools/sbvh_study.cpp).  No GPU.

usage: python tools/sbvh_rays.py [config] [out.npz]
The file holds the scene (positions, indices) and one row per live SD texel: o.xyz, d.xyz, TMin, TMax."""
import sys
import time

import numpy as np

sys.path[:0] = [".", "ray-traced-stochastic-depth-map_amd", "tests"]
import oracle.oracle as O  # noqa: E402  (study tool: the oracle is the CPU frame here, not a product path)
from helpers import to_oracle  # noqa: E402
from rsd.frame import CONFIGS, FrameConfig, make_camera, make_vao, sd_params, svao_params  # noqa: E402
from rsd.scenes import make_scene  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "suntemple_1080p_q"
out = sys.argv[2] if len(sys.argv) > 2 else f"/tmp/rays_{name}.npz"
kw, sc = CONFIGS[name]
cfg = FrameConfig(**kw)
scene = make_scene(sc)
cam = make_camera(scene, cfg)
vao, sdw, sdh = make_vao(cfg)
sdp = sd_params(cfg, vao.sdGuard)
svp = svao_params(cfg)
oc, ov, osd, osv = (to_oracle(cam, O.Camera), to_oracle(vao, O.VAOData), to_oracle(sdp, O.SDParams),
                    to_oracle(svp, O.SVAOParams))
t0 = time.time()
osc = O.Scene(scene.positions, scene.indices, scene.flags)
z, n = O.gbuffer(osc, oc, cfg.fb_w, cfg.fb_h, osd.cull_mode)
_, _, rmin, rmax = O.svao_pass1(oc, ov, osv, z, n, sdw, sdh)
ys, xs = np.nonzero(rmin != 0x7F7FFFFF)
rows = []
for y, x in zip(ys, xs):
    o, d, tmin, tmax, _ = O.sd_ray(oc, osd, z, rmin, rmax, sdw, sdh, int(x), int(y))
    if tmin <= tmax:
        rows.append([*o, *d, tmin, tmax])
rays = np.asarray(rows, np.float32)
print(f"{name}: {len(xs)} touched texels, {len(rays)} live rays, {time.time() - t0:.1f} s")
np.savez(out, positions=scene.positions.astype(np.float32), indices=scene.indices.astype(np.uint32), rays=rays)
