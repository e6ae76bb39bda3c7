"""Where pass 2's time goes (diagnostics): busy-tile / refined-pair statistics of a configs[1] frame
and the kernel time (HIP events, median of 60) with the busy-tile flags, without them, and with the
stencil cut to the first refined direction of each pixel.  usage: python tools/pass2_probe.py [config]"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ray-traced-stochastic-depth-map_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rsd import abi  # noqa: E402
from rsd.frame import CONFIGS, FrameConfig, Renderer  # noqa: E402
from rsd.scenes import make_scene  # noqa: E402

name = next((a for a in sys.argv[1:] if not a.startswith("--")), "suntemple_1080p_q")
kw, sc = CONFIGS[name]
r = Renderer(make_scene(sc), FrameConfig(**kw))
r.gbuffer()
r.clear_intervals()
r.pass1()
r.sd_trace()
torch.cuda.synchronize()
st = r.stencil.clone()
g = r.cfg.guard_band
s = st.cpu().numpy()[g:g + (r.cfg.visible_h + 31) // 32 * 32, g:r.cfg.fb_w - g].astype(np.uint32)
pairs = np.unpackbits(s.astype(np.uint8)[..., None], axis=-1).sum(-1)
th, tw = pairs.shape[0] // 16, (pairs.shape[1] + 15) // 16
pt = np.zeros((th, tw), np.int64)
for j in range(th):
    for i in range(tw):
        pt[j, i] = pairs[16 * j:16 * j + 16, 16 * i:16 * i + 16].sum()
busy = pt[pt > 0]


def timeit(prep, n=60):
    ts = []
    for _ in range(n):
        prep()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r.pass2()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return round(float(np.median(ts)), 2)


def restore(stencil=None, no_busy=False):
    """pass 1 again (the busy-tile list belongs to the pass 1 before each pass 2, svao.hip tile_gen;
    the SD map is unchanged), then optionally a different stencil / no busy tiles"""
    r.clear_intervals()
    r.pass1()
    if stencil is not None:
        r.stencil.copy_(stencil)
    if no_busy:
        r.tile_flags.zero_()


out = {"config": name, "tiles": int(pt.size), "busy_tiles": int(busy.size), "pairs": int(pairs.sum()),
       "stencilled_pixels": int((s != 0).sum()),
       "pairs_per_busy_tile": {"mean": round(float(busy.mean()), 1), "p50": int(np.median(busy)),
                               "p90": int(np.percentile(busy, 90)), "max": int(busy.max()),
                               "over_256": int((busy > 256).sum())}}
out["pass2_us_flags"] = timeit(restore)
svp_flags = r.svp
nf = abi.SVAOParams.from_buffer_copy(r.svp)
nf.tile_flags = None
r.svp = nf
out["pass2_us_no_flags"] = timeit(restore)
r.svp = svp_flags
# only the lowest refined direction of each pixel: the per-pair share of the time
st1 = torch.from_numpy((lambda a: a & (~a + 1))(st.cpu().numpy().astype(np.int32)).astype(np.uint8)).cuda()
out["pass2_us_one_dir_per_pixel"] = timeit(lambda: restore(st1))
out["pass2_us_no_busy_tiles"] = timeit(lambda: restore(no_busy=True))
print(json.dumps(out))
