"""Clean tiles (rsd_sd_params.d_tile_state, Renderer.keep_clean_tiles): the SD trace does not rewrite an 8x8 tile
it left at DEFAULT_DEPTH while the tile has no live ray.  The bar is the trace without it: every frame of a
moving camera gives the same SD map and AO bits, single-GPU and in the band frame whose re-splits move SD rows
between ranks.  A control shows the stores are really skipped (a map written behind librsd's back keeps the
foreign values until invalidate_sd_tiles())."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def bits(t):
    return np.ascontiguousarray(t.cpu().numpy()).view(np.uint32)


def _renderer(config):
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from rsd.frame import CONFIGS, FrameConfig, Renderer
    from rsd.scenes import make_scene
    kw, name = CONFIGS[config]
    return Renderer(make_scene(name), FrameConfig(**kw))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("config", ["suntemple_1080p_q", "bistro_1080p_full"])
def test_clean_tiles_equal_full_rewrite_along_camera_path(config):
    import torch
    from rsd.frame import camera_path
    r = _renderer(config)
    ref = r.frame_slot(own_gbuffer=True)   # every texel every frame
    cln = r.frame_slot(own_gbuffer=True)
    cln.keep_clean_tiles()
    poses = camera_path("orbit120")[::20]
    skipped = []
    for i, p in enumerate(poses):
        for s in (ref, cln):
            s.set_pose(*p)
            s.gbuffer()
            s.frame()
        torch.cuda.synchronize()
        assert np.array_equal(bits(cln.sd), bits(ref.sd)), f"pose {i}: SD map"
        assert torch.equal(cln.ao, ref.ao), f"pose {i}: AO"
        # the instrumented trace of the same pose reports the texels it did not rewrite
        cln.clear_intervals()
        cln.pass1()
        c = cln.sd_trace(counters=True)
        skipped.append(int(c.texels_clean))
        torch.cuda.synchronize()
        assert np.array_equal(bits(cln.sd), bits(ref.sd)), f"pose {i}: SD map (instrumented trace)"
    # after the first frame most tiles are clean (no live ray twice in a row)
    assert skipped[-1] > 0.3 * cln.sd_rays, skipped
    # a map written behind librsd's back keeps what was written in its clean tiles ...
    cln.sd.fill_(7.0)
    cln.frame()
    torch.cuda.synchronize()
    assert (cln.sd == 7.0).any()
    # ... until the stamps are voided: then the trace rewrites every tile
    cln.sd.fill_(7.0)
    cln.invalidate_sd_tiles()
    cln.frame()
    ref.frame()
    torch.cuda.synchronize()
    assert np.array_equal(bits(cln.sd), bits(ref.sd))
    r.close()


@pytest.mark.timeout(600)
def test_clean_tiles_band_frame_resplits():
    """4 rank threads (in-process communicator), SD rows split (a re-split moves SD rows between ranks), a moving
    camera: every rank's AO image equals the 1-GPU frame of the pose with clean tiles on."""
    import torch
    from rsd.frame import camera_path
    from rsd.shard import NativeComm, NativeHaloFrame, NativeHub
    r = _renderer("suntemple_1080p_q")
    poses = camera_path("orbit120")[:8]
    refs = []
    for p in poses:
        r.set_pose(*p)
        r.gbuffer()
        r.frame()
        refs.append(r.numpy()["ao"])
    world = 4
    hub = NativeHub(world)
    comms = [NativeComm.local(hub, k) for k in range(world)]
    slots = []
    for k in range(world):
        rr = r.frame_slot(own_gbuffer=True)
        rr.keep_clean_tiles()
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        slots.append((rr, st, NativeHaloFrame(rr, comms[k], sd_split="rows")))
    torch.cuda.synchronize()
    out, errors = {}, []

    def run(k):
        try:
            rr, st, f = slots[k]
            with torch.cuda.stream(st):
                for i, p in enumerate(poses):
                    rr.set_pose(*p)
                    rr.gbuffer()
                    f.frame()
                    out[(k, i)] = rr.ao.clone()
        except Exception:  # noqa: BLE001
            import traceback
            errors.append((k, traceback.format_exc()))

    threads = [threading.Thread(target=run, args=(k,)) for k in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=500)
    torch.cuda.synchronize()
    assert not errors, errors
    for k in range(world):
        for i in range(len(poses)):
            assert np.array_equal(out[(k, i)].cpu().numpy(), refs[i]), f"rank {k} pose {i}"
    for _, _, f in slots:
        f.close()
    for c in comms:
        c.close()
    hub.close()
    r.close()
