"""Participating medium on the device (k_ppm_eye<true>, k_ppm_photon<true>, orx_media.hip's
volumetric table, the DDA volumetric gather) against the oracle's restatement (parity unpinned
against the reference, which ships with ENABLE_PARTICIPATING_MEDIA 0 and holds no media fixture).

Bit-exact: RNG, hit points (the transmittances are the same fp32 operations), photon slots, the
volumetric photon table (per slot: the event count and the last event of the highest photon),
direct (zero).  The volumetric radiance sums the photons in the DDA's cell order on the device
and in slot order in the oracle: relative L2 <= 1e-5, like the indirect.
"""
import numpy as np
import pytest

import oracle_lib
from oppositerenderer_amd import _abi, scenes
from oppositerenderer_amd.renderer import OptixRenderer, RenderRequestDetails, next_ppm_radius

pytestmark = pytest.mark.gpu
SEED = 1645301512


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(((a - b) ** 2).sum()) / max(np.sqrt((b * b).sum()), 1e-30))


def pair(scene, W, H, P, **cfg):
    c = _abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P, enable_media=1,
                            max_photon_trace_depth=15, **cfg)
    gpu = OptixRenderer(c)
    gpu.initialize(0)
    gpu.initScene(scene)
    ora = oracle_lib.OracleRenderer(c)
    ora.init_scene(scene)
    cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
    det = RenderRequestDetails(cam, scene.name, _abi.PROGRESSIVE_PHOTON_MAPPING, W, H)
    return gpu, ora, det


def check(gpu, ora):
    for buf, dt in ((_abi.BUF_RNG, np.uint32), (_abi.BUF_HITPOINTS, np.uint32),
                    (_abi.BUF_VOLUMETRIC_PHOTONS, np.uint32), (_abi.BUF_DIRECT, np.uint32)):
        g, o = gpu.read_buffer(buf, dt), ora.read_buffer(buf, dt)
        assert g.shape == o.shape, buf
        mism = np.count_nonzero(g != o)
        assert mism == 0, f"buffer {buf}: {mism} of {g.size} words differ"
    # deposits: the valid slots (the oracle clears only power and position of the others)
    gs_, os_ = gpu.read_buffer(_abi.BUF_PHOTON_SLOTS).reshape(-1, 9), ora.read_buffer(_abi.BUF_PHOTON_SLOTS).reshape(-1, 9)
    valid = os_[:, 0:3].max(1) > 0
    assert np.array_equal(gs_[valid].view(np.uint32), os_[valid].view(np.uint32))
    assert not gs_[~valid].any()
    gv, ov = gpu.read_buffer(_abi.BUF_VOLUMETRIC), ora.read_buffer(_abi.BUF_VOLUMETRIC)
    assert rel_l2(gv, ov) <= 1e-5, rel_l2(gv, ov)
    gi, oi = gpu.read_buffer(_abi.BUF_INDIRECT), ora.read_buffer(_abi.BUF_INDIRECT)
    assert rel_l2(gi, oi) <= 1e-5, rel_l2(gi, oi)
    return float(np.abs(ov).sum())


@pytest.mark.parametrize("sigma_s,sigma_a,photon_map,W,H,P", [(0.001, 0.0, 0, 64, 64, 128),
                                                               (0.004, 0.001, 0, 96, 80, 96),
                                                               (0.004, 0.001, 2, 64, 48, 64)])
def test_media_parity_cornell(sigma_s, sigma_a, photon_map, W, H, P):
    sc = scenes.cornell_medium(sigma_s=sigma_s, sigma_a=sigma_a)
    gpu, ora, det = pair(sc, W, H, P, photon_map=photon_map)
    req = det.to_abi()
    r = sc.initial_ppm_radius()
    vol = []
    for it in range(4):
        gpu.renderNextIteration(it, it, r, True, det)
        ora.render_next_iteration(it, it, r, req)
        vol.append(check(gpu, ora))
        r = next_ppm_radius(r, it)
    assert vol[0] == 0 and vol[-1] > 0
    assert rel_l2(gpu.getOutputBuffer(), ora.output()) <= 1e-4
    gpu.destroy()
    ora.close()


def test_media_full_cornell_256():
    """Cornell + medium box at 256x256 with 256^2 photons (the reference's test block), two iterations"""
    sc = scenes.cornell_medium()
    gpu, ora, det = pair(sc, 256, 256, 256)
    req = det.to_abi()
    r = sc.initial_ppm_radius()
    for it in range(2):
        gpu.renderNextIteration(it, it, r, True, det)
        ora.render_next_iteration(it, it, r, req)
        check(gpu, ora)
        r = next_ppm_radius(r, it)
    assert rel_l2(gpu.getOutputBuffer(), ora.output()) <= 1e-4
    gpu.destroy()
    ora.close()


def test_media_unsupported_paths():
    sc = scenes.cornell_medium()
    c = _abi.default_config(seed=SEED, photon_launch_width=32, photon_launch_height=32, enable_media=1)
    gpu = OptixRenderer(c)
    gpu.initialize(0)
    gpu.initScene(sc)
    cam = sc.default_camera.set_aspect_ratio(1.0)
    for m in (_abi.PATH_TRACING, _abi.VCM_BIDIRECTIONAL_PATH_TRACING):
        with pytest.raises(Exception):
            gpu.renderNextIteration(0, 0, 1.0, True, RenderRequestDetails(cam, sc.name, m, 16, 16))
    gpu.destroy()
