"""Participating medium (ENABLE_PARTICIPATING_MEDIA, orx_config.enable_media), on the CPU oracle.

The reference ships with ENABLE_PARTICIPATING_MEDIA 0 (config.h:29) and holds no media fixture, so
the restatement (oracle/orx_oracle.c trace_radiance / trace_photon / vol_resolve / vol_gather,
ParticipatingMedium.cu, AAB.cu, VolumetricPhotonSphere*.cu) is parity unpinned: these tests
check its invariants; tests/test_gpu_media.py holds the device to it.
"""
import numpy as np
import pytest

import oracle_lib
from oppositerenderer_amd import _abi, scenes
from oppositerenderer_amd.renderer import RenderRequestDetails, next_ppm_radius

SEED = 1645301512


def run(scene, W, H, P, iters, **cfg):
    c = _abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P, **cfg)
    ora = oracle_lib.OracleRenderer(c)
    ora.init_scene(scene)
    cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
    req = RenderRequestDetails(cam, scene.name, _abi.PROGRESSIVE_PHOTON_MAPPING, W, H).to_abi()
    r = scene.initial_ppm_radius()
    snaps = []
    for it in range(iters):
        ora.render_next_iteration(it, it, r, req)
        snaps.append({k: ora.read_buffer(b) for k, b in (("vol", _abi.BUF_VOLUMETRIC),
                                                         ("table", _abi.BUF_VOLUMETRIC_PHOTONS),
                                                         ("direct", _abi.BUF_DIRECT),
                                                         ("ind", _abi.BUF_INDIRECT),
                                                         ("hp", _abi.BUF_HITPOINTS))})
        r = next_ppm_radius(r, it)
    out = ora.output()
    ora.close()
    return snaps, out


def test_media_iterations():
    """iteration 0 has no volumetric table yet; then every slot's numDeposits counts its photons'
    scatter events, the eye pass gathers volumetric radiance, the direct pass takes no shadow
    samples (DirectRadianceEstimation.cu:54) and the indirect holds volumetricRadiance/emitted"""
    sc = scenes.cornell_medium(sigma_s=0.004)
    snaps, out = run(sc, 48, 40, 96, 3, enable_media=1, max_photon_trace_depth=15)
    assert np.all(np.isfinite(out))
    assert not snaps[0]["vol"].any()
    for s in snaps:
        t = s["table"].reshape(-1, 7)
        n = t[:, 6].copy().view(np.uint32)
        assert n.sum() > 0 and np.all((n > 0) == (t[:, :3].max(1) > 0))
        hp = s["hp"].reshape(-1, 13)
        flags = hp[:, 12].copy().view(np.uint32)
        ns = (flags & (1 << 27)) != 0
        assert not s["direct"].reshape(-1, 3)[ns].any()
    vol = snaps[2]["vol"].reshape(-1, 3)
    assert (vol > 0).any() and np.all(vol >= 0)
    # indirect = gathered + vol/emitted: pixels without a non-specular hit carry exactly vol/emitted
    hp = snaps[2]["hp"].reshape(-1, 13)
    ns = (hp[:, 12].copy().view(np.uint32) & (1 << 27)) != 0
    inv = np.float32(1) / np.float32(96 * 96)
    ind = snaps[2]["ind"].reshape(-1, 3)
    np.testing.assert_array_equal(ind[~ns], (np.float32(0) + vol[~ns] * inv).astype(np.float32))


def test_media_off_ignores_box():
    """enable_media = 0 renders the scene without its medium box bit-identically"""
    a = scenes.cornell_medium(glass_sphere=False)
    b = scenes.cornell()
    _, oa = run(a, 32, 32, 64, 2)
    _, ob = run(b, 32, 32, 64, 2)
    np.testing.assert_array_equal(oa, ob)


def test_media_thin_fog_eye_pass():
    """sigma -> 0: iteration 0's eye pass (no table yet, the RNG not yet touched by a photon pass)
    hits the clear scene's points, with the attenuation times a transmittance of ~1.  (The photon
    pass differs: every medium hit counts a photon depth, so the first surface hit inside the box
    already deposits and the photon map carries the direct light the zero-shadow-sample direct
    pass leaves out.)"""
    a = scenes.cornell_medium(sigma_s=1e-7, glass_sphere=False)
    snaps, _ = run(a, 32, 32, 64, 1, enable_media=1)
    snaps_b, _ = run(scenes.cornell(), 32, 32, 64, 1)
    ha, hb = snaps[0]["hp"].reshape(-1, 13), snaps_b[0]["hp"].reshape(-1, 13)
    # the walk restarts at the box (hit = (o + t0 d) + t1 d): the same points up to fp32 rounding
    np.testing.assert_allclose(ha[:, :3], hb[:, :3], atol=2e-3)
    np.testing.assert_array_equal(ha[:, 3:6], hb[:, 3:6])
    np.testing.assert_array_equal(ha[:, 12], hb[:, 12])
    np.testing.assert_allclose(ha[:, 6:9], hb[:, 6:9], rtol=1e-3)
    assert not snaps[0]["vol"].any()


def test_media_errors():
    sc = scenes.cornell_medium()
    c = _abi.default_config(seed=SEED, photon_launch_width=32, photon_launch_height=32, enable_media=1)
    ora = oracle_lib.OracleRenderer(c)
    ora.init_scene(sc)
    cam = sc.default_camera.set_aspect_ratio(1.0)
    for m in (_abi.PATH_TRACING, _abi.VCM_BIDIRECTIONAL_PATH_TRACING):
        req = RenderRequestDetails(cam, sc.name, m, 16, 16).to_abi()
        with pytest.raises(RuntimeError):
            ora.render_next_iteration(0, 0, 1.0, req)
    ora.close()
    two = scenes.cornell_medium()
    two.add_medium_box((0, 0, 0), (1, 1, 1), 0.1, 0.0)
    ora = oracle_lib.OracleRenderer(c)
    with pytest.raises(RuntimeError):
        ora.init_scene(two)
    ora.close()
