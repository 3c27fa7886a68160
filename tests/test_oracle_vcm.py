"""CPU checks of the VCM restatement (oracle/orx_oracle_vcm.c.inc): determinism,
finiteness, the light-vertex cache invariants, error paths."""
import numpy as np
import pytest

import oracle_lib
from oppositerenderer_amd import _abi, scenes

SEED = 1645301512


def run(scene, W, H, iters, radius=0.05):
    cfg = _abi.default_config(seed=SEED, photon_launch_width=32, photon_launch_height=32)
    r = oracle_lib.OracleRenderer(cfg)
    r.init_scene(scene)
    req = _abi.OrxRequest()
    req.camera = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H))).to_abi()
    req.method = _abi.VCM_BIDIRECTIONAL_PATH_TRACING
    req.width, req.height, req.ppm_alpha = W, H, 2.0 / 3.0
    for it in range(iters):
        r.render_next_iteration(it, it, radius, req)
    return r


@pytest.mark.parametrize("name", ["Cornell", "CornellSmallLargeSphere", "CornellSmallSmallSpheres"])
def test_vcm_oracle_deterministic_and_finite(name):
    sc = scenes.scene_by_name(name)
    a = run(sc, 24, 20, 2)
    b = run(sc, 24, 20, 2)
    for buf in (_abi.BUF_RNG, _abi.BUF_VCM_CAMERA, _abi.BUF_VCM_VERTEX_COUNT):
        assert np.array_equal(a.read_buffer(buf, np.uint32), b.read_buffer(buf, np.uint32))
    out = a.output()
    assert np.isfinite(out).all() and out.min() >= 0 and out.max() > 0
    # splats are order-dependent sums, everything else is exact
    np.testing.assert_allclose(a.read_buffer(_abi.BUF_VCM_SPLAT), b.read_buffer(_abi.BUF_VCM_SPLAT), rtol=1e-5,
                               atol=1e-7)
    a.close()
    b.close()


def test_vcm_light_vertex_cache_invariants():
    """Stored vertices sit on non-specular surfaces (Diffuse/Glossy materials),
    at most VCM_MAX_PATH_LENGTH-1 per subpath, with finite positive throughput."""
    sc = scenes.scene_by_name("CornellSmallSmallSpheres")
    r = run(sc, 32, 32, 1)
    cnt = r.read_buffer(_abi.BUF_VCM_VERTEX_COUNT, np.uint32)
    assert cnt.max() <= 9 and cnt.mean() > 0.5
    v = r.read_buffer(_abi.BUF_VCM_VERTICES).reshape(9, -1, 16)
    valid = np.arange(9)[:, None] < cnt[None, :]
    sel = v[valid]
    mats = sel[:, 3].view(np.uint32)
    types = np.array([m.type for m in sc.materials])
    assert set(types[mats]) <= {_abi.MAT_DIFFUSE, _abi.MAT_GLOSSY}
    thr = sel[:, 4:7]
    assert np.isfinite(thr).all() and (thr >= 0).all()
    n = sel[:, 8:11]
    np.testing.assert_allclose(np.linalg.norm(n, axis=1), 1.0, atol=1e-5)
    assert (sel[:, 14] > 0).all()  # localDirFix.z = cos to the incoming direction
    r.close()


def test_vcm_spot_light_rejected():
    sc = scenes.cornell()
    sc.lights[0] = scenes.SpotLight((1.0, 1.0, 1.0), (278.0, 500.0, 279.5), (0.0, -1.0, 0.0), 30.0)
    with pytest.raises(RuntimeError, match="spot"):
        run(sc, 8, 8, 1)
