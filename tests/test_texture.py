"""Texture material on the CPU: the tex2D restatement (orx_detmath.h
orx_tex2d_linear) against an independent numpy statement of the CUDA
programming guide's linear-filtering rule, wrap-mode properties, and the
oracle rendering the TexturedRoom scene (every Texture.cu program) with each
method.  Parity of the sampler with NVIDIA hardware is unpinned (no CUDA
device or fixture exists here); GPU parity is tests/test_gpu_parity.py."""
import ctypes as C

import numpy as np
import pytest

import oracle_lib
from oppositerenderer_amd import _abi, scenes, synthetic
from oppositerenderer_amd.renderer import next_ppm_radius


def tex2d(img, u, v):
    lib = oracle_lib.load()
    lib.orc_tex2d.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_float, C.c_float, C.POINTER(C.c_float)]
    img = np.ascontiguousarray(img, np.uint8)
    out = (C.c_float * 4)()
    lib.orc_tex2d(img.ctypes.data, img.shape[1], img.shape[0], u, v, out)
    return np.array(out[:], np.float32)


def tex2d_numpy(img, u, v):
    """CUDA linear filtering, wrap addressing, normalised coordinates: 8-bit
    fractional weights, (1-a)(1-b)T00 + a(1-b)T10 + (1-a)bT01 + abT11."""
    h, w = img.shape[:2]
    f = np.float32
    u, v = f(u), f(v)
    uw, vw = f(u - np.floor(u)), f(v - np.floor(v))
    xb, yb = f(uw * f(w) - f(0.5)), f(vw * f(h) - f(0.5))
    i, j = int(np.floor(xb)), int(np.floor(yb))
    a = f(np.floor(f(f(xb - f(i)) * f(256)) + f(0.5)) / f(256))
    b = f(np.floor(f(f(yb - f(j)) * f(256)) + f(0.5)) / f(256))
    T = lambda ii, jj: img[jj % h, ii % w].astype(np.float32) / f(255)
    w00, w10, w01, w11 = f((f(1) - a) * (f(1) - b)), f(a * (f(1) - b)), f((f(1) - a) * b), f(a * b)
    return ((w00 * T(i, j) + w10 * T(i + 1, j)) + w01 * T(i, j + 1)) + w11 * T(i + 1, j + 1)


def test_tex2d_matches_cuda_rule():
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (7, 5, 4), dtype=np.uint8)
    for u, v in list(rng.uniform(-3, 3, (200, 2))) + [(0, 0), (1, 1), (0.5, 0.5), (-1e-9, 0.999999), (2.0, -2.0)]:
        got, ref = tex2d(img, u, v), tex2d_numpy(img, u, v)
        np.testing.assert_allclose(got, ref, rtol=0, atol=2e-7)


def test_tex2d_wrap_and_texel_centres():
    rng = np.random.default_rng(4)
    img = rng.integers(0, 256, (8, 16, 4), dtype=np.uint8)
    # texel centres return the texel exactly
    for x in range(16):
        for y in range(8):
            np.testing.assert_array_equal(tex2d(img, (x + 0.5) / 16, (y + 0.5) / 8), img[y, x] / np.float32(255))
    # integer shifts of the coordinates wrap
    for u, v in rng.uniform(0, 1, (50, 2)):
        np.testing.assert_array_equal(tex2d(img, u, v), tex2d(img, u + 3, v - 2))
    # non-finite coordinates do not read outside the image
    assert np.isfinite(tex2d(img, np.nan, np.inf)).all()


def test_texture_scene_validation():
    sc = synthetic.textured_room()
    sc.materials[0] = scenes.Texture(7)  # no such image
    r = oracle_lib.OracleRenderer(_abi.default_config(seed=1))
    with pytest.raises(RuntimeError):
        r.init_scene(sc)


@pytest.mark.parametrize("method", [_abi.PROGRESSIVE_PHOTON_MAPPING, _abi.PATH_TRACING,
                                    _abi.VCM_BIDIRECTIONAL_PATH_TRACING])
def test_oracle_renders_textured_room(method):
    sc = synthetic.textured_room()
    r = oracle_lib.OracleRenderer(_abi.default_config(seed=1645301512, photon_launch_width=48,
                                                      photon_launch_height=48))
    r.init_scene(sc)
    req = _abi.OrxRequest()
    req.camera = sc.default_camera.set_aspect_ratio(40 / 32).to_abi()
    req.method, req.width, req.height, req.ppm_alpha = method, 40, 32, 2.0 / 3.0
    radius = sc.initial_ppm_radius()
    for it in range(2):
        r.render_next_iteration(it, it, radius, req)
        radius = next_ppm_radius(radius, it)
    out = r.output()
    assert np.isfinite(out).all() and out.mean() > 0
    if method == _abi.PROGRESSIVE_PHOTON_MAPPING:
        hp = r.read_buffer(_abi.BUF_HITPOINTS).reshape(40 * 32, 13)
        flags = hp[:, 12].view(np.uint32)
        # the normal-mapped floor bends hitpoint normals away from +y
        pos, n = hp[:, 0:3], hp[:, 3:6]
        floor = ((flags & (1 << 27)) != 0) & (np.abs(pos[:, 1]) < 1e-3)  # PRD_HIT_NON_SPECULAR
        assert floor.sum() > 50
        assert np.allclose(np.linalg.norm(n[floor], axis=1), 1, atol=1e-5)
        assert (n[floor, 1] < 0.999).mean() > 0.3
