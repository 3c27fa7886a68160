"""GPU parity of the hot path's less common branches, each against the CPU oracle on the same
seeds (bars as in test_gpu_parity.py: RNG, hit points, grid, direct light bit-exact; indirect
rel-L2 <= 1e-5; output rel-L2 <= 1e-4; PT output bit-exact):

* thin-lens depth of field, camera.aperture > 0 (helpers/camera.h:11-27, used by
  RayGeneratorPPM.cu:49 and RayGeneratorPT.cu:61);
* spot lights: photon emission (PhotonGenerator.cu:73-78), direct light and PT next-event
  estimation (helpers/light.h:47-60), the constructor's by-value normalisation quirk
  (Light.cpp:39-49);
* imported scenes (scene/Scene.cpp:73-311, 487-565 restated in sceneio.py): an OBJ/MTL box with
  an emitter quad (PPM, PT, VCM), and a COLLADA scene with node transforms, a Glass material,
  an emitter mesh and a point light, with the reference's emitter double registration
  (Scene.cpp:141 + :508, duplicate_emitter_lights=True).
"""
import os
import tempfile

import numpy as np
import pytest

import oracle_lib
from oppositerenderer_amd import _abi, scenes, sceneio
from oppositerenderer_amd.renderer import next_ppm_radius
from test_gpu_parity import check_ppm_iteration, check_vcm_iteration, make_pair, rel_l2
from test_sceneio import BOX_MTL, BOX_OBJ, DAE

pytestmark = pytest.mark.gpu


def run_pair(scene, W, H, P, method, iters=2):
    gpu, ora, det = make_pair(scene, W, H, P, method)
    radius = scene.initial_ppm_radius()
    req = det.to_abi()
    for it in range(iters):
        gpu.renderNextIteration(it, it, radius, True, det)
        ora.render_next_iteration(it, it, radius, req)
        if method == _abi.PROGRESSIVE_PHOTON_MAPPING:
            check_ppm_iteration(gpu, ora)
        elif method == _abi.VCM_BIDIRECTIONAL_PATH_TRACING:
            check_vcm_iteration(gpu, ora)
        else:
            g, o = gpu.read_buffer(_abi.BUF_RNG, np.uint32), ora.read_buffer(_abi.BUF_RNG, np.uint32)
            assert np.array_equal(g, o)
        radius = next_ppm_radius(radius, it)
    g, o = gpu.getOutputBuffer(), ora.output()
    assert np.isfinite(g).all() and g.mean() > 0
    if method == _abi.PATH_TRACING:
        assert np.array_equal(g.view(np.uint32), o.view(np.uint32)), rel_l2(g, o)
    else:
        assert rel_l2(g, o) < 1e-4, rel_l2(g, o)
    gpu.destroy()
    ora.close()
    return g


@pytest.mark.parametrize("method", [_abi.PROGRESSIVE_PHOTON_MAPPING, _abi.PATH_TRACING])
def test_depth_of_field(method):
    scene = scenes.cornell()
    c = scene.default_camera
    scene.default_camera = scenes.Camera(c.eye, c.lookat, c.up, c.hfov, c.vfov, 12.0)
    img = run_pair(scene, 64, 48, 64, method)
    # the lens blurs: not the pinhole image
    scene.default_camera = c
    gpu, ora, det = make_pair(scene, 64, 48, 64, method)
    gpu.renderNextIteration(0, 0, scene.initial_ppm_radius(), True, det)
    assert not np.array_equal(gpu.getOutputBuffer(), img)
    gpu.destroy()
    ora.close()


def cornell_spot():
    """Cornell with its area light replaced by a spot light under the ceiling pointing down
    (the direction is deliberately not unit length: Light.cpp:41 normalises the by-value
    argument, so the member keeps it as given)."""
    sc = scenes.cornell()
    sc.name = "CornellSpot"
    sc.lights = [scenes.SpotLight(np.float32([4.0e5, 3.5e5, 3.0e5]), np.float32([278.0, 540.0, 279.5]),
                                  np.float32([0.1, -2.0, 0.05]), 50.0)]
    return sc


@pytest.mark.parametrize("method", [_abi.PROGRESSIVE_PHOTON_MAPPING, _abi.PATH_TRACING])
def test_spot_light(method):
    run_pair(cornell_spot(), 56, 48, 64, method)


def test_spot_light_vcm_is_rejected():
    """lightEmit (helpers/light.h:92-142) has no spot branch: VCM with a spot light is an error."""
    from oppositerenderer_amd.renderer import OrxError
    gpu, ora, det = make_pair(cornell_spot(), 32, 32, 32, _abi.VCM_BIDIRECTIONAL_PATH_TRACING)
    with pytest.raises(OrxError):
        gpu.renderNextIteration(0, 0, 1.0, True, det)
    gpu.destroy()
    ora.close()


def box_scene(**kw):
    d = tempfile.mkdtemp()
    with open(os.path.join(d, "box.mtl"), "w") as f:
        f.write(BOX_MTL)
    with open(os.path.join(d, "box.obj"), "w") as f:
        f.write(BOX_OBJ)
    sc = sceneio.load_scene(os.path.join(d, "box.obj"), **kw)
    sc.default_camera = scenes.Camera(np.float32([5, 4, -8]), np.float32([5, 4, 5]), np.float32([0, 1, 0]),
                                      50.0, 50.0, 0.0)
    return sc


@pytest.mark.parametrize("method", [_abi.PROGRESSIVE_PHOTON_MAPPING, _abi.PATH_TRACING,
                                    _abi.VCM_BIDIRECTIONAL_PATH_TRACING])
def test_imported_obj(method):
    run_pair(box_scene(), 48, 40, 64, method)


@pytest.mark.parametrize("duplicate", [False, True])
@pytest.mark.parametrize("method", [_abi.PROGRESSIVE_PHOTON_MAPPING, _abi.PATH_TRACING])
def test_imported_collada(method, duplicate):
    d = tempfile.mkdtemp()
    with open(os.path.join(d, "s.dae"), "w") as f:
        f.write(DAE)
    sc = sceneio.load_scene(os.path.join(d, "s.dae"), duplicate_emitter_lights=duplicate)
    assert len([l for l in sc.lights if l.type == _abi.LIGHT_AREA]) == (2 if duplicate else 1)
    # the file's camera looks down -z, away from the geometry: aim it at the scene
    sc.default_camera = scenes.Camera(np.float32([5, 4, -10]), np.float32([5, 2, 5]), np.float32([0, 1, 0]),
                                      45.0, 45.0, 0.0)
    run_pair(sc, 48, 36, 64, method)
