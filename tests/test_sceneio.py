"""Scene import: OBJ/MTL and COLLADA through the
restated Scene::createFromFile pipeline (scene/Scene.cpp:73-311), TGA/PIL
images (util/Image.cpp).  No reference asset exists here (README.md:15) and
assimp is absent: the files are written by these tests, so parity with
assimp's post-processing is unpinned; what is pinned is the reference's own
logic on top of it (material classification, emitter -> light, the AABB and
camera quirks)."""
import os
import tempfile

import numpy as np
import pytest

import oracle_lib
from oppositerenderer_amd import _abi, scenes, sceneio
from oppositerenderer_amd.renderer import next_ppm_radius

BOX_OBJ = """# cornell-like box, emitter quad under the ceiling
mtllib box.mtl
v 0 0 0
v 10 0 0
v 10 0 10
v 0 0 10
v 0 8 0
v 10 8 0
v 10 8 10
v 0 8 10
v 4 7.99 4
v 6 7.99 4
v 6 7.99 6
v 4 7.99 6
usemtl white
f 1 4 3 2
f 5 6 7 8
f 4 8 7 3
usemtl red
f 1 5 8 4
usemtl green
f 2 3 7 6
usemtl light
f 9 10 11 12
"""
BOX_MTL = """newmtl white
Kd 0.8 0.8 0.8
newmtl red
Kd 0.8 0.1 0.1
newmtl green
Kd 0.1 0.8 0.1
newmtl light
Kd 1 1 1
Ke 500 450 400
"""


def write(d, name, text):
    p = os.path.join(d, name)
    with open(p, "w") as f:
        f.write(text)
    return p


def render(sc, method, W=32, H=24, iters=2):
    r = oracle_lib.OracleRenderer(_abi.default_config(seed=1645301512, photon_launch_width=32,
                                                      photon_launch_height=32))
    r.init_scene(sc)
    req = _abi.OrxRequest()
    req.camera = sc.default_camera.set_aspect_ratio(W / H).to_abi()
    req.method, req.width, req.height, req.ppm_alpha = method, W, H, 2.0 / 3.0
    radius = sc.initial_ppm_radius()
    for it in range(iters):
        r.render_next_iteration(it, it, radius, req)
        radius = next_ppm_radius(radius, it)
    return r.output()


def test_tga_round_trip_and_reference_alpha():
    d = tempfile.mkdtemp()
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (5, 7, 4), dtype=np.uint8)
    sceneio.save_tga(os.path.join(d, "t.tga"), img)
    got = sceneio.load_tga(os.path.join(d, "t.tga"))
    assert got.shape == (5, 7, 4)
    assert np.array_equal(got[..., :3], img[..., :3])  # BGR(A) file bytes -> RGB
    assert (got[..., 3] == 1).all()                      # Image.cpp:105 alpha = 1


def test_tga_rejects_rle_and_colormap():
    d = tempfile.mkdtemp()
    p = os.path.join(d, "rle.tga")
    with open(p, "wb") as f:
        f.write(bytes([0, 0, 10] + [0] * 9 + [1, 0, 1, 0, 24, 0]) + bytes(3))
    with pytest.raises(ValueError, match="type '10'"):
        sceneio.load_tga(p)


def test_png_reference_channel_order():
    from PIL import Image
    d = tempfile.mkdtemp()
    img = np.zeros((2, 2, 4), np.uint8)
    img[..., 0], img[..., 1], img[..., 2], img[..., 3] = 10, 20, 30, 255
    Image.fromarray(img, "RGBA").save(os.path.join(d, "a.png"))
    ref = sceneio.load_image(os.path.join(d, "a.png"))
    assert tuple(ref[0, 0]) == (20, 10, 255, 30)  # QImage ARGB32 bytes 1,2,3,0 (Image.cpp:49-56)
    plain = sceneio.load_image(os.path.join(d, "a.png"), reference_channel_order=False)
    assert tuple(plain[0, 0]) == (10, 20, 30, 255)


def test_obj_box_materials_lights_aabb():
    d = tempfile.mkdtemp()
    write(d, "box.mtl", BOX_MTL)
    sc = sceneio.load_obj(write(d, "box.obj", BOX_OBJ))
    types = sorted(m.type for m in sc.materials)
    assert types == sorted([_abi.MAT_DIFFUSE] * 3 + [_abi.MAT_DIFFUSE_EMITTER])
    # loadMeshLightSource: first triangle of the emitter quad, power = Ke * Kd
    assert len(sc.lights) == 1
    L = sc.lights[0]
    np.testing.assert_array_equal(L.position, np.float32([4, 7.99, 4]))
    np.testing.assert_array_equal(L.v1, np.float32([2, 0, 0]))
    np.testing.assert_array_equal(L.v2, np.float32([2, 0, 2]))
    np.testing.assert_array_equal(L.power, np.float32([500, 450, 400]))
    em = [m for m in sc.materials if m.type == _abi.MAT_DIFFUSE_EMITTER][0]
    assert em.inverse_area == pytest.approx(L.inverse_area)
    # 6 quads triangulated as fans
    assert len(sc.triangles) == 12
    # the reference AABB uses the first corner of every face (Scene.cpp:151-153)
    firsts = sc.vertices[sc.triangles[:, 0]]
    np.testing.assert_array_equal(sc.aabb_min, firsts.min(axis=0))
    np.testing.assert_array_equal(sc.aabb_max, firsts.max(axis=0))
    # generated smooth normals are unit length
    assert np.allclose(np.linalg.norm(sc.normals, axis=1), 1, atol=1e-6)
    # emitters registered twice on request (Scene.cpp:141 + :508)
    sc2 = sceneio.load_obj(os.path.join(d, "box.obj"), duplicate_emitter_lights=True)
    assert len(sc2.lights) == 2


def test_obj_renders_with_every_method():
    d = tempfile.mkdtemp()
    write(d, "box.mtl", BOX_MTL)
    sc = sceneio.load_scene(write(d, "box.obj", BOX_OBJ))
    sc.default_camera = scenes.Camera(np.float32([5, 4, -8]), np.float32([5, 4, 5]), np.float32([0, 1, 0]),
                                      50.0, 50.0, 0.0)
    for method in (_abi.PROGRESSIVE_PHOTON_MAPPING, _abi.PATH_TRACING, _abi.VCM_BIDIRECTIONAL_PATH_TRACING):
        out = render(sc, method)
        assert np.isfinite(out).all() and out.mean() > 0, method


def test_obj_texture_material_and_tangents():
    d = tempfile.mkdtemp()
    rng = np.random.default_rng(1)
    sceneio.save_tga(os.path.join(d, "checker.tga"), rng.integers(0, 256, (8, 8, 4), dtype=np.uint8))
    sceneio.save_tga(os.path.join(d, "nrm.tga"), np.full((4, 4, 4), 128, np.uint8))
    write(d, "t.mtl", BOX_MTL + "newmtl tex\nmap_Kd checker.tga\nnorm nrm.tga\n")
    obj = BOX_OBJ.replace("usemtl white\nf 1 4 3 2\n", "usemtl tex\nvt 0 0\nvt 2 0\nvt 2 2\nvt 0 2\nf 1/1 4/2 3/3 2/4\nusemtl white\n")
    obj = obj.replace("mtllib box.mtl", "mtllib t.mtl")
    sc = sceneio.load_obj(write(d, "t.obj", obj))
    tex = [m for m in sc.materials if m.type == _abi.MAT_TEXTURE]
    assert len(tex) == 1 and len(sc.textures) == 1
    assert sc.textures[0].normal_rgba is not None
    assert sc.texcoords is not None and sc.tangents is not None
    # tangents on the textured floor follow +u (the x edge 1 -> 4 is z here: u grows along z)
    floor = sc.triangle_mat == sc.materials.index(tex[0])
    vi = np.unique(sc.triangles[floor])
    assert np.allclose(np.abs(sc.tangents[vi] @ np.float32([0, 0, 1])), 1, atol=1e-5)
    out = render(sc, _abi.PROGRESSIVE_PHOTON_MAPPING)
    assert np.isfinite(out).all()


DAE = """<?xml version="1.0" encoding="utf-8"?>
<COLLADA xmlns="http://www.collada.org/2005/11/COLLADASchema" version="1.4.1">
  <asset><up_axis>Y_UP</up_axis></asset>
  <library_effects>
    <effect id="white-fx"><profile_COMMON><technique sid="c"><lambert>
      <diffuse><color>0.7 0.7 0.7 1</color></diffuse></lambert></technique></profile_COMMON></effect>
    <effect id="glass-fx"><profile_COMMON><technique sid="c"><phong>
      <diffuse><color>1 1 1 1</color></diffuse>
      <index_of_refraction><float>1.5</float></index_of_refraction></phong></technique></profile_COMMON></effect>
    <effect id="light-fx"><profile_COMMON><technique sid="c"><lambert>
      <emission><color>100 100 100 1</color></emission>
      <diffuse><color>0.5 0.5 0.5 1</color></diffuse></lambert></technique></profile_COMMON></effect>
  </library_effects>
  <library_materials>
    <material id="white"><instance_effect url="#white-fx"/></material>
    <material id="glass"><instance_effect url="#glass-fx"/></material>
    <material id="light"><instance_effect url="#light-fx"/></material>
  </library_materials>
  <library_geometries>
    <geometry id="floor"><mesh>
      <source id="floor-pos"><float_array id="fa" count="12">0 0 0 1 0 0 1 0 1 0 0 1</float_array>
        <technique_common><accessor source="#fa" count="4" stride="3"/></technique_common></source>
      <vertices id="floor-v"><input semantic="POSITION" source="#floor-pos"/></vertices>
      <polylist material="m" count="1"><input semantic="VERTEX" source="#floor-v" offset="0"/>
        <vcount>4</vcount><p>0 3 2 1</p></polylist>
    </mesh></geometry>
  </library_geometries>
  <library_lights><light id="pl"><technique_common><point><color>5 6 7</color></point></technique_common></light></library_lights>
  <library_cameras><camera id="cam"><optics><technique_common><perspective><xfov>40</xfov></perspective></technique_common></optics></camera></library_cameras>
  <library_visual_scenes><visual_scene id="s">
    <node id="f1"><scale>10 1 10</scale><instance_geometry url="#floor"><bind_material><technique_common>
      <instance_material symbol="m" target="#white"/></technique_common></bind_material></instance_geometry></node>
    <node id="f2"><translate>0 3 0</translate><instance_geometry url="#floor"><bind_material><technique_common>
      <instance_material symbol="m" target="#glass"/></technique_common></bind_material></instance_geometry></node>
    <node id="em"><translate>4 7 4</translate><scale>2 1 2</scale><rotate>1 0 0 180</rotate>
      <instance_geometry url="#floor"><bind_material><technique_common>
      <instance_material symbol="m" target="#light"/></technique_common></bind_material></instance_geometry></node>
    <node id="lamp"><translate>5 6 5</translate><instance_light url="#pl"/></node>
    <node id="camnode"><translate>5 4 -10</translate><instance_camera url="#cam"/></node>
  </visual_scene></library_visual_scenes>
  <scene><instance_visual_scene url="#s"/></scene>
</COLLADA>
"""


def test_collada_transforms_materials_lights_camera():
    d = tempfile.mkdtemp()
    sc = sceneio.load_scene(write(d, "s.dae", DAE))
    kinds = sorted(m.type for m in sc.materials)
    assert kinds == sorted([_abi.MAT_DIFFUSE, _abi.MAT_GLASS, _abi.MAT_DIFFUSE_EMITTER])
    assert len(sc.triangles) == 6
    assert sc.vertices[:, 0].max() == pytest.approx(10.0)       # scaled floor
    assert (np.abs(sc.vertices[:, 1] - 3.0) < 1e-6).sum() == 4  # translated copy
    # one area light from the emitter (power = emission * Kd) + the point light
    area = [l for l in sc.lights if l.type == _abi.LIGHT_AREA]
    point = [l for l in sc.lights if l.type == _abi.LIGHT_POINT]
    assert len(area) == 1 and len(point) == 1
    np.testing.assert_allclose(area[0].power, [50, 50, 50])
    np.testing.assert_allclose(point[0].position, [5, 6, 5])
    # loadDefaultSceneCamera: fov = xfov(rad) * 365 / (2 pi), KeepHorizontal
    cam = sc.default_camera
    np.testing.assert_allclose(cam.eye, [5, 4, -10])
    np.testing.assert_allclose(cam.lookat, [5, 4, -11])
    assert cam.hfov == pytest.approx(40 * 365 / 360, rel=1e-5) and cam.aspect_mode == "KeepHorizontal"
    out = render(sc, _abi.PATH_TRACING)
    assert np.isfinite(out).all()


def test_synthetic_conference_scene():
    """Conference-class stand-in for configs[4]: ~331k triangles, two area
    lights registered once, a camera that sees lit geometry (oracle PT, tiny image)."""
    import numpy as np
    import oracle_lib
    from oppositerenderer_amd import _abi, scenes

    sc = scenes.scene_by_name("SyntheticConference")
    a = sc.to_abi()
    assert 320_000 <= a.n_triangles <= 340_000 and a.n_quads == 2 and len(sc.lights) == 2
    r = oracle_lib.OracleRenderer(_abi.default_config(seed=1645301512, photon_launch_width=16, photon_launch_height=16))
    oracle_lib.load().orc_set_threads(4)
    r.init_scene(sc)
    req = _abi.OrxRequest()
    req.camera = sc.default_camera.set_aspect_ratio(float(np.float32(32) / np.float32(18))).to_abi()
    req.method, req.width, req.height, req.ppm_alpha = _abi.PATH_TRACING, 32, 18, 2.0 / 3.0
    r.render_next_iteration(0, 0, sc.initial_ppm_radius(), req)
    img = r.output()
    assert np.isfinite(img).all() and (img.sum(-1) > 0).mean() > 0.3
