"""Scenes as flat primitive lists for the orx C ABI.

Replaces the reference's IScene implementations (RenderEngine/scene/IScene.h:16-29):
`getSceneRootGroup` built an OptiX node graph; here a scene is arrays of
parallelograms / spheres / triangles plus materials and lights, which
`orx_init_scene` deep-copies to the device.  Scalar arithmetic that the
reference performs in fp32 on the host (e.g. the `/ 220.f` block scaling in
CornellSmall.cpp) is reproduced in numpy float32 so both the renderer and
the oracle receive identical inputs.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field

import numpy as np

from . import _abi

f32 = np.float32


def _v(x, y, z):
    return np.array([x, y, z], dtype=np.float32)


def _vdiv_scalar(v, s):
    """optix float3 / float = v * (1.0f / s) (optixu_math_namespace.h)."""
    inv = f32(1.0) / f32(s)
    return (np.asarray(v, dtype=np.float32) * inv).astype(np.float32)


@dataclass
class Camera:
    """Camera inputs (renderer/Camera.h:72-79)."""
    eye: np.ndarray
    lookat: np.ndarray
    up: np.ndarray
    hfov: float = 60.0
    vfov: float = 60.0
    aperture: float = 0.0
    aspect_mode: str = "KeepVertical"

    def set_aspect_ratio(self, ratio):
        """Camera::setAspectRatio (renderer/Camera.cpp:294-318), in float32."""
        dtor = lambda d: f32(d) * (f32(math.pi) / f32(180.0))
        rtod = lambda r: f32(r) * (f32(180.0) / f32(math.pi))
        if self.aspect_mode == "KeepHorizontal":
            inp, real = self.hfov, f32(1.0) / f32(ratio)
            self.vfov = float(rtod(f32(2.0) * f32(math.atan(float(real * f32(math.tan(float(dtor(f32(0.5) * f32(inp))))))))))
        elif self.aspect_mode == "KeepVertical":
            inp, real = self.vfov, f32(ratio)
            self.hfov = float(rtod(f32(2.0) * f32(math.atan(float(real * f32(math.tan(float(dtor(f32(0.5) * f32(inp))))))))))
        return self

    def to_abi(self):
        c = _abi.OrxCamera()
        c.eye[:] = [float(v) for v in self.eye]
        c.lookat[:] = [float(v) for v in self.lookat]
        c.up[:] = [float(v) for v in self.up]
        c.hfov, c.vfov, c.aperture = float(self.hfov), float(self.vfov), float(self.aperture)
        return c


@dataclass
class Material:
    type: int
    Kd: tuple = (0.0, 0.0, 0.0)
    Ks: tuple = (0.0, 0.0, 0.0)
    Kr: tuple = (0.0, 0.0, 0.0)
    Kt: tuple = (0.0, 0.0, 0.0)
    ior: float = 1.0
    exponent: float = 1.0
    power: tuple = (0.0, 0.0, 0.0)
    inverse_area: float = 0.0
    texture: int = -1

    def to_abi(self):
        m = _abi.OrxMaterial()
        m.type = self.type
        m.Kd[:] = [float(v) for v in self.Kd]
        m.Ks[:] = [float(v) for v in self.Ks]
        m.Kr[:] = [float(v) for v in self.Kr]
        m.Kt[:] = [float(v) for v in self.Kt]
        m.ior, m.exponent = float(self.ior), float(self.exponent)
        m.power[:] = [float(v) for v in self.power]
        m.inverse_area = float(self.inverse_area)
        m.texture = int(self.texture)
        return m


@dataclass
class TextureImage:
    """Texture's diffuse map and optional normal map (material/Texture.cpp:18-29,
    util/Image.cpp): uint8 [h, w, 4] RGBA, row 0 first."""
    rgba: np.ndarray
    normal_rgba: np.ndarray | None = None


def Diffuse(Kd):
    return Material(_abi.MAT_DIFFUSE, Kd=tuple(np.broadcast_to(np.float32(Kd), 3)))


def Mirror(Kr):
    return Material(_abi.MAT_MIRROR, Kr=tuple(np.broadcast_to(np.float32(Kr), 3)))


def Glass(ior, Kr, Kt):
    return Material(_abi.MAT_GLASS, ior=float(f32(ior)), Kr=tuple(np.broadcast_to(np.float32(Kr), 3)),
                    Kt=tuple(np.broadcast_to(np.float32(Kt), 3)))


def Glossy(Kd, Ks, exponent):
    return Material(_abi.MAT_GLOSSY, Kd=tuple(np.broadcast_to(np.float32(Kd), 3)),
                    Ks=tuple(np.broadcast_to(np.float32(Ks), 3)), exponent=float(exponent))


def Texture(texture_index):
    """Texture material: Lambertian with Kd = tex2D(diffuseSampler, uv) (Texture.cu:83-110)."""
    return Material(_abi.MAT_TEXTURE, texture=int(texture_index))


def DiffuseEmitter(power, Kd, inverse_area):
    return Material(_abi.MAT_DIFFUSE_EMITTER, power=tuple(np.float32(power)),
                    Kd=tuple(np.broadcast_to(np.float32(Kd), 3)), inverse_area=float(inverse_area))


@dataclass
class Light:
    type: int
    power: np.ndarray
    position: np.ndarray
    v1: np.ndarray = field(default_factory=lambda: _v(0, 0, 0))
    v2: np.ndarray = field(default_factory=lambda: _v(0, 0, 0))
    direction: np.ndarray = field(default_factory=lambda: _v(0, 0, 0))
    angle: float = 0.0

    @property
    def inverse_area(self):
        """Light::Light area ctor (renderer/Light.cpp:14-28): 1/|v1 x v2| in fp32."""
        v1, v2 = self.v1.astype(np.float32), self.v2.astype(np.float32)
        c = np.array([v1[1] * v2[2] - v1[2] * v2[1], v1[2] * v2[0] - v1[0] * v2[2],
                      v1[0] * v2[1] - v1[1] * v2[0]], dtype=np.float32)
        d = f32(c[0] * c[0]) + f32(c[1] * c[1])
        d = f32(d + f32(c[2] * c[2]))
        area = np.sqrt(d, dtype=np.float32)
        return float(f32(1.0) / area)

    def to_abi(self):
        l = _abi.OrxLight()
        l.type = self.type
        for name in ("power", "position", "v1", "v2", "direction"):
            getattr(l, name)[:] = [float(v) for v in getattr(self, name)]
        l.angle = float(self.angle)
        return l


def AreaLight(power, anchor, v1, v2):
    return Light(_abi.LIGHT_AREA, np.float32(power), np.float32(anchor), np.float32(v1), np.float32(v2))


def PointLight(power, position):
    return Light(_abi.LIGHT_POINT, np.broadcast_to(np.float32(power), 3).copy(), np.float32(position))


def SpotLight(power, position, direction, angle):
    """Light::Light spot ctor (renderer/Light.cpp:39-49); angle in degrees."""
    return Light(_abi.LIGHT_SPOT, np.broadcast_to(np.float32(power), 3).copy(), np.float32(position),
                 direction=np.float32(direction), angle=float(angle))


class Scene:
    """Flat scene: what IScene::getSceneRootGroup + getSceneLights + getSceneAABB
    hand to OptixRenderer::initScene (OptixRenderer.cpp:436-485)."""

    def __init__(self, name):
        self.name = name
        self.materials: list[Material] = []
        self.quads: list[np.ndarray] = []
        self.quad_mat: list[int] = []
        self.spheres: list[np.ndarray] = []
        self.sphere_mat: list[int] = []
        self.vertices = np.zeros((0, 3), np.float32)
        self.normals = None
        self.texcoords = None
        self.tangents = None
        self.bitangents = None
        self.textures: list[TextureImage] = []
        self.triangles = np.zeros((0, 3), np.uint32)
        self.triangle_mat = np.zeros((0,), np.uint32)
        self.lights: list[Light] = []
        self.aabb_min = _v(0, 0, 0)
        self.aabb_max = _v(0, 0, 0)
        self.default_camera: Camera | None = None
        self.media: list[np.ndarray] = []  # [min xyz, max xyz, sigma_s, sigma_a] per medium box
        self._keep = []

    def add_material(self, m: Material) -> int:
        self.materials.append(m)
        return len(self.materials) - 1

    def add_parallelogram(self, anchor, offset1, offset2, mat: int):
        self.quads.append(np.concatenate([np.float32(anchor), np.float32(offset1), np.float32(offset2)]).astype(np.float32))
        self.quad_mat.append(mat)

    def add_sphere(self, center, radius, mat: int):
        self.spheres.append(np.array([*np.float32(center), f32(radius)], dtype=np.float32))
        self.sphere_mat.append(mat)

    def set_mesh(self, vertices, triangles, triangle_mat, normals=None, texcoords=None, tangents=None,
                 bitangents=None):
        f = lambda a: None if a is None else np.ascontiguousarray(a, dtype=np.float32)
        self.vertices = f(vertices)
        self.triangles = np.ascontiguousarray(triangles, dtype=np.uint32)
        self.triangle_mat = np.ascontiguousarray(triangle_mat, dtype=np.uint32)
        self.normals = f(normals)
        self.texcoords = f(texcoords)
        self.tangents = f(tangents)
        self.bitangents = f(bitangents)

    def add_medium_box(self, box_min, box_max, sigma_s, sigma_a):
        """AABInstance(ParticipatingMedium(sigma_s, sigma_a), AAB(min, max)) (Scene.cpp:337-350,
        Cornell.cpp:167-172): rendered when orx_config.enable_media is set."""
        self.media.append(np.array([*np.float32(box_min), *np.float32(box_max), f32(sigma_s), f32(sigma_a)],
                                   dtype=np.float32))

    def add_scene_fog(self, sigma_s=0.05, sigma_a=0.01):
        """The loaded-scene medium of Scene.cpp:337-350: ParticipatingMedium(0.05, 0.01) on the scene
        AABB with AAB::addPadding(0.01) (min -= 0.01, max += 0.01 in float, math/AAB.h:21-25)."""
        lo = (np.float32(self.aabb_min) - np.float32(0.01)).astype(np.float32)
        hi = (np.float32(self.aabb_max) + np.float32(0.01)).astype(np.float32)
        self.add_medium_box(lo, hi, sigma_s, sigma_a)

    def add_texture(self, rgba, normal_rgba=None) -> int:
        chk = lambda a: None if a is None else np.ascontiguousarray(a, dtype=np.uint8).reshape(
            np.shape(a)[0], np.shape(a)[1], 4)
        self.textures.append(TextureImage(chk(rgba), chk(normal_rgba)))
        return len(self.textures) - 1

    @property
    def num_primitives(self):
        return len(self.quads) + len(self.spheres) + len(self.triangles)

    def initial_ppm_radius(self) -> float:
        """IScene::getSceneInitialPPMRadiusEstimate (scene/IScene.cpp:51-59)."""
        ext = (self.aabb_max - self.aabb_min).astype(np.float32)
        volume = f32(f32(ext[0] * ext[1]) * ext[2])
        cubelength = f32(float(volume) ** (1.0 / 3.0))
        A = f32(f32(6) * cubelength * cubelength)
        return float(f32(float(A) * 3.94e-6))

    def to_abi(self) -> _abi.OrxScene:
        s = _abi.OrxScene()
        keep = []

        def arr(a, ctype):
            a = np.ascontiguousarray(a)
            keep.append(a)
            return a.ctypes.data_as(C.POINTER(ctype))

        q = np.array(self.quads, dtype=np.float32).reshape(-1, 9)
        s.n_quads = len(q)
        s.quads = arr(q, C.c_float)
        s.quad_material = arr(np.array(self.quad_mat, dtype=np.uint32), C.c_uint32)
        sp = np.array(self.spheres, dtype=np.float32).reshape(-1, 4)
        s.n_spheres = len(sp)
        s.spheres = arr(sp, C.c_float)
        s.sphere_material = arr(np.array(self.sphere_mat, dtype=np.uint32), C.c_uint32)
        s.n_vertices = len(self.vertices)
        s.vertices = arr(self.vertices, C.c_float)
        s.normals = arr(self.normals, C.c_float) if self.normals is not None else None
        s.n_triangles = len(self.triangles)
        s.triangles = arr(self.triangles, C.c_uint32)
        s.triangle_material = arr(self.triangle_mat, C.c_uint32)
        mats = (_abi.OrxMaterial * max(1, len(self.materials)))(*[m.to_abi() for m in self.materials])
        keep.append(mats)
        s.n_materials = len(self.materials)
        s.materials = C.cast(mats, C.POINTER(_abi.OrxMaterial))
        lights = (_abi.OrxLight * max(1, len(self.lights)))(*[l.to_abi() for l in self.lights])
        keep.append(lights)
        s.n_lights = len(self.lights)
        s.lights = C.cast(lights, C.POINTER(_abi.OrxLight))
        s.aabb_min[:] = [float(v) for v in self.aabb_min]
        s.aabb_max[:] = [float(v) for v in self.aabb_max]
        s.texcoords = arr(self.texcoords, C.c_float) if self.texcoords is not None else None
        s.tangents = arr(self.tangents, C.c_float) if self.tangents is not None else None
        s.bitangents = arr(self.bitangents, C.c_float) if self.bitangents is not None else None
        texs = (_abi.OrxTexture * max(1, len(self.textures)))()
        for i, t in enumerate(self.textures):
            texs[i].height, texs[i].width = t.rgba.shape[0], t.rgba.shape[1]
            texs[i].rgba = arr(t.rgba, C.c_uint8)
            if t.normal_rgba is not None:
                texs[i].normal_height, texs[i].normal_width = t.normal_rgba.shape[0], t.normal_rgba.shape[1]
                texs[i].normal_rgba = arr(t.normal_rgba, C.c_uint8)
        keep.append(texs)
        s.n_textures = len(self.textures)
        s.textures = C.cast(texs, C.POINTER(_abi.OrxTexture))
        med = np.array(self.media, dtype=np.float32).reshape(-1, 8)
        s.n_media = len(med)
        s.media = arr(med, C.c_float)
        self._keep = keep
        return s


def cornell() -> Scene:
    """Cornell (scene/Cornell.cpp:20-31, :66-192, :199-207)."""
    sc = Scene("Cornell")
    light = AreaLight((0.5e6, 0.4e6, 0.2e6), (343.0, 548.7999, 227.0), (0.0, 0.0, 105.0), (-130.0, 0.0, 0.0))
    sc.lights.append(light)
    sc.aabb_min = _v(-5, -5, -5)
    sc.aabb_max = (_v(556.0, 548.85, 559.2) + f32(5)).astype(np.float32)
    white = sc.add_material(Diffuse(0.8))
    green = sc.add_material(Diffuse((0.05, 0.8, 0.05)))
    red = sc.add_material(Diffuse((1.0, 0.05, 0.05)))
    sc.add_parallelogram((0, 0, 0), (0, 0, 559.2), (556.0, 0, 0), white)       # floor
    sc.add_parallelogram((0, 548.80, 0), (556.0, 0, 0), (0, 0, 559.2), white)  # ceiling
    sc.add_parallelogram((0, 0, 559.2), (0, 548.8, 0), (556.0, 0, 0), white)   # back wall
    sc.add_parallelogram((0, 0, 0), (0, 548.8, 0), (0, 0, 559.2), green)       # right wall
    sc.add_parallelogram((556.0, 0, 0), (0, 0, 559.2), (0, 548.8, 0), red)     # left wall
    emitter = sc.add_material(DiffuseEmitter(light.power, 1.0, light.inverse_area))
    sc.add_parallelogram(light.position, light.v1, light.v2, emitter)
    sc.default_camera = Camera(_v(278.0, 273.0, -850.0), _v(278.0, 273.0, 0.0), _v(0.0, 1.0, 0.0), 35.0, 35.0, 0.0)
    return sc


def cornell_medium(sigma_s=0.001, sigma_a=0.0, glass_sphere=True) -> Scene:
    """Cornell with a participating-medium box: the test block of Cornell.cpp:165-173 (compiled
    in under ENABLE_PARTICIPATING_MEDIA): ParticipatingMedium(0.001, 0.00) on
    AAB(Vector3(-1), Vector3(556.0f, 548.85f, 559.2f) - 1) and a glass sphere Sphere((250, 370, 250), 50)
    of Glass(1.5, 1) (Cornell.cpp:161).  The camera (z = -850) looks in through the box's open
    front, the light (y = 548.7999) sits just above its top face (547.85)."""
    sc = cornell()
    sc.name = "CornellMedium"
    sc.add_medium_box((-1.0, -1.0, -1.0), (555.0, f32(548.85) - f32(1.0), f32(559.2) - f32(1.0)), sigma_s, sigma_a)
    if glass_sphere:
        glass = sc.add_material(Glass(1.5, 1.0, 1.0))
        sc.add_sphere((250.0, 370.0, 250.0), 50.0, glass)
    return sc


class CornellSmallConfig:
    """CornellSmall::Config bits (scene/CornellSmall.h:18-41)."""
    SmallVCMColors = 1 << 0
    LightArea = 1 << 1
    LightAreaUpwards = 1 << 2
    LightPoint = 1 << 3
    LightPointStrong = 1 << 4
    LightPointDistant = 1 << 5
    BackwallBlue = 1 << 6
    FloorMirror = 1 << 7
    FloorGlossy = 1 << 8
    Blocks = 1 << 9
    LargeMirrorSphere = 1 << 10
    LargeGlassSphere = 1 << 11
    SmallMirrorSphere = 1 << 12
    SmallGlassSphere = 1 << 13
    Default = LightArea | Blocks


def cornell_small(config=CornellSmallConfig.Default, name="CornellSmall") -> Scene:
    """CornellSmall (scene/CornellSmall.cpp:25-330)."""
    K = CornellSmallConfig
    sc = Scene(name)
    if config & (K.LightArea | K.LightAreaUpwards):
        anchor, v1, v2 = _v(1.0, 2.499, 1.0), _v(0.5, 0, 0), _v(0, 0, 0.5)
        if config & K.LightAreaUpwards:
            v1, v2 = v2, v1
            anchor = (anchor - _v(0.0, 0.1, 0.0)).astype(np.float32)
        sc.lights.append(AreaLight(np.full(3, 19.661107023935260172519494336416, np.float32), anchor, v1, v2))
    elif config & (K.LightPoint | K.LightPointStrong | K.LightPointDistant):
        anchor = _v(1.25, 2.25, 1.25)
        power = 30.0
        if config & K.LightPointStrong:
            power = 70.0
        if config & K.LightPointDistant:
            power = 200.0
            anchor = (anchor + _v(0, 5, 0)).astype(np.float32)
        sc.lights.append(PointLight(power, anchor))
    sc.aabb_min = _v(-0.1, -0.1, -0.1)
    sc.aabb_max = (_v(2.5, 2.5, 2.5) + f32(0.1)).astype(np.float32)

    white = Diffuse(0.8)
    green = Diffuse((0.05, 0.8, 0.05))
    red = Diffuse((1.0, 0.05, 0.05))
    if config & K.SmallVCMColors:
        white = Diffuse((0.803922,) * 3)
        green = Diffuse((0.156863, 0.803922, 0.172549))
        red = Diffuse((0.803922, 0.152941, 0.152941))
    blue = Diffuse((0.156863, 0.172549, 0.803922))
    mirror = Mirror(1.0)
    glossy = Glossy(0.1, 0.7, 90.0)
    glass = Glass(1.6, 1.0, 1.0)
    ids = {}

    def mid(m):
        key = id(m)
        if key not in ids:
            ids[key] = sc.add_material(m)
        return ids[key]

    floor = mirror if config & K.FloorMirror else (glossy if config & K.FloorGlossy else white)
    back = blue if config & K.BackwallBlue else white
    rightw = red if config & K.SmallVCMColors else green
    leftw = green if config & K.SmallVCMColors else red
    sc.add_parallelogram((0, 0, 0), (0, 0, 2.5), (2.5, 0, 0), mid(floor))
    if not config & K.LightPointDistant:
        sc.add_parallelogram((0, 2.5, 0), (2.5, 0, 0), (0, 0, 2.5), mid(white))
    sc.add_parallelogram((0, 0, 2.5), (0, 2.5, 0), (2.5, 0, 0), mid(back))
    sc.add_parallelogram((0, 0, 0), (0, 2.5, 0), (0, 0, 2.5), mid(rightw))
    sc.add_parallelogram((2.5, 0, 0), (0, 0, 2.5), (0, 2.5, 0), mid(leftw))
    if config & K.Blocks:
        d = lambda *a: _vdiv_scalar(_v(*a), 220.0)
        blocks = [
            ((130.0, 165.0, 65.0), (-48.0, 0.0, 160.0), (160.0, 0.0, 49.0)),
            ((290.0, 0.0, 114.0), (0.0, 165.0, 0.0), (-50.0, 0.0, 158.0)),
            ((130.0, 0.0, 65.0), (0.0, 165.0, 0.0), (160.0, 0.0, 49.0)),
            ((82.0, 0.0, 225.0), (0.0, 165.0, 0.0), (48.0, 0.0, -160.0)),
            ((240.0, 0.0, 272.0), (0.0, 165.0, 0.0), (-158.0, 0.0, -47.0)),
            ((423.0, 340.0, 247.0), (-158.0, 0.0, 49.0), (49.0, 0.0, 159.0)),
            ((423.0, 0.0, 247.0), (0.0, 340.0, 0.0), (49.0, 0.0, 159.0)),
            ((472.0, 0.0, 406.0), (0.0, 340.0, 0.0), (-158.0, 0.0, 50.0)),
            ((314.0, 0.0, 456.0), (0.0, 340.0, 0.0), (-49.0, 0.0, -160.0)),
            ((265.0, 0.0, 296.0), (0.0, 340.1, 0.0), (158.0, 0.0, -49.0)),
        ]
        for a, b, c in blocks:
            sc.add_parallelogram(d(*a), d(*b), d(*c), mid(white))
    if config & (K.LightArea | K.LightAreaUpwards):
        l = sc.lights[0]
        em = sc.add_material(DiffuseEmitter(l.power, 1.0, l.inverse_area))
        sc.add_parallelogram(l.position, l.v1, l.v2, em)
    if config & (K.LargeMirrorSphere | K.LargeGlassSphere):
        m = glass if config & K.LargeGlassSphere else mirror
        sc.add_sphere((1.25, 0.8, 1.25), 0.8, mid(m))
    if config & K.SmallGlassSphere:
        sc.add_sphere((float(f32(1.25) - f32(0.535714269)), 0.5, 1.25), 0.5, mid(glass))
    if config & K.SmallMirrorSphere:
        sc.add_sphere((float(f32(1.25) + f32(0.535714269)), 0.5, 1.25), 0.5, mid(mirror))
    sc.default_camera = Camera(_v(1.25, 1.25, -2.85), _v(1.25, 1.25, 0.0), _v(0.0, 1.0, 0.0), 45.0, 45.0, 0.0)
    return sc


def scene_by_name(name: str) -> Scene:
    """SceneFactory::getSceneByName (Gui/scene/SceneFactory.cpp:24-70) for the
    built-in scenes; .dae loading is out of scope (assimp + assets absent)."""
    K = CornellSmallConfig
    table = {
        "Cornell": lambda: cornell(),
        "CornellMedium": lambda: cornell_medium(),
        "CornellSmall": lambda: cornell_small(K.Default, "CornellSmall"),
        "CornellSmallNoBlocks": lambda: cornell_small(K.LightArea, "CornellSmallNoBlocks"),
        "CornellSmallLargeSphere": lambda: cornell_small(
            K.SmallVCMColors | K.BackwallBlue | K.FloorGlossy | K.LargeMirrorSphere | K.LightArea,
            "CornellSmallLargeSphere"),
        "CornellSmallSmallSpheres": lambda: cornell_small(
            K.SmallVCMColors | K.BackwallBlue | K.FloorGlossy | K.LightPointStrong | K.SmallGlassSphere
            | K.SmallMirrorSphere, "CornellSmallSmallSpheres"),
        "CornellSmallLightUpwards": lambda: cornell_small(
            K.SmallVCMColors | K.BackwallBlue | K.LightAreaUpwards, "CornellSmallLightUpwards"),
        "CornellSmallPointDistant": lambda: cornell_small(
            K.SmallVCMColors | K.BackwallBlue | K.LightPointDistant | K.SmallGlassSphere | K.SmallMirrorSphere,
            "CornellSmallPointDistant"),
        "CornellSmallPointTest": lambda: cornell_small(
            K.SmallVCMColors | K.BackwallBlue | K.SmallGlassSphere | K.FloorGlossy | K.LightPointStrong,
            "CornellSmallPointTest"),
    }
    if name in table:
        return table[name]()
    if name.lower().endswith((".obj", ".dae")):  # SceneFactory: any other name is a scene file
        from .sceneio import load_scene
        return load_scene(name)
    if name == "TexturedRoom":
        from .synthetic import textured_room
        return textured_room()
    if name.startswith("SyntheticHall"):
        from .synthetic import synthetic_hall
        return synthetic_hall()
    if name.startswith("SyntheticConference"):
        from .synthetic import synthetic_conference
        return synthetic_conference()
    raise KeyError(f"unknown scene {name!r}")
