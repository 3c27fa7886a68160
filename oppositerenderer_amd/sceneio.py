"""Scene import: Wavefront OBJ/MTL and COLLADA (.dae) files -> flat `scenes.Scene`.

Restates what `Scene::createFromFile` (RenderEngine/scene/Scene.cpp:73-311,
:361-565) does through assimp 3.0 (README.md:30-37; absent here, so its
post-processing is restated and parity with it is unpinned):

* post-processing of the ReadFile call (Scene.cpp:93-104): polygons are
  triangulated as fans, node transforms are baked into the vertices
  (PreTransformVertices), missing normals are generated as smooth normals,
  tangents/bitangents are computed from the texture coordinates
  (CalcTangentSpace);
* `loadSceneMaterials` (:170-255): emissive -> DiffuseEmitter(emissive, Kd or 1);
  diffuse texture -> Texture (normal map from the NORMALS slot); IOR > 1 ->
  Glass(ior, 1, 1); reflective -> Mirror(reflective); diffuse colour ->
  Diffuse(Kd); otherwise red Diffuse(1, 0, 0).  `colorHasAnyComponent`
  (:563-566) requires EVERY component > 0, as the reference;
* `loadLightSources` (:257-273): point and spot lights of the file;
* `loadMeshLightSource` (:275-300): the first face (p0, p1, p2) of an emitter
  mesh becomes an area light anchored at p0 with v1 = p1 - p0, v2 = p2 - p0
  and the emitter's Kd-scaled power; the emitter gets its inverse area.  The
  reference registers every emitter twice (:141 and again from
  getSceneRootGroup :508); `duplicate_emitter_lights`
  reproduces that, the default registers each once;
* the scene AABB (:146-160) is built from `mIndices[0]` of every face three
  times (Appendix A.5); `reference_aabb=False` uses all three corners;
* `loadDefaultSceneCamera` (:469-485): eye, eye + lookAt, normalised up,
  hfov = vfov = mHorizontalFOV * 365 / (2 pi) (the reference's 365, Appendix
  A.9), KeepHorizontal.

Images (util/Image.cpp:14-158): TGA types 2/3 uncompressed are read in file
row order with alpha forced to 1 (:97-106); other formats go through PIL and
are reordered like the reference's QImage::Format_ARGB32 byte shuffle
(:49-56), which on a little-endian host yields (G, R, A, B) texels — a
reference bug reproduced unless `reference_channel_order=False`.
"""
from __future__ import annotations

import math
import os
import struct
import xml.etree.ElementTree as ET

import numpy as np

from . import scenes

f32 = np.float32


# ---------------------------------------------------------------------------
# images
# ---------------------------------------------------------------------------
def load_tga(path: str) -> np.ndarray:
    """Image::loadImageFromTga (util/Image.cpp:80-139) -> uint8 [h, w, 4]."""
    with open(path, "rb") as f:
        data = f.read()
    if len(data) < 18:
        raise ValueError(f"{path}: not a TGA file")
    id_len, cmap_type, img_type = data[0], data[1], data[2]
    cmap_len = struct.unpack_from("<H", data, 5)[0]
    cmap_depth = data[7]
    w, h = struct.unpack_from("<HH", data, 12)
    depth = data[16]
    if cmap_type == 1:
        raise ValueError(f"Does not support TGA color map for {path}")
    if img_type not in (2, 3):
        raise ValueError(f"Only supports RGB(A) type TGA textures - does not support type '{img_type}' for {path}")
    off = 18 + id_len + (cmap_len * ((cmap_depth + 7) // 8) if cmap_type else 0)
    bpp = depth // 8
    if bpp not in (1, 3, 4) or (img_type == 2 and bpp == 1):
        raise ValueError(f"{path}: unsupported TGA depth {depth}")
    px = np.frombuffer(data, np.uint8, w * h * bpp, off).reshape(h, w, bpp)
    out = np.empty((h, w, 4), np.uint8)
    if bpp == 1:  # grayscale: expanded to RGB (libtga's conversion is unpinned)
        out[..., 0] = out[..., 1] = out[..., 2] = px[..., 0]
    else:  # TGA_RGB: BGR(A) file order -> RGB
        out[..., 0], out[..., 1], out[..., 2] = px[..., 2], px[..., 1], px[..., 0]
    out[..., 3] = 1  # m_imageData[... + 3] = 1 (Image.cpp:105)
    return out  # rows in file order: yOut = y (Image.cpp:99)


def save_tga(path: str, rgba: np.ndarray) -> None:
    """Uncompressed 32-bit TGA, rows written in array order (inverse of load_tga)."""
    rgba = np.ascontiguousarray(rgba, np.uint8)
    h, w = rgba.shape[:2]
    hdr = struct.pack("<BBBHHBHHHHBB", 0, 0, 2, 0, 0, 0, 0, 0, w, h, 32, 8)
    bgra = rgba[..., [2, 1, 0, 3]]
    with open(path, "wb") as f:
        f.write(hdr)
        f.write(bgra.tobytes())


def load_image(path: str, reference_channel_order: bool = True) -> np.ndarray:
    """Image::Image (util/Image.cpp:14-72) -> uint8 [h, w, 4]."""
    if not os.path.exists(path):
        raise FileNotFoundError(f"The file {path} does not exist.")
    if path.lower().endswith(".tga"):
        return load_tga(path)
    from PIL import Image as PILImage
    with PILImage.open(path) as im:
        rgba = np.asarray(im.convert("RGBA"), np.uint8)
    if not reference_channel_order:
        return rgba.copy()
    # QImage ARGB32 on a little-endian host holds B, G, R, A bytes; the
    # reference copies bytes 1, 2, 3, 0 of each texel: G, R, A, B
    return np.ascontiguousarray(rgba[..., [1, 0, 3, 2]])


# ---------------------------------------------------------------------------
# geometry post-processing (assimp ReadFile flags, Scene.cpp:93-104)
# ---------------------------------------------------------------------------
class _Mesh:
    def __init__(self, material: int):
        self.material = material
        self.positions: list = []   # per corner
        self.normals: list = []
        self.uvs: list = []
        self.faces: list = []       # lists of corner indices


def _smooth_normals(P, tris):
    """GenSmoothNormals: per-vertex mean of the unit face normals of the faces
    that share the vertex position."""
    fn = np.cross(P[tris[:, 1]] - P[tris[:, 0]], P[tris[:, 2]] - P[tris[:, 0]])
    ln = np.linalg.norm(fn, axis=1, keepdims=True)
    fn = np.where(ln > 0, fn / np.maximum(ln, 1e-30), 0.0)
    _, key = np.unique(P, axis=0, return_inverse=True)
    key = key.reshape(-1)
    acc = np.zeros((key.max() + 1 if len(key) else 0, 3))
    for k in range(3):
        np.add.at(acc, key[tris[:, k]], fn)
    n = acc[key]
    ln = np.linalg.norm(n, axis=1, keepdims=True)
    return np.where(ln > 0, n / np.maximum(ln, 1e-30), 0.0)


def _tangent_space(P, N, UV, tris):
    """CalcTangentSpace: per-face tangent/bitangent from the texture-coordinate
    derivatives, summed per vertex, tangent made orthogonal to the normal."""
    T = np.zeros_like(P)
    B = np.zeros_like(P)
    p0, p1, p2 = P[tris[:, 0]], P[tris[:, 1]], P[tris[:, 2]]
    w0, w1, w2 = UV[tris[:, 0]], UV[tris[:, 1]], UV[tris[:, 2]]
    e1, e2 = p1 - p0, p2 - p0
    d1, d2 = w1 - w0, w2 - w0
    det = d1[:, 0] * d2[:, 1] - d2[:, 0] * d1[:, 1]
    r = np.where(np.abs(det) > 1e-20, 1.0 / np.where(det == 0, 1, det), 0.0)[:, None]
    ft = (e1 * d2[:, 1:2] - e2 * d1[:, 1:2]) * r
    fb = (e2 * d1[:, 0:1] - e1 * d2[:, 0:1]) * r
    for k in range(3):
        np.add.at(T, tris[:, k], ft)
        np.add.at(B, tris[:, k], fb)
    T = T - N * np.sum(N * T, axis=1, keepdims=True)
    nt = np.linalg.norm(T, axis=1, keepdims=True)
    nb = np.linalg.norm(B, axis=1, keepdims=True)
    return np.where(nt > 0, T / np.maximum(nt, 1e-30), 0.0), np.where(nb > 0, B / np.maximum(nb, 1e-30), 0.0)


class _Material:
    def __init__(self, name):
        self.name = name
        self.diffuse = None
        self.emissive = None
        self.reflective = None
        self.ior = None
        self.tex_diffuse = None
        self.tex_normals = None


def _all_positive(c):
    return c is not None and all(v > 0 for v in c)  # colorHasAnyComponent (Scene.cpp:563-566)


def _build(name, meshes, materials, lights, camera, base_dir, duplicate_emitter_lights, reference_aabb,
           reference_channel_order):
    sc = scenes.Scene(name)
    # loadSceneMaterials (Scene.cpp:170-255)
    mat_ids, emitters, texcache = [], {}, {}

    def texture(path_main, path_norm):
        key = (path_main, path_norm)
        if key not in texcache:
            img = load_image(os.path.join(base_dir, path_main), reference_channel_order)
            nimg = load_image(os.path.join(base_dir, path_norm), reference_channel_order) if path_norm else None
            texcache[key] = sc.add_texture(img, nimg)
        return texcache[key]

    for i, m in enumerate(materials):
        if _all_positive(m.emissive):
            kd = m.diffuse if m.diffuse is not None else (1.0, 1.0, 1.0)
            emitters[i] = (np.float32(m.emissive), np.float32(kd))
            mat_ids.append(None)  # created with its light's inverse area below
        elif m.tex_diffuse:
            mat_ids.append(sc.add_material(scenes.Texture(texture(m.tex_diffuse, m.tex_normals))))
        elif m.ior is not None and m.ior > 1.0:
            mat_ids.append(sc.add_material(scenes.Glass(m.ior, 1.0, 1.0)))
        elif _all_positive(m.reflective):
            mat_ids.append(sc.add_material(scenes.Mirror(tuple(m.reflective))))
        elif m.diffuse is not None:
            mat_ids.append(sc.add_material(scenes.Diffuse(tuple(m.diffuse))))
        else:
            mat_ids.append(sc.add_material(scenes.Diffuse((1.0, 0.0, 0.0))))
    sc.lights.extend(lights)  # loadLightSources
    # emitter meshes -> area lights (loadMeshLightSource, Scene.cpp:275-300)
    for i, (emissive, kd) in emitters.items():
        power = (emissive * kd).astype(np.float32)  # DiffuseEmitter ctor scales power by Kd
        light = None
        for mesh in meshes:
            if mesh.material != i or not mesh.faces:
                continue
            f0 = mesh.faces[0]
            anchor = np.float32(mesh.positions[f0[0]])
            v1 = (np.float32(mesh.positions[f0[1]]) - anchor).astype(np.float32)
            v2 = (np.float32(mesh.positions[f0[2]]) - anchor).astype(np.float32)
            light = scenes.AreaLight(power, anchor, v1, v2)
            for _ in range(2 if duplicate_emitter_lights else 1):
                sc.lights.append(light)
        mat_ids[i] = sc.add_material(scenes.DiffuseEmitter(tuple(emissive), tuple(kd),
                                                          light.inverse_area if light is not None else 0.0))
    # triangle soup -> shared vertices (JoinIdenticalVertices) per mesh
    V, Nn, UV, T, M = [], [], [], [], []
    base = 0
    any_uv = any(m.uvs for m in meshes)
    aabb_pts = []
    for mesh in meshes:
        if not mesh.faces:
            continue
        tris = []
        for f in mesh.faces:
            for k in range(1, len(f) - 1):  # Triangulate: fan
                tris.append((f[0], f[k], f[k + 1]))
        tris = np.array(tris, np.int64)
        P = np.array(mesh.positions, np.float64)
        has_n = len(mesh.normals) == len(mesh.positions) and len(mesh.normals) > 0
        has_uv = len(mesh.uvs) == len(mesh.positions) and len(mesh.uvs) > 0
        Nm = np.array(mesh.normals, np.float64) if has_n else None
        Um = np.array(mesh.uvs, np.float64) if has_uv else np.zeros((len(P), 2))
        attrs = np.concatenate([P, Nm if has_n else np.zeros_like(P), Um], axis=1)
        uniq, inv = np.unique(attrs, axis=0, return_inverse=True)
        inv = inv.reshape(-1)
        tris = inv[tris]
        P, Um = uniq[:, 0:3], uniq[:, 6:8]
        Nm = uniq[:, 3:6] if has_n else _smooth_normals(P, tris)
        V.append(P)
        Nn.append(Nm)
        UV.append(Um)
        T.append(tris + base)
        M.append(np.full(len(tris), mat_ids[mesh.material], np.uint32))
        aabb_pts.append(P[tris[:, 0]] if reference_aabb else P[tris.reshape(-1)])
        base += len(P)
    if V:
        P = np.concatenate(V)
        N = np.concatenate(Nn)
        UVa = np.concatenate(UV)
        tris = np.concatenate(T)
        tan, btan = _tangent_space(P, N, UVa, tris) if any_uv else (None, None)
        sc.set_mesh(P.astype(np.float32), tris.astype(np.uint32), np.concatenate(M), N.astype(np.float32),
                    texcoords=UVa.astype(np.float32) if any_uv else None,
                    tangents=None if tan is None else tan.astype(np.float32),
                    bitangents=None if btan is None else btan.astype(np.float32))
        pts = np.concatenate(aabb_pts).astype(np.float32)
        sc.aabb_min, sc.aabb_max = pts.min(axis=0), pts.max(axis=0)
    else:
        sc.aabb_min = np.full(3, 1e33, np.float32)
        sc.aabb_max = np.full(3, -1e33, np.float32)
    if camera is not None:
        eye, look, up, hfov_rad = camera
        fov = float(f32(hfov_rad) * f32(365.0) / (f32(2.0) * f32(math.pi)))
        upn = np.float32(up) / np.float32(np.linalg.norm(np.float32(up)))
        sc.default_camera = scenes.Camera(np.float32(eye), (np.float32(eye) + np.float32(look)).astype(np.float32),
                                          upn.astype(np.float32), fov, fov, 0.0, "KeepHorizontal")
    else:
        c = (sc.aabb_min + sc.aabb_max) * 0.5
        ext = float(np.max(sc.aabb_max - sc.aabb_min)) if V else 1.0
        sc.default_camera = scenes.Camera(np.float32(c + [0, 0, -2 * ext]), np.float32(c), np.float32([0, 1, 0]),
                                          45.0, 45.0, 0.0)
    if not sc.lights:
        raise ValueError("No lights exists in this scene.")
    return sc


# ---------------------------------------------------------------------------
# Wavefront OBJ / MTL
# ---------------------------------------------------------------------------
def _parse_mtl(path):
    mats, cur = {}, None
    if not os.path.exists(path):
        return mats
    for line in open(path, encoding="utf-8", errors="replace"):
        t = line.split()
        if not t or t[0].startswith("#"):
            continue
        k = t[0].lower()
        if k == "newmtl":
            cur = _Material(" ".join(t[1:]))
            mats[cur.name] = cur
        elif cur is None:
            continue
        elif k == "kd":
            cur.diffuse = tuple(float(v) for v in t[1:4])
        elif k == "ke":
            cur.emissive = tuple(float(v) for v in t[1:4])
        elif k == "kr":  # reflective colour (assimp AI_MATKEY_COLOR_REFLECTIVE)
            cur.reflective = tuple(float(v) for v in t[1:4])
        elif k == "ni":
            cur.ior = float(t[1])
        elif k == "map_kd":
            cur.tex_diffuse = t[-1]
        elif k in ("norm", "map_kn"):  # aiTextureType_NORMALS
            cur.tex_normals = t[-1]
    return mats


def load_obj(path: str, duplicate_emitter_lights: bool = False, reference_aabb: bool = True,
             reference_channel_order: bool = True) -> scenes.Scene:
    """Wavefront OBJ (+ MTL) through Scene::createFromFile's pipeline."""
    base_dir = os.path.dirname(os.path.abspath(path))
    vs, vns, vts = [], [], []
    materials: list[_Material] = []
    mat_index: dict[str, int] = {}
    libs: dict[str, _Material] = {}
    meshes: dict[int, _Mesh] = {}
    lights = []
    current = None

    def mesh_for(mi):
        if mi not in meshes:
            meshes[mi] = _Mesh(mi)
        return meshes[mi]

    def use(name):
        if name not in mat_index:
            m = libs.get(name)
            if m is None:
                m = _Material(name)
                m.diffuse = (0.6, 0.6, 0.6)  # assimp ObjFile default material
            mat_index[name] = len(materials)
            materials.append(m)
        return mat_index[name]

    for line in open(path, encoding="utf-8", errors="replace"):
        t = line.split()
        if not t or t[0].startswith("#"):
            continue
        k = t[0]
        if k == "v":
            vs.append([float(x) for x in t[1:4]])
        elif k == "vn":
            vns.append([float(x) for x in t[1:4]])
        elif k == "vt":
            vts.append([float(x) for x in t[1:3]] + ([0.0] if len(t) < 3 else []))
        elif k == "mtllib":
            libs.update(_parse_mtl(os.path.join(base_dir, " ".join(t[1:]))))
        elif k == "usemtl":
            current = use(" ".join(t[1:]))
        elif k == "f":
            if current is None:
                current = use("__default__")
            m = mesh_for(current)
            corners = []
            for c in t[1:]:
                parts = c.split("/")
                vi = int(parts[0])
                vi = vi - 1 if vi > 0 else len(vs) + vi
                m.positions.append(vs[vi])
                ti = parts[1] if len(parts) > 1 and parts[1] else None
                ni = parts[2] if len(parts) > 2 and parts[2] else None
                if ni is not None:
                    n = int(ni)
                    m.normals.append(vns[n - 1 if n > 0 else len(vns) + n])
                if ti is not None:
                    q = int(ti)
                    m.uvs.append(vts[q - 1 if q > 0 else len(vts) + q][:2])
                corners.append(len(m.positions) - 1)
            if len(corners) >= 3:
                m.faces.append(corners)
    return _build(os.path.abspath(path), [meshes[k] for k in sorted(meshes)], materials, lights, None, base_dir,
                  duplicate_emitter_lights, reference_aabb, reference_channel_order)


# ---------------------------------------------------------------------------
# COLLADA 1.4 (the reference's Sponza / Conference scenes are .dae)
# ---------------------------------------------------------------------------
def _strip(tag):
    return tag.split("}", 1)[1] if "}" in tag else tag


def _floats(text):
    return [float(x) for x in (text or "").split()]


def _node_matrix(node):
    M = np.eye(4)
    for ch in node:
        tag = _strip(ch.tag)
        v = _floats(ch.text)
        if tag == "matrix":
            M = M @ np.array(v, np.float64).reshape(4, 4)
        elif tag == "translate":
            T = np.eye(4)
            T[:3, 3] = v[:3]
            M = M @ T
        elif tag == "scale":
            M = M @ np.diag([v[0], v[1], v[2], 1.0])
        elif tag == "rotate":
            ax = np.array(v[:3], np.float64)
            ax = ax / max(np.linalg.norm(ax), 1e-30)
            a = math.radians(v[3])
            c, s = math.cos(a), math.sin(a)
            x, y, z = ax
            R = np.array([[c + x * x * (1 - c), x * y * (1 - c) - z * s, x * z * (1 - c) + y * s, 0],
                          [y * x * (1 - c) + z * s, c + y * y * (1 - c), y * z * (1 - c) - x * s, 0],
                          [z * x * (1 - c) - y * s, z * y * (1 - c) + x * s, c + z * z * (1 - c), 0],
                          [0, 0, 0, 1]])
            M = M @ R
        elif tag == "lookat":
            pass  # cameras only; handled where cameras are resolved
    return M


def load_collada(path: str, duplicate_emitter_lights: bool = False, reference_aabb: bool = True,
                 reference_channel_order: bool = True) -> scenes.Scene:
    """COLLADA subset: <triangles>/<polylist>/<polygons> meshes with VERTEX,
    NORMAL and TEXCOORD inputs; lambert/phong/blinn/constant effects (emission,
    diffuse colour or texture, reflective, index_of_refraction, an extra bump
    texture as normal map); node matrix/translate/rotate/scale transforms baked
    in; point/spot lights; the first perspective camera."""
    base_dir = os.path.dirname(os.path.abspath(path))
    root = ET.parse(path).getroot()
    ns = {"c": root.tag.split("}")[0][1:]} if root.tag.startswith("{") else {}
    q = (lambda p: p.replace("c:", "")) if not ns else (lambda p: p)

    def find(el, p):
        return el.find(q(p), ns)

    def findall(el, p):
        return el.findall(q(p), ns)

    byid = {}
    for el in root.iter():
        i = el.get("id")
        if i is not None:
            byid[i] = el
    ref = lambda url: byid.get(url.lstrip("#")) if url else None
    # images
    images = {}
    for im in findall(root, ".//c:library_images/c:image"):
        init = find(im, "c:init_from")
        if init is not None and init.text:
            images[im.get("id")] = init.text.strip().replace("file://", "")

    def effect_texture(prof, slot_el):
        if slot_el is None:
            return None
        tex = find(slot_el, "c:texture")
        if tex is None:
            return None
        sampler = tex.get("texture")
        # texture -> sampler2D newparam -> surface newparam -> image, or directly an image id
        for _ in range(3):
            if sampler in images:
                return images[sampler]
            np_el = None
            for p in findall(prof, ".//c:newparam"):
                if p.get("sid") == sampler:
                    np_el = p
            if np_el is None:
                return None
            src = np_el.find(".//" + q("c:source"), ns)
            init = np_el.find(".//" + q("c:init_from"), ns)
            sampler = (src.text if src is not None else init.text if init is not None else "").strip()
        return images.get(sampler)

    def color(el):
        if el is None:
            return None
        c = find(el, "c:color")
        return tuple(_floats(c.text)[:3]) if c is not None else None

    def material_of(mid):
        m = _Material(mid)
        mel = byid.get(mid)
        eff = ref(find(mel, "c:instance_effect").get("url")) if mel is not None and find(mel, "c:instance_effect") is not None else None
        if eff is None:
            m.diffuse = None
            return m
        prof = find(eff, "c:profile_COMMON")
        tech = find(prof, "c:technique") if prof is not None else None
        shade = None
        if tech is not None:
            for kind in ("phong", "blinn", "lambert", "constant"):
                shade = find(tech, "c:" + kind)
                if shade is not None:
                    break
        if shade is None:
            return m
        m.emissive = color(find(shade, "c:emission"))
        m.diffuse = color(find(shade, "c:diffuse"))
        m.reflective = color(find(shade, "c:reflective"))
        ior = find(shade, "c:index_of_refraction")
        if ior is not None and find(ior, "c:float") is not None:
            m.ior = float(find(ior, "c:float").text)
        m.tex_diffuse = effect_texture(prof, find(shade, "c:diffuse"))
        bump = tech.find(".//" + q("c:bump"), ns) if tech is not None else None
        m.tex_normals = effect_texture(prof, bump)
        return m

    materials: list[_Material] = []
    mat_index: dict[str, int] = {}

    def use(mid):
        if mid not in mat_index:
            mat_index[mid] = len(materials)
            materials.append(material_of(mid))
        return mat_index[mid]

    def source_array(src_id):
        s = byid.get(src_id.lstrip("#"))
        if s is not None and _strip(s.tag) == "vertices":
            inp = [i for i in findall(s, "c:input") if i.get("semantic") == "POSITION"][0]
            s = byid.get(inp.get("source").lstrip("#"))
        arr = _floats(find(s, "c:float_array").text)
        acc = s.find(".//" + q("c:accessor"), ns)
        stride = int(acc.get("stride", "1")) if acc is not None else 3
        return np.array(arr, np.float64).reshape(-1, stride)

    meshes: dict[int, _Mesh] = {}
    lights = []
    camera = None

    def walk(node, M):
        nonlocal camera
        M = M @ _node_matrix(node)
        Nm = np.linalg.inv(M[:3, :3]).T
        for ig in findall(node, "c:instance_geometry"):
            geo = ref(ig.get("url"))
            bind = {}
            for im in ig.findall(".//" + q("c:instance_material"), ns):
                bind[im.get("symbol")] = im.get("target").lstrip("#")
            mesh_el = find(geo, "c:mesh")
            if mesh_el is None:
                continue
            for prim in list(mesh_el):
                tag = _strip(prim.tag)
                if tag not in ("triangles", "polylist", "polygons"):
                    continue
                mi = use(bind.get(prim.get("material"), prim.get("material") or "__default__"))
                inputs = findall(prim, "c:input")
                stride = max(int(i.get("offset", "0")) for i in inputs) + 1
                P = Nrm = T = None
                offs = {}
                for i in inputs:
                    sem, off = i.get("semantic"), int(i.get("offset", "0"))
                    if sem == "VERTEX":
                        P, offs["p"] = source_array(i.get("source")), off
                        vel = byid.get(i.get("source").lstrip("#"))
                        for vi in findall(vel, "c:input"):
                            if vi.get("semantic") == "NORMAL":
                                Nrm, offs["n"] = source_array(vi.get("source")), off
                            if vi.get("semantic") == "TEXCOORD":
                                T, offs["t"] = source_array(vi.get("source")), off
                    elif sem == "NORMAL":
                        Nrm, offs["n"] = source_array(i.get("source")), off
                    elif sem == "TEXCOORD" and i.get("set", "0") == "0" and "t" not in offs:
                        T, offs["t"] = source_array(i.get("source")), off
                if tag == "polygons":
                    plist = [np.array(_floats(p.text), np.int64) for p in findall(prim, "c:p")]
                    counts = [len(p) // stride for p in plist]
                    idx = np.concatenate(plist) if plist else np.zeros(0, np.int64)
                else:
                    idx = np.array(_floats(find(prim, "c:p").text), np.int64)
                    if tag == "polylist":
                        counts = [int(v) for v in _floats(find(prim, "c:vcount").text)]
                    else:
                        counts = [3] * (len(idx) // (3 * stride))
                idx = idx.reshape(-1, stride)
                m = meshes.setdefault(mi, _Mesh(mi))
                pos = (np.c_[P[idx[:, offs["p"]]][:, :3], np.ones(len(idx))] @ M.T)[:, :3]
                nrm = None
                if Nrm is not None:
                    nrm = Nrm[idx[:, offs["n"]]][:, :3] @ Nm.T
                    nrm = nrm / np.maximum(np.linalg.norm(nrm, axis=1, keepdims=True), 1e-30)
                uv = T[idx[:, offs["t"]]][:, :2] if T is not None else None
                start = 0
                for cnt in counts:
                    corners = []
                    for k in range(start, start + cnt):
                        m.positions.append(pos[k].tolist())
                        if nrm is not None:
                            m.normals.append(nrm[k].tolist())
                        if uv is not None:
                            m.uvs.append(uv[k].tolist())
                        corners.append(len(m.positions) - 1)
                    start += cnt
                    if len(corners) >= 3:
                        m.faces.append(corners)
        for il in findall(node, "c:instance_light"):
            lel = ref(il.get("url"))
            tech = find(lel, "c:technique_common")
            pos = (M @ np.array([0, 0, 0, 1.0]))[:3]
            dirn = (M[:3, :3] @ np.array([0, 0, -1.0]))
            for ch in tech:
                kind = _strip(ch.tag)
                col = color(ch) or (1.0, 1.0, 1.0)
                if kind == "point":
                    lights.append(scenes.PointLight(col, pos))
                elif kind == "spot":
                    fa = find(ch, "c:falloff_angle")
                    ang = float(fa.text) if fa is not None else 45.0
                    # aiLight::mAngleInnerCone (radians) passed as Light's angle (Scene.cpp:266)
                    lights.append(scenes.SpotLight(col, pos, dirn / np.linalg.norm(dirn), math.radians(ang)))
        for ic in findall(node, "c:instance_camera"):
            if camera is None:
                cel = ref(ic.get("url"))
                persp = cel.find(".//" + q("c:perspective"), ns)
                xfov = find(persp, "c:xfov") if persp is not None else None
                yfov = find(persp, "c:yfov") if persp is not None else None
                ar = find(persp, "c:aspect_ratio") if persp is not None else None
                if xfov is not None:
                    h = math.radians(float(xfov.text))
                elif yfov is not None:
                    a = float(ar.text) if ar is not None else 1.0
                    h = 2 * math.atan(math.tan(math.radians(float(yfov.text)) / 2) * a)
                else:
                    h = math.radians(45.0)
                eye = (M @ np.array([0, 0, 0, 1.0]))[:3]
                look = M[:3, :3] @ np.array([0, 0, -1.0])
                up = M[:3, :3] @ np.array([0, 1.0, 0])
                camera = (eye, look, up, h)
        for ch in findall(node, "c:node"):
            walk(ch, M)
        for inode in findall(node, "c:instance_node"):
            n2 = ref(inode.get("url"))
            if n2 is not None:
                walk(n2, M)

    vs = root.find(".//" + q("c:library_visual_scenes/c:visual_scene"), ns)
    up_axis = root.find(".//" + q("c:asset/c:up_axis"), ns)
    M0 = np.eye(4)
    if up_axis is not None and up_axis.text.strip() == "Z_UP":  # assimp converts to Y-up
        M0 = np.array([[1, 0, 0, 0], [0, 0, 1, 0], [0, -1, 0, 0], [0, 0, 0, 1.0]])
    for node in findall(vs, "c:node") if vs is not None else []:
        walk(node, M0)
    return _build(os.path.abspath(path), [meshes[k] for k in sorted(meshes)], materials, lights, camera, base_dir,
                  duplicate_emitter_lights, reference_aabb, reference_channel_order)


def load_scene(path: str, **kw) -> scenes.Scene:
    """Scene::createFromFile by extension (.obj / .dae)."""
    ext = os.path.splitext(path)[1].lower()
    if ext == ".obj":
        return load_obj(path, **kw)
    if ext == ".dae":
        return load_collada(path, **kw)
    raise ValueError(f"unsupported scene file {path!r} (.obj, .dae)")
