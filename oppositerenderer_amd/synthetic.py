"""Seeded synthetic "Sponza-class" scene (BASELINE configs[2]/[3] stand-in).

The real Sponza / Conference .dae assets are unavailable (dead Dropbox link,
README.md:15; assimp absent), so SURVEY.md 8(d) prescribes a procedurally
tessellated hall: floor, ceiling and walls as triangle grids, two rows of
smooth-shaded columns, arcades of boxes, Lambert materials, one quad area
light registered once.  Geometry is generated deterministically from a numpy
PCG64 stream seeded with 42; nothing is stored as data.
"""
from __future__ import annotations

import numpy as np

from . import scenes

f32 = np.float32


def _grid(origin, du, dv, nu, nv):
    """Tessellated parallelogram: (nu x nv) quads -> 2*nu*nv triangles, face normal."""
    o, du, dv = (np.asarray(a, np.float64) for a in (origin, du, dv))
    u = np.linspace(0, 1, nu + 1)
    v = np.linspace(0, 1, nv + 1)
    uu, vv = np.meshgrid(u, v, indexing="ij")
    verts = o + uu[..., None] * du + vv[..., None] * dv
    verts = verts.reshape(-1, 3)
    n = np.cross(du, dv)
    n /= np.linalg.norm(n)
    norms = np.broadcast_to(n, verts.shape)
    idx = np.arange((nu + 1) * (nv + 1)).reshape(nu + 1, nv + 1)
    a, b, c, d = idx[:-1, :-1], idx[1:, :-1], idx[1:, 1:], idx[:-1, 1:]
    tris = np.concatenate([np.stack([a, b, c], -1).reshape(-1, 3), np.stack([a, c, d], -1).reshape(-1, 3)])
    return verts, norms, tris


def _cylinder(center, radius, height, nseg, nstack):
    """Open cylinder along +y with outward smooth normals."""
    th = np.linspace(0, 2 * np.pi, nseg + 1)[:-1]
    y = np.linspace(0, height, nstack + 1)
    tt, yy = np.meshgrid(th, y, indexing="ij")
    x = center[0] + radius * np.cos(tt)
    z = center[2] + radius * np.sin(tt)
    verts = np.stack([x, center[1] + yy, z], -1).reshape(-1, 3)
    norms = np.stack([np.cos(tt), np.zeros_like(tt), np.sin(tt)], -1).reshape(-1, 3)
    idx = np.arange(nseg * (nstack + 1)).reshape(nseg, nstack + 1)
    nxt = np.roll(idx, -1, axis=0)
    a, b, c, d = idx[:, :-1], nxt[:, :-1], nxt[:, 1:], idx[:, 1:]
    # winding so that the geometric normal cross(p0-p2, p1-p0) points outward
    tris = np.concatenate([np.stack([a, c, b], -1).reshape(-1, 3), np.stack([a, d, c], -1).reshape(-1, 3)])
    return verts, norms, tris


def _box(lo, hi, n):
    lo, hi = np.asarray(lo, float), np.asarray(hi, float)
    e = hi - lo
    parts = []
    X, Y, Z = np.eye(3)
    faces = [
        (lo, Z * e[2], Y * e[1]),                       # x = lo, normal -x
        (lo + X * e[0], Y * e[1], Z * e[2]),            # x = hi, normal +x
        (lo, X * e[0], Z * e[2]),                       # y = lo, normal -y
        (lo + Y * e[1], Z * e[2], X * e[0]),            # y = hi, normal +y
        (lo, Y * e[1], X * e[0]),                       # z = lo, normal -z
        (lo + Z * e[2], X * e[0], Y * e[1]),            # z = hi, normal +z
    ]
    for o, du, dv in faces:
        parts.append(_grid(o, du, dv, n, n))
    return parts


def synthetic_hall(grid_n=64, column_seg=64, column_stack=56, box_n=8, seed=42, scale=1.0 / 3.0) -> scenes.Scene:
    rng = np.random.default_rng(seed)
    # Sponza-like proportions; `scale` puts the hall in Cornell-like units so that
    # IScene::getSceneInitialPPMRadiusEstimate (A*3.94e-6, IScene.cpp:51-59),
    # which grows with the scene's linear size, stays ~1.4 grid cells as in Cornell
    S = scale
    L, Wd, Hh = 3000.0 * S, 1300.0 * S, 1400.0 * S
    sc = scenes.Scene("SyntheticHall")
    mats = {
        "floor": sc.add_material(scenes.Diffuse((0.55, 0.50, 0.45))),
        "wall": sc.add_material(scenes.Diffuse((0.75, 0.70, 0.62))),
        "ceiling": sc.add_material(scenes.Diffuse((0.8, 0.8, 0.8))),
        "column": sc.add_material(scenes.Diffuse((0.7, 0.65, 0.55))),
        "red": sc.add_material(scenes.Diffuse((0.7, 0.12, 0.10))),
        "green": sc.add_material(scenes.Diffuse((0.15, 0.55, 0.18))),
        "blue": sc.add_material(scenes.Diffuse((0.15, 0.2, 0.6))),
    }
    parts = []  # (verts, norms, tris, material)

    def add(vnt, m):
        parts.append((*vnt, m))

    add(_grid((0, 0, 0), (0, 0, Wd), (L, 0, 0), grid_n, grid_n), mats["floor"])          # floor, +y
    add(_grid((0, Hh, 0), (L, 0, 0), (0, 0, Wd), grid_n, grid_n), mats["ceiling"])       # ceiling, -y
    add(_grid((0, 0, Wd), (0, Hh, 0), (L, 0, 0), grid_n, grid_n), mats["wall"])          # back (z=Wd), -z
    add(_grid((0, 0, 0), (L, 0, 0), (0, Hh, 0), grid_n, grid_n), mats["wall"])           # front (z=0), +z
    add(_grid((0, 0, 0), (0, Hh, 0), (0, 0, Wd), grid_n, grid_n), mats["green"])         # x=0, +x
    add(_grid((L, 0, 0), (0, 0, Wd), (0, Hh, 0), grid_n, grid_n), mats["red"])           # x=L, -x
    # two colonnades
    ncol = 12
    for row, zc in enumerate((Wd * 0.27, Wd * 0.73)):
        for k in range(ncol):
            xc = L * (k + 0.5) / ncol + rng.uniform(-8, 8) * S
            r = (55.0 + rng.uniform(-5, 5)) * S
            add(_cylinder((xc, 0.0, zc), r, 900.0 * S, column_seg, column_stack), mats["column"])
            # capital + arcade beam segment as boxes
            for lo, hi in (((xc - 80 * S, 900 * S, zc - 80 * S), (xc + 80 * S, 960 * S, zc + 80 * S)),):
                for p in _box(lo, hi, box_n):
                    add(p, mats["column"])
        for k in range(ncol - 1):
            x0 = L * (k + 0.5) / ncol + 80 * S
            x1 = L * (k + 1.5) / ncol - 80 * S
            for p in _box((x0, 1040 * S, zc - 60 * S), (x1, 1120 * S, zc + 60 * S), box_n):
                add(p, mats["column"])
    # a few coloured blocks on the floor
    for _ in range(6):
        x, z = rng.uniform(300 * S, L - 300 * S), rng.uniform(350 * S, Wd - 350 * S)
        s = rng.uniform(60, 140) * S
        m = mats[("red", "green", "blue")[rng.integers(0, 3)]]
        for p in _box((x - s, 0, z - s), (x + s, 2 * s, z + s), box_n):
            add(p, m)
    verts, norms, tris, tmat = [], [], [], []
    base = 0
    for v, n, t, m in parts:
        verts.append(v)
        norms.append(n)
        tris.append(t + base)
        tmat.append(np.full(len(t), m, np.uint32))
        base += len(v)
    sc.set_mesh(np.concatenate(verts).astype(np.float32), np.concatenate(tris).astype(np.uint32),
                np.concatenate(tmat), np.concatenate(norms).astype(np.float32))
    # one quad area light under the ceiling, facing down, registered once
    anchor = (L * 0.5 - 250.0 * S, Hh - 2.0 * S, Wd * 0.5 - 150.0 * S)
    v1, v2 = (500.0 * S, 0.0, 0.0), (0.0, 0.0, 300.0 * S)   # Light normal = normalize(cross(v1, v2)) = -y
    light = scenes.AreaLight((3.0e5, 2.8e5, 2.4e5), anchor, v1, v2)
    sc.lights.append(light)
    em = sc.add_material(scenes.DiffuseEmitter(light.power, 1.0, light.inverse_area))
    sc.add_parallelogram(light.position, light.v1, light.v2, em)
    sc.aabb_min = np.array([-5, -5, -5], np.float32)
    sc.aabb_max = np.array([L + 5, Hh + 5, Wd + 5], np.float32)
    sc.default_camera = scenes.Camera(np.array([150.0 * S, 600.0 * S, Wd * 0.5], np.float32),
                                      np.array([L, 450.0 * S, Wd * 0.5], np.float32),
                                      np.array([0.0, 1.0, 0.0], np.float32), 60.0, 45.0, 0.0)
    return sc


def synthetic_conference(grid_n=80, box_n=4, seed=43, scale=1.0 / 3.0) -> scenes.Scene:
    """Seeded "Conference-class" room (BASELINE configs[4] stand-in, SURVEY 8(d) C5: ~331k
    triangles): tessellated floor, ceiling and walls, rows of tables with chairs, a podium and a
    projection wall, ceiling light fixtures; Lambert materials; two quad area lights, each
    registered once."""
    rng = np.random.default_rng(seed)
    S = scale
    L, Wd, Hh = 3200.0 * S, 2000.0 * S, 900.0 * S
    sc = scenes.Scene("SyntheticConference")
    mats = {
        "floor": sc.add_material(scenes.Diffuse((0.35, 0.30, 0.28))),
        "wall": sc.add_material(scenes.Diffuse((0.80, 0.78, 0.72))),
        "ceiling": sc.add_material(scenes.Diffuse((0.85, 0.85, 0.85))),
        "table": sc.add_material(scenes.Diffuse((0.55, 0.38, 0.22))),
        "chair": sc.add_material(scenes.Diffuse((0.15, 0.18, 0.45))),
        "metal": sc.add_material(scenes.Diffuse((0.6, 0.6, 0.62))),
        "screen": sc.add_material(scenes.Diffuse((0.9, 0.9, 0.9))),
    }
    parts = []

    def add(vnt, m):
        parts.append((*vnt, m))

    def box(lo, hi, m, n=box_n):
        for p in _box(lo, hi, n):
            add(p, m)

    add(_grid((0, 0, 0), (0, 0, Wd), (L, 0, 0), grid_n, grid_n), mats["floor"])
    add(_grid((0, Hh, 0), (L, 0, 0), (0, 0, Wd), grid_n, grid_n), mats["ceiling"])
    add(_grid((0, 0, Wd), (0, Hh, 0), (L, 0, 0), grid_n, grid_n), mats["wall"])
    add(_grid((0, 0, 0), (L, 0, 0), (0, Hh, 0), grid_n, grid_n), mats["wall"])
    add(_grid((0, 0, 0), (0, Hh, 0), (0, 0, Wd), grid_n, grid_n), mats["screen"])  # projection wall, x=0
    add(_grid((L, 0, 0), (0, 0, Wd), (0, Hh, 0), grid_n, grid_n), mats["wall"])
    # podium in front of the projection wall
    box((150 * S, 0, Wd * 0.5 - 150 * S), (300 * S, 110 * S, Wd * 0.5 + 150 * S), mats["table"], 8)
    # rows of tables, each with chairs on the far side
    nrow, ntab = 7, 3
    for i in range(nrow):
        x0 = 700 * S + i * 330 * S
        for j in range(ntab):
            z0 = 200 * S + j * 560 * S
            tl, tw, th = 120 * S, 480 * S, 75 * S
            box((x0, th - 5 * S, z0), (x0 + tl, th, z0 + tw), mats["table"], 8)
            for lx, lz in ((x0 + 5 * S, z0 + 5 * S), (x0 + tl - 10 * S, z0 + 5 * S),
                           (x0 + 5 * S, z0 + tw - 10 * S), (x0 + tl - 10 * S, z0 + tw - 10 * S)):
                box((lx, 0, lz), (lx + 5 * S, th - 5 * S, lz + 5 * S), mats["metal"])
            for c in range(8):
                cz = z0 + (c + 0.5) * tw / 8 + rng.uniform(-4, 4) * S
                cx = x0 + tl + 50 * S + rng.uniform(-8, 8) * S
                sw = 45 * S
                box((cx - sw / 2, 45 * S, cz - sw / 2), (cx + sw / 2, 50 * S, cz + sw / 2), mats["chair"])   # seat
                box((cx + sw / 2, 50 * S, cz - sw / 2), (cx + sw / 2 + 5 * S, 95 * S, cz + sw / 2), mats["chair"])  # back
                for dx, dz in ((-1, -1), (1, -1), (-1, 1), (1, 1)):
                    lx, lz = cx + dx * (sw / 2 - 3 * S), cz + dz * (sw / 2 - 3 * S)
                    box((lx - 2 * S, 0, lz - 2 * S), (lx + 2 * S, 45 * S, lz + 2 * S), mats["metal"])
    # ceiling light fixtures
    for i in range(6):
        for j in range(4):
            x, z = (500 + i * 450) * S, (300 + j * 470) * S
            box((x - 60 * S, Hh - 25 * S, z - 20 * S), (x + 60 * S, Hh, z + 20 * S), mats["metal"], 10)
    verts, norms, tris, tmat = [], [], [], []
    base = 0
    for v, n, t, m in parts:
        verts.append(v)
        norms.append(n)
        tris.append(t + base)
        tmat.append(np.full(len(t), m, np.uint32))
        base += len(v)
    sc.set_mesh(np.concatenate(verts).astype(np.float32), np.concatenate(tris).astype(np.uint32),
                np.concatenate(tmat), np.concatenate(norms).astype(np.float32))
    for ax in (L * 0.35, L * 0.7):  # two quad area lights under the ceiling, facing down
        anchor = (ax - 200.0 * S, Hh - 30.0 * S, Wd * 0.5 - 150.0 * S)
        light = scenes.AreaLight((2.0e5, 1.9e5, 1.7e5), anchor, (400.0 * S, 0.0, 0.0), (0.0, 0.0, 300.0 * S))
        sc.lights.append(light)
        em = sc.add_material(scenes.DiffuseEmitter(light.power, 1.0, light.inverse_area))
        sc.add_parallelogram(light.position, light.v1, light.v2, em)
    sc.aabb_min = np.array([-5, -5, -5], np.float32)
    sc.aabb_max = np.array([L + 5, Hh + 5, Wd + 5], np.float32)
    sc.default_camera = scenes.Camera(np.array([L - 100.0 * S, 300.0 * S, Wd * 0.5], np.float32),
                                      np.array([0.0, 250.0 * S, Wd * 0.5], np.float32),
                                      np.array([0.0, 1.0, 0.0], np.float32), 70.0, 45.0, 0.0)
    return sc


def _checker(n, cells, c0, c1, seed):
    """RGBA8 checkerboard with per-texel noise (uint8 [n, n, 4])."""
    rng = np.random.default_rng(seed)
    i, j = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    pick = ((i * cells // n) + (j * cells // n)) % 2
    rgb = np.where(pick[..., None] == 0, np.float64(c0), np.float64(c1)) * 255.0
    rgb = np.clip(rgb + rng.uniform(-12, 12, rgb.shape), 0, 255)
    return np.concatenate([rgb, np.full((n, n, 1), 255.0)], -1).astype(np.uint8)


def _bump_normal_map(n, freq):
    """Tangent-space normal map of a sinusoidal height field, encoded (N+1)/2*255."""
    y, x = np.meshgrid(np.arange(n) / n, np.arange(n) / n, indexing="ij")
    dhx = 0.6 * np.cos(2 * np.pi * freq * x) * np.sin(2 * np.pi * freq * y)
    dhy = 0.6 * np.sin(2 * np.pi * freq * x) * np.cos(2 * np.pi * freq * y)
    nrm = np.stack([-dhx, -dhy, np.ones_like(x)], -1)
    nrm /= np.linalg.norm(nrm, axis=-1, keepdims=True)
    rgb = np.round((nrm + 1.0) * 0.5 * 255.0)
    return np.concatenate([rgb, np.full((n, n, 1), 255.0)], -1).astype(np.uint8)


def textured_room(grid_n=6, tex_n=32, seed=7) -> scenes.Scene:
    """Small triangle-mesh room whose walls use the Texture material
    (material/Texture.cu): checker diffuse maps sampled with wrapping
    texcoords (uv up to 3), vertex normals, tangents/bitangents and a
    normal map on the floor; a textured parallelogram (no texcoord attribute)
    and a Diffuse block for contrast; one quad area light.  Procedural and
    seeded; exercises every Texture code path of the hot passes."""
    sc = scenes.Scene("TexturedRoom")
    L, Hh = 10.0, 8.0
    t_floor = sc.add_texture(_checker(tex_n, 4, (0.85, 0.8, 0.7), (0.25, 0.3, 0.5), seed),
                             _bump_normal_map(tex_n, 2))
    t_wall = sc.add_texture(_checker(tex_n, 2, (0.8, 0.2, 0.15), (0.9, 0.85, 0.8), seed + 1))
    t_back = sc.add_texture(_checker(tex_n // 2, 8, (0.2, 0.7, 0.25), (0.85, 0.85, 0.85), seed + 2))
    m_floor = sc.add_material(scenes.Texture(t_floor))
    m_wall = sc.add_material(scenes.Texture(t_wall))
    m_back = sc.add_material(scenes.Texture(t_back))
    m_white = sc.add_material(scenes.Diffuse(0.75))
    verts, norms, uvs, tans, btans, tris, tmat = [], [], [], [], [], [], []
    base = 0

    def add(origin, du, dv, m, rep):
        nonlocal base
        v, n, t = _grid(origin, du, dv, grid_n, grid_n)
        uu, vv = np.meshgrid(np.linspace(0, rep, grid_n + 1), np.linspace(0, rep, grid_n + 1), indexing="ij")
        verts.append(v)
        norms.append(n)
        uvs.append(np.stack([uu, vv], -1).reshape(-1, 2))
        tans.append(np.broadcast_to(np.float64(du) / np.linalg.norm(du), v.shape))
        btans.append(np.broadcast_to(np.float64(dv) / np.linalg.norm(dv), v.shape))
        tris.append(t + base)
        tmat.append(np.full(len(t), m, np.uint32))
        base += len(v)

    add((0, 0, 0), (0, 0, L), (L, 0, 0), m_floor, 3.0)       # floor, +y
    add((0, Hh, 0), (L, 0, 0), (0, 0, L), m_white, 1.0)      # ceiling, -y
    add((0, 0, L), (0, Hh, 0), (L, 0, 0), m_back, 2.0)       # back wall, -z
    add((0, 0, 0), (0, Hh, 0), (0, 0, L), m_wall, 1.5)       # x=0, +x
    add((L, 0, 0), (0, 0, L), (0, Hh, 0), m_wall, 1.5)       # x=L, -x
    for p in _box((6.0, 0.0, 5.5), (8.0, 2.5, 7.5), 2):
        v, n, t = p
        verts.append(v)
        norms.append(n)
        uvs.append(np.zeros((len(v), 2)))
        tans.append(np.tile([1.0, 0.0, 0.0], (len(v), 1)))
        btans.append(np.tile([0.0, 1.0, 0.0], (len(v), 1)))
        tris.append(t + base)
        tmat.append(np.full(len(t), m_white, np.uint32))
        base += len(v)
    cat = lambda a: np.concatenate(a).astype(np.float32)
    sc.set_mesh(cat(verts), np.concatenate(tris).astype(np.uint32), np.concatenate(tmat), cat(norms),
                texcoords=cat(uvs), tangents=cat(tans), bitangents=cat(btans))
    sc.add_parallelogram((1.5, 0.01, 6.0), (0.0, 0.0, 2.5), (2.5, 0.0, 0.0), m_wall)   # textured quad, +y
    light = scenes.AreaLight((1.2e3, 1.1e3, 0.9e3), (6.0, Hh - 0.01, 4.0), (0.0, 0.0, 2.0), (-2.0, 0.0, 0.0))
    sc.lights.append(light)
    em = sc.add_material(scenes.DiffuseEmitter(light.power, 1.0, light.inverse_area))
    sc.add_parallelogram(light.position, light.v1, light.v2, em)
    sc.aabb_min = np.array([-0.1, -0.1, -0.1], np.float32)
    sc.aabb_max = np.array([L + 0.1, Hh + 0.1, L + 0.1], np.float32)
    sc.default_camera = scenes.Camera(np.array([5.0, 4.0, -6.0], np.float32), np.array([5.0, 3.0, 5.0], np.float32),
                                      np.array([0.0, 1.0, 0.0], np.float32), 50.0, 50.0, 0.0)
    return sc
