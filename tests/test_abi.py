"""CPU-side checks of the drop-in boundary: liborx.so loads without a GPU and
exports every symbol include/orx.h declares; the ctypes mirror matches the C
struct layouts (compiled probe); host-side logic (radius schedule, scene
construction) matches the reference formulas."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import numpy as np

from oppositerenderer_amd import _abi, renderer, scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols(header="orx.h"):
    src = open(os.path.join(ROOT, "include", header)).read()
    return sorted(set(re.findall(r"\b(orx_[a-z_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = renderer.load_library()
    syms = declared_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), s
    assert set(renderer.EXPORTED_SYMBOLS) <= set(syms)


def test_library_exports_every_wire_symbol():
    from oppositerenderer_amd import wire
    lib = renderer.load_library()
    syms = declared_symbols("orx_wire.h")
    assert len(syms) >= 19
    for s in syms:
        assert hasattr(lib, s), s
    assert set(wire.WIRE_SYMBOLS) == set(syms)


def test_wire_struct_layouts_match_c():
    from oppositerenderer_amd import wire
    probe = r"""
#include <stdio.h>
#include "orx_wire.h"
int main(void){
 printf("%zu %zu %zu %zu %zu %zu\n", sizeof(orx_wire_request), sizeof(orx_wire_request_info), sizeof(orx_wire_result),
        sizeof(orx_wire_result_info), offsetof(orx_wire_request, ppm_alpha), offsetof(orx_wire_result, output_bytes));
 return 0;}
"""
    d = tempfile.mkdtemp()
    c = os.path.join(d, "w.c")
    exe = os.path.join(d, "w")
    open(c, "w").write(probe)
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
    vals = [int(v) for v in subprocess.check_output([exe]).split()]
    py = [C.sizeof(wire.OrxWireRequest), C.sizeof(wire.OrxWireRequestInfo), C.sizeof(wire.OrxWireResult),
          C.sizeof(wire.OrxWireResultInfo), wire.OrxWireRequest.ppm_alpha.offset, wire.OrxWireResult.output_bytes.offset]
    assert vals == py


def test_no_gpu_create_fails_cleanly():
    lib = renderer.load_library()
    h = C.c_void_p()
    cfg = _abi.default_config()
    st = lib.orx_create(0, C.byref(cfg), C.byref(h))
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if not has_gpu:
        assert st == _abi.ORX_ERR_DEVICE and not h.value


def test_struct_layouts_match_c():
    probe = r"""
#include <stdio.h>
#include <stddef.h>
#include "orx.h"
int main(void){
 printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(orx_camera), sizeof(orx_request), sizeof(orx_material),
        sizeof(orx_light), sizeof(orx_scene), sizeof(orx_config), sizeof(orx_stats), offsetof(orx_stats, pass_ms),
        sizeof(orx_texture), offsetof(orx_scene, textures));
 return 0;}
"""
    d = tempfile.mkdtemp()
    c = os.path.join(d, "p.c")
    exe = os.path.join(d, "p")
    open(c, "w").write(probe)
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
    vals = [int(v) for v in subprocess.check_output([exe]).split()]
    py = [C.sizeof(_abi.OrxCamera), C.sizeof(_abi.OrxRequest), C.sizeof(_abi.OrxMaterial), C.sizeof(_abi.OrxLight),
          C.sizeof(_abi.OrxScene), C.sizeof(_abi.OrxConfig), C.sizeof(_abi.OrxStats), _abi.OrxStats.pass_ms.offset,
          C.sizeof(_abi.OrxTexture), _abi.OrxScene.textures.offset]
    assert vals == py


def test_ppm_radius_schedule():
    """StandaloneRenderManager.cpp:105-107, alpha = 2/3."""
    r = 7.5375776
    r2 = r * r
    for i in range(10):
        r = renderer.next_ppm_radius(r, i)
        r2 = r2 * (i + 2.0 / 3.0) / (i + 1)
        assert abs(r * r - r2) < 1e-9 * r2


def test_cornell_initial_radius():
    """IScene::getSceneInitialPPMRadiusEstimate on Cornell's AABB (7.5376)."""
    assert abs(scenes.cornell().initial_ppm_radius() - 7.5376) < 1e-3


def test_scene_factory_builtins():
    for name in ("Cornell", "CornellSmall", "CornellSmallNoBlocks", "CornellSmallLargeSphere", "CornellSmallSmallSpheres",
                 "CornellSmallLightUpwards", "CornellSmallPointDistant", "CornellSmallPointTest"):
        sc = scenes.scene_by_name(name)
        assert sc.lights and sc.num_primitives > 0
        abi = sc.to_abi()
        assert abi.n_lights == len(sc.lights)
