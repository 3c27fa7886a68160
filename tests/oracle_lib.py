"""Loader for the CPU oracle (oracle/liborx_oracle.so) — TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from oppositerenderer_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "liborx_oracle.so")
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        lib = C.CDLL(LIB)
        _abi.declare_common(lib, "orc")
        lib.orc_create.argtypes = [C.POINTER(_abi.OrxConfig), C.POINTER(C.c_void_p)]
        lib.orc_create.restype = C.c_int
        lib.orc_xorwow_init.argtypes = [C.c_uint64, C.POINTER(C.c_uint32)]
        lib.orc_xorwow_next.argtypes = [C.POINTER(C.c_uint32)]
        lib.orc_xorwow_next.restype = C.c_uint32
        lib.orc_uniform.argtypes = [C.POINTER(C.c_uint32)]
        lib.orc_uniform.restype = C.c_float
        lib.orc_trace_closest.argtypes = [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_float,
                                          C.c_float, C.POINTER(C.c_float)]
        lib.orc_trace_closest.restype = C.c_int32
        lib.orc_trace_any.argtypes = [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_float, C.c_float]
        lib.orc_trace_any.restype = C.c_int32
        lib.orc_sample_unit_hemisphere_cos.argtypes = [C.POINTER(C.c_float), C.c_float, C.c_float, C.POINTER(C.c_float)]
        lib.orc_sample_unit_hemisphere.argtypes = [C.POINTER(C.c_float), C.c_float, C.c_float, C.POINTER(C.c_float)]
        lib.orc_camera_setup.argtypes = [C.POINTER(_abi.OrxCamera)] + [C.POINTER(C.c_float)] * 3
        lib.orc_set_threads.argtypes = [C.c_int]
        _lib = lib
    return _lib


class OracleRenderer:
    """Same call surface as oppositerenderer_amd.renderer.OptixRenderer."""

    def __init__(self, cfg=None):
        self.lib = load()
        self.cfg = cfg or _abi.default_config()
        h = C.c_void_p()
        st = self.lib.orc_create(C.byref(self.cfg), C.byref(h))
        assert st == 0, st
        self.h = h
        self.width = self.height = 0

    def _check(self, st):
        if st != 0:
            raise RuntimeError(self.lib.orc_last_error(self.h).decode())

    def init_scene(self, scene):
        self._scene_abi = scene.to_abi()
        self._scene_ref = scene
        self._check(self.lib.orc_init_scene(self.h, C.byref(self._scene_abi)))

    def render_next_iteration(self, it, local_it, radius, request):
        self.width, self.height = request.width, request.height
        self._check(self.lib.orc_render_next_iteration(self.h, it, local_it, radius, 1, C.byref(request)))

    def read_buffer(self, buf_id, dtype=np.float32):
        n = C.c_size_t()
        self._check(self.lib.orc_read_buffer(self.h, buf_id, None, 0, C.byref(n)))
        out = np.empty(n.value // np.dtype(dtype).itemsize, dtype=dtype)
        self._check(self.lib.orc_read_buffer(self.h, buf_id, out.ctypes.data, n.value, C.byref(n)))
        return out

    def output(self):
        out = np.empty(self.width * self.height * 3, np.float32)
        self._check(self.lib.orc_get_output(self.h, out.ctypes.data, out.nbytes))
        return out.reshape(self.height, self.width, 3)

    def stats(self):
        s = _abi.OrxStats()
        self._check(self.lib.orc_get_stats(self.h, C.byref(s)))
        return s

    def close(self):
        if self.h:
            self.lib.orc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
