"""Loader for the CPU oracle (oracle/liborx_oracle.so) — TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from oppositerenderer_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# ORACLE_LIB: another build of the same sources (the ASan/UBSan one, tests/test_sanitizers.py)
LIB = os.environ.get("ORACLE_LIB") or os.path.join(ROOT, "oracle", "liborx_oracle.so")
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


class OracleShard:
    """CPU backend for oppositerenderer_amd.multigpu.ShardedPPM (gloo tests)."""

    def __init__(self, renderer: OracleRenderer, torch):
        self.r, self.torch = renderer, torch
        lib = renderer.lib
        for name, args, res in (
            ("orc_set_shard", [C.c_void_p, C.c_uint32, C.c_uint32], C.c_int),
            ("orc_ppm_local_passes", [C.c_void_p, C.c_uint64, C.c_uint64, C.c_float, C.c_void_p], C.c_int),
            ("orc_export_hitpoints", [C.c_void_p, C.c_void_p, C.c_size_t], C.c_int),
            ("orc_ppm_gather_external", [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_size_t], C.c_int),
            ("orc_ppm_finish", [C.c_void_p, C.c_void_p, C.c_size_t], C.c_int),
            ("orc_vcm_local_light", [C.c_void_p, C.c_uint64, C.c_uint64, C.c_float, C.c_void_p], C.c_int),
            ("orc_export_vcm_splats", [C.c_void_p, C.c_void_p, C.c_size_t], C.c_int),
            ("orc_vcm_finish", [C.c_void_p, C.c_void_p, C.c_size_t], C.c_int),
            ("orc_ppm_local_trace", [C.c_void_p, C.c_uint64, C.c_uint64, C.c_float, C.c_void_p], C.c_int),
            ("orc_ppm_slab_histogram", [C.c_void_p, C.c_void_p, C.c_uint32], C.c_int),
            ("orc_ppm_slab_pack", [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p,
                                   C.c_uint64, C.c_void_p], C.c_int),
            ("orc_ppm_slab_import", [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32, C.c_uint32,
                                     C.c_uint32, C.c_uint32], C.c_int),
            ("orc_ppm_slab_halo", [C.c_void_p, C.c_uint32, C.c_uint32, C.c_float], C.c_uint32),
        ):
            f = getattr(lib, name)
            f.argtypes, f.restype = args, res
        self.lib = lib

    def set_shard(self, rank, world):
        self.r._check(self.lib.orc_set_shard(self.r.h, rank, world))
        self.rank_world = (rank, world)

    # -- slab mode (orx_set_slab_partition's phases on the oracle) --
    def enable_slab(self):
        pass

    def slot_capacity(self):
        cfg = self.r.cfg
        rank, world = self.rank_world
        prows = (cfg.photon_launch_height - rank + world - 1) // world if cfg.photon_launch_height > rank else 0
        return (cfg.photon_launch_width * prows * cfg.max_photon_deposits,
                cfg.photon_launch_width * cfg.photon_launch_height * cfg.max_photon_deposits)

    def alloc_i32(self, n):
        return self.torch.zeros(n, dtype=self.torch.int32)

    def local_trace(self, it, local_it, radius, request):
        self.r.width, self.r.height = request.width, request.height
        self.r._check(self.lib.orc_ppm_local_trace(self.r.h, it, local_it, radius, C.byref(request)))

    def slab_histogram(self, hist, nb):
        self.r._check(self.lib.orc_ppm_slab_histogram(self.r.h, C.c_void_p(hist.data_ptr()), nb))

    def slab_halo(self, nb, axis, radius):
        return int(self.lib.orc_ppm_slab_halo(self.r.h, nb, axis, radius))

    def slab_pack(self, bin_dest, nb, axis, halo, base, n_records, send):
        bd = np.ascontiguousarray(bin_dest, np.uint8)
        bs = np.ascontiguousarray(base, np.uint32)
        self.r._check(self.lib.orc_ppm_slab_pack(self.r.h, bd.ctypes.data, nb, axis, halo, bs.ctypes.data,
                                                 n_records, C.c_void_p(send.data_ptr())))

    def slab_import(self, recv, n_records, box, axis, nb, own):
        bx = None if box is None else np.ascontiguousarray(box, np.uint32)
        self.r._check(self.lib.orc_ppm_slab_import(self.r.h, C.c_void_p(recv.data_ptr()), n_records,
                                                   None if bx is None else bx.ctypes.data, axis, nb, own[0],
                                                   own[1]))

    def alloc(self, nfloat):
        return self.torch.zeros(nfloat, dtype=self.torch.float32)

    def local_passes(self, it, local_it, radius, request):
        self.r.width, self.r.height = request.width, request.height
        self.r._check(self.lib.orc_ppm_local_passes(self.r.h, it, local_it, radius, C.byref(request)))

    def export_hitpoints(self, t):
        self.r._check(self.lib.orc_export_hitpoints(self.r.h, C.c_void_p(t.data_ptr()), t.numel() * 4))

    def gather_external(self, hp_all, segments, out):
        self.r._check(self.lib.orc_ppm_gather_external(self.r.h, C.c_void_p(hp_all.data_ptr()), segments,
                                                       C.c_void_p(out.data_ptr()), out.numel() * 4))

    def finish(self, ind_local):
        self.r._check(self.lib.orc_ppm_finish(self.r.h, C.c_void_p(ind_local.data_ptr()), ind_local.numel() * 4))

    def render_next(self, it, local_it, radius, request):
        self.r.width, self.r.height = request.width, request.height
        self.r._check(self.lib.orc_render_next_iteration(self.r.h, it, local_it, radius, 1, C.byref(request)))

    def vcm_local_light(self, it, local_it, radius, request):
        self.r.width, self.r.height = request.width, request.height
        self.r._check(self.lib.orc_vcm_local_light(self.r.h, it, local_it, radius, C.byref(request)))

    def export_vcm_splats(self, t):
        self.r._check(self.lib.orc_export_vcm_splats(self.r.h, C.c_void_p(t.data_ptr()), t.numel() * 4))

    def vcm_finish(self, splat_own):
        self.r._check(self.lib.orc_vcm_finish(self.r.h, C.c_void_p(splat_own.data_ptr()), splat_own.numel() * 4))

    def output_local_tensor(self, max_rows):
        t = self.alloc(max_rows * self.r.width * 3)
        n = C.c_size_t()
        self.r._check(self.lib.orc_read_buffer(self.r.h, 6, None, 0, C.byref(n)))
        self.r._check(self.lib.orc_read_buffer(self.r.h, 6, C.c_void_p(t.data_ptr()), t.numel() * 4, C.byref(n)))
        return t
