"""Python mirror of OppositeRenderer's `OptixRenderer` (RenderEngine/renderer/OptixRenderer.h:21-43)
and `StandaloneRenderManager`'s progressive loop (Standalone/StandaloneRenderManager.cpp:75-140),
bound to liborx.so through the C ABI in include/orx.h.

There is no CPU fallback: if liborx.so is missing or no HIP device is present
every entry point raises.  The oracle under oracle/ is test infrastructure and
is never imported here.
"""
from __future__ import annotations

import ctypes as C
import math
import os

import numpy as np

from . import _abi
from .scenes import Camera, Scene

_HERE = os.path.dirname(os.path.abspath(__file__))
# ORX_LIB selects an alternative in-tree build (e.g. liborx_fp32.so) for A/B measurements
LIB_PATH = os.environ.get("ORX_LIB") or os.path.join(_HERE, "liborx.so")
_lib = None


class OrxError(RuntimeError):
    """Raised where the reference throws std::exception (OptixRenderer.cpp:816-820)."""

    def __init__(self, status, message):
        super().__init__(f"[orx status {status}] {message}")
        self.status = status


def load_library(path: str = LIB_PATH):
    """Load liborx.so (built in-tree by __graft_entry__.build / `make -C oppositerenderer_amd/csrc`)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise OrxError(_abi.ORX_ERR_STATE,
                       f"liborx.so not found at {path}; build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = C.CDLL(path)
    _abi.declare_common(lib, "orx")
    lib.orx_default_config.argtypes = [C.POINTER(_abi.OrxConfig)]
    lib.orx_default_config.restype = None
    lib.orx_create.argtypes = [C.c_int, C.POINTER(_abi.OrxConfig), C.POINTER(C.c_void_p)]
    lib.orx_create.restype = C.c_int
    lib.orx_get_output_device.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    lib.orx_get_output_device.restype = C.c_int
    for name in ("orx_width", "orx_height", "orx_emitted_photons_per_iteration"):
        getattr(lib, name).argtypes = [C.c_void_p]
        getattr(lib, name).restype = C.c_uint32
    lib.orx_output_bytes.argtypes = [C.c_void_p]
    lib.orx_output_bytes.restype = C.c_size_t
    lib.orx_set_shard.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
    lib.orx_set_shard.restype = C.c_int
    lib.orx_reset_timing.argtypes = [C.c_void_p]
    lib.orx_reset_timing.restype = C.c_int
    lib.orx_ppm_pipelined.argtypes = [C.c_void_p]
    lib.orx_ppm_pipelined.restype = C.c_int
    lib.orx_ppm_grid_schedule.argtypes = [C.c_void_p, C.POINTER(C.c_float)]
    lib.orx_ppm_grid_schedule.restype = C.c_int
    lib.orx_set_iteration_pipelining.argtypes = [C.c_void_p, C.c_int]
    lib.orx_set_iteration_pipelining.restype = C.c_int
    lib.orx_stream.argtypes = [C.c_void_p]
    lib.orx_stream.restype = C.c_void_p
    _lib = lib
    return lib


EXPORTED_SYMBOLS = (
    "orx_default_config", "orx_create", "orx_init_scene", "orx_render_next_iteration", "orx_get_output",
    "orx_get_output_device", "orx_width", "orx_height", "orx_output_bytes", "orx_emitted_photons_per_iteration",
    "orx_last_error", "orx_destroy", "orx_read_buffer", "orx_get_stats", "orx_reset_timing", "orx_ppm_pipelined",
    "orx_set_iteration_pipelining", "orx_ppm_grid_schedule",
    "orx_set_shard", "orx_set_ppm_pipeline",
    "orx_stream",
)


class RenderRequestDetails:
    """RenderServerRenderRequestDetails (clientserver/RenderServerRenderRequestDetails.h:15-33)."""

    def __init__(self, camera: Camera, scene_name: str, render_method: int, width: int, height: int,
                 ppm_alpha: float = 2.0 / 3.0):
        self.camera = camera
        self.scene_name = scene_name
        self.render_method = render_method
        self.width = width
        self.height = height
        self.ppm_alpha = ppm_alpha

    def to_abi(self) -> _abi.OrxRequest:
        r = _abi.OrxRequest()
        r.camera = self.camera.to_abi()
        r.method = self.render_method
        r.width = self.width
        r.height = self.height
        r.ppm_alpha = self.ppm_alpha
        return r


class OptixRenderer:
    """Drop-in for the reference's OptixRenderer, HIP/gfx950 underneath.

    initialize(device)                -> OptixRenderer::initialize(ComputeDevice)   (OptixRenderer.cpp:113-400)
    initScene(scene)                  -> OptixRenderer::initScene(IScene&)           (:436-485)
    renderNextIteration(...)          -> OptixRenderer::renderNextIteration          (:507-821)
    getOutputBuffer()                 -> OptixRenderer::getOutputBuffer              (:860-865)
    getWidth/getHeight/getScreenBufferSizeBytes                                      (:850-870)
    """

    PHOTON_LAUNCH_WIDTH = 1024
    PHOTON_LAUNCH_HEIGHT = 1024
    EMITTED_PHOTONS_PER_ITERATION = PHOTON_LAUNCH_WIDTH * PHOTON_LAUNCH_HEIGHT

    def __init__(self, config: _abi.OrxConfig | None = None):
        self._lib = load_library()
        self._cfg = config if config is not None else _abi.default_config()
        self._h = None
        self._initialized = False
        self._scene_abi = None

    # -- error plumbing ------------------------------------------------
    def _check(self, status):
        if status != _abi.ORX_OK:
            msg = self._lib.orx_last_error(self._h).decode() if self._h else "orx call failed"
            raise OrxError(status, msg)

    # -- reference API -------------------------------------------------
    def initialize(self, device: int = 0):
        if self._initialized:
            raise OrxError(_abi.ORX_ERR_STATE, "ERROR: Multiple OptixRenderer::initialize!")
        h = C.c_void_p()
        st = self._lib.orx_create(int(device), C.byref(self._cfg), C.byref(h))
        if st != _abi.ORX_OK:
            raise OrxError(st, f"orx_create failed on HIP device {device}")
        self._h = h
        self._initialized = True
        return self

    def initScene(self, scene: Scene):
        if not self._initialized:
            raise OrxError(_abi.ORX_ERR_STATE, "Cannot initialize scene before OptixRenderer.")
        self._scene_abi = scene.to_abi()
        self._scene = scene
        self._check(self._lib.orx_init_scene(self._h, C.byref(self._scene_abi)))

    def renderNextIteration(self, iterationNumber: int, localIterationNumber: int, PPMRadius: float,
                            createOutput: bool, details: RenderRequestDetails):
        if not self._initialized:
            raise OrxError(_abi.ORX_ERR_STATE, "Traced before OptixRenderer was initialized.")
        req = details.to_abi() if isinstance(details, RenderRequestDetails) else details
        self._check(self._lib.orx_render_next_iteration(self._h, int(iterationNumber), int(localIterationNumber),
                                                         float(PPMRadius), int(bool(createOutput)), C.byref(req)))

    def getOutputBuffer(self, out: np.ndarray | None = None) -> np.ndarray:
        """W*H*3 float32 SUM over local iterations (divide by N to display, RenderWidget.cpp:197)."""
        n = self.getScreenBufferSizeBytes()
        if out is None:
            out = np.empty(n // 4, np.float32)
        assert out.nbytes >= n and out.dtype == np.float32 and out.flags.c_contiguous
        self._check(self._lib.orx_get_output(self._h, out.ctypes.data, out.nbytes))
        return out[: n // 4].reshape(self.getHeight(), self.getWidth(), 3)

    def getOutputBufferDevice(self, dst_ptr: int, nbytes: int):
        """Device-to-device copy of the accumulation buffer (multi-GPU harness)."""
        self._check(self._lib.orx_get_output_device(self._h, C.c_void_p(dst_ptr), nbytes))

    def getWidth(self) -> int:
        return self._lib.orx_width(self._h)

    def getHeight(self) -> int:
        return self._lib.orx_height(self._h)

    def getScreenBufferSizeBytes(self) -> int:
        return self._lib.orx_output_bytes(self._h)

    def emittedPhotonsPerIteration(self) -> int:
        return self._lib.orx_emitted_photons_per_iteration(self._h)

    # -- extensions ----------------------------------------------------
    def set_shard(self, rank: int, world: int):
        self._check(self._lib.orx_set_shard(self._h, rank, world))

    def stream_handle(self) -> int:
        return self._lib.orx_stream(self._h) or 0

    def read_buffer(self, buf_id: int, dtype=np.float32) -> np.ndarray:
        n = C.c_size_t()
        self._check(self._lib.orx_read_buffer(self._h, buf_id, None, 0, C.byref(n)))
        out = np.empty(n.value // np.dtype(dtype).itemsize, dtype=dtype)
        self._check(self._lib.orx_read_buffer(self._h, buf_id, out.ctypes.data, n.value, C.byref(n)))
        return out

    def stats(self) -> _abi.OrxStats:
        s = _abi.OrxStats()
        self._check(self._lib.orx_get_stats(self._h, C.byref(s)))
        return s

    def pipelined(self) -> bool:
        """Whether the last iteration overlapped part of its work with the next one's passes (PPM: the
        gather + output; VCM: the deferred shadow rays + colours)."""
        return bool(self._lib.orx_ppm_pipelined(self._h))

    def grid_schedule(self):
        """The pipelined PPM grid build's schedule (orx_ppm_grid_schedule): (0 synchronous / 1 asynchronous /
        -1 not chosen yet, (photon + grid ms, gather ms) as measured, or zeros)."""
        ms = (C.c_float * 2)()
        mode = self._lib.orx_ppm_grid_schedule(self._h, ms)
        return mode, (float(ms[0]), float(ms[1]))

    def set_iteration_pipelining(self, mode: int):
        """Single-device PPM pipelining and VCM shadow-ray overlap: 1 on, 0 serial passes, -1 the
        ORX_PIPELINE default."""
        self._check(self._lib.orx_set_iteration_pipelining(self._h, mode))

    def reset_timing(self):
        """Start a new timed region for stats().pass_ms / *_total (HIP events, no host timing)."""
        self._check(self._lib.orx_reset_timing(self._h))

    def destroy(self):
        if self._h:
            self._lib.orx_destroy(self._h)
            self._h = None
            self._initialized = False

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


def next_ppm_radius(radius: float, iteration: int, alpha: float = 2.0 / 3.0) -> float:
    """StandaloneRenderManager.cpp:105-107: r^2 <- r^2 (i + alpha) / (i + 1), in double."""
    r2 = radius * radius
    return math.sqrt(r2 * (iteration + alpha) / float(iteration + 1))


class StandaloneRenderManager:
    """Headless restatement of Standalone/StandaloneRenderManager.cpp:55-140: one
    renderNextIteration per call, PPM radius schedule with alpha = 2/3, output
    fetched every `output_every` iterations (5 in the reference)."""

    PPM_ALPHA = 2.0 / 3.0

    def __init__(self, renderer, scene: Scene, method: int, width: int, height: int, camera: Camera | None = None,
                 output_every: int = 5):
        self.renderer = renderer
        self.scene = scene
        self.camera = camera or scene.default_camera
        self.camera.set_aspect_ratio(float(np.float32(width) / np.float32(height)))
        self.details = RenderRequestDetails(self.camera, scene.name, method, width, height, self.PPM_ALPHA)
        self.radius = scene.initial_ppm_radius()
        self.iteration = 0
        self.output_every = output_every
        self._compiled = False

    def render_next_iteration(self):
        if not self._compiled:
            self.renderer.initScene(self.scene)
            self._compiled = True
        out = self.iteration % self.output_every == 0
        self.renderer.renderNextIteration(self.iteration, self.iteration, self.radius, out, self.details)
        self.radius = next_ppm_radius(self.radius, self.iteration, self.PPM_ALPHA)
        self.iteration += 1
