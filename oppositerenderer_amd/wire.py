"""Client/server distribution of OppositeRenderer, MI355X-side.

The reference farms iterations out to render servers over Qt TCP
(Client/DistributedApplication.cpp:96-122, Server/server/RenderServer.cpp:93-150):
the client sends RenderServerRenderRequests (a run of iteration numbers with
their precomputed PPM radii), a server renders the run with local iteration
numbers 0..n-1 and answers with a RenderResultPacket (its output buffer, the
sum over the run), and the client merges packets in iteration order
(Client/client/RenderResultPacketReceiver.cpp).  Here the same frames -- byte
for byte the reference's QDataStream layout, encoded and merged by liborx.so
(include/orx_wire.h, oppositerenderer_amd/csrc/orx_wire.cpp) -- travel over
torch.distributed point-to-point messages (RCCL / gloo, so across nodes over
RoCE/IB instead of TCP sockets): rank 0 is the client, every other rank a
render server driving one GPU.

Classes mirror the reference's names: RenderServerRenderRequest,
RenderServerRenderRequestDetails, RenderResultPacket,
RenderResultPacketReceiver, and the client's request generator.
"""
from __future__ import annotations

import ctypes as C
import os
import math
import time
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from . import _abi
from .renderer import OrxError, load_library


# --- C ABI (include/orx_wire.h) -------------------------------------------
class OrxWireRequest(C.Structure):
    _fields_ = [("sequence_number", C.c_uint64), ("n_iterations", C.c_uint32), ("n_radii", C.c_uint32),
                ("iteration_numbers", C.POINTER(C.c_uint64)), ("ppm_radii", C.POINTER(C.c_double)),
                ("camera", _abi.OrxCamera), ("scene_name", C.c_void_p), ("scene_name_len", C.c_uint32),
                ("render_method", C.c_uint32), ("width", C.c_uint32), ("height", C.c_uint32),
                ("ppm_alpha", C.c_double)]


class OrxWireRequestInfo(C.Structure):
    _fields_ = [("frame_bytes", C.c_uint64), ("n_iterations", C.c_uint32), ("n_radii", C.c_uint32),
                ("scene_name_len", C.c_uint32), ("scene_name_null", C.c_int32)]


class OrxWireResult(C.Structure):
    _fields_ = [("sequence_number", C.c_uint64), ("n_iterations", C.c_uint32), ("reserved", C.c_uint32),
                ("iteration_numbers", C.POINTER(C.c_uint64)), ("render_time_seconds", C.c_float),
                ("total_time_seconds", C.c_float), ("output", C.POINTER(C.c_float)), ("output_bytes", C.c_uint64)]


class OrxWireResultInfo(C.Structure):
    _fields_ = [("frame_bytes", C.c_uint64), ("n_iterations", C.c_uint32), ("reserved", C.c_uint32),
                ("output_bytes", C.c_uint64)]


WIRE_SYMBOLS = (
    "orx_wire_request_bytes", "orx_wire_encode_request", "orx_wire_peek_request", "orx_wire_decode_request",
    "orx_wire_result_bytes", "orx_wire_encode_result", "orx_wire_peek_result", "orx_wire_decode_result",
    "orx_receiver_create", "orx_receiver_destroy", "orx_receiver_push", "orx_receiver_push_encoded",
    "orx_receiver_front", "orx_receiver_iteration_number", "orx_receiver_next_expected",
    "orx_receiver_backbuffer_iterations", "orx_receiver_backbuffer_bytes", "orx_receiver_peak_backbuffer_bytes",
    "orx_receiver_backbuffer_is_not_filled",
)

_declared = False
_wire_lib = None


def _lib():
    """liborx.so (the wire codec and receiver are host code in it), or ORX_WIRE_LIB: a library of the codec
    alone, e.g. the ASan/UBSan build tests/test_sanitizers.py runs the wire tests against"""
    global _declared, _wire_lib
    if os.environ.get("ORX_WIRE_LIB"):
        if _wire_lib is None:
            _wire_lib = C.CDLL(os.environ["ORX_WIRE_LIB"])
        lib = _wire_lib
    else:
        lib = load_library()
    if _declared:
        return lib
    P, u64, u32, i32 = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int32
    sig = {
        "orx_wire_request_bytes": ([C.POINTER(OrxWireRequest)], u64),
        "orx_wire_encode_request": ([C.POINTER(OrxWireRequest), P, u64, C.POINTER(u64)], C.c_int),
        "orx_wire_peek_request": ([P, u64, C.POINTER(OrxWireRequestInfo)], C.c_int),
        "orx_wire_decode_request": ([P, u64, C.POINTER(OrxWireRequest), C.POINTER(u64), C.POINTER(C.c_double), P],
                                    C.c_int),
        "orx_wire_result_bytes": ([C.POINTER(OrxWireResult)], u64),
        "orx_wire_encode_result": ([C.POINTER(OrxWireResult), P, u64, C.POINTER(u64)], C.c_int),
        "orx_wire_peek_result": ([P, u64, C.POINTER(OrxWireResultInfo)], C.c_int),
        "orx_wire_decode_result": ([P, u64, C.POINTER(OrxWireResult), C.POINTER(u64), C.POINTER(C.c_float)], C.c_int),
        "orx_receiver_create": ([i32, C.POINTER(P)], C.c_int),
        "orx_receiver_destroy": ([P], None),
        "orx_receiver_push": ([P, C.POINTER(OrxWireResult), u64, C.POINTER(i32)], C.c_int),
        "orx_receiver_push_encoded": ([P, P, u64, u64, C.POINTER(i32)], C.c_int),
        "orx_receiver_front": ([P, C.POINTER(u64)], C.POINTER(C.c_float)),
        "orx_receiver_iteration_number": ([P], u64),
        "orx_receiver_next_expected": ([P], u64),
        "orx_receiver_backbuffer_iterations": ([P], u32),
        "orx_receiver_backbuffer_bytes": ([P], u64),
        "orx_receiver_peak_backbuffer_bytes": ([P], u64),
        "orx_receiver_backbuffer_is_not_filled": ([P, u64], i32),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    _declared = True
    return lib


def _check(status: int, what: str):
    if status != _abi.ORX_OK:
        raise OrxError(status, what)



# --- messages ---------------------------------------------------------------
@dataclass
class RenderServerRenderRequestDetails:
    """clientserver/RenderServerRenderRequestDetails.h:15-33 (camera as the 12 streamed floats)."""
    camera: Sequence[float] = (0, 0, 0, 0, 0, -1, 0, 1, 0, 60, 60, 0)
    scene_name: Optional[bytes] = b""
    render_method: int = _abi.PROGRESSIVE_PHOTON_MAPPING
    width: int = 0
    height: int = 0
    ppm_alpha: float = 2.0 / 3.0

    @classmethod
    def from_camera(cls, camera, scene_name, render_method, width, height, ppm_alpha=2.0 / 3.0):
        vals = [*map(float, camera.eye), *map(float, camera.lookat), *map(float, camera.up),
                float(camera.hfov), float(camera.vfov), float(camera.aperture)]
        name = scene_name.encode() if isinstance(scene_name, str) else scene_name
        return cls(vals, name, render_method, width, height, ppm_alpha)

    def camera_abi(self) -> _abi.OrxCamera:
        c = _abi.OrxCamera()
        v = [float(x) for x in self.camera]
        c.eye[:] = v[0:3]
        c.lookat[:] = v[3:6]
        c.up[:] = v[6:9]
        c.hfov, c.vfov, c.aperture = v[9], v[10], v[11]
        return c


@dataclass
class RenderServerRenderRequest:
    """clientserver/RenderServerRenderRequest.h:13-37."""
    sequence_number: int
    iteration_numbers: List[int]
    ppm_radii: List[float]
    details: RenderServerRenderRequestDetails = field(default_factory=RenderServerRenderRequestDetails)

    def getSequenceNumber(self) -> int:
        return self.sequence_number

    def getIterationNumbers(self) -> List[int]:
        return self.iteration_numbers

    def getPPMRadii(self) -> List[float]:
        return self.ppm_radii

    def getNumIterations(self) -> int:
        return len(self.iteration_numbers)

    def getFirstIterationNumber(self) -> int:
        return self.iteration_numbers[0]

    def getDetails(self) -> RenderServerRenderRequestDetails:
        return self.details

    def encode(self) -> bytes:
        lib = _lib()
        its = (C.c_uint64 * max(1, len(self.iteration_numbers)))(*self.iteration_numbers)
        rad = (C.c_double * max(1, len(self.ppm_radii)))(*self.ppm_radii)
        r = OrxWireRequest()
        r.sequence_number = self.sequence_number
        r.n_iterations, r.n_radii = len(self.iteration_numbers), len(self.ppm_radii)
        r.iteration_numbers, r.ppm_radii = its, rad
        r.camera = self.details.camera_abi()
        name = self.details.scene_name
        name_buf = C.create_string_buffer(bytes(name or b""), max(1, len(name or b"")))
        r.scene_name = C.cast(name_buf, C.c_void_p) if name is not None else None
        r.scene_name_len = len(name or b"")
        r.render_method = self.details.render_method & 0xFFFFFFFF
        r.width, r.height, r.ppm_alpha = self.details.width, self.details.height, self.details.ppm_alpha
        n = lib.orx_wire_request_bytes(C.byref(r))
        out = C.create_string_buffer(n)
        written = C.c_uint64()
        _check(lib.orx_wire_encode_request(C.byref(r), out, n, C.byref(written)), "encode request")
        return out.raw[:written.value]

    @classmethod
    def decode(cls, data: bytes) -> "RenderServerRenderRequest":
        lib = _lib()
        src = C.create_string_buffer(bytes(data), max(1, len(data)))
        info = OrxWireRequestInfo()
        _check(lib.orx_wire_peek_request(src, len(data), C.byref(info)), "truncated or malformed request frame")
        its = (C.c_uint64 * max(1, info.n_iterations))()
        rad = (C.c_double * max(1, info.n_radii))()
        name = C.create_string_buffer(max(1, info.scene_name_len))
        r = OrxWireRequest()
        _check(lib.orx_wire_decode_request(src, len(data), C.byref(r), its, rad, name), "decode request")
        c = r.camera
        cam = [*c.eye, *c.lookat, *c.up, c.hfov, c.vfov, c.aperture]
        scene = None if info.scene_name_null else name.raw[:info.scene_name_len]
        det = RenderServerRenderRequestDetails(cam, scene, r.render_method, r.width, r.height, r.ppm_alpha)
        return cls(r.sequence_number, list(its[:info.n_iterations]), list(rad[:info.n_radii]), det)


@dataclass
class RenderResultPacket:
    """clientserver/RenderResultPacket.h:19-48: a server's output for a run of iterations."""
    sequence_number: int
    iteration_numbers: List[int]
    output: np.ndarray
    render_time_seconds: float = 0.0
    total_time_seconds: float = 0.0

    def getSequenceNumber(self) -> int:
        return self.sequence_number

    def getIterationNumbersInPacket(self) -> List[int]:
        return self.iteration_numbers

    def getNumIterationsInPacket(self) -> int:
        return len(self.iteration_numbers)

    def getFirstIterationNumber(self) -> int:
        return self.iteration_numbers[0]

    def getLastIterationNumber(self) -> int:
        return self.iteration_numbers[-1]

    def getOutput(self) -> np.ndarray:
        return self.output

    def _abi(self):
        out = np.ascontiguousarray(self.output, dtype=np.float32)
        its = (C.c_uint64 * max(1, len(self.iteration_numbers)))(*self.iteration_numbers)
        p = OrxWireResult()
        p.sequence_number = self.sequence_number
        p.n_iterations = len(self.iteration_numbers)
        p.iteration_numbers = its
        p.render_time_seconds = self.render_time_seconds
        p.total_time_seconds = self.total_time_seconds
        p.output = out.ctypes.data_as(C.POINTER(C.c_float))
        p.output_bytes = out.nbytes
        return p, (out, its)

    def encode(self) -> bytes:
        lib = _lib()
        p, keep = self._abi()
        n = lib.orx_wire_result_bytes(C.byref(p))
        buf = np.empty(n, dtype=np.uint8)
        written = C.c_uint64()
        _check(lib.orx_wire_encode_result(C.byref(p), buf.ctypes.data_as(C.c_void_p), n, C.byref(written)),
               "encode result")
        return buf[:written.value].tobytes()

    @classmethod
    def decode(cls, data) -> "RenderResultPacket":
        lib = _lib()
        src = np.frombuffer(bytes(data), dtype=np.uint8)
        ptr = src.ctypes.data_as(C.c_void_p)
        info = OrxWireResultInfo()
        _check(lib.orx_wire_peek_result(ptr, src.size, C.byref(info)), "truncated or malformed result frame")
        its = (C.c_uint64 * max(1, info.n_iterations))()
        out = np.empty(info.output_bytes // 4, dtype=np.float32)
        p = OrxWireResult()
        _check(lib.orx_wire_decode_result(ptr, src.size, C.byref(p), its,
                                          out.ctypes.data_as(C.POINTER(C.c_float))), "decode result")
        return cls(p.sequence_number, list(its[:info.n_iterations]), out, p.render_time_seconds,
                   p.total_time_seconds)


class RenderResultPacketReceiver:
    """Client/client/RenderResultPacketReceiver.hxx: merges packets into the front buffer."""

    def __init__(self, render_method: int):
        self._l = _lib()
        h = C.c_void_p()
        _check(self._l.orx_receiver_create(render_method, C.byref(h)), "receiver create")
        self._h = h

    def onRenderResultPacketReceived(self, packet: RenderResultPacket, current_sequence: int) -> bool:
        p, keep = packet._abi()
        acc = C.c_int32()
        _check(self._l.orx_receiver_push(self._h, C.byref(p), current_sequence, C.byref(acc)), "receiver push")
        return bool(acc.value)

    def push_encoded(self, data: bytes, current_sequence: int) -> bool:
        src = np.frombuffer(bytes(data), dtype=np.uint8)
        acc = C.c_int32()
        _check(self._l.orx_receiver_push_encoded(self._h, src.ctypes.data_as(C.c_void_p), src.size,
                                                 current_sequence, C.byref(acc)), "receiver push")
        return bool(acc.value)

    def front(self) -> Optional[np.ndarray]:
        n = C.c_uint64()
        ptr = self._l.orx_receiver_front(self._h, C.byref(n))
        if not ptr:
            return None
        return np.ctypeslib.as_array(ptr, shape=(n.value,)).copy()

    def getIterationNumber(self) -> int:
        return self._l.orx_receiver_iteration_number(self._h)

    def next_expected_iteration(self) -> int:
        return self._l.orx_receiver_next_expected(self._h)

    def getBackBufferNumIterations(self) -> int:
        return self._l.orx_receiver_backbuffer_iterations(self._h)

    def getBackBufferSizeBytes(self) -> int:
        return self._l.orx_receiver_backbuffer_bytes(self._h)

    def getPeakBackBufferSizeBytes(self) -> int:
        return self._l.orx_receiver_peak_backbuffer_bytes(self._h)

    def backBufferIsNotFilled(self, current_sequence: int) -> bool:
        return bool(self._l.orx_receiver_backbuffer_is_not_filled(self._h, current_sequence))

    def close(self):
        if getattr(self, "_h", None):
            self._l.orx_receiver_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RequestGenerator:
    """DistributedApplication::getNextRenderServerRenderRequest (Client/DistributedApplication.cpp:96-122)
    and onSequenceNumberIncremented (:141-149): consecutive iteration numbers with the PPM radius of
    each, r^2 <- r^2 (i + alpha) / (i + 1) in double; a new sequence restarts at iteration 0 and r0."""

    PPM_ALPHA = 2.0 / 3.0

    def __init__(self, initial_radius: float, details: RenderServerRenderRequestDetails, sequence_number: int = 1):
        self.initial_radius = initial_radius
        self.details = details
        self.sequence_number = sequence_number
        self.next_iteration = 0
        self.radius = initial_radius

    def increment_sequence(self):
        self.sequence_number += 1
        self.next_iteration = 0
        self.radius = self.initial_radius

    def next_request(self, num_iterations: int) -> RenderServerRenderRequest:
        its, radii = [], []
        for _ in range(num_iterations):
            its.append(self.next_iteration)
            radii.append(self.radius)
            r2 = self.radius * self.radius
            self.radius = math.sqrt(r2 * (self.next_iteration + self.PPM_ALPHA) / (self.next_iteration + 1))
            self.next_iteration += 1
        return RenderServerRenderRequest(self.sequence_number, its, radii, self.details)


def render_request(renderer, request: RenderServerRenderRequest, details_abi) -> RenderResultPacket:
    """RenderServerRenderer::onNewRenderCommandInQueue + createRenderResultPacket
    (Server/server/RenderServerRenderer.cpp:73-178): the run is rendered with local iteration
    numbers 0..n-1 and the packet carries getOutputBuffer (the sum over the run).  `renderer`
    is anything with renderNextIteration(iteration, local, radius, create_output, details) and
    getOutputBuffer() (OptixRenderer here; the tests' oracle adapter on CPU)."""
    t0 = time.perf_counter()
    n = request.getNumIterations()
    for i in range(n):
        renderer.renderNextIteration(request.iteration_numbers[i], i, request.ppm_radii[i], i == n - 1, details_abi)
    out = np.ascontiguousarray(renderer.getOutputBuffer(), dtype=np.float32).reshape(-1)
    dt = time.perf_counter() - t0
    return RenderResultPacket(request.sequence_number, list(request.iteration_numbers), out, dt, dt)


# --- transport: torch.distributed point-to-point -----------------------------
def send_frame(frame: bytes, dst: int, device=None):
    import torch
    import torch.distributed as dist
    n = torch.tensor([len(frame)], dtype=torch.int64, device=device)
    dist.send(n, dst)
    dist.send(torch.frombuffer(bytearray(frame), dtype=torch.uint8).to(device), dst)


def recv_frame(src: int, device=None) -> bytes:
    import torch
    import torch.distributed as dist
    n = torch.empty(1, dtype=torch.int64, device=device)
    dist.recv(n, src)
    buf = torch.empty(int(n.item()), dtype=torch.uint8, device=device)
    dist.recv(buf, src)
    return buf.cpu().numpy().tobytes()


STOP = b"STOP"


def serve(renderer, details_abi, device=None):
    """Render-server loop (rank > 0): receive request frames from rank 0 until STOP,
    answer each with a result frame (RenderServer::onDataFromClient / onNewRenderResultPacket)."""
    while True:
        frame = recv_frame(0, device)
        if frame == STOP:
            return
        req = RenderServerRenderRequest.decode(frame)
        send_frame(render_request(renderer, req, details_abi).encode(), 0, device)


def run_client(generator: RequestGenerator, world: int, packets_per_server: int, iterations_per_packet: int,
               render_method: int, device=None) -> RenderResultPacketReceiver:
    """The client (rank 0): issue packets_per_server requests of iterations_per_packet iterations to
    each server round-robin, merge every answer through the receiver, then stop the servers."""
    rx = RenderResultPacketReceiver(render_method)
    for _ in range(packets_per_server):
        for s in range(1, world):
            send_frame(generator.next_request(iterations_per_packet).encode(), s, device)
        for s in range(1, world):
            rx.push_encoded(recv_frame(s, device), generator.sequence_number)
    for s in range(1, world):
        send_frame(STOP, s, device)
    return rx
