"""wire_oracle.py -- CPU restatement of OppositeRenderer's client/server wire
format and of the client's iteration-order merge.

TEST INFRASTRUCTURE ONLY.  tests/ use it to check the product codec and
receiver (oppositerenderer_amd/csrc/orx_wire.cpp through liborx.so); nothing
in the product imports it.

What it restates:
  * QDataStream serialisation as the reference uses it (Qt 5 stream version,
    big-endian): quint32/quint64/int are big-endian integers; QByteArray is a
    quint32 length (0xFFFFFFFF for a null array) followed by the bytes;
    QVector<T> is a quint32 count followed by the elements; float and double
    are written with the stream's floating-point precision (Qt >= 4.6): 8-byte
    IEEE doubles for a default-constructed stream, 4-byte floats for a stream
    set to SinglePrecision.
  * RenderServerRenderRequest operator<< (clientserver/RenderServerRenderRequest.cpp:61-74):
    an inner default stream (double precision) holding quint64 sequence
    number, QVector<unsigned long long> iteration numbers, QVector<double> PPM
    radii and the details, framed on the socket stream as
    int(inner size + 2*sizeof(int)) followed by the inner QByteArray.
  * RenderServerRenderRequestDetails operator<< (RenderServerRenderRequestDetails.cpp:56-69):
    its own inner default stream: Camera (Camera.cpp:411-416: eye, lookat,
    up, hfov, vfov, aperture -- floats, hence doubles here), QByteArray scene
    name, quint32 render method, quint32 width, quint32 height, double
    ppmAlpha; written as a QByteArray.
  * RenderResultPacket operator<< (clientserver/RenderResultPacket.cpp:124-146)
    on the socket stream, which both ends set to SinglePrecision
    (RenderServerConnection.cpp:42, RenderServer.cpp:59): quint64 size (the
    bytes that follow it), quint64 sequence number, the iteration numbers
    sorted ascending (qSort), float render time, float total time (4 bytes
    each), QByteArray output (the renderer's raw host float32 buffer).
  * RenderResultPacket::merge (RenderResultPacket.cpp:104-121) and the
    client's RenderResultPacketReceiver (Client/client/RenderResultPacketReceiver.cpp:30-200):
    PPM packets wait in a back buffer sorted by first iteration, adjacent
    runs are merged, and the run that starts at the next expected iteration
    is folded into the front buffer as a running average; path-tracing (and
    VCM) packets are folded in arrival order.  Packets of another sequence
    number are dropped; a newer sequence number resets the receiver.
    All float arithmetic is float32 in the reference's operation order
    (numpy float32, no fused multiply-add).

Parity: the framing is restated from Qt's documented QDataStream format and
the reference's operators; no Qt build exists here, so agreement with bytes
produced by a real Qt is UNPINNED (pinned instead by hand-derived
known-answer vectors in tests/test_wire.py).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

NULL_BYTEARRAY = 0xFFFFFFFF


# --- QDataStream primitives (big-endian) ---------------------------------
def qbytearray(b: Optional[bytes]) -> bytes:
    if b is None:
        return struct.pack(">I", NULL_BYTEARRAY)
    return struct.pack(">I", len(b)) + bytes(b)


def qvector_u64(v: Sequence[int]) -> bytes:
    return struct.pack(">I", len(v)) + b"".join(struct.pack(">Q", int(x)) for x in v)


def qvector_f64(v: Sequence[float]) -> bytes:
    return struct.pack(">I", len(v)) + b"".join(struct.pack(">d", float(x)) for x in v)


def qfloat(x: float, single: bool) -> bytes:
    """operator<<(float): the stream precision decides the width."""
    f = float(np.float32(x))
    return struct.pack(">f", f) if single else struct.pack(">d", f)


@dataclass
class Camera:
    eye: Sequence[float] = (0.0, 0.0, 0.0)
    lookat: Sequence[float] = (0.0, 0.0, -1.0)
    up: Sequence[float] = (0.0, 1.0, 0.0)
    hfov: float = 60.0
    vfov: float = 60.0
    aperture: float = 0.0

    def values(self) -> List[float]:
        return [*self.eye, *self.lookat, *self.up, self.hfov, self.vfov, self.aperture]


@dataclass
class RequestDetails:
    camera: Camera = field(default_factory=Camera)
    scene_name: Optional[bytes] = b""
    render_method: int = 2
    width: int = 0
    height: int = 0
    ppm_alpha: float = 2.0 / 3.0


@dataclass
class RenderRequest:
    sequence_number: int
    iteration_numbers: List[int]
    ppm_radii: List[float]
    details: RequestDetails


def encode_details(d: RequestDetails) -> bytes:
    """RenderServerRenderRequestDetails.cpp:56-69 (inner default stream)."""
    inner = b"".join(qfloat(v, single=False) for v in d.camera.values())
    inner += qbytearray(d.scene_name)
    inner += struct.pack(">III", d.render_method & 0xFFFFFFFF, d.width, d.height)
    inner += struct.pack(">d", float(d.ppm_alpha))
    return qbytearray(inner)


def encode_request(r: RenderRequest) -> bytes:
    """RenderServerRenderRequest.cpp:61-74: int(size + 8) then QByteArray."""
    inner = struct.pack(">Q", r.sequence_number)
    inner += qvector_u64(r.iteration_numbers)
    inner += qvector_f64(r.ppm_radii)
    inner += encode_details(r.details)
    return struct.pack(">i", len(inner) + 8) + qbytearray(inner)


class _Reader:
    def __init__(self, b: bytes):
        self.b, self.o = b, 0

    def take(self, n: int) -> bytes:
        if self.o + n > len(self.b):
            raise ValueError("truncated stream")
        s = self.b[self.o:self.o + n]
        self.o += n
        return s

    def u32(self) -> int:
        return struct.unpack(">I", self.take(4))[0]

    def i32(self) -> int:
        return struct.unpack(">i", self.take(4))[0]

    def u64(self) -> int:
        return struct.unpack(">Q", self.take(8))[0]

    def f64(self) -> float:
        return struct.unpack(">d", self.take(8))[0]

    def f32(self) -> float:
        return struct.unpack(">f", self.take(4))[0]

    def bytearray_(self) -> Optional[bytes]:
        n = self.u32()
        return None if n == NULL_BYTEARRAY else self.take(n)


def decode_request(b: bytes) -> RenderRequest:
    r = _Reader(b)
    r.i32()
    inner = _Reader(r.bytearray_() or b"")
    seq = inner.u64()
    its = [inner.u64() for _ in range(inner.u32())]
    radii = [inner.f64() for _ in range(inner.u32())]
    d = _Reader(inner.bytearray_() or b"")
    cam = [float(np.float32(d.f64())) for _ in range(12)]
    name = d.bytearray_()
    method, w, h = d.u32(), d.u32(), d.u32()
    alpha = d.f64()
    return RenderRequest(seq, its, radii, RequestDetails(
        Camera(cam[0:3], cam[3:6], cam[6:9], cam[9], cam[10], cam[11]), name, method, w, h, alpha))


@dataclass
class ResultPacket:
    sequence_number: int
    iteration_numbers: List[int]
    output: np.ndarray              # float32, W*H*3
    render_time: float = 0.0
    total_time: float = 0.0

    def first(self) -> int:
        return self.iteration_numbers[0]

    def last(self) -> int:
        return self.iteration_numbers[-1]


def encode_result(p: ResultPacket) -> bytes:
    """RenderResultPacket.cpp:124-146 on a SinglePrecision socket stream."""
    out = np.ascontiguousarray(p.output, dtype=np.float32).tobytes()
    its = sorted(int(x) for x in p.iteration_numbers)
    size = (len(out) + 4) + (len(its) * 8 + 4) + 8 + 2 * 4
    return (struct.pack(">QQ", size, p.sequence_number) + qvector_u64(its) + qfloat(p.render_time, True)
            + qfloat(p.total_time, True) + qbytearray(out))


def decode_result(b: bytes) -> ResultPacket:
    r = _Reader(b)
    r.u64()
    seq = r.u64()
    its = [r.u64() for _ in range(r.u32())]
    rt, tt = r.f32(), r.f32()
    out = np.frombuffer(r.bytearray_() or b"", dtype=np.float32).copy()
    return ResultPacket(seq, its, out, rt, tt)


# --- client-side merge ----------------------------------------------------
f32 = np.float32


def packet_merge(a: ResultPacket, b: ResultPacket) -> None:
    """RenderResultPacket::merge (RenderResultPacket.cpp:104-121): a absorbs b."""
    ta, tb = len(a.iteration_numbers), len(b.iteration_numbers)
    scale = f32(1.0) / f32(ta + tb)
    x, y = a.output, b.output
    a.output = ((f32(ta) * x + f32(tb) * y) * scale).astype(np.float32)
    a.iteration_numbers = a.iteration_numbers + b.iteration_numbers


def running_average(inp: np.ndarray, n_in: int, out: np.ndarray, n_out: int) -> np.ndarray:
    """mergeBufferRunningAverage (RenderResultPacketReceiver.cpp:166-190)."""
    if n_out == 0:
        return inp.astype(np.float32).copy()
    ratio = f32(n_in) / f32(n_out + n_in)
    return (out + (inp - out) * ratio).astype(np.float32)


class Receiver:
    """RenderResultPacketReceiver (PPM: iteration order; otherwise arrival order)."""

    def __init__(self, ppm: bool):
        self.ppm = ppm
        self.reset()
        self.last_sequence = 0

    def reset(self):
        self.front: Optional[np.ndarray] = None
        self.iteration = 0
        self.next_expected = 0
        self.back: List[ResultPacket] = []

    def push(self, p: ResultPacket, current_sequence: int) -> bool:
        if p.sequence_number != current_sequence:
            return False
        if p.sequence_number > self.last_sequence:
            self.reset()
            self.last_sequence = p.sequence_number
        p = ResultPacket(p.sequence_number, sorted(p.iteration_numbers), p.output.astype(np.float32).copy(),
                         p.render_time, p.total_time)
        if self.front is None:
            self.front = np.zeros_like(p.output)
        if self.ppm:
            self.back.append(p)
            self.back.sort(key=lambda q: q.first())        # qSort, operator< on the first iteration
            merged = True
            while merged:
                merged = False
                for k in range(len(self.back) - 1):
                    if self.back[k].last() + 1 == self.back[k + 1].first():
                        packet_merge(self.back[k], self.back[k + 1])
                        del self.back[k + 1]
                        merged = True
                        break
            if self.back[0].first() == self.next_expected:
                b = self.back.pop(0)
                self.front = running_average(b.output, len(b.iteration_numbers), self.front, self.next_expected)
                self.next_expected = b.last() + 1
            self.iteration = self.next_expected - 1 if self.next_expected > 0 else 0
        else:
            self.front = running_average(p.output, len(p.iteration_numbers), self.front, self.iteration)
            self.iteration += len(p.iteration_numbers)
        return True


def next_request_radii(r0: float, first_iteration: int, n: int, alpha: float = 2.0 / 3.0) -> List[float]:
    """DistributedApplication::getNextRenderServerRenderRequest (DistributedApplication.cpp:96-122):
    radius of iteration i, then r^2 <- r^2 (i + alpha) / (i + 1), in double."""
    import math
    radii, r = [], r0
    for i in range(first_iteration + n):
        if i >= first_iteration:
            radii.append(r)
        r = math.sqrt(r * r * (i + alpha) / (i + 1))
    return radii
