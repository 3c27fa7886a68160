"""Client/server wire format and the client's merge.

The product codec and receiver (liborx.so: include/orx_wire.h) are checked
byte for byte / bit for bit against the restatement in oracle/wire_oracle.py,
which is itself pinned by hand-derived known-answer frames below (Qt's
QDataStream layout: big-endian, QByteArray = u32 length + bytes, QVector =
u32 count + elements, floats as doubles on a default stream and as floats on
the SinglePrecision socket stream).  A gloo run drives the client/server loop
of oppositerenderer_amd.wire over torch.distributed with oracle-backed
render servers.  No GPU is needed: the codec is host code in liborx.so."""
import os
import socket
import struct
import sys
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import wire_oracle as wo  # noqa: E402

import oracle_lib  # noqa: E402
from oppositerenderer_amd import _abi, scenes, wire  # noqa: E402
from oppositerenderer_amd.renderer import OrxError  # noqa: E402

SEED = 1645301512


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def to_oracle(req: wire.RenderServerRenderRequest) -> wo.RenderRequest:
    c = [float(np.float32(v)) for v in req.details.camera]
    d = req.details
    return wo.RenderRequest(req.sequence_number, list(req.iteration_numbers), list(req.ppm_radii),
                            wo.RequestDetails(wo.Camera(c[0:3], c[3:6], c[6:9], c[9], c[10], c[11]), d.scene_name,
                                              d.render_method, d.width, d.height, d.ppm_alpha))


# --- known-answer frames ------------------------------------------------------
def test_request_known_answer():
    """sequence 5, iterations [7], radii [0.5], camera hfov = vfov = 35 (others 0), scene "A",
    PPM (2), 2x1, alpha 0.5 -- every field written out by hand."""
    det = wire.RenderServerRenderRequestDetails([0] * 9 + [35.0, 35.0, 0.0], b"A", 2, 2, 1, 0.5)
    req = wire.RenderServerRenderRequest(5, [7], [0.5], det)
    details = ("0000000000000000" * 9 + "4041800000000000" * 2 + "0000000000000000"  # 12 floats as doubles
               + "00000001" + "41"                        # QByteArray "A"
               + "00000002" + "00000002" + "00000001"     # method, width, height
               + "3fe0000000000000")                      # ppmAlpha 0.5
    inner = ("0000000000000005"                           # quint64 sequence number
             + "00000001" + "0000000000000007"            # QVector<u64> {7}
             + "00000001" + "3fe0000000000000"            # QVector<double> {0.5}
             + "%08x" % (len(details) // 2) + details)     # details QByteArray
    frame = "%08x" % (len(inner) // 2 + 8) + "%08x" % (len(inner) // 2) + inner
    assert len(details) // 2 == 121 and len(inner) // 2 == 157
    assert req.encode().hex() == frame
    assert wo.encode_request(to_oracle(req)).hex() == frame


def test_result_known_answer():
    """sequence 3, iterations {9, 8} (sent sorted), times 1.5 s / 2 s as 4-byte floats,
    output [1.0, -2.0] as raw little-endian float32 bytes; size counts what follows it."""
    p = wire.RenderResultPacket(3, [9, 8], np.array([1.0, -2.0], np.float32), 1.5, 2.0)
    body = ("0000000000000003" + "00000002" + "0000000000000008" + "0000000000000009"
            + "3fc00000" + "40000000" + "00000008" + "0000803f" + "000000c0")
    frame = "%016x" % (len(body) // 2) + body
    assert p.encode().hex() == frame
    assert wo.encode_result(wo.ResultPacket(3, [9, 8], p.output, 1.5, 2.0)).hex() == frame


# --- codec == oracle, round trips, edge cases ---------------------------------
@pytest.mark.parametrize("n_it,name", [(0, b""), (1, None), (4, b"Cornell"), (17, b"sponza/sponza.dae")])
def test_request_codec_matches_oracle(n_it, name):
    rng = np.random.default_rng(n_it)
    cam = list(rng.normal(size=12).astype(np.float32))
    det = wire.RenderServerRenderRequestDetails(cam, name, int(rng.integers(0, 3)), 1920, 1080, 2.0 / 3.0)
    req = wire.RenderServerRenderRequest(int(rng.integers(1, 1 << 62)), [int(x) for x in rng.integers(0, 1 << 40, n_it)],
                                         list(rng.uniform(0.1, 10, n_it)), det)
    b = req.encode()
    assert b == wo.encode_request(to_oracle(req))
    back = wire.RenderServerRenderRequest.decode(b)
    assert back.sequence_number == req.sequence_number
    assert back.iteration_numbers == req.iteration_numbers
    assert back.ppm_radii == req.ppm_radii
    assert back.details.scene_name == name
    assert [np.float32(v) for v in back.details.camera] == [np.float32(v) for v in cam]
    assert (back.details.render_method, back.details.width, back.details.height) == (det.render_method, 1920, 1080)
    assert back.details.ppm_alpha == det.ppm_alpha
    o = wo.decode_request(b)
    assert o.iteration_numbers == req.iteration_numbers and o.details.scene_name == name


@pytest.mark.parametrize("n_px", [0, 1, 4096])
def test_result_codec_matches_oracle(n_px):
    rng = np.random.default_rng(n_px)
    out = rng.normal(size=3 * n_px).astype(np.float32)
    its = [int(x) for x in rng.permutation(50)[:5]]
    p = wire.RenderResultPacket(11, its, out, 0.25, 7.5)
    b = p.encode()
    assert b == wo.encode_result(wo.ResultPacket(11, its, out, 0.25, 7.5))
    assert struct.unpack(">Q", b[:8])[0] == len(b) - 8
    q = wire.RenderResultPacket.decode(b)
    assert q.iteration_numbers == sorted(its)
    assert np.array_equal(q.output.view(np.uint32), out.view(np.uint32))
    assert (q.render_time_seconds, q.total_time_seconds) == (0.25, 7.5)


def test_malformed_frames_raise():
    req = wire.RenderServerRenderRequest(1, [0, 1], [1.0, 0.9], wire.RenderServerRenderRequestDetails())
    b = req.encode()
    for cut in (0, 3, 8, len(b) - 1):
        with pytest.raises(OrxError):
            wire.RenderServerRenderRequest.decode(b[:cut])
    bad = bytearray(b)
    bad[3] ^= 1  # leading int no longer inner size + 8
    with pytest.raises(OrxError):
        wire.RenderServerRenderRequest.decode(bytes(bad))
    r = wire.RenderResultPacket(1, [0], np.ones(6, np.float32)).encode()
    for cut in (0, 7, 20, len(r) - 1):
        with pytest.raises(OrxError):
            wire.RenderResultPacket.decode(r[:cut])


def test_mutated_frames_decode_or_raise():
    """Every truncation and 2000 seeded byte mutations of a request and a result frame: the decoder either
    returns a frame or raises OrxError -- it never reads past the buffer (tests/test_sanitizers.py runs this
    under AddressSanitizer, which turns any out-of-bounds read of the codec into a failure)."""
    rng = np.random.default_rng(5)
    req = wire.RenderServerRenderRequest(7, [3, 4, 5], [1.0, 0.9, 0.8], wire.RenderServerRenderRequestDetails())
    res = wire.RenderResultPacket(7, [3, 4, 5], rng.uniform(0, 1, 3 * 17).astype(np.float32))
    for frame, cls in ((req.encode(), wire.RenderServerRenderRequest), (res.encode(), wire.RenderResultPacket)):
        for cut in range(len(frame)):
            with pytest.raises(OrxError):
                cls.decode(frame[:cut])
        for _ in range(1000):
            bad = bytearray(frame)
            for _ in range(int(rng.integers(1, 4))):
                k = int(rng.integers(0, len(bad)))
                bad[k] = int(rng.integers(0, 256)) if rng.random() < 0.5 else bad[k] ^ 0xFF
            try:
                cls.decode(bytes(bad))
            except OrxError:
                pass


# --- receiver == oracle -------------------------------------------------------
def _packets(rng, n_iters, sizes, n_px):
    its, k, out = list(range(n_iters)), 0, []
    while k < n_iters:
        m = int(rng.choice(sizes))
        run = its[k:k + m]
        out.append((run, rng.uniform(0, 4, 3 * n_px).astype(np.float32)))
        k += m
    return out


@pytest.mark.parametrize("ppm", [True, False])
def test_receiver_matches_oracle_out_of_order(ppm):
    rng = np.random.default_rng(3)
    method = _abi.PROGRESSIVE_PHOTON_MAPPING if ppm else _abi.PATH_TRACING
    rx = wire.RenderResultPacketReceiver(method)
    ox = wo.Receiver(ppm)
    pk = _packets(rng, 40, [1, 2, 3, 4], 257)
    order = rng.permutation(len(pk))
    for i in order:
        run, data = pk[i]
        a = rx.onRenderResultPacketReceived(wire.RenderResultPacket(1, list(reversed(run)), data), 1)
        b = ox.push(wo.ResultPacket(1, list(reversed(run)), data), 1)
        assert a and b
        assert rx.getIterationNumber() == ox.iteration
        if ppm:
            assert rx.next_expected_iteration() == ox.next_expected
            assert rx.getBackBufferNumIterations() == sum(len(p.iteration_numbers) for p in ox.back)
        f = rx.front()
        if ox.next_expected or not ppm:
            assert np.array_equal(f.view(np.uint32), ox.front.view(np.uint32))
    if ppm:
        assert rx.next_expected_iteration() == 40 and rx.getIterationNumber() == 39
        assert rx.getBackBufferNumIterations() == 0 and rx.getPeakBackBufferSizeBytes() >= 0
        # every iteration weighs the same: the front is close to the plain mean of per-iteration buffers
        per_it = np.concatenate([[d] * len(r) for r, d in pk]).reshape(40, -1)
        assert np.allclose(rx.front(), per_it.mean(0), rtol=1e-5, atol=1e-5)
    else:
        assert rx.getIterationNumber() == 40


def test_receiver_sequences():
    rx = wire.RenderResultPacketReceiver(_abi.PROGRESSIVE_PHOTON_MAPPING)
    a = np.full(6, 2.0, np.float32)
    assert not rx.onRenderResultPacketReceived(wire.RenderResultPacket(1, [0], a), 2)  # stale: dropped
    assert rx.front() is None
    assert rx.onRenderResultPacketReceived(wire.RenderResultPacket(2, [1], a), 2)     # waits for 0
    assert rx.next_expected_iteration() == 0 and rx.getBackBufferNumIterations() == 1
    assert rx.backBufferIsNotFilled(2)
    assert rx.onRenderResultPacketReceived(wire.RenderResultPacket(2, [0], 2 * a), 2)
    assert rx.next_expected_iteration() == 2 and rx.getIterationNumber() == 1
    assert np.allclose(rx.front(), 3.0)  # (2*2 + 1*2... merged run [0,1] = (4 + 2)/2)
    assert rx.onRenderResultPacketReceived(wire.RenderResultPacket(3, [0], a), 3)     # newer: reset
    assert rx.next_expected_iteration() == 1 and np.allclose(rx.front(), 2.0)
    with pytest.raises(OrxError):  # a different frame size inside one sequence
        rx.onRenderResultPacketReceived(wire.RenderResultPacket(3, [1], np.ones(9, np.float32)), 3)


def test_request_generator_radii():
    det = wire.RenderServerRenderRequestDetails()
    g = wire.RequestGenerator(7.5376, det)
    a, b = g.next_request(4), g.next_request(3)
    assert a.iteration_numbers == [0, 1, 2, 3] and b.iteration_numbers == [4, 5, 6]
    assert a.ppm_radii + b.ppm_radii == wo.next_request_radii(7.5376, 0, 7)
    g.increment_sequence()
    c = g.next_request(2)
    assert c.sequence_number == 2 and c.iteration_numbers == [0, 1] and c.ppm_radii[0] == 7.5376


def test_wire_symbols_exported():
    lib = wire._lib()
    for name in wire.WIRE_SYMBOLS:
        assert hasattr(lib, name), name


# --- the client/server loop over torch.distributed (gloo) ---------------------
class OracleServerRenderer:
    """The render server's renderer on CPU: the oracle behind OptixRenderer's call names."""

    def __init__(self, seed, P):
        self.r = oracle_lib.OracleRenderer(_abi.default_config(seed=seed, photon_launch_width=P,
                                                               photon_launch_height=P))
        oracle_lib.load().orc_set_threads(2)
        self.r.init_scene(scenes.cornell())

    def renderNextIteration(self, it, local, radius, create_output, details):
        self.r.render_next_iteration(it, local, radius, details)

    def getOutputBuffer(self):
        return self.r.output().reshape(-1)


def _details(W, H):
    sc = scenes.cornell()
    cam = sc.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
    d = wire.RenderServerRenderRequestDetails.from_camera(cam, sc.name, _abi.PROGRESSIVE_PHOTON_MAPPING, W, H)
    req = _abi.OrxRequest()
    req.camera = cam.to_abi()
    req.method, req.width, req.height, req.ppm_alpha = _abi.PROGRESSIVE_PHOTON_MAPPING, W, H, 2.0 / 3.0
    return d, req, sc.initial_ppm_radius()


def _loop_worker(rank, world, port, out_path, W, H, P, packets, per_packet):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d, req, r0 = _details(W, H)
    if rank == 0:
        rx = wire.run_client(wire.RequestGenerator(r0, d), world, packets, per_packet, _abi.PROGRESSIVE_PHOTON_MAPPING)
        np.save(out_path, np.concatenate([[rx.getIterationNumber()], rx.front()]).astype(np.float64))
    else:
        wire.serve(OracleServerRenderer(SEED + 7919 * rank, P), req)
    dist.barrier()
    dist.destroy_process_group()


def test_client_server_loop_gloo():
    world, W, H, P, packets, per_packet = 3, 24, 20, 16, 2, 2
    out = os.path.join(tempfile.mkdtemp(), "front.npy")
    mp.spawn(_loop_worker, args=(world, free_port(), out, W, H, P, packets, per_packet), nprocs=world, join=True)
    got = np.load(out)
    # replay: the same requests rendered by the same per-server renderers, merged by the oracle receiver
    d, req, r0 = _details(W, H)
    gen = wire.RequestGenerator(r0, d)
    servers = {s: OracleServerRenderer(SEED + 7919 * s, P) for s in range(1, world)}
    ox = wo.Receiver(True)
    for _ in range(packets):
        reqs = {s: gen.next_request(per_packet) for s in range(1, world)}
        for s in range(1, world):
            p = wire.render_request(servers[s], reqs[s], req)
            ox.push(wo.ResultPacket(p.sequence_number, p.iteration_numbers, p.output), gen.sequence_number)
    assert int(got[0]) == packets * (world - 1) * per_packet - 1
    assert np.array_equal(got[1:].astype(np.float32).view(np.uint32), ox.front.view(np.uint32))
    assert ox.front.mean() > 0
