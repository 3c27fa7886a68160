"""What bench.py actually times, against the oracle (TEST: GPU).

1. The bench's timed schedule at the bench's own size.  bench.py issues
   renderNextIteration(it, it, r, False, det) back to back with no read in between
   (StandaloneRenderManager.cpp:75-140 without its every-5th output fetch), so every PPM
   iteration after the first runs pipelined: the gather + output of iteration i on the second
   stream beside the eye / photon / grid passes of i+1, with the two buffer sets alternating
   (OptixRenderer.cpp:569-673 restated as orx_render_next_iteration).  The full-size tests of
   test_gpu_fullsize.py read buffers between iterations, which breaks that chain every time;
   here configs[2] (hall 1920x1080, 2048^2 photons) runs six iterations from iteration 0 with
   no read and no synchronisation, then the running-sum output (rel-L2 <= 1e-4, north_star),
   the last iteration's indirect radiance (rel-L2 <= 1e-5: fp32 summation order only) and the
   RNG state (bit-exact) are compared with the oracle's six iterations.  configs[3] (hall VCM)
   runs three iterations the same way (iteration 0 carries the light-vertex-count estimate
   launch, OptixRenderer.cpp:699-773): camera colours and RNG bit-exact, output <= 1e-4.

2. The RCCL sharded path on a real GPU.  Two RCCL ranks cannot share the one GPU of a test box,
   so multigpu.ShardedPPM / ShardedVCM run at world 1 over torch.distributed's "nccl" backend
   (RCCL) in a fresh child process: all_gather_into_tensor of the hit points issued async and
   waited on the side stream, reduce_scatter_tensor of the indirect radiance, the slab
   partition's histogram all-gather and photon all_to_all_single, and the image all_gather —
   the calls bench.py --gpus N makes (DistributedApplication.cpp:96-122 is the reference's
   distribution point).  Each variant runs three iterations at 480x270 (hall, 256^2 photons)
   and is compared with the oracle's single renderer: PPM rows pipelined, rows serial, slab
   pipelined, slab serial (rel-L2 <= 1e-5), VCM (rel-L2 <= 1e-5) and PT (bit-exact).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle_lib
from oppositerenderer_amd import _abi, synthetic
from oppositerenderer_amd.renderer import OptixRenderer, RenderRequestDetails, next_ppm_radius

pytestmark = pytest.mark.gpu
SEED = 1645301512
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(((a - b) ** 2).sum()) / max(np.sqrt((b * b).sum()), 1e-30))


def _bench_schedule(method, iters, P=2048, W=1920, H=1080):
    """bench.py main()'s loop: same config, same calls, createOutput False, no reads."""
    scene = synthetic.synthetic_hall()
    cfg = _abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P)
    gpu = OptixRenderer(cfg)
    gpu.initialize(0)
    gpu.initScene(scene)
    cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
    det = RenderRequestDetails(cam, scene.name, method, W, H)
    radius = scene.initial_ppm_radius()
    for it in range(iters):
        gpu.renderNextIteration(it, it, radius, False, det)
        radius = next_ppm_radius(radius, it)
    pipelined = gpu.pipelined()  # before any read: a read ends the pipelined chain
    ora = oracle_lib.OracleRenderer(_abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P))
    ora.init_scene(scene)
    radius = scene.initial_ppm_radius()
    req = det.to_abi()
    for it in range(iters):
        ora.render_next_iteration(it, it, radius, req)
        radius = next_ppm_radius(radius, it)
    return gpu, ora, pipelined


def test_bench_schedule_configs2_hall_ppm_six_pipelined_iterations():
    gpu, ora, pipelined = _bench_schedule(_abi.PROGRESSIVE_PHOTON_MAPPING, 6)
    assert pipelined, "bench.py's default schedule must be the pipelined one (ORX_PIPELINE unset)"
    g, o = gpu.getOutputBuffer(), ora.output()
    assert np.isfinite(g).all() and g.mean() > 0
    assert rel_l2(g, o) < 1e-4, rel_l2(g, o)
    gi, oi = gpu.read_buffer(_abi.BUF_INDIRECT), ora.read_buffer(_abi.BUF_INDIRECT)
    assert rel_l2(gi, oi) < 1e-5, rel_l2(gi, oi)
    gr, orr = gpu.read_buffer(_abi.BUF_RNG, np.uint32), ora.read_buffer(_abi.BUF_RNG, np.uint32)
    assert np.array_equal(gr, orr), f"rng: {np.count_nonzero(gr != orr)} words differ"
    gs, os_ = gpu.stats(), ora.stats()
    assert gs.valid_photons == os_.valid_photons  # the last iteration's deposits
    gpu.destroy()
    ora.close()


def test_bench_schedule_configs3_hall_vcm_three_iterations():
    gpu, ora, overlapped = _bench_schedule(_abi.VCM_BIDIRECTIONAL_PATH_TRACING, 3)
    assert overlapped, "bench.py's VCM schedule overlaps the shadow rays with the next light pass"
    for buf, name in ((_abi.BUF_RNG, "rng"), (_abi.BUF_VCM_CAMERA, "camera colours"),
                      (_abi.BUF_VCM_VERTEX_COUNT, "vertex counts")):
        g, o = gpu.read_buffer(buf, np.uint32), ora.read_buffer(buf, np.uint32)
        assert np.array_equal(g, o), f"{name}: {np.count_nonzero(g != o)} of {g.size} words differ"
    g, o = gpu.getOutputBuffer(), ora.output()
    assert np.isfinite(g).all() and g.mean() > 0
    assert rel_l2(g, o) < 1e-4, rel_l2(g, o)
    # the light pass's camera connections went to the resolve, none back to in-place tracing
    st = gpu.stats()
    assert st.vcm_light_connections > 0 and st.vcm_light_inplace == 0, (st.vcm_light_connections, st.vcm_light_inplace)
    assert st.vcm_shadow_rays > 0 and st.vcm_shadow_overflow == 0
    gpu.destroy()
    ora.close()


@pytest.mark.fresh_process
def test_rccl_world1_sharded_paths_match_oracle(tmp_path):
    """tests/rccl_world1_child.py in a fresh process (conftest runs this test before any other,
    so the child starts before this process has made a HIP call)."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("ORX_PIPELINE", None)
    out = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "rccl_world1_child.py"),
                          str(tmp_path / "store")], env=env, capture_output=True, text=True, timeout=170, cwd=ROOT)
    assert out.returncode == 0, (out.stdout[-2000:], out.stderr[-3000:])
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["backend"] == "nccl", res
    for name, r in res["variants"].items():
        if name == "pt":
            assert r["bit_exact"], (name, r)
        else:
            assert r["rel_l2"] < 1e-5, (name, r)
        assert r["mean"] > 0, (name, r)
        if r.get("expect_pipelined"):
            assert r["pipelined"], (name, r)
    assert {"ppm_batch", "vcm_batch", "pt_batch", "ppm_batch2_emulated"} <= set(res["variants"]), res
    assert res["variants"]["pt_batch"]["bit_exact"], res["variants"]["pt_batch"]
    assert res["variants"]["ppm_batch2_emulated"]["rank_images_differ"], res["variants"]["ppm_batch2_emulated"]
