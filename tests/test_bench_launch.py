"""`python bench.py --gpus 2` with no launcher: bench.py starts the two rank processes itself,
they rendezvous on 127.0.0.1, run the sharded PPM iteration (multigpu.ShardedPPM) under gloo on
the CPU oracle backend (tests/shard_backends.py; the product backend is liborx.so on HIP), take
the max over ranks of the timed region, and rank 0 prints exactly one JSON line."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _launch(extra):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["ORX_SHARD_BACKEND"] = "shard_backends:oracle_shard"
    env["ORX_BATCH_BACKEND"] = "shard_backends:oracle_batch"
    env["PYTHONPATH"] = os.pathsep.join([os.path.join(ROOT, "tests"), ROOT, env.get("PYTHONPATH", "")])
    env["OMP_NUM_THREADS"] = "2"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--scene", "Cornell", "--width", "48", "--height", "40", "--photon-launch", "32",
           "--no-cpu-baseline"] + extra
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["world_size"] == 2
    assert "launcher test" in out["backend"]
    return out


def test_bench_gpus2_self_launch_prints_one_json_line():
    """the default multi-GPU partition: photon batches (every rank its own whole iterations)"""
    out = _launch([])
    assert out["value"] > 0 and out["steps"] == 2 and out["scaling"] == "weak"
    assert out["config"]["photons_per_iteration"] == 32 * 32
    assert out["config"]["paths_per_iteration"] == 2 * (48 * 40 + 32 * 32)
    assert "photon-batch" in out["config"]["parallelism"]


def test_bench_gpus2_rows_partition():
    out = _launch(["--partition", "rows"])
    assert out["value"] > 0 and out["steps"] == 2 and out["scaling"] == "strong"
    assert out["config"]["photons_per_iteration"] == 32 * 32
    assert out["config"]["paths_per_iteration"] == 48 * 40 + 32 * 32


def test_bench_config4_defaults_to_the_rows_partition():
    """--config 4 (BASELINE configs[4]: a pixel-tile shard over 8 GPUs) runs the strong-scaling row
    partition by default; the sizes are overridden so that the oracle backend finishes quickly."""
    out = _launch(["--config", "4"])
    assert out["scaling"] == "strong"
    assert "row-interleaved" in out["config"]["parallelism"]
    assert out["config"]["paths_per_iteration"] == 48 * 40 + 32 * 32
    import bench
    assert bench.parse(["--config", "4"]).partition == "rows"
    assert bench.parse(["--config", "4", "--partition", "batch"]).partition == "batch"
    assert bench.parse([]).partition == "batch"
    assert bench.parse(["--config", "3"]).partition == "batch"


def test_bench_rank_failure_ends_the_launch():
    """A rank that fails (here: an unknown scene) ends the launch with its exit code instead of
    leaving the other rank waiting in a collective."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    env["ORX_SHARD_BACKEND"] = "shard_backends:oracle_shard"
    env["PYTHONPATH"] = os.pathsep.join([os.path.join(ROOT, "tests"), ROOT, env.get("PYTHONPATH", "")])
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1",
           "--scene", "NoSuchScene", "--width", "16", "--height", "16", "--photon-launch", "16", "--no-cpu-baseline"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode != 0
    assert not p.stdout.strip()
