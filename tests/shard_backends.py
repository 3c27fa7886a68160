"""Shard backends for tests only (TEST INFRASTRUCTURE): the CPU oracle behind the multi-GPU
bench's orchestration, so the launcher, the gloo collectives, the max-over-ranks timing and the
JSON line of `bench.py --gpus N` run on CPU (tests/test_bench_launch.py).  Selected with
ORX_SHARD_BACKEND=shard_backends:oracle_shard; the product backend is liborx.so on HIP."""
import torch

import oracle_lib


def oracle_shard(cfg, rank, world, local_rank, scene):
    r = oracle_lib.OracleRenderer(cfg)
    oracle_lib.load().orc_set_threads(2)
    r.init_scene(scene)
    b = oracle_lib.OracleShard(r, torch)
    b.set_shard(rank, world)
    return b
