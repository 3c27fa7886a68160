"""Shard backends for tests only (TEST INFRASTRUCTURE): the CPU oracle behind the multi-GPU
bench's orchestration, so the launcher, the gloo collectives, the max-over-ranks timing and the
JSON line of `bench.py --gpus N` run on CPU (tests/test_bench_launch.py).  Selected with
ORX_SHARD_BACKEND=shard_backends:oracle_shard (row partition) and ORX_BATCH_BACKEND=shard_backends:oracle_batch
(photon-batch partition); the product backends are liborx.so on HIP."""
import torch

import oracle_lib
from oppositerenderer_amd import multigpu


def oracle_shard(cfg, rank, world, local_rank, scene):
    r = oracle_lib.OracleRenderer(cfg)
    oracle_lib.load().orc_set_threads(2)
    r.init_scene(scene)
    b = oracle_lib.OracleShard(r, torch)
    b.set_shard(rank, world)
    return b


def oracle_batch(cfg, rank, world, local_rank, scene):
    """photon-batch partition on the oracle: a whole-frame renderer with the rank's seed"""
    c = type(cfg).from_buffer_copy(cfg)
    c.seed = multigpu.batch_seed(cfg.seed, rank)
    r = oracle_lib.OracleRenderer(c)
    oracle_lib.load().orc_set_threads(2)
    r.init_scene(scene)
    b = oracle_lib.OracleShard(r, torch)
    b.set_shard(0, 1)
    return b
