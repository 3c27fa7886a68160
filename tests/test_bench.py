"""bench.py's workload table and host-CPU accounting (CPU only: no GPU is touched)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_default_is_the_metric_workload():
    a = bench.parse([])
    assert (a.config, a.scene, a.width, a.height, a.method, a.photon_launch) == (
        2, "SyntheticHall", 1920, 1080, "ppm", 2048)
    assert a.scaling == "strong"


def test_configs_match_baseline():
    # BASELINE.json configs[0..4]
    want = {0: ("Cornell", 256, 256, "pt"), 1: ("Cornell", 1024, 1024, "ppm"),
            2: ("SyntheticHall", 1920, 1080, "ppm"), 3: ("SyntheticHall", 1920, 1080, "vcm"),
            4: ("SyntheticConference", 3840, 2160, "ppm")}
    for c, w in want.items():
        a = bench.parse(["--config", str(c)])
        assert (a.scene, a.width, a.height, a.method) == w
    assert bench.parse(["--config", "4"]).photon_launch ** 2 == 16777216
    assert bench.parse(["--config", "2"]).photon_launch ** 2 == 4194304
    assert bench.parse(["--config", "1"]).photon_launch ** 2 == 1048576


def test_overrides_win():
    a = bench.parse(["--config", "4", "--width", "640", "--scaling", "weak"])
    assert a.width == 640 and a.height == 2160 and a.scaling == "weak"


def test_host_cpu_accounting():
    n, info = bench.host_cpu()
    assert 1 <= n <= info["affinity_cpus"]
    if info["omp_num_threads"]:
        assert n <= info["omp_num_threads"]
