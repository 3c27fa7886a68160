import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

# torch's HIP runtime is loaded before liborx.so's first HIP call whatever tests a run selects:
# loaded only after liborx had initialised HIP, torch's lazy device init reported "No HIP GPUs are
# available" (a -k selection whose first torch user came after liborx tests)
import torch  # noqa: E402,F401


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through liborx.so on HIP)")
    config.addinivalue_line("markers", "slow: longer CPU-oracle runs")
    config.addinivalue_line("markers", "fresh_process: spawns a child that must start before this process "
                                       "makes its first HIP call (run first)")


def pytest_collection_modifyitems(session, config, items):
    # tests that start a fresh GPU child process go first, before any test of this process has
    # initialised HIP (tests/test_gpu_steady_state.py::test_rccl_world1_sharded_paths_match_oracle)
    items.sort(key=lambda it: 0 if it.get_closest_marker("fresh_process") else 1)
