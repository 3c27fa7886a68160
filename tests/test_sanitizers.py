"""The CPU-side C/C++ under AddressSanitizer + UndefinedBehaviorSanitizer (sanitizers on the
CPU restatement): the wire codec and receiver (oppositerenderer_amd/csrc/orx_wire.cpp, the host code that parses
bytes from a network peer) and the oracle (oracle/orx_oracle.c), each built with -fsanitize=address,undefined
(`make wire-asan`, `make -C oracle asan`), run under tests/test_wire.py (known-answer frames, malformed frames,
the receiver against its restatement) and tests/test_xorwow_kat.py in a child Python with the sanitizer runtimes
preloaded.  Any ASan report or UBSan runtime error fails the test (UBSan built non-recovering).  CPU only; the
HIP kernels are not sanitizer targets on this pool."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def runtime(name):
    p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.mark.skipif(bool(os.environ.get("LD_PRELOAD")), reason="a preload is already set (ASan must come first)")
def test_wire_and_oracle_rng_under_asan_ubsan():
    asan, ubsan = runtime("libasan.so"), runtime("libubsan.so")
    if not asan or not ubsan:
        pytest.skip("gcc sanitizer runtimes not installed")
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oppositerenderer_amd", "csrc"), "wire-asan"])
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"])
    env = dict(os.environ,
               LD_PRELOAD=f"{asan}:{ubsan}",
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               ORX_WIRE_LIB=os.path.join(ROOT, "oppositerenderer_amd", "liborx_wire_asan.so"),
               ORACLE_LIB=os.path.join(ROOT, "oracle", "liborx_oracle_asan.so"))
    out = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider", "-m", "not gpu",
                          "tests/test_wire.py", "tests/test_xorwow_kat.py", "-k", "not gloo"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    log = out.stdout + out.stderr
    assert out.returncode == 0, log[-4000:]
    assert "AddressSanitizer" not in log and "runtime error" not in log, log[-4000:]
    assert " passed" in out.stdout, log[-2000:]
