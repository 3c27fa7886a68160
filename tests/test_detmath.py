"""Accuracy of the deterministic math (include/orx_detmath.h) against libm/numpy.

The functions only need to be (a) deterministic and (b) accurate enough to
stand in for CUDA's fast-math intrinsics (__sinf etc. are 2^-21.4 absolute on
[-pi, pi]); both properties are checked here through a tiny C harness compiled
from the header, with the same flags as the oracle.
"""
import ctypes as C
import os
import subprocess
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = r"""
#include "orx_detmath.h"
void dm_sin(const float* x, float* y, int n){for(int i=0;i<n;i++) y[i]=orx_sinf(x[i]);}
void dm_cos(const float* x, float* y, int n){for(int i=0;i<n;i++) y[i]=orx_cosf(x[i]);}
void dm_exp(const float* x, float* y, int n){for(int i=0;i<n;i++) y[i]=orx_expf(x[i]);}
void dm_acos(const float* x, float* y, int n){for(int i=0;i<n;i++) y[i]=orx_acosf(x[i]);}
void dm_asin(const float* x, float* y, int n){for(int i=0;i<n;i++) y[i]=orx_asinf(x[i]);}
void dm_pow(const float* x, const float* e, float* y, int n){for(int i=0;i<n;i++) y[i]=orx_powf(x[i], e[i]);}
void dm_floor(const float* x, float* y, int n){for(int i=0;i<n;i++) y[i]=orx_floorf(x[i]);}
void dm_ceil(const float* x, float* y, int n){for(int i=0;i<n;i++) y[i]=orx_ceilf(x[i]);}
"""


@pytest.fixture(scope="module")
def dm():
    d = tempfile.mkdtemp()
    c = os.path.join(d, "dm.c")
    so = os.path.join(d, "libdm.so")
    open(c, "w").write(SRC)
    subprocess.check_call(["gcc", "-O2", "-fPIC", "-shared", "-ffp-contract=off", "-I", os.path.join(ROOT, "include"),
                           c, "-o", so, "-lm"])
    lib = C.CDLL(so)
    return lib


def run1(lib, name, x):
    x = np.ascontiguousarray(x, np.float32)
    y = np.empty_like(x)
    getattr(lib, name)(x.ctypes.data_as(C.c_void_p), y.ctypes.data_as(C.c_void_p), C.c_int(len(x)))
    return y


def test_sin_cos_abs_error(dm):
    x = np.linspace(-2 * np.pi, 2 * np.pi, 200001, dtype=np.float32)
    for name, ref in (("dm_sin", np.sin), ("dm_cos", np.cos)):
        y = run1(dm, name, x)
        err = np.abs(y.astype(np.float64) - ref(x.astype(np.float64)))
        assert err.max() < 4e-7, (name, err.max())


def test_exp_rel_error(dm):
    x = np.linspace(-20, 20, 100001, dtype=np.float32)
    y = run1(dm, "dm_exp", x)
    ref = np.exp(x.astype(np.float64))
    assert (np.abs(y - ref) / ref).max() < 3e-7
    assert run1(dm, "dm_exp", np.array([-200, 200, 0], np.float32)).tolist() == [0.0, float("inf"), 1.0]


def test_acos_asin(dm):
    x = np.linspace(-1, 1, 100001, dtype=np.float32)
    assert np.abs(run1(dm, "dm_acos", x) - np.arccos(x.astype(np.float64))).max() < 5e-7
    assert np.abs(run1(dm, "dm_asin", x) - np.arcsin(x.astype(np.float64))).max() < 5e-7


def test_pow(dm):
    rng = np.random.default_rng(0)
    b = rng.uniform(1e-3, 10, 20000).astype(np.float32)
    e = rng.uniform(-3, 100, 20000).astype(np.float32)
    y = np.empty_like(b)
    dm.dm_pow(b.ctypes.data_as(C.c_void_p), e.ctypes.data_as(C.c_void_p), y.ctypes.data_as(C.c_void_p), C.c_int(len(b)))
    ref = np.power(b.astype(np.float64), e.astype(np.float64))
    ok = np.isfinite(ref) & (ref < 3e38) & (ref > 1e-37)
    assert (np.abs(y[ok] - ref[ok]) / ref[ok]).max() < 2e-7


def test_floor_ceil_exact(dm):
    x = np.concatenate([np.linspace(-1e3, 1e3, 100003, dtype=np.float32),
                        np.array([-0.0, 0.0, 0.5, -0.5, 8388607.5, -8388607.5, 1e20, -1e20], np.float32)])
    assert np.array_equal(run1(dm, "dm_floor", x), np.floor(x))
    assert np.array_equal(run1(dm, "dm_ceil", x), np.ceil(x))


def test_gather_weight_polynomial():
    """The gather's kernel weight (orx_kernels.hip weight2: a degree-5 polynomial in u = d^2/r^2,
    Horner with fused multiply-adds in fp32) against photonPower's closed form
    (IndirectRadianceEstimation.cu:59-67, alpha = 1.818, beta = 1.953) over the whole accepted
    range u in [0, 1]: relative error within 2e-6, far inside the indirect bar of 1e-5 rel-L2."""
    import re

    src = open(os.path.join(ROOT, "oppositerenderer_amd", "csrc", "orx_kernels.hip")).read()
    coef = {int(k): float(v) for k, v in re.findall(r"ORX_W5_C(\d) = ([-0-9.e]+)f", src)}
    assert sorted(coef) == list(range(6))
    c = [np.float32(coef[k]) for k in range(6)]
    u = np.linspace(0.0, 1.0, 200001).astype(np.float32)
    p = np.full_like(u, c[5])
    for k in (4, 3, 2, 1, 0):  # fma in float64 of float32 operands, rounded once: fp32 FMA
        p = (p.astype(np.float64) * u.astype(np.float64) + np.float64(c[k])).astype(np.float32)
    alpha, beta, enb = 1.818, 1.953, 0.141847
    w = alpha * (1.0 - (1.0 - np.exp(-beta * u.astype(np.float64) / 2.0)) / (1.0 - enb))
    err = np.abs(p.astype(np.float64) - w) / w
    assert err.max() < 2e-6, err.max()
