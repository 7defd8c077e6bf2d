"""GPU: the device libm restatement (rsc_math.h — fdlibm-style sin/cos/acos/cbrt/log used by the
Sim3 angles, MLPnP and MapPoint::PredictScale in SearchBySim3) evaluated ON THE GPU through
rsc_selftest_math, checked (a) bit-for-bit against the same functions compiled for the host (the
oracle's ora_dm_*: device code generation changes nothing) and (b) within 1 ulp of glibc (Python's
math module), the CPU test's bar (tests/test_cpu_mlpnp.py), on the ranges the kernels feed them."""
import math

import numpy as np
import pytest

import oracle_lib as ol
from gpu_common import ctx as gpu_ctx

pytestmark = pytest.mark.gpu


def _inputs(rng):
    xs = np.concatenate([rng.uniform(-1, 1, 20000) * s for s in (1e-8, 1e-3, 1.0, 3.2, 50.0, 1e4)])
    edge = np.array([0.0, -0.0, math.pi / 4, -math.pi / 4, math.pi / 2, math.pi, 2 * math.pi, 1e-300, 5e-324])
    return np.concatenate([xs, edge])


def _ulp_close(a, b, k):
    return abs(a - b) <= k * math.ulp(b) + 1e-300


@pytest.mark.parametrize("name", ["sin", "cos", "acos", "cbrt", "log", "logf"])
def test_device_libm_matches_host_restatement_and_glibc(name):
    rng = np.random.default_rng(42)
    if name == "acos":
        x = np.concatenate([rng.uniform(-1, 1, 60000), [-1.0, 1.0, 0.0, 0.5, -0.5, 1 - 2**-52, -1 + 2**-52]])
    elif name == "cbrt":
        x = np.abs(_inputs(rng)) + 1e-300
    elif name in ("log", "logf"):
        # SearchBySim3's PredictScale ratios and a wide sweep
        x = np.concatenate([rng.uniform(0.5, 3.0, 30000), 10.0 ** rng.uniform(-30, 30, 30000), [1.0, 2.0, 1.2]])
    else:
        x = _inputs(rng)
    dev = gpu_ctx().selftest_math(name, x)
    L = ol.lib()
    host_fn = {"sin": L.ora_dm_sin, "cos": L.ora_dm_cos, "acos": L.ora_dm_acos, "cbrt": L.ora_dm_cbrt,
               "log": L.ora_dm_log, "logf": L.ora_dm_log}[name]
    if name == "logf":
        host = np.array([float(np.float32(host_fn(float(np.float32(v))))) for v in x])
    else:
        host = np.array([host_fn(float(v)) for v in x])
    assert np.array_equal(dev.view(np.uint64), host.view(np.uint64)), name
    glibc = {"sin": math.sin, "cos": math.cos, "acos": math.acos,
             "cbrt": lambda v: float(np.cbrt(v)), "log": math.log,
             "logf": lambda v: float(np.float32(math.log(float(np.float32(v)))))}[name]
    k = 1
    for xi, di in zip(x, dev):
        gi = glibc(float(xi))
        if name == "logf":
            assert abs(di - gi) <= math.ulp(np.float32(gi)) + 1e-300, (name, xi, di, gi)
        else:
            assert _ulp_close(di, gi, k), (name, xi, di, gi)
