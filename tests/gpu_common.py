"""Shared helpers of the GPU parity tests (GPU result vs oracle on identical inputs and seeds)."""
import numpy as np
import pytest

_ctx = None


def ctx():
    global _ctx
    if _ctx is None:
        from rsc import engine
        _ctx = engine.Context(0)
    return _ctx


def bits(a):
    return np.ascontiguousarray(np.asarray(a, np.float32)).view(np.uint32)


def assert_pnp_equal(g, o, where=""):
    """Bit-exact parity of one PnPsolver::iterate() result."""
    assert g["ok"] == o["ok"], f"{where} ok {g['ok']} vs {o['ok']}"
    assert g["no_more"] == o["no_more"], f"{where} no_more"
    assert g["n_inliers"] == o["n_inliers"], f"{where} n_inliers {g['n_inliers']} vs {o['n_inliers']}"
    if o["ok"]:
        assert np.array_equal(bits(g["T"]), bits(o["T"])), f"{where} T\n{g['T']}\n{o['T']}"
        assert np.array_equal(g["inliers"], o["inliers"]), f"{where} inlier mask"
    else:
        assert len(g["inliers"]) == 0 and len(o["inliers"]) == 0


def assert_sim3_equal(g, o, where=""):
    assert g["ok"] == o["ok"], f"{where} ok"
    assert g["no_more"] == o["no_more"], f"{where} no_more"
    assert g["n_inliers"] == o["n_inliers"], f"{where} n_inliers {g['n_inliers']} vs {o['n_inliers']}"
    assert np.array_equal(bits(g["R"]), bits(o["R"])), f"{where} R"
    assert np.array_equal(bits(g["t"]), bits(o["t"])), f"{where} t"
    assert np.array_equal(g["inliers"], o["inliers"]), f"{where} inliers"


# Scenes where PnPsolver::Refine() FAILS at least once in 20 rounds of iterate(5) (found by scanning
# the generator; they exercise re-speculation after a failed Refine with stale EPnP rows, Q6).
REFINE_FAIL_CASES = [1, 4, 17, 43, 66, 72, 74, 83, 95, 98]


def refine_fail_scene(s):
    from rsc import synth
    rng = np.random.default_rng(5000 + s)
    n = int(rng.integers(40, 300))
    ratio = float(rng.uniform(0.5, 0.6))
    return synth.make_pnp_scene(rng, n, ratio), s + 1
