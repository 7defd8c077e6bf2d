"""The product's per-lane device numerics (rsc_core.h / rsc_epnp.h / rsc_sim3.h) and its iterate()
replay logic (rsc_engine.h), compiled for the HOST by the test-only emulation library, against the
oracle.  Bar: bit-exact.  (The same sources run on the MI355X in the -m gpu tests.)"""
import ctypes
import json
import os

import numpy as np
import pytest

import hostemu_lib as he
import oracle_lib as ol
from rsc import synth

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
RELOC = (0.99, 10, 300, 4, 0.5, 5.991)


def bits(a):
    return np.ascontiguousarray(np.asarray(a, np.float32)).view(np.uint32)


def test_rng_jump_table_matches_glibc():
    with open(os.path.join(GOLD, "glibc_rand.json")) as f:
        g = json.load(f)
    for seed, ref in g["rand"].items():
        assert np.array_equal(he.rand_stream(int(seed), len(ref)), np.array(ref, np.int32))
    # long stream: crosses the jump-table window (re-basing in RngStream::ensure)
    assert np.array_equal(he.rand_stream(77, 40000), ol.glibc_rand(77, 40000))


@pytest.mark.parametrize("ms", [4, 5, 6])
@pytest.mark.parametrize("k", range(3))
def test_hypotheses_bitexact(ms, k):
    rng = np.random.default_rng(10 * ms + k)
    sc = synth.make_pnp_scene(rng, int(rng.integers(50, 700)), float(rng.uniform(0.3, 0.6)))
    seed = 100 + k
    o = ol.OraclePnP(sc, seed)
    o.set_ransac_parameters(0.99, 10, 300, ms, 0.5, 5.991)
    o.enable_trace()
    o.iterate(40)
    ints, fl = o.trace()
    for h in range(len(ints)):
        idx, R, t = he.pnp_hypothesis(sc, seed, h, ns=ms)
        assert np.array_equal(idx, ints[h, :ms]), h
        assert np.array_equal(bits(R.ravel()), bits(fl[h, :9])) and np.array_equal(bits(t), bits(fl[h, 9:])), h
        c, _ = he.pnp_count(sc, R, t)
        assert c == ints[h, 8], h
        if ints[h, 9]:
            break  # the oracle's Refine changes the EPnP buffers for later hypotheses


def _nan_equal(a, b):
    a = np.ascontiguousarray(a, np.float32).ravel()
    b = np.ascontiguousarray(b, np.float32).ravel()
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(a.view(np.uint32)[~na], b.view(np.uint32)[~nb])


@pytest.mark.parametrize("plane", ["floor", "wall", "tilted"])
def test_planar_hypotheses_nan_exit_bitexact(plane):
    """Coplanar samples (Q4): NaN control points, a 12x12 / 4x4 eigen-solve that never deflates.
    The product's QR sweep ends after the first all-NaN sweep (rsc_core.h tridiag_qr), the oracle
    runs Eigen's full 30 n sweeps: the poses must agree (NaN as NaN) and the counts exactly."""
    rng = np.random.default_rng({"floor": 1, "wall": 2, "tilted": 3}[plane])
    sc = synth.make_planar_pnp_scene(rng, 300, 0.7, plane)
    o = ol.OraclePnP(sc, 7)
    o.set_ransac_parameters(*RELOC)
    o.enable_trace()
    o.iterate(40)
    ints, fl = o.trace()
    n_nan = 0
    for h in range(len(ints)):
        idx, R, t = he.pnp_hypothesis(sc, 7, h)
        assert np.array_equal(idx, ints[h, :4]), h
        assert _nan_equal(np.concatenate([R.ravel(), t]), fl[h]), h
        c, _ = he.pnp_count(sc, R, t)
        assert c == ints[h, 8], h
        n_nan += bool(np.isnan(fl[h]).any())
        if ints[h, 9]:
            break
    assert n_nan > 0


def test_refine_rows_and_stale_rows_bitexact():
    rng = np.random.default_rng(5)
    sc = synth.make_pnp_scene(rng, 400, 0.6)
    K = np.array([sc.fx, sc.fy, sc.cx, sc.cy], np.float32)
    for nbig in (150, 251, 90):
        o = ol.OraclePnP(sc, 1)
        o.set_ransac_parameters(*RELOC)
        big = np.sort(rng.choice(sc.n, nbig, replace=False)).astype(np.int32)
        Ro, to, eo = o.compute_pose(big)
        pws = sc.p3dw[big].astype(np.float64).copy()
        us = sc.p2d[big].astype(np.float64).copy()
        als = np.zeros((nbig, 4))
        R = np.zeros(9, np.float32)
        t = np.zeros(3, np.float32)
        e = he.lib().he_pnp_rows(nbig, nbig, pws.reshape(-1), us.reshape(-1), als.reshape(-1), K, R, t)
        assert np.array_equal(bits(R), bits(Ro.ravel())) and np.array_equal(bits(t), bits(to)) and e == eo
        small = rng.choice(sc.n, 4, replace=False).astype(np.int32)
        R2o, t2o, e2o = o.compute_pose(small)
        pws4, als4, us4 = pws.copy(), als.copy(), np.zeros((nbig, 2))
        pws4[:4] = sc.p3dw[small]
        us4[:4] = sc.p2d[small]
        e2 = he.lib().he_pnp_rows(4, nbig, pws4.reshape(-1), us4.reshape(-1), als4.reshape(-1), K, R, t)
        assert np.array_equal(bits(R), bits(R2o.ravel())) and np.array_equal(bits(t), bits(t2o)) and e2 == e2o


def test_sim3_hypotheses_bitexact():
    rng = np.random.default_rng(8)
    for k in range(3):
        pair = synth.make_sim3_pair(rng, 500, 150, invalid_frac=0.1)
        o = ol.OracleSim3(pair, 5 + k)
        o.set_ransac_parameters(0.99, 20, 300)
        o.enable_trace()
        o.iterate(40)
        ints, fl = o.trace()
        p = o.prepared()
        N = o.N
        w, g0 = he.window(5 + k)
        K = pair.K1.astype(np.float32)
        for h in range(len(ints)):
            idx = np.zeros(3, np.int32)
            pose = np.zeros(24, np.float32)
            he.lib().he_sim3_hypothesis(w, g0, h, N, p["X1c"].reshape(-1), p["X2c"].reshape(-1), idx, pose)
            assert np.array_equal(idx, ints[h, :3])
            assert np.array_equal(bits(pose[:12]), bits(fl[h]))
            m = np.zeros(N, np.uint8)
            c = he.lib().he_sim3_count(pose, K, pair.K2.astype(np.float32), N, p["X1c"].reshape(-1),
                                       p["X2c"].reshape(-1), p["P1im1"].reshape(-1), p["P2im2"].reshape(-1),
                                       p["maxerr1"], p["maxerr2"], m)
            assert c == ints[h, 3]


def _assert_pnp(a, b, where):
    assert (a["ok"], a["no_more"], a["n_inliers"]) == (b["ok"], b["no_more"], b["n_inliers"]), where
    if b["ok"]:
        assert np.array_equal(bits(a["T"]), bits(b["T"])), where
        assert np.array_equal(a["inliers"], b["inliers"]), where


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_replay_emulation_matches_oracle(seed):
    """rsc_engine.h's speculate/replay/refine/respeculate logic vs the sequential oracle, on
    relocalization-shaped rounds of iterate(5) (Refine successes and failures, stale rows)."""
    rng = np.random.default_rng(40 + seed)
    scenes = [synth.make_pnp_scene(rng, int(rng.integers(40, 500)), float(rng.uniform(0.35, 0.85)),
                                   n_points=None) for _ in range(4)]
    emus = [he.EmuPnP(sc, seed * 10 + i) for i, sc in enumerate(scenes)]
    oras = [ol.OraclePnP(sc, seed * 10 + i) for i, sc in enumerate(scenes)]
    for e, o in zip(emus, oras):
        e.set_ransac_parameters(*RELOC)
        o.set_ransac_parameters(*RELOC)
    for rnd in range(12):
        outs = he.iterate_many(emus, 5)
        for i, o in enumerate(oras):
            _assert_pnp(outs[i], o.iterate(5), f"round {rnd} cand {i}")
            se, so = emus[i].state(), o.info()
            assert se["iterations"] == so["iterations"] and se["max_rows"] == so["max_rows"]
            assert se["best_inliers"] == so["best_inliers"]


def test_replay_emulation_long_iterate():
    rng = np.random.default_rng(99)
    sc = synth.make_pnp_scene(rng, 600, 0.62, n_points=650)
    e, o = he.EmuPnP(sc, 4), ol.OraclePnP(sc, 4)
    e.set_ransac_parameters(*RELOC)
    o.set_ransac_parameters(*RELOC)
    _assert_pnp(e.iterate(300), o.iterate(300), "iterate(300)")


@pytest.mark.parametrize("case", [1, 4, 17, 43, 66])
def test_replay_emulation_refine_failures(case):
    from gpu_common import refine_fail_scene
    sc, seed = refine_fail_scene(case)
    e, o = he.EmuPnP(sc, seed), ol.OraclePnP(sc, seed)
    e.set_ransac_parameters(*RELOC)
    o.set_ransac_parameters(*RELOC)
    o.enable_trace()
    for rnd in range(20):
        _assert_pnp(e.iterate(5), o.iterate(5), f"round {rnd}")
        assert e.state()["max_rows"] == o.info()["max_rows"]
    ints, _ = o.trace()
    assert ((ints[:, 9] == 1) & (ints[:, 11] == 0)).any(), "case must contain a failed Refine"


def test_split_wait_gives_up_after_its_limit():
    """rsc_core.h poll_until, the split eigen stage's bounded hand-off wait (split_wait), compiled for
    the host: it returns as soon as the flag is ready, and at a spin limit of 1 a flag that is not yet
    ready makes it give up after one load (the device then raises the launch's fault word, which the
    host returns as RSC_ERR_INTERNAL — tests/test_gpu_fault.py runs that path on the device)."""
    assert he.poll_until(1, 1) == (True, 1, 0)
    assert he.poll_until(1, 2) == (False, 1, 1)  # the give-up path at limit 1
    assert he.poll_until(1 << 24, 5) == (True, 5, 4)
    assert he.poll_until(3, 5) == (False, 3, 3)
    assert he.poll_until(0, 1) == (False, 0, 0)
