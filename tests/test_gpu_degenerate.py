"""GPU parity on the reference's degenerate inputs (VERDICT r3 "Next round" 2) — scenes that
rsc/synth.py's frustum generator never produces but real EuRoC frames do (walls, floors, poles,
repeated points):

* PnP on exactly planar map points (floor Y = 1.5 / wall Z = 6): every 4-point sample is coplanar,
  the PCA's smallest eigenvalue is 0 or a rounding residue, and the control points / 3x3 inverse
  give NaN (Q4, PnPsolver.cpp:311-331); NaN poses score 0 inliers (NaN compares false, :258).  The
  12x12 and 4x4 eigen-solves of such a hypothesis never deflate: the kernels end them after the first
  all-NaN sweep (rsc_core.h tridiag_qr), the oracle runs Eigen's 360 / 120 sweeps — identical results;
* PnP on a tilted plane (coplanar up to rounding: NaN and ill-conditioned finite samples mixed) and
  with 25 % repeated correspondences;
* Sim3 with 40 % collinear matches (Horn on collinear triples, Sim3Solver.cpp:139-151, :196-266) and
  with repeated matches;
* MLPnP on planes through the world origin ("floor0" / "wall0"): the planar branch of computePose
  (FullPivHouseholderQR rank 2 on the uncentred points, the 9-column system, 4-way sign test,
  MLPnPsolver.cpp:346-364, :404-435, :497-558) on the device, the branch confirmed per hypothesis by
  the oracle's trace; and on offset planes, which MLPnP's uncentred rank test keeps on the general
  branch.

Bit-exact as everywhere (samples, counts, masks, poses), with NaN poses compared as NaN (the sign /
payload of a NaN is not an IEEE-specified result: x86 produces the negative default NaN, gfx950 the
positive one)."""
import numpy as np
import pytest

from gpu_common import assert_pnp_equal, assert_sim3_equal, ctx
import oracle_lib as ol
from rsc import synth
from rsc import workloads as wl

pytestmark = pytest.mark.gpu


def nan_equal(a, b):
    """Bitwise equal, except that NaN matches NaN (same positions)."""
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(a.view(np.uint32)[~na], b.view(np.uint32)[~nb])


@pytest.mark.parametrize("plane", ["floor", "wall", "tilted", "duplicates"])
def test_pnp_degenerate_every_hypothesis(plane):
    from rsc import engine
    # exhaustive: at most 45 % inliers, so minInliers = N/2 is unreachable and the 300 speculated
    # hypotheses are the 300 the reference evaluates (Refine paths: the round-robin test below)
    scenes = [synth.make_planar_pnp_scene(np.random.default_rng(700 + i), n, r, plane)
              for i, (n, r) in enumerate([(600, 0.45), (1500, 0.4), (250, 0.45), (2000, 0.3)])]
    seeds = [11, 12, 13, 14]
    gs = [engine.PnPSolver(ctx(), sc, s) for sc, s in zip(scenes, seeds)]
    b = engine.SolverBatch(gs)
    b.set_ransac_parameters(*wl.RELOC)
    outs = b.iterate(300, with_masks=True)
    n_nan = n_hyp = 0
    for i, (sc, s) in enumerate(zip(scenes, seeds)):
        o = ol.OraclePnP(sc, s)
        o.set_ransac_parameters(*wl.RELOC)
        o.enable_trace()
        ro = o.iterate(300)
        assert_pnp_equal(outs[i], ro, f"{plane} cand {i}")
        assert not ro["ok"] and ro["iterations"] == 300
        ints, fl = o.trace()
        cnt, pos = gs[i].last_hypotheses(400)
        smp = gs[i].last_samples(400)
        assert len(cnt) == len(ints)
        assert np.array_equal(smp[:, :4], ints[:, :4]), f"{plane} cand {i} samples"
        assert np.array_equal(cnt, ints[:, 8]), f"{plane} cand {i} counts"
        assert nan_equal(pos, fl), f"{plane} cand {i} poses"
        n_nan += int(np.isnan(fl).any(1).sum())
        n_hyp += len(ints)
    if plane in ("floor", "wall"):
        assert n_nan > 0.8 * n_hyp  # the Q4 NaN path dominates
    if plane == "tilted":
        assert n_nan > 0


@pytest.mark.parametrize("plane", ["floor", "tilted"])
def test_pnp_planar_round_robin_with_refine(plane):
    """iterate(5) rounds (Tracking.cpp:1239-1262) on planar candidates mixed with regular ones, so
    NaN hypotheses, Refines and stale EPnP rows (Q6) meet in the same launches."""
    from rsc import engine
    rng = np.random.default_rng(31)
    scenes = [synth.make_planar_pnp_scene(rng, 500, 0.75, plane), synth.make_pnp_scene(rng, 400, 0.7),
              synth.make_planar_pnp_scene(rng, 900, 0.7, plane), synth.make_pnp_scene(rng, 300, 0.8)]
    pairs = []
    for i, sc in enumerate(scenes):
        g = engine.PnPSolver(ctx(), sc, 50 + i)
        g.set_ransac_parameters(*wl.RELOC)
        o = ol.OraclePnP(sc, 50 + i)
        o.set_ransac_parameters(*wl.RELOC)
        pairs.append((g, o))
    for rnd in range(8):
        outs = engine.pnp_iterate_many([p[0] for p in pairs], 5)
        for i, (g, o) in enumerate(pairs):
            assert_pnp_equal(outs[i], o.iterate(5), f"{plane} round {rnd} cand {i}")
            assert g.state()["max_rows"] == o.info()["max_rows"]


@pytest.mark.parametrize("kind", ["collinear", "duplicates"])
def test_sim3_degenerate_every_hypothesis(kind):
    from rsc import engine
    pairs = [synth.make_sim3_pair(np.random.default_rng(800 + i), n, k, degenerate=kind)
             for i, (n, k) in enumerate([(500, 200), (1000, 15), (300, 150)])]
    seeds = [21, 22, 23]
    gs = [engine.Sim3Solver(ctx(), p, s) for p, s in zip(pairs, seeds)]
    b = engine.SolverBatch(gs)
    b.set_ransac_parameters(*wl.LOOP)
    outs = b.iterate(300, with_masks=True)
    for i, (p, s) in enumerate(zip(pairs, seeds)):
        o = ol.OracleSim3(p, s)
        o.set_ransac_parameters(*wl.LOOP)
        o.enable_trace()
        ro = o.iterate(300)
        assert_sim3_equal(outs[i], ro, f"{kind} pair {i}")
        ints, fl = o.trace()
        cnt, pos = gs[i].last_hypotheses(400)
        # one speculation of all 300; the reference stops at its first success (Q12)
        h = len(ints)
        assert len(cnt) >= h
        assert np.array_equal(cnt[:h], ints[:, 3]), f"{kind} pair {i} counts"
        assert nan_equal(pos[:h], fl), f"{kind} pair {i} poses"


@pytest.mark.parametrize("plane", ["floor", "wall", "tilted"])
def test_mlpnp_offset_planes_on_device(plane):
    """Coplanar scenes whose plane misses the world origin: MLPnP's rank test on the UNCENTRED
    points3 * points3^T (MLPnPsolver.cpp:346-364) gives rank 3, so these stay on the general branch
    with ill-conditioned samples (the planar branch itself: test_mlpnp_planar_branch_on_device)."""
    from rsc import engine
    rng = np.random.default_rng(900)
    sc = synth.make_planar_pnp_scene(rng, 800, 0.6, plane)
    params = (0.99, 10, 300, 6, 0.5, 5.991)
    g = engine.MLPnPSolver(ctx(), sc, 9)
    g.set_ransac_parameters(*params)
    o = ol.OracleMLPnP(sc, 9)
    o.set_ransac_parameters(*params)
    o.enable_trace()
    rg, ro = g.iterate(60), o.iterate(60)
    assert rg["ok"] == ro["ok"] and rg["n_inliers"] == ro["n_inliers"] and rg["iterations"] == ro["iterations"]
    assert nan_equal(rg["T"], ro["T"])
    if ro["ok"]:
        assert np.array_equal(rg["inliers"], ro["inliers"])
    ints, dbl = o.trace()
    smp, pos = g.last_hypotheses()
    h = len(ints)
    assert len(smp) >= h
    assert np.array_equal(smp[:h, :6], ints[:, :6])
    da, db = pos[:h].astype(np.float64), dbl.astype(np.float64)
    na, nb = np.isnan(da), np.isnan(db)
    assert np.array_equal(na, nb) and np.array_equal(da.view(np.uint64)[~na], db.view(np.uint64)[~nb])


def _ml_planar_compare(g, o, n_its, where):
    rg, ro = g.iterate(n_its), o.iterate(n_its)
    assert (rg["ok"], rg["n_inliers"], rg["iterations"]) == (ro["ok"], ro["n_inliers"], ro["iterations"]), where
    assert nan_equal(rg["T"], ro["T"]), where
    if ro["ok"]:
        assert np.array_equal(rg["inliers"], ro["inliers"]), where
    ints, dbl = o.trace()
    planar = o.trace_planar()
    smp, pos = g.last_hypotheses()
    h = len(ints)
    assert len(smp) >= h and len(planar) == h
    assert np.array_equal(smp[:h, :6], ints[:, :6]), where
    da, db = pos[:h].astype(np.float64), dbl.astype(np.float64)
    na, nb = np.isnan(da), np.isnan(db)
    assert np.array_equal(na, nb) and np.array_equal(da.view(np.uint64)[~na], db.view(np.uint64)[~nb]), where
    return ro, planar


@pytest.mark.parametrize("plane,ratio,seeds,min_ok", [("floor0", 0.75, (9, 10, 11), 2), ("wall0", 0.6, (9, 10), 0)])
def test_mlpnp_planar_branch_on_device(plane, ratio, seeds, min_ok):
    """MLPnP's planar branch on the device: map points on a plane THROUGH THE WORLD ORIGIN (world
    Y = 0 / Z = 0 exactly, rsc.synth "floor0" / "wall0"), so rank(points3 * points3^T) == 2 for every
    sample (MLPnPsolver.cpp:346-364) and computePose rotates the points into the plane, solves the
    9-column system (:404-435) and runs the 4-way sign test (:497-558).  The oracle's trace confirms
    the branch was taken for EVERY hypothesis; the device's samples and double poses are bit-exact
    against it (a general-branch solve would give other bits), and on the floor scene the planar
    hypotheses reach Refine and succeed."""
    from rsc import engine
    rng = np.random.default_rng(900)
    sc = synth.make_planar_pnp_scene(rng, 800, ratio, plane)
    assert not np.any(sc.p3dw[:, 1 if plane == "floor0" else 2])
    params = (0.99, 10, 300, 6, 0.5, 5.991)
    n_ok = 0
    for seed in seeds:
        g = engine.MLPnPSolver(ctx(), sc, seed)
        g.set_ransac_parameters(*params)
        o = ol.OracleMLPnP(sc, seed)
        o.set_ransac_parameters(*params)
        o.enable_trace()
        ro, planar = _ml_planar_compare(g, o, 60, f"{plane} seed {seed}")
        assert planar.all() and len(planar) > 0
        n_ok += ro["ok"]
    assert n_ok >= min_ok


def test_mlpnp_planar_and_general_candidates_in_one_launch():
    """Planar-branch candidates (origin floor) and general ones in the same mlpnp_iterate_many
    launches, iterate(5) rounds as the reference's round-robin would call them."""
    from rsc import engine
    rng = np.random.default_rng(901)
    scs = [synth.make_planar_pnp_scene(rng, 600, 0.75, "floor0"), synth.make_pnp_scene(rng, 700, 0.6),
           synth.make_planar_pnp_scene(rng, 500, 0.7, "wall0"), synth.make_pnp_scene(rng, 400, 0.5)]
    params = (0.99, 10, 300, 6, 0.5, 5.991)
    pairs = []
    for i, sc in enumerate(scs):
        g = engine.MLPnPSolver(ctx(), sc, 30 + i)
        g.set_ransac_parameters(*params)
        o = ol.OracleMLPnP(sc, 30 + i)
        o.set_ransac_parameters(*params)
        pairs.append((g, o))
    for rnd in range(8):
        outs = engine.mlpnp_iterate_many([p[0] for p in pairs], 5)
        for i, (g, o) in enumerate(pairs):
            ro = o.iterate(5)
            got = outs[i]
            assert (got["ok"], got["no_more"], got["n_inliers"]) == (ro["ok"], ro["no_more"], ro["n_inliers"]), \
                f"round {rnd} cand {i}"
            assert nan_equal(got["T"], ro["T"]) and np.array_equal(got["inliers"], ro["inliers"]), f"round {rnd} cand {i}"
