"""GPU: rsc_optimize_sim3_many (Optimizer::OptimizeSim3 on the MI355X) == the oracle, bit for bit
(nIn, g2oS12 quaternion / translation / scale bits, the NULLed vpMatches1 entries, LM iteration and
trial counts), across sizes, outlier ratios, the < 10 rule, empty problems and a 32-pair batch, in
both forms (one workgroup per pair; the cooperative form with helper workgroups, the default)."""
import numpy as np
import pytest

import oracle_lib as ol
from gpu_common import ctx
from rsc import engine, synth

pytestmark = pytest.mark.gpu


def check(problems, c=None):
    res = engine.optimize_sim3_many(c or ctx(), problems)
    for k, (p, g) in enumerate(zip(problems, res)):
        r, S, keep, st = ol.optimize_sim3(p)
        assert g["n_inliers"] == r, f"pair {k}: nIn {g['n_inliers']} vs {r}"
        assert g["n_correspondences"] == st[0] and g["n_bad"] == st[1], f"pair {k}"
        assert np.array_equal(g["S"].view(np.uint64), S.view(np.uint64)), f"pair {k}: S\n{g['S']}\n{S}"
        assert np.array_equal(g["keep"], keep), f"pair {k}: keep"
        if st[0]:
            assert [g["lm_iterations"], g["lm_trials"]] == list(st[2:]), f"pair {k}: stats"
    return res


def test_random_pairs_bitexact():
    rng = np.random.default_rng(91)
    probs = [synth.make_sim3opt_problem(rng, int(rng.integers(5, 1500)), valid_frac=float(rng.uniform(0.4, 1.0)),
                                        outlier_frac=float(rng.uniform(0.0, 0.6)), noise=bool(rng.random() < 0.8),
                                        pose_noise=float(rng.uniform(0.0, 0.08))) for _ in range(40)]
    check(probs)


def test_rules_and_degenerate_pairs():
    rng = np.random.default_rng(92)
    probs = [synth.make_sim3opt_problem(rng, 40, noise=False, outlier_frac=0.9),   # < 10 after removal
             synth.make_sim3opt_problem(rng, 20, valid_frac=0.0),                  # no correspondence
             synth.make_sim3opt_problem(rng, 12, noise=False, outlier_frac=0.0),   # tiny
             synth.make_sim3opt_problem(rng, 300, noise=False, outlier_frac=0.0)]  # no outlier: 5 + 5
    res = check(probs)
    assert res[0]["n_inliers"] == 0 and res[1]["n_inliers"] == 0 and res[3]["n_bad"] == 0


def test_loop_closure_batch_32_pairs():
    """The bench shape: 32 KeyFrame pairs x ~1000 correspondences (config-3 pairs)."""
    rng = np.random.default_rng(93)
    check([synth.make_sim3opt_problem(rng, 1000, outlier_frac=0.25) for _ in range(32)])


@pytest.fixture
def form_ctx():
    """The shared context in a given OptimizeSim3 form, restored to automatic afterwards."""
    c = ctx()
    yield c
    c.set_sim3opt_helpers(-1)


@pytest.mark.parametrize("helpers", [0, 1, 3, 7])
def test_forms_bitexact(form_ctx, helpers):
    """The one-workgroup form and the cooperative form at 1, 3 and 7 helpers per pair: every chunk
    claimed by a helper or by the master, the same bits."""
    form_ctx.set_sim3opt_helpers(helpers)
    rng = np.random.default_rng(94 + helpers)
    probs = [synth.make_sim3opt_problem(rng, int(rng.integers(5, 2500)), valid_frac=float(rng.uniform(0.5, 1.0)),
                                        outlier_frac=float(rng.uniform(0.0, 0.5)), noise=True,
                                        pose_noise=float(rng.uniform(0.0, 0.05))) for _ in range(12)]
    check(probs, form_ctx)


def test_cooperative_maximum_pair(form_ctx):
    """8192 correspondences (16,384 edges, the 256-chunk maximum of the hand-off) and a single pair
    (the loop-closure event's launch: 7 helpers), with the automatic form."""
    rng = np.random.default_rng(98)
    check([synth.make_sim3opt_problem(rng, 8192, outlier_frac=0.2)], form_ctx)
    check([synth.make_sim3opt_problem(rng, 8192, outlier_frac=0.2, valid_frac=1.0),
           synth.make_sim3opt_problem(rng, 33, outlier_frac=0.0)], form_ctx)


def test_cooperative_many_pairs(form_ctx):
    """72 pairs: 72 master blocks leave room for 2 helpers each; 160 pairs: none (the
    one-workgroup form)."""
    rng = np.random.default_rng(99)
    check([synth.make_sim3opt_problem(rng, int(rng.integers(20, 600)), outlier_frac=0.2) for _ in range(72)], form_ctx)
    check([synth.make_sim3opt_problem(rng, int(rng.integers(20, 200)), outlier_frac=0.2) for _ in range(160)],
          form_ctx)
