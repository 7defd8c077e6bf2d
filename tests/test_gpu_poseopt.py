"""GPU: rsc_pose_optimization_many (Optimizer::PoseOptimization on the MI355X) == the oracle, bit for
bit (pose bits, nGood, mvbOutlier flags, LM iteration and trial counts), across sizes, outlier
ratios, slots without map points, the < 3 and < 10 edge rules and a 64-frame batch."""
import numpy as np
import pytest

import oracle_lib as ol
from gpu_common import bits, ctx
from rsc import engine, synth

pytestmark = pytest.mark.gpu


def check(frames):
    res = engine.pose_optimization_many(ctx(), frames)
    for k, (f, g) in enumerate(zip(frames, res)):
        r, T, out, st = ol.pose_optimization(f)
        sel = f.has_mp == 1
        assert g["n_good"] == r, f"frame {k}: nGood {g['n_good']} vs {r}"
        assert g["n_initial"] == int(sel.sum())
        assert np.array_equal(bits(g["Tcw"]), bits(T)), f"frame {k}: Tcw\n{g['Tcw']}\n{T}"
        assert np.array_equal(g["outlier"][sel], out[sel]), f"frame {k}: outliers"
        assert (g["outlier"][~sel] == 255).all()
        if g["n_initial"] >= 3:
            assert [g["rounds"], g["lm_iterations"], g["lm_trials"]] == list(st), f"frame {k}: stats"
    return res


def test_random_frames_bitexact():
    rng = np.random.default_rng(77)
    frames = []
    for _ in range(48):
        n = int(rng.integers(3, 900))
        frames.append(synth.make_poseopt_frame(rng, n, float(rng.uniform(0.3, 1.0)),
                                               rot_noise=float(rng.uniform(0, 0.15)),
                                               trans_noise=float(rng.uniform(0, 0.4)),
                                               no_mp_frac=float(rng.choice([0.0, 0.25]))))
    check(frames)


def test_small_and_degenerate_frames():
    rng = np.random.default_rng(78)
    frames = [synth.make_poseopt_frame(rng, n, 1.0) for n in (3, 4, 9, 10, 11)]
    f = synth.make_poseopt_frame(rng, 8, 1.0)
    f.has_mp[:] = 0
    f.has_mp[:2] = 1                       # 2 edges: returns 0, pose untouched
    frames.append(f)
    f = synth.make_poseopt_frame(rng, 200, 1.0, noise=False)  # noise-free known answer
    frames.append(f)
    res = check(frames)
    assert res[5]["n_good"] == 0 and np.array_equal(res[5]["Tcw"], frames[5].Tcw)
    assert np.abs(res[6]["Tcw"][:3, 3] - frames[6].t_true).max() < 1e-5


def test_relocalization_batch_64x2000():
    """The bench shape: 64 Frames x 2000 map-point matches (60 % inliers)."""
    rng = np.random.default_rng(79)
    frames = [synth.make_poseopt_frame(rng, 2000, 0.6) for _ in range(64)]
    check(frames)


def test_stereo_frames_bitexact():
    """EdgeStereoSE3ProjectXYZOnlyPose (Optimizer.cpp:290-323; the reference's stereo_euroc /
    stereo_kitti builds): Frames with 60-100 % stereo slots, mixed sizes and outlier ratios."""
    rng = np.random.default_rng(81)
    frames = []
    for _ in range(40):
        n = int(rng.integers(3, 1200))
        frames.append(synth.make_poseopt_frame(rng, n, float(rng.uniform(0.3, 1.0)),
                                               rot_noise=float(rng.uniform(0, 0.15)),
                                               trans_noise=float(rng.uniform(0, 0.4)),
                                               no_mp_frac=float(rng.choice([0.0, 0.25])),
                                               stereo_frac=float(rng.uniform(0.6, 1.0))))
    check(frames)


def test_stereo_relocalization_batch_64x2000():
    rng = np.random.default_rng(82)
    frames = [synth.make_poseopt_frame(rng, 2000, 0.6, stereo_frac=0.8) for _ in range(64)]
    check(frames)
