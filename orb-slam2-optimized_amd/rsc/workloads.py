"""The BASELINE.json configurations as concrete, seed-fixed inputs.

One definition shared by ``bench.py`` (the timed workloads) and ``tests/test_gpu_configs.py`` (the
same inputs compared bit-exactly against the oracle), so the shapes the bench reports are the shapes
the parity tests check.
"""
from __future__ import annotations

import numpy as np

from . import synth

RELOC = (0.99, 10, 300, 4, 0.5, 5.991)        # Tracking.cpp:1226
LOOP = (0.99, 20, 300)                        # LoopClosing.cpp:261
MLPNP = (0.99, 10, 300, 6, 0.5, 5.991)        # commented call Tracking.cpp:1227-1228

# config 2: 64 candidates x 2000 correspondences; exhaustive mode = 40 % inliers (minInliers
# floor(0.5 N) = 1000 is unreachable -> exactly 300 hypotheses per candidate, Q1); parity mode = 60 %.
CONFIG2 = dict(candidates=64, corrs=2000, iters=300, exhaustive_ratio=0.4, parity_ratio=0.6)
# config 3: 32 KeyFrame pairs x 1000 matches; exhaustive = 15 true inliers (<= 20 never passes the
# "> minInliers" test, Q12); parity mode = 300 true inliers.
CONFIG3 = dict(pairs=32, corrs=1000, iters=300, exhaustive_inliers=15, parity_inliers=300)
# config 4: 128 candidates x 4096, MLPnP, exhaustive (40 % inliers), sharded across the ranks (the
# BASELINE quotes 4 GPUs = 32 per GPU; the parity test checks the first 32).
CONFIG4 = dict(candidates=128, candidates_per_gpu=32, corrs=4096, iters=300, ratio=0.4)


def config2_scenes(rank: int = 0, candidates: int = 64, corrs: int = 2000, ratio: float = 0.4, seed: int = 20240):
    """The PnP relocalization batch of one rank (bench.py headline)."""
    rng = np.random.default_rng(seed + rank)
    return [synth.make_pnp_scene(rng, corrs, ratio) for _ in range(candidates)]


def config2_seeds(step: int, rank: int = 0, candidates: int = 64) -> np.ndarray:
    """srand() seed of every candidate at bench step ``step`` (H4: one stream per candidate)."""
    return (1 + np.arange(candidates) + candidates * (step + 1000 * rank)).astype(np.uint32)


def config3_pairs(n_inliers: int = 15, pairs: int = 32, corrs: int = 1000, seed: int = 77):
    rng = np.random.default_rng(seed)
    return [synth.make_sim3_pair(rng, corrs, n_inliers) for _ in range(pairs)]


def config4_scenes(candidates: int = 32, corrs: int = 4096, ratio: float = 0.4, seed: int = 78):
    rng = np.random.default_rng(seed)
    return [synth.make_pnp_scene(rng, corrs, ratio) for _ in range(candidates)]


def config4_covariances(sc):
    """Bearing-vector covariances of config 4's "with bearing-vector covariances" variant: the
    keypoint's pixel variance (mvLevelSigma2) through the bearing map ((u - cx) / fx, (v - cy) / fy, 1)
    plus a tiny isotropic term — computePose's covMats (MLPnPsolver.cpp:375-388)."""
    s2 = np.asarray(sc.sigma2, np.float64)
    cov = np.zeros((sc.n, 3, 3))
    cov[:, 0, 0] = s2 / float(sc.fx) ** 2
    cov[:, 1, 1] = s2 / float(sc.fy) ** 2
    return cov + np.eye(3) * 1e-9


def step_seeds(step: int, count: int) -> np.ndarray:
    return (1 + np.arange(count) + count * step).astype(np.uint32)
