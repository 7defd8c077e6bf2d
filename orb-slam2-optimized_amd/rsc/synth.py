"""Synthetic relocalization / loop-closure scenes shaped like the reference's EuRoC runs.

No dataset is fetched (there is no network): every scene is generated from a seeded
``numpy.random.Generator`` (SURVEY.md §8(d) "Synthetic inputs").

Constants follow the reference's configuration:
  * EuRoC intrinsics fx=fy=435.2046959714599, cx=367.4517211914062, cy=252.2008514404297,
    image 752x480 (Examples/Stereo/EuRoC.yaml:8-11,18-19).  ``Frame::fx`` etc. are *static float*
    members (include/Frame.hpp:102-105), so the values are rounded to float32 before the solvers
    widen them to double (PnPsolver.hpp:71).
  * ORB pyramid: 8 levels, scale factor 1.2f, sigma^2(L) = scale(L)^2 computed in float
    (src/ORBextractor.cpp:353-360); keypoints per level follow the geometric per-level budget
    (src/ORBextractor.cpp:372-383).
"""
from __future__ import annotations

import dataclasses
import numpy as np

FX = np.float32(435.2046959714599)
FY = np.float32(435.2046959714599)
CX = np.float32(367.4517211914062)
CY = np.float32(252.2008514404297)
WIDTH, HEIGHT = 752, 480
N_LEVELS = 8
SCALE_FACTOR = np.float32(1.2)


def level_sigma2() -> np.ndarray:
    """mvLevelSigma2 exactly as ORBextractor computes it (float32 products)."""
    sf = [np.float32(1.0)]
    for _ in range(1, N_LEVELS):
        sf.append(np.float32(sf[-1] * SCALE_FACTOR))
    return np.array([np.float32(s * s) for s in sf], dtype=np.float32)


def level_probabilities(nfeatures: int = 1200) -> np.ndarray:
    factor = 1.0 / float(SCALE_FACTOR)
    n_desired = nfeatures * (1 - factor) / (1 - factor ** N_LEVELS)
    per = []
    for _ in range(N_LEVELS - 1):
        per.append(round(n_desired))
        n_desired *= factor
    per.append(max(nfeatures - sum(per), 0))
    p = np.array(per, dtype=np.float64)
    return p / p.sum()


def random_rotation(rng: np.random.Generator, max_angle: float = np.pi) -> np.ndarray:
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    ang = rng.uniform(-max_angle, max_angle)
    K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    return np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * (K @ K)


@dataclasses.dataclass
class PnPScene:
    """Compacted PnPsolver inputs (PnPsolver.cpp:22-44) for one relocalization candidate."""
    p2d: np.ndarray      # float32 [n,2]  mvKeysUn[i].pt
    p3dw: np.ndarray     # float32 [n,3]  MapPoint::GetWorldPos()
    sigma2: np.ndarray   # float32 [n]    mvLevelSigma2[octave]
    kp_index: np.ndarray  # int32 [n]     index of the keypoint in the Frame
    n_points: int        # F.N (size of the output inlier vector)
    R_true: np.ndarray   # float64 [3,3] Tcw rotation
    t_true: np.ndarray   # float64 [3]
    inlier_true: np.ndarray  # bool [n]
    fx: np.float32 = FX
    fy: np.float32 = FY
    cx: np.float32 = CX
    cy: np.float32 = CY

    @property
    def n(self) -> int:
        return int(self.p2d.shape[0])


def make_pnp_scene(rng: np.random.Generator, n: int, inlier_ratio: float, noise: bool = True,
                   n_points: int | None = None, depth=(0.5, 8.0)) -> PnPScene:
    """Random Tcw, inliers = noisy projections of frustum points, outliers = uniform pixels."""
    R = random_rotation(rng)
    t = rng.uniform(-2.0, 2.0, size=3)
    u = rng.uniform(0, WIDTH, size=n)
    v = rng.uniform(0, HEIGHT, size=n)
    d = rng.uniform(depth[0], depth[1], size=n)
    fx, fy, cx, cy = float(FX), float(FY), float(CX), float(CY)
    Xc = np.stack([(u - cx) / fx * d, (v - cy) / fy * d, d], axis=1)
    Xw = (Xc - t) @ R  # R^T (Xc - t)
    levels = rng.choice(N_LEVELS, size=n, p=level_probabilities())
    s2 = level_sigma2()[levels]
    n_in = int(round(inlier_ratio * n))
    inl = np.zeros(n, dtype=bool)
    inl[rng.permutation(n)[:n_in]] = True
    obs_u = u.copy()
    obs_v = v.copy()
    if noise:
        sig = np.sqrt(s2.astype(np.float64))
        obs_u[inl] += rng.normal(size=n_in) * sig[inl]
        obs_v[inl] += rng.normal(size=n_in) * sig[inl]
    n_out = n - n_in
    obs_u[~inl] = rng.uniform(0, WIDTH, size=n_out)
    obs_v[~inl] = rng.uniform(0, HEIGHT, size=n_out)
    if n_points is None:
        n_points = n
    kp = np.sort(rng.choice(n_points, size=n, replace=False)).astype(np.int32) if n_points > n \
        else np.arange(n, dtype=np.int32)
    return PnPScene(p2d=np.stack([obs_u, obs_v], 1).astype(np.float32),
                    p3dw=Xw.astype(np.float32), sigma2=s2.astype(np.float32), kp_index=kp,
                    n_points=int(n_points), R_true=R, t_true=t, inlier_true=inl)


def _observe(rng, R, t, Xw, inlier_ratio, noise, n_points):
    """Projections of world points Xw (float64 [n,3]) by Tcw = (R, t) as a PnPScene: inliers noisy
    by sigma(level), outliers uniform in the image (as make_pnp_scene)."""
    n = len(Xw)
    Xc = Xw @ R.T + t
    fx, fy, cx, cy = float(FX), float(FY), float(CX), float(CY)
    u = fx * Xc[:, 0] / Xc[:, 2] + cx
    v = fy * Xc[:, 1] / Xc[:, 2] + cy
    levels = rng.choice(N_LEVELS, size=n, p=level_probabilities())
    s2 = level_sigma2()[levels]
    n_in = int(round(inlier_ratio * n))
    inl = np.zeros(n, dtype=bool)
    inl[rng.permutation(n)[:n_in]] = True
    if noise:
        sig = np.sqrt(s2.astype(np.float64))
        u[inl] += rng.normal(size=n_in) * sig[inl]
        v[inl] += rng.normal(size=n_in) * sig[inl]
    u[~inl] = rng.uniform(0, WIDTH, size=n - n_in)
    v[~inl] = rng.uniform(0, HEIGHT, size=n - n_in)
    n_points = n if n_points is None else n_points
    kp = np.sort(rng.choice(n_points, size=n, replace=False)).astype(np.int32) if n_points > n \
        else np.arange(n, dtype=np.int32)
    return PnPScene(p2d=np.stack([u, v], 1).astype(np.float32), p3dw=Xw.astype(np.float32),
                    sigma2=s2.astype(np.float32), kp_index=kp, n_points=int(n_points), R_true=R, t_true=t,
                    inlier_true=inl)


def make_planar_pnp_scene(rng: np.random.Generator, n: int, inlier_ratio: float, plane: str = "floor",
                          noise: bool = True, n_points: int | None = None) -> PnPScene:
    """Relocalization candidate whose map points lie on one plane — the walls and floors of EuRoC's
    rooms, which make_pnp_scene avoids by drawing a frustum volume.

    plane = "floor": world Y = 1.5 exactly (representable), so every 4-point sample is exactly
            coplanar in float: the PCA's smallest eigenvalue is 0 (or a rounding residue of either
            sign), sqrt(lambda / n) and the 3x3 inverse of the control points give NaN or inf, and
            the hypothesis ends with NaN poses and 0 inliers (Q4, PnPsolver.cpp:311-331);
    plane = "wall":  world Z = 6 exactly (the same, facing the camera);
    plane = "tilted": a random plane through the view, coplanar up to float rounding (ill-conditioned
            but mostly finite samples);
    plane = "duplicates": a frustum scene in which 25 % of the correspondences repeat another one
            exactly (3D and 2D), so samples with repeated points are rank-deficient;
    plane = "floor0" / "wall0": the floor / wall moved into a plane THROUGH THE WORLD ORIGIN (world
            Y = 0 / Z = 0 exactly; the camera pose carries the offset, so the images are the same
            geometry).  MLPnP's planarity test is rank(points3 * points3^T) == 2 on uncentred world
            points (MLPnPsolver.cpp:346-364), which only such a plane passes: its samples take the
            planar branch (9-column A, :404-435; 4-way sign test, :497-558).
    The camera looks at the plane from 1.5-9 m; points outside the image are redrawn."""
    if plane == "duplicates":
        sc = make_pnp_scene(rng, n, inlier_ratio, noise=noise, n_points=n_points)
        k = n // 4
        src = rng.choice(n - k, size=k)
        dst = n - k + np.arange(k)
        for a in (sc.p2d, sc.p3dw, sc.sigma2):
            a[dst] = a[src]
        sc.inlier_true[dst] = sc.inlier_true[src]
        return sc
    origin_off = {"floor0": np.array([0.0, 1.5, 0.0]), "wall0": np.array([0.0, 0.0, 6.0])}.get(plane)
    if origin_off is not None:
        plane = plane[:-1]
    R = random_rotation(rng, 0.25)
    t = rng.uniform(-0.5, 0.5, size=3)
    if plane == "tilted":
        nrm = np.array([0.0, -1.0, -0.4]) + rng.normal(size=3) * 0.3
        nrm /= np.linalg.norm(nrm)
        e1 = np.cross(nrm, [1.0, 0.0, 0.0])
        e1 /= np.linalg.norm(e1)
        e2 = np.cross(nrm, e1)
        p0 = R.T @ (np.array([0.0, 0.5, 5.0]) - t)
    pts = []
    while sum(len(p) for p in pts) < n:
        m = 4 * n
        if plane == "floor":
            W = np.stack([rng.uniform(-6, 6, m), np.full(m, 1.5), rng.uniform(0.5, 12, m)], 1)
        elif plane == "wall":
            W = np.stack([rng.uniform(-6, 6, m), rng.uniform(-4, 4, m), np.full(m, 6.0)], 1)
        elif plane == "tilted":
            a, b = rng.uniform(-6, 6, m), rng.uniform(-6, 6, m)
            W = p0 + a[:, None] * e1 + b[:, None] * e2
        else:
            raise ValueError(plane)
        W = W.astype(np.float32).astype(np.float64)
        Xc = W @ R.T + t
        z = Xc[:, 2]
        with np.errstate(divide="ignore", invalid="ignore"):
            u = float(FX) * Xc[:, 0] / z + float(CX)
            v = float(FY) * Xc[:, 1] / z + float(CY)
        ok = (z > 1.5) & (z < 9.0) & (u >= 0) & (u < WIDTH) & (v >= 0) & (v < HEIGHT)
        pts.append(W[ok])
    Xw = np.concatenate(pts)[:n]
    if origin_off is not None:  # same camera-frame points: Xc = R (Xw - off) + (t + R off)
        Xw = Xw - origin_off    # exact: the plane coordinate becomes +0.0
        t = t + R @ origin_off
    return _observe(rng, R, t, Xw, inlier_ratio, noise, n_points)


@dataclasses.dataclass
class Sim3Pair:
    """Raw Sim3Solver constructor inputs (Sim3Solver.cpp:6-85) for one keyframe pair."""
    valid: np.ndarray    # uint8 [n1]
    Xw1: np.ndarray      # float32 [n1,3]  pMP1->GetWorldPos()
    Xw2: np.ndarray      # float32 [n1,3]  pMP2->GetWorldPos()
    sigma2_1: np.ndarray  # float32 [n1]
    sigma2_2: np.ndarray  # float32 [n1]
    R1: np.ndarray       # float32 [3,3]  KF1 Rcw
    t1: np.ndarray       # float32 [3]
    R2: np.ndarray
    t2: np.ndarray
    K1: np.ndarray       # float32 [4] fx, fy, cx, cy
    K2: np.ndarray
    inlier_true: np.ndarray  # bool [n1]

    @property
    def n1(self) -> int:
        return int(self.valid.shape[0])


def make_sim3_pair(rng: np.random.Generator, n1: int, n_inliers: int, invalid_frac: float = 0.0,
                   noise3d: float = 0.01, degenerate: str | None = None) -> Sim3Pair:
    """Two keyframes seeing the same points; map 2 carries a rigid loop drift (Rd, td).

    Physical point P: Xw1 = P (+noise), Xw2 = Rd P + td (+noise).  KF1: Xc1 = R1 P + t1.
    KF2 is displaced by (Rrel, trel) from KF1, expressed in map-2 coordinates, so that
    Xc2 = Rrel Xc1 + trel for inliers.  Outliers of map 2 are unrelated points in front of KF2.

    degenerate = "collinear": 40 % of the matches lie on one 3D line (a pole, a door edge) in
    both maps, so 3-point samples drawn from them are collinear (Horn's M has rank 1, the 4x4 N
    repeated eigenvalues: Sim3Solver.cpp:139-151, :196-266); "duplicates": 30 % of the matches
    repeat another match exactly, so samples can hold the same point twice.
    """
    R1 = random_rotation(rng, 0.3)
    t1 = rng.uniform(-1, 1, size=3)
    Rd = random_rotation(rng, 0.2)
    td = rng.uniform(-0.5, 0.5, size=3)
    Rrel = random_rotation(rng, 0.15)
    trel = rng.uniform(-0.3, 0.3, size=3)
    R2 = Rrel @ R1 @ Rd.T
    t2 = Rrel @ (t1 - R1 @ Rd.T @ td) + trel
    fx, fy, cx, cy = float(FX), float(FY), float(CX), float(CY)
    u = rng.uniform(0, WIDTH, size=n1)
    v = rng.uniform(0, HEIGHT, size=n1)
    d = rng.uniform(1.0, 8.0, size=n1)
    Xc1 = np.stack([(u - cx) / fx * d, (v - cy) / fy * d, d], axis=1)
    P = (Xc1 - t1) @ R1
    if degenerate == "collinear":
        k = (2 * n1) // 5
        a = P[0]
        dirn = rng.normal(size=3)
        dirn /= np.linalg.norm(dirn)
        P[:k] = a + rng.uniform(-1.0, 1.0, size=k)[:, None] * dirn
    Xw1 = P + rng.normal(size=P.shape) * noise3d
    Xw2 = P @ Rd.T + td + rng.normal(size=P.shape) * noise3d
    if degenerate == "collinear":  # exactly collinear in both maps (no 3D noise on the line)
        Xw1[:k] = P[:k]
        Xw2[:k] = P[:k] @ Rd.T + td
    if degenerate == "duplicates":
        k = (3 * n1) // 10
        src = rng.choice(n1 - k, size=k)
        Xw1[n1 - k:] = Xw1[src]
        Xw2[n1 - k:] = Xw2[src]
    inl = np.zeros(n1, dtype=bool)
    inl[rng.permutation(n1)[:n_inliers]] = True
    nout = int((~inl).sum())
    uo = rng.uniform(0, WIDTH, size=nout)
    vo = rng.uniform(0, HEIGHT, size=nout)
    do = rng.uniform(1.0, 8.0, size=nout)
    Xc2o = np.stack([(uo - cx) / fx * do, (vo - cy) / fy * do, do], axis=1)
    Xw2[~inl] = (Xc2o - t2) @ R2
    levels1 = rng.choice(N_LEVELS, size=n1, p=level_probabilities())
    levels2 = rng.choice(N_LEVELS, size=n1, p=level_probabilities())
    s2 = level_sigma2()
    valid = np.ones(n1, dtype=np.uint8)
    if invalid_frac > 0:
        valid[rng.random(n1) < invalid_frac] = 0
    K = np.array([FX, FY, CX, CY], dtype=np.float32)
    return Sim3Pair(valid=valid, Xw1=Xw1.astype(np.float32), Xw2=Xw2.astype(np.float32),
                    sigma2_1=s2[levels1].astype(np.float32), sigma2_2=s2[levels2].astype(np.float32),
                    R1=R1.astype(np.float32), t1=t1.astype(np.float32), R2=R2.astype(np.float32),
                    t2=t2.astype(np.float32), K1=K, K2=K.copy(), inlier_true=inl)


@dataclasses.dataclass
class PoseOptFrame:
    """Optimizer::PoseOptimization inputs (Optimizer.cpp:205-325) for one Frame (monocular, or stereo
    slots where u_right >= 0)."""
    has_mp: np.ndarray      # uint8 [n]   mvpMapPoints[i] != NULL
    uv: np.ndarray          # float32 [n,2] mvKeysUn[i].pt
    Xw: np.ndarray          # float32 [n,3] MapPoint::GetWorldPos() (0 where has_mp == 0)
    inv_sigma2: np.ndarray  # float32 [n]   mvInvLevelSigma2[octave] = 1.0f / mvLevelSigma2
    Tcw: np.ndarray         # float32 [4,4] initial pFrame->mTcw (e.g. the RANSAC pose)
    R_true: np.ndarray
    t_true: np.ndarray
    inlier_true: np.ndarray  # bool [n]
    fx: np.float32 = FX
    fy: np.float32 = FY
    cx: np.float32 = CX
    cy: np.float32 = CY
    u_right: np.ndarray = None  # float32 [n] mvuRight (-1: monocular slot), None: monocular Frame
    bf: np.float32 = np.float32(0.0)

    @property
    def n(self) -> int:
        return int(self.uv.shape[0])


# EuRoC.yaml stereo rig (Camera.bf: baseline 0.110 m x fx)
EUROC_BF = np.float32(47.90639384423901)


def make_poseopt_frame(rng: np.random.Generator, n: int, inlier_ratio: float = 0.8, rot_noise: float = 0.02,
                       trans_noise: float = 0.05, no_mp_frac: float = 0.0, noise: bool = True,
                       stereo_frac: float = 0.0) -> PoseOptFrame:
    """A PnP-shaped scene whose initial Tcw is the true pose perturbed like a RANSAC estimate.
    stereo_frac > 0: that share of the slots carries a right-image coordinate mvuRight = u - bf/z
    (+ the same pixel noise, outliers displaced), the rest are monocular (-1)."""
    sc = make_pnp_scene(rng, n, inlier_ratio, noise=noise)
    dR = random_rotation(rng, rot_noise)
    R0 = dR @ sc.R_true
    t0 = sc.t_true + rng.normal(size=3) * trans_noise
    T = np.eye(4, dtype=np.float32)
    T[:3, :3] = R0.astype(np.float32)
    T[:3, 3] = t0.astype(np.float32)
    has = np.ones(n, dtype=np.uint8)
    if no_mp_frac > 0:
        has[rng.random(n) < no_mp_frac] = 0
    Xw = sc.p3dw.copy()
    Xw[has == 0] = 0.0
    inv = (np.float32(1.0) / sc.sigma2).astype(np.float32)
    fr = PoseOptFrame(has_mp=has, uv=sc.p2d, Xw=Xw, inv_sigma2=inv, Tcw=T, R_true=sc.R_true, t_true=sc.t_true,
                      inlier_true=sc.inlier_true)
    if stereo_frac > 0:
        pc = sc.p3dw.astype(np.float64) @ sc.R_true.T + sc.t_true
        z = np.maximum(pc[:, 2], 1e-3)
        ur = sc.p2d[:, 0].astype(np.float64) - float(EUROC_BF) / z
        if noise:
            ur = ur + rng.normal(size=n) * np.sqrt(sc.sigma2)
        ur = np.where(sc.inlier_true, ur, ur + rng.uniform(-40, 40, size=n))
        st = (rng.random(n) < stereo_frac) & (ur >= 0.0)  # no right match off the image: monocular slot
        fr.u_right = np.where(st, ur, -1.0).astype(np.float32)
        fr.bf = EUROC_BF
    return fr


@dataclasses.dataclass
class BowFeatures:
    """One view's ORBmatcher::SearchByBoW inputs: ORB descriptors (mDescriptors, 32 B rows),
    keypoint angles, map-point validity (GetMapPointMatches()[i] && !isBad()) and the DBoW2
    FeatureVector (mFeatVec: node id -> ascending feature indices) as CSR."""
    n: int
    desc: np.ndarray        # uint8 [n,32]
    angle: np.ndarray       # float32 [n] degrees in [0, 360)
    valid: np.ndarray       # uint8 [n]
    node_id: np.ndarray     # uint32 [nodes] ascending
    node_begin: np.ndarray  # int32 [nodes+1]
    feat: np.ndarray        # uint32 [n]


# DBoW2 ORB vocabulary shape (k = 10, L = 6, ORBvoc.txt) and Frame::ComputeBoW's levelsup = 4
# (src/Frame.cpp: transform(..., 4)): FeatureVector keys are node ids of depth 2, i.e. 11..110 with
# the vocabulary's breadth-first numbering.
BOW_NODE_IDS = np.arange(11, 111, dtype=np.uint32)


def _feature_vector(nodes: np.ndarray):
    """CSR of node -> ascending feature indices from a per-feature node id (DBoW2 adds features in
    index order, so each node's vector is ascending)."""
    order = np.lexsort((np.arange(len(nodes)), nodes))
    ids, counts = np.unique(nodes[order], return_counts=True)
    begin = np.zeros(len(ids) + 1, np.int32)
    begin[1:] = np.cumsum(counts)
    return ids.astype(np.uint32), begin, order.astype(np.uint32)


def _node_draw(rng: np.random.Generator, n: int, skew: float) -> np.ndarray:
    w = 1.0 / np.arange(1, len(BOW_NODE_IDS) + 1) ** skew
    w = rng.permutation(w / w.sum())
    return rng.choice(BOW_NODE_IDS, size=n, p=w)


def make_bow_view(rng: np.random.Generator, n: int, valid_frac: float = 1.0, skew: float = 0.8,
                  nodes: np.ndarray | None = None) -> BowFeatures:
    """Random ORB view: uniform 256-bit descriptors and angles, Zipf-skewed node occupancy."""
    if nodes is None:
        nodes = _node_draw(rng, n, skew)
    node_id, begin, feat = _feature_vector(np.asarray(nodes, np.uint32))
    return BowFeatures(n, rng.integers(0, 256, size=(n, 32), dtype=np.uint8),
                       rng.uniform(0, 360, n).astype(np.float32),
                       (rng.random(n) < valid_frac).astype(np.uint8), node_id, begin, feat)


def _flip_bits(rng: np.random.Generator, desc: np.ndarray, flips: np.ndarray) -> np.ndarray:
    out = desc.copy()
    for i, k in enumerate(flips):
        bits = rng.choice(256, size=int(k), replace=False)
        np.bitwise_xor.at(out[i], bits // 8, (1 << (bits % 8)).astype(np.uint8))
    return out


def make_bow_related(rng: np.random.Generator, src: BowFeatures, n: int, overlap: float, rot_deg: float,
                     valid_frac: float = 0.85, same_node: float = 0.9, mean_flips: float = 18.0,
                     skew: float = 0.8) -> BowFeatures:
    """A second view sharing ~overlap*n features with `src`: a shared feature copies a source
    descriptor with Poisson(mean_flips) bit flips, its angle rotated by rot_deg (+ 2 degree noise),
    and keeps the source node with probability `same_node` (quantisation noise otherwise)."""
    k = min(int(round(overlap * n)), src.n)
    nodes = _node_draw(rng, n, skew)
    v = make_bow_view(rng, n, valid_frac, skew, nodes)
    src_nodes = np.empty(src.n, np.uint32)
    for j in range(len(src.node_id)):
        src_nodes[src.feat[src.node_begin[j]:src.node_begin[j + 1]]] = src.node_id[j]
    dst = rng.choice(n, size=k, replace=False)
    srcs = rng.choice(src.n, size=k, replace=False)
    v.desc[dst] = _flip_bits(rng, src.desc[srcs], np.minimum(rng.poisson(mean_flips, k), 255))
    v.angle[dst] = np.mod(src.angle[srcs] + np.float32(rot_deg) + rng.normal(0, 2, k), 360).astype(np.float32)
    keep = rng.random(k) < same_node
    nodes[dst[keep]] = src_nodes[srcs[keep]]
    v.node_id, v.node_begin, v.feat = _feature_vector(nodes)
    return v


# ---- ORBmatcher::SearchBySim3 inputs ----------------------------------------------------------
GRID_COLS, GRID_ROWS = 64, 48  # FRAME_GRID_COLS / ROWS (include/Frame.hpp:20-21)


@dataclasses.dataclass
class Sim3KF:
    """One KeyFrame as SearchBySim3 reads it (rsc_sim3_kf, include/rsc.h)."""
    n: int
    kp: np.ndarray          # float32 [n,2] mvKeysUn[i].pt
    octave: np.ndarray      # int32 [n]
    desc: np.ndarray        # uint8 [n,32]
    cell_begin: np.ndarray  # int32 [64*48+1]
    cell_feat: np.ndarray   # int32 []
    Rcw: np.ndarray         # float32 [3,3]
    tcw: np.ndarray         # float32 [3]
    mp_state: np.ndarray    # uint8 [n] 0 NULL, 1 good, 2 bad
    mp_pos: np.ndarray      # float32 [n,3]
    mp_dmax: np.ndarray     # float32 [n]
    mp_dmin: np.ndarray     # float32 [n]
    mp_desc: np.ndarray     # uint8 [n,32]
    mp_id: np.ndarray       # int64 [n] MapPoint identity (-1 = none), to build matched12
    fx: float = float(FX)
    fy: float = float(FY)
    cx: float = float(CX)
    cy: float = float(CY)
    min_x: float = 0.0
    max_x: float = float(WIDTH)
    min_y: float = 0.0
    max_y: float = float(HEIGHT)


def scale_factors() -> np.ndarray:
    sf = [np.float32(1.0)]
    for _ in range(1, N_LEVELS):
        sf.append(np.float32(sf[-1] * SCALE_FACTOR))
    return np.array(sf, np.float32)


LOG_SCALE_FACTOR = np.float32(np.log(np.float32(1.2)))
GRID_W_INV = np.float32(np.float32(GRID_COLS) / np.float32(WIDTH))   # mfGridElementWidthInv (Frame.cpp)
GRID_H_INV = np.float32(np.float32(GRID_ROWS) / np.float32(HEIGHT))


def build_grid(kp: np.ndarray):
    """Frame::AssignFeaturesToGrid (PosInGrid with round()), as CSR over cell = ix * 48 + iy."""
    px = np.floor((kp[:, 0] - 0.0) * GRID_W_INV + 0.5).astype(np.int64)
    py = np.floor((kp[:, 1] - 0.0) * GRID_H_INV + 0.5).astype(np.int64)
    ok = (px >= 0) & (px < GRID_COLS) & (py >= 0) & (py < GRID_ROWS)
    cell = np.where(ok, px * GRID_ROWS + py, -1)
    idx = np.nonzero(ok)[0]
    order = idx[np.lexsort((idx, cell[idx]))]
    counts = np.bincount(cell[order], minlength=GRID_COLS * GRID_ROWS)
    begin = np.zeros(GRID_COLS * GRID_ROWS + 1, np.int32)
    begin[1:] = np.cumsum(counts)
    return begin, order.astype(np.int32)


def _flip(rng, d, mean):
    out = d.copy()
    for i in range(len(out)):
        k = min(int(rng.poisson(mean)), 255)
        bits = rng.choice(256, size=k, replace=False)
        np.bitwise_xor.at(out[i], bits // 8, (1 << (bits % 8)).astype(np.uint8))
    return out


def make_sim3match_pair(rng: np.random.Generator, n_points: int = 1000, n_extra: int = 300,
                        matched_frac: float = 0.3, bad_frac: float = 0.03, noise_px: float = 1.0,
                        pose_noise: float = 0.002):
    """Two KeyFrames observing n_points common world points (plus n_extra unmatched keypoints each),
    the relative pose (R12, t12) with a small error (a Sim3 RANSAC estimate), and the matched12 input
    (a `matched_frac` share of common points already matched).  Returns (kf1, kf2, R12, t12, matched12)."""
    sf = scale_factors()
    P = np.stack([rng.uniform(-3, 3, n_points), rng.uniform(-2, 2, n_points), rng.uniform(2, 10, n_points)], 1)
    R1 = random_rotation(rng, 0.2)
    t1 = -R1 @ np.array([0.0, 0.0, 0.0])
    R2 = random_rotation(rng, 0.15) @ R1
    c2 = rng.normal(0, 0.3, 3)
    t2 = -R2 @ c2
    mp_ids = np.arange(n_points)
    mp_desc = rng.integers(0, 256, (n_points, 32), dtype=np.uint8)
    kfs = []
    for R, t in ((R1, t1), (R2, t2)):
        Xc = P @ R.T + t
        uv = np.stack([FX * Xc[:, 0] / Xc[:, 2] + CX, FY * Xc[:, 1] / Xc[:, 2] + CY], 1)
        vis = (Xc[:, 2] > 0.1) & (uv[:, 0] >= 0) & (uv[:, 0] < WIDTH) & (uv[:, 1] >= 0) & (uv[:, 1] < HEIGHT)
        ids = np.nonzero(vis)[0]
        m = len(ids) + n_extra
        kp = np.zeros((m, 2), np.float32)
        kp[:len(ids)] = uv[ids] + rng.normal(0, noise_px, (len(ids), 2))
        kp[len(ids):] = np.stack([rng.uniform(0, WIDTH, n_extra), rng.uniform(0, HEIGHT, n_extra)], 1)
        kp = np.clip(kp, 0, [WIDTH - 1e-3, HEIGHT - 1e-3]).astype(np.float32)
        octave = rng.choice(N_LEVELS, size=m, p=level_probabilities()).astype(np.int32)
        desc = rng.integers(0, 256, (m, 32), dtype=np.uint8)
        desc[:len(ids)] = _flip(rng, mp_desc[ids], 8.0)
        perm = rng.permutation(m)  # keypoint order unrelated to point order
        kp, octave, desc = kp[perm], octave[perm], desc[perm]
        mp_id = np.full(m, -1, np.int64)
        src = np.concatenate([ids, np.full(n_extra, -1)])[perm]
        mp_id[:] = src
        has = mp_id >= 0
        state = np.where(has, 1, 0).astype(np.uint8)
        state[has & (rng.random(m) < bad_frac)] = 2
        pos = np.zeros((m, 3), np.float32)
        pos[has] = P[mp_id[has]]
        dist = np.linalg.norm(P[np.maximum(mp_id, 0)] - (-R.T @ t), axis=1)
        dmax = np.where(has, dist * sf[octave], 0).astype(np.float32)   # MapPoint::UpdateNormalAndDepth
        dmin = (dmax / sf[N_LEVELS - 1]).astype(np.float32)
        mdesc = np.zeros((m, 32), np.uint8)
        mdesc[has] = mp_desc[mp_id[has]]
        begin, feat = build_grid(kp)
        kfs.append(Sim3KF(m, kp, octave, desc, begin, feat, R.astype(np.float32), t.astype(np.float32), state,
                          pos, dmax, dmin, mdesc, mp_id))
    kf1, kf2 = kfs
    # p1 = R12 p2 + t12 (camera 2 -> camera 1), perturbed like a RANSAC estimate
    R12 = (random_rotation(rng, pose_noise) @ (R1 @ R2.T)).astype(np.float32)
    t12 = (t1 - (R1 @ R2.T) @ t2 + rng.normal(0, pose_noise, 3)).astype(np.float32)
    where2 = {int(i): j for j, i in enumerate(kf2.mp_id) if i >= 0}
    matched12 = np.full(kf1.n, -1, np.int32)
    for i, mid in enumerate(kf1.mp_id):
        if mid >= 0 and rng.random() < matched_frac:
            matched12[i] = where2.get(int(mid), -2)
    return kf1, kf2, R12, t12, matched12


# ---- Optimizer::OptimizeSim3 inputs ----------------------------------------------------------------
def quat_from_R(m) -> np.ndarray:
    """Quaterniond(Matrix3d) (Eigen's trace / largest-diagonal algorithm), coefficients (x, y, z, w)."""
    m = np.asarray(m, np.float64)
    t = m[0, 0] + m[1, 1] + m[2, 2]
    if t > 0.0:
        t = np.sqrt(t + 1.0)
        w = 0.5 * t
        t = 0.5 / t
        return np.array([(m[2, 1] - m[1, 2]) * t, (m[0, 2] - m[2, 0]) * t, (m[1, 0] - m[0, 1]) * t, w])
    i = 0
    if m[1, 1] > m[0, 0]:
        i = 1
    if m[2, 2] > m[i, i]:
        i = 2
    j, k = (i + 1) % 3, (i + 2) % 3
    c = np.zeros(3)
    t = np.sqrt(m[i, i] - m[j, j] - m[k, k] + 1.0)
    c[i] = 0.5 * t
    t = 0.5 / t
    w = (m[k, j] - m[j, k]) * t
    c[j] = (m[j, i] + m[i, j]) * t
    c[k] = (m[k, i] + m[i, k]) * t
    return np.array([c[0], c[1], c[2], w])


@dataclasses.dataclass
class Sim3OptProblem:
    """Optimizer::OptimizeSim3(pKF1, pKF2, vpMatches1, g2oS12, th2) inputs (Optimizer.cpp:1054-1145),
    per KF1 keypoint slot i: valid (a correspondence: both MapPoints present, not bad, i2 >= 0),
    X1w = vpMapPoints1[i]->GetWorldPos(), X2w = vpMatches1[i]->GetWorldPos(), uv1 = KF1 mvKeysUn[i],
    uv2 = KF2 mvKeysUn[i2], inv1/inv2 = mvInvLevelSigma2 of the octaves."""
    valid: np.ndarray   # uint8 [n]
    X1w: np.ndarray     # float32 [n,3]
    X2w: np.ndarray     # float32 [n,3]
    uv1: np.ndarray     # float32 [n,2]
    uv2: np.ndarray     # float32 [n,2]
    inv1: np.ndarray    # float32 [n]
    inv2: np.ndarray    # float32 [n]
    R1w: np.ndarray     # float32 [3,3]
    t1w: np.ndarray     # float32 [3]
    R2w: np.ndarray
    t2w: np.ndarray
    S0: np.ndarray      # float64 [8] g2oS12 on entry: q (x, y, z, w), t, s
    R12_true: np.ndarray
    t12_true: np.ndarray
    inlier_true: np.ndarray  # bool [n]
    K1: np.ndarray = dataclasses.field(default_factory=lambda: np.array([FX, FY, CX, CY], np.float32))
    K2: np.ndarray = dataclasses.field(default_factory=lambda: np.array([FX, FY, CX, CY], np.float32))
    th2: float = 10.0   # LoopClosing.cpp:311

    @property
    def n(self) -> int:
        return int(self.valid.shape[0])

    def poses24(self) -> np.ndarray:
        return np.ascontiguousarray(np.concatenate([np.asarray(self.R1w, np.float32).ravel(),
                                                    np.asarray(self.t1w, np.float32),
                                                    np.asarray(self.R2w, np.float32).ravel(),
                                                    np.asarray(self.t2w, np.float32)]), np.float32)

    def K8(self) -> np.ndarray:
        return np.ascontiguousarray(np.concatenate([self.K1, self.K2]), np.float32)


def make_sim3opt_problem(rng: np.random.Generator, n: int, valid_frac: float = 0.9, outlier_frac: float = 0.1,
                         pose_noise: float = 0.01, noise: bool = True, drift: float = 0.01) -> Sim3OptProblem:
    """A loop-closure pair: KF2-camera points X2c, the true relative pose S12 (scale 1, as Sim3Solver
    fixes it), X1c = S12 X2c (+ map drift noise), both KeyFrames' world poses, observations with
    pyramid-level pixel noise, outliers displaced, and the initial g2oS12 = a perturbed S12 as
    Sim3Solver would return it (float R, t -> Sim3(R.cast<double>(), t.cast<double>(), 1))."""
    s2 = level_sigma2()
    X2c = np.stack([rng.uniform(-3, 3, n), rng.uniform(-2, 2, n), rng.uniform(1.5, 9, n)], 1)
    R12 = random_rotation(rng, 0.3)
    t12 = rng.normal(0, 0.4, 3)
    X1c = X2c @ R12.T + t12 + (rng.normal(0, drift, (n, 3)) if noise else 0.0)
    R1w, R2w = random_rotation(rng), random_rotation(rng)
    t1w, t2w = rng.normal(0, 2, 3), rng.normal(0, 2, 3)
    X1w = ((X1c - t1w) @ R1w).astype(np.float32)   # R^T (Xc - t)
    X2w = ((X2c - t2w) @ R2w).astype(np.float32)
    probs = level_probabilities()
    o1 = rng.choice(N_LEVELS, size=n, p=probs)
    o2 = rng.choice(N_LEVELS, size=n, p=probs)
    uv1 = np.stack([FX * X1c[:, 0] / X1c[:, 2] + CX, FY * X1c[:, 1] / X1c[:, 2] + CY], 1)
    uv2 = np.stack([FX * X2c[:, 0] / X2c[:, 2] + CX, FY * X2c[:, 1] / X2c[:, 2] + CY], 1)
    if noise:
        uv1 = uv1 + rng.normal(size=(n, 2)) * np.sqrt(s2[o1])[:, None]
        uv2 = uv2 + rng.normal(size=(n, 2)) * np.sqrt(s2[o2])[:, None]
    inl = rng.random(n) >= outlier_frac
    bad = ~inl
    nb = int(bad.sum())
    uv1[bad] += rng.choice([-1.0, 1.0], (nb, 2)) * rng.uniform(12, 60, (nb, 2))  # gross: >= 12 px
    valid = (rng.random(n) < valid_frac).astype(np.uint8)
    Rp = (random_rotation(rng, pose_noise) @ R12).astype(np.float32)
    tp = (t12 + rng.normal(0, pose_noise, 3)).astype(np.float32)
    S0 = np.concatenate([quat_from_R(Rp.astype(np.float64)), tp.astype(np.float64), [1.0]])
    inv = (np.float32(1.0) / s2).astype(np.float32)
    return Sim3OptProblem(valid=valid, X1w=X1w, X2w=X2w, uv1=uv1.astype(np.float32), uv2=uv2.astype(np.float32),
                          inv1=inv[o1], inv2=inv[o2], R1w=R1w.astype(np.float32), t1w=t1w.astype(np.float32),
                          R2w=R2w.astype(np.float32), t2w=t2w.astype(np.float32), S0=S0, R12_true=R12,
                          t12_true=t12, inlier_true=inl)


# ---- KeyFrameDatabase scenes (KeyFrameDatabase.cpp) ---------------------------------------------
VOCAB_WORDS = 10 ** 6  # ORBvoc.txt: k = 10, L = 6 -> up to 10^6 leaves


@dataclasses.dataclass
class KFDBScene:
    """KeyFrames along a trajectory: bows[k] = (word ids ascending uint32, L1-normalised float64
    TF-IDF values), covis[k] = GetBestCovisibilityKeyFrames(10) (nearest along the trajectory);
    the place-word pools make neighbouring KeyFrames share words and a small set of frequent words
    makes most KeyFrames share a few (the inverted file's long lists)."""
    bows: list
    covis: list
    pools: np.ndarray
    frequent: np.ndarray
    step: int
    span: int
    places: int = 0  # distinct places (n_kfs / revisits)


def _bow_from(rng: np.random.Generator, words: np.ndarray):
    ids = np.unique(words.astype(np.uint32))
    vals = rng.exponential(1.0, len(ids)) * rng.uniform(0.5, 3.0, len(ids))  # tf * idf
    s = vals.sum()
    return ids, (vals / s if s > 0 else vals).astype(np.float64)


def _place_words(rng, sc: KFDBScene, pos: float, n_words: int, noise_frac: float = 0.1):
    c = int(round(pos * sc.step))
    lo = max(0, min(len(sc.pools) - sc.span, c))
    own = rng.choice(sc.pools[lo:lo + sc.span], size=int(n_words * (1 - noise_frac)), replace=False)
    noise = rng.integers(0, VOCAB_WORDS, int(n_words * noise_frac))
    freq = sc.frequent[rng.random(len(sc.frequent)) < 0.3]
    return np.concatenate([own, noise, freq])


def make_kfdb_scene(rng: np.random.Generator, n_kfs: int, words_per_kf: int = 600, step: int = 150,
                    n_frequent: int = 40, revisits: int = 1) -> KFDBScene:
    """KeyFrames along a trajectory; KeyFrame k observes the words of place k (consecutive places
    share words).  revisits > 1: the trajectory covers the same n_kfs / revisits places that many
    times (a map built over repeated passes, as EuRoC's MH / V sequences), with a jittered place per
    pass, so a relocalization query matches one covisibility group per pass."""
    span = 2 * words_per_kf
    places = -(-n_kfs // revisits)
    pools = rng.permutation(VOCAB_WORDS)[: places * step + span].astype(np.uint32)
    frequent = rng.integers(0, VOCAB_WORDS, n_frequent).astype(np.uint32)
    sc = KFDBScene([], [], pools, frequent, step, span)
    sc.places = places
    for k in range(n_kfs):
        pos = k if revisits == 1 else (k % places) + rng.uniform(-0.3, 0.3)
        sc.bows.append(_bow_from(rng, _place_words(rng, sc, pos, words_per_kf)))
    for k in range(n_kfs):
        near = sorted((j for j in range(max(0, k - 8), min(n_kfs, k + 9)) if j != k), key=lambda j: (abs(j - k), j))
        sc.covis.append(np.array(near[:10], np.int32))
    return sc


def make_kfdb_query(rng: np.random.Generator, sc: KFDBScene, pos: float, words: int = 600):
    """A Frame's (or new KeyFrame's) BowVector observed at trajectory position pos."""
    return _bow_from(rng, _place_words(rng, sc, pos, words))


# ---- Gated events (rsc_reloc_events_gated / rsc_loop_events_gated) -------------------------------
def make_reloc_gate_event(rng: np.random.Generator, n_frame: int, cands, poisoned=(), stereo_frac: float = 0.0):
    """One Tracking::Relocalization() call: candidate scenes (n, inlier ratio) whose matches are subsets
    of one current Frame's n_frame keypoint slots (kp_index), and the Frame's mvuRight / mbf.
    Candidates listed in `poisoned` have a right-image coordinate on every slot they match that
    disagrees with their pose by 100+ px (a wrong stereo match), so PoseOptimization classifies those
    stereo edges as outliers (chi2 > 7.815) and the RANSAC pose is rejected (nGood < 10); with
    stereo_frac > 0 that share of the other candidates' slots carries a consistent mvuRight.
    Returns (scenes, u_right float32 [n_frame] (-1 = monocular slot), bf)."""
    scenes = [make_pnp_scene(rng, int(n), float(r), n_points=n_frame) for n, r in cands]
    ur = np.full(n_frame, -1.0, np.float32)
    for c, sc in enumerate(scenes):
        if c in poisoned:
            continue
        pc = sc.p3dw.astype(np.float64) @ sc.R_true.T + sc.t_true
        u = sc.p2d[:, 0].astype(np.float64) - float(EUROC_BF) / np.maximum(pc[:, 2], 1e-3)
        st = (rng.random(sc.n) < stereo_frac) & (u >= 0.0) & sc.inlier_true
        ur[sc.kp_index[st]] = u[st].astype(np.float32)
    for c in poisoned:
        sc = scenes[c]
        ur[sc.kp_index] = (sc.p2d[:, 0] + rng.uniform(100.0, 200.0, sc.n)).astype(np.float32)
    return scenes, ur, EUROC_BF


def _make_kf(rng, P, mp_desc, R, t, n_extra, bad_frac, noise_px):
    """A KeyFrame (Sim3KF) observing the world points P from pose (R, t): keypoints of the visible points
    (+ pixel noise) and n_extra unmatched ones in a random order, octaves, descriptors, MapPoints."""
    sf = scale_factors()
    Xc = P @ R.T + t
    uv = np.stack([FX * Xc[:, 0] / Xc[:, 2] + CX, FY * Xc[:, 1] / Xc[:, 2] + CY], 1)
    vis = (Xc[:, 2] > 0.1) & (uv[:, 0] >= 0) & (uv[:, 0] < WIDTH) & (uv[:, 1] >= 0) & (uv[:, 1] < HEIGHT)
    ids = np.nonzero(vis)[0]
    m = len(ids) + n_extra
    kp = np.zeros((m, 2), np.float32)
    kp[:len(ids)] = uv[ids] + rng.normal(0, noise_px, (len(ids), 2))
    kp[len(ids):] = np.stack([rng.uniform(0, WIDTH, n_extra), rng.uniform(0, HEIGHT, n_extra)], 1)
    kp = np.clip(kp, 0, [WIDTH - 1e-3, HEIGHT - 1e-3]).astype(np.float32)
    octave = rng.choice(N_LEVELS, size=m, p=level_probabilities()).astype(np.int32)
    desc = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    desc[:len(ids)] = _flip(rng, mp_desc[ids], 8.0)
    perm = rng.permutation(m)
    kp, octave, desc = kp[perm], octave[perm], desc[perm]
    mp_id = np.concatenate([ids, np.full(n_extra, -1)])[perm].astype(np.int64)
    has = mp_id >= 0
    state = np.where(has, 1, 0).astype(np.uint8)
    state[has & (rng.random(m) < bad_frac)] = 2
    pos = np.zeros((m, 3), np.float32)
    pos[has] = P[mp_id[has]]
    dist = np.linalg.norm(P[np.maximum(mp_id, 0)] - (-R.T @ t), axis=1)
    dmax = np.where(has, dist * sf[octave], 0).astype(np.float32)
    dmin = (dmax / sf[N_LEVELS - 1]).astype(np.float32)
    mdesc = np.zeros((m, 32), np.uint8)
    mdesc[has] = mp_desc[mp_id[has]]
    begin, feat = build_grid(kp)
    return Sim3KF(m, kp, octave, desc, begin, feat, R.astype(np.float32), t.astype(np.float32), state, pos, dmax,
                  dmin, mdesc, mp_id)


def sim3_pair_from_kfs(kf1: Sim3KF, kf2: Sim3KF, matches12: np.ndarray) -> Sim3Pair:
    """Sim3Solver(pKF1, pKF2, vpMatched12) constructor inputs (Sim3Solver.cpp:6-85) from two KeyFrame
    views and the BoW matches (KF2 keypoint index per KF1 slot, -1 none): a slot is usable when both
    MapPoints exist and neither is bad; sigma^2 from the keypoints' octaves."""
    s2 = level_sigma2()
    n1 = kf1.n
    m = np.asarray(matches12)
    y = np.maximum(m, 0)
    valid = (m >= 0) & (kf1.mp_state == 1) & (kf2.mp_state[y] == 1)
    K = np.array([kf1.fx, kf1.fy, kf1.cx, kf1.cy], np.float32)
    return Sim3Pair(valid=valid.astype(np.uint8), Xw1=np.ascontiguousarray(kf1.mp_pos, np.float32),
                    Xw2=np.ascontiguousarray(kf2.mp_pos[y], np.float32),
                    sigma2_1=s2[kf1.octave].astype(np.float32), sigma2_2=s2[kf2.octave[y]].astype(np.float32),
                    R1=kf1.Rcw, t1=kf1.tcw, R2=kf2.Rcw, t2=kf2.tcw, K1=K, K2=K.copy(),
                    inlier_true=np.zeros(n1, bool))


def make_loop_gate_event(rng: np.random.Generator, cands, n_points: int = 700, n_extra: int = 150,
                         match_frac: float = 0.6, poisoned=()):
    """One LoopClosing::ComputeSim3() call: the current KeyFrame and candidate KeyFrames observing a
    shared world (no map drift, scale 1), with BoW-style matches12 per candidate: cands = [right-match
    share, ...] of the matched KF1 MapPoints (the rest matched to a random KF2 MapPoint).  Candidates in
    `poisoned` carry keypoints displaced by 30-60 px from their MapPoints' projections (their Sim3
    RANSAC, which projects 3D points and never reads keypoints, still succeeds; OptimizeSim3's
    KF2-side reprojection edges all exceed th2, so the gate rejects it).
    Returns (kf1, [(kf2, matches12, Sim3Pair)])."""
    P = np.stack([rng.uniform(-3, 3, n_points), rng.uniform(-2, 2, n_points), rng.uniform(2, 9, n_points)], 1)
    mp_desc = rng.integers(0, 256, (n_points, 32), dtype=np.uint8)
    R1 = random_rotation(rng, 0.2)
    t1 = np.zeros(3)
    kf1 = _make_kf(rng, P, mp_desc, R1, t1, n_extra, 0.02, 1.0)
    out = []
    for c, good in enumerate(cands):
        R2 = random_rotation(rng, 0.12) @ R1
        t2 = -R2 @ rng.normal(0, 0.25, 3)
        kf2 = _make_kf(rng, P, mp_desc, R2, t2, n_extra, 0.02, 1.0)
        if c in poisoned:
            has = kf2.mp_id >= 0
            k = int(has.sum())
            off = rng.choice([-1.0, 1.0], (k, 2)) * rng.uniform(30.0, 60.0, (k, 2))
            kp = kf2.kp.copy()
            kp[has] = np.clip(kp[has] + off, 0, [WIDTH - 1e-3, HEIGHT - 1e-3])
            kf2.kp = kp.astype(np.float32)
            kf2.cell_begin, kf2.cell_feat = build_grid(kf2.kp)
        where2 = {int(i): j for j, i in enumerate(kf2.mp_id) if i >= 0}
        with_mp2 = np.nonzero(kf2.mp_id >= 0)[0]
        m12 = np.full(kf1.n, -1, np.int32)
        for i, mid in enumerate(kf1.mp_id):
            if mid < 0 or int(mid) not in where2 or rng.random() >= match_frac:
                continue
            m12[i] = where2[int(mid)] if rng.random() < good else int(rng.choice(with_mp2))
        out.append((kf2, m12, sim3_pair_from_kfs(kf1, kf2, m12)))
    return kf1, out
