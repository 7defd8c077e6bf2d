#!/usr/bin/env python3
"""Write the bench's 64 config-2 scenes (seeded as in bench.py) to tools/data/scenes.bin for the
diagnostic tools: int32 C, N; float32 [C*N][4] (x, y, z, sigma2); float32 [C*N][2] (u, v)."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-slam2-optimized_amd"))
from rsc import synth  # noqa: E402
rng = np.random.default_rng(20240)
sc = [synth.make_pnp_scene(rng, 2000, 0.4) for _ in range(64)]
os.makedirs(os.path.join(ROOT, "tools", "data"), exist_ok=True)
with open(os.path.join(ROOT, "tools", "data", "scenes.bin"), "wb") as f:
    np.array([64, 2000], np.int32).tofile(f)
    np.concatenate([np.concatenate([s.p3dw, s.sigma2[:, None]], 1) for s in sc]).astype(np.float32).tofile(f)
    np.concatenate([s.p2d for s in sc]).astype(np.float32).tofile(f)
