"""The split eigen stage's fail-loudly path on the device.

pnp_eig_split_kernel's chase wave and row wave hand each QR step over through LDS flags; a wait that
gives up (split_wait, rsc_quad.h) must never return eigenvectors built from stale rotations with
RSC_OK.  The test-only build orb-slam2-optimized_amd/lib/librsc_spin1.so (Makefile: the same sources
with RSC_SPLIT_SPIN_LIMIT=1) gives up after one poll, so the hand-offs of a split-form launch fail:
the call must return RSC_ERR_INTERNAL, and the next call of the same context (fault word cleared)
must fail the same way rather than hang.  Runs in a child process (a second librsc in its own
process).  The product library's split launches are covered by every config-2 parity test."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "orb-slam2-optimized_amd", "lib", "librsc_spin1.so")

CHILD = r"""
import sys
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import numpy as np
from rsc import engine, synth
ctx = engine.Context(0)
rng = np.random.default_rng(7)
# 8 candidates x 300 hypotheses = 2,400: 120 eigen workgroups, beyond the rows form's 64 -> split form
scenes = [synth.make_pnp_scene(rng, 600, 0.4) for _ in range(8)]
gs = [engine.PnPSolver(ctx, sc, 11 + i) for i, sc in enumerate(scenes)]
b = engine.SolverBatch(gs)
b.set_ransac_parameters(0.99, 10, 300, 4, 0.5, 5.991)  # minInliers 0.5 N: unreachable at 40 %
for call in range(2):
    try:
        b.iterate_raw(300)
        print("call", call, "returned OK")
        sys.exit(3)
    except RuntimeError as e:
        msg = str(e)
        print("call", call, "raised:", msg)
        if "hand-off" not in msg:
            sys.exit(4)
print("fault path ok")
"""


def test_split_hand_off_give_up_is_an_error():
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} missing: run make (build() builds it)")
    env = dict(os.environ, RSC_LIBRSC=LIB)
    r = subprocess.run([sys.executable, "-c", CHILD, os.path.join(ROOT, "orb-slam2-optimized_amd"),
                        os.path.join(ROOT, "tests")], env=env, capture_output=True, text=True, timeout=150)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert "fault path ok" in r.stdout
