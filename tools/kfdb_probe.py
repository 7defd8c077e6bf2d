#!/usr/bin/env python3
"""Diagnostic: timeline of the KeyFrameDatabase count kernel (bench.py's kfdb section: 2000 KeyFrames
x ~612 words, relocalization queries) from rsc_diag_kfdb_stamps — needs a library built with
RSC_KFDB_STAMPS=1 (HIPFLAGS with -DRSC_KFDB_STAMPS=1)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orb-slam2-optimized_amd"), ROOT]
import numpy as np  # noqa: E402
import bench  # noqa: E402
from rsc import engine  # noqa: E402

ctx = engine.Context(0)
sc, queries = bench.kfdb_scene()
n = len(sc.bows)
db = engine.KeyFrameDatabase(ctx, bench.KFDB_CAPACITY)
for k in range(n):
    db.add(k, *sc.bows[k])
kfs = np.arange(n, dtype=np.int32)
cnt = np.array([len(c) for c in sc.covis], np.int32)
tab = np.zeros((n, 10), np.int32)
for k, c in enumerate(sc.covis):
    tab[k, :len(c)] = c
db.set_covisibility_table(kfs, cnt, tab)
st = np.zeros(4096 * 4, np.uint64)
rows = []
for i, (ids, vals) in enumerate(queries[:16]):
    db.detect_relocalization(100 + i, ids, vals)
    engine._check(engine.load_library().rsc_diag_kfdb_stamps(ctx.h, st, st.size), "kfdb stamps")
    s = st.reshape(4096, 4)[:n].astype(np.int64)
    t0 = s[:, 0].min()
    rows.append([(s[:, 0] - t0).max(), (s[:, 1] - s[:, 0]).mean(), (s[:, 2] - s[:, 1]).mean(),
                 (s[:, 3] - s[:, 2]).mean(), (s[:, 3] - s[:, 2]).max(), (s[:, 3] - t0).max()])
r = np.array(rows, np.float64).mean(0) / 100.0
print(f"count kernel (us, mean of 16 queries): last wave start {r[0]:.2f}; per wave: staging {r[1]:.2f}, "
      f"count {r[2]:.2f}, state+score {r[3]:.2f} (max {r[4]:.2f}); first entry -> last exit {r[5]:.2f}")
