"""KeyFrameDatabase operation scripts (test infrastructure): one random sequence of add / erase /
clear / covisibility updates and DetectRelocalizationCandidates / DetectLoopCandidates queries,
replayed identically on the oracle (tests/oracle_lib.OracleKFDB), the pure-Python restatement
(test_cpu_kfdb.PyKFDB) and the device database (rsc.engine.KeyFrameDatabase).  The per-KeyFrame
query state persists across the sequence, so the scripts exercise the reference's cross-query
behaviour (KeyFrameDatabase.cpp:181-196, :245-252)."""
import numpy as np

from rsc import synth

OPS = {"add": 0, "erase": 1, "clear": 2, "covis": 3, "reloc": 4, "loop": 5}


def make_script(seed: int, n_kfs: int = 60, n_queries: int = 40, words: int = 300):
    rng = np.random.default_rng(seed)
    sc = synth.make_kfdb_scene(rng, n_kfs, words_per_kf=words, step=words // 4)
    ops = []
    for k in range(n_kfs):
        ops.append(("add", k, *sc.bows[k]))
    for k in range(n_kfs):
        ops.append(("covis", k, sc.covis[k]))
    fid, kid = 1, 1000
    for q in range(n_queries):
        r = rng.random()
        pos = rng.uniform(0, n_kfs - 1)
        if r < 0.08:  # erase and re-add later in the list order (a new position in every list)
            k = int(rng.integers(0, n_kfs))
            ops.append(("erase", k))
            if rng.random() < 0.7:
                ops.append(("add", k, *sc.bows[k]))
        if r < 0.5:
            same = q > 0 and rng.random() < 0.1  # the same Frame id twice
            ids, vals = synth.make_kfdb_query(rng, sc, pos, words)
            ops.append(("reloc", fid if not same else fid - 1, ids, vals))
            fid += 0 if same else 1
        else:
            ids, vals = synth.make_kfdb_query(rng, sc, pos, words)
            near = int(round(pos))
            conn = np.array(sorted({near, *sc.covis[near][:int(rng.integers(0, 6))]}), np.int32)
            ms = float(rng.choice([0.0, 0.01, 0.03, 0.2]))
            ops.append(("loop", kid, ids, vals, conn, ms))
            kid += 1
    # a Frame with id 0 (every KeyFrame's initial mnRelocQuery) and a cleared database
    ids, vals = synth.make_kfdb_query(rng, sc, n_kfs / 2, words)
    ops.append(("reloc", 0, ids, vals))
    ops.append(("clear",))
    for k in range(0, n_kfs, 3):
        ops.append(("add", k, *sc.bows[k]))
    for _ in range(4):
        ids, vals = synth.make_kfdb_query(rng, sc, rng.uniform(0, n_kfs - 1), words)
        ops.append(("reloc", fid, ids, vals))
        fid += 1
    return ops


def run_script(db, ops):
    """Apply ops to db; returns the list of candidate arrays of the queries, in order."""
    out = []
    for op in ops:
        kind = op[0]
        if kind == "add":
            db.add(op[1], op[2], op[3])
        elif kind == "erase":
            db.erase(op[1])
        elif kind == "clear":
            db.clear()
        elif kind == "covis":
            db.set_covisibility(op[1], op[2])
        elif kind == "reloc":
            out.append(np.asarray(db.detect_relocalization(op[1], op[2], op[3]), np.int32))
        elif kind == "loop":
            out.append(np.asarray(db.detect_loop(op[1], op[2], op[3], op[4], op[5]), np.int32))
    return out


def save_script(prefix: str, ops, store: dict):
    store[f"{prefix}_n"] = np.int32(len(ops))
    for i, op in enumerate(ops):
        p = f"{prefix}_{i}"
        store[p + "_k"] = np.int32(OPS[op[0]])
        kind = op[0]
        if kind == "add":
            store[p + "_a"] = np.int64(op[1]); store[p + "_ids"] = op[2]; store[p + "_vals"] = op[3]
        elif kind == "erase":
            store[p + "_a"] = np.int64(op[1])
        elif kind == "covis":
            store[p + "_a"] = np.int64(op[1]); store[p + "_best"] = op[2]
        elif kind == "reloc":
            store[p + "_a"] = np.int64(op[1]); store[p + "_ids"] = op[2]; store[p + "_vals"] = op[3]
        elif kind == "loop":
            store[p + "_a"] = np.int64(op[1]); store[p + "_ids"] = op[2]; store[p + "_vals"] = op[3]
            store[p + "_conn"] = op[4]; store[p + "_ms"] = np.float32(op[5])


def load_script(prefix: str, z):
    names = {v: k for k, v in OPS.items()}
    ops = []
    for i in range(int(z[f"{prefix}_n"])):
        p = f"{prefix}_{i}"
        kind = names[int(z[p + "_k"])]
        if kind == "add":
            ops.append((kind, int(z[p + "_a"]), z[p + "_ids"], z[p + "_vals"]))
        elif kind == "erase":
            ops.append((kind, int(z[p + "_a"])))
        elif kind == "clear":
            ops.append((kind,))
        elif kind == "covis":
            ops.append((kind, int(z[p + "_a"]), z[p + "_best"]))
        elif kind == "reloc":
            ops.append((kind, int(z[p + "_a"]), z[p + "_ids"], z[p + "_vals"]))
        else:
            ops.append((kind, int(z[p + "_a"]), z[p + "_ids"], z[p + "_vals"], z[p + "_conn"], float(z[p + "_ms"])))
    return ops
