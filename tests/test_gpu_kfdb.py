"""GPU parity of the KeyFrameDatabase candidate queries (KeyFrameDatabase.cpp:52-283) through the
C ABI (rsc_kfdb_*) against the oracle: candidate lists bit-exact (same slots, same order) and every
slot's persistent query state (mnLoopQuery/Words/Score, mnRelocQuery/Words/Score) identical after
each script — on the golden fixture, on random operation scripts, on the hand-built known answers
of test_cpu_kfdb.py, and on a bench-sized database; plus the ABI's error behaviour."""
import os

import numpy as np
import pytest

import kfdb_script as ks
import oracle_lib as ol
import test_cpu_kfdb as tk
from gpu_common import ctx
from rsc import engine, synth

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def gpu_db(cap, max_words=4096):
    return engine.KeyFrameDatabase(ctx(), cap, max_words)


def states(db, n):
    return [db.state(k) for k in range(n)]


def compare_script(ops, cap):
    g, o = gpu_db(cap), ol.OracleKFDB(cap)
    a, b = ks.run_script(g, ops), ks.run_script(o, ops)
    assert len(a) == len(b)
    for i, (x, y) in enumerate(zip(a, b)):
        assert list(x) == list(y), i
    assert states(g, cap) == states(o, cap)
    return a


def test_golden_fixture():
    z = np.load(os.path.join(ROOT, "tests", "golden", "kfdb_traces.npz"))
    for c in range(int(z["cases"])):
        ops = ks.load_script(f"c{c}", z)
        got = compare_script(ops, int(z[f"c{c}_cap"]))
        want = [z[f"c{c}_r{i}"] for i in range(int(z[f"c{c}_nr"]))]
        for g, w in zip(got, want):
            assert list(g) == list(w)


@pytest.mark.parametrize("seed", [4, 5, 6, 7])
def test_random_scripts(seed):
    compare_script(ks.make_script(seed, n_kfs=80, n_queries=40, words=400), 96)


class GpuTiny:
    """test_cpu_kfdb's hand-built cases on the device database."""

    def __new__(cls, cap):
        return gpu_db(cap)


@pytest.mark.parametrize("case", ["test_relocalization_known_answers", "test_relocalization_stale_score",
                                  "test_loop_known_answers", "test_empty_database_and_no_common_words",
                                  "test_erase_and_order"])
def test_known_answers(case, monkeypatch):
    # the CPU known-answer tests iterate over (PyKFDB, OracleKFDB); run them with the device class
    monkeypatch.setattr(tk.ol, "OracleKFDB", GpuTiny)
    monkeypatch.setattr(tk, "PyKFDB", GpuTiny)
    getattr(tk, case)()


def test_bench_sized_database():
    rng = np.random.default_rng(21)
    n = 2000
    sc = synth.make_kfdb_scene(rng, n, words_per_kf=600)
    g, o = gpu_db(n), ol.OracleKFDB(n)
    for k in range(n):
        for db in (g, o):
            db.add(k, *sc.bows[k])
            db.set_covisibility(k, sc.covis[k])
    for f in range(1, 25):
        ids, vals = synth.make_kfdb_query(rng, sc, rng.uniform(0, n - 1))
        if f % 3:
            a, b = g.detect_relocalization(f, ids, vals), o.detect_relocalization(f, ids, vals)
        else:
            near = int(rng.integers(0, n))
            conn = sc.covis[near]
            a, b = g.detect_loop(5000 + f, ids, vals, conn, 0.01), o.detect_loop(5000 + f, ids, vals, conn, 0.01)
        assert list(a) == list(b), f
    assert states(g, n) == states(o, n)


def test_abi_errors():
    db = gpu_db(8, max_words=16)
    ids, vals = np.array([1, 5, 9], np.uint32), np.array([0.2, 0.3, 0.5])
    db.add(0, ids, vals)
    with pytest.raises(RuntimeError):
        db.add(0, ids, vals)  # already present (the reference would list it twice)
    with pytest.raises(RuntimeError):
        db.add(1, ids[::-1], vals)  # not a BowVector (ids must ascend)
    with pytest.raises(RuntimeError):
        db.add(8, ids, vals)  # slot out of range
    with pytest.raises(RuntimeError):
        db.add(2, np.arange(17, dtype=np.uint32), np.ones(17))  # more words than max_words
    with pytest.raises(RuntimeError):
        db.add(3, np.array([1, 10 ** 6], np.uint32), np.ones(2))  # not a word of the vocabulary
    with pytest.raises(RuntimeError):
        db.detect_relocalization(2, np.array([10 ** 6], np.uint32), np.ones(1))
    with pytest.raises(RuntimeError):
        db.set_covisibility(0, np.arange(11, dtype=np.int32) % 8)  # more than 10
    with pytest.raises(RuntimeError):
        db.detect_loop(3, ids, vals, np.array([9], np.int32), 0.0)  # connected slot out of range
    assert list(db.detect_relocalization(1, ids, vals)) == [0]


def test_more_than_4096_slots_in_use():
    """The finish kernel's select loop beyond its 4 x 1024 register-held list entries (slots in
    use > 4096), with a sparse high slot added last (the sweeps cover every slot up to it)."""
    rng = np.random.default_rng(31)
    n = 4600
    sc = synth.make_kfdb_scene(rng, n, words_per_kf=60, step=12, n_frequent=8)
    g, o = gpu_db(n + 300, max_words=128), ol.OracleKFDB(n + 300)
    order = list(range(n))
    for k in order:
        for db in (g, o):
            db.add(k, *sc.bows[k])
            db.set_covisibility(k, sc.covis[k])
    for db in (g, o):
        db.add(n + 250, *sc.bows[n - 1])
    for f in range(1, 9):
        ids, vals = synth.make_kfdb_query(rng, sc, rng.uniform(n - 900, n - 1), words=60)
        if f % 2:
            a, b = g.detect_relocalization(f, ids, vals), o.detect_relocalization(f, ids, vals)
        else:
            conn = sc.covis[int(rng.integers(n - 900, n))]
            a, b = g.detect_loop(7000 + f, ids, vals, conn, 0.0), o.detect_loop(7000 + f, ids, vals, conn, 0.0)
        assert list(a) == list(b), f
    assert states(g, n + 300) == states(o, n + 300)


def test_more_than_1024_scored_slots():
    """A query every one of 1,500 KeyFrames shares all its words with (all pass minCommonWords):
    the finish kernel ranks and scores more slots than its LDS ranking holds (1,024)."""
    rng = np.random.default_rng(32)
    n = 1500
    words = np.sort(rng.choice(10 ** 6, 40, replace=False)).astype(np.uint32)
    g, o = gpu_db(n, max_words=64), ol.OracleKFDB(n)
    for k in range(n):
        vals = rng.uniform(0.1, 1.0, 40)
        vals = vals / vals.sum()
        extra = np.sort(rng.choice(10 ** 6, 10, replace=False)).astype(np.uint32)
        ids = np.unique(np.concatenate([words, extra]))
        v = np.concatenate([vals, rng.uniform(0.01, 0.05, len(ids) - 40)])
        for db in (g, o):
            db.add(k, ids, v[:len(ids)])
            db.set_covisibility(k, np.array([(k + j) % n for j in range(1, 6)], np.int32))
    qv = rng.uniform(0.1, 1.0, 40)
    for f in range(1, 4):
        a, b = g.detect_relocalization(f, words, qv), o.detect_relocalization(f, words, qv)
        assert list(a) == list(b) and len(a) > 0, f
        a, b = g.detect_loop(9000 + f, words, qv, np.array([1, 2], np.int32), 0.0), \
            o.detect_loop(9000 + f, words, qv, np.array([1, 2], np.int32), 0.0)
        assert list(a) == list(b), f
    assert states(g, n) == states(o, n)


def test_release_resets_the_slot():
    """rsc_kfdb_release (the facade's erase): the slot leaves the inverted file and its query
    state and covisibility row return to a fresh KeyFrame's, so another KeyFrame can take it."""
    rng = np.random.default_rng(33)
    sc = synth.make_kfdb_scene(rng, 40, words_per_kf=100, step=30)
    g, o = gpu_db(64, max_words=128), ol.OracleKFDB(64)
    for k in range(40):
        for db in (g, o):
            db.add(k, *sc.bows[k])
            db.set_covisibility(k, sc.covis[k])
    ids, vals = synth.make_kfdb_query(rng, sc, 20.0, words=100)
    assert list(g.detect_relocalization(3, ids, vals)) == list(o.detect_relocalization(3, ids, vals))
    touched = [k for k in range(40) if g.state(k)[0][1] == 3]
    assert touched
    k = touched[0]
    g.release(k)
    assert g.state(k) == ((0, 0), (0, 0), (0.0, 0.0))
    # the slot now hosts another KeyFrame: the database behaves as the oracle with that KeyFrame
    # in a fresh slot
    o.erase(k)
    g.add(k, *sc.bows[39])
    o.add(50, *sc.bows[39])
    a = g.detect_relocalization(4, ids, vals)
    b = o.detect_relocalization(4, ids, vals)
    assert [50 if x == k else x for x in a] == list(b)


def test_long_bow_vectors_and_queries():
    """BowVectors over 1,024 words (the count kernel's second batch of ids: counts and the L1 score
    carried across batches) and queries up to the 4,096-word bound (the largest LDS hash, 8,192
    entries, above the default 64 KB of dynamic LDS)."""
    rng = np.random.default_rng(34)
    n = 60
    sc = synth.make_kfdb_scene(rng, n, words_per_kf=1800, step=300, n_frequent=40)
    g, o = gpu_db(n + 4), ol.OracleKFDB(n + 4)
    for k in range(n):
        for db in (g, o):
            db.add(k, *sc.bows[k])
            db.set_covisibility(k, sc.covis[k])
    # one KeyFrame at the 4,096-word bound, sharing its words with the long queries below
    big = np.unique(np.concatenate([sc.bows[30][0], rng.choice(10 ** 6, 3000, replace=False).astype(np.uint32)]))[:4096]
    bv = rng.uniform(0.01, 1.0, len(big))
    for db in (g, o):
        db.add(n, big, bv / bv.sum())
    assert max(len(b[0]) for b in sc.bows) > 1024
    for f, words in enumerate((1200, 2500, 4096, 3000), 1):
        if words == 4096:
            ids, vals = big, rng.uniform(0.01, 1.0, len(big))
        else:
            ids, vals = synth.make_kfdb_query(rng, sc, rng.uniform(10, n - 10), words=words)
        assert len(ids) > 1024
        a, b = g.detect_relocalization(f, ids, vals), o.detect_relocalization(f, ids, vals)
        assert list(a) == list(b) and len(a) > 0, f
        conn = sc.covis[int(rng.integers(0, n))]
        a, b = g.detect_loop(100 + f, ids, vals, conn, 0.0), o.detect_loop(100 + f, ids, vals, conn, 0.0)
        assert list(a) == list(b), f
    assert states(g, n + 4) == states(o, n + 4)
