"""The reference's shared rand() stream (Q3) on the device, bit-exact against oracle replays that call
libc's real rand() in the reference's order.

DUtils::Random::RandomInt (Random.cpp:47-50) draws from glibc's process-global rand(), unseeded in the
reference (= srand(1)).  Tracking::Relocalization (Tracking.cpp:1239-1262) and
LoopClosing::ComputeSim3 (LoopClosing.cpp:271-286) call iterate(5) on their candidates round by round,
so every call continues the stream where the previous one stopped.  rsc_stream is that stream:

* Stream.peek / skip against glibc (restated and libc), including jumps across the jump table's reach;
* solvers bound to one stream, called one at a time in the round-robin order (the facade's path);
* *_iterate_many over bound solvers (calls in list order);
* whole events through rsc_reloc_events_shared / rsc_loop_events_shared (all events' rounds in the
  same launches, each call positioned where the previous call of its event ends): winner records,
  poses and the final stream position equal the oracle's libc replay.
"""
import numpy as np
import pytest

from gpu_common import bits, ctx
import events_oracle as eo
import oracle_lib as ol
from rsc import events as rev
from rsc import synth

pytestmark = pytest.mark.gpu


def test_stream_peek_and_skip_match_glibc():
    from rsc import engine
    for seed in (1, 2, 12345):
        st = engine.Stream(ctx(), seed)
        ref = ol.glibc_rand(seed, 1000)
        assert np.array_equal(st.peek(1000), ref)
        ol.libc_srand(seed)
        assert [ol.libc_rand() for _ in range(50)] == ref[:50].tolist()
    st = engine.Stream(ctx(), 1)
    total = 0
    ref = ol.glibc_rand(1, 1_100_000)
    for k in (1, 309, 16383, 16384, 16704, 33000, 1_000_000):
        st.skip(k)
        total += k
        assert st.position == total
        n = min(64, len(ref) - total)
        assert np.array_equal(st.peek(n), ref[total:total + n]), k


def _rr_pnp(n_rounds, solvers, oracles, bound_many=False):
    """Round-robin iterate(5) over the live candidates (Tracking.cpp:1241-1262 without the gate)."""
    from rsc import engine
    live = list(range(len(solvers)))
    for rnd in range(n_rounds):
        if not live:
            break
        if bound_many:
            outs = engine.pnp_iterate_many([solvers[i] for i in live], 5)
        else:
            outs = [solvers[i].iterate(5) for i in live]
        nxt = []
        for i, g in zip(live, outs):
            o = oracles[i].iterate(5)
            assert (g["ok"], g["no_more"], g["n_inliers"], g["iterations"]) == \
                (o["ok"], o["no_more"], o["n_inliers"], o["iterations"]), f"round {rnd} cand {i}"
            if o["ok"]:
                assert np.array_equal(bits(g["T"]), bits(o["T"])) and np.array_equal(g["inliers"], o["inliers"])
            if not o["no_more"]:
                nxt.append(i)
        live = nxt


@pytest.mark.parametrize("bound_many", [False, True])
def test_bound_pnp_solvers_round_robin(bound_many):
    """Candidates bound to ONE stream, called in the reference's order (one call at a time, or a
    round as one rsc_pnp_iterate_many over bound solvers): every call equals the oracle's call on
    libc's rand() after srand(1), and the stream ends where libc's does."""
    from rsc import engine
    rng = np.random.default_rng(41)
    scenes = [synth.make_pnp_scene(rng, int(rng.integers(200, 900)), r) for r in (0.3, 0.62, 0.2, 0.7, 0.5)]
    st = engine.Stream(ctx(), 1)
    gs, os_ = [], []
    for sc in scenes:
        g = engine.PnPSolver(ctx(), sc, 99)
        g.set_ransac_parameters(0.99, 10, 60, 4, 0.5, 5.991)
        g.bind_stream(st)
        o = ol.OraclePnP(sc, 99)
        o.set_ransac_parameters(0.99, 10, 60, 4, 0.5, 5.991)
        o.use_libc_rand()
        gs.append(g)
        os_.append(o)
    ol.libc_srand(1)
    _rr_pnp(6, gs, os_, bound_many)
    assert st.peek(1)[0] == ol.libc_rand()


def test_bound_sim3_and_mlpnp_solvers():
    from rsc import engine
    rng = np.random.default_rng(42)
    pairs = [synth.make_sim3_pair(rng, 500, k) for k in (30, 150, 60)]
    scenes = [synth.make_pnp_scene(rng, 400, r) for r in (0.4, 0.7)]
    st = engine.Stream(ctx(), 1)
    gs = [engine.Sim3Solver(ctx(), p, 5) for p in pairs] + [engine.MLPnPSolver(ctx(), sc, 5) for sc in scenes]
    os_ = [ol.OracleSim3(p, 5) for p in pairs] + [ol.OracleMLPnP(sc, 5) for sc in scenes]
    for g, o in zip(gs, os_):
        args = (0.99, 20, 300) if isinstance(g, engine.Sim3Solver) else (0.99, 10, 300, 6, 0.5, 5.991)
        g.set_ransac_parameters(*args)
        o.set_ransac_parameters(*args)
        g.bind_stream(st)
        o.use_libc_rand()
    ol.libc_srand(1)
    for rnd in range(5):
        for i, (g, o) in enumerate(zip(gs, os_)):
            a, b = g.iterate(5), o.iterate(5)
            assert (a["ok"], a["no_more"], a["n_inliers"], a["iterations"]) == \
                (b["ok"], b["no_more"], b["n_inliers"], b["iterations"]), f"round {rnd} solver {i}"
            if "R" in a:
                assert np.array_equal(bits(a["R"]), bits(b["R"])) and np.array_equal(a["inliers"], b["inliers"])
            elif b["ok"]:
                assert np.array_equal(bits(a["T"]), bits(b["T"])) and np.array_equal(a["inliers"], b["inliers"])
    assert st.peek(1)[0] == ol.libc_rand()


@pytest.mark.parametrize("kind", ["reloc", "loop"])
def test_events_on_the_shared_stream(kind):
    """Whole events on the reference's stream: every event's calls draw from its own srand(1) stream
    in round-robin order, all events batched in the same launches; winner record, winner pose and the
    stream position after the event equal the oracle's libc replay."""
    from rsc import engine
    evs = [ev for ev in rev.make_event_stream(seed=29, n_reloc=12, n_loop=10) if ev.kind == kind]
    ins = [rev.event_inputs(ev) for ev in evs]
    cls = engine.PnPSolver if kind == "reloc" else engine.Sim3Solver
    eb = engine.EventBatch([[cls(ctx(), x, 1) for x in xs] for xs in ins])
    eb.batch.set_ransac_parameters(*(rev.RELOC_PARAMS if kind == "reloc" else rev.LOOP_PARAMS))
    streams = [engine.Stream(ctx(), 1) for _ in evs]
    eb.run(streams=streams)
    poses = eb.winner_poses()
    n_win = 0
    for e, (ev, xs) in enumerate(zip(evs, ins)):
        rec, pose, used = eo.run_event_shared(ev, 1, xs)
        got = eb.per_event[e]
        assert (int(got["winner"]), int(got["round"]), int(got["hypothesis"]), int(got["n_inliers"])) == \
            (rec["winner"], rec["round"], rec["hypothesis"], rec["n_inliers"]), f"event {ev.eid}"
        assert np.array_equal(poses[e].view(np.uint32), pose.view(np.uint32)), f"event {ev.eid}"
        assert streams[e].position == used, f"event {ev.eid}"
        assert streams[e].peek(1)[0] == ol.libc_rand(), f"event {ev.eid}"
        n_win += rec["winner"] >= 0
    assert n_win >= 2


@pytest.mark.parametrize("kind", ["pnp", "sim3", "mlpnp"])
def test_unbind_resumes_the_own_stream(kind):
    """include/rsc.h rsc_*_bind_stream: unbinding (NULL) returns a solver to its own srand(seed) stream
    where it stopped: own calls, bound calls on the shared stream, own calls again, a reset
    while bound (reseeds the parked stream), unbind — every call equals the oracle that switches between
    its own stream and libc's rand() at the same points."""
    from rsc import engine
    rng = np.random.default_rng(43)
    if kind == "sim3":
        x = synth.make_sim3_pair(rng, 500, 60)
        g, o = engine.Sim3Solver(ctx(), x, 77), ol.OracleSim3(x, 77)
        args = (0.99, 20, 300)
    else:
        x = synth.make_pnp_scene(rng, 500, 0.3)
        cls, ocls = (engine.PnPSolver, ol.OraclePnP) if kind == "pnp" else (engine.MLPnPSolver, ol.OracleMLPnP)
        g, o = cls(ctx(), x, 77), ocls(x, 77)
        args = (0.99, 10, 300, 4 if kind == "pnp" else 6, 0.5, 5.991)
    for s in (g, o):
        s.set_ransac_parameters(*args)
    st = engine.Stream(ctx(), 1)
    ol.libc_srand(1)

    def step(tag):
        a, b = g.iterate(5), o.iterate(5)
        assert (a["ok"], a["no_more"], a["n_inliers"], a["iterations"]) == \
            (b["ok"], b["no_more"], b["n_inliers"], b["iterations"]), tag
        key = "R" if kind == "sim3" else "T"
        if b["ok"] or kind == "sim3":
            assert np.array_equal(bits(a[key]), bits(b[key])), tag

    step("own 1")
    g.bind_stream(st)
    o.use_libc_rand(True)
    step("bound 1")
    step("bound 2")
    g.bind_stream(None)
    o.use_libc_rand(False)
    step("own 2")
    step("own 3")
    assert st.peek(1)[0] == ol.libc_rand()  # the unbound calls did not touch the shared stream
    # reset while bound reseeds the parked own stream
    g.bind_stream(st)
    g.reset(91)
    o2 = type(o)(x, 91)
    o2.set_ransac_parameters(*args)
    o = o2
    for s in (g, o):
        s.set_ransac_parameters(*args)
    g.bind_stream(None)
    step("own after reset")
