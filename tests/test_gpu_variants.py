"""GPU parity of the product's alternative kernel forms forced on EVERY launch — each must give the
default path's bits, so each is checked against the oracle exactly like the default path.

* the eigen stage in the Refine's rows form (`rsc_context_set_eig_rows`, rsc_quad.h
  pnp_eig_rows_body: a 12-lane group per hypothesis, Q rows in VGPRs) — the default for small
  launches since round 5 (<= 64 workgroups), forced here onto large ones too: every hypothesis of
  exhaustive batches (min sets 4..6, a planar scene for the NaN path), and a relocalization event
  stream;
* the split form (`rsc_context_set_eig_split`, pnp_eig_split_body: chase wave + row wave per unit,
  the default beyond the rows form's range) and the lane-pair form, each forced onto every launch,
  small ones included (set_eig_rows(0)): the same batches and event stream.
First run on hardware in round 5 (profiles/r05/gpu_tests_variants_r5b.txt)."""
import numpy as np
import pytest

import oracle_lib as ol
from rsc import synth

pytestmark = pytest.mark.gpu


def _nan_equal(a, b):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(a.view(np.uint32)[~na], b.view(np.uint32)[~nb])


def _rows_ctx(rows=True, split=True):
    from rsc import engine
    c = engine.Context(0)
    c.set_eig_rows(1 << 20 if rows else 0)  # every launch in the rows form / in the split or pair form
    c.set_eig_split(split)
    return c


@pytest.mark.parametrize("form", ["rows", "split", "pairs"])
@pytest.mark.parametrize("ms", [4, 5, 6])
def test_eig_rows_every_hypothesis(ms, form):
    from rsc import engine
    c = _rows_ctx(form == "rows", form == "split")
    rng = np.random.default_rng(900 + ms)
    scenes = [synth.make_pnp_scene(rng, 700, 0.4), synth.make_pnp_scene(rng, 1900, 0.35),
              synth.make_planar_pnp_scene(rng, 500, 0.4, "floor"), synth.make_pnp_scene(rng, 230, 0.45)]
    params = (0.99, 10, 300, ms, 0.5, 5.991)  # at most 45 % inliers: minInliers N/2 unreachable
    seeds = [31 + i for i in range(len(scenes))]
    gs = [engine.PnPSolver(c, sc, s) for sc, s in zip(scenes, seeds)]
    b = engine.SolverBatch(gs)
    b.set_ransac_parameters(*params)
    b.iterate(300)
    for i, (sc, s) in enumerate(zip(scenes, seeds)):
        o = ol.OraclePnP(sc, s)
        o.set_ransac_parameters(*params)
        o.enable_trace()
        ro = o.iterate(300)
        assert not ro["ok"] and ro["iterations"] == 300
        ints, fl = o.trace()
        cnt, pos = gs[i].last_hypotheses(400)
        smp = gs[i].last_samples(400)
        assert len(cnt) == len(ints) == 300
        assert np.array_equal(smp[:, :ms], ints[:, :ms]), f"ms={ms} cand {i} samples"
        assert np.array_equal(cnt, ints[:, 8]), f"ms={ms} cand {i} counts"
        assert _nan_equal(pos, fl), f"ms={ms} cand {i} poses"
    c.close()


@pytest.mark.parametrize("form", ["rows", "split", "pairs"])
def test_eig_rows_reloc_events(form):
    from rsc import engine, events as rev
    import events_oracle as eo
    c = _rows_ctx(form == "rows", form == "split")
    evs = [ev for ev in rev.make_event_stream(seed=23, n_reloc=8, n_loop=0) if ev.kind == "reloc"]
    eb = engine.EventBatch([[engine.PnPSolver(c, x, s) for x, s in zip(rev.event_inputs(ev), ev.seeds)] for ev in evs])
    eb.batch.set_ransac_parameters(*rev.RELOC_PARAMS)
    eb.run()
    got = rev.pack_events([ev.eid for ev in evs], eb.per_event, eb.winner_poses())
    assert np.array_equal(got.view(np.uint32), eo.run_events(evs).view(np.uint32))
    c.close()
