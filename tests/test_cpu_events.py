"""The oracle's C event runners (config-5 CPU baseline: ora_reloc_events_batch / ora_loop_events_batch)
replay the reference order exactly like the Python round-robin driver of events_oracle.run_events, on
one thread and on several."""
import numpy as np

import events_oracle as eo
from rsc import events as rev


def test_c_event_runner_equals_python_replay():
    evs = rev.make_event_stream(seed=11, n_reloc=16, n_loop=6)
    ref = eo.run_events(evs)
    for nt in (1, 3):
        parts = [eo.PackedEvents([ev for ev in evs if ev.kind == k]).run(nt).records() for k in ("reloc", "loop")]
        got = np.concatenate(parts)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), nt
    assert (ref[:, 1] >= 0).any() and (ref[:, 1] < 0).any()
