"""The per-dispatch device busy span (fi_debug_dispatch_span_ms) beside the
HIP-event time of the same dispatch: the span covers only the waves that ran
a trial, so it is never longer than the event pair around the launch, and a
dispatch with no trial to run reports 0."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REGS_PC = ((1 << 32) - 2) | (1 << 32)


@pytest.mark.parametrize("name", ["crc32", "qsort"])
def test_dispatch_spans(engine_factory, name):
    e = engine_factory(name)
    e.set_campaign(0x5EED0002, REGS_PC, 1)
    e.set_protect(0)
    e.run_trials(0, 20000, want_outcomes=False)
    e.kernel_timer_reset()
    e.run_trials(0, 20000, want_outcomes=False)
    ev, sp, kinds = e.debug_dispatch_ms(), e.debug_dispatch_span_ms(), e.debug_dispatch_kinds()
    assert len(ev) == len(sp) == len(kinds) >= 2
    for t, s, k in zip(ev, sp, kinds):
        assert 0.0 <= s <= t + 0.05, (k, t, s)   # (s_memrealtime: 10 ns ticks; event resolution)
    # the 64-lane epoch runs every trial: its span is most of its event time
    t0 = [(t, s) for t, s, k in zip(ev, sp, kinds) if k == 0]
    assert t0 and all(s > 0.5 * t for t, s in t0)
