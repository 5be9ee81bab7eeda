"""GPU: the launch profiler behind bench.py's roofline (kt_profile_*).

Two sweep lanes complete out of the order the host recorded their events
in; the union of the launch intervals is formed over every launch at once,
so overlapping launches of pipelined calls count once and the union never
exceeds the wall time around them."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def kra():
    import krylov_robustness_amd as kra
    return kra


def test_lane_finishing_last_was_recorded_first(kra, monkeypatch):
    """Lane 0 is held busy before the call, so its sweep -- whose events the
    host recorded FIRST -- finishes after lane 1's.  The next submission folds
    the first call's events in (waiting on every event of the batch, not only
    the last recorded); collect and the profile reads return without error,
    the forms equal an unprofiled run, and the union is <= the wall time."""
    from krylov_robustness_amd import graphs
    monkeypatch.setenv("KT_SLQ_LANES", "2")
    A = graphs.chung_lu(100_000, 1_000_000, seed=2)
    ctx = kra.Context(0)
    D = kra.DeviceMatrix(A, ctx)
    ref = [kra.slq_quadforms(D, 32, 20, seed=s, block=16, ctx=ctx)[2] for s in (1, 2)]
    ctx.profile_reset()
    ctx.profile(True)
    t0 = time.perf_counter()
    ctx.debug_delay(0, 200_000)  # 200 ms on lane 0
    p1 = kra.slq_submit(D, 32, 20, seed=1, block=16, ctx=ctx)   # sweep 0 on lane 0, sweep 1 on lane 1
    p2 = kra.slq_submit(D, 32, 20, seed=2, block=16, ctx=ctx)   # folds p1's events in
    q1 = kra.slq_collect(p1)[2]
    q2 = kra.slq_collect(p2)[2]
    wall_ms = (time.perf_counter() - t0) * 1e3
    ctx.profile(False)
    launches, summed = ctx.profile_read(0)
    busy = ctx.profile_busy(0)
    assert np.array_equal(q1, ref[0]) and np.array_equal(q2, ref[1])
    assert launches == 2 * 2 * 19  # 2 calls x 2 sweeps x (m - 1) passes
    # (interval ends are fp32 ms after the anchor event: ~1e-5 ms each)
    assert 0 < busy <= summed + 1e-4 * launches
    assert busy <= wall_ms
    # lane 0 waited 200 ms: its passes ran after lane 1's, so the union is
    # about twice a lane's busy time, not its overlap -- and the delay
    # itself is no profiled launch
    assert busy < 200.0


def test_pipelined_union_counts_overlap_once(kra, monkeypatch):
    """Calls submitted one deep (the bench pipeline): with two lanes, the
    union over all calls is <= the wall time and <= the summed durations."""
    from krylov_robustness_amd import graphs
    monkeypatch.setenv("KT_SLQ_LANES", "2")
    A = graphs.chung_lu(200_000, 2_000_000, seed=3)
    ctx = kra.Context(0)
    D = kra.DeviceMatrix(A, ctx)
    kra.slq_quadforms(D, 64, 30, seed=0, block=16, ctx=ctx)  # warm
    ctx.profile_reset()
    ctx.profile(True)
    t0 = time.perf_counter()
    pend = None
    for s in range(6):
        nxt = kra.slq_submit(D, 64, 30, seed=s, block=16, ctx=ctx)
        if pend is not None:
            kra.slq_collect(pend)
        pend = nxt
    kra.slq_collect(pend)
    wall_ms = (time.perf_counter() - t0) * 1e3
    ctx.profile(False)
    launches, summed = ctx.profile_read(0)
    busy = ctx.profile_busy(0)
    assert launches == 6 * 4 * 29
    assert busy <= wall_ms and busy <= summed + 1e-4 * launches
    # every launch carries its sweep's width
    assert ctx.profile_read_width(0, 16) == (launches, summed)
    assert ctx.profile_read_width(0, 32) == (0, 0.0)
    assert ctx.profile_read_width(2, 16)[0] == 6 * 4  # one start pass per sweep


def test_destroyed_matrix_ticket_fails_cleanly(kra):
    """kt_matrix_destroy drains every lane before releasing the CSR; a ticket
    of the destroyed matrix then fails to collect instead of reading it, and
    a ticket collected with another matrix is refused without being consumed
    (collected with its own matrix afterwards, it gives the sweeps' forms)."""
    from krylov_robustness_amd import _lib, graphs
    A = graphs.chung_lu(50_000, 500_000, seed=1)
    ctx = kra.Context(0)
    D1 = kra.DeviceMatrix(A, ctx)
    D2 = kra.DeviceMatrix(A, ctx)
    p = kra.slq_submit(D1, 32, 20, seed=1, block=16, ctx=ctx)
    with pytest.raises(_lib.KrylovError, match="another matrix"):
        _lib.check(_lib.load().kt_slq_collect(D2.handle, p[1], None, None, None))
    q1 = kra.slq_collect(p)[2]  # the right matrix: still collectable
    assert np.array_equal(q1, kra.slq_quadforms(D1, 32, 20, seed=1, block=16, ctx=ctx)[2])
    p = kra.slq_submit(D1, 32, 20, seed=1, block=16, ctx=ctx)
    D1.close()
    with pytest.raises(_lib.KrylovError, match="destroyed"):
        _lib.check(_lib.load().kt_slq_collect(D2.handle, p[1], None, None, None))
    q = kra.slq_quadforms(D2, 32, 20, seed=1, block=16, ctx=ctx)[2]
    assert np.all(np.isfinite(q))
