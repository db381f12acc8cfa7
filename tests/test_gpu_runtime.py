"""The native Model::run runtime (csrc/cfd_runtime.cpp, cfd_run_* in
include/cfd.h; reference model.rs:57-117, 1282-1332) on the GPU: the worker
steps while unpaused, publishes one residual record per step, snapshots on
request (at most one per command drain, carrying the paused flag), applies
parameters between steps, and hands the model back on stop — with the state
bit-identical to the oracle after the same number of steps."""
import time

import numpy as np
import pytest

from _util import assert_bitwise

pytestmark = pytest.mark.gpu


def _wait(pred, limit=30.0):
    t0 = time.time()
    while not pred():
        if time.time() - t0 > limit:
            raise AssertionError("timed out")
        time.sleep(0.005)


def test_runtime_steps_pauses_snapshots_and_stops():
    import cfdamd
    from oracle import OracleModel
    g = cfdamd.Grid(64, 48, 3.0, 2.0, cfdamd.Cylinder(1.0, 1.0, 0.3))
    m = cfdamd.Model(g, cfdamd.SimulationParams())
    h = m.run()
    log = []
    _wait(lambda: log.extend(h.get_new_log_messages()) or len(log) >= 5)
    h.pause()
    h.request_snapshot()
    snap = []
    _wait(lambda: snap.append(h.get_last_available_snapshot()) or snap[-1] is not None)
    s = snap[-1]
    assert s.paused and s.u.size == 65 * 48 and s.v.size == 64 * 49 and s.p.size == 64 * 48
    assert h.get_last_available_snapshot() is None          # taken once
    n_paused = h.steps
    time.sleep(0.1)
    assert h.steps == n_paused                               # no stepping while paused
    log.extend(h.get_new_log_messages())
    steps = [r.simulation_step for r in log]
    assert steps == list(range(1, len(steps) + 1))           # one record per step, in order
    assert len(steps) == n_paused
    # parameters take effect between steps (model.rs:1297-1299)
    h.set_params(cfdamd.SimulationParams(dt=0.004, viscosity=1e-3))
    h.resume()
    _wait(lambda: h.steps >= n_paused + 3)
    h.stop()
    st = m.get_state()                                       # the model is ours again
    k = st["simulation_step"]
    assert k >= n_paused + 3
    o = OracleModel(64, 48, 3.0, 2.0, cylinder=(1.0, 1.0, 0.3))
    for _ in range(n_paused):
        o.update()
    o.set_params(dt=0.004, viscosity=1e-3)
    for _ in range(k - n_paused):
        o.update()
    for f in ("u", "v", "p", "p_prime"):
        assert_bitwise(f, st[f], o.field(f))
    # snapshot fields equal get_state at the pause point
    o2 = OracleModel(64, 48, 3.0, 2.0, cylinder=(1.0, 1.0, 0.3))
    for _ in range(n_paused):
        o2.update()
    assert_bitwise("snapshot u", s.u, o2.field("u"))
    assert_bitwise("snapshot p", s.p, o2.field("p"))


def test_runtime_rejects_bad_params_synchronously():
    """The reference's set_parameters cannot fail (model.rs:1250-1257), so
    parameters the model would refuse are rejected by cfd_run_set_params
    itself, before the worker sees them: the caller gets the error, the
    model's parameters are unchanged and the worker keeps stepping.  (A
    worker that fails mid-run, e.g. on a non-finite field, is reported by
    cfd_run_status: tests/test_gpu_long.py::test_nonfinite_velocity_is_reported.)"""
    import cfdamd
    m = cfdamd.Model(cfdamd.Grid(32, 16, 1.0, 1.0), cfdamd.SimulationParams())
    h = m.run()
    before = m.params
    bad = cfdamd.SimulationParams(jacobi_iters=10 ** 6)
    with pytest.raises(cfdamd.CfdError) as e:
        h.set_params(bad)
    assert e.value.code == -1 and "jacobi_iters" in str(e.value)
    assert m.params is before
    n = h.steps
    _wait(lambda: h.steps > n + 2)
    assert h.status()[0] == 0
    with pytest.raises(cfdamd.CfdError):   # the worker owns the handle
        m.update()
    h.stop()
    m.update()                               # handed back after stop
    m.close()
