"""GPU: speculative temporal blocking of the reference's tolerance mode.

With the tolerance on (model.rs:748-819: <= 50 sweeps, early exit once
max |dp'| < p_tol, up to 20 re-correction passes) a single-domain Jacobi
solve runs T = 8 sweeps per kind-5 launch and publishes every sweep's
residual; k_spec_check finds the first sweep below p_tol, stops the later
launches and, when that sweep is not the launch's last, re-runs the launch
from its untouched source buffer with exactly that many sweeps.  The result
must be the reference's bit for bit: every field, every scalar, and the sweep
count (jacobi_sweeps_total), step by step against the oracle, on grids and
tolerances that make solves stop at every possible stage of a launch.
"""
import os

import numpy as np
import pytest

from _util import assert_bitwise

pytestmark = pytest.mark.gpu

STATE = ("u", "v", "p", "u_star", "v_star", "p_prime", "rhs")


@pytest.fixture(autouse=True)
def _oracle_threads():
    import oracle
    try:
        n = max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:
        n = 4
    oracle.set_threads(n)
    yield
    oracle.set_threads(1)


def _compare(tag, m, o):
    st = m.get_state()
    for f in STATE:
        assert_bitwise(f"{tag}:{f}", st[f], o.field(f))
    s = o.scalars()
    assert st["simulation_step"] == s.step, tag
    assert st["jacobi_sweeps_total"] == s.jacobi_sweeps_total, (tag, st["jacobi_sweeps_total"],
                                                               s.jacobi_sweeps_total)
    for k, want in (("simulation_time", s.time), ("dt", s.dt), ("last_p_residual", s.p),
                    ("last_u_residual", s.u), ("last_v_residual", s.v)):
        assert np.float32(st[k]).view(np.uint32) == np.float32(want).view(np.uint32), (tag, k)
    return int(s.jacobi_sweeps_total)


@pytest.fixture(params=["resident", "launches"])
def solve_form(request, monkeypatch):
    """Every parity case runs twice: as the small-grid default, the whole
    solve in one resident launch (k_jacobi_resident), and as the per-launch
    speculative path (CFD_RESIDENT=0: k_jacobi_lds MODE 2 with the lagged
    check, the r6 default, + redo); test_gpu_spec_lag_slabs.py compares it
    with the k_spec_check launches (CFD_SPEC_LAG=0)."""
    monkeypatch.setenv("CFD_RESIDENT", "1" if request.param == "resident" else "0")
    return request.param


def _run(grid, params, okw, steps, tag):
    import cfdamd
    from oracle import OracleModel
    c = grid.obstacle
    m = cfdamd.Model(grid, params, device=0)
    assert m.kernel_config["temporal"] == 8, m.kernel_config
    if os.environ.get("CFD_RESIDENT") == "1":
        assert m.jacobi_kernel["name"].startswith("k_jacobi_resident<"), m.jacobi_kernel
        assert m.jacobi_kernel["kind"] == 6
    else:
        assert m.jacobi_kernel["name"].startswith("k_jacobi_lds<8,"), m.jacobi_kernel
    o = OracleModel(grid.nx, grid.ny, grid.lx, grid.ly,
                    cylinder=(c.center_x, c.center_y, c.radius) if c else None, **okw)
    sweeps = []
    try:
        prev = 0
        for k in range(steps):
            m.update()
            o.update()
            tot = _compare(f"{tag} step {k + 1}", m, o)
            sweeps.append(tot - prev)
            prev = tot
        # the form that ran, from the device: resident solves launched
        if os.environ.get("CFD_RESIDENT") == "1":
            assert m.resident_solves >= steps, (m.resident_solves, steps)
        elif os.environ.get("CFD_RESIDENT") == "0":
            assert m.resident_solves == 0
    finally:
        m.close()
    return sweeps


@pytest.mark.parametrize("p_tol", [1e-4, 1e-3, 3e-5])
def test_spec_cavity_parity_mode(p_tol, solve_form):
    """128^2 cavity, Re 100, the reference's control flow at three tolerances:
    solves end early at varying sweeps (the re-run with 1..7 sweeps)."""
    import cfdamd
    params = cfdamd.SimulationParams.cavity(100.0, 50, p_tol=p_tol)
    sweeps = _run(cfdamd.cavity_grid(128), params,
                  dict(bc_kind=1, viscosity=0.01, p_tol=p_tol), 40, f"cavity tol {p_tol}")
    # the early exit was taken: not every step ran whole 8-sweep launches
    assert any(s % 8 for s in sweeps), sweeps


def test_spec_channel_default_grid_cylinder(solve_form):
    """The reference's default grid (800 x 264 channel, cylinder, src/app.rs
    :33-53) with its default parameters (SimulationParams::default)."""
    import cfdamd
    _run(cfdamd.default_grid(), cfdamd.SimulationParams(), {}, 12, "default channel")


def test_spec_channel_second_order_parabolic(solve_form):
    import cfdamd
    grid = cfdamd.Grid(256, 96, 30.0, 10.0, cfdamd.Cylinder(7.5, 5.0, 1.5))
    params = cfdamd.SimulationParams(velocity_scheme=cfdamd.VelocityScheme.SecondOrder,
                                     inlet_profile=cfdamd.InletProfile.Parabolic)
    _run(grid, params, dict(scheme=1, inlet_profile=1), 20, "channel SO")


def test_spec_c2_parity_mode(solve_form):
    """C2 (1024^2 cavity, Re 400) in the reference's control flow."""
    import cfdamd
    params = cfdamd.SimulationParams.cavity(400.0, 50)
    _run(cfdamd.cavity_grid(1024), params, dict(bc_kind=1, viscosity=0.0025), 6, "C2 parity")


def test_spec_off_matches_spec_on(monkeypatch):
    """CFD_SPEC=0 (one launch per sweep with the per-sweep early exit) and the
    speculative path give the same bits and sweep counts."""
    import cfdamd
    grid = cfdamd.cavity_grid(256, 128)
    params = cfdamd.SimulationParams.cavity(400.0, 50, p_tol=2e-4)
    states = []
    for env in ("0", "1"):
        monkeypatch.setenv("CFD_SPEC", env)
        m = cfdamd.Model(grid, params, device=0)
        assert m.kernel_config["temporal"] == (1 if env == "0" else 8)
        m.update_n(15)
        states.append(m.get_state())
        m.close()
    for f in STATE:
        assert_bitwise(f"spec on/off:{f}", states[1][f], states[0][f])
    assert states[0]["jacobi_sweeps_total"] == states[1]["jacobi_sweeps_total"]


def test_fused_pass_head_matches_two_launches(monkeypatch):
    """The corrector-pass head fused into one launch (k_copy_star_div) and the
    two launches it replaces (CFD_COPY_DIV=0) give the same bits, with passes
    running (tolerance on, channel with a cylinder)."""
    import cfdamd
    grid = cfdamd.Grid(256, 96, 30.0, 10.0, cfdamd.Cylinder(7.5, 5.0, 1.5))
    params = cfdamd.SimulationParams(jacobi_iters=30, corrector_passes=6)
    states = []
    for env in ("0", "1"):
        monkeypatch.setenv("CFD_COPY_DIV", env)
        m = cfdamd.Model(grid, params, device=0)
        m.update_n(12)
        states.append(m.get_state())
        m.close()
    for f in STATE:
        assert_bitwise(f"pass head fused/unfused:{f}", states[1][f], states[0][f])


@pytest.mark.parametrize("grid_kind", ["channel", "cavity"])
def test_vector_corrector_matches_scalar(monkeypatch, grid_kind):
    """The corrector passes' 4-cells-per-thread kernel (k_corrector4) and the
    one-float-per-thread k_corrector (CFD_CORR_VEC=0) give the same bits with
    passes running: u faces incl. the Q9 tail, v faces, p += p'."""
    import cfdamd
    if grid_kind == "channel":
        grid = cfdamd.Grid(256, 96, 30.0, 10.0, cfdamd.Cylinder(7.5, 5.0, 1.5))
        params = cfdamd.SimulationParams(jacobi_iters=30, corrector_passes=6)
    else:
        grid = cfdamd.cavity_grid(192, 128)
        params = cfdamd.SimulationParams.cavity(400.0, 50, p_tol=2e-4)
    states = []
    for env in ("0", "1"):
        monkeypatch.setenv("CFD_CORR_VEC", env)
        m = cfdamd.Model(grid, params, device=0)
        m.update_n(10)
        states.append(m.get_state())
        m.close()
    for f in STATE:
        assert_bitwise(f"corrector vec/scalar {grid_kind}:{f}", states[1][f], states[0][f])


def test_resident_deadline_fault_is_loud_and_recoverable(monkeypatch):
    """A barrier wait past the deadline (forced: CFD_PERSIST_DEADLINE_US=0)
    aborts the resident solve.  r5: the model recovers by itself (checkpoint
    restored, the steps since re-run per launch), reports it once
    (CFD_ETIMEOUT), and with NO set_state by the caller every later step
    equals the oracle, sweep counts included."""
    import cfdamd
    from cfdamd._lib import CFD_ETIMEOUT, CfdError
    from oracle import OracleModel
    monkeypatch.setenv("CFD_RESIDENT", "1")
    grid = cfdamd.cavity_grid(256, 128)
    params = cfdamd.SimulationParams.cavity(400.0, 50, p_tol=2e-4)
    o = OracleModel(grid.nx, grid.ny, grid.lx, grid.ly, bc_kind=1, viscosity=1.0 / 400.0,
                    p_tol=2e-4)
    m = cfdamd.Model(grid, params, device=0)
    try:
        for k in range(3):
            m.update()
            o.update()
            _compare(f"resident before fault {k}", m, o)
        monkeypatch.setenv("CFD_PERSIST_DEADLINE_US", "0")
        monkeypatch.setenv("CFD_PERSIST_LATE", "3")   # workgroups 1, 4, ... arrive 2 ms late
        steps = 0
        with pytest.raises(CfdError) as ei:
            for _ in range(5):   # the first barrier wait faults
                m.update()
                steps += 1
                m.synchronize()
        assert ei.value.code == CFD_ETIMEOUT, ei.value
        assert "resident" in str(ei.value) and "recovered" in str(ei.value), ei.value
        assert m.recoveries == 1
        monkeypatch.delenv("CFD_PERSIST_DEADLINE_US")
        monkeypatch.delenv("CFD_PERSIST_LATE")
        for k in range(steps):
            o.update()
        _compare("resident recovered", m, o)
        assert m.jacobi_kernel["kind"] == 5   # per launch after the fault
        for k in range(3):
            m.update()
            o.update()
            _compare(f"after resident fault {k}", m, o)
    finally:
        m.close()


def test_resident_late_workgroups_bitwise(monkeypatch):
    """Workgroups that reach the first barrier 2 ms late (CFD_PERSIST_LATE=3)
    hold the others at the barrier and change no bit."""
    monkeypatch.setenv("CFD_PERSIST_LATE", "3")
    import cfdamd
    monkeypatch.setenv("CFD_RESIDENT", "1")
    params = cfdamd.SimulationParams.cavity(400.0, 50)
    _run(cfdamd.cavity_grid(1024), params, dict(bc_kind=1, viscosity=0.0025), 3, "C2 late")


def test_resident_two_models_interleaved(monkeypatch):
    """Two models' resident solves enqueued back to back on their own streams
    (ordered by the device's launch gate) give each model's own sequential
    bits."""
    import cfdamd
    monkeypatch.setenv("CFD_RESIDENT", "1")
    grids = [cfdamd.cavity_grid(256, 128), cfdamd.default_grid()]
    params = [cfdamd.SimulationParams.cavity(400.0, 50, p_tol=2e-4), cfdamd.SimulationParams()]
    alone = []
    for g, p in zip(grids, params):
        m = cfdamd.Model(g, p, device=0)
        m.update_n(8)
        alone.append(m.get_state())
        m.close()
    ms = [cfdamd.Model(g, p, device=0) for g, p in zip(grids, params)]
    try:
        for _ in range(8):
            for m in ms:
                m.update()   # no synchronisation between the models
        for m, ref in zip(ms, alone):
            st = m.get_state()
            for f in STATE:
                assert_bitwise(f"interleaved:{f}", st[f], ref[f])
            assert st["jacobi_sweeps_total"] == ref["jacobi_sweeps_total"]
    finally:
        for m in ms:
            m.close()


def test_resident_guarded_fma_division_tiny_values(monkeypatch):
    """On the reference's default grid no divisor has an exact reciprocal or
    FMA-corrected form for all inputs, but form 3 -- FMA-corrected for
    |x| >= 2^-96, IEEE `/` below, proven on the device for all 2^32 inputs --
    holds, and the resident solve can use it (CFD_RESIDENT_DIV=3: measured
    slower than IEEE division, so opt-in).  p' scaled to 1e-33 in half the
    domain (sums far below the threshold: the IEEE branch, in waves mixed with
    the FMA branch) and a developed state elsewhere: three steps bitwise
    against the oracle, sweep counts included."""
    import cfdamd
    from oracle import OracleModel
    monkeypatch.setenv("CFD_RESIDENT", "1")
    monkeypatch.setenv("CFD_RESIDENT_DIV", "3")   # opt-in (slower than IEEE here)
    grid = cfdamd.default_grid()
    m = cfdamd.Model(grid, cfdamd.SimulationParams(), device=0)
    try:
        assert m.jacobi_kernel["name"] == "k_jacobi_resident<3>", m.jacobi_kernel
        m.update_n(6)
        st = m.get_state()
        pp = st["p_prime"].copy().reshape(grid.ny, grid.nx)
        pp[:, : grid.nx // 2] *= np.float32(1e-33)
        st["p_prime"] = pp.ravel()
        m.set_state(**st)
        c = grid.obstacle
        o = OracleModel(grid.nx, grid.ny, grid.lx, grid.ly, cylinder=(c.center_x, c.center_y, c.radius))
        for k in STATE:
            o.field(k)[:] = st[k]
        sc = o.scalars()
        sc.step, sc.time, sc.dt = st["simulation_step"], st["simulation_time"], st["dt"]
        sc.jacobi_sweeps_total = st["jacobi_sweeps_total"]
        o.set_scalars(sc)
        for k in range(3):
            m.update()
            o.update()
            _compare(f"tiny p' step {k + 1}", m, o)
        assert m.resident_solves >= 3
    finally:
        m.close()
