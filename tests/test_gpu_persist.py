"""GPU: the persistent fixed-count solve (k_jacobi_persist, CFD_PERSIST=1).

One launch runs all but the last 8-sweep block of a solve; workgroups hand
rows to their neighbours through per-workgroup flags inside the launch
(write-through p' stores, L1-bypassing loads).  Every field must equal the
per-launch form bit for bit -- across grids whose tiles split unevenly, with
the obstacle masks, the second-order scheme, corrector passes, the IEEE
division path, and a developed 4096^2 state -- and the oracle.
"""
import numpy as np
import pytest

from _util import assert_bitwise

pytestmark = pytest.mark.gpu

STATE = ("u", "v", "p", "u_star", "v_star", "p_prime", "rhs")


def _states(monkeypatch, grid, params, steps, develop=0):
    import cfdamd
    out = []
    for env in ("0", "1"):
        monkeypatch.setenv("CFD_PERSIST", env)
        m = cfdamd.Model(grid, params, device=0)
        try:
            if develop:
                m.update_n(develop)
            m.update_n(steps)
            out.append(m.get_state())
        finally:
            m.close()
    return out


@pytest.mark.parametrize("nx,ny,iters", [(256, 200, 50), (1024, 1024, 100), (640, 1000, 200), (1024, 1024, 1200),
                                          (2048, 384, 40)])
def test_persist_matches_launches_cavity(monkeypatch, nx, ny, iters):
    import cfdamd
    params = cfdamd.SimulationParams.cavity(400.0, iters, corrector_passes=0, tol_enabled=False)
    a, b = _states(monkeypatch, cfdamd.cavity_grid(nx, ny), params, 12)
    for f in STATE:
        assert_bitwise(f"persist cavity {nx}x{ny}:{f}", b[f], a[f])


def test_persist_matches_launches_channel_so_passes(monkeypatch):
    """Channel with a cylinder (masks), second order, 3 corrector passes
    (each pass's solve is persistent), non-power-of-two spacing."""
    import cfdamd
    grid = cfdamd.Grid(800, 264, 30.0, 10.0, cfdamd.Cylinder(7.5, 5.0, 1.5))
    params = cfdamd.SimulationParams(velocity_scheme=cfdamd.VelocityScheme.SecondOrder,
                                     jacobi_iters=64, corrector_passes=3, tol_enabled=False)
    a, b = _states(monkeypatch, grid, params, 10)
    for f in STATE:
        assert_bitwise(f"persist channel:{f}", b[f], a[f])


@pytest.mark.timeout(300)
def test_persist_developed_4096(monkeypatch):
    """The bench workload from a developed state (99 % of p' non-zero)."""
    import cfdamd
    params = cfdamd.SimulationParams.cavity(1000.0, 200, corrector_passes=0, tol_enabled=False)
    a, b = _states(monkeypatch, cfdamd.cavity_grid(4096), params, 3, develop=400)
    for f in STATE:
        assert_bitwise(f"persist 4096:{f}", b[f], a[f])
    assert np.count_nonzero(a["p_prime"]) > 0.9 * a["p_prime"].size


def test_persist_matches_oracle(monkeypatch):
    import cfdamd
    from oracle import OracleModel
    monkeypatch.setenv("CFD_PERSIST", "1")
    grid = cfdamd.cavity_grid(384, 256)
    params = cfdamd.SimulationParams.cavity(100.0, 48, corrector_passes=0, tol_enabled=False)
    m = cfdamd.Model(grid, params, device=0)
    o = OracleModel(grid.nx, grid.ny, grid.lx, grid.ly, bc_kind=1, viscosity=0.01, jacobi_iters=48,
                    tol_enabled=False, corrector_passes=0)
    try:
        for k in range(6):
            m.update()
            o.update()
        st = m.get_state()
        for f in STATE:
            assert_bitwise(f"persist oracle:{f}", st[f], o.field(f))
    finally:
        m.close()


def test_persist_off_under_graph_replay(monkeypatch):
    """CFD_GRAPH=1 replays captured steps with frozen kernel arguments, so
    the captured solves run per launch (a replayed persistent launch would
    reuse its flag epoch); the replay equals the eager persistent run."""
    import cfdamd
    grid = cfdamd.cavity_grid(512, 384)
    params = cfdamd.SimulationParams.cavity(400.0, 64, corrector_passes=0, tol_enabled=False)
    states = []
    for graph in ("0", "1"):
        monkeypatch.setenv("CFD_GRAPH", graph)
        m = cfdamd.Model(grid, params, device=0)
        try:
            m.update_n(13)
            states.append(m.get_state())
        finally:
            m.close()
    for f in STATE:
        assert_bitwise(f"persist graph:{f}", states[1][f], states[0][f])


def _run_slabs(monkeypatch, n, grid, params, steps, depth, sharded_env):
    import threading
    import cfdamd
    monkeypatch.setenv("CFD_HALO_DEPTH", str(depth))
    monkeypatch.setenv("CFD_PERSIST_SHARDED", sharded_env)
    hub = cfdamd.LocalHub(n)
    out, models, errors = [None] * n, [None] * n, []

    def worker(r):
        try:
            m = cfdamd.Model(grid, params, device=0, n_ranks=n, rank=r, local_hub=hub)
            models[r] = m
            m.update_n(steps)
            m.synchronize()
            out[r] = (m.get_state(), m.persist_blocks)
        except Exception as e:   # surfaced below
            errors.append(e)

    ts = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(600)
    for m in models:
        if m is not None:
            m.close()
    hub.close()
    if errors:
        raise errors[0]
    return out


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n", [2, 4])
def test_persist_runs_between_exchanges_on_slabs(monkeypatch, n):
    """Slabs with 32 ghost rows: the 8-sweep blocks between two p' exchanges
    run as one persistent launch over the first block's band (later blocks
    recompute ghost rows past their valid band, which the exchange replaces);
    owned rows equal the per-launch slabs bit for bit."""
    import cfdamd
    grid = cfdamd.cavity_grid(512, 1024 * n // 2)
    params = cfdamd.SimulationParams.cavity(400.0, 200, corrector_passes=0, tol_enabled=False)
    a = _run_slabs(monkeypatch, n, grid, params, 6, 32, "0")
    b = _run_slabs(monkeypatch, n, grid, params, 6, 32, "1")
    assert all(pb == 0 for _, pb in a), [pb for _, pb in a]
    assert all(pb >= 2 for _, pb in b), [pb for _, pb in b]
    for r in range(n):
        for f in STATE:
            assert_bitwise(f"slab {r}/{n}:{f}", b[r][0][f], a[r][0][f])


@pytest.mark.timeout(300)
def test_kind5_fields_over_1GiB(monkeypatch):
    """A single-domain grid whose p' field exceeds 1 GiB (16384 x 17408,
    1.14 GiB per field): kind 5 -- per-wave buffer windows, so a parked
    lane's offset never wraps -- runs it (persistently) and equals kind 1
    (CFD_TB_KIND=1, the former fallback) bit for bit."""
    import cfdamd
    grid = cfdamd.cavity_grid(16384, 17408)
    params = cfdamd.SimulationParams.cavity(1000.0, 16, corrector_passes=0, tol_enabled=False)
    states = []
    for kind in ("1", "5"):
        monkeypatch.setenv("CFD_TB_KIND", kind)
        m = cfdamd.Model(grid, params, device=0)
        try:
            assert m.jacobi_kernel["kind"] == int(kind), m.jacobi_kernel
            m.update_n(8)   # past the inlet ramp's first steps: p' non-zero under the lid
            st = m.get_state()
            states.append({f: st[f] for f in ("u", "v", "p_prime", "rhs")})
            del st
        finally:
            m.close()
    for f in ("u", "v", "p_prime", "rhs"):
        assert_bitwise(f"kind5 >1GiB:{f}", states[1][f], states[0][f])
    assert np.count_nonzero(states[1]["p_prime"]) > 0
