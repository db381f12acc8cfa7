"""GPU: the row-slab decomposition (cfd_create_sharded's kernels, row plans,
ghost layouts and deep-halo sweeps) against the single-domain oracle, bit for
bit, on ONE device.  The slabs live in one process and talk through the
in-process LocalHub transport (cfd_create_sharded_local) instead of RCCL —
RCCL refuses two ranks on one GPU — so everything but the RCCL calls
themselves is exercised here; bench.py drives the RCCL transport on N GPUs."""
import os
import threading

import numpy as np
import pytest

from _util import assert_bitwise

pytestmark = pytest.mark.gpu


def run_sharded(n, grid, params, steps, halo_depth, geoms=None, extra=None):
    """geoms: a list that receives every slab's Jacobi tile geometry
    (Model.jacobi_geometry, persistent form); extra(model) -> value stored per
    rank in the list's .extra attribute."""
    import cfdamd
    if halo_depth is not None:   # None: the library's default depth (bench.py's)
        os.environ["CFD_HALO_DEPTH"] = str(halo_depth)
    hub = cfdamd.LocalHub(n)
    states, models, errors = [None] * n, [None] * n, []
    extras = [None] * n

    def worker(r):
        try:
            m = cfdamd.Model(grid, params, device=0, n_ranks=n, rank=r, local_hub=hub)
            models[r] = m
            if geoms is not None:
                geoms.append(m.jacobi_geometry())
            for _ in range(steps):
                m.update()
            m.synchronize()
            states[r] = (m.j0, m.j1, m.get_state(), m.halo_depth)
            if extra is not None:
                extras[r] = extra(m)
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
    os.environ.pop("CFD_HALO_DEPTH", None)
    if errors:
        raise errors[0]
    if extra is not None:
        return states, extras
    return states


def assemble(states, nx):
    """Owned rows of every slab -> global flat arrays (v gets the top face
    from the last slab)."""
    out = {}
    for f in ("u", "p", "p_prime", "u_star", "rhs"):
        out[f] = np.concatenate([s[f] for (_, _, s, _) in states])
    for f in ("v", "v_star"):
        parts = []
        for k, (j0, j1, s, _) in enumerate(states):
            rows = s[f].reshape(j1 - j0 + 1, nx)
            parts.append(rows if k == len(states) - 1 else rows[:-1])
            if k < len(states) - 1:
                # the shared face row is held (and computed) by both ranks
                nxt = states[k + 1][2][f].reshape(-1, nx)[0]
                assert_bitwise(f"{f} shared face row {j1}", rows[-1], nxt)
        out[f] = np.concatenate(parts).ravel()
    return out


def check_against_oracle(states, grid, oracle_kw, steps, fields):
    from oracle import OracleModel
    c = grid.obstacle
    o = OracleModel(grid.nx, grid.ny, grid.lx, grid.ly,
                    cylinder=(c.center_x, c.center_y, c.radius) if c else None, **oracle_kw)
    for _ in range(steps):
        o.update()
    got = assemble(states, grid.nx)
    for f in fields:
        assert_bitwise(f, got[f], o.field(f))
    s = o.scalars()
    for (_, _, st, _) in states:
        assert np.float32(st["dt"]) == np.float32(s.dt)
        assert np.float32(st["last_p_residual"]) == np.float32(s.p)
        assert np.float32(st["last_u_residual"]) == np.float32(s.u)
        assert np.float32(st["last_v_residual"]) == np.float32(s.v)
        assert st["simulation_step"] == s.step


FIELDS = ("u", "v", "p", "p_prime", "u_star", "v_star")


@pytest.mark.parametrize("n,depth", [(2, 1), (3, 3), (4, 8), (2, 5)])
def test_sharded_fixed_mode_cavity(n, depth):
    import cfdamd
    grid = cfdamd.cavity_grid(64, 96)
    params = cfdamd.SimulationParams.cavity(100.0, 30, corrector_passes=2, tol_enabled=False)
    st = run_sharded(n, grid, params, 5, depth)
    assert all(s[3] == min(depth, 96 // n - 2) for s in st)
    check_against_oracle(st, grid, dict(bc_kind=1, viscosity=0.01, jacobi_iters=30,
                                        corrector_passes=2, tol_enabled=0), 5, FIELDS)


@pytest.mark.parametrize("n,scheme", [(2, 1), (3, 0)])
def test_sharded_parity_mode_channel_cylinder_across_slabs(n, scheme):
    """Reference defaults (tolerance on, 20 corrector passes): host-driven
    early exits with an all-reduced residual every sweep; the cylinder
    straddles the slab boundary."""
    import cfdamd
    grid = cfdamd.Grid(128, 60, 30.0, 10.0, cfdamd.Cylinder(7.5, 5.0, 1.9))
    params = cfdamd.SimulationParams(velocity_scheme=cfdamd.VelocityScheme(scheme))
    st = run_sharded(n, grid, params, 4, 8)
    check_against_oracle(st, grid, dict(scheme=scheme), 4, FIELDS)


def test_sharded_bench_like_config():
    """The bench's timed mode (200 sweeps, tolerance off, no extra passes) with
    the default halo depth 8, four slabs."""
    import cfdamd
    grid = cfdamd.cavity_grid(256, 256)
    params = cfdamd.SimulationParams.cavity(1000.0, 200, corrector_passes=0, tol_enabled=False)
    st = run_sharded(4, grid, params, 3, 8)
    check_against_oracle(st, grid, dict(bc_kind=1, viscosity=0.001, jacobi_iters=200,
                                        corrector_passes=0, tol_enabled=0), 3, FIELDS)


@pytest.mark.parametrize("n,tol", [(2, False), (3, True)])
def test_sharded_fused_finish_channel_cylinder(n, tol):
    """No extra corrector passes: the fused corrector/boundary/residual kernel
    on slabs, outflow + obstacle faces across the slab boundary, residual maxima
    all-reduced; tolerance on takes the host-driven solve."""
    import cfdamd
    grid = cfdamd.Grid(128, 60, 30.0, 10.0, cfdamd.Cylinder(7.5, 5.0, 1.9))
    params = cfdamd.SimulationParams(velocity_scheme=cfdamd.VelocityScheme(1),
                                     inlet_profile=cfdamd.InletProfile(1), jacobi_iters=40,
                                     corrector_passes=0, tol_enabled=tol)
    st = run_sharded(n, grid, params, 5, 4)
    check_against_oracle(st, grid, dict(scheme=1, inlet_profile=1, jacobi_iters=40,
                                        corrector_passes=0, tol_enabled=int(tol)), 5,
                         FIELDS + ("rhs",))


@pytest.mark.parametrize("n,nx,ny,steps", [(2, 8192, 4096, 4), (8, 16384, 8192, 4)])
def test_sharded_bench_geometry_matches_single_domain(n, nx, ny, steps):
    """bench.py's exact multi-GPU workloads (C4: 8192x4096 on 2 slabs, C5:
    16384x8192 on 8 slabs of 16.78 M cells, default halo depth nyl/32 = 32)
    for 4 timed-mode steps: the assembled slabs equal a single-domain model of
    the same grid bit for bit (the single domain is itself oracle-exact at the
    sizes the oracle can run).  Only the transport differs from the N-GPU
    bench: LocalHub copies instead of RCCL send/recv.  This pins allocation,
    slab split, row plans and the default depth at full size; four steps from
    rest leave the rows near the lower slab boundaries at zero, so the halo
    data itself is checked by the small-grid tests above (non-zero across
    every boundary, depths 1-8)."""
    import cfdamd
    grid = cfdamd.cavity_grid(nx, ny)
    params = cfdamd.SimulationParams.cavity(1000.0, 200, corrector_passes=0, tol_enabled=False)
    geoms = []
    st = run_sharded(n, grid, params, steps, None, geoms)
    assert all(s[3] == 32 for s in st), [s[3] for s in st]
    # one Jacobi geometry along the weak-scaling series (r4): every slab runs
    # the padded 3-workgroups-per-CU round of the single-domain 4096^2 model
    # (keyed on owned rows; the C5 slab's 32 ghost rows used to tip it over)
    c3 = cfdamd.Model(cfdamd.cavity_grid(4096), params, device=0)
    try:
        want = c3.jacobi_geometry()
    finally:
        c3.close()
    assert want["lds_pad"] == 24 * 1024, want
    for gm in geoms:
        assert (gm["lds_pad"], gm["wgs_per_cu"]) == (want["lds_pad"], want["wgs_per_cu"]), (gm, want)
    got = assemble(st, nx)
    del st
    m = cfdamd.Model(grid, params, device=0)
    try:
        for _ in range(steps):
            m.update()
        ref = m.get_state()
    finally:
        m.close()
    assert np.count_nonzero(ref["p_prime"]) > 0 and np.count_nonzero(ref["u"]) > 0
    for f in ("u", "v", "p", "p_prime"):
        assert_bitwise(f"{f} ({n} slabs vs single domain, {nx}x{ny})", got[f], ref[f])


def test_sharded_tolerance_toggle_keeps_deep_ghosts():
    """set_parameters flips the tolerance on (host-driven solves refresh one
    p' ghost row per sweep) and back off (deep-halo fixed-count solves read
    hg ghost rows): the fixed-count solve after the toggle must re-exchange
    the deep ghosts first, or the slabs drift from the single domain."""
    import cfdamd
    from oracle import OracleModel
    n, depth = 3, 6
    grid = cfdamd.cavity_grid(96, 96)
    fixed = cfdamd.SimulationParams.cavity(100.0, 24, corrector_passes=1, tol_enabled=False)
    tol = cfdamd.SimulationParams.cavity(100.0, 24, corrector_passes=1, tol_enabled=True)
    schedule = [fixed, fixed, tol, tol, fixed, fixed, fixed]
    os.environ["CFD_HALO_DEPTH"] = str(depth)
    hub = cfdamd.LocalHub(n)
    states, models, errors = [None] * n, [None] * n, []

    def worker(r):
        try:
            m = cfdamd.Model(grid, schedule[0], device=0, n_ranks=n, rank=r, local_hub=hub)
            models[r] = m
            for k, p in enumerate(schedule):
                if k and p is not schedule[k - 1]:
                    m.set_parameters(p)
                m.update()
            m.synchronize()
            states[r] = (m.j0, m.j1, m.get_state(), m.halo_depth)
        except Exception as e:
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
    os.environ.pop("CFD_HALO_DEPTH", None)
    if errors:
        raise errors[0]
    kw = dict(bc_kind=1, viscosity=0.01, jacobi_iters=24, corrector_passes=1)
    o = OracleModel(96, 96, 1.0, 1.0, tol_enabled=0, **kw)
    for k, p in enumerate(schedule):
        if k and p is not schedule[k - 1]:
            o.set_params(tol_enabled=int(p.tol_enabled), **kw)
        o.update()
    got = assemble(states, 96)
    for f in FIELDS:
        assert_bitwise(f"toggle:{f}", got[f], o.field(f))


@pytest.mark.parametrize("n,tol,depth", [(2, False, 4), (3, True, 2), (4, False, 8), (4, True, 3)])
def test_sharded_sor_matches_oracle(n, tol, depth):
    """SOR (pressure_solver 1, the JS variant's solver) on slabs: k_sor_fused
    over each slab's interior rows, 2 p' ghost rows exchanged after every
    iteration, the residual all-reduced (every iteration, host-checked one
    iteration behind, with the tolerance on; the last one otherwise), the
    cylinder across a slab boundary, corrector passes: bitwise against the
    single-domain oracle."""
    import cfdamd
    grid = cfdamd.Grid(128, 96, 30.0, 10.0, cfdamd.Cylinder(7.5, 5.0, 1.9))
    params = cfdamd.SimulationParams(pressure_solver=cfdamd.PressureSolver.Sor, jacobi_iters=30,
                                     corrector_passes=3, tol_enabled=tol)
    st = run_sharded(n, grid, params, 4, depth)
    check_against_oracle(st, grid, dict(pressure_solver=1, jacobi_iters=30, corrector_passes=3,
                                        tol_enabled=int(tol)), 4, FIELDS + ("rhs",))


@pytest.mark.parametrize("n,tol,smooth", [(2, False, None), (3, True, None), (4, False, None),
                                          (3, False, "2")])
def test_sharded_multigrid_matches_oracle(monkeypatch, n, tol, smooth):
    """Multigrid (pressure_solver 2) on slabs: the rhs is gathered to every
    rank, the whole grid is solved redundantly with the single-domain kernels
    and each slab keeps its rows (plus exact deep ghosts): bitwise against the
    single-domain oracle, fixed and tolerance (host-driven) modes, cylinder
    across a slab boundary, corrector passes."""
    import cfdamd
    if smooth is not None:
        monkeypatch.setenv("CFD_MG_SMOOTH", smooth)   # 2: the row-march smoother
    grid = cfdamd.Grid(128, 96, 30.0, 10.0, cfdamd.Cylinder(7.5, 5.0, 1.9))
    params = cfdamd.SimulationParams(pressure_solver=cfdamd.PressureSolver.Multigrid,
                                     corrector_passes=3, tol_enabled=tol)
    st = run_sharded(n, grid, params, 4, 4)
    check_against_oracle(st, grid, dict(pressure_solver=2, corrector_passes=3,
                                        tol_enabled=int(tol)), 4, FIELDS + ("rhs",))


def _slab_slices(st, nx, j0, j1):
    out = {}
    for k in ("u", "u_star"):
        out[k] = st[k].reshape(-1, nx + 1)[j0:j1].ravel().copy()
    for k in ("v", "v_star"):
        out[k] = st[k].reshape(-1, nx)[j0:j1 + 1].ravel().copy()
    for k in ("p", "p_prime", "rhs"):
        out[k] = st[k].reshape(-1, nx)[j0:j1].ravel().copy()
    for k in ("dt", "simulation_time", "simulation_step", "last_p_residual", "last_u_residual",
              "last_v_residual", "jacobi_sweeps_total"):
        out[k] = st[k]
    return out


def run_sharded_from_state(n, grid, params, state, steps):
    """LocalHub slabs started from a single-domain state (cfd_set_state on
    every slab, collective: it exchanges the ghosts)."""
    import cfdamd
    hub = cfdamd.LocalHub(n)
    states, models, errors = [None] * n, [None] * n, []

    def worker(r):
        try:
            m = cfdamd.Model(grid, params, device=0, n_ranks=n, rank=r, local_hub=hub)
            models[r] = m
            m.set_state(**_slab_slices(state, grid.nx, m.j0, m.j1))
            m.update_n(steps)
            m.synchronize()
            states[r] = (m.j0, m.j1, m.get_state(), m.halo_depth)
        except Exception as e:   # surfaced below
            errors.append(e)

    ts = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(900)
    for m in models:
        if m is not None:
            m.close()
    hub.close()
    if errors:
        raise errors[0]
    return states


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n,nx,ny", [(2, 8192, 4096), (8, 16384, 8192)])
def test_sharded_full_size_developed_across_boundaries(n, nx, ny):
    """C4 (2 slabs of 8192x2048) and C5 (8 slabs of 16384x1024) at bench.py's
    default halo depth (32) from a DEVELOPED cavity: the single-domain model
    runs 400 timed-mode steps, the state gets a seeded 1e-3 perturbation (so
    boundaries deep below the lid, where p' has underflowed to 0, carry data
    too), it is injected into the slabs, and two more steps on the slabs
    equal two more single-domain steps bit for bit.  Unlike 4 steps from
    rest, the rows either side of every slab boundary carry non-zero p'
    (>= 90 %), so the deep-halo exchange, the overlapped bands and the
    rhs/u/v ghosts move real data.  For C4 one step is also checked against
    the oracle from the same state."""
    import cfdamd
    grid = cfdamd.cavity_grid(nx, ny)
    params = cfdamd.SimulationParams.cavity(1000.0, 200, corrector_passes=0, tol_enabled=False)
    m = cfdamd.Model(grid, params, device=0)
    try:
        m.update_n(400)
        st0 = m.get_state()
        # the cavity develops from the lid down (p' underflows to 0 far below
        # it): a seeded 1e-3 perturbation puts data in every boundary row
        rng = np.random.default_rng(1234)
        for k in ("u", "v", "u_star", "v_star", "p_prime"):
            st0[k] = (st0[k] + (1e-3 * rng.uniform(-1.0, 1.0, st0[k].size)).astype(
                np.float32)).astype(np.float32)
        m.set_state(**st0)
        m.update_n(2)
        ref = m.get_state()
    finally:
        m.close()
    assert np.isfinite(ref["u"]).all() and np.isfinite(ref["p_prime"]).all()
    pp = st0["p_prime"].reshape(ny, nx)
    import ctypes as C
    L = cfdamd.load()
    j0, j1 = C.c_uint64(), C.c_uint64()
    bounds = []
    for r in range(1, n):
        L.cfd_plan_slab(ny, n, r, C.byref(j0), C.byref(j1))
        bounds.append(int(j0.value))
    rows = sorted({b + d for b in bounds for d in (-1, 0)})
    frac = np.count_nonzero(pp[rows]) / float(len(rows) * nx)
    assert frac >= 0.9, f"boundary rows {rows}: only {frac:.3f} of p' non-zero"
    st = run_sharded_from_state(n, grid, params, st0, 2)
    assert all(s[3] == 32 for s in st), [s[3] for s in st]
    got = assemble(st, nx)
    del st
    for f in FIELDS + ("rhs",):
        assert_bitwise(f"{f} ({n} slabs, developed, vs single domain {nx}x{ny})", got[f], ref[f])
    del got, ref
    if n == 2:
        from oracle import OracleModel
        import oracle as orc
        orc.set_threads(min(16, os.cpu_count() or 1))
        o = OracleModel(nx, ny, float(nx) / ny, 1.0, bc_kind=1, viscosity=0.001,
                        jacobi_iters=200, corrector_passes=0, tol_enabled=0)
        for k in ("u", "v", "p", "u_star", "v_star", "p_prime", "rhs"):
            o.field(k)[:] = st0[k]
        sc = o.scalars()
        sc.step, sc.time, sc.dt = st0["simulation_step"], st0["simulation_time"], st0["dt"]
        sc.jacobi_sweeps_total = st0["jacobi_sweeps_total"]
        o.set_scalars(sc)
        o.update()
        orc.set_threads(1)
        one = run_sharded_from_state(n, grid, params, st0, 1)
        got1 = assemble(one, nx)
        for f in FIELDS + ("rhs",):
            assert_bitwise(f"{f} (2 slabs, 1 developed step) vs oracle", got1[f], o.field(f))


@pytest.mark.parametrize("n,nx,ny,tol,part", [(4, 512, 512, False, "1"), (2, 512, 384, True, "1"),
                                              (3, 384, 192, False, "1"), (4, 512, 512, False, "0")])
def test_sharded_multigrid_partitioned_levels(monkeypatch, n, nx, ny, tol, part):
    """Multigrid on slabs with the fine levels partitioned (each rank smooths,
    restricts and prolongs its own rows of levels 0..P-1, with ghost-row
    exchanges; the coarse levels are gathered whole): 512^2 on 4 slabs
    partitions levels 0-2 (level 3 = the tail's), 512x384 on 2 slabs levels
    0-2, 384x192 on 3 slabs levels 0-1; CFD_MG_PARTITION=0 keeps the
    whole-grid-per-rank form.  Bitwise against the single-domain oracle, with
    corrector passes, tolerance off and on."""
    import cfdamd
    monkeypatch.setenv("CFD_MG_PARTITION", part)
    grid = cfdamd.cavity_grid(nx, ny)
    params = cfdamd.SimulationParams.cavity(400.0, 50, pressure_solver=cfdamd.PressureSolver.Multigrid,
                                            corrector_passes=2, tol_enabled=tol)
    st = run_sharded(n, grid, params, 3, 4)
    check_against_oracle(st, grid, dict(bc_kind=1, viscosity=1.0 / 400.0, pressure_solver=2,
                                        corrector_passes=2, tol_enabled=int(tol)), 3,
                         FIELDS + ("rhs",))
