"""GPU parity of the JavaScript variant's pressure solvers (SURVEY.md §8(f)
row 3) selected through cfd_params.pressure_solver:

* multigrid (index.html:775-795, 1344-1470): bit-exact against the reference
  script itself, executed by node on the same inputs
  (tests/golden/js_mg_*.npz, make_js_golden.py), for every split of the
  V-cycle between grid-wide launches and the single-workgroup tail;
* red-black SOR (index.html:741-774 per-cell formula): bit-exact against the
  C restatement (oracle/cfd_oracle_solvers.c), itself cross-checked by numpy;
* whole Model::update steps with either solver, tolerance on and off, channel
  and cavity: bit-exact against the oracle.
"""
import json
import os

import numpy as np
import pytest

from _util import assert_bitwise

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
JS = json.load(open(os.path.join(GOLD, "js_manifest.json")))["fixtures"]


def _cfd():
    import cfdamd
    return cfdamd


def _oracle(nx, ny, lx, ly, cylinder=None, **p):
    from oracle import OracleModel
    return OracleModel(nx, ny, lx, ly, cylinder=cylinder, **p)


@pytest.mark.parametrize("tail,tb,smooth", [("default", "1", None), ("0", "1", None),
                                            ("100000000", "1", None), ("0", "0", None),
                                            ("0", "1", "2"), ("0", "1", "1")])
@pytest.mark.parametrize("name", sorted(JS))
def test_multigrid_solve_matches_reference_javascript(monkeypatch, name, tail, tb, smooth):
    """tail: levels run in the single-workgroup tail (0: only the coarsest);
    tb: five smoothing sweeps per launch (1) or one per launch (0); smooth:
    CFD_MG_SMOOTH (2: the row march on every level, 1: the LDS block form)."""
    c = _cfd()
    if smooth is not None:
        monkeypatch.setenv("CFD_MG_SMOOTH", smooth)
    if tail != "default":
        monkeypatch.setenv("CFD_MG_TAIL", tail)
    monkeypatch.setenv("CFD_MG_TB", tb)
    meta = JS[name]
    fx = np.load(os.path.join(GOLD, name + ".npz"))
    nx, ny = meta["nx"], meta["ny"]
    m = c.Model(c.Grid(nx, ny, meta["lx"], meta["ly"]),
                c.SimulationParams(pressure_solver=c.PressureSolver.Multigrid))
    m.set_state(rhs=fx["in_rhs"], p_prime=np.full(nx * ny, 7.0, np.float32))
    r = m.pressure_solve()
    st = m.get_state()
    assert_bitwise(f"{name} tail={tail} tb={tb}: p'", st["p_prime"], fx["out_solve"])
    assert np.float32(r) == np.float32(fx["out_residual_f64"][0])
    assert st["jacobi_sweeps_total"] == 1


@pytest.mark.parametrize("fused", ["1", "0"])
@pytest.mark.parametrize("nx,ny,lx,ly,iters,tol,scale", [
    (64, 48, 4.0 / 3.0, 1.0, 40, False, 1.0),     # IEEE double division
    (128, 128, 1.0, 1.0, 60, False, 1.0),         # power-of-two divisors: reciprocal multiply
    (96, 72, 30.0, 10.0, 500, True, 1e-2),        # converges and exits early
    (264, 150, 2.64, 1.5, 33, False, 1.0),        # 3 wave columns, ragged last segment
    (256, 19, 1.0, 1.0, 7, True, 1.0),            # one 16-row segment, tolerance on
    (16, 4, 1.0, 1.0, 5, False, 1.0),             # smallest grid (two color passes)
])
def test_sor_solve_matches_oracle(monkeypatch, fused, nx, ny, lx, ly, iters, tol, scale):
    """k_sor_fused (one launch per red-black iteration, ping-pong buffers;
    CFD_SOR_FUSED=1, the default where it applies) and the in-place two color
    passes (=0) against the oracle's red-black restatement, bitwise."""
    monkeypatch.setenv("CFD_SOR_FUSED", fused)
    c = _cfd()
    import oracle
    rng = np.random.default_rng(nx + ny)
    rhs = (rng.uniform(-1, 1, nx * ny) * scale).astype(np.float32)
    m = c.Model(c.Grid(nx, ny, lx, ly),
                c.SimulationParams(pressure_solver=c.PressureSolver.Sor, jacobi_iters=iters,
                                   tol_enabled=tol))
    m.set_state(rhs=rhs, p_prime=rng.uniform(-1, 1, nx * ny).astype(np.float32))
    r = m.pressure_solve()
    want = np.empty(nx * ny, np.float32)
    dx, dy = np.float32(lx) / np.float32(nx), np.float32(ly) / np.float32(ny)
    r2, n = oracle.sor_solve(want, rhs, nx, ny, dx, dy, iters, tol, 1e-4)
    st = m.get_state()
    assert_bitwise(f"sor {nx}x{ny}", st["p_prime"], want)
    assert np.float32(r) == np.float32(r2)
    assert st["jacobi_sweeps_total"] == n
    if tol:
        assert n < iters


@pytest.mark.parametrize("solver", [1, 2])
@pytest.mark.parametrize("case", ["channel_ref", "channel_fused", "cavity_fixed"])
def test_steps_with_solver_match_oracle(solver, case):
    c = _cfd()
    if case == "channel_ref":      # reference knobs: tolerance on, 20 corrector passes
        g = dict(nx=128, ny=64, lx=30.0, ly=10.0, cylinder=(7.5, 5.0, 0.75))
        kw = dict(scheme=1)
    elif case == "channel_fused":  # corrector_passes 0: fused corrector/boundary/residuals
        g = dict(nx=192, ny=96, lx=30.0, ly=10.0, cylinder=(7.5, 5.0, 1.5))
        kw = dict(jacobi_iters=30, corrector_passes=0, tol_enabled=0, inlet_profile=1)
    else:
        g = dict(nx=128, ny=128, lx=1.0, ly=1.0, cylinder=None)
        kw = dict(bc_kind=1, viscosity=0.01, jacobi_iters=25, corrector_passes=2, tol_enabled=0)
    o = _oracle(g["nx"], g["ny"], g["lx"], g["ly"], g["cylinder"], pressure_solver=solver, **kw)
    cyl = g["cylinder"]
    m = c.Model(c.Grid(g["nx"], g["ny"], g["lx"], g["ly"], c.Cylinder(*cyl) if cyl else None),
                c.SimulationParams(
                    velocity_scheme=c.VelocityScheme(kw.get("scheme", 0)),
                    inlet_profile=c.InletProfile(kw.get("inlet_profile", 0)),
                    pressure_solver=c.PressureSolver(solver),
                    viscosity=kw.get("viscosity", 1e-6),
                    jacobi_iters=kw.get("jacobi_iters", 50),
                    corrector_passes=kw.get("corrector_passes", 20),
                    tol_enabled=bool(kw.get("tol_enabled", 1)),
                    bc_kind=c.BoundaryKind(kw.get("bc_kind", 0))))
    for step in range(5):
        o.update()
        m.update()
        s, r = o.scalars(), m.get_residuals()
        for a, b in ((s.p, r.p), (s.u, r.u), (s.v, r.v), (s.dt, r.dt)):
            assert np.float32(a).view(np.uint32) == np.float32(b).view(np.uint32), (case, step)
        assert s.jacobi_sweeps_total == r.jacobi_sweeps_total
    st = m.get_state()
    for f in ("u", "v", "p", "u_star", "v_star", "p_prime", "rhs"):
        assert_bitwise(f"{case} solver={solver}: {f}", st[f], o.field(f))


def test_switching_solvers_mid_run():
    """set_parameters may change the solver between steps (model.rs:1255)."""
    c = _cfd()
    g = dict(nx=64, ny=48, lx=3.0, ly=2.0, cylinder=(1.0, 1.0, 0.3))
    o = _oracle(g["nx"], g["ny"], g["lx"], g["ly"], g["cylinder"])
    m = c.Model(c.Grid(64, 48, 3.0, 2.0, c.Cylinder(1.0, 1.0, 0.3)), c.SimulationParams())
    for solver in (0, 2, 1, 0, 1):
        o.set_params(pressure_solver=solver)
        m.set_parameters(c.SimulationParams(pressure_solver=c.PressureSolver(solver)))
        for _ in range(2):
            o.update()
            m.update()
    st = m.get_state()
    for f in ("u", "v", "p", "p_prime"):
        assert_bitwise(f, st[f], o.field(f))


@pytest.mark.parametrize("smooth", ["default", "2", "3"])
@pytest.mark.parametrize("nx,ny,lx,ly", [(1024, 1024, 1.0, 1.0), (1048, 1000, 30.0, 10.0)])
def test_multigrid_large_grids_match_oracle(monkeypatch, nx, ny, lx, ly, smooth):
    """Grids of >= 2^20 cells: deep hierarchies, many smoothing tiles and deep
    hierarchies (power-of-two divisors and IEEE double division).  smooth:
    CFD_MG_SMOOTH (2: the row march k_mg_smooth5m on every level, 3: the wave
    windows k_mg_smooth5w on every level)."""
    if smooth != "default":
        monkeypatch.setenv("CFD_MG_SMOOTH", smooth)
    c = _cfd()
    import oracle
    rng = np.random.default_rng(nx)
    rhs = (rng.uniform(-1, 1, nx * ny) * 50.0).astype(np.float32)
    m = c.Model(c.Grid(nx, ny, lx, ly),
                c.SimulationParams(pressure_solver=c.PressureSolver.Multigrid))
    m.set_state(rhs=rhs)
    r = m.pressure_solve()
    want = np.empty(nx * ny, np.float32)
    dx, dy = np.float32(lx) / np.float32(nx), np.float32(ly) / np.float32(ny)
    r2 = oracle.mg_solve(want, rhs, nx, ny, dx, dy)
    assert_bitwise(f"mg {nx}x{ny}", m.get_state()["p_prime"], want)
    assert np.float32(r) == np.float32(r2)


def test_multigrid_march_on_big_level_matches_windows(monkeypatch):
    """The default smoother form on a level of >= 2^22 cells is the row march
    (k_mg_smooth5m); it must give the same bits as the wave-window form
    (CFD_MG_SMOOTH=3), which the oracle tests above pin at smaller sizes (and
    the march too, under CFD_MG_SMOOTH=2)."""
    c = _cfd()
    nx, ny = 4096, 2048
    rng = np.random.default_rng(7)
    rhs = (rng.uniform(-1, 1, nx * ny) * 50.0).astype(np.float32)
    out = {}
    for smooth in ("0", "3"):
        monkeypatch.setenv("CFD_MG_SMOOTH", smooth)
        m = c.Model(c.Grid(nx, ny, 2.0, 1.0),
                    c.SimulationParams(pressure_solver=c.PressureSolver.Multigrid))
        m.set_state(rhs=rhs)
        r = m.pressure_solve()
        out[smooth] = (m.get_state()["p_prime"], np.float32(r))
        m.close()
    assert_bitwise("march vs windows 4096x2048", out["0"][0], out["3"][0])
    assert out["0"][1] == out["3"][1]
