"""CPU: the restatement of the JavaScript variant's pressure solvers
(oracle/cfd_oracle_solvers.c) against the reference's own script and an
independent numpy restatement.

* Multigrid: bit-exact against the script's mgSmooth / mgRestrict /
  mgProlongate / mgVcycle and its multigrid branch (index.html:775-795,
  1344-1470) as executed by node (tests/golden/js_mg_*.npz,
  make_js_golden.py).
* Red-black SOR (index.html:741-774 per-cell formula; the script's
  lexicographic order is not reproducible in parallel, so parity with the
  script itself is unpinned for SOR): bit-exact against numpy.
"""
import json
import os

import numpy as np
import pytest

from _util import assert_bitwise

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
JS = json.load(open(os.path.join(GOLD, "js_manifest.json")))["fixtures"]


def _orc():
    import oracle
    return oracle


@pytest.mark.parametrize("name", sorted(JS))
def test_multigrid_matches_reference_javascript(name):
    o = _orc()
    meta = JS[name]
    fx = np.load(os.path.join(GOLD, name + ".npz"))
    nx, ny = meta["nx"], meta["ny"]
    dx, dy = meta["dx"], meta["dy"]
    nx_c, ny_c = (nx + 1) // 2, (ny + 1) // 2
    p, rhs = fx["in_p"], fx["in_rhs"]
    s = p.copy()
    o.mg_smooth(s, rhs, nx, ny, dx, dy, 5)
    assert_bitwise("mgSmooth", s, fx["out_smooth"])
    assert_bitwise("mgRestrict", o.mg_restrict(p, nx, ny, nx_c, ny_c), fx["out_restrict"])
    assert_bitwise("mgProlongate", o.mg_prolongate(fx["in_coarse"], nx_c, ny_c, nx, ny),
                   fx["out_prolong"])
    v = p.copy()
    o.mg_vcycle(v, rhs, nx, ny, dx, dy)
    assert_bitwise("mgVcycle", v, fx["out_vcycle"])
    pp = np.full(nx * ny, 7.0, np.float32)
    r = o.mg_solve(pp, rhs, nx, ny, np.float32(dx), np.float32(dy))
    assert_bitwise("multigrid branch p'", pp, fx["out_solve"])
    assert np.float32(r) == np.float32(fx["out_residual_f64"][0])


def np_sor(rhs, nx, ny, dx, dy, iters, tol_enabled, p_tol):
    """Independent red-black restatement: each color is one vectorised update
    (a color reads only the other color), double arithmetic, f32 storage."""
    f64 = np.float64
    P = np.zeros((ny, nx), np.float32)
    R = rhs.reshape(ny, nx)
    dx, dy = f64(np.float32(dx)), f64(np.float32(dy))
    denom = 2.0 / (dx * dx) + 2.0 / (dy * dy)
    jj, ii = np.mgrid[1:ny - 1, 1:nx - 1]
    res, n = np.float32(0), 0
    for _ in range(iters):
        me = 0.0
        for color in (0, 1):
            m = ((ii + jj) & 1) == color
            J, I = jj[m], ii[m]
            old = P[J, I].astype(f64)
            upd = (((P[J, I + 1].astype(f64) + P[J, I - 1]) / (dx * dx) +
                    (P[J + 1, I].astype(f64) + P[J - 1, I]) / (dy * dy) - R[J, I]) / denom)
            new = ((1.0 - 1.7) * old + 1.7 * upd).astype(np.float32)
            P[J, I] = new
            err = np.abs(new.astype(f64) - old)
            err = err[~np.isnan(err)]
            if err.size:
                me = max(me, float(err.max()))
        P[0, :] = P[1, :]
        P[ny - 1, :] = P[ny - 2, :]
        P[:, 0] = P[:, 1]
        P[:, nx - 1] = 0.0
        n += 1
        res = np.float32(me)
        if tol_enabled and res < np.float32(p_tol):
            break
    return P.ravel(), res, n


@pytest.mark.parametrize("nx,ny,lx,ly,iters,tol,scale", [
    (32, 16, 2.0, 1.0, 40, False, 1.0),
    (48, 40, 30.0, 10.0, 200, True, 1e-2),
    (64, 64, 1.0, 1.0, 7, True, 10.0),
    (16, 4, 1.0, 1.0, 5, False, 1.0),
])
def test_red_black_sor_matches_numpy(nx, ny, lx, ly, iters, tol, scale):
    o = _orc()
    rng = np.random.default_rng(nx * 1000 + ny)
    rhs = (rng.uniform(-1, 1, nx * ny) * scale).astype(np.float32)
    dx, dy = np.float32(lx) / np.float32(nx), np.float32(ly) / np.float32(ny)
    pp = rng.uniform(-1, 1, nx * ny).astype(np.float32)   # zeroed by the solver
    r, n = o.sor_solve(pp, rhs, nx, ny, dx, dy, iters, tol, 1e-4)
    want, r2, n2 = np_sor(rhs, nx, ny, dx, dy, iters, tol, 1e-4)
    assert n == n2
    assert np.float32(r) == r2
    assert_bitwise("sor p'", pp, want)
    if tol and iters == 200:
        assert n < iters   # converged and stopped early


def test_model_dispatches_selected_solver():
    """OracleModel.pressure_solve runs the selected solver on the model's rhs
    and counts sweeps (SOR: iterations, multigrid: one per solve)."""
    o = _orc()
    nx, ny = 64, 48
    rng = np.random.default_rng(3)
    rhs = rng.uniform(-1, 1, nx * ny).astype(np.float32)
    for solver in (1, 2):
        m = o.OracleModel(nx, ny, 2.0, 1.5, pressure_solver=solver, jacobi_iters=30, tol_enabled=0)
        m.field("rhs")[:] = rhs
        r = m.pressure_solve()
        pp = np.empty(nx * ny, np.float32)
        dx, dy = np.float32(2.0) / np.float32(nx), np.float32(1.5) / np.float32(ny)
        if solver == 1:
            r2, n = o.sor_solve(pp, rhs, nx, ny, dx, dy, 30, False, 1e-4)
        else:
            r2, n = o.mg_solve(pp, rhs, nx, ny, dx, dy), 1
        assert np.float32(r) == np.float32(r2)
        assert_bitwise(f"solver {solver}", m.field("p_prime"), pp)
        assert m.scalars().jacobi_sweeps_total == n


@pytest.mark.parametrize("solver", [1, 2])
def test_model_steps_with_alternative_solvers_stay_finite(solver):
    o = _orc()
    m = o.OracleModel(64, 32, 30.0, 10.0, cylinder=(7.5, 5.0, 1.5), pressure_solver=solver)
    for _ in range(5):
        m.update()
    for f in ("u", "v", "p", "p_prime"):
        assert np.isfinite(m.field(f)).all(), f
    assert np.abs(m.field("u")).max() > 0
