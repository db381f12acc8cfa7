"""GPU: the chained 8-sweep march (k_jacobi_chain, cfd_jacobi_chain.hip, r5;
opt-in CFD_JACOBI_CHAIN=1) against the oracle and against the per-launch march it replaces.  A
workgroup's four wave segments alternate direction and hand each other the
boundary row each stage needs (start and end meetings through LDS); the
first/last row group of every wave column runs the per-launch march.  Every
field must be the reference's, bit for bit: grids whose chain plan has one or
many chain groups, ragged wave columns, the channel with its cylinder (IEEE
division), the second-order scheme, corrector passes, developed fields, and
the optimistic SUMS form's fallback."""
import numpy as np
import pytest

from _util import assert_bitwise

pytestmark = pytest.mark.gpu
STATE = ("u", "v", "p", "u_star", "v_star", "p_prime", "rhs")


def _oracle(nx, ny, lx, ly, **kw):
    from oracle import OracleModel
    return OracleModel(nx, ny, lx, ly, **kw)


CASES = [
    # nx, ny, lx, ly, cylinder, oracle/model params
    (256, 128, 2.0, 1.0, None, dict(bc_kind=1, viscosity=0.001, jacobi_iters=40, corrector_passes=0,
                                    tol_enabled=0)),
    (800, 264, 30.0, 10.0, (7.5, 5.0, 1.5), dict(jacobi_iters=32, corrector_passes=2, tol_enabled=0)),
    (800, 264, 30.0, 10.0, (7.5, 5.0, 1.5), dict(jacobi_iters=24, corrector_passes=1, tol_enabled=0,
                                                 scheme=1)),
    (1000, 700, 1.0, 0.7, None, dict(bc_kind=1, viscosity=0.002, jacobi_iters=48, corrector_passes=1,
                                     tol_enabled=0)),
    (1536, 1024, 1.5, 1.0, None, dict(bc_kind=1, viscosity=0.001, jacobi_iters=64, corrector_passes=0,
                                      tol_enabled=0)),
]


def _model(nx, ny, lx, ly, cyl, kw):
    import cfdamd
    grid = cfdamd.Grid(nx, ny, lx, ly, cfdamd.Cylinder(*cyl) if cyl else None)
    params = cfdamd.SimulationParams(
        dt=0.005, viscosity=kw.get("viscosity", 1e-6),
        velocity_scheme=cfdamd.VelocityScheme(kw.get("scheme", 0)),
        jacobi_iters=kw["jacobi_iters"], corrector_passes=kw["corrector_passes"],
        tol_enabled=bool(kw["tol_enabled"]), bc_kind=cfdamd.BoundaryKind(kw.get("bc_kind", 0)))
    return cfdamd.Model(grid, params, device=0)


@pytest.mark.parametrize("case", range(len(CASES)))
def test_chain_matches_oracle(monkeypatch, case):
    nx, ny, lx, ly, cyl, kw = CASES[case]
    # kind 5 at 8 sweeps per launch on every grid (IEEE-division grids select
    # kind 4 at T = 4 by default): the chain in all three division forms
    monkeypatch.setenv("CFD_TB_KIND", "5")
    monkeypatch.setenv("CFD_TEMPORAL", "8")
    monkeypatch.setenv("CFD_JACOBI_CHAIN", "1")
    m = _model(nx, ny, lx, ly, cyl, kw)
    try:
        assert m.jacobi_kernel["name"].startswith("k_jacobi_chain"), m.jacobi_kernel
        o = _oracle(nx, ny, lx, ly, cylinder=cyl, **kw)
        for _ in range(5):
            m.update()
            o.update()
        st = m.get_state()
        for f in ("u", "v", "p", "p_prime", "rhs"):
            assert_bitwise(f"chain {nx}x{ny}:{f}", st[f], o.field(f))
        assert m.chain_stats["launches"] > 0
    finally:
        m.close()


@pytest.mark.parametrize("n", [2048, 4096])
def test_chain_equals_per_launch_on_developed_fields(monkeypatch, n):
    """A developed cavity (300 steps), then 2 steps from the same state with
    the chain (SUMS and reference form) and with the per-launch march: every
    field identical."""
    import cfdamd
    grid = cfdamd.cavity_grid(n)
    params = cfdamd.SimulationParams.cavity(1000.0, 200, corrector_passes=0, tol_enabled=False)
    m = cfdamd.Model(grid, params, device=0)
    try:
        m.update_n(300)
        st0 = m.get_state()
    finally:
        m.close()
    assert np.count_nonzero(st0["p_prime"]) > 0.5 * st0["p_prime"].size
    out = {}
    for key, env in {"per_launch": ("0", "0"), "chain_ref": ("1", "0"), "chain_sums": ("1", "1")}.items():
        monkeypatch.setenv("CFD_JACOBI_CHAIN", env[0])
        monkeypatch.setenv("CFD_JACOBI_SUMS", env[1])
        mm = cfdamd.Model(grid, params, device=0)
        try:
            mm.set_state(**st0)
            mm.update_n(2)
            out[key] = (mm.get_state(), mm.chain_stats, mm.jacobi_kernel["name"])
        finally:
            mm.close()
    assert out["per_launch"][1]["launches"] == 0 and out["per_launch"][2].startswith("k_jacobi_lds")
    for key in ("chain_ref", "chain_sums"):
        assert out[key][1]["launches"] == 50 and out[key][1]["fallbacks"] == 0, out[key][1]
        for f in STATE:
            assert_bitwise(f"{n} {key}:{f}", out[key][0][f], out["per_launch"][0][f])


def test_chain_sums_guard_falls_back_on_huge_values(monkeypatch):
    """p' = 2^110 and rhs = 2^126 deep inside the grid (chain row groups): the
    optimistic SUMS form's bound fails there and those groups re-run in the
    reference's form; the solve equals the per-launch reference-form march
    and the oracle's sweeps."""
    import cfdamd
    n = 1024
    grid = cfdamd.cavity_grid(n)
    params = cfdamd.SimulationParams.cavity(400.0, 64, corrector_passes=0, tol_enabled=False)
    m = cfdamd.Model(grid, params, device=0)
    try:
        m.update_n(20)
        base = m.get_state()
    finally:
        m.close()
    pp = base["p_prime"].copy().reshape(-1, n)
    pp[400:430, 300:420] = np.float32(2.0 ** 110)
    rhs = base["rhs"].copy().reshape(-1, n)
    rhs[700:712, 500:540] = np.float32(2.0 ** 126)
    inject = dict(base, p_prime=pp.ravel(), rhs=rhs.ravel())
    out = {}
    for key, env in {"per_launch": ("0", "0"), "chain_sums": ("1", "1")}.items():
        monkeypatch.setenv("CFD_JACOBI_CHAIN", env[0])
        monkeypatch.setenv("CFD_JACOBI_SUMS", env[1])
        mm = cfdamd.Model(grid, params, device=0)
        try:
            mm.set_state(**inject)
            mm.jacobi_pressure()
            out[key] = (mm.get_state()["p_prime"], mm.chain_stats)
        finally:
            mm.close()
    assert_bitwise("chain sums fallback:p_prime", out["chain_sums"][0], out["per_launch"][0])
    cs = out["chain_sums"][1]
    assert cs["launches"] == 8 and cs["fallbacks"] > 0, cs
    # and the oracle's 64 sweeps from the same state
    from oracle import OracleModel
    o = OracleModel(n, n, 1.0, 1.0, bc_kind=1, viscosity=1.0 / 400.0, jacobi_iters=64,
                    corrector_passes=0, tol_enabled=0)
    for k in ("u", "v", "p", "u_star", "v_star", "p_prime", "rhs"):
        o.field(k)[:] = inject[k]
    o.jacobi()
    assert_bitwise("chain sums fallback vs oracle:p_prime", out["chain_sums"][0], o.field("p_prime"))
