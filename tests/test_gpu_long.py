"""Parity of the HIP path on full configurations and long horizons.

test_gpu_parity.py pins every kernel on short runs; this file covers what a
short run cannot:
  * BASELINE.json configs[1] (C2): the 1024 x 1024 lid-driven cavity at
    Re = 400 with 100 Poisson sweeps per step, in the bench's timed mode and in
    the reference's parity mode (early exits, corrector passes);
  * hundreds of steps from rest through the transient front, where p', u and
    v carry subnormal values (the tests assert they do, so the denormal
    behaviour of the packed VOP3P Jacobi march and of every other kernel is
    compared bit for bit), into developed flow;
  * single steps from DEVELOPED 4096^2 / 8192^2 states (the bench's workloads,
    T = 4 and T = 8 sweeps per launch), where nearly every p' cell is non-zero.

Bar: bit-exact on every f32 word of the state and on the scalars, against the
C restatement (oracle/cfd_oracle.c, parity unpinned against the Rust binary:
see DESIGN.md §4).  The oracle runs multi-threaded here (orc_set_threads,
bit-identical results) to keep the file within a couple of minutes.
"""
import os

import numpy as np
import pytest

from _util import assert_bitwise, rel_l2

pytestmark = pytest.mark.gpu

STATE = ("u", "v", "p", "u_star", "v_star", "p_prime", "rhs")
TINY = np.finfo(np.float32).tiny


def _threads():
    try:
        return max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:
        return 4


@pytest.fixture(autouse=True)
def _oracle_threads():
    import oracle
    oracle.set_threads(_threads())
    yield
    oracle.set_threads(1)


def subnormals(a):
    a = np.abs(np.asarray(a, np.float32))
    return int(((a > 0) & (a < TINY)).sum())


def compare_state(tag, m, o):
    st = m.get_state()
    for f in STATE:
        assert_bitwise(f"{tag}:{f}", st[f], o.field(f))
    s = o.scalars()
    assert st["simulation_step"] == s.step, tag
    assert st["jacobi_sweeps_total"] == s.jacobi_sweeps_total, tag
    for k, want in (("simulation_time", s.time), ("dt", s.dt), ("last_p_residual", s.p),
                    ("last_u_residual", s.u), ("last_v_residual", s.v)):
        assert np.float32(st[k]).view(np.uint32) == np.float32(want).view(np.uint32), (tag, k)
    return st


def cavity(nx, ny, re, **kw):
    import cfdamd
    from oracle import OracleModel
    g = cfdamd.cavity_grid(nx, ny)
    m = cfdamd.Model(g, cfdamd.SimulationParams.cavity(re, kw.pop("jacobi_iters", 50), **kw))
    okw = dict(bc_kind=1, viscosity=np.float32(1.0 / re), jacobi_iters=m.params.jacobi_iters,
               corrector_passes=m.params.corrector_passes, tol_enabled=int(m.params.tol_enabled))
    o = OracleModel(nx, ny, g.lx, g.ly, **okw)
    return m, o


# ------------------------------------------------------------------ C2

def test_c2_timed_mode_bitwise():
    """configs[1]: 1024^2 cavity, Re = 400, 100 sweeps per step, tolerance off,
    no extra corrector passes (the bench's timed mode at C2); scalars every
    step, the whole state at steps 4 and 10."""
    m, o = cavity(1024, 1024, 400.0, jacobi_iters=100, corrector_passes=0, tol_enabled=False)
    assert m.kernel_config == {"fastdiv": 1, "temporal": 8}
    for step in range(1, 11):
        m.update()
        o.update()
        r, s = m.get_residuals(), o.scalars()
        for a, b in ((r.u, s.u), (r.v, s.v), (r.p, s.p), (r.dt, s.dt)):
            assert np.float32(a).view(np.uint32) == np.float32(b).view(np.uint32), step
        if step in (4, 10):
            st = compare_state(f"C2 step {step}", m, o)
    assert np.abs(st["u"]).max() > 0
    assert rel_l2(st["u"], o.field("u")) <= 1e-5 and rel_l2(st["v"], o.field("v")) <= 1e-5
    m.close()


def test_c2_parity_mode_bitwise():
    """configs[1] with the reference's control flow: 100-sweep solves with the
    early exit at 1e-4 and up to 20 re-correction passes (model.rs:696-724)."""
    m, o = cavity(1024, 1024, 400.0, jacobi_iters=100)
    assert m.params.tol_enabled and m.params.corrector_passes == 20
    for step in range(1, 4):
        m.update()
        o.update()
    compare_state("C2 parity mode", m, o)
    m.close()


# --------------------------------------------------------- long horizons

LONG = {
    # name: (grid, oracle kwargs, steps, checkpoints)
    "cavity128_re100_parity": (dict(nx=128, ny=128, lx=1.0, ly=1.0, cylinder=None),
                               dict(bc_kind=1, viscosity=0.01), 400),
    "cavity256x128_re400_parity": (dict(nx=256, ny=128, lx=2.0, ly=1.0, cylinder=None),
                                   dict(bc_kind=1, viscosity=0.0025), 400),
    "cavity128_re1000_fixed50": (dict(nx=128, ny=128, lx=1.0, ly=1.0, cylinder=None),
                                 dict(bc_kind=1, viscosity=0.001, jacobi_iters=50,
                                      corrector_passes=0, tol_enabled=0), 400),
    "channel128x64_so_cylinder": (dict(nx=128, ny=64, lx=30.0, ly=10.0, cylinder=(7.5, 5.0, 0.75)),
                                  dict(scheme=1), 200),
}
CHECKPOINTS = (3, 4, 5, 6, 8, 10, 15, 25, 50, 100, 200, 300, 400)


@pytest.mark.parametrize("name", list(LONG))
def test_long_horizon_bitwise_through_subnormals(name):
    """Hundreds of steps from rest, the whole state compared at checkpoints
    along the way.  The transient front carries subnormal p', u and v values
    in the first steps (asserted), the later checkpoints are developed flow."""
    import cfdamd
    from oracle import OracleModel
    g, kw, steps = LONG[name]
    o = OracleModel(g["nx"], g["ny"], g["lx"], g["ly"], cylinder=g["cylinder"], **kw)
    cyl = g["cylinder"]
    grid = cfdamd.Grid(g["nx"], g["ny"], g["lx"], g["ly"], cfdamd.Cylinder(*cyl) if cyl else None)
    params = cfdamd.SimulationParams(
        viscosity=float(kw.get("viscosity", 1e-6)),
        velocity_scheme=cfdamd.VelocityScheme(kw.get("scheme", 0)),
        jacobi_iters=kw.get("jacobi_iters", 50), corrector_passes=kw.get("corrector_passes", 20),
        tol_enabled=bool(kw.get("tol_enabled", 1)), bc_kind=cfdamd.BoundaryKind(kw.get("bc_kind", 0)))
    m = cfdamd.Model(grid, params)
    seen = {"p_prime": 0, "u": 0, "v": 0}
    for step in range(1, steps + 1):
        m.update()
        o.update()
        if step in CHECKPOINTS:
            st = compare_state(f"{name} step {step}", m, o)
            for f in seen:
                seen[f] += subnormals(st[f])
    m.close()
    for f, n in seen.items():
        assert n > 0, f"{name}: no subnormal {f} value at any checkpoint"


# ------------------------------------------------------ developed states

@pytest.mark.parametrize("n,develop,kind,temporal,nz_min", [
    (4096, 400, None, 8, 0.9), (4096, 400, "4", 4, 0.9), (8192, 400, None, 8, 0.25)])
def test_step_from_developed_state_bitwise(monkeypatch, n, develop, kind, temporal, nz_min):
    """The bench workloads developed on the GPU (4096^2 with the default march,
    kind 5 at T = 8, MALL-resident, and with kind 4 at T = 4; 8192^2, whose
    Jacobi working set is 3x the Infinity Cache), then ONE more step on the
    GPU and on the oracle from the same state; every field bitwise."""
    import cfdamd
    from oracle import OracleModel
    if kind:
        monkeypatch.setenv("CFD_TB_KIND", kind)
        monkeypatch.setenv("CFD_TEMPORAL", str(temporal))
    m = cfdamd.Model(cfdamd.cavity_grid(n), cfdamd.SimulationParams.cavity(
        1000.0, 200, corrector_passes=0, tol_enabled=False))
    assert m.kernel_config["temporal"] == temporal
    assert m.jacobi_kernel["kind"] == (int(kind) if kind else 5)
    m.update_n(develop)
    st = m.get_state()
    nz = np.count_nonzero(st["p_prime"]) / st["p_prime"].size
    print(f"{n}^2 after {develop} steps: {nz:.1%} of p' non-zero, "
          f"{subnormals(st['p_prime'])} subnormal")
    assert nz > nz_min, f"p' only {nz:.0%} non-zero after {develop} steps"
    assert np.isfinite(st["u"]).all() and np.isfinite(st["v"]).all()
    o = OracleModel(n, n, 1.0, 1.0, bc_kind=1, viscosity=np.float32(0.001), jacobi_iters=200,
                    corrector_passes=0, tol_enabled=0)
    for f in STATE:
        o.field(f)[:] = st[f]
    sc = o.scalars()
    sc.step, sc.time, sc.dt = st["simulation_step"], st["simulation_time"], st["dt"]
    sc.jacobi_sweeps_total = st["jacobi_sweeps_total"]
    o.set_scalars(sc)
    m.update()
    o.update()
    compare_state(f"{n}^2 from step {develop}", m, o)
    m.close()


# ---------------------------------------------------- failure detection

def test_nonfinite_velocity_is_reported():
    """SURVEY.md §5 failure detection: a NaN injected into u spreads through
    the next step; cfd_get_residuals and then cfd_update report
    CFD_ENONFINITE (the reference keeps stepping silently), the runner's status
    too, and injecting a finite state clears it."""
    import cfdamd
    m, o = cavity(64, 64, 100.0)
    m.update_n(3)
    good = m.get_state()
    bad_u = good["u"].copy()
    bad_u[65 * 20 + 30] = np.nan
    m.set_state(u=bad_u)
    m.update()
    with pytest.raises(cfdamd.CfdError) as e:
        m.get_residuals()
    assert e.value.code == cfdamd.CFD_ENONFINITE
    with pytest.raises(cfdamd.CfdError) as e:
        m.update()
    assert e.value.code == cfdamd.CFD_ENONFINITE
    # an Inf is caught the same way; the runner surfaces it as its status
    inf_v = good["v"].copy()
    inf_v[64 * 10 + 7] = np.inf
    m.set_state(**{k: good[k] for k in STATE if k != "v"}, v=inf_v,
                simulation_step=good["simulation_step"])
    h = m.run()
    import time
    t0 = time.time()
    while h.status()[0] == 0 and time.time() - t0 < 30:
        time.sleep(0.01)
    rc, msg = h.status()
    h.stop()
    assert rc == cfdamd.CFD_ENONFINITE, (rc, msg)
    # a finite state: stepping resumes and matches the oracle
    m.set_state(**{k: good[k] for k in STATE}, simulation_step=good["simulation_step"],
                simulation_time=good["simulation_time"], dt=good["dt"],
                jacobi_sweeps_total=good["jacobi_sweeps_total"])
    for _ in range(3):
        o.update()
    m.update_n(2)
    for _ in range(2):
        o.update()
    compare_state("after reset", m, o)
    m.close()
