"""Parity of the HIP path (through the C ABI) against the CPU restatement.

Bar: bit-exact on every f32 word of the state (u, v, p, u*, v*, p', rhs) and
on the scalars (dt, time, residuals) — the reference's arithmetic is pure f32
with order-independent maxima, so nothing looser is needed.  The north star's
1e-5 relative-L2 velocity tolerance (BASELINE.json) is also asserted where a
test talks about velocity, as the stated contract.
"""
import json
import os
import time

import numpy as np
import pytest

from _util import assert_bitwise, rel_l2

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
MANIFEST = json.load(open(os.path.join(GOLD, "manifest.json")))
L2_TOL = 1e-5   # BASELINE.json north_star: <= 1e-5 relative L2 on velocity


def _cfd():
    import cfdamd
    return cfdamd


def _grid(g):
    c = _cfd()
    cyl = g.get("cylinder")
    return c.Grid(g["nx"], g["ny"], g["lx"], g["ly"], c.Cylinder(*cyl) if cyl else None)


def _params(p):
    c = _cfd()
    return c.SimulationParams(
        dt=0.005, viscosity=p.get("viscosity", 1e-6),
        velocity_scheme=c.VelocityScheme(p.get("scheme", 0)),
        inlet_profile=c.InletProfile(p.get("inlet_profile", 0)),
        jacobi_iters=p.get("jacobi_iters", 50), corrector_passes=p.get("corrector_passes", 20),
        tol_enabled=bool(p.get("tol_enabled", 1)), bc_kind=c.BoundaryKind(p.get("bc_kind", 0)))


def _oracle(g, **p):
    from oracle import OracleModel
    return OracleModel(g["nx"], g["ny"], g["lx"], g["ly"], cylinder=g.get("cylinder"), **p)


# --------------------------------------------------------------------- KATs

@pytest.mark.parametrize("name", [k for k, v in MANIFEST["fixtures"].items() if v["kind"] == "kat"])
def test_phase_kats_match_golden(name):
    c = _cfd()
    meta = MANIFEST["fixtures"][name]
    fx = np.load(os.path.join(GOLD, name + ".npz"))
    dt = np.float32(MANIFEST["kat_dt"])
    m = c.Model(_grid(meta["grid"]), c.SimulationParams(
        velocity_scheme=c.VelocityScheme(meta["scheme"])))
    mu, mv = m.get_masks()
    assert_bitwise("mask_u", mu.view(np.uint8).astype(np.float32), fx["mask_u"].astype(np.float32))
    assert_bitwise("mask_v", mv.astype(np.float32), fx["mask_v"].astype(np.float32))
    m.set_state(u=fx["in_u"], v=fx["in_v"], u_star=fx["in_u_star"], v_star=fx["in_v_star"],
                p_prime=fx["in_p_prime"], p=fx["in_p"])
    m.run_phase(0, dt)
    assert_bitwise("u_star (u predictor)", m.get_state()["u_star"], fx["out_u_star"])
    m.run_phase(1, dt)
    assert_bitwise("v_star (v predictor)", m.get_state()["v_star"], fx["out_v_star"])
    m.run_phase(2, dt)
    assert_bitwise("rhs (divergence)", m.get_state()["rhs"], fx["out_rhs"])
    r = m.jacobi_pressure()
    assert np.float32(r) == fx["out_jacobi_residual"][0]
    st = m.get_state()
    assert_bitwise("p_prime (jacobi)", st["p_prime"], fx["out_p_prime"])
    assert st["jacobi_sweeps_total"] == int(fx["out_jacobi_sweeps"][0])
    m.run_phase(3, dt)
    st = m.get_state()
    assert_bitwise("u (corrector)", st["u"], fx["out_corr_u"])
    assert_bitwise("v (corrector)", st["v"], fx["out_corr_v"])
    assert_bitwise("p (corrector)", st["p"], fx["out_corr_p"])
    m.run_phase(4, dt)
    st = m.get_state()
    assert_bitwise("u (boundary)", st["u"], fx["out_bc_u"])
    assert_bitwise("v (boundary)", st["v"], fx["out_bc_v"])


# ------------------------------------------------------------ whole steps

def _check_run(m, fx, tag):
    st = m.get_state()
    for f in ("u", "v", "p", "u_star", "v_star", "p_prime", "rhs"):
        assert_bitwise(f"{tag}:{f}", st[f], fx[f])
    t, dt, p, u, v = fx["scalars_f32"]
    step, sweeps = fx["scalars_i64"]
    assert st["simulation_step"] == step
    assert st["jacobi_sweeps_total"] == sweeps
    for k, want in (("simulation_time", t), ("dt", dt), ("last_p_residual", p),
                    ("last_u_residual", u), ("last_v_residual", v)):
        assert np.float32(st[k]).view(np.uint32) == np.float32(want).view(np.uint32), k
    assert rel_l2(st["u"], fx["u"]) <= L2_TOL and rel_l2(st["v"], fx["v"]) <= L2_TOL


@pytest.mark.parametrize("name", [k for k, v in MANIFEST["fixtures"].items() if v["kind"] == "run"])
def test_runs_match_golden(name):
    c = _cfd()
    meta = MANIFEST["fixtures"][name]
    fx = np.load(os.path.join(GOLD, name + ".npz"))
    m = c.Model(_grid(meta["grid"]), _params(meta["params"]))
    for _ in range(meta["steps"]):
        m.update()
    _check_run(m, fx, name)


@pytest.mark.parametrize("scheme", [0, 1])
def test_live_oracle_channel_nonsquare(scheme):
    """256 x 200 channel with the cylinder, 6 steps: GPU vs live oracle."""
    c = _cfd()
    g = dict(nx=256, ny=200, lx=30.0, ly=10.0, cylinder=(7.5, 5.0, 0.75))
    o = _oracle(g, scheme=scheme)
    m = c.Model(_grid(g), c.SimulationParams(velocity_scheme=c.VelocityScheme(scheme)))
    for _ in range(6):
        o.update()
        m.update()
    st = m.get_state()
    for f in ("u", "v", "p", "u_star", "v_star", "p_prime"):
        assert_bitwise(f, st[f], o.field(f))
    s = o.scalars()
    r = m.get_residuals()
    assert (r.simulation_step, np.float32(r.dt), np.float32(r.p)) == (s.step, np.float32(s.dt), np.float32(s.p))


@pytest.mark.parametrize("scheme,profile,tol", [(0, 0, 1), (1, 1, 0), (0, 1, 0), (1, 0, 1)])
def test_fused_finish_channel(scheme, profile, tol):
    """corrector_passes 0 runs corrector + boundaries + step residuals as one fused
    kernel (k_correct_finish): channel with the cylinder (outflow copy, obstacle
    faces, uniform/parabolic inlet), residuals compared every step."""
    c = _cfd()
    g = dict(nx=192, ny=96, lx=30.0, ly=10.0, cylinder=(7.5, 5.0, 1.5))
    kw = dict(scheme=scheme, inlet_profile=profile, jacobi_iters=40, corrector_passes=0,
              tol_enabled=tol)
    o = _oracle(g, **kw)
    m = c.Model(_grid(g), _params(kw))
    for step in range(8):
        o.update()
        m.update()
        s, r = o.scalars(), m.get_residuals()
        for a, b in ((s.u, r.u), (s.v, r.v), (s.p, r.p), (s.dt, r.dt)):
            assert np.float32(a).view(np.uint32) == np.float32(b).view(np.uint32), step
    st = m.get_state()
    for f in ("u", "v", "p", "u_star", "v_star", "p_prime", "rhs"):
        assert_bitwise(f, st[f], o.field(f))


@pytest.mark.parametrize("case", ["cavity", "channel_fo", "channel_passes", "wide_ragged",
                                  "cavity_so", "channel_so", "wide_ragged_so", "tall_so"])
def test_predict_div_fused_matches_unfused(monkeypatch, case):
    """The fused predictor + divergence kernels vs the separate predictor and
    k_divergence launches, every field bitwise: k_predict_march (CFD_PRED_DIV=2,
    both schemes) and k_predict_div (=1, first order).  Covers segment edges
    (ny not a multiple of the segment), wave columns of 62 / 63 chunks (nx/4 + 1
    not a multiple), face 0 / face nx / column 0, the flat wrap reads of the
    last chunk, obstacle masks, corrector passes (later divergences unfused)."""
    c = _cfd()
    so = c.VelocityScheme.SecondOrder
    cases = {
        "cavity": (c.cavity_grid(64, 48), c.SimulationParams.cavity(100.0, 30, tol_enabled=False), 6),
        "channel_fo": (c.Grid(256, 200, 30.0, 10.0, c.Cylinder(7.5, 5.0, 0.75)),
                       c.SimulationParams(corrector_passes=0), 6),
        "channel_passes": (c.Grid(192, 96, 30.0, 10.0, c.Cylinder(7.5, 5.0, 1.5)),
                           c.SimulationParams(corrector_passes=3, jacobi_iters=20), 4),
        "wide_ragged": (c.cavity_grid(1016, 37), c.SimulationParams.cavity(400.0, 12, tol_enabled=False), 3),
        "cavity_so": (c.cavity_grid(64, 48), c.SimulationParams.cavity(100.0, 30, tol_enabled=False,
                                                                      velocity_scheme=so), 8),
        "channel_so": (c.Grid(256, 200, 30.0, 10.0, c.Cylinder(7.5, 5.0, 0.75)),
                       c.SimulationParams(corrector_passes=2, velocity_scheme=so), 6),
        "wide_ragged_so": (c.cavity_grid(1016, 37), c.SimulationParams.cavity(
            400.0, 12, tol_enabled=False, velocity_scheme=so), 4),
        "tall_so": (c.Grid(248, 301, 8.0, 10.0, c.Cylinder(4.0, 5.0, 1.0)),
                    c.SimulationParams(corrector_passes=0, jacobi_iters=15, velocity_scheme=so), 5),
    }
    grid, params, steps = cases[case]
    modes = ("0", "2") if params.velocity_scheme == so else ("0", "1", "2")
    out = {}
    for fused in modes:
        monkeypatch.setenv("CFD_PRED_DIV", fused)
        m = c.Model(grid, params)
        for _ in range(steps):
            m.update()
        out[fused] = m.get_state()
        m.close()
    for mode in modes[1:]:
        for f in ("u", "v", "p", "u_star", "v_star", "p_prime", "rhs"):
            assert_bitwise(f"{f} (CFD_PRED_DIV={mode})", out[mode][f], out["0"][f])


def test_jacobi_tolerance_and_fixed_paths():
    """jacobi_pressure with random p'/rhs: early-exit (tol on) and fixed count."""
    c = _cfd()
    g = dict(nx=96, ny=72, lx=2.0, ly=1.5, cylinder=None)
    rng = np.random.default_rng(7)
    for tol, iters in ((1, 50), (0, 37), (1, 400)):
        o = _oracle(g, jacobi_iters=iters, tol_enabled=tol)
        m = c.Model(_grid(g), c.SimulationParams(jacobi_iters=iters, tol_enabled=bool(tol)))
        pp = rng.uniform(-1e-3, 1e-3, 96 * 72).astype(np.float32)
        rhs = rng.uniform(-1, 1, 96 * 72).astype(np.float32) * np.float32(1e-3)
        o.field("p_prime")[:] = pp
        o.field("rhs")[:] = rhs
        m.set_state(p_prime=pp, rhs=rhs)
        r0 = o.jacobi()
        r1 = m.jacobi_pressure()
        assert np.float32(r0) == np.float32(r1), (tol, iters)
        assert_bitwise(f"p_prime tol={tol} iters={iters}", m.get_state()["p_prime"], o.field("p_prime"))
        assert m.get_state()["jacobi_sweeps_total"] == o.scalars().jacobi_sweeps_total


def test_bench_config_full_size_bitwise():
    """BASELINE configs[2] workload (4096^2 cavity, Re=1000, 200 sweeps/step, tolerance
    off, no extra corrector passes) for 3 steps: bit-exact against the oracle at full size."""
    c = _cfd()
    n = 4096
    g = dict(nx=n, ny=n, lx=1.0, ly=1.0, cylinder=None)
    kw = dict(bc_kind=1, viscosity=0.001, jacobi_iters=200, corrector_passes=0, tol_enabled=0)
    o = _oracle(g, **kw)
    m = c.Model(c.cavity_grid(n), c.SimulationParams.cavity(1000.0, 200, corrector_passes=0,
                                                            tol_enabled=False))
    for _ in range(3):
        o.update()
        m.update()
    st = m.get_state()
    for f in ("u", "v", "p", "p_prime"):
        assert_bitwise(f, st[f], o.field(f))
    assert np.isfinite(st["u"]).all() and np.abs(st["u"]).max() > 0
    assert rel_l2(st["u"], o.field("u")) <= L2_TOL


def test_set_parameters_and_resume_bitwise():
    """set_parameters mid-run and state save/restore reproduce the oracle."""
    c = _cfd()
    g = dict(nx=64, ny=48, lx=3.0, ly=2.0, cylinder=(1.0, 1.0, 0.3))
    o = _oracle(g)
    m = c.Model(_grid(g), c.SimulationParams())
    for _ in range(3):
        o.update(); m.update()
    o.set_params(dt=0.004, viscosity=1e-3, target_inlet_velocity=2.0, scheme=1)
    m.set_parameters(c.SimulationParams(dt=0.004, viscosity=1e-3, target_inlet_velocity=2.0,
                                        velocity_scheme=c.VelocityScheme.SecondOrder))
    for _ in range(3):
        o.update(); m.update()
    saved = m.get_state()
    m2 = c.Model(_grid(g), m.params)
    m2.set_state(**saved)
    for _ in range(2):
        o.update(); m2.update()
    st = m2.get_state()
    for f in ("u", "v", "p", "p_prime"):
        assert_bitwise(f, st[f], o.field(f))


def test_invalid_shapes_fail_loudly():
    c = _cfd()
    with pytest.raises(c.CfdError):
        c.Model(c.Grid(100, 64, 1.0, 1.0), c.SimulationParams())    # nx % 8 != 0
    with pytest.raises(c.CfdError):
        c.Model(c.Grid(64, 3, 1.0, 1.0), c.SimulationParams())      # ny too small
    with pytest.raises(c.CfdError):
        c.Model(c.Grid(64, 64, 1.0, 1.0), c.SimulationParams(jacobi_iters=100000))


def test_smallest_grid_and_zero_iterations():
    c = _cfd()
    for nx, ny, iters, passes in ((16, 4, 50, 20), (16, 5, 0, 0), (24, 9, 3, 2)):
        g = dict(nx=nx, ny=ny, lx=1.0, ly=1.0, cylinder=None)
        o = _oracle(g, jacobi_iters=iters, corrector_passes=passes, bc_kind=1, viscosity=0.01)
        m = c.Model(_grid(g), c.SimulationParams(jacobi_iters=iters, corrector_passes=passes,
                                                 bc_kind=c.BoundaryKind.Cavity, viscosity=0.01))
        for _ in range(4):
            o.update(); m.update()
        st = m.get_state()
        for f in ("u", "v", "p", "p_prime"):
            assert_bitwise(f"{nx}x{ny}:{f}", st[f], o.field(f))


def test_control_handle_run_loop():
    """Model::run contract (model.rs:1282-1332): steps while unpaused,
    snapshot on request, parameters applied between steps, stop ends it."""
    c = _cfd()
    m = c.Model(c.Grid(64, 32, 2.0, 1.0), c.SimulationParams())
    h = m.run()
    t0 = time.time()
    while len(h.get_new_log_messages()) < 1 and time.time() - t0 < 30:
        time.sleep(0.01)
    h.pause()
    time.sleep(0.2)
    h.request_snapshot()
    snap = None
    while snap is None and time.time() - t0 < 30:
        snap = h.get_last_available_snapshot()
        time.sleep(0.01)
    assert snap is not None and snap.paused and snap.u.size == 65 * 32
    h.stop()
    h.join(10)


@pytest.mark.parametrize("fastdiv,temporal,kind", [
    ("0", "1", "1"), ("0", "4", "1"), ("1", "1", "1"), ("1", "3", "1"), ("1", "4", "1"),
    ("1", "8", "3"), ("0", "8", "3"), ("1", "5", "3"), ("1", "6", "3"), ("1", "7", "3"),
    ("1", "4", "3"), ("1", "3", "3"), ("1", "2", "3"), ("1", "1", "3"), ("2", "8", "3"),
    ("2", "4", "1"), ("1", "6", "4"), ("1", "8", "4"), ("0", "8", "4"), ("1", "4", "4"),
    ("1", "7", "4"), ("1", "5", "4"), ("1", "3", "4"), ("1", "2", "4"), ("1", "1", "4"),
    ("2", "6", "4"),
    ("1", "8", "5"), ("1", "7", "5"), ("1", "6", "5"), ("1", "5", "5"), ("1", "4", "5"),
    ("1", "3", "5"), ("1", "2", "5"), ("1", "1", "5"), ("0", "8", "5"), ("2", "8", "5"),
    ("0", "4", "5"), ("2", "5", "5")])
def test_kernel_variants_bitwise(monkeypatch, fastdiv, temporal, kind):
    """Every Jacobi kernel variant (IEEE or proven-exact fast division; 1..8
    sweeps per launch; kinds 1, 3, 4 and 5) gives the oracle's bits, on a power-of-two cavity (where
    the reciprocal multiply is exact) and on the reference's default channel
    grid (non-power-of-two divisors)."""
    c = _cfd()
    monkeypatch.setenv("CFD_FASTDIV", fastdiv)
    monkeypatch.setenv("CFD_TEMPORAL", temporal)
    monkeypatch.setenv("CFD_TB_KIND", kind)
    if kind == "1":
        monkeypatch.setenv("CFD_TB_ROWS", "32")
    cases = [
        (dict(nx=256, ny=128, lx=2.0, ly=1.0, cylinder=None),
         dict(bc_kind=1, viscosity=0.001, jacobi_iters=23, corrector_passes=1, tol_enabled=0)),
        (dict(nx=800, ny=264, lx=30.0, ly=10.0, cylinder=(7.5, 5.0, 0.75)),
         dict(jacobi_iters=30, corrector_passes=2, tol_enabled=0)),
    ]
    for g, kw in cases:
        o = _oracle(g, **kw)
        m = c.Model(_grid(g), _params(kw))
        cfg = m.kernel_config
        assert cfg["temporal"] == int(temporal)
        if fastdiv == "0":
            assert cfg["fastdiv"] == 0
        for _ in range(4):
            o.update()
            m.update()
        st = m.get_state()
        for f in ("u", "v", "p", "p_prime"):
            assert_bitwise(f"{g['nx']}x{g['ny']} fd={cfg['fastdiv']} T={temporal}:{f}", st[f],
                           o.field(f))


def test_power_of_two_cavity_uses_reciprocal_multiply():
    """The bench grid proves the reciprocal multiply exact and so runs the
    default march: kind 5 (rhs window in LDS) at 8 sweeps per launch."""
    c = _cfd()
    m = c.Model(c.cavity_grid(4096), c.SimulationParams.cavity(1000.0, 200, corrector_passes=0,
                                                               tol_enabled=False))
    assert m.kernel_config == {"fastdiv": 1, "temporal": 8}
    assert m.jacobi_kernel == {"kind": 5, "name": "k_jacobi_lds<8, 1, 0>"}


def test_kernel_selection_rules(monkeypatch):
    """Kind 4 keeps T = 4 inside the 256 MB Infinity Cache and goes to T = 8
    beyond it (its launch is then HBM-bound); IEEE division (a grid whose
    divisors have no proven-exact reciprocal form, CFD_FASTDIV=0 here) keeps
    kind 4 at T = 4.  Every variant is parity-tested in
    test_kernel_variants_bitwise."""
    c = _cfd()
    p = c.SimulationParams.cavity(1000.0, 200, corrector_passes=0, tol_enabled=False)
    monkeypatch.setenv("CFD_TB_KIND", "4")
    m = c.Model(c.cavity_grid(8192, 4096), p)
    assert m.kernel_config == {"fastdiv": 1, "temporal": 8}
    m.close()
    m = c.Model(c.cavity_grid(4096), p)
    assert m.kernel_config == {"fastdiv": 1, "temporal": 4}
    m.close()
    monkeypatch.delenv("CFD_TB_KIND")
    monkeypatch.setenv("CFD_FASTDIV", "0")
    m = c.Model(c.cavity_grid(1024), p)
    assert m.kernel_config == {"fastdiv": 0, "temporal": 4} and m.jacobi_kernel["kind"] == 4
    m.close()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("passes", [2, 3])
def test_corrector_head_bands_full_width(monkeypatch, passes):
    """The corrector head on a grid wide and tall enough for its 16-row bands
    (cf_rows: 4096 x 2048 gives 4 x 129 = 516 workgroups >= 2 per CU) -- the
    software-pipelined owned rows, the edge lanes' selected faces -- bitwise
    against the separate corrector + copy + divergence launches
    (CFD_CORR_HEAD=0), the loop ending on an even and on an odd pass; one step
    also against the oracle."""
    c = _cfd()
    g = dict(nx=4096, ny=2048, lx=2.0, ly=1.0, cylinder=None)
    kw = dict(bc_kind=1, viscosity=0.001, jacobi_iters=16, corrector_passes=passes, tol_enabled=False)
    fields = ("u", "v", "p", "p_prime", "u_star", "v_star", "rhs")
    got = {}
    for env in ("0", "1"):
        monkeypatch.setenv("CFD_CORR_HEAD", env)
        m = c.Model(_grid(g), _params(kw))
        try:
            for _ in range(3):
                m.update()
            got[env] = m.get_state()
        finally:
            m.close()
    for f in fields:
        assert_bitwise(f"4096x2048 passes={passes} head bands vs separate:{f}", got["1"][f], got["0"][f])
    if passes == 3:
        o = _oracle(g, **kw)
        for _ in range(3):
            o.update()
        for f in fields:
            assert_bitwise(f"4096x2048 passes={passes} head bands vs oracle:{f}", got["1"][f], o.field(f))


@pytest.mark.parametrize("passes,tol", [(1, False), (2, False), (3, False), (20, True)])
def test_corrector_head_fused_matches_separate(monkeypatch, passes, tol):
    """k_correct_head4 (r4): the corrector of pass k with pass k+1's copy and
    divergence in one launch, the passes alternating the u* / v* arrays, u / v
    written only by the loop's last corrector.  Bitwise against the separate
    launches (CFD_CORR_HEAD=0) in every field the step leaves -- u* and v*
    included -- with the loop ending on odd and even passes, fixed (1-3
    passes) and by the reference's early exit (20 passes, tolerance on), on
    the cavity and on the channel with the cylinder, and against the oracle."""
    c = _cfd()
    cases = [
        (dict(nx=256, ny=128, lx=2.0, ly=1.0, cylinder=None),
         dict(bc_kind=1, viscosity=0.001, jacobi_iters=23, corrector_passes=passes, tol_enabled=tol)),
        (dict(nx=800, ny=264, lx=30.0, ly=10.0, cylinder=(7.5, 5.0, 0.75)),
         dict(jacobi_iters=30, corrector_passes=passes, tol_enabled=tol, scheme=1)),
    ]
    fields = ("u", "v", "p", "p_prime", "u_star", "v_star", "rhs")
    for g, kw in cases:
        got = {}
        for env in ("0", "1"):
            monkeypatch.setenv("CFD_CORR_HEAD", env)
            m = c.Model(_grid(g), _params(kw))
            for _ in range(6):
                m.update()
            got[env] = m.get_state()
            m.close()
        o = _oracle(g, **kw)
        for _ in range(6):
            o.update()
        for f in fields:
            assert_bitwise(f"{g['nx']}x{g['ny']} passes={passes} fused vs separate:{f}", got["1"][f],
                           got["0"][f])
            assert_bitwise(f"{g['nx']}x{g['ny']} passes={passes} fused vs oracle:{f}", got["1"][f],
                           o.field(f))
