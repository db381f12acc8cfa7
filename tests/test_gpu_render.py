"""GPU: cfd_render / cfd_derive_field (device-side snapshot derivation,
SURVEY.md §8(f) row 1) against the numpy restatement of src/app.rs:235-403
(oracle/render.py) applied to the same model's snapshot — pixel- and
bit-exact, including NaN values, the obstacle overlay and sharded slabs."""
import numpy as np
import pytest

from _util import assert_bitwise

pytestmark = pytest.mark.gpu

MODES = (0, 1, 2)


def _check_model(m, cylinder=None):
    from render import derive, render
    g = m.grid
    snap = m.get_snapshot()
    for mode in MODES:
        img, mm = m.render(mode)
        want, wmm = render(mode, snap.u, snap.v, snap.p, g.nx, g.ny, g.dx, g.dy, cylinder)
        bad = np.argwhere((img != want).any(-1))
        assert bad.size == 0, f"mode {mode}: {len(bad)} pixels differ, first {bad[0]}"
        assert np.float32(mm[0]) == wmm[0] and np.float32(mm[1]) == wmm[1], (mode, mm, wmm)
        fld, fmm = m.derive_field(mode)
        assert_bitwise(f"field mode {mode}", fld,
                       derive(mode, snap.u, snap.v, snap.p, g.nx, g.ny, g.dx, g.dy), nan_equal=True)
        assert fmm == mm


def test_render_channel_with_cylinder():
    import cfdamd
    m = cfdamd.Model(cfdamd.default_grid(), cfdamd.SimulationParams(
        velocity_scheme=cfdamd.VelocityScheme.SecondOrder))
    for _ in range(4):
        m.update()
    c = m.grid.obstacle
    _check_model(m, (c.center_x, c.center_y, c.radius))
    m.close()


def test_render_cavity_and_injected_nans():
    import cfdamd
    n = 256
    m = cfdamd.Model(cfdamd.cavity_grid(n, 128),
                     cfdamd.SimulationParams.cavity(400.0, 100, corrector_passes=0,
                                                    tol_enabled=False))
    m.update_n(6)
    _check_model(m)
    # random state with NaNs, infinities and signed zeros
    rng = np.random.default_rng(7)
    st = m.get_state()
    kw = {}
    for k in ("u", "v", "p"):
        a = rng.standard_normal(st[k].size).astype(np.float32)
        a[rng.integers(0, a.size, 50)] = np.nan
        a[rng.integers(0, a.size, 5)] = np.inf
        a[rng.integers(0, a.size, 50)] = -0.0
        kw[k] = a
    m.set_state(**kw)
    _check_model(m)
    # constant (all-zero) field: the 1e-6 range widening
    m.set_state(u=np.zeros_like(st["u"]), v=np.zeros_like(st["v"]), p=np.zeros_like(st["p"]))
    _check_model(m)
    m.close()


def test_render_sharded_slabs_equal_single():
    """Each slab renders its own rows with the global min/max (all-reduced),
    so the stacked slab images equal the single-domain image."""
    import threading
    import cfdamd
    grid = cfdamd.Grid(128, 60, 30.0, 10.0, cfdamd.Cylinder(7.5, 5.0, 1.9))
    params = cfdamd.SimulationParams(jacobi_iters=30, corrector_passes=1, tol_enabled=False)
    single = cfdamd.Model(grid, params)
    single.update_n(4)
    want = [single.render(mode) for mode in MODES]
    single.close()
    n = 3
    hub = cfdamd.LocalHub(n)
    out, errors = [None] * n, []

    def worker(r):
        try:
            m = cfdamd.Model(grid, params, device=0, n_ranks=n, rank=r, local_hub=hub)
            m.update_n(4)
            out[r] = [m.render(mode) for mode in MODES]
            m.synchronize()
            m.close()
        except Exception as e:
            errors.append(e)

    ts = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(300)
    hub.close()
    if errors:
        raise errors[0]
    for k, mode in enumerate(MODES):
        img = np.concatenate([out[r][k][0] for r in range(n)])
        assert np.array_equal(img, want[k][0]), f"mode {mode}"
        assert all(out[r][k][1] == want[k][1] for r in range(n))
