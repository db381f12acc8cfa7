"""GPU: round-5 paths measured on the hardware in r6 (this file runs last,
after the multi-process files, so a failure here cannot hide any default-path
test under -x):
* the lagged early-exit check of single-domain speculative solves
  (spec_lag_first, cfd_jacobi_lds.h; the default since r6, CFD_SPEC_LAG=0
  restores a k_spec_check launch after every speculative launch): each
  speculative launch checks the previous launch's residuals, the re-run
  checks the last launch's;
* CFD_SPEC_SLABS=1 -- the tolerance mode on slabs as speculative T-sweep
  blocks (enqueue_spec_slabs, cfd_model.hip) instead of the host-driven loop,
  stopping on the host's read of each block's all-reduced residuals (r6).
Every case is bitwise against the oracle and against the other path.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from _util import assert_bitwise
from test_gpu_sharded import FIELDS, assemble, check_against_oracle, run_sharded
from test_gpu_spec import STATE, _run

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ---------------------------------------------------------------- CFD_SPEC_LAG

@pytest.mark.parametrize("case", ["cavity_1e-4", "cavity_1e-3", "cavity_3e-5", "default_channel", "c2"])
def test_spec_lag_matches_oracle(monkeypatch, case):
    """The parity cases of test_gpu_spec.py with the lagged check: every
    step's fields, sweep count and residuals equal the oracle's."""
    import cfdamd
    monkeypatch.setenv("CFD_RESIDENT", "0")
    monkeypatch.setenv("CFD_SPEC_LAG", "1")
    if case.startswith("cavity"):
        p_tol = float(case.split("_")[1])
        params = cfdamd.SimulationParams.cavity(100.0, 50, p_tol=p_tol)
        sweeps = _run(cfdamd.cavity_grid(128), params, dict(bc_kind=1, viscosity=0.01, p_tol=p_tol),
                      40, f"lag cavity tol {p_tol}")
        assert any(s % 8 for s in sweeps), sweeps
    elif case == "default_channel":
        _run(cfdamd.default_grid(), cfdamd.SimulationParams(), {}, 12, "lag default channel")
    else:
        params = cfdamd.SimulationParams.cavity(400.0, 50)
        _run(cfdamd.cavity_grid(1024), params, dict(bc_kind=1, viscosity=0.0025), 6, "lag C2")


def test_spec_lag_matches_check_launch_at_every_exit(monkeypatch):
    """The lagged check (each speculative launch decides whether the previous
    one converged; the re-run decides for the last) against k_spec_check
    launches (CFD_SPEC_LAG=0) on a sweep of tolerances that puts the early exit
    at every position of an 8-sweep launch, the first and last launch
    included: identical bits, sweep counts and residuals."""
    import cfdamd
    monkeypatch.setenv("CFD_RESIDENT", "0")
    grid = cfdamd.cavity_grid(192, 160)
    seen = set()
    for p_tol in (3e-3, 1e-3, 5e-4, 2e-4, 1e-4, 5e-5):
        params = cfdamd.SimulationParams.cavity(200.0, 50, p_tol=p_tol)
        out = []
        for env in ("0", "1"):
            monkeypatch.setenv("CFD_SPEC_LAG", env)
            m = cfdamd.Model(grid, params, device=0)
            sw = []
            prev = 0
            for _ in range(12):
                m.update()
                tot = m.get_residuals().jacobi_sweeps_total
                sw.append(tot - prev)
                prev = tot
            out.append((m.get_state(), sw))
            m.close()
        for f in STATE + ("last_p_residual",):
            assert_bitwise(f"lag vs check tol {p_tol}:{f}", out[1][0][f], out[0][0][f])
        assert out[0][1] == out[1][1], (p_tol, out[0][1], out[1][1])
        seen.update(out[1][1])
    # early exits were taken (per-step totals over the corrector passes'
    # solves that are not whole 50-sweep solves), at several positions
    assert len({s % 8 for s in seen}) >= 4 and any(s % 50 for s in seen), sorted(seen)


# -------------------------------------------------------------- CFD_SPEC_SLABS

@pytest.mark.timeout(300)
@pytest.mark.parametrize("n,p_tol,depth", [(2, 1e-4, 8), (4, 1e-3, 8), (3, 3e-5, 6), (2, 2e-4, 4)])
def test_sharded_spec_tolerance_mode(monkeypatch, n, p_tol, depth):
    """r5: the reference's tolerance mode on slabs as speculative T-sweep
    blocks (one T-row p' exchange, one speculative launch, one all-reduce of
    the block's residuals and a device-side check per block; the converged
    block re-run and aligned to the host-counted buffer) equals the oracle --
    early exits at every p_tol, 20 corrector passes -- and the host-driven
    per-sweep loop it replaces (CFD_SPEC_SLABS=0).  From rest every solve
    ends in its first sweeps: r6's host-side stop makes no more collective
    calls than the host-driven loop there (r5 enqueued every block of every
    pass: 1,014 calls against 30)."""
    import cfdamd
    grid = cfdamd.cavity_grid(128, 128)
    params = cfdamd.SimulationParams.cavity(100.0, 50, p_tol=p_tol)
    calls = {}
    states = {}
    for env in ("1", "0"):
        monkeypatch.setenv("CFD_SPEC_SLABS", env)   # "0": the host-driven default
        st, ex = run_sharded(n, grid, params, 3, depth, extra=lambda m: m.comm_calls)
        states[env] = st
        calls[env] = ex[0]
    check_against_oracle(states["1"], grid, dict(bc_kind=1, viscosity=0.01, p_tol=p_tol), 3,
                         FIELDS + ("rhs",))
    a, b = assemble(states["1"], grid.nx), assemble(states["0"], grid.nx)
    for f in FIELDS:
        assert_bitwise(f"spec vs host-driven:{f}", a[f], b[f])
    assert calls["1"] <= calls["0"], calls


@pytest.mark.timeout(300)
def test_sharded_spec_long_solves_fewer_collectives(monkeypatch):
    """A developed cavity injected into 2 slabs (set_state) with a tolerance
    no sweep reaches (p_tol 1e-9): every solve runs its 50 sweeps and the
    pass loop all 20 passes, the regime the speculative blocks are for.  The
    blocks (7 exchanges + 7 all-reduces + 1 ghost row per solve) make at most
    a third of the host-driven loop's collective calls (2 per sweep), and
    both equal the single-domain model bit for bit."""
    import cfdamd
    from test_gpu_sharded import _slab_slices
    import threading
    grid = cfdamd.cavity_grid(128, 128)
    base = cfdamd.SimulationParams.cavity(100.0, 50)
    m = cfdamd.Model(grid, base, device=0)
    m.update_n(30)
    st0 = m.get_state()
    m.close()
    params = cfdamd.SimulationParams.cavity(100.0, 50, p_tol=1e-9)
    ref = cfdamd.Model(grid, params, device=0)
    ref.set_state(**st0)
    ref.update_n(2)
    want = ref.get_state()
    ref.close()
    calls = {}
    for env in ("1", "0"):
        monkeypatch.setenv("CFD_SPEC_SLABS", env)
        hub = cfdamd.LocalHub(2)
        out, models, errors = [None] * 2, [None] * 2, []

        def worker(r):
            try:
                mm = cfdamd.Model(grid, params, device=0, n_ranks=2, rank=r, local_hub=hub)
                models[r] = mm
                mm.set_state(**_slab_slices(st0, grid.nx, mm.j0, mm.j1))
                c0 = mm.comm_calls
                mm.update_n(2)
                mm.synchronize()
                out[r] = (mm.j0, mm.j1, mm.get_state(), mm.comm_calls - c0)
            except Exception as e:   # surfaced below
                errors.append(e)

        ts = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(240)
        for mm in models:
            if mm is not None:
                mm.close()
        hub.close()
        if errors:
            raise errors[0]
        calls[env] = out[0][3]
        p = np.concatenate([s["p"] for (_, _, s, _) in out])
        pp = np.concatenate([s["p_prime"] for (_, _, s, _) in out])
        assert_bitwise(f"long solves [{env}]:p", p, want["p"])
        assert_bitwise(f"long solves [{env}]:p_prime", pp, want["p_prime"])
    # 2 steps x 21 solves of 50 sweeps: 100 calls per solve host-driven, 15
    # with the blocks (plus the per-step u/v exchange and all-reduce)
    assert calls["1"] * 3 <= calls["0"], calls


@pytest.mark.parametrize("n,scheme", [(2, 1), (3, 0)])
def test_spec_slabs_channel_cylinder_across_slabs(monkeypatch, n, scheme):
    """test_gpu_sharded's reference-defaults channel (cylinder straddling the
    slab boundary, 20 corrector passes) through the speculative slab blocks."""
    import cfdamd
    monkeypatch.setenv("CFD_SPEC_SLABS", "1")
    grid = cfdamd.Grid(128, 60, 30.0, 10.0, cfdamd.Cylinder(7.5, 5.0, 1.9))
    params = cfdamd.SimulationParams(velocity_scheme=cfdamd.VelocityScheme(scheme))
    st = run_sharded(n, grid, params, 4, 8)
    check_against_oracle(st, grid, dict(scheme=scheme), 4, FIELDS)


@pytest.mark.timeout(600)
def test_spec_slabs_rccl_loopback_fewer_collectives():
    """Two RCCL ranks (socket transport on the one GPU, tools/rccl_loopback.py)
    in the reference's tolerance mode on the channel: bitwise the single-domain
    model with the speculative slab blocks and with the host-driven loop, and
    the blocks make no more collective calls per step."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from jsonl import records
    calls = {}
    for env in ("1", "0"):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rccl_loopback.py"),
                            "--n", "2", "--steps", "3", "--mode", "tol"],
                           env=dict(os.environ, CFD_SPEC_SLABS=env), capture_output=True, text=True,
                           timeout=280)
        lines = records(r.stdout)
        assert r.returncode == 0 and len(lines) == 1, (r.stdout[-2000:], r.stderr[-3000:])
        assert lines[0]["bitwise_equal_single_domain"], lines
        calls[env] = lines[0]["collective_calls_per_step_rank0"]
    # from rest: no more calls than the host-driven loop (r6 host-side stop)
    assert calls["1"] <= calls["0"], calls
