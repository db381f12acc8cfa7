"""GPU: the persistent fixed-count solve (k_jacobi_persist, CFD_PERSIST=1).

One launch runs the 8-sweep blocks of a solve; workgroups take (block, tile)
tasks by ticket and hand rows to their neighbours through per-tile flags
inside the launch (write-through p' stores, agent acquire after each poll).
Every field must equal the per-launch form bit for bit -- across grids whose
tiles split unevenly, with the obstacle masks, the second-order scheme,
corrector passes, the IEEE division path, and a developed 4096^2 state -- and
the oracle; every persistent case asserts that the persistent path ran.
Since r4 the launch completes with any number of its workgroups resident
(owned tiles, claims, stealing): late owners, forced stealing, a grid larger
than the GPU holds, and two models' launches running at once on one GPU are
bitwise too.
"""
import os

import numpy as np
import pytest

from _util import assert_bitwise

pytestmark = pytest.mark.gpu

STATE = ("u", "v", "p", "u_star", "v_star", "p_prime", "rhs")


@pytest.fixture(autouse=True)
def _persistent_on(monkeypatch):
    """Single-domain persistence is opt-in since r4 (the per-launch march
    with the guarded SUMS form is the default there); these tests ask for it
    unless they set CFD_PERSIST themselves."""
    monkeypatch.setenv("CFD_PERSIST", "1")


def pow2_grid(nx, ny, inv=512):
    """A cavity-type grid whose spacings are 1/inv (a power of two) whatever
    nx, ny are: the reciprocal-multiply division is proven exact there, so
    the default kernel is kind 5 and fixed-count solves run persistently
    (cavity_grid(nx, ny) has spacing 1/ny, which for ny = 200, 384, 1000 gives
    IEEE division, kind 4 and no persistent launch)."""
    import cfdamd
    return cfdamd.Grid(nx, ny, nx / inv, ny / inv, None)


def _states(monkeypatch, grid, params, steps, develop=0, envs=("0", "1"), persistent=True,
            steals=None):
    """States after `steps` steps with CFD_PERSIST=0 then =1 (or `envs`: a
    list of CFD_PERSIST values or dicts of variables); asserts which path each
    solve took (persist_blocks 0 per launch, > 0 persistent -- or 0 when
    `persistent` is False: a solve with fewer than two leading 8-sweep blocks
    has nothing to run persistently)."""
    import cfdamd
    out = []
    for env in envs:
        env = env if isinstance(env, dict) else {"CFD_PERSIST": env}
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        m = cfdamd.Model(grid, params, device=0)
        try:
            if develop:
                m.update_n(develop)
            m.update_n(steps)
            st = m.get_state()
            pb = m.persist_blocks
            if steals is not None:
                steals.append(m.persist_steals)
            if env.get("CFD_PERSIST", "1") == "0" or not persistent:
                assert pb == 0, (env, pb)
            else:
                assert pb > 0, (env, pb)
            out.append(st)
        finally:
            m.close()
    return out


@pytest.mark.parametrize("nx,ny,iters", [(256, 200, 50), (256, 200, 48), (1024, 1024, 100), (640, 1000, 200),
                                          (1024, 1024, 1200), (2048, 384, 40)])
def test_persist_matches_launches_cavity(monkeypatch, nx, ny, iters):
    """50 sweeps split 8 + 6 x 7 (one leading 8-sweep block: per launch);
    100 = 9 x 8 + 4 x 7 (9 persistent blocks, the 7-sweep ones per launch)."""
    import cfdamd
    params = cfdamd.SimulationParams.cavity(400.0, iters, corrector_passes=0, tol_enabled=False)
    a, b = _states(monkeypatch, pow2_grid(nx, ny), params, 12, persistent=iters != 50)
    for f in STATE:
        assert_bitwise(f"persist cavity {nx}x{ny}:{f}", b[f], a[f])


@pytest.mark.parametrize("kind", ["5", "default"])
def test_persist_matches_launches_channel_so_passes(monkeypatch, kind):
    """Channel with a cylinder (masks), second order, 3 corrector passes
    (each pass's solve is persistent), non-power-of-two spacing: kind 5 forced
    (CFD_TB_KIND=5), so the persistent launch runs its IEEE / FMA-corrected
    division instantiation; by default such grids run kind 4 per launch."""
    import cfdamd
    grid = cfdamd.Grid(800, 264, 30.0, 10.0, cfdamd.Cylinder(7.5, 5.0, 1.5))
    params = cfdamd.SimulationParams(velocity_scheme=cfdamd.VelocityScheme.SecondOrder,
                                     jacobi_iters=64, corrector_passes=3, tol_enabled=False)
    if kind == "5":
        monkeypatch.setenv("CFD_TB_KIND", "5")
    a, b = _states(monkeypatch, grid, params, 10, persistent=kind == "5")
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
        assert m.persist_blocks == 6, m.persist_blocks
        for f in STATE:
            assert_bitwise(f"persist oracle:{f}", st[f], o.field(f))
    finally:
        m.close()


@pytest.mark.parametrize("env", [{"CFD_PERSIST_GRID": "5000"}, {"CFD_PERSIST_LATE": "7"},
                                 {"CFD_PERSIST_LATE": "3", "CFD_PERSIST_STEAL_US": "0"},
                                 {"CFD_PERSIST_STEAL_US": "0"}])
def test_persist_stealing_bitwise(monkeypatch, env):
    """Each workgroup owns a tile; a neighbour block nobody has claimed for
    CFD_PERSIST_STEAL_US is claimed and run by the waiting workgroup.  Forced
    here: owners of every 7th / 3rd tile start 2 ms late (CFD_PERSIST_LATE,
    as a non-resident owner would), stealing at once (STEAL_US=0), and a grid
    of 5000 workgroups (more than the GPU holds; the surplus owns nothing).
    Every task still runs exactly once, in dependency order: bitwise vs per
    launch."""
    import cfdamd
    params = cfdamd.SimulationParams.cavity(400.0, 64, corrector_passes=0, tol_enabled=False)
    steals = []
    a, b = _states(monkeypatch, pow2_grid(640, 1000), params, 4,
                   envs=("0", dict(env, CFD_PERSIST="1")), steals=steals)
    for f in STATE:
        assert_bitwise(f"persist {env}:{f}", b[f], a[f])
    if "CFD_PERSIST_LATE" in env:
        assert steals[-1] > 0, steals   # the late owners' blocks were stolen


@pytest.mark.timeout(300)
def test_persist_two_models_at_once(monkeypatch):
    """Two 4096^2 models step at the same time on one GPU, each on its own
    stream from its own thread, with persistent solves and no gate between
    them: 2 x 740 workgroups, more than the GPU holds at once (the co-tenant
    case that stranded the r3 launch until its spin limit).  Owners that are
    not resident have their blocks stolen; each model equals its per-launch
    run bit for bit."""
    import threading
    import cfdamd
    grid = cfdamd.cavity_grid(4096)
    params = [cfdamd.SimulationParams.cavity(re, 200, corrector_passes=0, tol_enabled=False)
              for re in (1000.0, 400.0)]
    monkeypatch.setenv("CFD_PERSIST", "0")
    want = []
    for p in params:
        m = cfdamd.Model(grid, p, device=0)
        try:
            m.update_n(6)
            want.append(m.get_state())
        finally:
            m.close()
    monkeypatch.setenv("CFD_PERSIST", "1")
    monkeypatch.setenv("CFD_PERSIST_GATE", "0")
    models = [cfdamd.Model(grid, p, device=0) for p in params]
    got, errors = [None, None], []

    def run(k):
        try:
            for _ in range(6):   # one step per call: the two streams interleave
                models[k].update()
            got[k] = (models[k].get_state(), models[k].persist_blocks)
        except Exception as e:   # surfaced below
            errors.append(e)

    try:
        ts = [threading.Thread(target=run, args=(k,), daemon=True) for k in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(240)
    finally:
        for m in models:
            m.close()
    assert not errors, errors
    for k in range(2):
        assert got[k][1] == 25, got[k][1]   # (steals are possible, not required: residency varies)
        for f in STATE:
            assert_bitwise(f"two models [{k}]:{f}", got[k][0][f], want[k][f])


def test_persist_deadline_fault_is_loud_and_recoverable(monkeypatch):
    """A wait past the deadline (forced here: CFD_PERSIST_DEADLINE_US=0, so
    any neighbour not yet done counts as a fault) aborts the launch.  r5: the
    model recovers by itself -- the synchronisation that sees the fault
    restores the checkpoint the model took after its last synchronisation
    and re-runs the steps since with one launch per block -- and reports it
    once (CFD_ETIMEOUT).  With NO set_state by the caller, every later step
    equals the oracle, and the model's solves run per launch from then on."""
    import cfdamd
    from cfdamd._lib import CFD_ETIMEOUT, CfdError
    from oracle import OracleModel
    grid = cfdamd.cavity_grid(1024, 1024)
    params = cfdamd.SimulationParams.cavity(400.0, 200, corrector_passes=0, tol_enabled=False)
    o = OracleModel(grid.nx, grid.ny, grid.lx, grid.ly, bc_kind=1, viscosity=1.0 / 400.0,
                    jacobi_iters=200, tol_enabled=False, corrector_passes=0)
    monkeypatch.setenv("CFD_PERSIST", "1")
    m = cfdamd.Model(grid, params, device=0)
    try:
        for _ in range(3):
            m.update()
            o.update()
        monkeypatch.setenv("CFD_PERSIST_DEADLINE_US", "0")
        steps = 0   # updates the model accepted
        with pytest.raises(CfdError) as ei:
            for _ in range(20):   # a fault on the first persistent solve is near-certain
                m.update()
                steps += 1
                m.synchronize()
        assert ei.value.code == CFD_ETIMEOUT, ei.value
        assert "recovered" in str(ei.value), ei.value
        assert m.recoveries == 1
        monkeypatch.delenv("CFD_PERSIST_DEADLINE_US")
        for _ in range(steps):
            o.update()
        st = m.get_state()
        for f in STATE:
            assert_bitwise(f"recovered state:{f}", st[f], o.field(f))
        for _ in range(2):
            m.update()
            o.update()
        st = m.get_state()
        assert m.persist_blocks == 0   # per launch after the fault
        for f in STATE:
            assert_bitwise(f"after deadline fault:{f}", st[f], o.field(f))
    finally:
        m.close()


def test_persist_deadline_fault_recovers_batched_steps(monkeypatch):
    """The same fault inside a cfd_update_n batch of 4 steps: the batch is
    re-run whole from the checkpoint (taken at its start) and equals the
    oracle's 4 steps."""
    import cfdamd
    from cfdamd._lib import CFD_ETIMEOUT, CfdError
    from oracle import OracleModel
    grid = pow2_grid(512, 384)
    params = cfdamd.SimulationParams.cavity(400.0, 64, corrector_passes=0, tol_enabled=False)
    o = OracleModel(grid.nx, grid.ny, grid.lx, grid.ly, bc_kind=1, viscosity=1.0 / 400.0,
                    jacobi_iters=64, tol_enabled=False, corrector_passes=0)
    monkeypatch.setenv("CFD_PERSIST", "1")
    m = cfdamd.Model(grid, params, device=0)
    try:
        m.update_n(2)
        m.synchronize()
        for _ in range(2):
            o.update()
        monkeypatch.setenv("CFD_PERSIST_DEADLINE_US", "0")
        m.update_n(4)
        with pytest.raises(CfdError) as ei:
            m.synchronize()
        assert ei.value.code == CFD_ETIMEOUT and m.recoveries == 1, ei.value
        monkeypatch.delenv("CFD_PERSIST_DEADLINE_US")
        for _ in range(4):
            o.update()
        st = m.get_state()
        for f in STATE:
            assert_bitwise(f"batch recovered:{f}", st[f], o.field(f))
    finally:
        m.close()


@pytest.mark.timeout(300)
def test_persist_deadline_fault_on_slabs_recovers_every_rank(monkeypatch):
    """Slabs with persistent runs (CFD_PERSIST_SHARDED=1) and a forced
    deadline fault: the rank that timed out tells the others through the
    step all-reduce (Ctl::red[6]), every rank recovers at the same
    synchronisation and re-runs the same steps, and the slabs equal the
    single-domain per-launch model bit for bit."""
    import threading
    import cfdamd
    from cfdamd._lib import CFD_ETIMEOUT, CfdError
    n = 2
    grid = cfdamd.cavity_grid(512, 1024)
    params = cfdamd.SimulationParams.cavity(400.0, 200, corrector_passes=0, tol_enabled=False)
    ref = cfdamd.Model(grid, params, device=0)
    try:
        ref.update_n(5)
        want = ref.get_state()
    finally:
        ref.close()
    monkeypatch.setenv("CFD_HALO_DEPTH", "32")
    monkeypatch.setenv("CFD_PERSIST_SHARDED", "1")
    hub = cfdamd.LocalHub(n)
    out, codes, models, errors = [None] * n, [None] * n, [None] * n, []

    def worker(r):
        try:
            m = cfdamd.Model(grid, params, device=0, n_ranks=n, rank=r, local_hub=hub)
            models[r] = m
            m.update_n(5)
            try:
                m.synchronize()
                codes[r] = 0
            except CfdError as e:
                codes[r] = e.code
            out[r] = (m.get_state(), m.j0, m.j1, m.recoveries)
        except Exception as e:   # surfaced below
            errors.append(e)

    monkeypatch.setenv("CFD_PERSIST_DEADLINE_US", "0")   # every wait faults
    ts = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(240)
    for m in models:
        if m is not None:
            m.close()
    hub.close()
    if errors:
        raise errors[0]
    assert codes == [CFD_ETIMEOUT] * n, codes
    nx = grid.nx
    for st, j0, j1, rec in out:
        assert rec == 1
        for f in ("p_prime", "p", "rhs"):
            assert_bitwise(f"slab recovered {j0}:{f}", st[f], want[f].reshape(-1, nx)[j0:j1].ravel())
        assert_bitwise(f"slab recovered {j0}:u", st["u"], want["u"].reshape(-1, nx + 1)[j0:j1].ravel())

@pytest.mark.timeout(300)
def test_persist_deadline_fault_in_slab_pressure_solve(monkeypatch):
    """cfd_pressure_solve on slabs with persistent runs and a forced deadline
    fault: the entry point all-reduces the abort word itself
    (no step all-reduce runs), so every rank reports CFD_ETIMEOUT, recovers
    once and replays the same solve; p' then equals the single-domain
    per-launch model's bit for bit."""
    import threading
    import cfdamd
    from cfdamd._lib import CFD_ETIMEOUT, CfdError
    n = 2
    grid = cfdamd.cavity_grid(512, 1024)
    params = cfdamd.SimulationParams.cavity(400.0, 200, corrector_passes=0, tol_enabled=False)
    ref = cfdamd.Model(grid, params, device=0)
    try:
        ref.update_n(3)
        ref.pressure_solve()
        want = ref.get_state()
    finally:
        ref.close()
    monkeypatch.setenv("CFD_HALO_DEPTH", "32")
    monkeypatch.setenv("CFD_PERSIST_SHARDED", "1")
    hub = cfdamd.LocalHub(n)
    out, codes, models, errors = [None] * n, [None] * n, [None] * n, []
    ready = threading.Barrier(n)

    def worker(r):
        try:
            m = cfdamd.Model(grid, params, device=0, n_ranks=n, rank=r, local_hub=hub)
            models[r] = m
            m.update_n(3)
            m.synchronize()
            ready.wait(60)
            if r == 0:
                os.environ["CFD_PERSIST_DEADLINE_US"] = "0"   # every wait faults
            ready.wait(60)
            try:
                m.pressure_solve()
                m.synchronize()
                codes[r] = 0
            except CfdError as e:
                codes[r] = e.code
            out[r] = (m.get_state(), m.j0, m.j1, m.recoveries)
        except Exception as e:   # surfaced below
            errors.append(e)

    ts = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(n)]
    try:
        for t in ts:
            t.start()
        for t in ts:
            t.join(240)
    finally:
        os.environ.pop("CFD_PERSIST_DEADLINE_US", None)
        for m in models:
            if m is not None:
                m.close()
        hub.close()
    if errors:
        raise errors[0]
    assert codes == [CFD_ETIMEOUT] * n, codes
    nx = grid.nx
    for st, j0, j1, rec in out:
        assert rec == 1
        assert_bitwise(f"slab solve recovered {j0}:p_prime", st["p_prime"],
                       want["p_prime"].reshape(-1, nx)[j0:j1].ravel())


def test_persist_off_under_graph_replay(monkeypatch):
    """CFD_GRAPH=1 replays captured steps with frozen kernel arguments, so
    the captured solves run per launch (a replayed persistent launch would
    reuse its flag epoch); the replay equals the eager persistent run."""
    import cfdamd
    grid = pow2_grid(512, 384)
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
    lane's offset never wraps -- runs it persistently (4,410 tiles, more
    than one round of workgroups) and equals kind 1 (CFD_TB_KIND=1, the
    former fallback) bit for bit."""
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
            if kind == "5":
                assert m.persist_blocks == 2, m.persist_blocks
            states.append({f: st[f] for f in ("u", "v", "p_prime", "rhs")})
            del st
        finally:
            m.close()
    for f in ("u", "v", "p_prime", "rhs"):
        assert_bitwise(f"kind5 >1GiB:{f}", states[1][f], states[0][f])
    assert np.count_nonzero(states[1]["p_prime"]) > 0


def test_persist_sums_form_runs_and_guard_falls_back(monkeypatch):
    """The SUMS form ((h + v) / dx^2 for h / dx^2 + v / dy^2, bitwise while
    every value stays far below overflow) runs on a power-of-two square grid,
    and the per-task guard falls back to the reference's form where a task
    reads a huge value: p' = 2^110 in one corner (the tiles there and those
    its values reach), rhs = 2^126 (> the 2^124 limit) in one patch (the
    tiles that read it); distant tiles keep SUMS.  Every case bitwise vs
    per-launch solves (CFD_PERSIST=0, always the reference's form since r6)."""
    import cfdamd
    grid = cfdamd.cavity_grid(1024)
    params = cfdamd.SimulationParams.cavity(400.0, 200, corrector_passes=0, tol_enabled=False)
    m = cfdamd.Model(grid, params, device=0)
    try:
        m.update_n(20)
        base = m.get_state()
    finally:
        m.close()
    n = grid.nx
    pp_huge = base["p_prime"].copy().reshape(-1, n)
    pp_huge[5:40, 5:60] = np.float32(2.0 ** 110)
    rhs_huge = base["rhs"].copy().reshape(-1, n)
    rhs_huge[500:520, 300:340] = np.float32(2.0 ** 126)
    cases = {"plain": {}, "huge_pp": {"p_prime": pp_huge.ravel()},
             "huge_rhs": {"rhs": rhs_huge.ravel()}}
    envs = {"per_launch": {"CFD_PERSIST": "0", "CFD_JACOBI_SUMS": "0"},
            "no_sums": {"CFD_PERSIST": "1", "CFD_JACOBI_SUMS": "0"},
            "sums": {"CFD_PERSIST": "1", "CFD_JACOBI_SUMS": "1"}}
    sums = {}
    for name, inject in cases.items():
        out = {}
        for key, env in envs.items():
            for k, v in env.items():
                monkeypatch.setenv(k, v)
            mm = cfdamd.Model(grid, params, device=0)
            try:
                mm.set_state(**dict(base, **inject))
                mm.jacobi_pressure()
                out[key] = (mm.get_state()["p_prime"], mm.persist_blocks, mm.persist_sums)
            finally:
                mm.close()
        for key, (pp, _, _) in out.items():
            assert_bitwise(f"sums {name} [{key}]:p_prime", pp, out["per_launch"][0])
        assert out["sums"][1] == 25 and out["no_sums"][2] == 0, (out["sums"][1:], out["no_sums"][1:])
        assert out["per_launch"][1:] == (0, 0), out["per_launch"][1:]
        sums[name] = out["sums"][2]
    # plain: the owned tiles' blocks 2..24 (blocks 0 and 1 measure the inputs)
    assert sums["plain"] > 0, sums
    assert 0 < sums["huge_pp"] < sums["plain"] and 0 < sums["huge_rhs"] < sums["plain"], sums
