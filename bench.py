#!/usr/bin/env python3
"""Benchmark of the MI355X pressure-projection hot path (cfd-demo src/model.rs).

BASELINE.json metric: Poisson cell-updates/s + ms/timestep on the lid-driven
cavity.  N=1 runs configs[2] (4096 x 4096, Re=1000, 200 Jacobi sweeps/step);
N>1 is the weak-scaling series of SURVEY.md §8(d): every GPU holds a
4096 x 4096-cell slab of a global grid (N=2: 8192 x 4096, N=4: 8192 x 8192,
N=8: 16384 x 8192), 1D row slabs with RCCL halo exchange over xGMI.

A step = one full Model::update (model.rs:304-379) in the reference's timed
mode: first-order upwind predictor, divergence, ONE pressure solve of K=200
sweeps (tolerance off, no extra corrector passes), corrector, boundaries,
residual/CFL reductions.  value = global cells x 200 sweeps x steps /
max-over-ranks wall time of the timed steps (inputs resident in HBM).

The timed data does not depend on --warmup: every run first develops the
cavity for --develop (400) untimed steps from rest (97 % of p' non-zero, vs 3 %
after 20), then runs the W warm-up steps, then times K steps.  After timing, one
more step runs on the GPU and on the CPU oracle from the same developed state
and the two are compared bit for bit (`parity_developed_step`).

roofline: `achieved` is the one-pass HBM bytes of a Jacobi launch (read p',
read rhs, write p' once: 12 B x slab cells) over the measured
launch time; a launch performs T sweeps on chip, so `algorithmic_sweep_equiv`
reports the 12 B x cells x T figure separately.  At N=1 a second entry,
`roofline_control`, times the same kernel family on 8192^2 (T = 8), whose
768 MB Jacobi working set cannot live in the 256 MB Infinity Cache.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

`--gpus N` with N > 1 and no external launcher (WORLD_SIZE unset): this
process spawns the N ranks itself (one child per GPU, RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR / MASTER_PORT set) before anything touches the GPU,
and prints rank 0's JSON line; it never measures fewer ranks than asked.
"""
import argparse
import json
import os
import platform
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cfd-demo_amd"))

METRIC = "cell-updates/s (Poisson iter) + ms/timestep, 4096² grid, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BYTES_PER_CELL_UPDATE = 12     # read p', read rhs, write p'_new (f32)
WEAK_GRIDS = {1: (4096, 4096), 2: (8192, 4096), 4: (8192, 8192), 8: (16384, 8192)}


def global_grid(n):
    if n in WEAK_GRIDS:
        return WEAK_GRIDS[n]
    return 4096, 4096 * n


def cpu_info():
    model = platform.processor() or "unknown"
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True).stdout
        for line in out.splitlines():
            if line.startswith("Model name"):
                model = line.split(":", 1)[1].strip()
    except Exception:
        pass
    return model, os.cpu_count()


def cpu_threads():
    """Host threads this job may use: the box's CPU share (OMP_NUM_THREADS is
    set to it on the GPU box), else the affinity mask, capped at 16."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:
        return 1


def cpu_baseline(nx, ny, iters, re, budget_s, state, threads=1, max_steps=5):
    """The oracle (scalar/auto-vectorised C restatement) on the same workload,
    started from the GPU model's final state (so it sweeps the same developed,
    mostly non-zero fields, subnormals included, as the reference would).
    threads=1 is the reference's single worker thread (model.rs:1287);
    threads>1 splits the row loops over OpenMP threads, bit-identical results
    (oracle/cfd_oracle.h orc_set_threads).  SURVEY.md §8(d): median of the
    per-step times of up to max_steps steps (stopping early only when the
    budget runs out) after 1 warm-up step."""
    m, orc = oracle_from_state(nx, ny, iters, re, state, threads)
    m.update()   # untimed warm-up step: touches every page
    times, t_start = [], time.perf_counter()
    while True:
        t0 = time.perf_counter()
        m.update()
        times.append(time.perf_counter() - t0)
        if time.perf_counter() - t_start >= budget_s or len(times) >= max_steps:
            break
    orc.set_threads(1)
    model, ncpu = cpu_info()
    med = sorted(times)[len(times) // 2]
    return {"value": nx * ny * iters / med, "unit": "cell-updates/s", "cores": threads,
            "kind": "port",
            "sample": f"median of {len(times)} full update() step(s) of the same {nx}x{ny} cavity "
                      f"({iters} sweeps/step) from the GPU run's final state (step "
                      f"{state['simulation_step']}) after 1 warm-up step, oracle/cfd_oracle.c, "
                      f"{threads} thread(s)"
                      + (" (the reference's single worker thread)" if threads == 1 else
                         " (OpenMP row split, same bits)")
                      + f"; ms/step median {1e3 * med:.0f} (min {1e3 * min(times):.0f}, max "
                        f"{1e3 * max(times):.0f}); host {model}, {ncpu} cpus"}


def oracle_from_state(nx, ny, iters, re, state, threads, scheme=0, passes=0, tol=0, grid=None,
                      params=None):
    """The oracle at `state`: the nx x ny cavity (Re, iters, scheme, passes,
    tol), or `grid` / `params` (cfdamd Grid / SimulationParams) when given."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    from oracle import OracleModel
    orc.set_threads(threads)
    if grid is not None:
        c = grid.obstacle
        p = params
        m = OracleModel(grid.nx, grid.ny, grid.lx, grid.ly,
                        cylinder=(c.center_x, c.center_y, c.radius) if c else None,
                        dt=p.dt, viscosity=p.viscosity, target_inlet_velocity=p.target_inlet_velocity,
                        scheme=int(p.velocity_scheme), inlet_profile=int(p.inlet_profile),
                        jacobi_iters=p.jacobi_iters, corrector_passes=p.corrector_passes,
                        tol_enabled=int(p.tol_enabled), p_tol=p.p_tol, bc_kind=int(p.bc_kind),
                        pressure_solver=int(p.pressure_solver))
    else:
        m = OracleModel(nx, ny, float(nx) / float(ny), 1.0, bc_kind=1, viscosity=1.0 / re,
                        jacobi_iters=iters, corrector_passes=passes, tol_enabled=tol, scheme=scheme)
    for k in ("u", "v", "p", "u_star", "v_star", "p_prime", "rhs"):
        m.field(k)[:] = state[k]
    sc = m.scalars()
    sc.step, sc.time, sc.dt = state["simulation_step"], state["simulation_time"], state["dt"]
    sc.jacobi_sweeps_total = state["jacobi_sweeps_total"]
    m.set_scalars(sc)
    return m, orc


def parity_developed_step(model, nx, ny, iters, re, state, threads, **mode):
    """One GPU step and one oracle step from the same developed state; True
    when every field word and every scalar agree."""
    import numpy as np
    o, orc = oracle_from_state(nx, ny, iters, re, state, threads, **mode)
    model.update()
    o.update()
    orc.set_threads(1)
    g = model.get_state()
    bad = [k for k in ("u", "v", "p", "u_star", "v_star", "p_prime", "rhs")
           if not np.array_equal(g[k].view(np.uint32), o.field(k).view(np.uint32))]
    s = o.scalars()
    for k, want in (("dt", s.dt), ("last_p_residual", s.p), ("last_u_residual", s.u),
                    ("last_v_residual", s.v), ("simulation_time", s.time)):
        if np.float32(g[k]).view(np.uint32) != np.float32(want).view(np.uint32):
            bad.append(k)
    if int(g["jacobi_sweeps_total"]) != int(s.jacobi_sweeps_total):
        bad.append("jacobi_sweeps_total")
    return not bad, bad


def reference_default_leg(args, cfdamd, device, develop=200, steps=20, cpu_steps=3):
    """The reference's own design point: default_grid() -- the 800 x 264
    channel with the cylinder, lx 30, ly 10 (src/app.rs:33-53) -- under the
    default SimulationParams (model.rs:44-55: dt 0.005, nu 1e-6, <= 50 sweeps
    per solve with the 1e-4 early exit, <= 20 corrector passes,
    model.rs:696-724, 748-819), FirstOrder and SecondOrder.  Developed from
    rest for `develop` untimed steps, then `steps` timed; the kernel names the
    solve runs (its spacings are not powers of two: the IEEE or FMA-corrected
    division forms), one step bitwise against the oracle from the developed
    state, and the oracle's 1-thread ms/step on the same state beside it."""
    out = {"workload": "default_grid() 800x264 channel, cylinder r 0.75 at (7.5, 5), lx 30, ly 10 "
                       "(app.rs:33-53); SimulationParams::default() (model.rs:44-55): <=50 "
                       "sweeps/solve, early exit 1e-4, <=20 corrector passes",
           "developed": f"{develop} steps from rest"}
    for scheme in (cfdamd.VelocityScheme.FirstOrder, cfdamd.VelocityScheme.SecondOrder):
        grid = cfdamd.default_grid()
        params = cfdamd.SimulationParams(velocity_scheme=scheme)
        m = cfdamd.Model(grid, params, device=device)
        m.update_n(develop)
        m.synchronize()
        s0 = m.get_residuals().jacobi_sweeps_total
        t0 = time.perf_counter()
        m.update_n(steps)
        m.synchronize()
        el = time.perf_counter() - t0
        sweeps = m.get_residuals().jacobi_sweeps_total - s0
        kc = m.kernel_config
        kname = m.jacobi_kernel["name"]
        division = ["IEEE", "reciprocal multiply (proven exact, 2^32 inputs)",
                    "FMA-corrected (proven exact, 2^32 inputs)"][kc["fastdiv"]]
        if kname == "k_jacobi_resident<3>":   # the resident solve's guarded form
            division = "FMA-corrected for |x| >= 2^-96, IEEE below (proven exact, 2^32 inputs)"
        e = {"steps": steps, "ms_per_step": 1e3 * el / steps, "sweeps_per_step": sweeps / steps,
             "cell_updates_per_s": grid.nx * grid.ny * sweeps / el,
             "kernel": kname, "division": division}
        state = m.get_state()
        if not args.no_parity:
            o, orc = oracle_from_state(0, 0, 0, 0, state, cpu_threads(), grid=grid, params=params)
            m.update()
            o.update()
            orc.set_threads(1)
            g = m.get_state()
            import numpy as np
            bad = [k for k in ("u", "v", "p", "u_star", "v_star", "p_prime", "rhs")
                   if not np.array_equal(g[k].view(np.uint32), o.field(k).view(np.uint32))]
            sc = o.scalars()
            if int(g["jacobi_sweeps_total"]) != int(sc.jacobi_sweeps_total):
                bad.append("jacobi_sweeps_total")
            for k, want in (("dt", sc.dt), ("last_p_residual", sc.p), ("simulation_time", sc.time)):
                if np.float32(g[k]).view(np.uint32) != np.float32(want).view(np.uint32):
                    bad.append(k)
            e["parity_developed_step"] = not bad
            if bad:
                e["parity_differ"] = bad
        m.close()
        if not args.no_cpu_baseline:
            o, orc = oracle_from_state(0, 0, 0, 0, state, 1, grid=grid, params=params)
            ts = []
            for _ in range(cpu_steps):
                t0 = time.perf_counter()
                o.update()
                ts.append(time.perf_counter() - t0)
            med = sorted(ts)[len(ts) // 2]
            e["cpu_oracle_1thread_ms_per_step"] = 1e3 * med
            e["gpu_over_cpu"] = med / (el / steps)
        out[scheme.name] = e
    return out


def phase_window(model, steps):
    """Per-phase device time of `steps` more steps (a separate window after
    the timed one: the extra event records would perturb the headline)."""
    model.synchronize()
    model.timing_phases(True)
    model.timing_begin()
    model.update_n(steps)
    tm = model.timing_end()
    ph = model.timing_phase_ms()
    model.timing_phases(False)
    k = max(tm["steps"], 1)
    return {"steps": k, "predict_march_us": 1e3 * ph["predict_ms"] / k,
            "correct_finish_us": 1e3 * ph["finish_ms"] / k,
            "solve_us": 1e3 * tm["solve_ms"] / k, "step_us_events": 1e3 * tm["step_ms"] / k}


def so_leg(args, cfdamd, device, nx, ny, steps=10):
    """The same timed-mode step with second-order upwind advection
    (VelocityScheme::SecondOrder, model.rs:910-1053, 1097-1248): developed
    like the headline run, timed, per-phase times, and one step bitwise
    against the oracle from the developed state."""
    params = cfdamd.SimulationParams.cavity(
        args.re, args.iters, corrector_passes=0, tol_enabled=False,
        velocity_scheme=cfdamd.VelocityScheme.SecondOrder)
    model = cfdamd.Model(cfdamd.cavity_grid(nx, ny), params, device=device)
    model.update_n(args.develop + args.warmup)
    model.synchronize()
    t0 = time.perf_counter()
    model.update_n(steps)
    model.synchronize()
    el = time.perf_counter() - t0
    out = {"workload": f"{nx}x{ny} cavity Re={args.re:g}, SecondOrder upwind, {args.iters} "
                       f"sweeps/step, tolerance off, developed {args.develop} steps",
           "steps": steps, "ms_per_step": 1e3 * el / steps,
           "value": nx * ny * args.iters * steps / el, "unit": "cell-updates/s",
           "phases": phase_window(model, 5)}
    if not args.no_parity:
        state = model.get_state()
        ok, bad = parity_developed_step(model, nx, ny, args.iters, args.re, state, cpu_threads(),
                                        scheme=1)
        out["parity_developed_step"] = ok
        if not ok:
            out["parity_differ"] = bad
    model.close()
    return out


def parity_mode_leg(args, cfdamd, device, n, re, fixed_iters, steps=5):
    """The reference's own control flow (model.rs:696-724, 748-819): 50-sweep
    solves with the 1e-4 early exit and up to 20 re-correction passes.  The
    cavity is developed in the fixed-count mode (args.develop steps), its state
    injected into a model with the reference's parameters, then 2 warm-up and
    `steps` timed steps; sweeps/step counts the sweeps the reference's loop
    runs (early exits included).  One more step is compared bitwise with the
    oracle in the same mode."""
    grid = cfdamd.cavity_grid(n)
    dev = cfdamd.Model(grid, cfdamd.SimulationParams.cavity(
        re, fixed_iters, corrector_passes=0, tol_enabled=False), device=device)
    dev.update_n(args.develop)
    st = dev.get_state()
    dev.close()
    ref = cfdamd.SimulationParams.cavity(re, 50)   # jacobi 50, passes 20, tol 1e-4
    m = cfdamd.Model(grid, ref, device=device)
    m.set_state(**st)
    m.update_n(2)
    s0 = m.get_residuals().jacobi_sweeps_total
    m.synchronize()
    t0 = time.perf_counter()
    m.update_n(steps)
    m.synchronize()
    el = time.perf_counter() - t0
    sweeps = m.get_residuals().jacobi_sweeps_total - s0
    out = {"workload": f"{n}x{n} cavity Re={re:g}, reference control flow: <=50 sweeps/solve, "
                       f"early exit at 1e-4, <=20 corrector passes (model.rs:696-724, 748-819)",
           "developed": f"{args.develop} fixed-count steps ({fixed_iters} sweeps), state injected",
           "kernel": m.jacobi_kernel["name"],
           "steps": steps, "ms_per_step": 1e3 * el / steps, "sweeps_per_step": sweeps / steps,
           "cell_updates_per_s": n * n * sweeps / el,
           "us_per_sweep": 1e6 * el / max(sweeps, 1)}
    if not args.no_parity:
        state = m.get_state()
        ok, bad = parity_developed_step(m, n, n, 50, re, state, cpu_threads(), passes=20, tol=1)
        out["parity_developed_step"] = ok
        if not ok:
            out["parity_differ"] = bad
    m.close()
    return out


STATE_KEYS = ("u", "v", "p", "u_star", "v_star", "p_prime", "rhs")
SCALAR_KEYS = ("dt", "simulation_time", "simulation_step", "last_p_residual", "last_u_residual",
               "last_v_residual", "jacobi_sweeps_total")


def parity_sharded_step(model, dist, rank, world, grid, params, device):
    """N > 1: one more step on the slabs, checked against the same step of a
    single-domain GPU model of the whole grid started from the gathered slab
    state (rank 0; 16384 x 8192 fits one MI355X).  The single domain is
    itself bitwise against the oracle (parity_developed_step at N = 1, the
    test suite), so a True here carries the oracle's parity to the N-GPU run
    that was just timed: every word of u, v, p, u*, v*, p', rhs and every
    scalar of every rank.  Collective: every rank calls it."""
    import numpy as np
    import cfdamd
    pre = model.get_state()
    model.update()
    post = model.get_state()
    mine = (model.j0, model.j1, {k: pre[k] for k in STATE_KEYS}, {k: post[k] for k in STATE_KEYS},
            {k: pre[k] for k in SCALAR_KEYS}, {k: post[k] for k in SCALAR_KEYS})
    del pre, post
    objs = [None] * world if rank == 0 else None
    dist.gather_object(mine, objs, dst=0)
    del mine
    if rank != 0:
        return None
    t0 = time.perf_counter()
    try:
        g_pre = cfdamd.assemble_slabs([(o[0], o[1], o[2]) for o in objs], grid.nx)
        g_post = cfdamd.assemble_slabs([(o[0], o[1], o[3]) for o in objs], grid.nx)
    except ValueError as e:   # a shared v face row differs between two slabs
        return {"ok": False, "differ": [str(e)]}
    sc_pre, sc_post = objs[0][4], [o[5] for o in objs]
    del objs
    ref = cfdamd.Model(grid, params, device=device)
    try:
        ref.set_state(**g_pre, **sc_pre)
        del g_pre
        ref.update()
        r = ref.get_state()
    finally:
        ref.close()
    bad = [k for k in STATE_KEYS if not np.array_equal(r[k].view(np.uint32), g_post[k].view(np.uint32))]

    def same(a, b):
        return (np.float32(a).view(np.uint32) == np.float32(b).view(np.uint32)
                if isinstance(a, (float, np.floating)) else int(a) == int(b))
    for rk, sp in enumerate(sc_post):
        bad += [f"{k} (rank {rk})" for k in SCALAR_KEYS if not same(sp[k], r[k])]
    return {"ok": not bad, "differ": bad,
            "detail": f"1 step from step {int(sc_pre['simulation_step'])} on the {world} slabs vs "
                      f"a single-domain {grid.nx}x{grid.ny} model on device {device} from the "
                      f"gathered slab state: every word of u, v, p, u*, v*, p', rhs and the "
                      f"scalars of every rank compared ({time.perf_counter() - t0:.1f} s)"}


def time_jacobi(model, steps):
    """Average Jacobi launch time (ms) over `steps` timed-mode steps: HIP events
    on the model's stream around each step's launch sequence."""
    model.synchronize()
    model.timing_begin()
    model.update_n(steps)
    tm = model.timing_end()
    launches = max(steps * model.launches_per_solve(), 1)
    return tm, tm["solve_ms"] / launches


def block_kernel(model):
    """The solve's dominant kernel as rocprofv3 names it, and the T-sweep
    blocks one dispatch of it runs: the persistent launch (k_jacobi_persist,
    all blocks but the last) when the model's last solve used it, else the
    one-block launch.  PMC figures per dispatch are divided by the blocks."""
    nb = model.persist_blocks
    if nb > 0:
        return f"k_jacobi_persist<8, {model.kernel_config['fastdiv']}>", nb
    return model.jacobi_kernel["name"], 1


def roofline_entry(model, nx, nyl, launch_ms, bench_kernel_note=None):
    kname, nblk = block_kernel(model)
    T = model.kernel_config["temporal"]
    cells = nx * nyl
    one_pass = BYTES_PER_CELL_UPDATE * cells
    achieved = one_pass / (launch_ms * 1e-3) / 1e9 if launch_ms > 0 else 0.0
    traffic, traffic_src, pmc_blocks = pmc_traffic(kname, f"{nx}x{nyl}")
    if traffic:
        traffic /= pmc_blocks or nblk   # per 8-sweep block of the profiled dispatch
    meas = traffic / (launch_ms * 1e-3) / 1e9 if traffic and launch_ms > 0 else None
    return {
        "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
        "measured_hbm_GBps": meas,
        "measured_hbm_frac": meas / HBM_PEAK_GBS if meas else None,
        "kernel": kname, "blocks_per_dispatch": nblk, "slab": [nx, nyl], "sweeps_per_launch": T,
        "avg_launch_us": launch_ms * 1e3,
        "us_per_sweep": launch_ms * 1e3 / T,
        "jacobi_cell_updates_per_s": cells * T / (launch_ms * 1e-3) if launch_ms > 0 else 0.0,
        "bytes_per_launch": one_pass,
        "algorithmic_sweep_equiv": {
            "GBps": achieved * T, "frac": achieved * T / HBM_PEAK_GBS,
            "note": "12 B per cell-update x T sweeps per launch: the single-sweep figure "
                    "the launch's on-chip temporal blocking replaces"},
        "timing": "HIP events on the model stream around each step's Jacobi launch sequence "
                  "/ T-sweep blocks (includes inter-launch gaps; with the persistent launch a "
                  "'launch' is one of its blocks)",
        "note": "achieved = one-pass bytes (read p', read rhs, write p' once per launch) / "
                "launch time; traffic = PMC bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, "
                "gfx950 correction); FETCH_SIZE counts Infinity-Cache hits too "
                "(MI355X_MICROARCH.md HBM section), so on MALL-resident slabs it is fabric, "
                "not HBM, traffic",
    }


VALU_ISSUE_PEAK = 1024 * 2.4e9 / 4   # wave64 VALU instructions/s: 256 CUs x 4 SIMDs, one per 4 cycles at 2.4 GHz


def roofline_valu(kernel, slab, launch_ms, blocks=1):
    """The Jacobi launch's binding resource on a MALL-resident slab is VALU
    issue: SQ_INSTS_VALU per launch from the newest committed
    PMC pass on this slab (tools/pmc_valu.py) over the measured launch time,
    against the chip's wave64 VALU issue rate at the 2.4 GHz max clock."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_valu*.json")), reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        k = d.get("kernels", {}).get(kernel)
        if k and d.get("workload") == slab and k.get("SQ_INSTS_VALU") and launch_ms > 0:
            blocks = k.get("blocks_per_dispatch") or blocks   # the profiled run's own count
            rate = k["SQ_INSTS_VALU"] / blocks / (launch_ms * 1e-3)
            return {"bound": "valu", "achieved": rate / 1e9, "peak": VALU_ISSUE_PEAK / 1e9,
                    "unit": "G wave64-VALU-instructions/s", "frac": rate / VALU_ISSUE_PEAK,
                    "valu_insts_per_launch": k["SQ_INSTS_VALU"] / blocks,
                    "source": os.path.relpath(path, ROOT),
                    "note": "SQ_INSTS_VALU (PMC, same kernel and slab) / launch time; peak = 1024 "
                            "SIMDs x 1 wave64 instruction per 4 cycles x 2.4 GHz (the chip holds "
                            "a lower clock under load, so frac is conservative)"}
    return None


def pmc_traffic(kernel, slab):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/*/pmc_traffic.json, tools/pmc_traffic.py: 2 x FETCH_SIZE +
    WRITE_SIZE per the gfx950 correction) measured on this slab shape."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_traffic*.json")),
                       reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        k = d.get("kernels", {}).get(kernel)
        if k and d.get("workload") == slab:
            return k["traffic_bytes"], os.path.relpath(path, ROOT), k.get("blocks_per_dispatch")
    return None, None, None


def control_run(args, cfdamd, device, n=8192, steps=10):
    """The same timed-mode step on an 8192^2 cavity (one GPU): the Jacobi
    working set (2 p' + rhs = 768 MB) is 3x the Infinity Cache, so its
    launches stream from HBM; developed for args.develop steps like the main run."""
    model = cfdamd.Model(cfdamd.cavity_grid(n), cfdamd.SimulationParams.cavity(
        args.re, args.iters, corrector_passes=0, tol_enabled=False), device=device)
    model.update_n(args.develop)
    model.update_n(2)
    tm, launch_ms = time_jacobi(model, steps)
    e = roofline_entry(model, n, n, launch_ms)
    e["workload"] = (f"{n}x{n} cavity Re={args.re:g}, {args.iters} sweeps/step, developed "
                     f"{args.develop} steps, {steps} timed steps; Jacobi working set "
                     f"{3 * n * n * 4 / 2**20:.0f} MiB > 256 MiB Infinity Cache")
    e["ms_per_step"] = tm["step_ms"] / max(tm["steps"], 1)
    model.close()
    return e


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n, timeout_s):
    """`--gpus N` without an external launcher: run N copies of this script,
    one rank per GPU, and relay rank 0's JSON line.  The parent never loads
    the HIP library or torch's GPU runtime (children are separate processes,
    never exec'd from a process that touched the GPU).  A rank that fails
    ends the job: the others are terminated and the exit status is non-zero."""
    import threading
    port = free_port()
    procs, lines = [], []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   CFD_BENCH_LAUNCHER="bench.py")
        procs.append(subprocess.Popen(
            [sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
            stdout=subprocess.PIPE if r == 0 else sys.stderr, text=True))

    def relay():
        for line in procs[0].stdout:
            lines.append(line)
            sys.stdout.write(line)
            sys.stdout.flush()
    th = threading.Thread(target=relay, daemon=True)
    th.start()
    t_end = time.monotonic() + timeout_s
    rcs = [None] * n
    failed = None
    while any(rc is None for rc in rcs):
        for r, p in enumerate(procs):
            if rcs[r] is None:
                rcs[r] = p.poll()
                if rcs[r] not in (None, 0) and failed is None:
                    failed = r
        if failed is not None or time.monotonic() > t_end:
            break
        time.sleep(0.2)
    if failed is not None or any(rc is None for rc in rcs):
        why = (f"rank {failed} exited with status {rcs[failed]}" if failed is not None
               else f"ranks still running after {timeout_s:.0f} s")
        print(f"bench.py launcher: {why}; terminating the other ranks", file=sys.stderr,
              flush=True)
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        th.join(timeout=5)
        raise SystemExit(1)
    th.join(timeout=30)
    if not any(l.lstrip().startswith("{") for l in lines):
        print("bench.py launcher: rank 0 printed no JSON line", file=sys.stderr, flush=True)
        raise SystemExit(1)
    raise SystemExit(max(rcs))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    # 400 steps from rest: the fields are developed (97 % of p' non-zero, vs
    # 4 % at step 20), so the timed steps sweep representative data
    ap.add_argument("--warmup", type=int, default=5)
    # untimed steps from rest before the warm-up, whatever --warmup is: the
    # timed steps then sweep developed fields (97 % of p' non-zero at 400)
    ap.add_argument("--develop", type=int, default=400)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--re", type=float, default=1000.0)
    ap.add_argument("--nx", type=int, default=0)
    ap.add_argument("--ny", type=int, default=0)
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--clock-warmup", type=float, default=0.0,
                    help="seconds of steps on a scratch model before the measured one is "
                         "created, so the GPU clocks have left their idle state")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-control", action="store_true",
                    help="skip the 8192^2 (non-MALL-resident) roofline control at N=1")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-so", action="store_true",
                    help="skip the second-order upwind leg at N=1")
    ap.add_argument("--no-parity-mode", action="store_true",
                    help="skip the reference-control-flow legs (C2, C3) at N=1")
    ap.add_argument("--no-reference-default", action="store_true",
                    help="skip the reference's default_grid() channel leg at N=1")
    ap.add_argument("--launch-timeout", type=float, default=1800.0,
                    help="seconds the self-launched ranks of --gpus N may take")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher and rank plumbing only (gloo, no GPU, no HIP library): "
                         "prints a line with dry_run true and no measurement")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        launch_ranks(args.gpus, args.launch_timeout)   # does not return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("CFD_BENCH_LOOPBACK") == "1" and world > 1:
        # rehearsal of the N-GPU run on a one-GPU box (tools/rccl_loopback.py's
        # trick): every rank on device 0, each its own RCCL "host" so RCCL
        # connects them through its socket transport; set before RCCL loads
        os.environ["NCCL_HOSTID"] = f"cfd-bench-rank{rank}"
        # persistent solves stay on: the ticketed launch completes with the
        # ranks' kernels sharing the GPU (the exact SCALE configuration)
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
        os.environ.setdefault("NCCL_NET", "Socket")
        local = 0
    n = max(world, 1)
    if args.gpus != n:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")

    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
    launcher = os.environ.get("CFD_BENCH_LAUNCHER", "external" if world > 1 else "none")
    if args.dry_run:
        ranks = dist.get_world_size() if dist is not None else 1
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": None, "unit": "cell-updates/s",
                              "n_gpus": n, "ranks_seen": ranks, "launcher": launcher,
                              "dry_run": True}), flush=True)
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return
    import cfdamd
    if world > 1 and os.environ.get("CFD_BENCH_LOOPBACK") != "1":
        ndev = cfdamd.device_count()
        if ndev < world or local >= ndev:
            print(f"bench.py rank {rank}: --gpus {world} needs {world} GPUs, this process sees "
                  f"{ndev}", file=sys.stderr, flush=True)
            raise SystemExit(3)

    nx, ny = global_grid(n)
    if args.nx:
        nx = args.nx
    if args.ny:
        ny = args.ny
    grid = cfdamd.cavity_grid(nx, ny)
    params = cfdamd.SimulationParams.cavity(args.re, args.iters, corrector_passes=0,
                                            tol_enabled=False)
    uid = None
    if world > 1:
        obj = [cfdamd.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        uid = obj[0]
    if args.clock_warmup > 0 and world == 1:
        scratch = cfdamd.Model(grid, params, device=local)
        t_end = time.perf_counter() + args.clock_warmup
        while time.perf_counter() < t_end:
            scratch.update_n(4)
            scratch.synchronize()
        scratch.close()
        del scratch
    model = cfdamd.Model(grid, params, device=local, n_ranks=n, rank=rank, unique_id=uid)

    def barrier():
        model.synchronize()
        if dist is not None:
            dist.barrier()

    model.update_n(args.develop + args.warmup)
    barrier()
    model.timing_begin()
    t0 = time.perf_counter()
    model.update_n(args.steps)
    model.synchronize()
    t1 = time.perf_counter()
    barrier()
    tm = model.timing_end()
    elapsed = t1 - t0
    rank_elapsed = [elapsed]
    if dist is not None:
        gathered = [None] * world
        dist.all_gather_object(gathered, elapsed)
        rank_elapsed = [float(x) for x in gathered]
        elapsed = max(rank_elapsed)
    ranks_seen = model.comm_size

    import numpy as np
    try:
        res = model.get_residuals()
    except cfdamd.CfdError as e:   # CFD_ENONFINITE: reported, not hidden
        if e.code != cfdamd.CFD_ENONFINITE:
            raise
        res = None
    state = model.get_state()   # this rank's slab
    finite = bool(np.isfinite(state["u"]).all() and np.isfinite(state["v"]).all())
    nonzero = float(np.count_nonzero(state["p_prime"])) / max(state["p_prime"].size, 1)
    subn = int(((np.abs(state["p_prime"]) > 0) &
                (np.abs(state["p_prime"]) < np.finfo(np.float32).tiny)).sum())

    kcfg = model.kernel_config
    kern = model.jacobi_kernel
    T = kcfg["temporal"]
    launches = max(args.steps * model.launches_per_solve(), 1)
    launch_ms = tm["solve_ms"] / launches
    roof = roofline_entry(model, nx, model.nyl, launch_ms)
    kname, nblk = block_kernel(model)
    roof_valu = roofline_valu(kname, f"{nx}x{model.nyl}", launch_ms, nblk)
    geometry = model.jacobi_geometry(persist=nblk > 1)
    multi = {}
    if n > 1:
        # collective legs, after the timed steps (every rank takes part):
        # per-rank phase and RCCL exchange times, then the sharded parity step
        ph = phase_window(model, 5)
        ex = model.timing_exchange_ms()
        mine = {"rank": rank, "predict_march_us": ph["predict_march_us"],
                "correct_finish_us": ph["correct_finish_us"], "solve_us": ph["solve_us"],
                "step_us_events": ph["step_us_events"],
                "exchange_us_per_step": 1e3 * ex["exchange_ms"] / ph["steps"],
                "exchanges_per_step": ex["exchanges"] / ph["steps"], "geometry": geometry}
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
        multi["rank_phases"] = gathered
        if not args.no_parity:
            multi["parity_sharded_step"] = parity_sharded_step(model, dist, rank, world, grid,
                                                               params, local)
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": nx * ny * args.iters * args.steps / elapsed,
            "unit": "cell-updates/s",
            "n_gpus": n,
            "ranks_seen": ranks_seen,
            "launcher": launcher,
            "rank_ms_per_step": [1e3 * e / args.steps for e in rank_elapsed],
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic (lid-driven cavity from rest, build-defined BCs, SURVEY.md §8(d); "
                    f"{args.develop} untimed developing steps + {args.warmup} warm-up, timed "
                    f"steps {args.develop + args.warmup}..{args.develop + args.warmup + args.steps}"
                    f" on the developed fields: {100 * nonzero:.1f}% of p' non-zero, "
                    f"{subn} subnormal)",
            "config": {
                "workload": f"{nx}x{ny} lid-driven cavity Re={args.re:g}, first-order upwind "
                            f"advection (VelocityScheme::FirstOrder), {args.iters} Jacobi "
                            "sweeps/step, tolerance off, 0 extra corrector passes",
                "velocity_scheme": "FirstOrder",
                "grid": [nx, ny], "slab_per_gpu": [nx, model.nyl], "jacobi_iters": args.iters,
                "parallelism": f"row-slab x{n}" + (f", halo depth {model.halo_depth}" if n > 1 else ""),
                "kernel": (f"{kname} ({nblk} blocks of {T} sweeps in one persistent launch"
                           + (", the residual block included)" if nblk >= model.launches_per_solve()
                              else f") + {kern['name']} launches for the rest") if nblk > 1 else
                           f"{kern['name']} ({T} sweep(s)/launch, kind {kern['kind']})"),
                "division": ["IEEE", "reciprocal multiply (proven exact, 2^32 inputs)",
                             "FMA-corrected (proven exact, 2^32 inputs)"][kcfg["fastdiv"]],
            },
            "roofline": roof,
            "roofline_valu": roof_valu,
            "jacobi_geometry": geometry,
            "solve_fraction_of_step": tm["solve_ms"] / tm["step_ms"] if tm["step_ms"] else None,
            # a timed-mode step moves 2,498 B per pressure cell
            # when every pass streams its fields (P = 1 solve, K = 200 sweeps);
            # that byte count over the measured step time, against the HBM peak
            # (above 1 = on-chip temporal blocking, not a roofline fraction)
            "step_algorithmic": {
                "bytes_per_cell": 16 + 26 + 12 + 28 + 12 * args.iters + 16,
                "GBps": (16 + 26 + 12 + 28 + 12 * args.iters + 16) * nx * ny /
                        (elapsed / args.steps) / 1e9,
                "x_hbm_peak": (16 + 26 + 12 + 28 + 12 * args.iters + 16) * nx * ny /
                              (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS},
            "final_step": int(state["simulation_step"]), "final_dt": float(state["dt"]),
            "fields_finite": finite and res is not None,
        }
        if n > 1:
            out["rank_phases"] = multi["rank_phases"]
            ps = multi.get("parity_sharded_step")
            if ps is not None:
                out["parity_sharded_step"] = ps["ok"]
                out["parity_sharded_step_detail"] = ps.get("detail", "") + (
                    "" if ps["ok"] else f"; differ: {ps['differ']}")
        if n == 1 and not args.no_parity and out["fields_finite"]:
            ok, bad = parity_developed_step(model, nx, ny, args.iters, args.re, state,
                                            cpu_threads())
            out["parity_developed_step"] = ok
            out["parity_developed_step_detail"] = (
                f"1 step from step {state['simulation_step']} on GPU and oracle "
                f"(oracle/cfd_oracle.c), every word of u, v, p, u*, v*, p', rhs and the "
                f"scalars compared" + ("" if ok else f"; differ: {bad}"))
        if n == 1:
            out["phases"] = phase_window(model, 5)
        if n == 1 and not args.no_so:
            out["so_step"] = so_leg(args, cfdamd, local, nx, ny)
        if n == 1 and not args.no_parity_mode:
            out["parity_mode"] = {
                "C2": parity_mode_leg(args, cfdamd, local, 1024, 400.0, 100),
                "C3": parity_mode_leg(args, cfdamd, local, 4096, 1000.0, 200)}
        if n == 1 and not args.no_control:
            out["roofline_control"] = control_run(args, cfdamd, local)
        if n == 1 and not args.no_reference_default:
            out["reference_default"] = reference_default_leg(args, cfdamd, local)
        if n == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(nx, ny, args.iters, args.re, args.cpu_budget, state)
            nt = cpu_threads()
            if nt > 1:
                # the same restatement over all of this job's host cores
                out["cpu_baseline_multicore"] = cpu_baseline(
                    nx, ny, args.iters, args.re, args.cpu_budget / 2, state, threads=nt,
                    max_steps=9)
        # ONE write for the whole line: other ranks share this stdout under an
        # external launcher, and a line split over several writes can be cut
        sys.stdout.flush()
        data = (json.dumps(out) + "\n").encode()
        while data:
            data = data[os.write(1, data):]
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    model.close()


if __name__ == "__main__":
    main()
