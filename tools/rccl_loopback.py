#!/usr/bin/env python3
"""Execute the RCCL transport of cfd_create_sharded on a ONE-GPU box.

RCCL refuses two ranks of one communicator on one device ("Duplicate GPU
detected") when it sees them on one host.  Each rank here gets its own
NCCL_HOSTID, so RCCL takes them for two hosts and connects them through its
socket network transport over the loopback interface (no xGMI, host-staged
copies): slow, but every ncclSend / ncclRecv / ncclAllReduce the sharded model
issues runs for real, with the row offsets, group pairing and slab heights of
the production path.  Both slabs run on device 0; the gathered result is
compared bit for bit with a single-domain model of the same grid.

    python tools/rccl_loopback.py [--n 2] [--nx 256 --ny 200] [--steps 4]

Diagnostic for the multi-GPU path (the 8-GPU run belongs to the driver).
"""
import argparse
import os
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import jsonl  # noqa: E402


def result(args, rank, obj):
    """A rank's verdict goes to its own file; the launcher prints the merged
    records from one process after every rank has exited (r4: two ranks'
    prints into one inherited pipe interleaved)."""
    jsonl.append_record(os.path.join(args.result_dir, f"rank{rank}.jsonl"), obj)


def selftest(args, rank):
    """CPU guard for the output path (tests/test_bench_helpers.py): each rank
    emits --lines records straight to the shared stdout through jsonl.emit and
    the same number through its result file."""
    for i in range(args.lines):
        rec = {"rank": rank, "i": i, "via": "stdout", "pad": "x" * (64 + 37 * (i % 7))}
        jsonl.emit(rec)
        result(args, rank, dict(rec, via="file"))


def worker(args):
    rank, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if args.mode == "selftest":
        selftest(args, rank)
        return
    # before the RCCL library initialises: one "host" per rank, sockets on lo
    os.environ["NCCL_HOSTID"] = f"cfd-loopback-rank{rank}"
    # the ranks share one GPU
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    os.environ.setdefault("NCCL_NET", "Socket")
    os.environ.setdefault("CFD_RCCL_TIMEOUT_S", "60")
    sys.path.insert(0, os.path.join(ROOT, "cfd-demo_amd"))
    import numpy as np
    import torch.distributed as dist
    import cfdamd
    dist.init_process_group("gloo", rank=rank, world_size=n)
    cases = []
    if args.mode in ("fixed", "both"):
        cases.append(("cavity fixed-count (deep halos, overlapped exchange)",
                      cfdamd.cavity_grid(args.nx, args.ny),
                      cfdamd.SimulationParams.cavity(1000.0, 64, corrector_passes=0, tol_enabled=False)))
    if args.mode in ("tol", "both"):
        cases.append(("channel with cylinder, reference tolerance mode (lagged convergence)",
                      cfdamd.Grid(args.nx, args.ny, 30.0, 10.0, cfdamd.Cylinder(7.5, 5.0, 1.5)),
                      cfdamd.SimulationParams()))
    if args.mode == "solvers":
        # the JS variant's solvers on slabs: SOR (2-row exchange every
        # iteration, all-reduced residuals) and multigrid (rhs all-gathered by
        # point-to-point sends, whole grid solved on every rank)
        for solver, label in ((cfdamd.PressureSolver.Sor, "SOR"),
                              (cfdamd.PressureSolver.Multigrid, "multigrid")):
            for tol in (False, True):
                cases.append((f"channel with cylinder, {label}, tolerance {'on' if tol else 'off'}",
                              cfdamd.Grid(args.nx, args.ny, 30.0, 10.0, cfdamd.Cylinder(7.5, 5.0, 1.5)),
                              cfdamd.SimulationParams(pressure_solver=solver, jacobi_iters=40,
                                                      corrector_passes=2, tol_enabled=tol)))
    if args.mode == "developed":
        developed(args, rank, n, cfdamd, dist, np)
        return
    if args.mode == "tolbench":
        tolbench(args, rank, n, cfdamd, dist, np)
        return
    report = []
    for name, grid, params in cases:
        if rank == 0:
            obj = [cfdamd.rccl_unique_id()]
        else:
            obj = [None]
        dist.broadcast_object_list(obj, src=0)
        t0 = time.perf_counter()
        m = cfdamd.Model(grid, params, device=0, n_ranks=n, rank=rank, unique_id=obj[0])
        for _ in range(args.steps):
            m.update()
        m.synchronize()
        el = time.perf_counter() - t0
        st = m.get_state()
        mine = {k: st[k] for k in ("u", "v", "p", "p_prime")}
        slab = (m.j0, m.j1)
        calls = m.comm_calls / max(1, args.steps)
        m.close()
        gathered = [None] * n
        dist.all_gather_object(gathered, (slab, mine, calls))
        if rank == 0:
            ref = cfdamd.Model(grid, params, device=0)
            for _ in range(args.steps):
                ref.update()
            want = ref.get_state()
            ref.close()
            nx = grid.nx
            ok = True
            for k in ("u", "v", "p", "p_prime"):
                parts = []
                for i, ((j0, j1), f, _) in enumerate(gathered):
                    if k == "v":
                        rows = f[k].reshape(j1 - j0 + 1, nx)
                        parts.append(rows if i == n - 1 else rows[:-1])
                    else:
                        parts.append(f[k])
                got = np.concatenate([np.ravel(x) for x in parts])
                same = np.array_equal(got.view(np.uint32), want[k].view(np.uint32))
                ok &= same
            report.append({"case": name, "ranks": n, "grid": [grid.nx, grid.ny],
                           "steps": args.steps, "bitwise_equal_single_domain": bool(ok),
                           "sharded_wall_s": round(el, 3),
                           "collective_calls_per_step_rank0": gathered[0][2]})
    if rank == 0:
        for r in report:
            result(args, rank, r)
        if not all(r["bitwise_equal_single_domain"] for r in report):
            sys.exit(1)
    dist.barrier()
    dist.destroy_process_group()


def slab_slices(st, nx, j0, j1):
    """Rows [j0, j1) of a single-domain state (v and v* with face row j1)."""
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


def perturb(st, np, seed=1234, amp=1e-3):
    """Add a seeded f32 perturbation of amplitude `amp` to the developed u, v,
    u*, v* and p' (the same bits on every rank).  The cavity develops from the
    lid down and p' underflows to exactly 0 far below it, so slab boundaries
    deep in the grid would otherwise carry zeros; this puts non-zero data in
    every row a halo exchange moves."""
    rng = np.random.default_rng(seed)
    for k in ("u", "v", "u_star", "v_star", "p_prime"):
        st[k] = (st[k] + (amp * rng.uniform(-1.0, 1.0, st[k].size)).astype(np.float32)).astype(
            np.float32)


def developed(args, rank, n, cfdamd, dist, np):
    """The bench's timed mode on a DEVELOPED cavity: every rank develops the
    single-domain model for --develop steps (deterministic, so every rank
    holds the same bits), perturbs it (perturb), injects its slab rows into the
    RCCL-sharded model
    (cfd_set_state exchanges the ghosts), and runs --steps steps; its rows
    must equal the single-domain continuation bit for bit.  The slab
    boundaries carry developed p' (the non-zero fraction of the rows either
    side of each boundary is reported)."""
    grid = cfdamd.cavity_grid(args.nx, args.ny)
    params = cfdamd.SimulationParams.cavity(1000.0, 200, corrector_passes=0, tol_enabled=False)
    nx = args.nx
    ref = cfdamd.Model(grid, params, device=0)
    ref.update_n(args.develop)
    st0 = ref.get_state()
    nz_dev = float(np.count_nonzero(st0["p_prime"])) / st0["p_prime"].size
    perturb(st0, np)
    ref.set_state(**st0)
    ref.update_n(args.steps)
    want = ref.get_state()
    ref.close()
    obj = [cfdamd.rccl_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    t0 = time.perf_counter()
    m = cfdamd.Model(grid, params, device=0, n_ranks=n, rank=rank, unique_id=obj[0])
    j0, j1 = m.j0, m.j1
    m.set_state(**slab_slices(st0, nx, j0, j1))
    m.update_n(args.steps)
    m.synchronize()
    el = time.perf_counter() - t0
    got = m.get_state()
    ranks_seen = m.comm_size
    persist_blocks = m.persist_blocks   # persistent blocks (0: per launch, the SCALE config)
    m.close()
    exp = slab_slices(want, nx, j0, j1)
    bad = [k for k in ("u", "v", "p", "p_prime", "u_star", "v_star", "rhs")
           if not np.array_equal(got[k].view(np.uint32), exp[k].view(np.uint32))]
    pp = st0["p_prime"].reshape(-1, nx)
    # the p' rows either side of this slab's internal boundaries
    rows = ([j0 - 1, j0] if j0 > 0 else []) + ([j1 - 1, j1] if j1 < args.ny else [])
    nzf = float(np.count_nonzero(pp[rows])) / max(len(rows) * nx, 1) if rows else None
    result(args, rank, {"case": "developed cavity, fixed-count (deep halos, overlapped exchange)",
                      "rank": rank, "ranks": n, "ranks_seen": ranks_seen,
                      "grid": [args.nx, args.ny], "slab": [j0, j1], "develop": args.develop,
                      "steps": args.steps, "boundary_rows": rows,
                      "boundary_pprime_nonzero_frac": nzf,
                      "developed_pprime_nonzero_frac": nz_dev,
                      "bitwise_equal_single_domain": not bad, "differ": bad,
                      "persist_blocks": persist_blocks,
                      "sharded_wall_s": round(el, 3)})
    dist.barrier()
    dist.destroy_process_group()
    if bad:
        sys.exit(1)


def tolbench(args, rank, n, cfdamd, dist, np):
    """The reference's design point in its own control flow on slabs: the
    default_grid() channel (800 x 264, cylinder, SimulationParams::default():
    <= 50 sweeps, early exit 1e-4, <= 20 corrector passes), --develop steps
    from rest untimed, then --steps steps timed: wall ms and collective calls
    per step, and the state after them bit for bit against the single-domain
    model.  Run once per solve schedule (CFD_SPEC_SLABS=0: the host-driven
    per-sweep loop; 1: the speculative blocks)."""
    grid = cfdamd.default_grid()
    params = cfdamd.SimulationParams()
    obj = [cfdamd.rccl_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    m = cfdamd.Model(grid, params, device=0, n_ranks=n, rank=rank, unique_id=obj[0])
    m.update_n(args.develop)
    m.synchronize()
    dist.barrier()
    c0 = m.comm_calls
    s0 = m.get_residuals().jacobi_sweeps_total
    t0 = time.perf_counter()
    m.update_n(args.steps)
    m.synchronize()
    el = time.perf_counter() - t0
    calls = (m.comm_calls - c0) / args.steps
    sweeps = (m.get_residuals().jacobi_sweeps_total - s0) / args.steps
    st = m.get_state()
    mine = (m.j0, m.j1, {k: st[k] for k in ("u", "p", "p_prime")})
    m.close()
    gathered = [None] * n
    dist.all_gather_object(gathered, (mine, el))
    if rank == 0:
        ref = cfdamd.Model(grid, params, device=0)
        ref.update_n(args.develop + args.steps)
        want = ref.get_state()
        ref.close()
        ok = all(np.array_equal(np.concatenate([g[0][2][k] for g in gathered]).view(np.uint32),
                                want[k].view(np.uint32)) for k in ("u", "p", "p_prime"))
        wall = max(g[1] for g in gathered)
        result(args, rank, {"case": "default_grid() channel, reference control flow",
                            "schedule": "speculative blocks" if os.environ.get("CFD_SPEC_SLABS") == "1"
                            else "host-driven per sweep",
                            "ranks": n, "develop": args.develop, "steps": args.steps,
                            "ms_per_step": 1e3 * wall / args.steps,
                            "collective_calls_per_step_rank0": calls,
                            "ms_per_collective_call": 1e3 * wall / args.steps / max(calls, 1e-9),
                            "sweeps_per_step": sweeps,
                            "bitwise_equal_single_domain": bool(ok)})
        if not ok:
            sys.exit(1)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2)
    ap.add_argument("--nx", type=int, default=256)
    ap.add_argument("--ny", type=int, default=200)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--mode", default="both",
                    choices=["fixed", "tol", "both", "solvers", "developed", "tolbench", "selftest"])
    ap.add_argument("--develop", type=int, default=400)
    ap.add_argument("--timeout", type=float, default=240.0)
    ap.add_argument("--lines", type=int, default=200)
    ap.add_argument("--result-dir", default=None)
    ap.add_argument("--worker", action="store_true")
    args = ap.parse_args()
    if args.worker:
        worker(args)
        return
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    rdir = tempfile.mkdtemp(prefix="cfd_rccl_loopback_")
    procs = []
    for r in range(args.n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(args.n), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), LOCAL_RANK="0")
        cmd = [sys.executable, os.path.abspath(__file__), "--worker", "--n", str(args.n),
               "--nx", str(args.nx), "--ny", str(args.ny), "--steps", str(args.steps),
               "--mode", args.mode, "--develop", str(args.develop),
               "--lines", str(args.lines), "--result-dir", rdir]
        procs.append(subprocess.Popen(cmd, env=env))
    rc = 0
    for p in procs:
        try:
            rc |= p.wait(timeout=args.timeout)
        except subprocess.TimeoutExpired:
            p.kill()
            rc |= 1
    # one process prints every rank's records, in rank order, one write each
    for r in range(args.n):
        path = os.path.join(rdir, f"rank{r}.jsonl")
        for rec in jsonl.read_records(path):
            jsonl.emit(rec)
        if os.path.exists(path):
            os.remove(path)
    os.rmdir(rdir)
    sys.exit(rc)


if __name__ == "__main__":
    main()
