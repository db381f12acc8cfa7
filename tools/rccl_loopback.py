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
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def worker(args):
    rank, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    # before the RCCL library initialises: one "host" per rank, sockets on lo
    os.environ["NCCL_HOSTID"] = f"cfd-loopback-rank{rank}"
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
        m.close()
        gathered = [None] * n
        dist.all_gather_object(gathered, (slab, mine))
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
                for i, ((j0, j1), f) in enumerate(gathered):
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
                           "sharded_wall_s": round(el, 3)})
    if rank == 0:
        for r in report:
            print(json.dumps(r), flush=True)
        if not all(r["bitwise_equal_single_domain"] for r in report):
            sys.exit(1)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2)
    ap.add_argument("--nx", type=int, default=256)
    ap.add_argument("--ny", type=int, default=200)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--mode", default="both", choices=["fixed", "tol", "both", "solvers"])
    ap.add_argument("--worker", action="store_true")
    args = ap.parse_args()
    if args.worker:
        worker(args)
        return
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(args.n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(args.n), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), LOCAL_RANK="0")
        cmd = [sys.executable, os.path.abspath(__file__), "--worker", "--n", str(args.n),
               "--nx", str(args.nx), "--ny", str(args.ny), "--steps", str(args.steps),
               "--mode", args.mode]
        procs.append(subprocess.Popen(cmd, env=env))
    rc = 0
    for p in procs:
        try:
            rc |= p.wait(timeout=240)
        except subprocess.TimeoutExpired:
            p.kill()
            rc |= 1
    sys.exit(rc)


if __name__ == "__main__":
    main()
