#!/usr/bin/env python3
"""Timing of the pressure solvers (Jacobi, red-black SOR, multigrid) on one
MI355X: one solve on a fixed random rhs, repeated, HIP events on the model's
stream (cfd_timing_*).  Prints one JSON line per solver.

    python tools/bench_solvers.py [--n 4096] [--iters 200] [--reps 10]

Algorithmic HBM bytes (f32 fields; neighbour reuse assumed perfect):
  Jacobi / SOR iteration: 12 B per cell (read p', read rhs, write p');
  multigrid V-cycle: per level 10 smooths x 12 B + residual 12 B + restrict
  4 B + prolong-add 8 B = 144 B per cell, x 4/3 over the levels; 3 V-cycles
  per solve plus the zero fill (4 B) and the final residual (8 B).
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cfd-demo_amd"))

import cfdamd  # noqa: E402

HBM = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--solvers", default="0,1,2")
    a = ap.parse_args()
    n = a.n
    rng = np.random.default_rng(1)
    rhs = rng.uniform(-1, 1, n * n).astype(np.float32)
    for solver in (int(s) for s in a.solvers.split(",")):
        p = cfdamd.SimulationParams.cavity(1000.0, a.iters, corrector_passes=0, tol_enabled=False)
        p.pressure_solver = cfdamd.PressureSolver(solver)
        m = cfdamd.Model(cfdamd.cavity_grid(n), p)
        m.set_state(rhs=rhs)
        m.pressure_solve()   # warm-up (builds the multigrid hierarchy)
        m.synchronize()
        m.timing_begin()
        for _ in range(a.reps):
            r = m.pressure_solve()
        t = m.timing_end()
        ms = t["solve_ms"] / a.reps
        cells = n * n
        if solver == 2:
            alg = cells * (3 * 144.0 * 4.0 / 3.0 + 12.0)
            units = {"v_cycles_per_solve": 3}
        else:
            alg = cells * 12.0 * a.iters
            units = {"iterations": a.iters,
                     "cell_updates_per_s": cells * a.iters / (ms * 1e-3)}
        out = {"solver": cfdamd.PressureSolver(solver).name, "grid": [n, n],
               "ms_per_solve": ms, "residual": float(r),
               "algorithmic_GBps": alg / (ms * 1e-3) / 1e9,
               "frac_of_8TBps": alg / (ms * 1e-3) / 1e9 / HBM, **units}
        print(json.dumps(out), flush=True)
        m.close()


if __name__ == "__main__":
    main()
