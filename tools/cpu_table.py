#!/usr/bin/env python3
"""BASELINE.md's CPU table: the reference CPU path (oracle/cfd_oracle.c, the C
restatement of src/model.rs; the Rust binary cannot be built here) timed on
this host for C1-C3 in the timed mode (K sweeps/step, tolerance off, no extra
corrector passes), 1 thread (the reference's one worker thread,
model.rs:1287) and all of this job's threads (OpenMP row split, same bits).

Each config is developed on the GPU (--develop steps, so the CPU sweeps the
same mostly non-zero fields the GPU bench times), its state handed to the
oracle, one warm-up step, then the median of up to --max-steps timed steps
within --budget seconds.  Prints one JSON line per config and thread count.

    python tools/cpu_table.py [--develop 400] [--budget 20]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "cfd-demo_amd"))

CONFIGS = [("C1", 128, 100.0, 50), ("C2", 1024, 400.0, 100), ("C3", 4096, 1000.0, 200)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--develop", type=int, default=400)
    ap.add_argument("--budget", type=float, default=20.0)
    ap.add_argument("--max-steps", type=int, default=5)
    a = ap.parse_args()
    import bench
    import cfdamd
    host, ncpu = bench.cpu_info()
    nt = bench.cpu_threads()
    for name, n, re, iters in CONFIGS:
        m = cfdamd.Model(cfdamd.cavity_grid(n), cfdamd.SimulationParams.cavity(
            re, iters, corrector_passes=0, tol_enabled=False), device=0)
        m.update_n(a.develop)
        m.synchronize()
        t0 = time.perf_counter()
        m.update_n(20)
        m.synchronize()
        gpu_ms = 1e3 * (time.perf_counter() - t0) / 20
        st = m.get_state()
        m.close()
        for threads in (1, nt):
            r = bench.cpu_baseline(n, n, iters, re, a.budget, st, threads=threads,
                                   max_steps=a.max_steps)
            print(json.dumps({"config": name, "grid": [n, n], "re": re, "sweeps_per_step": iters,
                              "threads": threads, "cell_updates_per_s": r["value"],
                              "ms_per_step": 1e3 * n * n * iters / r["value"],
                              "gpu_ms_per_step": gpu_ms, "host": host, "host_cpus": ncpu,
                              "sample": r["sample"]}), flush=True)


if __name__ == "__main__":
    main()
