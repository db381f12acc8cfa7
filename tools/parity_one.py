"""The reference's control flow (tolerance on: <= 50 sweeps, early exit at
p_tol, <= 20 corrector passes; model.rs:696-724, 748-819) on a developed
n x n cavity, for kernel traces: develop --develop fixed-count steps, inject
the state into a model with the reference's parameters, run --steps steps.
Prints one JSON line (ms/step, sweeps/step).  Usage: parity_one.py [n] [steps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cfd-demo_amd"))
import cfdamd  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
re_ = {128: 100.0, 1024: 400.0}.get(n, 1000.0)
dev = cfdamd.Model(cfdamd.cavity_grid(n), cfdamd.SimulationParams.cavity(
    re_, 200, corrector_passes=0, tol_enabled=False))
dev.update_n(int(os.environ.get("TB_WARMUP", "100")))
st = dev.get_state()
dev.close()
m = cfdamd.Model(cfdamd.cavity_grid(n), cfdamd.SimulationParams.cavity(re_, 50))
m.set_state(**st)
m.update_n(1)
s0 = m.get_residuals().jacobi_sweeps_total
m.synchronize()
t0 = time.perf_counter()
m.update_n(steps)
m.synchronize()
el = time.perf_counter() - t0
s1 = m.get_residuals().jacobi_sweeps_total
print(json.dumps({"n": n, "steps": steps, "ms_per_step": 1e3 * el / steps,
                  "sweeps_per_step": (s1 - s0) / steps, "kernel": m.jacobi_kernel}), flush=True)
m.close()
