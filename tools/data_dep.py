"""Is the Jacobi launch time data-dependent?  Runs the bench workload (4096^2
cavity, 200 sweeps/step) for many steps, printing the solve time per sweep as
the fields evolve, then times single sweeps on the evolved state with its
subnormal values kept, flushed to zero, and replaced by random normals.
Usage: python tools/data_dep.py [steps] [chunk]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cfd-demo_amd"))
import cfdamd  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 25
n = 4096
params = cfdamd.SimulationParams.cavity(1000.0, 200, corrector_passes=0, tol_enabled=False)
m = cfdamd.Model(cfdamd.cavity_grid(n), params)


def stats(a):
    a = np.asarray(a, np.float32)
    fin = np.isfinite(a)
    sub = fin & (a != 0) & (np.abs(a) < np.finfo(np.float32).tiny)
    return {"zero": float((a == 0).mean()), "subnormal": float(sub.mean()),
            "nonfinite": float((~fin).mean()),
            "max_abs": float(np.abs(a[fin]).max()) if fin.any() else None}


def ftz(a):
    a = a.copy()
    a[np.isfinite(a) & (np.abs(a) < np.finfo(np.float32).tiny)] = 0.0
    return a


done = 0
while done < steps:
    m.timing_begin()
    m.update_n(chunk)
    tm = m.timing_end()
    done += chunk
    line = {"step": done, "us_per_sweep": round(tm["solve_ms"] / tm["sweeps"] * 1e3, 3),
            "ms_per_step": round(tm["step_ms"] / tm["steps"], 4)}
    if done % 100 == 0 or done == chunk:
        st = m.get_state()
        line.update({k: stats(st[k]) for k in ("p_prime", "rhs", "u", "v")})
    print(json.dumps(line), flush=True)

st = m.get_state()
res = {"kept": m.profile_sweeps(40) * 1e3}
m.set_state(p_prime=ftz(st["p_prime"]), rhs=ftz(st["rhs"]))
res["p_rhs_flushed"] = m.profile_sweeps(40) * 1e3
rng = np.random.default_rng(1)
m.set_state(p_prime=rng.uniform(-1, 1, st["p_prime"].size).astype(np.float32),
            rhs=rng.uniform(-1, 1, st["rhs"].size).astype(np.float32))
res["random_normals"] = m.profile_sweeps(40) * 1e3
m.set_state(p_prime=np.zeros_like(st["p_prime"]), rhs=np.zeros_like(st["rhs"]))
res["zeros"] = m.profile_sweeps(40) * 1e3
print(json.dumps({"single_sweep_us": res}), flush=True)
# whole steps with every field's subnormals flushed
m.set_state(**{k: ftz(st[k]) for k in ("u", "v", "p", "u_star", "v_star", "p_prime", "rhs")})
m.timing_begin()
m.update_n(2)
tm = m.timing_end()
print(json.dumps({"after_full_flush_us_per_sweep": tm["solve_ms"] / tm["sweeps"] * 1e3}), flush=True)
m.close()
