"""Diagnostic: one Jacobi solve (jacobi_pressure) with the chained march vs the
per-launch march from the same random state; prints where p' differs."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cfd-demo_amd"))
import cfdamd  # noqa: E402

nx, ny = (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "256x128").split("x"))
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 8
grid = cfdamd.Grid(nx, ny, nx / 128.0, ny / 128.0, None)
params = cfdamd.SimulationParams.cavity(1000.0, iters, corrector_passes=0, tol_enabled=False)
rng = np.random.default_rng(5)
out = {}
for key, env in {"per_launch": ("0", "0"), "chain_ref": ("1", "0"), "chain_sums": ("1", "1")}.items():
    os.environ["CFD_JACOBI_CHAIN"], os.environ["CFD_JACOBI_SUMS"] = env
    m = cfdamd.Model(grid, params, device=0)
    st = m.get_state()
    st["p_prime"] = rng.standard_normal(st["p_prime"].size).astype(np.float32) if key == "per_launch" else out["per_launch"][1]
    st["rhs"] = (0.01 * np.random.default_rng(6).standard_normal(st["rhs"].size)).astype(np.float32)
    m.set_state(**st)
    m.jacobi_pressure()
    out[key] = (m.get_state()["p_prime"].reshape(ny, nx), st["p_prime"], m.jacobi_kernel["name"], m.chain_stats)
    m.close()
lib = cfdamd.load()
import ctypes as C
v = [C.c_int() for _ in range(5)]
ok = lib.cfd_plan_chain(nx, ny, 256, 3, 1, ny - 1, *(C.byref(x) for x in v))
print("plan", ok, [x.value for x in v])
for key in ("chain_ref", "chain_sums"):
    a, b = out[key][0], out["per_launch"][0]
    d = a.view(np.uint32) != b.view(np.uint32)
    rows = np.nonzero(d.any(axis=1))[0]
    cols = np.nonzero(d.any(axis=0))[0]
    print(key, out[key][2], out[key][3], "differ", int(d.sum()), "rows", rows[:40].tolist(), "cols", cols[:12].tolist(), cols[-4:].tolist())
