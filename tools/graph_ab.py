"""Wall-clock of K timed-mode steps on the bench workload without solve
timing (so CFD_GRAPH=1 replays captured steps): develop 400 steps, then
time K steps between synchronizations, best of R.  Prints one JSON line.
Usage: CFD_GRAPH=0|1 python tools/graph_ab.py [K] [R]"""
import json
import os
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cfd-demo_amd"))
import cfdamd  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
R = int(sys.argv[2]) if len(sys.argv) > 2 else 5
m = cfdamd.Model(cfdamd.cavity_grid(4096),
                 cfdamd.SimulationParams.cavity(1000.0, 200, corrector_passes=0, tol_enabled=False))
m.update_n(400)
m.synchronize()
best = 1e9
for _ in range(R):
    t0 = time.perf_counter()
    m.update_n(K)
    m.synchronize()
    best = min(best, (time.perf_counter() - t0) / K)
st = m.get_state()
crc = zlib.crc32(b"".join(st[k].tobytes() for k in ("u", "v", "p", "p_prime")))
print(json.dumps({"graph": os.environ.get("CFD_GRAPH", "0"), "ms_per_step": best * 1e3,
                  "steps": int(st["simulation_step"]), "state_crc32": crc}), flush=True)
m.close()
