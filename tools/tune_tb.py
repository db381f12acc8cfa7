"""Sweep k_jacobi_tb launch geometry on the GPU (one process, interleaved
rounds, median per config).  Usage: python tools/tune_tb.py [n]"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cfd-demo_amd"))
import cfdamd  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
# r > 0: fixed rows per wave; r < 0: balanced segmentation with -r blocks per CU
configs = [(1, 4, r) for r in (12, 18, 24, 30, 36, 42, 32)] + \
          [(3, 8, r) for r in (18, 24, 30, 36)] + [(3, 6, r) for r in (24, 30, 36)] + \
          [(1, 3, r) for r in (24, 30)]
if os.environ.get("TUNE_CONFIGS"):
    configs = [tuple(int(x) for x in c.split(",")) for c in os.environ["TUNE_CONFIGS"].split(";")]
grid = cfdamd.cavity_grid(n)
params = cfdamd.SimulationParams.cavity(1000.0, 200, corrector_passes=0, tol_enabled=False)
models = {}
configs = [c if len(c) == 4 else tuple(c) + (1,) for c in configs]
for kind, t, r, x in configs:
    os.environ["CFD_XCD_REMAP"] = str(x)
    os.environ["CFD_TB_KIND"] = str(kind)
    os.environ["CFD_TEMPORAL"] = str(t)
    if r > 0:
        os.environ["CFD_TB_ROWS"] = str(r)
        os.environ.pop("CFD_TB_BPC", None)
    else:
        os.environ.pop("CFD_TB_ROWS", None)
        os.environ["CFD_TB_BPC"] = str(-r)
    m = cfdamd.Model(grid, params)
    m.update_n(2)
    m.synchronize()
    models[(kind, t, r, x)] = m
res = {c: [] for c in configs}
for rnd in range(3):
    for c in configs:
        m = models[c]
        m.timing_begin()
        m.update_n(3)
        tm = m.timing_end()
        res[c].append(tm["solve_ms"] / tm["sweeps"] * 1e3)
out = []
for c in configs:
    us = statistics.median(res[c])
    out.append({"kind": c[0], "T": c[1], "R": c[2], "xcd": c[3], "us_per_sweep": us,
                "cell_updates_per_s": n * n / (us * 1e-6)})
    print(json.dumps(out[-1]), flush=True)
