"""Where the developed bench field keeps its subnormals: p' and rhs values
below 2^-126 (non-zero) per tenth of the rows, after the bench's 400
developing steps of the 4096^2 cavity.  Diagnostic for the per-XCD cycle
spread of the Jacobi launch (tools/lds_stamps.py).  Usage: subnormal_bands.py [n] [steps]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cfd-demo_amd"))
import cfdamd  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 400
m = cfdamd.Model(cfdamd.cavity_grid(n),
                 cfdamd.SimulationParams.cavity(1000.0, 200, corrector_passes=0, tol_enabled=False))
m.update_n(steps)
st = m.get_state()
tiny = np.finfo(np.float32).tiny
out = {"n": n, "steps": steps, "bands": []}
for f in ("p_prime", "rhs"):
    a = np.abs(st[f].reshape(n, n))
    for b in range(10):
        rows = a[b * n // 10:(b + 1) * n // 10]
        sub = int(((rows > 0) & (rows < tiny)).sum())
        zero = int((rows == 0).sum())
        out["bands"].append({"field": f, "band": b, "subnormal": sub, "zero": zero,
                             "frac_subnormal": sub / rows.size})
print(json.dumps(out))
m.close()
