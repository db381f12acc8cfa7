"""Diagnostic: the fused corrector head (CFD_CORR_HEAD) vs the separate
launches vs the oracle, per field and step, on a small cavity with corrector
passes.  Usage: diag_corr_head.py [fastdiv] [temporal] [kind] [passes]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cfd-demo_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
fd, T, kind, passes = (sys.argv[1:5] + ["0", "1", "1", "1"][len(sys.argv) - 1:])[:4]
os.environ.update(CFD_FASTDIV=fd, CFD_TEMPORAL=T, CFD_TB_KIND=kind)
if kind == "1":
    os.environ["CFD_TB_ROWS"] = "32"
import cfdamd  # noqa: E402
from oracle import OracleModel  # noqa: E402

g = cfdamd.Grid(256, 128, 2.0, 1.0, None)
kw = dict(bc_kind=1, viscosity=0.001, jacobi_iters=23, corrector_passes=int(passes), tol_enabled=0)
out = {}
for head in ("0", "1"):
    os.environ["CFD_CORR_HEAD"] = head
    m = cfdamd.Model(g, cfdamd.SimulationParams(dt=0.005, viscosity=0.001, jacobi_iters=23,
                                                corrector_passes=int(passes), tol_enabled=False,
                                                bc_kind=cfdamd.BoundaryKind.Cavity))
    o = OracleModel(256, 128, 2.0, 1.0, **kw)
    rows = []
    for step in range(4):
        m.update()
        o.update()
        st = m.get_state()
        diff = {f: int(np.count_nonzero(st[f].view(np.uint32) != o.field(f).view(np.uint32)))
                for f in ("u", "v", "p", "p_prime", "u_star", "v_star", "rhs")}
        rows.append(diff)
    out[head] = rows
    m.close()
print(json.dumps(out))
