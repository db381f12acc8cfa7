"""Phase timeline of the resident tolerance-mode solve (k_jacobi_resident) on
the reference's default design point, from a diagnostic build with
-DCFD_RES_STAMP=1 (loaded through CFD_LIB): per block, the median and max over
workgroups of load / sweeps / store issue / store drain + residual atomics /
grid barrier / residual read, and the gap to the next block.  Answers where a
solve's ~140 us go.  Usage: CFD_LIB=... python tools/res_stamps.py [develop]"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cfd-demo_amd"))
import cfdamd  # noqa: E402
from cfdamd import _lib  # noqa: E402

develop = int(sys.argv[1]) if len(sys.argv) > 1 else 200
m = cfdamd.Model(cfdamd.default_grid(), cfdamd.SimulationParams())
m.update_n(develop)
m.update_n(1)
m.synchronize()
geo = m.kernel_config
L = _lib.load()
fn = L.cfd_diag_res_stamps
fn.argtypes = [C.c_void_p, C.c_int]
NWG, NS = 256, 64
buf = np.zeros(NWG * NS, dtype=np.uint64)
got = fn(buf.ctypes.data, NWG * NS)
m.close()
s = buf[:got].reshape(NWG, NS).astype(np.int64)
rows = s[s[:, 0] > 0]                       # workgroups that ran
base = rows[:, 0].min()
us = (rows - base) * 0.01                    # 100 MHz ticks -> us
n = int((rows > 0).sum(axis=1).min())        # stamps every workgroup has
PH = ["load", "sweeps", "store_issue", "drain+atomics", "barrier", "err_read"]
out = {"workgroups": int(rows.shape[0]), "stamps": n, "kernel_config": geo,
       "entry_spread_us": float(us[:, 0].max()), "blocks": []}
k = 0
i = 1
while i + 6 < n:
    d = np.diff(us[:, i:i + 7], axis=1)      # 6 phases
    blk = {ph: [round(float(np.median(d[:, j])), 2), round(float(d[:, j].max()), 2)]
           for j, ph in enumerate(PH)}
    if i + 7 < n:
        gap = us[:, i + 7] - us[:, i + 6]
        blk["to_next"] = [round(float(np.median(gap)), 2), round(float(gap.max()), 2)]
    blk["start_median_us"] = round(float(np.median(us[:, i])), 2)
    out["blocks"].append(blk)
    i += 7
    k += 1
out["end_max_us"] = round(float(us[:, n - 1].max()), 2)
print(json.dumps(out, indent=1))
