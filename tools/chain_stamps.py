"""Per-wave timeline of one k_jacobi_chain launch (diagnostic build with
-DCFD_CHAIN_STAMP=1, loaded through CFD_LIB): per role (chain waves 0-3, edge
groups 4) the time in the opening, the steady slots, the closing slots and
waiting at exit, and the spread of wave end times.
Usage: CFD_LIB=... python tools/chain_stamps.py [n]"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cfd-demo_amd"))
import cfdamd  # noqa: E402
from cfdamd import _lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
m = cfdamd.Model(cfdamd.cavity_grid(n),
                 cfdamd.SimulationParams.cavity(1000.0, 200, corrector_passes=0, tol_enabled=False))
m.update_n(int(os.environ.get("TB_WARMUP", "20")))
m.synchronize()
L = _lib.load()
fn = L.cfd_diag_chain_stamps
fn.argtypes = [C.c_void_p, C.c_int]
cap = 1 << 15
buf = np.zeros(cap * 8, dtype=np.uint64)
got = fn(buf.ctypes.data, cap)
s = buf[: got * 8].reshape(-1, 8).astype(np.int64)
s = s[s[:, 4] > 0]
base = s[:, 0].min()
us = lambda c: (c - base) * 0.01   # 100 MHz ticks -> us
role = s[:, 6] & 0xFF
q = lambda a: [round(float(np.percentile(a, p)), 2) for p in (0, 10, 50, 90, 100)] if len(a) else []
out = {"waves": int(len(s)), "span_us": round(float(us(s[:, 4]).max()), 2), "roles": {}}
for r in range(5):
    k = s[role == r]
    if not len(k):
        continue
    d = {"n": int(len(k)), "start": q(us(k[:, 0])), "end": q(us(k[:, 4]))}
    if r < 4:
        d["opening"] = q((k[:, 1] - k[:, 0]) * 0.01)
        d["steady"] = q((k[:, 2] - k[:, 1]) * 0.01)
        d["closing"] = q((k[:, 3] - k[:, 2]) * 0.01)
        d["exit_wait"] = q((k[:, 4] - k[:, 3]) * 0.01)
    else:
        d["life"] = q((k[:, 4] - k[:, 0]) * 0.01)
    hw = s[role == r][:, 5] & 0xFFFFFFFF
    d["simd_hist"] = np.bincount(((hw >> 4) & 3).astype(np.int64), minlength=4).tolist()
    out["roles"][str(r)] = d
print(json.dumps(out), flush=True)
m.close()
