"""Per-wave timeline of one kind-5 Jacobi launch (diagnostic build with
-DCFD_LDS_STAMP=1, loaded through CFD_LIB): start/end of every wave relative to
the first start, lifetime, shader-clock rate, and the waves per CU/SIMD.
Answers whether a launch's time goes to the waves' own work or to their
dispatch ramp / tail.  Usage: CFD_LIB=... python tools/lds_stamps.py [n]"""
import collections
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
fn = L.cfd_diag_lds_stamps
fn.argtypes = [C.c_void_p, C.c_int]
cap = 1 << 15
buf = np.zeros(cap * 4, dtype=np.uint64)
got = fn(buf.ctypes.data, cap)
s = buf[: got * 4].reshape(-1, 4)
s = s[s[:, 1] > 0]
t0 = s[:, 0].astype(np.int64)
t1 = s[:, 1].astype(np.int64)
base = t0.min()
st = (t0 - base) * 10.0 / 1000.0     # us (100 MHz)
en = (t1 - base) * 10.0 / 1000.0
life = en - st
clk = (s[:, 2] & 0xFFFFFFFFFF).astype(np.float64) / np.maximum(life, 1e-3) / 1e3   # GHz
bid = (s[:, 2] >> 40).astype(np.int64)
hw = (s[:, 3] & 0xFFFFFFFF).astype(np.int64)
xcc = (s[:, 3] >> 32).astype(np.int64) & 0xF
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
sh = (hw >> 12) & 1
se = (hw >> 13) & 7
cukey = xcc * 1000 + se * 100 + sh * 20 + cu
per_cu = collections.Counter(cukey.tolist())
per_simd = collections.Counter((cukey * 4 + simd).tolist())
q = lambda a: [round(float(np.percentile(a, p)), 2) for p in (0, 10, 50, 90, 100)]
out = {"waves": int(len(s)), "span_us": round(float(en.max()), 2),
       "start_us_pct0_10_50_90_100": q(st), "end_us_pct": q(en), "life_us_pct": q(life),
       "clock_GHz_pct": q(clk), "cus_used": len(per_cu),
       "waves_per_cu_hist": dict(sorted(collections.Counter(per_cu.values()).items())),
       "waves_per_simd_hist": dict(sorted(collections.Counter(per_simd.values()).items())),
       "kernel": m.kernel_config}
# which waves end last: the wave's (column, segment) from its XCD-renumbered
# block and wave index (the stamp's slot is blockIdx * 4 + wave, in order)
geo = m.jacobi_geometry(False)
nwc, nseg = geo["wave_cols"], geo["segments"]
slot = np.nonzero(buf[: got * 4].reshape(-1, 4)[:, 1] > 0)[0]
wave = slot % 4
if len(s) > nwc * nseg:   # the filled round (lds_fill_waves)
    wtot = len(s)
    gw = bid * 4 + wave
    q_, rem = wtot // nwc, wtot % nwc
    big = rem * (q_ + 1)
    wc = np.where(gw < big, gw // (q_ + 1), rem + (gw - big) // max(q_, 1))
    seg = np.where(gw < big, gw - wc * (q_ + 1), gw - big - (wc - rem) * q_)
    ns = np.where(wc < rem, q_ + 1, q_)
else:
    wc = bid % nwc
    seg = (bid // nwc) * 4 + wave
    ns = np.full_like(seg, nseg)
row_edge = (seg == 0) | (seg == ns - 1)
col_edge = (wc == 0) | (wc == nwc - 1)
simd_load = np.array([per_simd[k] for k in (cukey * 4 + simd).tolist()])
cats = {"interior": ~row_edge & ~col_edge, "row_edge": row_edge & ~col_edge,
        "col_edge": col_edge & ~row_edge, "corner": row_edge & col_edge}
for w_ in sorted(set(simd_load.tolist())):
    cats[f"simd_{w_}_waves"] = simd_load == w_
for par in (0, 1):
    cats[f"seg_parity_{par}"] = (seg % 2 == par) & ~row_edge & ~col_edge
last = en >= np.percentile(en, 95)
out["by_kind"] = {k: {"n": int(v.sum()), "end_us_pct": q(en[v]) if v.any() else None,
                      "in_last_5pct": int((v & last).sum())} for k, v in cats.items()}
# time histogram of live waves (10 bins over the span)
edges = np.linspace(0, en.max(), 11)
out["live_waves_at"] = [int(((st <= x) & (en > x)).sum()) for x in (edges[:-1] + edges[1:]) / 2]
print(json.dumps(out), flush=True)
np.save(os.path.join(ROOT, "gpurun_out", "lds_stamps.npy"), s)
m.close()
