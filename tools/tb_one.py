"""One model, one launch geometry (CFD_TB_KIND / CFD_TEMPORAL / CFD_TB_ROWS /
CFD_XCD_REMAP from the environment) on the bench workload, in its own
process: prints one JSON line with the solve time per sweep and the step time.
Also the unit rocprofv3 PMC passes attach to.  Usage: tb_one.py [n] [steps]
n: N (N x N cavity) or NXxNY[@S]: an NX x NY cavity-type grid with spacing 1/S
(default S = NY), e.g. 16384x1088@8192 -- the shape of one C5 slab with its
32 + 32 ghost rows at the C5 grid's power-of-two spacing."""
import json
import os
import sys
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cfd-demo_amd"))
import cfdamd  # noqa: E402

spec = sys.argv[1] if len(sys.argv) > 1 else "4096"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
if "x" in spec:
    shape, _, inv = spec.partition("@")
    nx, ny = (int(v) for v in shape.split("x"))
    inv = float(inv) if inv else float(ny)
    grid = cfdamd.Grid(nx, ny, nx / inv, ny / inv, None)
else:
    grid = cfdamd.cavity_grid(int(spec))
m = cfdamd.Model(grid,
                 cfdamd.SimulationParams.cavity(1000.0, 200, corrector_passes=0, tol_enabled=False))
m.update_n(int(os.environ.get("TB_WARMUP", "150")))
m.synchronize()
m.timing_begin()
m.update_n(steps)
tm = m.timing_end()
st = m.get_state()
# state checksum: variants of one kernel must agree bit for bit
crc = zlib.crc32(b"".join(st[k].tobytes() for k in ("u", "v", "p", "p_prime")))
print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith("CFD_")},
                  "grid": [grid.nx, grid.ny], "geometry": m.jacobi_geometry(),
                  "persist_blocks": m.persist_blocks, "persist_steals": m.persist_steals,
                  "kernel": m.kernel_config, "us_per_sweep": tm["solve_ms"] / tm["sweeps"] * 1e3,
                  "ms_per_step": tm["step_ms"] / tm["steps"], "state_crc32": crc}), flush=True)
m.close()
