"""The reference's default design point (default_grid() 800 x 264 channel with
the cylinder, SimulationParams::default(): <= 50 sweeps, early exit 1e-4, <= 20
corrector passes) for kernel traces: develop REFDEF_DEVELOP steps from rest,
time `steps` steps.  Prints one JSON line.  Usage: refdef_one.py [steps] [so]"""
import json
import os
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cfd-demo_amd"))
import cfdamd  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
scheme = cfdamd.VelocityScheme.SecondOrder if len(sys.argv) > 2 and sys.argv[2] == "so" \
    else cfdamd.VelocityScheme.FirstOrder
m = cfdamd.Model(cfdamd.default_grid(), cfdamd.SimulationParams(velocity_scheme=scheme))
m.update_n(int(os.environ.get("REFDEF_DEVELOP", "200")))
m.synchronize()
s0 = m.get_residuals().jacobi_sweeps_total
t0 = time.perf_counter()
m.update_n(steps)
m.synchronize()
el = time.perf_counter() - t0
s1 = m.get_residuals().jacobi_sweeps_total
st = m.get_state()
crc = zlib.crc32(b"".join(st[k].tobytes() for k in ("u", "v", "p", "p_prime")))
print(json.dumps({"state_crc32": crc, "steps": steps, "ms_per_step": 1e3 * el / steps,
                  "sweeps_per_step": (s1 - s0) / steps, "kernel": m.jacobi_kernel,
                  "config": m.kernel_config}), flush=True)
m.close()
