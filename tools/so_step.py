"""The bench workload with the second-order scheme (velocity_scheme 1):
150 warm-up steps + 5, one process; the unit rocprofv3 attaches to when
timing the SO predictor (CFD_PRED_VEC=0: one face per thread)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cfd-demo_amd"))
import cfdamd  # noqa: E402

m = cfdamd.Model(cfdamd.cavity_grid(4096),
                 cfdamd.SimulationParams.cavity(1000.0, 200, corrector_passes=0, tol_enabled=False,
                                                velocity_scheme=cfdamd.VelocityScheme.SecondOrder))
m.update_n(155)
m.synchronize()
m.close()
