"""One model, one launch geometry (CFD_TB_KIND / CFD_TEMPORAL / CFD_TB_ROWS from
the environment), a few bench steps: the unit rocprofv3 PMC passes attach to."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cfd-demo_amd"))
import cfdamd  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
m = cfdamd.Model(cfdamd.cavity_grid(n),
                 cfdamd.SimulationParams.cavity(1000.0, 200, corrector_passes=0, tol_enabled=False))
m.update_n(steps)
m.synchronize()
print(m.kernel_config, m.get_residuals().simulation_step)
m.close()
