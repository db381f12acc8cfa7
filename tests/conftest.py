import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "cfd-demo_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

# Files whose tests start several processes on the GPU (RCCL over loopback,
# bench.py self-launch).  They run after every single-process parity file, so
# a harness fault there cannot hide the oracle checks behind it under -x (r4).
MULTI_PROCESS_FILES = ("test_gpu_rccl.py",)
# r5's lagged check and speculative slab blocks (first run on the hardware in
# r6): after everything else
LAST_FILES = ("test_gpu_spec_lag_slabs.py",)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests proper")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(session, config, items):
    def rank(it):
        name = os.path.basename(str(it.fspath))
        return 2 if name in LAST_FILES else 1 if name in MULTI_PROCESS_FILES else 0
    items[:] = sorted(items, key=rank)   # stable: file order kept within each group
