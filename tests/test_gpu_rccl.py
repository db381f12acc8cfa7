"""GPU: the RCCL transport itself.  tests/test_gpu_sharded.py checks the
decomposition through the in-process LocalHub; here two processes drive
cfd_create_sharded through real RCCL calls (ncclSend / ncclRecv groups for the
halos, ncclAllReduce for the residual and CFL maxima) on the one GPU of the
box: each rank gets its own NCCL_HOSTID, so RCCL connects them through its
socket transport over loopback instead of refusing two ranks on one device
(tools/rccl_loopback.py).  The gathered slabs must equal the single-domain
model bit for bit, in the bench's fixed-count mode (deep halos, overlapped
band exchange) and in the reference's tolerance mode (lagged convergence)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rccl_two_ranks_bitwise_single_domain():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rccl_loopback.py"),
                        "--n", "2", "--steps", "4"], capture_output=True, text=True, timeout=300)
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert r.returncode == 0 and len(lines) == 2, (r.stdout[-2000:], r.stderr[-3000:])
    assert all(x["bitwise_equal_single_domain"] for x in lines), lines


def test_rccl_two_ranks_solvers_bitwise_single_domain():
    """SOR and multigrid on two RCCL ranks (socket transport on one GPU), with
    the tolerance off and on: the gathered slabs equal a single-domain model."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rccl_loopback.py"),
                        "--n", "2", "--steps", "3", "--mode", "solvers"], capture_output=True,
                       text=True, timeout=300)
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert r.returncode == 0 and len(lines) == 4, (r.stdout[-2000:], r.stderr[-3000:])
    assert all(x["bitwise_equal_single_domain"] for x in lines), lines
