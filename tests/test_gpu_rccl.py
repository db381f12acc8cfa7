"""GPU: the RCCL transport itself.  tests/test_gpu_sharded.py checks the
decomposition through the in-process LocalHub; here two processes drive
cfd_create_sharded through real RCCL calls (ncclSend / ncclRecv groups for the
halos, ncclAllReduce for the residual and CFL maxima) on the one GPU of the
box: each rank gets its own NCCL_HOSTID, so RCCL connects them through its
socket transport over loopback instead of refusing two ranks on one device
(tools/rccl_loopback.py).  The gathered slabs must equal the single-domain
model bit for bit, in the bench's fixed-count mode (deep halos, overlapped
band exchange, persistent runs between exchanges -- since r4 with the ranks'
kernels sharing the GPU) and in the reference's tolerance mode (lagged
convergence)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from jsonl import records  # noqa: E402  (tolerant: several objects per line)


def test_rccl_two_ranks_bitwise_single_domain():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rccl_loopback.py"),
                        "--n", "2", "--steps", "4"], capture_output=True, text=True, timeout=300)
    lines = records(r.stdout)
    assert r.returncode == 0 and len(lines) == 2, (r.stdout[-2000:], r.stderr[-3000:])
    assert all(x["bitwise_equal_single_domain"] for x in lines), lines


def test_rccl_two_ranks_solvers_bitwise_single_domain():
    """SOR and multigrid on two RCCL ranks (socket transport on one GPU), with
    the tolerance off and on: the gathered slabs equal a single-domain model."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rccl_loopback.py"),
                        "--n", "2", "--steps", "3", "--mode", "solvers"], capture_output=True,
                       text=True, timeout=300)
    lines = records(r.stdout)
    assert r.returncode == 0 and len(lines) == 4, (r.stdout[-2000:], r.stderr[-3000:])
    assert all(x["bitwise_equal_single_domain"] for x in lines), lines


_NEVER_JOINS = r"""
import os, sys, time
sys.path.insert(0, os.path.join(os.environ["CFD_ROOT"], "cfd-demo_amd"))
os.environ["NCCL_HOSTID"] = "cfd-lonely-rank0"
os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
os.environ.setdefault("NCCL_IB_DISABLE", "1")
os.environ.setdefault("NCCL_NET", "Socket")
import cfdamd
uid = cfdamd.rccl_unique_id()
t0 = time.monotonic()
try:
    cfdamd.Model(cfdamd.cavity_grid(64), cfdamd.SimulationParams.cavity(100.0, 8), device=0,
                 n_ranks=2, rank=0, unique_id=uid)
    print("CREATED")
except cfdamd.CfdError as e:
    print("CODE", e.code, round(time.monotonic() - t0, 1), str(e)[:200])
"""


@pytest.mark.timeout(200)
def test_comm_init_deadline_when_a_rank_never_joins():
    """ncclCommInitRank has a deadline (non-blocking ncclCommInitRankConfig
    polled under CFD_RCCL_TIMEOUT_S): rank 0 of 2 whose peer never arrives
    gets CFD_ERCCL within the deadline instead of hanging in
    cfd_create_sharded."""
    env = dict(os.environ, CFD_ROOT=ROOT, CFD_RCCL_TIMEOUT_S="5")
    r = subprocess.run([sys.executable, "-c", _NEVER_JOINS], env=env, capture_output=True,
                       text=True, timeout=150)
    out = [l for l in r.stdout.splitlines() if l.startswith(("CODE", "CREATED"))]
    assert out and out[0].startswith("CODE -3"), (r.stdout[-2000:], r.stderr[-2000:])
    assert float(out[0].split()[2]) < 30.0, out


@pytest.mark.timeout(600)
def test_bench_self_launch_two_ranks_loopback():
    """`python bench.py --gpus 2` exactly as the driver invokes it (no external
    launcher): bench.py spawns both ranks itself; with CFD_BENCH_LOOPBACK=1
    both sit on device 0 and RCCL connects them over its socket transport.
    One line, n_gpus 2, and the RCCL communicator reports 2 ranks."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(CFD_BENCH_LOOPBACK="1", CFD_RCCL_TIMEOUT_S="60")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "3", "--warmup", "1", "--develop", "10", "--nx", "1024",
                        "--ny", "512", "--iters", "64"], env=env, capture_output=True,
                       text=True, timeout=300)
    lines = records(r.stdout)
    assert r.returncode == 0 and len(lines) == 1, (r.stdout[-2000:], r.stderr[-3000:])
    assert lines[0]["n_gpus"] == 2 and lines[0]["ranks_seen"] == 2, lines[0]
    assert lines[0]["launcher"] == "bench.py" and len(lines[0]["rank_ms_per_step"]) == 2
    # r4: the N > 1 line verifies itself -- one more step on the slabs equals
    # a single-domain model's step from the gathered state -- and carries
    # every rank's phase and RCCL exchange times and its Jacobi geometry
    out = lines[0]
    assert out["parity_sharded_step"] is True, out.get("parity_sharded_step_detail")
    assert len(out["rank_phases"]) == 2, out["rank_phases"]
    for rp in out["rank_phases"]:
        assert rp["exchange_us_per_step"] > 0 and rp["exchanges_per_step"] >= 3, rp
        assert rp["geometry"]["wave_cols"] > 0, rp
    assert out["jacobi_geometry"]["segments"] > 0


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n,nx,ny", [(2, 8192, 4096), (4, 8192, 8192)])
def test_rccl_developed_full_size_slabs_bitwise(n, nx, ny):
    """C4 (2 ranks, 8192x4096) and the 4-GPU weak-scaling grid (4 ranks,
    8192^2) over real RCCL calls: a cavity developed for 400 steps (plus a
    seeded 1e-3 perturbation, tools/rccl_loopback.py perturb) is injected
    into the slabs and stepped twice; every rank's rows equal the
    single-domain continuation bit for bit, with non-zero p' (>= 90 %) in
    the rows either side of every slab boundary."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rccl_loopback.py"),
                        "--n", str(n), "--nx", str(nx), "--ny", str(ny), "--steps", "2",
                        "--develop", "400", "--mode", "developed", "--timeout", "400"],
                       capture_output=True, text=True, timeout=480)
    lines = records(r.stdout)
    assert r.returncode == 0 and len(lines) == n, (r.stdout[-2000:], r.stderr[-3000:])
    for x in lines:
        assert x["bitwise_equal_single_domain"], x
        assert x["ranks_seen"] == n
        assert x["boundary_pprime_nonzero_frac"] >= 0.9, x
        # the SCALE configuration since r5: one launch per 8-sweep block
        # between the p' exchanges (the same-geometry A/B)
        assert x["persist_blocks"] == 0, x
