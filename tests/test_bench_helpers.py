"""CPU checks of bench.py's bookkeeping against the committed profiles: the
HBM-traffic and VALU-issue figures the driver's bench line carries are found
for the bench kernel on the bench slab (and not for other slabs), and the
roofline fractions stay fractions."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_pmc_traffic_found_for_bench_slab():
    b = _bench()
    t, src = b.pmc_traffic("k_jacobi_lds<8, 1, false>", "4096x4096")
    assert t is not None and src.startswith("profiles/")
    # one-pass bytes of the launch are 201.3 MB; the measured traffic is within 1.25x
    assert 201326592 <= t <= 1.25 * 201326592
    assert b.pmc_traffic("k_jacobi_lds<8, 1, false>", "123x45") == (None, None)


def test_roofline_valu_is_a_fraction():
    b = _bench()
    r = b.roofline_valu("k_jacobi_lds<8, 1, false>", "4096x4096", 0.040)   # 40 us launch
    assert r is not None and r["bound"] == "valu"
    assert 0.3 < r["frac"] <= 1.0
    assert r["valu_insts_per_launch"] > 1e7
    assert b.roofline_valu("k_jacobi_lds<8, 1, false>", "123x45", 0.040) is None


def test_weak_scaling_grids_keep_the_slab():
    b = _bench()
    for n, (nx, ny) in b.WEAK_GRIDS.items():
        assert nx * ny == n * 4096 * 4096


def _run_bench(args, env_extra=None, timeout=240):
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                       capture_output=True, text=True, timeout=timeout)
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.lstrip().startswith("{")]
    return p, lines


def test_bench_gpus_n_self_launches_n_ranks():
    """`python bench.py --gpus 2` with no external launcher spawns 2 ranks
    (RANK/WORLD_SIZE/MASTER_* set by bench.py itself) and prints exactly one
    line, rank 0's, with n_gpus 2 and 2 ranks in the transport group (the
    dry run stops before the HIP library: gloo group only)."""
    p, lines = _run_bench(["--gpus", "2", "--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert len(lines) == 1
    assert lines[0]["n_gpus"] == 2 and lines[0]["ranks_seen"] == 2
    assert lines[0]["launcher"] == "bench.py" and lines[0]["dry_run"] is True


def test_bench_gpus_n_never_reports_fewer_ranks():
    """Without enough GPUs (this container has none) every launched rank
    refuses to run: the job fails and no line with n_gpus 1 appears."""
    p, lines = _run_bench(["--gpus", "2", "--no-cpu-baseline", "--no-control", "--no-parity"])
    assert p.returncode != 0
    assert not any(l.get("n_gpus") == 1 for l in lines)
    assert "needs 2 GPUs" in p.stderr
