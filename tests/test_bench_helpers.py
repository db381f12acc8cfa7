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
    t, src, blocks = b.pmc_traffic("k_jacobi_lds<8, 1, false>", "4096x4096")
    assert t is not None and src.startswith("profiles/")
    # one-pass bytes of the launch are 201.3 MB; the measured traffic is within 1.25x
    assert 201326592 <= t <= 1.25 * 201326592
    assert blocks is None   # a one-block kernel: no per-dispatch block count recorded
    assert b.pmc_traffic("k_jacobi_lds<8, 1, false>", "123x45") == (None, None, None)


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


def test_assemble_slabs_owned_rows_and_shared_v_face():
    """cfdamd.assemble_slabs (bench.py's N > 1 parity step gathers with it):
    owned rows concatenate; the v face row j1 both neighbours hold comes once,
    and a mismatch between the two copies is an error, not a silent pick."""
    import sys
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "cfd-demo_amd"))
    import cfdamd
    nx, ny = 8, 10
    rng = np.random.default_rng(3)
    g = {f: rng.standard_normal(n).astype(np.float32) for f, n in
         (("u", (nx + 1) * ny), ("p", nx * ny), ("p_prime", nx * ny), ("u_star", (nx + 1) * ny),
          ("rhs", nx * ny), ("v", nx * (ny + 1)), ("v_star", nx * (ny + 1)))}
    cuts = [0, 3, 7, 10]
    slabs = []
    for j0, j1 in zip(cuts[:-1], cuts[1:]):
        st = {f: g[f].reshape(-1, nx + 1)[j0:j1].ravel() for f in ("u", "u_star")}
        st.update({f: g[f].reshape(-1, nx)[j0:j1].ravel() for f in ("p", "p_prime", "rhs")})
        st.update({f: g[f].reshape(-1, nx)[j0:j1 + 1].ravel() for f in ("v", "v_star")})
        slabs.append((j0, j1, st))
    out = cfdamd.assemble_slabs(slabs, nx)
    for f in g:
        assert np.array_equal(out[f], g[f]), f
    slabs[1][2]["v"] = slabs[1][2]["v"].copy()
    slabs[1][2]["v"][-nx] += 1.0   # slab 1's copy of face row 7 differs from slab 2's
    try:
        cfdamd.assemble_slabs(slabs, nx)
    except ValueError as e:
        assert "face row 7" in str(e)
    else:
        raise AssertionError("a differing shared face row must raise")
