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
