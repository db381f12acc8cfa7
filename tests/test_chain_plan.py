"""CPU: the chained march's row plan (cfd_plan_chain, cfd_jacobi_chain.hip).
Every row of [out_lo, out_hi) belongs to exactly one row group; chain groups
have 4D + 2 - 2T rows with D >= 2T - 1 (opening and closing hand-offs never
overlap); the edge groups keep >= 8 rows per wave and hold every row whose
march could reach a global boundary row (chain waves carry no row patches);
the chain groups and the edge groups take the same number of slots."""
import ctypes as C

import pytest

T = 8


def _plan(nx, ny, n_cu=256, occ=3, lo=1, hi=None):
    import cfdamd
    lib = cfdamd.load()
    hi = ny - 1 if hi is None else hi
    v = [C.c_int() for _ in range(5)]
    ok = lib.cfd_plan_chain(nx, ny, n_cu, occ, lo, hi, *(C.byref(x) for x in v))
    assert ok in (0, 1)
    return ok, lo, hi, [x.value for x in v]


@pytest.mark.parametrize("nx,ny", [(4096, 4096), (8192, 8192), (256, 128), (800, 264), (1024, 1024),
                                   (3000, 1777), (16384, 1088), (640, 4000), (130, 1000)])
def test_chain_plan_covers_rows(nx, ny):
    ok, lo, hi, (nwc, ngrp, d0, nhi, elo) = _plan(nx, ny)
    if not ok:
        return
    M = ngrp - 2
    assert ngrp >= 3 and d0 >= 2 * T - 1 and 0 <= nhi <= M
    rows = [4 * (d0 + (k < nhi)) + 2 - 2 * T for k in range(M)]
    ehi = (hi - lo) - elo - sum(rows)
    assert elo >= 32 and ehi >= 32
    # chain cones stay off the global boundary rows 0, 1, ny-2, ny-1
    assert lo + elo - T - 1 > 1 and hi - ehi + T < ny - 2
    # balance: an edge wave of D + 1 - T rows takes the chain's D + T + 1 slots
    for e in (elo, ehi):
        assert abs(e / 4 - (d0 + 1 - T)) <= 0.25 * (d0 + 1 - T) + 8, (e, d0)
    assert nwc == -(-(nx // 2) // (64 - 2 * ((T + 1) // 2)))


def test_chain_plan_bench_grid():
    """The bench's 4096^2 cavity at 3 workgroups per CU: 20 row groups per
    column (one round of 256 x 3 workgroups over 37 wave columns)."""
    ok, lo, hi, (nwc, ngrp, d0, nhi, elo) = _plan(4096, 4096)
    assert ok and nwc == 37 and ngrp == 20 and d0 >= 50


def test_chain_plan_refuses_small_grids():
    assert _plan(64, 48)[0] == 0
    assert _plan(4096, 40)[0] == 0
