"""CPU: the product library loads and exports every entry point declared in
include/cfd.h; host-only entry points behave (no GPU compute here)."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "cfd.h")


def header_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(cfd_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from cfdamd import _lib
    L = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert sorted(_lib.EXPORTS) == syms
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    for s in syms:
        assert re.search(rf"\bT {s}\b", out), s


def test_library_is_gfx950_code_object():
    from cfdamd import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_defaults_mirror_reference():
    from cfdamd import _lib
    L = _lib.load()
    p = _lib.CfdParams()
    L.cfd_default_params(C.byref(p))
    # SimulationParams::default (model.rs:44-55) and the hardcoded solver constants
    assert (p.dt, p.target_inlet_velocity) == (pytest.approx(0.005), 1.0)
    assert p.viscosity == pytest.approx(1e-6)
    assert (p.velocity_scheme, p.inlet_profile, p.pressure_solver) == (0, 0, 0)
    assert (p.jacobi_iters, p.corrector_passes, p.tol_enabled) == (50, 20, 1)
    assert p.p_tol == pytest.approx(1e-4)
    g = _lib.CfdGrid()
    L.cfd_default_grid(C.byref(g))
    # default_grid (src/app.rs:32-53)
    assert (g.nx, g.ny, g.lx, g.ly, g.has_cylinder) == (800, 264, 30.0, 10.0, 1)
    assert (g.cylinder_x, g.cylinder_y, g.cylinder_radius) == (7.5, 5.0, 0.75)
    assert L.cfd_abi_version() == 1


def test_python_mirror_defaults():
    import cfdamd
    p = cfdamd.SimulationParams()
    assert p._c().jacobi_iters == 50 and p.velocity_scheme == cfdamd.VelocityScheme.FirstOrder
    g = cfdamd.default_grid()
    assert (g.nx, g.ny, g.obstacle.radius) == (800, 264, 0.75)
    assert g.dx == pytest.approx(30.0 / 800)
    cav = cfdamd.SimulationParams.cavity(1000.0, 200)
    assert cav.viscosity == pytest.approx(1e-3) and cav.bc_kind == cfdamd.BoundaryKind.Cavity


def test_errors_are_loud_without_a_device():
    """No HIP device in this container: creation must fail with a status and a
    message, never silently compute elsewhere."""
    import cfdamd
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    with pytest.raises(cfdamd.CfdError) as e:
        cfdamd.Model(cfdamd.Grid(64, 32, 1.0, 1.0), cfdamd.SimulationParams())
    assert e.value.code in (-1, -2)


def test_invalid_arguments_rejected_before_device():
    import cfdamd
    for g in (cfdamd.Grid(100, 64, 1.0, 1.0), cfdamd.Grid(64, 2, 1.0, 1.0)):
        with pytest.raises(cfdamd.CfdError) as e:
            cfdamd.Model(g, cfdamd.SimulationParams())
        assert e.value.code == -1


def test_solver_choice_validated_before_device():
    """pressure_solver 0..2 (all three run on slabs since r2:
    tests/test_gpu_sharded.py); anything else is rejected before the device."""
    import cfdamd
    with pytest.raises(cfdamd.CfdError) as e:
        cfdamd.Model(cfdamd.Grid(64, 32, 1.0, 1.0),
                     cfdamd.SimulationParams(pressure_solver=3))
    assert e.value.code == -1
    with pytest.raises(cfdamd.CfdError) as e:
        cfdamd.Model(cfdamd.Grid(64, 32, 1.0, 1.0), cfdamd.SimulationParams(pressure_solver=-1),
                     n_ranks=2, rank=0, unique_id=bytes(128))
    assert e.value.code == -1