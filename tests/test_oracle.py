"""CPU: the oracle is pinned by (a) bitwise agreement of two independent
restatements (C: oracle/cfd_oracle.c, numpy: oracle/np_model.py) and (b) the
committed golden fixtures.  The reference itself cannot be built here (no
Rust toolchain), so parity against it is unpinned (DESIGN.md "Oracle")."""
import json
import os

import numpy as np
import pytest

from _util import assert_bitwise
from np_model import NpModel
from oracle import OracleModel

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
MANIFEST = json.load(open(os.path.join(GOLD, "manifest.json")))
NPF = {"u": "u", "v": "v", "p": "p", "u_star": "u_star", "v_star": "v_star",
       "p_prime": "pp", "rhs": "rhs"}


def pair(nx, ny, lx, ly, cylinder=None, **p):
    return (OracleModel(nx, ny, lx, ly, cylinder=cylinder, **p),
            NpModel(nx, ny, lx, ly, cylinder=cylinder, **p))


def same(o, n, fields=tuple(NPF)):
    for f in fields:
        assert_bitwise(f, o.field(f), getattr(n, NPF[f]))


@pytest.mark.parametrize("scheme", [0, 1])
@pytest.mark.parametrize("cyl", [None, (7.5, 5.0, 2.5), (0.5, 9.9, 1.2)])
def test_phases_agree_on_random_state(scheme, cyl):
    o, n = pair(40, 24, 30.0, 10.0, cylinder=cyl, scheme=scheme)
    assert np.array_equal(o.mask("u"), n.mask_u) and np.array_equal(o.mask("v"), n.mask_v)
    rng = np.random.default_rng(11 + scheme)
    for f in ("u", "v", "u_star", "v_star", "p_prime", "p"):
        x = rng.uniform(-1, 1, o.field(f).size).astype(np.float32)
        o.field(f)[:] = x
        getattr(n, NPF[f])[:] = x
    dt = np.float32(0.013)
    o.u_predictor(dt); n.u_predictor(dt); same(o, n, ("u_star",))
    o.v_predictor(dt); n.v_predictor(dt); same(o, n, ("v_star",))
    o.divergence(dt); n.divergence(dt); same(o, n, ("rhs",))
    assert np.float32(o.jacobi()) == n.jacobi()
    same(o, n, ("p_prime",))
    o.corrector(dt); n.corrector(dt); same(o, n, ("u", "v", "p"))
    o.boundary(); n.boundary(); same(o, n, ("u", "v"))


@pytest.mark.parametrize("cfg", [
    dict(nx=64, ny=40, lx=30.0, ly=10.0, cylinder=(7.5, 5.0, 2.0), scheme=0),
    dict(nx=64, ny=40, lx=30.0, ly=10.0, cylinder=(7.5, 5.0, 2.0), scheme=1, inlet_profile=1),
    dict(nx=48, ny=48, lx=1.0, ly=1.0, bc_kind=1, viscosity=0.01, scheme=1),
    dict(nx=32, ny=16, lx=1.0, ly=1.0, bc_kind=1, viscosity=0.01, jacobi_iters=13,
         corrector_passes=3, tol_enabled=0),
    dict(nx=16, ny=4, lx=1.0, ly=1.0),
])
def test_full_steps_agree(cfg):
    o, n = pair(**cfg)
    for _ in range(8):
        o.update(); n.update()
        s = o.scalars()
        assert (s.step, np.float32(s.dt), np.float32(s.p), np.float32(s.u), np.float32(s.v)) == \
            (n.step, n.dt, n.res_p, n.res_u, n.res_v)
    same(o, n)


def test_jacobi_residual_excludes_tail_columns():
    """Q6: a disturbance only in the scalar-tail columns nx-7..nx-1 moves p'
    but never the returned residual (model.rs:755-772)."""
    o = OracleModel(32, 16, 1.0, 1.0, jacobi_iters=1)
    rhs = o.field("rhs")
    rhs[:] = 0
    rhs[5 * 32 + 27] = 1e3    # column 27 = nx-5
    assert o.jacobi() == 0.0
    assert o.field("p_prime")[5 * 32 + 27] != 0.0
    o2 = OracleModel(32, 16, 1.0, 1.0, jacobi_iters=1)
    o2.field("rhs")[5 * 32 + 24] = 1e3   # column 24 = nx-8: inside the chunks
    assert o2.jacobi() > 0.0


def test_corrector_tail_association():
    """Q9: columns nx-7..nx-1 use (dt*dp)/dx, others dt*(dp/dx)."""
    o = OracleModel(16, 4, 3.0, 1.0)
    pp = o.field("p_prime")
    rng = np.random.default_rng(3)
    pp[:] = rng.uniform(-1, 1, pp.size).astype(np.float32)
    o.field("u_star")[:] = 0
    dt = np.float32(0.0123)
    o.corrector(dt)
    u = o.field("u").reshape(4, 17)
    P = pp.reshape(4, 16)
    dx = np.float32(np.float32(3.0) / np.float32(16))
    for i in range(1, 16):
        dp = P[1, i] - P[1, i - 1]
        corr = (dt * dp) / dx if i >= 16 - 7 else dt * (dp / dx)
        assert np.float32(u[1, i]).view(np.uint32) == np.float32(np.float32(0) - corr).view(np.uint32)


@pytest.mark.parametrize("name", sorted(MANIFEST["fixtures"]))
def test_oracle_reproduces_golden(name):
    meta = MANIFEST["fixtures"][name]
    fx = np.load(os.path.join(GOLD, name + ".npz"))
    g = meta["grid"]
    if meta["kind"] == "kat":
        o = OracleModel(g["nx"], g["ny"], g["lx"], g["ly"], cylinder=g["cylinder"],
                        scheme=meta["scheme"])
        for f in ("u", "v", "u_star", "v_star", "p_prime", "p"):
            o.field(f)[:] = fx["in_" + f]
        dt = np.float32(MANIFEST["kat_dt"])
        o.u_predictor(dt); assert_bitwise("u_star", o.field("u_star"), fx["out_u_star"])
        o.v_predictor(dt); assert_bitwise("v_star", o.field("v_star"), fx["out_v_star"])
        o.divergence(dt); assert_bitwise("rhs", o.field("rhs"), fx["out_rhs"])
        assert np.float32(o.jacobi()) == fx["out_jacobi_residual"][0]
        assert_bitwise("p_prime", o.field("p_prime"), fx["out_p_prime"])
        o.corrector(dt)
        assert_bitwise("u", o.field("u"), fx["out_corr_u"])
        o.boundary()
        assert_bitwise("v", o.field("v"), fx["out_bc_v"])
    else:
        o = OracleModel(g["nx"], g["ny"], g["lx"], g["ly"], cylinder=g["cylinder"],
                        **meta["params"])
        for _ in range(meta["steps"]):
            o.update()
        for f in ("u", "v", "p", "u_star", "v_star", "p_prime", "rhs"):
            assert_bitwise(f, o.field(f), fx[f])
        s = o.scalars()
        assert np.array_equal(np.array([s.time, s.dt, s.p, s.u, s.v], np.float32),
                              fx["scalars_f32"])
