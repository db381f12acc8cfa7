"""Generate the golden fixtures under tests/golden/ (test infrastructure).

The reference itself cannot run here (Rust toolchain absent),
so the fixtures are outputs of the C restatement oracle/cfd_oracle.c; this
script refuses to write a fixture unless the independent numpy restatement
oracle/np_model.py reproduces it bit for bit.  PARITY UNPINNED against the
reference binary — see DESIGN.md "Oracle".

    python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from np_model import NpModel  # noqa: E402
from oracle import OracleModel  # noqa: E402

F = np.float32
FIELDS = ("u", "v", "p", "u_star", "v_star", "p_prime", "rhs")
NPF = {"u": "u", "v": "v", "p": "p", "u_star": "u_star", "v_star": "v_star",
       "p_prime": "pp", "rhs": "rhs"}

# name -> (grid kwargs, params kwargs, steps)
CHANNEL = dict(lx=30.0, ly=10.0, cylinder=(7.5, 5.0, 0.75))
RUNS = {
    "run_channel_128x64_fo": (dict(nx=128, ny=64, **CHANNEL), dict(scheme=0), 10),
    "run_channel_128x64_so": (dict(nx=128, ny=64, **CHANNEL), dict(scheme=1), 10),
    "run_channel_128x64_parabolic": (dict(nx=128, ny=64, **CHANNEL),
                                     dict(scheme=0, inlet_profile=1), 10),
    "run_cavity_128x128_re100": (dict(nx=128, ny=128, lx=1.0, ly=1.0, cylinder=None),
                                 dict(bc_kind=1, viscosity=0.01), 20),
    "run_cavity_128x128_fixed50": (dict(nx=128, ny=128, lx=1.0, ly=1.0, cylinder=None),
                                   dict(bc_kind=1, viscosity=0.01, jacobi_iters=50,
                                        corrector_passes=0, tol_enabled=0), 20),
}
KATS = {  # name -> (grid kwargs, scheme)
    "kat_32x16_fo": (dict(nx=32, ny=16, lx=30.0, ly=10.0, cylinder=(7.5, 5.0, 2.5)), 0),
    "kat_32x16_so": (dict(nx=32, ny=16, lx=30.0, ly=10.0, cylinder=(7.5, 5.0, 2.5)), 1),
}
KAT_DT = F(0.01)


def pair(g, p):
    o = OracleModel(g["nx"], g["ny"], g["lx"], g["ly"], cylinder=g["cylinder"], **p)
    n = NpModel(g["nx"], g["ny"], g["lx"], g["ly"], cylinder=g["cylinder"], **p)
    return o, n


def check(tag, o, n, fields=FIELDS):
    for f in fields:
        a, b = o.field(f), getattr(n, NPF[f])
        if not np.array_equal(a.view(np.uint32), b.view(np.uint32)):
            raise SystemExit(f"{tag}: C and numpy restatements disagree on {f}")


def kat(name, g, scheme, seed):
    o, n = pair(g, dict(scheme=scheme))
    rng = np.random.default_rng(seed)
    inp = {}
    for f in ("u", "v", "u_star", "v_star", "p_prime", "p"):
        x = rng.uniform(-1, 1, o.field(f).size).astype(F)
        o.field(f)[:] = x
        getattr(n, NPF[f])[:] = x
        inp["in_" + f] = x.copy()
    out = {}
    o.u_predictor(KAT_DT); n.u_predictor(KAT_DT); check(name, o, n, ("u_star",))
    out["out_u_star"] = o.field("u_star").copy()
    o.v_predictor(KAT_DT); n.v_predictor(KAT_DT); check(name, o, n, ("v_star",))
    out["out_v_star"] = o.field("v_star").copy()
    o.divergence(KAT_DT); n.divergence(KAT_DT); check(name, o, n, ("rhs",))
    out["out_rhs"] = o.field("rhs").copy()
    r1, r2 = o.jacobi(), n.jacobi()
    assert np.float32(r1) == r2
    check(name, o, n, ("p_prime",))
    out["out_p_prime"] = o.field("p_prime").copy()
    out["out_jacobi_residual"] = np.array([r1], F)
    out["out_jacobi_sweeps"] = np.array([o.scalars().jacobi_sweeps_total], np.int64)
    o.corrector(KAT_DT); n.corrector(KAT_DT); check(name, o, n, ("u", "v", "p"))
    out["out_corr_u"], out["out_corr_v"], out["out_corr_p"] = (
        o.field("u").copy(), o.field("v").copy(), o.field("p").copy())
    o.boundary(); n.boundary(); check(name, o, n, ("u", "v"))
    out["out_bc_u"], out["out_bc_v"] = o.field("u").copy(), o.field("v").copy()
    out["mask_u"], out["mask_v"] = o.mask("u").copy(), o.mask("v").copy()
    return {**inp, **out}


def run(name, g, p, steps):
    o, n = pair(g, p)
    for _ in range(steps):
        o.update()
        n.update()
    check(name, o, n)
    s = o.scalars()
    assert s.dt == n.dt and s.p == n.res_p and s.u == n.res_u and s.v == n.res_v
    out = {f: o.field(f).copy() for f in FIELDS}
    out["scalars_f32"] = np.array([s.time, s.dt, s.p, s.u, s.v], F)
    out["scalars_i64"] = np.array([s.step, s.jacobi_sweeps_total], np.int64)
    return out


def main():
    manifest = {"generator": "tests/golden/make_golden.py",
                "oracle": "oracle/cfd_oracle.c (cross-checked bitwise by oracle/np_model.py)",
                "parity": "unpinned against the reference binary (Rust toolchain absent)",
                "kat_dt": float(KAT_DT), "fixtures": {}}
    for k, (name, (g, scheme)) in enumerate(KATS.items()):
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **kat(name, g, scheme, 1234 + k))
        manifest["fixtures"][name] = {"grid": g, "scheme": scheme, "seed": 1234 + k,
                                      "kind": "kat"}
    for name, (g, p, steps) in RUNS.items():
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **run(name, g, p, steps))
        manifest["fixtures"][name] = {"grid": g, "params": p, "steps": steps, "kind": "run"}
    with open(os.path.join(HERE, "manifest.json"), "w") as fh:
        json.dump(manifest, fh, indent=1)
    print("wrote", len(manifest["fixtures"]), "fixtures")


if __name__ == "__main__":
    main()
