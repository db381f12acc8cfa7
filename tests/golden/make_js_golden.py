"""Golden vectors for the multigrid pressure solver, produced by the
reference's OWN JavaScript (test infrastructure).

The reference's multigrid solver lives in its JavaScript variant
(/root/reference/index.html): mgSmooth / mgRestrict / mgProlongate /
mgVcycle (:1344-1470) and the multigrid branch of the pressure correction
(:775-795).  Those functions are pure (typed arrays in, typed arrays out), so
this script reads their text from the reference at generation time, runs them
under node (v12, present in this image) on seeded inputs, and stores inputs
and outputs as small fixtures tests/golden/js_mg_*.npz.  No reference source
is written to the repository: only the numbers.  The GPU path and the C
restatement (oracle/cfd_oracle_solvers.c) must reproduce them bit for bit.

    python tests/golden/make_js_golden.py
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_HTML = "/root/reference/index.html"

# name -> (nx, ny, lx, ly): dx = f32(lx) / f32(nx) as the model forms it (src/app.rs:37-38)
CASES = {
    "js_mg_64x48": (64, 48, 4.0 / 3.0, 1.0),          # non-power-of-two spacing
    "js_mg_128x128": (128, 128, 1.0, 1.0),            # power-of-two spacing (cavity)
    "js_mg_136x72": (136, 72, 30.0, 10.0),            # odd coarse sizes (17, 9, 5, 3)
    "js_mg_40x24": (40, 24, 30.0, 10.0),              # shallow hierarchy
}

HARNESS = r"""
'use strict';
const fs = require('fs');
const fnText = fs.readFileSync(process.argv[2], 'utf8');
const branchText = fs.readFileSync(process.argv[3], 'utf8');
const job = JSON.parse(fs.readFileSync(process.argv[4], 'utf8'));
const dir = process.argv[5];
const mg = new Function(fnText +
  '\nreturn {mgSmooth, mgRestrict, mgProlongate, mgVcycle};')();
const { mgSmooth, mgRestrict, mgProlongate, mgVcycle } = mg;
function rd(name, n) {
  const b = fs.readFileSync(dir + '/' + name);
  return new Float32Array(b.buffer.slice(b.byteOffset, b.byteOffset + 4 * n));
}
function wr(name, a) { fs.writeFileSync(dir + '/' + name, Buffer.from(a.buffer)); }
const nx = job.nx, ny = job.ny, dx = job.dx, dy = job.dy;
const nx_c = Math.floor((nx + 1) / 2), ny_c = Math.floor((ny + 1) / 2);
const p = rd('p.bin', nx * ny), rhs = rd('rhs.bin', nx * ny), coarse = rd('coarse.bin', nx_c * ny_c);
const s = p.slice(); mgSmooth(s, rhs, nx, ny, dx, dy, 5); wr('smooth.bin', s);
wr('restrict.bin', mgRestrict(p, nx, ny, nx_c, ny_c));
wr('prolong.bin', mgProlongate(coarse, nx_c, ny_c, nx, ny));
const v = p.slice(); mgVcycle(v, rhs, nx, ny, dx, dy); wr('vcycle.bin', v);
// the multigrid branch of the pressure correction, with the script's own names
const branch = new Function('pPrime', 'rhs', 'Nx', 'Ny', 'dx', 'dy', 'mgVcycle',
  'let lastPResidual;\n' + branchText + '\nreturn lastPResidual;');
const pPrime = new Float32Array(nx * ny).fill(7);   // the branch zeroes it itself
const res = branch(pPrime, rhs, nx, ny, dx, dy, mgVcycle);
wr('solve.bin', pPrime);
fs.writeFileSync(dir + '/residual.json', JSON.stringify({ residual: res }));
"""


def extract():
    html = open(REF_HTML).read()
    a = html.index("// Simple Jacobi smoother for multigrid")
    b = html.index("// **************** NEW: Tracer Particles")
    fns = html[a:b]
    c0 = html.index('} else if (currentPressureSolver === "multigrid") {')
    c0 = html.index("{", c0) + 1
    c1 = html.index("} else { // Default: Pressure Correction using Jacobi", c0)
    return fns, html[c0:c1]


def main():
    fns, branch = extract()
    for name in ("mgSmooth", "mgRestrict", "mgProlongate", "mgVcycle"):
        assert f"function {name}(" in fns, name
    assert "mgVcycle(pPrime, rhs, Nx, Ny, dx, dy)" in branch
    manifest = {"generator": "tests/golden/make_js_golden.py",
                "source": "reference index.html:1344-1470 (mg*), :775-795 (multigrid branch), "
                          "executed by node " + subprocess.run(["node", "--version"],
                                                               capture_output=True,
                                                               text=True).stdout.strip(),
                "fixtures": {}}
    for k, (name, (nx, ny, lx, ly)) in enumerate(CASES.items()):
        dx = np.float32(lx) / np.float32(nx)
        dy = np.float32(ly) / np.float32(ny)
        rng = np.random.default_rng(4242 + k)
        nx_c, ny_c = (nx + 1) // 2, (ny + 1) // 2
        p = rng.uniform(-1, 1, nx * ny).astype(np.float32)
        rhs = (rng.uniform(-1, 1, nx * ny) * 100.0).astype(np.float32)
        coarse = rng.uniform(-1, 1, nx_c * ny_c).astype(np.float32)
        with tempfile.TemporaryDirectory() as d:
            for fn, txt in (("fns.js", fns), ("branch.js", branch), ("harness.js", HARNESS)):
                open(os.path.join(d, fn), "w").write(txt)
            for fn, arr in (("p.bin", p), ("rhs.bin", rhs), ("coarse.bin", coarse)):
                arr.tofile(os.path.join(d, fn))
            json.dump({"nx": nx, "ny": ny, "dx": float(dx), "dy": float(dy)},
                      open(os.path.join(d, "job.json"), "w"))
            subprocess.run(["node", os.path.join(d, "harness.js"), os.path.join(d, "fns.js"),
                            os.path.join(d, "branch.js"), os.path.join(d, "job.json"), d],
                           check=True)
            out = {f: np.fromfile(os.path.join(d, f + ".bin"), np.float32)
                   for f in ("smooth", "restrict", "prolong", "vcycle", "solve")}
            res = json.load(open(os.path.join(d, "residual.json")))["residual"]
        np.savez_compressed(os.path.join(HERE, name + ".npz"), in_p=p, in_rhs=rhs,
                            in_coarse=coarse, out_residual_f64=np.array([res], np.float64),
                            **{"out_" + f: a for f, a in out.items()})
        manifest["fixtures"][name] = {"nx": nx, "ny": ny, "lx": lx, "ly": ly,
                                      "dx": float(dx), "dy": float(dy), "seed": 4242 + k}
        print(name, "residual", res)
    json.dump(manifest, open(os.path.join(HERE, "js_manifest.json"), "w"), indent=1)


if __name__ == "__main__":
    sys.exit(main())
