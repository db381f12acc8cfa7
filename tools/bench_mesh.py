#!/usr/bin/env python3
"""Mesh::from_quad_tree (mesh.rs:51-227) on one MI355X against the CPU
restatement (oracle/quad_mesh_ref.py, numpy-vectorised neighbour search, one
process), for the reference's default polygon (views/mesh_view.rs:140-152)
at shrinking feature sizes.  One JSON line per size.

    python tools/bench_mesh.py [--cpu-max-cells 60000]

Work unit: a cell pair of the O(n^2) face-neighbour search (n^2 - n per
build); the GPU time is the device time of the build's kernels (HIP events),
the tesselation (host) is reported beside it.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cfd-demo_amd"), os.path.join(ROOT, "oracle")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cpu-max-cells", type=int, default=20000)
    a = ap.parse_args()
    from cfdamd import quad_mesh as qm
    for feature, max_cell in ((0.1, 0.5), (0.02, 0.5), (0.01, 0.25), (0.005, 0.1)):
        poly = qm.default_polygon()
        t0 = time.perf_counter()
        tree = qm.tesselate(poly, feature, max_cell)
        t_tess = time.perf_counter() - t0
        qm.Mesh.from_quad_tree(tree, poly)            # warm-up (module load, allocations)
        mesh = qm.Mesh.from_quad_tree(tree, poly)
        n = mesh.num_cells
        out = {"feature_size": feature, "max_cell_size": max_cell, "leaves": tree.n_leaves,
               "cells": n, "gpu_build_ms": mesh.build_ms,
               "gpu_pairs_per_s": (n * n - n) / (mesh.build_ms * 1e-3),
               "host_tesselate_ms": 1e3 * t_tess}
        if n <= a.cpu_max_cells:
            import quad_mesh_ref as qr
            op = qr.default_polygon()
            otree = qr.tesselate(op, feature, max_cell)
            t0 = time.perf_counter()
            qr.Mesh(otree, op)
            el = time.perf_counter() - t0
            out["cpu_port_build_ms"] = 1e3 * el
            out["cpu_port"] = "oracle/quad_mesh_ref.py (numpy over j, 1 process)"
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
