"""ctypes binding of include/cfd.h (libcfd_amd.so, built in-tree by
cfd-demo_amd/Makefile).  No fallback: if the HIP library is missing or cannot
load, every entry point raises."""
from __future__ import annotations

import ctypes as C
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
# CFD_LIB: an alternative build of the same library (tools/build_variants.sh, tuning only)
LIB_PATH = os.environ.get("CFD_LIB") or os.path.join(ROOT, "lib", "libcfd_amd.so")

# Every entry point include/cfd.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "cfd_default_params", "cfd_default_grid", "cfd_create", "cfd_rccl_unique_id",
    "cfd_create_sharded", "cfd_local_hub_create", "cfd_local_hub_destroy",
    "cfd_create_sharded_local", "cfd_device_count", "cfd_get_comm_size", "cfd_get_slab", "cfd_update", "cfd_update_n", "cfd_piso_step",
    "cfd_pressure_solve", "cfd_run_phase", "cfd_set_params", "cfd_get_snapshot",
    "cfd_get_residuals", "cfd_get_state", "cfd_set_state", "cfd_get_masks", "cfd_synchronize",
    "cfd_profile_sweeps", "cfd_timing_begin", "cfd_timing_end", "cfd_timing_phases",
    "cfd_timing_phase_ms", "cfd_timing_exchange_ms", "cfd_get_halo_depth",
    "cfd_get_kernel_config", "cfd_get_jacobi_kernel", "cfd_get_persist_blocks", "cfd_get_persist_steals", "cfd_get_persist_sums", "cfd_get_recoveries", "cfd_get_comm_calls", "cfd_get_resident_solves", "cfd_get_jacobi_geometry", "cfd_plan_slab", "cfd_plan_sweep", "cfd_plan_halo", "cfd_plan_block", "cfd_plan_overlap",
    "cfd_render", "cfd_derive_field", "cfd_last_error", "cfd_abi_version", "cfd_destroy",
    "cfd_get_config", "cfd_run_start", "cfd_run_stop", "cfd_run_pause", "cfd_run_resume",
    "cfd_run_set_params", "cfd_run_request_snapshot", "cfd_run_last_snapshot",
    "cfd_run_new_residuals", "cfd_run_status", "cfd_run_steps",
    "cfd_polygon_new", "cfd_polygon_new_rect", "cfd_polygon_new_regular", "cfd_polygon_add_hole",
    "cfd_polygon_contains_point", "cfd_polygon_intersects_aabb",
    "cfd_polygon_edges_intersect_aabb", "cfd_polygon_bounding_box",
    "cfd_polygon_bounding_square", "cfd_polygon_edges", "cfd_polygon_destroy",
    "cfd_geom_do_intersect", "cfd_geom_segment_intersection", "cfd_geom_intersect_quad_edge",
    "cfd_tesselate", "cfd_quadtree_size", "cfd_quadtree_nodes", "cfd_quadtree_destroy",
    "cfd_mesh_from_quadtree", "cfd_mesh_sizes", "cfd_mesh_cells", "cfd_mesh_neighbors",
    "cfd_mesh_intersections", "cfd_mesh_full_bounding_box", "cfd_mesh_build_ms",
    "cfd_mesh_destroy",
]


class CfdGrid(C.Structure):
    _fields_ = [("nx", C.c_uint64), ("ny", C.c_uint64), ("lx", C.c_float), ("ly", C.c_float),
                ("has_cylinder", C.c_int32), ("cylinder_x", C.c_float),
                ("cylinder_y", C.c_float), ("cylinder_radius", C.c_float)]


class CfdParams(C.Structure):
    _fields_ = [("dt", C.c_float), ("viscosity", C.c_float),
                ("target_inlet_velocity", C.c_float), ("velocity_scheme", C.c_int32),
                ("inlet_profile", C.c_int32), ("pressure_solver", C.c_int32),
                ("jacobi_iters", C.c_int32), ("corrector_passes", C.c_int32),
                ("tol_enabled", C.c_int32), ("p_tol", C.c_float), ("bc_kind", C.c_int32)]


class CfdResiduals(C.Structure):
    _fields_ = [("simulation_step", C.c_uint64), ("simulation_time", C.c_float),
                ("dt", C.c_float), ("p", C.c_float), ("u", C.c_float), ("v", C.c_float),
                ("step_time_s", C.c_double), ("piso_substeps", C.c_uint32),
                ("jacobi_sweeps_total", C.c_uint64)]


FP = C.POINTER(C.c_float)


class CfdState(C.Structure):
    _fields_ = [("u", FP), ("v", FP), ("p", FP), ("u_star", FP), ("v_star", FP),
                ("p_prime", FP), ("rhs", FP), ("dt", C.c_float), ("simulation_time", C.c_float),
                ("simulation_step", C.c_uint64), ("last_p_residual", C.c_float),
                ("last_u_residual", C.c_float), ("last_v_residual", C.c_float),
                ("jacobi_sweeps_total", C.c_uint64)]


class CfdPoint(C.Structure):
    _fields_ = [("x", C.c_double), ("y", C.c_double)]


class CfdAabb(C.Structure):
    _fields_ = [("center", CfdPoint), ("half_width", C.c_double), ("half_height", C.c_double)]


# cfd_status (include/cfd.h)
CFD_EINVAL, CFD_EHIP, CFD_ERCCL, CFD_ESTATE, CFD_ENONFINITE, CFD_ETIMEOUT = -1, -2, -3, -4, -5, -6


class CfdError(RuntimeError):
    def __init__(self, fn: str, code: int, msg: str):
        super().__init__(f"{fn} failed ({code}): {msg}")
        self.code = code


_lib = None


def load():
    """Load libcfd_amd.so; raise (never fall back) when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"HIP library {LIB_PATH} not built: run `make -C {ROOT}` "
            "(or __graft_entry__.build()). There is no CPU fallback.")
    L = C.CDLL(LIB_PATH)
    vp, i32, f32 = C.c_void_p, C.c_int, C.c_float
    sig = {
        "cfd_default_params": (None, [C.POINTER(CfdParams)]),
        "cfd_default_grid": (None, [C.POINTER(CfdGrid)]),
        "cfd_create": (i32, [C.POINTER(CfdGrid), C.POINTER(CfdParams), i32, C.POINTER(vp)]),
        "cfd_rccl_unique_id": (i32, [C.c_char_p]),
        "cfd_create_sharded": (i32, [C.POINTER(CfdGrid), C.POINTER(CfdParams), i32, i32, i32,
                                     C.c_char_p, C.POINTER(vp)]),
        "cfd_local_hub_create": (vp, [i32]),
        "cfd_local_hub_destroy": (None, [vp]),
        "cfd_create_sharded_local": (i32, [C.POINTER(CfdGrid), C.POINTER(CfdParams), i32, i32,
                                           i32, vp, C.POINTER(vp)]),
        "cfd_device_count": (i32, [C.POINTER(i32)]),
        "cfd_get_comm_size": (i32, [vp, C.POINTER(i32)]),
        "cfd_get_slab": (i32, [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
        "cfd_update": (i32, [vp]),
        "cfd_update_n": (i32, [vp, i32]),
        "cfd_piso_step": (i32, [vp, f32]),
        "cfd_pressure_solve": (i32, [vp, FP]),
        "cfd_run_phase": (i32, [vp, i32, f32]),
        "cfd_set_params": (i32, [vp, C.POINTER(CfdParams)]),
        "cfd_get_snapshot": (i32, [vp, FP, FP, FP, FP]),
        "cfd_get_residuals": (i32, [vp, C.POINTER(CfdResiduals)]),
        "cfd_get_state": (i32, [vp, C.POINTER(CfdState)]),
        "cfd_set_state": (i32, [vp, C.POINTER(CfdState)]),
        "cfd_get_masks": (i32, [vp, C.POINTER(C.c_uint8), C.POINTER(C.c_uint8)]),
        "cfd_synchronize": (i32, [vp]),
        "cfd_profile_sweeps": (i32, [vp, i32, C.POINTER(C.c_double)]),
        "cfd_timing_begin": (i32, [vp]),
        "cfd_timing_end": (i32, [vp, C.POINTER(C.c_double), C.POINTER(C.c_uint64),
                                 C.POINTER(C.c_double), C.POINTER(C.c_uint64)]),
        "cfd_timing_phases": (i32, [vp, i32]),
        "cfd_timing_phase_ms": (i32, [vp, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
        "cfd_timing_exchange_ms": (i32, [vp, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]),
        "cfd_get_halo_depth": (i32, [vp]),
        "cfd_get_kernel_config": (i32, [vp, C.POINTER(i32), C.POINTER(i32)]),
        "cfd_get_jacobi_kernel": (i32, [vp, C.POINTER(i32), C.c_char_p, C.c_size_t]),
        "cfd_get_persist_blocks": (i32, [vp, C.POINTER(i32)]),
        "cfd_get_persist_steals": (i32, [vp, C.POINTER(C.c_uint64)]),
        "cfd_get_persist_sums": (i32, [vp, C.POINTER(C.c_uint64)]),
        "cfd_get_recoveries": (i32, [vp, C.POINTER(C.c_uint64)]),
        "cfd_get_comm_calls": (i32, [vp, C.POINTER(C.c_uint64)]),
        "cfd_get_resident_solves": (i32, [vp, C.POINTER(C.c_uint64)]),
        "cfd_get_jacobi_geometry": (i32, [vp, i32, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32),
                                          C.POINTER(i32)]),
        "cfd_plan_slab": (i32, [C.c_uint64, i32, i32, C.POINTER(C.c_uint64),
                                C.POINTER(C.c_uint64)]),
        "cfd_plan_sweep": (i32, [i32, i32, i32, i32, i32, i32, C.POINTER(i32), C.POINTER(i32),
                                 C.POINTER(i32)]),
        "cfd_plan_halo": (i32, [i32, i32, i32, i32, i32, C.POINTER(i32)]),
        "cfd_plan_overlap": (i32, [i32, i32, i32, i32, i32, i32, C.POINTER(i32)]),
        "cfd_plan_block": (i32, [i32, i32, i32, i32, i32, i32, i32, C.POINTER(i32),
                                 C.POINTER(i32), C.POINTER(i32), C.POINTER(i32)]),
        "cfd_render": (i32, [vp, i32, C.POINTER(C.c_uint8), FP]),
        "cfd_derive_field": (i32, [vp, i32, FP, FP]),
        "cfd_last_error": (C.c_char_p, []),
        "cfd_abi_version": (i32, []),
        "cfd_destroy": (None, [vp]),
        "cfd_get_config": (i32, [vp, C.POINTER(CfdGrid), C.POINTER(CfdParams)]),
        "cfd_run_start": (i32, [vp, C.POINTER(vp)]),
        "cfd_run_stop": (i32, [vp]),
        "cfd_run_pause": (i32, [vp]),
        "cfd_run_resume": (i32, [vp]),
        "cfd_run_set_params": (i32, [vp, C.POINTER(CfdParams)]),
        "cfd_run_request_snapshot": (i32, [vp]),
        "cfd_run_last_snapshot": (i32, [vp, FP, FP, FP, FP, C.POINTER(i32), C.POINTER(i32)]),
        "cfd_run_new_residuals": (i32, [vp, C.POINTER(CfdResiduals), i32, C.POINTER(i32)]),
        "cfd_run_status": (i32, [vp, C.c_char_p, C.c_size_t]),
        "cfd_run_steps": (C.c_uint64, [vp]),
        # quadtree mesher
        "cfd_polygon_new": (i32, [C.POINTER(CfdPoint), C.c_size_t, C.POINTER(C.c_uint64),
                                  C.c_size_t, C.POINTER(vp), C.POINTER(i32)]),
        "cfd_polygon_new_rect": (i32, [C.c_double] * 4 + [C.POINTER(vp)]),
        "cfd_polygon_new_regular": (i32, [CfdPoint, C.c_double, C.c_size_t, C.c_double,
                                          C.POINTER(vp)]),
        "cfd_polygon_add_hole": (i32, [vp, vp, C.POINTER(i32)]),
        "cfd_polygon_contains_point": (i32, [vp, CfdPoint, C.POINTER(i32)]),
        "cfd_polygon_intersects_aabb": (i32, [vp, C.POINTER(CfdAabb), C.POINTER(i32)]),
        "cfd_polygon_edges_intersect_aabb": (i32, [vp, C.POINTER(CfdAabb), C.POINTER(i32)]),
        "cfd_polygon_bounding_box": (i32, [vp, C.POINTER(CfdAabb)]),
        "cfd_polygon_bounding_square": (i32, [vp, C.POINTER(CfdAabb)]),
        "cfd_polygon_edges": (i32, [vp, C.POINTER(CfdPoint), C.c_size_t, C.POINTER(C.c_size_t)]),
        "cfd_polygon_destroy": (None, [vp]),
        "cfd_geom_do_intersect": (i32, [CfdPoint] * 4 + [C.POINTER(i32)]),
        "cfd_geom_segment_intersection": (i32, [CfdPoint] * 4 + [C.POINTER(CfdPoint),
                                                                 C.POINTER(i32)]),
        "cfd_geom_intersect_quad_edge": (i32, [CfdPoint, C.c_double, C.c_double, CfdPoint,
                                               CfdPoint, C.POINTER(CfdPoint), C.POINTER(i32)]),
        "cfd_tesselate": (i32, [vp, C.c_double, C.c_double, C.POINTER(vp)]),
        "cfd_quadtree_size": (i32, [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
        "cfd_quadtree_nodes": (i32, [vp, C.POINTER(CfdAabb), C.POINTER(C.c_int64)]),
        "cfd_quadtree_destroy": (None, [vp]),
        "cfd_mesh_from_quadtree": (i32, [vp, vp, i32, C.POINTER(vp)]),
        "cfd_mesh_sizes": (i32, [vp, C.POINTER(C.c_uint64)]),
        "cfd_mesh_cells": (i32, [vp] + [C.POINTER(C.c_double)] * 4),
        "cfd_mesh_neighbors": (i32, [vp, i32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
        "cfd_mesh_intersections": (i32, [vp, C.POINTER(C.c_uint64), C.POINTER(CfdPoint)]),
        "cfd_mesh_full_bounding_box": (i32, [vp, C.POINTER(CfdAabb)]),
        "cfd_mesh_build_ms": (i32, [vp, C.POINTER(C.c_double)]),
        "cfd_mesh_destroy": (None, [vp]),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("CFD_LIB") and not hasattr(L, name):
            continue   # an older tuning variant (tools/build_variants.sh) may predate a symbol
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(fn: str, rc: int):
    if rc != 0:
        msg = load().cfd_last_error()
        raise CfdError(fn, rc, msg.decode() if msg else "")
