"""cfdamd.quad_mesh — host-side mirror of the reference's mesher
(/root/reference/src/quad_mesh, src/utils/intersection.rs) over the C ABI
(include/cfd.h, cfd-demo_amd/csrc/cfd_mesh.hip).

Names follow the reference:

    Point, AABB                                  point.rs, aabb.rs
    Polygon.new / new_rect / new_polygon /
      add_hole / contains_point / intersects_aabb /
      edges_intersect_aabb / bounding_box /
      bounding_square / edges, PolygonError       polygon.rs:4-198
    do_intersect, line_segment_intersection,
      intersect_quad_edge                         utils/intersection.rs:20-129
    tesselate -> QuadTree                         quad_tree.rs:17-100
    Mesh.from_quad_tree (on the GPU),
      visit_cell, full_bounding_box               mesh.rs:51-338

Geometry and tesselation run on the host; Mesh.from_quad_tree runs its
leaf filter, O(n^2) neighbour search and intersections as HIP kernels.
"""
from __future__ import annotations

import ctypes as C
import enum
from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np

from ._lib import CfdAabb, CfdError, CfdPoint, check, load

__all__ = ["Point", "AABB", "Polygon", "PolygonError", "PolygonException", "do_intersect",
           "line_segment_intersection", "intersect_quad_edge", "tesselate", "QuadTree", "Mesh",
           "Cell", "default_polygon"]


@dataclass(frozen=True)
class Point:                                   # point.rs
    x: float
    y: float

    def _c(self) -> CfdPoint:
        return CfdPoint(self.x, self.y)


@dataclass(frozen=True)
class AABB:                                    # aabb.rs:4-9
    center: Point
    half_width: float
    half_height: float

    def _c(self) -> CfdAabb:
        return CfdAabb(self.center._c(), self.half_width, self.half_height)

    @staticmethod
    def _from(c: CfdAabb) -> "AABB":
        return AABB(Point(c.center.x, c.center.y), c.half_width, c.half_height)

    def width(self) -> float:
        return 2.0 * self.half_width

    def height(self) -> float:
        return 2.0 * self.half_height


class PolygonError(enum.IntEnum):              # polygon.rs:12-16
    NotEnoughVertices = 1
    SelfIntersecting = 2
    InvalidHole = 3


class PolygonException(ValueError):
    def __init__(self, kind: PolygonError):
        super().__init__(kind.name)
        self.kind = kind


def _pt(p) -> CfdPoint:
    return CfdPoint(p.x, p.y) if isinstance(p, Point) else CfdPoint(*p)


class Polygon:
    """Polygon with holes (polygon.rs:4-10); owns a native cfd_polygon."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def new(cls, vertex_buffer, vertices) -> "Polygon":
        """Polygon::new (polygon.rs:19-40); raises PolygonException like Err."""
        pts = (CfdPoint * max(len(vertex_buffer), 1))(*[_pt(p) for p in vertex_buffer])
        idx = (C.c_uint64 * max(len(vertices), 1))(*vertices)
        h, pe = C.c_void_p(), C.c_int()
        check("cfd_polygon_new", load().cfd_polygon_new(pts, len(vertex_buffer), idx, len(vertices),
                                                        C.byref(h), C.byref(pe)))
        if pe.value:
            raise PolygonException(PolygonError(pe.value))
        return cls(h)

    @classmethod
    def new_rect(cls, x: float, y: float, w: float, h: float) -> "Polygon":
        out = C.c_void_p()
        check("cfd_polygon_new_rect", load().cfd_polygon_new_rect(x, y, w, h, C.byref(out)))
        return cls(out)

    @classmethod
    def new_polygon(cls, center: Point, radius: float, n: int, start_angle: float) -> "Polygon":
        out = C.c_void_p()
        check("cfd_polygon_new_regular", load().cfd_polygon_new_regular(
            _pt(center), radius, n, start_angle, C.byref(out)))
        return cls(out)

    def add_hole(self, hole: "Polygon") -> None:
        """add_hole (polygon.rs:69-79); the hole is moved into this polygon."""
        pe = C.c_int()
        check("cfd_polygon_add_hole", load().cfd_polygon_add_hole(self._h, hole._h, C.byref(pe)))
        if pe.value:
            raise PolygonException(PolygonError(pe.value))
        hole._h = None   # owned by self now

    def contains_point(self, p) -> bool:
        r = C.c_int()
        check("cfd_polygon_contains_point",
              load().cfd_polygon_contains_point(self._h, _pt(p), C.byref(r)))
        return bool(r.value)

    def intersects_aabb(self, box: AABB) -> bool:
        r, b = C.c_int(), box._c()
        check("cfd_polygon_intersects_aabb",
              load().cfd_polygon_intersects_aabb(self._h, C.byref(b), C.byref(r)))
        return bool(r.value)

    def edges_intersect_aabb(self, box: AABB) -> bool:
        r, b = C.c_int(), box._c()
        check("cfd_polygon_edges_intersect_aabb",
              load().cfd_polygon_edges_intersect_aabb(self._h, C.byref(b), C.byref(r)))
        return bool(r.value)

    def bounding_box(self) -> AABB:
        b = CfdAabb()
        check("cfd_polygon_bounding_box", load().cfd_polygon_bounding_box(self._h, C.byref(b)))
        return AABB._from(b)

    def bounding_square(self) -> AABB:
        b = CfdAabb()
        check("cfd_polygon_bounding_square",
              load().cfd_polygon_bounding_square(self._h, C.byref(b)))
        return AABB._from(b)

    def edges(self) -> List[Tuple[Point, Point]]:
        n = C.c_size_t()
        check("cfd_polygon_edges", load().cfd_polygon_edges(self._h, None, 0, C.byref(n)))
        buf = (CfdPoint * max(2 * n.value, 1))()
        check("cfd_polygon_edges", load().cfd_polygon_edges(self._h, buf, n.value, C.byref(n)))
        return [(Point(buf[2 * k].x, buf[2 * k].y), Point(buf[2 * k + 1].x, buf[2 * k + 1].y))
                for k in range(n.value)]

    def __del__(self):
        if getattr(self, "_h", None):
            try:
                load().cfd_polygon_destroy(self._h)
            except Exception:
                pass
            self._h = None


def default_polygon() -> Polygon:
    """views/mesh_view.rs:140-152: 30 x 10 rectangle with a square hole of
    circumradius 1 at (5, 5), rotated by TAU / 8."""
    poly = Polygon.new_rect(0.0, 0.0, 30.0, 10.0)
    poly.add_hole(Polygon.new_polygon(Point(5.0, 5.0), 1.0, 4, 2.0 * np.pi / 8.0))
    return poly


def do_intersect(p, q, a, b) -> bool:
    r = C.c_int()
    check("cfd_geom_do_intersect", load().cfd_geom_do_intersect(_pt(p), _pt(q), _pt(a), _pt(b),
                                                                C.byref(r)))
    return bool(r.value)


def line_segment_intersection(p, q, a, b) -> Optional[Point]:
    out, found = CfdPoint(), C.c_int()
    check("cfd_geom_segment_intersection", load().cfd_geom_segment_intersection(
        _pt(p), _pt(q), _pt(a), _pt(b), C.byref(out), C.byref(found)))
    return Point(out.x, out.y) if found.value else None


def intersect_quad_edge(center, half_width: float, half_height: float, p1, p2) -> List[Point]:
    """intersect_quad_edge with quad = Quad::new_rect(center, hw, hh)."""
    buf, n = (CfdPoint * 8)(), C.c_int()
    check("cfd_geom_intersect_quad_edge", load().cfd_geom_intersect_quad_edge(
        _pt(center), half_width, half_height, _pt(p1), _pt(p2), buf, C.byref(n)))
    return [Point(buf[k].x, buf[k].y) for k in range(n.value)]


class QuadTree:
    """quad_tree.rs:7-15, flattened: nodes in depth-first pre-order."""

    def __init__(self, handle):
        self._h = handle
        nn, nl = C.c_uint64(), C.c_uint64()
        check("cfd_quadtree_size", load().cfd_quadtree_size(self._h, C.byref(nn), C.byref(nl)))
        self.n_nodes, self.n_leaves = int(nn.value), int(nl.value)
        # (center.x, center.y, half_width, half_height) per node: cfd_aabb's layout
        self.box_array = np.empty((max(self.n_nodes, 1), 4), np.float64)
        self.children = np.empty((max(self.n_nodes, 1), 4), np.int64)
        check("cfd_quadtree_nodes", load().cfd_quadtree_nodes(
            self._h, self.box_array.ctypes.data_as(C.POINTER(CfdAabb)),
            self.children.ctypes.data_as(C.POINTER(C.c_int64))))

    def box(self, node: int) -> AABB:
        x, y, hw, hh = (float(v) for v in self.box_array[node])
        return AABB(Point(x, y), hw, hh)

    @property
    def boxes(self) -> List[AABB]:
        return [self.box(k) for k in range(self.n_nodes)]

    @property
    def boundary(self) -> AABB:
        return self.box(0)

    def is_leaf(self, node: int = 0) -> bool:
        return bool(self.children[node, 0] < 0)

    def child_nodes(self, node: int = 0) -> Optional[List[int]]:
        return None if self.is_leaf(node) else [int(c) for c in self.children[node]]

    def __del__(self):
        if getattr(self, "_h", None):
            try:
                load().cfd_quadtree_destroy(self._h)
            except Exception:
                pass
            self._h = None


def tesselate(polygon: Polygon, feature_size: float, max_cell_size: float) -> QuadTree:
    """tesselate (quad_tree.rs:17-20)."""
    out = C.c_void_p()
    check("cfd_tesselate", load().cfd_tesselate(polygon._h, feature_size, max_cell_size,
                                                C.byref(out)))
    return QuadTree(out)


@dataclass
class Cell:                                    # mesh.rs:31-37
    center: Point
    half_width: float
    half_height: float
    east: np.ndarray
    west: np.ndarray
    north: np.ndarray
    south: np.ndarray
    intersections: np.ndarray


class Mesh:
    """The reference's SoA Mesh (mesh.rs:9-29), built on the GPU."""

    FACES = ("east", "west", "north", "south")

    def __init__(self):
        raise TypeError("use Mesh.from_quad_tree")

    @classmethod
    def from_quad_tree(cls, root: QuadTree, polygon: Polygon, device: int = 0) -> "Mesh":
        L = load()
        h = C.c_void_p()
        check("cfd_mesh_from_quadtree", L.cfd_mesh_from_quadtree(root._h, polygon._h, device,
                                                                 C.byref(h)))
        m = object.__new__(cls)
        try:
            sizes = (C.c_uint64 * 6)()
            check("cfd_mesh_sizes", L.cfd_mesh_sizes(h, sizes))
            n = int(sizes[0])
            dp = C.POINTER(C.c_double)
            m.cell_centers_x, m.cell_centers_y, m.cell_half_width, m.cell_half_height = (
                np.empty(n, np.float64) for _ in range(4))
            check("cfd_mesh_cells", L.cfd_mesh_cells(
                h, m.cell_centers_x.ctypes.data_as(dp), m.cell_centers_y.ctypes.data_as(dp),
                m.cell_half_width.ctypes.data_as(dp), m.cell_half_height.ctypes.data_as(dp)))
            up = C.POINTER(C.c_uint64)
            for face, name in enumerate(cls.FACES):
                rng = np.empty((n, 2), np.uint64)
                idx = np.empty(int(sizes[1 + face]), np.uint64)
                check("cfd_mesh_neighbors", L.cfd_mesh_neighbors(
                    h, face, rng.ctypes.data_as(up), idx.ctypes.data_as(up)))
                setattr(m, f"neighbors_{name}_range", rng)
                setattr(m, f"neighbors_{name}_indexes", idx)
            m.cell_intersections_range = np.empty((n, 2), np.uint64)
            pts = np.empty((int(sizes[5]), 2), np.float64)
            check("cfd_mesh_intersections", L.cfd_mesh_intersections(
                h, m.cell_intersections_range.ctypes.data_as(up),
                pts.ctypes.data_as(C.POINTER(CfdPoint))))
            m.cell_intersections_points = pts
            box = CfdAabb()
            check("cfd_mesh_full_bounding_box", L.cfd_mesh_full_bounding_box(h, C.byref(box)))
            m._bbox = AABB._from(box)
            ms = C.c_double()
            check("cfd_mesh_build_ms", L.cfd_mesh_build_ms(h, C.byref(ms)))
            m.build_ms = float(ms.value)
        finally:
            L.cfd_mesh_destroy(h)
        return m

    @property
    def num_cells(self) -> int:
        return int(self.cell_centers_x.size)

    def cell_geometry_intersections(self, i: int) -> np.ndarray:
        a, b = self.cell_intersections_range[i]
        return self.cell_intersections_points[int(a):int(b)]

    def visit_cell(self, i: int, visit) -> None:
        """visit_cell (mesh.rs:230-281)."""
        nb = {}
        for name in self.FACES:
            a, b = getattr(self, f"neighbors_{name}_range")[i]
            nb[name] = getattr(self, f"neighbors_{name}_indexes")[int(a):int(b)]
        visit(Cell(Point(float(self.cell_centers_x[i]), float(self.cell_centers_y[i])),
                   float(self.cell_half_width[i]), float(self.cell_half_height[i]),
                   nb["east"], nb["west"], nb["north"], nb["south"],
                   self.cell_geometry_intersections(i)))

    def visit_all_cells(self, visit) -> None:
        for i in range(self.num_cells):
            self.visit_cell(i, visit)

    def full_bounding_box(self) -> AABB:
        return self._bbox
