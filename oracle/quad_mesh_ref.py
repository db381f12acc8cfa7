"""Pure-Python restatement of the reference's mesher — TEST INFRASTRUCTURE ONLY
(imported by tests/ alone, never by the product package).

Follows /root/reference/src/quad_mesh/{aabb,polygon,quad_tree,mesh}.rs and
src/utils/intersection.rs line by line, in Python floats (IEEE double, the
reference's f64; Python never contracts a*b+c).  The O(n^2) neighbour search
of Mesh::from_quad_tree is vectorised over j with numpy (same f64 compares,
same ascending-j order).  Pinned by the reference's own 33 unit tests
(tests/test_quad_mesh.py runs them against this module and the product).
"""
from __future__ import annotations

import math
import sys
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

EPS = sys.float_info.epsilon   # std::f64::EPSILON


@dataclass(frozen=True)
class Point:
    x: float
    y: float


# ------------------------------------------------------- intersection.rs

def orientation(p, q, r) -> int:                       # :3-13
    val = (q.y - p.y) * (r.x - q.x) - (q.x - p.x) * (r.y - q.y)
    if abs(val) < EPS:
        return 0
    return 1 if val > 0.0 else 2


def _fmax(a, b):   # f64::max: a NaN operand loses
    if a != a:
        return b
    if b != b:
        return a
    return a if a > b else b


def _fmin(a, b):
    if a != a:
        return b
    if b != b:
        return a
    return a if a < b else b


def on_segment(p, q, r) -> bool:                       # :15-18
    return (q.x <= _fmax(p.x, r.x) + EPS and q.x >= _fmin(p.x, r.x) - EPS) and \
           (q.y <= _fmax(p.y, r.y) + EPS and q.y >= _fmin(p.y, r.y) - EPS)


def do_intersect(p, q, a, b) -> bool:                  # :20-38
    o1, o2 = orientation(p, q, a), orientation(p, q, b)
    o3, o4 = orientation(a, b, p), orientation(a, b, q)
    if o1 != o2 and o3 != o4:
        return True
    if o1 == 0 and on_segment(p, a, q):
        return True
    if o2 == 0 and on_segment(p, b, q):
        return True
    if o3 == 0 and on_segment(a, p, b):
        return True
    if o4 == 0 and on_segment(a, q, b):
        return True
    return False


def line_segment_intersection(p, q, a, b) -> Optional[Point]:   # :41-63
    if not do_intersect(p, q, a, b):
        return None
    a1 = q.y - p.y
    b1 = p.x - q.x
    c1 = a1 * p.x + b1 * p.y
    a2 = b.y - a.y
    b2 = a.x - b.x
    c2 = a2 * a.x + b2 * a.y
    det = a1 * b2 - a2 * b1
    if abs(det) < EPS:
        return None
    return Point((b2 * c1 - b1 * c2) / det, (a1 * c2 - a2 * c1) / det)


def quad_new_rect(center, hw, hh):                     # quad.rs:24-35
    left, right = center.x - hw, center.x + hw
    bottom, top = center.y - hh, center.y + hh
    return [Point(left, bottom), Point(right, bottom), Point(right, top), Point(left, top)]


def intersect_quad_edge(quad, p1, p2) -> List[Point]:  # :68-129
    out: List[Point] = []

    def seen(x):
        return any(abs(p.x - x.x) < EPS and abs(p.y - x.y) < EPS for p in out)

    for i in range(4):
        v1, v2 = quad[i], quad[(i + 1) % 4]
        if orientation(p1, p2, v1) == 0 and orientation(p1, p2, v2) == 0:
            d_x, d_y = p2.x - p1.x, p2.y - p1.y
            norm = d_x * d_x + d_y * d_y
            if abs(norm) < EPS:
                continue
            t_v1 = ((v1.x - p1.x) * d_x + (v1.y - p1.y) * d_y) / norm
            t_v2 = ((v2.x - p1.x) * d_x + (v2.y - p1.y) * d_y) / norm
            t_start = _fmax(_fmin(t_v1, t_v2), 0.0)
            t_end = _fmin(_fmax(t_v1, t_v2), 1.0)
            if t_start <= t_end + EPS:
                s = Point(p1.x + t_start * d_x, p1.y + t_start * d_y)
                e = Point(p1.x + t_end * d_x, p1.y + t_end * d_y)
                if not seen(s):
                    out.append(s)
                if not seen(e):
                    out.append(e)
                continue
        x = line_segment_intersection(p1, p2, v1, v2)
        if x is not None and not seen(x):
            out.append(x)
    return out


# ---------------------------------------------------------------- aabb.rs

@dataclass(frozen=True)
class AABB:
    center: Point
    half_width: float
    half_height: float

    def width(self):
        return 2.0 * self.half_width

    def height(self):
        return 2.0 * self.half_height

    def top_left(self):
        return Point(self.center.x - self.half_width, self.center.y - self.half_height)

    def top_right(self):
        return Point(self.center.x + self.half_width, self.center.y - self.half_height)

    def bottom_left(self):
        return Point(self.center.x - self.half_width, self.center.y + self.half_height)

    def bottom_right(self):
        return Point(self.center.x + self.half_width, self.center.y + self.half_height)

    def intersects_segment(self, a, b):                # :78-89
        tl, tr, bl, br = self.top_left(), self.top_right(), self.bottom_left(), self.bottom_right()
        return (do_intersect(a, b, tl, tr) or do_intersect(a, b, tr, br) or
                do_intersect(a, b, br, bl) or do_intersect(a, b, bl, tl))


# ------------------------------------------------------------- polygon.rs

class PolygonError(Exception):
    def __init__(self, kind: str):
        super().__init__(kind)
        self.kind = kind


def polygon_is_self_intersecting(pts) -> bool:         # :208-231
    n = len(pts)
    if n < 4:
        return False
    for i in range(n):
        p1, q1 = pts[i], pts[(i + 1) % n]
        for j in range(i + 1, n):
            if j == i or (j + 1) % n == i or (i + 1) % n == j:
                continue
            if do_intersect(p1, q1, pts[j], pts[(j + 1) % n]):
                return True
    return False


class Polygon:
    def __init__(self, vertex_buffer, vertices):       # new :19-40
        if len(vertices) < 3:
            raise PolygonError("NotEnoughVertices")
        pts = [vertex_buffer[i] for i in vertices]
        if polygon_is_self_intersecting(pts):
            raise PolygonError("SelfIntersecting")
        self.vertex_buffer = list(vertex_buffer)
        self.vertices = list(vertices)
        self.holes: List["Polygon"] = []

    @classmethod
    def new(cls, vertex_buffer, vertices):
        return cls(vertex_buffer, vertices)

    @classmethod
    def new_rect(cls, x, y, w, h):                     # :42-53
        return cls([Point(x, y), Point(x + w, y), Point(x + w, y + h), Point(x, y + h)],
                   [0, 1, 2, 3])

    @classmethod
    def new_polygon(cls, center, radius, n, start_angle):   # :55-67
        vb = []
        for i in range(n):
            theta = float(i) * (2.0 * math.pi) / float(n) + start_angle
            vb.append(Point(center.x + radius * math.cos(theta),
                            center.y + radius * math.sin(theta)))
        return cls(vb, list(range(n)))

    def add_hole(self, hole):                          # :69-79
        for idx in hole.vertices:
            if not self.contains_point(hole.vertex_buffer[idx]):
                raise PolygonError("InvalidHole")
        self.holes.append(hole)

    def contains_point(self, p) -> bool:               # :81-103
        count = 0
        n = len(self.vertices)
        for i in range(n):
            j = (i + 1) % n
            a = self.vertex_buffer[self.vertices[i]]
            b = self.vertex_buffer[self.vertices[j]]
            if (a.y > p.y) != (b.y > p.y):
                x_intersect = a.x + (p.y - a.y) * (b.x - a.x) / (b.y - a.y)
                if p.x < x_intersect:
                    count += 1
        if count % 2 != 1:
            return False
        return not any(h.contains_point(p) for h in self.holes)

    def intersects_aabb(self, o: AABB) -> bool:        # :105-117
        return (self.contains_point(o.top_left()) or self.contains_point(o.top_right()) or
                self.contains_point(o.bottom_left()) or self.contains_point(o.bottom_right()) or
                self.contains_point(o.center))

    def edges(self):                                   # :186-196 (index quirk kept)
        n = len(self.vertices)
        return [(self.vertex_buffer[i], self.vertex_buffer[(i + 1) % n]) for i in self.vertices]

    def edges_intersect_aabb(self, o: AABB) -> bool:   # :119-133
        for a, b in self.edges():
            if o.intersects_segment(a, b):
                return True
        return any(h.edges_intersect_aabb(o) for h in self.holes)

    def bounding_box(self) -> AABB:                    # :150-178
        min_x, max_x, min_y, max_y = math.inf, -math.inf, math.inf, -math.inf
        for p in self.vertex_buffer:
            min_x = _fmin(min_x, p.x)
            max_x = _fmax(max_x, p.x)
            min_y = _fmin(min_y, p.y)
            max_y = _fmax(max_y, p.y)
        return AABB(Point((min_x + max_x) / 2.0, (min_y + max_y) / 2.0),
                    (max_x - min_x) / 2.0, (max_y - min_y) / 2.0)

    def bounding_square(self) -> AABB:                 # :180-184
        b = self.bounding_box()
        m = _fmax(b.width(), b.height())
        return AABB(b.center, m / 2.0, m / 2.0)


def default_polygon() -> Polygon:                      # views/mesh_view.rs:140-152
    poly = Polygon.new_rect(0.0, 0.0, 30.0, 10.0)
    poly.add_hole(Polygon.new_polygon(Point(5.0, 5.0), 1.0, 4, (2.0 * math.pi) / 8.0))
    return poly


# ----------------------------------------------------------- quad_tree.rs

class QuadTree:
    def __init__(self, boundary: AABB, children=None):
        self.boundary = boundary
        self.children = children

    def is_leaf(self):
        return self.children is None


def tesselate(polygon: Polygon, feature_size: float, max_cell_size: float) -> QuadTree:
    return _tesselate(polygon, polygon.bounding_square(), feature_size, max_cell_size)


def _tesselate(polygon, b: AABB, feature_size, max_cell_size) -> QuadTree:   # :22-100
    cell_size = _fmin(b.width(), b.height())
    intersects = polygon.edges_intersect_aabb(b)
    if (cell_size <= feature_size or not intersects) and cell_size <= max_cell_size:
        return QuadTree(b)
    nhw, nhh = b.half_width / 2.0, b.half_height / 2.0
    cx, cy = b.center.x, b.center.y
    return QuadTree(b, [
        _tesselate(polygon, AABB(Point(cx - nhw, cy - nhh), nhw, nhh), feature_size, max_cell_size),
        _tesselate(polygon, AABB(Point(cx + nhw, cy - nhh), nhw, nhh), feature_size, max_cell_size),
        _tesselate(polygon, AABB(Point(cx - nhw, cy + nhh), nhw, nhh), feature_size, max_cell_size),
        _tesselate(polygon, AABB(Point(cx + nhw, cy + nhh), nhw, nhh), feature_size, max_cell_size),
    ])


def preorder(t: QuadTree):
    """Nodes in depth-first pre-order (the product's flattening)."""
    out = [t]
    if t.children:
        for c in t.children:
            out.extend(preorder(c))
    return out


# ---------------------------------------------------------------- mesh.rs

class Mesh:
    def __init__(self, root: QuadTree, polygon: Polygon):   # from_quad_tree :51-227
        leaves = [n.boundary for n in preorder(root) if n.is_leaf()]   # gather_leaves :352-370
        valid = []
        for c in leaves:                                   # :57-78
            center_inside = polygon.contains_point(c.center)
            left, right = c.center.x - c.half_width, c.center.x + c.half_width
            bottom, top = c.center.y - c.half_height, c.center.y + c.half_height
            vertex_inside = (polygon.contains_point(Point(left, bottom)) or
                             polygon.contains_point(Point(left, top)) or
                             polygon.contains_point(Point(right, bottom)) or
                             polygon.contains_point(Point(right, top)))
            if center_inside or vertex_inside:
                valid.append(c)
        n = len(valid)
        self.cell_centers_x = np.array([c.center.x for c in valid], np.float64)
        self.cell_centers_y = np.array([c.center.y for c in valid], np.float64)
        self.cell_half_width = np.array([c.half_width for c in valid], np.float64)
        self.cell_half_height = np.array([c.half_height for c in valid], np.float64)
        xmin = self.cell_centers_x - self.cell_half_width
        xmax = self.cell_centers_x + self.cell_half_width
        ymin = self.cell_centers_y - self.cell_half_height
        ymax = self.cell_centers_y + self.cell_half_height
        eps = 1e-6
        lists = {k: [] for k in ("east", "west", "north", "south")}
        idx = np.arange(n)
        for i in range(n):                                 # :124-154
            y_ov = (ymin[i] < ymax) & (ymax[i] > ymin)
            x_ov = (xmin[i] < xmax) & (xmax[i] > xmin)
            not_me = idx != i
            lists["east"].append(idx[(np.abs(xmin - xmax[i]) < eps) & y_ov & not_me])
            lists["west"].append(idx[(np.abs(xmax - xmin[i]) < eps) & y_ov & not_me])
            lists["north"].append(idx[(np.abs(ymin - ymax[i]) < eps) & x_ov & not_me])
            lists["south"].append(idx[(np.abs(ymax - ymin[i]) < eps) & x_ov & not_me])
        for name, ls in lists.items():                     # :156-184
            rng = np.zeros((n, 2), np.uint64)
            flat = []
            for i, l in enumerate(ls):
                rng[i] = (len(flat), len(flat) + len(l))
                flat.extend(int(j) for j in l)
            setattr(self, f"neighbors_{name}_range", rng)
            setattr(self, f"neighbors_{name}_indexes", np.array(flat, np.uint64))
        edges = list(polygon.edges())                      # :186-210
        for h in polygon.holes:
            edges.extend(h.edges())
        pts, rng = [], np.zeros((n, 2), np.uint64)
        for i, c in enumerate(valid):
            quad = quad_new_rect(c.center, c.half_width, c.half_height)
            start = len(pts)
            for p1, p2 in edges:
                pts.extend(intersect_quad_edge(quad, p1, p2))
            rng[i] = (start, len(pts))
        self.cell_intersections_range = rng
        self.cell_intersections_points = np.array([(p.x, p.y) for p in pts],
                                                  np.float64).reshape(-1, 2)

    def full_bounding_box(self) -> AABB:                   # :294-338
        if self.cell_centers_x.size == 0:
            return AABB(Point(0.0, 0.0), 0.0, 0.0)
        min_x, max_x, min_y, max_y = math.inf, -math.inf, math.inf, -math.inf
        for i in range(self.cell_centers_x.size):
            q = quad_new_rect(Point(float(self.cell_centers_x[i]), float(self.cell_centers_y[i])),
                              float(self.cell_half_width[i]), float(self.cell_half_height[i]))
            cmin_x = cmin_y = math.inf
            cmax_x = cmax_y = -math.inf
            for v in q:
                cmin_x, cmax_x = _fmin(cmin_x, v.x), _fmax(cmax_x, v.x)
                cmin_y, cmax_y = _fmin(cmin_y, v.y), _fmax(cmax_y, v.y)
            min_x = cmin_x if cmin_x < min_x else min_x
            max_x = cmax_x if cmax_x > max_x else max_x
            min_y = cmin_y if cmin_y < min_y else min_y
            max_y = cmax_y if cmax_y > max_y else max_y
        return AABB(Point(0.5 * (min_x + max_x), 0.5 * (min_y + max_y)),
                    0.5 * (max_x - min_x), 0.5 * (max_y - min_y))
