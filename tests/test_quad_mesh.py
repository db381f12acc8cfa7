"""CPU: the mesher (src/quad_mesh, src/utils/intersection.rs).

1. The reference's own 33 unit tests (polygon.rs:235-461, quad_tree.rs:102-138,
   intersection.rs:132-391), restated one for one, run against BOTH the
   product's host code (cfdamd.quad_mesh over the C ABI) and the oracle
   restatement (oracle/quad_mesh_ref.py).
2. Product vs oracle, bit for bit in f64: tesselations (every node box in
   depth-first order), point membership and quad/edge intersections on random
   inputs.

The GPU half (Mesh.from_quad_tree) is tests/test_gpu_mesh.py.
"""
import math
import random

import pytest


def _product():
    from cfdamd import quad_mesh as qm
    return qm


def _oracle():
    import quad_mesh_ref as qr
    return qr


class Impl:
    def __init__(self, name):
        self.name = name
        self.m = _product() if name == "product" else _oracle()
        self.P = self.m.Point

    def polygon(self, vb, v):
        return self.m.Polygon.new(vb, v)

    def rect(self, x, y, w, h):
        return self.m.Polygon.new_rect(x, y, w, h)

    def errors(self):
        return (self.m.PolygonException,) if self.name == "product" else (self.m.PolygonError,)

    def kind(self, e):
        return e.kind.name if self.name == "product" else e.kind

    def lsi(self, p, q, a, b):
        return self.m.line_segment_intersection(p, q, a, b)

    def di(self, p, q, a, b):
        return self.m.do_intersect(p, q, a, b)

    def iqe(self, center, hw, hh, p1, p2):
        if self.name == "product":
            return self.m.intersect_quad_edge(center, hw, hh, p1, p2)
        return self.m.intersect_quad_edge(self.m.quad_new_rect(center, hw, hh), p1, p2)

    def tess(self, poly, f, mx):
        return self.m.tesselate(poly, f, mx)

    def root_children_all_leaves(self, t):
        if self.name == "product":
            ch = t.child_nodes(0)
            return ch is not None and all(t.is_leaf(c) for c in ch)
        return t.children is not None and all(c.is_leaf() for c in t.children)

    def root_has_children(self, t):
        return (t.child_nodes(0) is not None) if self.name == "product" else t.children is not None


@pytest.fixture(params=["product", "oracle"])
def im(request):
    return Impl(request.param)


def _err(im, fn):
    try:
        fn()
    except im.errors() as e:
        return im.kind(e)
    return None


EPS = 2.220446049250313e-16


# -------------------------------------------------- polygon.rs:235-461 (12)

def test_line(im):
    P = im.P
    assert _err(im, lambda: im.polygon([P(0.0, 0.0), P(1.0, 1.0)], [0, 1])) == "NotEnoughVertices"


def test_non_intersecting_polygon(im):
    P = im.P
    assert _err(im, lambda: im.polygon([P(0, 0), P(1, 0), P(1, 1), P(0, 1)], [0, 1, 2, 3])) is None


def test_self_intersecting_polygon(im):
    P = im.P
    assert _err(im, lambda: im.polygon([P(0.0, 0.0), P(1.0, 1.0), P(0.0, 1.0), P(1.0, 0.0)],
                                       [0, 1, 2, 3])) == "SelfIntersecting"


def test_triangle(im):
    P = im.P
    assert _err(im, lambda: im.polygon([P(0.0, 0.0), P(1.0, 0.0), P(0.0, 1.0)], [0, 1, 2])) is None


def test_concave_polygon(im):
    P = im.P
    vb = [P(0.0, 0.0), P(4.0, 0.0), P(4.0, 3.0), P(2.0, 1.0), P(0.0, 3.0)]
    assert _err(im, lambda: im.polygon(vb, [0, 1, 2, 3, 4])) is None


def test_complex_self_intersecting_polygon(im):
    P = im.P
    vb = [P(-1.0, -1.0), P(1.0, -1.0), P(-1.0, 0.0), P(1.0, 0.0), P(0.0, 1.0)]
    assert _err(im, lambda: im.polygon(vb, [0, 3, 2, 1, 4])) == "SelfIntersecting"


def _square4(im):
    P = im.P
    return im.polygon([P(0.0, 0.0), P(4.0, 0.0), P(4.0, 4.0), P(0.0, 4.0)], [0, 1, 2, 3])


def test_point_in_polygon_inside(im):
    assert _square4(im).contains_point(im.P(2.0, 2.0))


def test_point_in_polygon_outside(im):
    assert not _square4(im).contains_point(im.P(5.0, 5.0))


def _outer_and_hole(im, hole_pts):
    P = im.P
    outer = im.polygon([P(0.0, 0.0), P(10.0, 0.0), P(10.0, 10.0), P(0.0, 10.0)], [0, 1, 2, 3])
    hole = im.polygon([P(*xy) for xy in hole_pts], [0, 1, 2, 3])
    return outer, hole


def test_contains_point_with_hole(im):
    outer, hole = _outer_and_hole(im, [(3.0, 3.0), (7.0, 3.0), (7.0, 7.0), (3.0, 7.0)])
    outer.add_hole(hole)
    P = im.P
    assert not outer.contains_point(P(5.0, 5.0))
    assert outer.contains_point(P(2.0, 2.0))
    assert not outer.contains_point(P(3.0, 5.0))


def test_add_valid_hole(im):
    outer, hole = _outer_and_hole(im, [(3.0, 3.0), (7.0, 3.0), (7.0, 7.0), (3.0, 7.0)])
    assert _err(im, lambda: outer.add_hole(hole)) is None


def test_add_valid_hole2(im):
    outer = im.rect(0.0, 0.0, 10.0, 10.0)
    hole = im.rect(3.0, 3.0, 4.0, 4.0)
    assert _err(im, lambda: outer.add_hole(hole)) is None


def test_add_invalid_hole(im):
    outer, hole = _outer_and_hole(im, [(3.0, 3.0), (11.0, 3.0), (11.0, 7.0), (3.0, 7.0)])
    assert _err(im, lambda: outer.add_hole(hole)) == "InvalidHole"


# ------------------------------------------------ quad_tree.rs:102-138 (2)

def test_tesselate_rect_one_sub(im):
    t = im.tess(im.rect(0.0, 0.0, 10.0, 10.0), 5.0, 5.0)
    assert im.root_children_all_leaves(t)


def test_tesselate_octagon_subdivision(im):
    P = im.P
    vb = [P(5.0 + 4.0 * math.cos(i * (2 * math.pi) / 8), 5.0 + 4.0 * math.sin(i * (2 * math.pi) / 8))
          for i in range(8)]
    t = im.tess(im.polygon(vb, list(range(8))), 0.5, 5.0)
    assert im.root_has_children(t)


# --------------------------------------------- intersection.rs:132-391 (19)

def _close(p, x, y):
    return abs(p.x - x) < EPS and abs(p.y - y) < EPS


def test_line_intersection_intersecting(im):
    P = im.P
    assert im.lsi(P(0.0, 0.0), P(1.0, 1.0), P(0.0, 1.0), P(1.0, 0.0)) is not None


def test_line_intersection_non_intersecting_but_lines_do(im):
    P = im.P
    assert im.lsi(P(0.0, 0.0), P(0.5, 0.5), P(2.0, 0.0), P(3.0, -1.0)) is None


def test_line_intersection_parallel(im):
    P = im.P
    assert im.lsi(P(0.0, 0.0), P(1.0, 0.0), P(0.0, 1.0), P(1.0, 1.0)) is None


def test_line_intersection_collinear(im):
    P = im.P
    assert im.lsi(P(0.0, 0.0), P(1.0, 1.0), P(2.0, 2.0), P(3.0, 3.0)) is None


def test_line_intersection_endpoint(im):
    P = im.P
    ip = im.lsi(P(0.0, 0.0), P(1.0, 1.0), P(1.0, 1.0), P(2.0, 0.0))
    assert ip is not None and _close(ip, 1.0, 1.0)


def test_line_intersection_overlapping_collinear(im):
    P = im.P
    assert im.lsi(P(0.0, 0.0), P(2.0, 2.0), P(1.0, 1.0), P(3.0, 3.0)) is None


def test_line_intersection_nearly_parallel(im):
    P = im.P
    assert im.lsi(P(0.0, 0.0), P(10.0, 0.0001), P(0.0, 1.0), P(10.0, 1.0001)) is None


def test_line_intersection_exact_intersection(im):
    P = im.P
    ip = im.lsi(P(0.0, 0.0), P(2.0, 2.0), P(0.0, 2.0), P(2.0, 0.0))
    assert ip is not None and _close(ip, 1.0, 1.0)


def test_intersecting_segments(im):
    P = im.P
    assert im.di(P(0.0, 0.0), P(1.0, 1.0), P(0.0, 1.0), P(1.0, 0.0))


def test_non_intersecting_segments(im):
    P = im.P
    assert not im.di(P(0.0, 0.0), P(0.5, 0.5), P(2.0, 0.0), P(3.0, -1.0))


def test_collinear_but_disjoint(im):
    P = im.P
    assert not im.di(P(0.0, 0.0), P(1.0, 1.0), P(2.0, 2.0), P(3.0, 3.0))


def test_sharing_endpoint(im):
    P = im.P
    assert im.di(P(0.0, 0.0), P(1.0, 1.0), P(1.0, 1.0), P(2.0, 0.0))


def test_intersect_quad_edge_no_intersection(im):
    P = im.P
    assert len(im.iqe(P(0.0, 0.0), 1.0, 1.0, P(-3.0, -3.0), P(-2.0, -2.0))) == 0


def test_intersect_quad_edge_one_intersection(im):
    P = im.P
    r = im.iqe(P(0.0, 0.0), 1.0, 1.0, P(-2.0, 0.0), P(0.0, 0.0))
    assert len(r) == 1 and _close(r[0], -1.0, 0.0)


def test_intersect_quad_edge_two_intersections(im):
    P = im.P
    r = sorted(im.iqe(P(0.0, 0.0), 1.0, 1.0, P(-2.0, 0.0), P(2.0, 0.0)), key=lambda p: p.x)
    assert len(r) == 2 and _close(r[0], -1.0, 0.0) and _close(r[1], 1.0, 0.0)


def test_intersect_quad_edge_through_vertex(im):
    P = im.P
    r = im.iqe(P(0.0, 0.0), 1.0, 1.0, P(-2.0, -2.0), P(2.0, 2.0))
    assert len(r) == 2
    for x, y in ((-1.0, -1.0), (1.0, 1.0)):
        assert any(_close(p, x, y) for p in r)


def test_intersect_quad_edge_along_edge(im):
    P = im.P
    r = sorted(im.iqe(P(0.0, 0.0), 1.0, 1.0, P(-1.0, 1.0), P(1.0, 1.0)), key=lambda p: p.x)
    assert len(r) == 2 and _close(r[0], -1.0, 1.0) and _close(r[1], 1.0, 1.0)


def test_intersect_quad_edge_inside_quad(im):
    P = im.P
    assert len(im.iqe(P(0.0, 0.0), 1.0, 1.0, P(-0.5, -0.5), P(0.5, 0.5))) == 0


def test_intersect_quad_edge_diagonal(im):
    P = im.P
    r = im.iqe(P(0.0, 0.0), 1.0, 1.0, P(-2.0, -1.0), P(0.0, 1.0))
    assert len(r) == 2
    for x, y in ((-1.0, 0.0), (0.0, 1.0)):
        assert any(_close(p, x, y) for p in r)


# ------------------------------------------ product vs oracle, bit for bit

def _pair_default():
    return _product().default_polygon(), _oracle().default_polygon()


@pytest.mark.parametrize("feature,max_cell", [(0.1, 0.5), (0.3, 1.0), (0.05, 0.5)])
def test_tesselation_matches_oracle(feature, max_cell):
    """views/mesh_view.rs defaults (0.1, 0.5) and two other settings."""
    pp, op = _pair_default()
    t = _product().tesselate(pp, feature, max_cell)
    nodes = _oracle().preorder(_oracle().tesselate(op, feature, max_cell))
    assert t.n_nodes == len(nodes)
    assert t.n_leaves == sum(1 for n in nodes if n.is_leaf())
    for k, (b, n) in enumerate(zip(t.boxes, nodes)):
        o = n.boundary
        assert (b.center.x, b.center.y, b.half_width, b.half_height) == \
               (o.center.x, o.center.y, o.half_width, o.half_height), k
        assert t.is_leaf(k) == n.is_leaf(), k


def test_polygon_queries_match_oracle():
    pm, om = _product(), _oracle()
    pp, op = _pair_default()
    for a, b in ((pp.bounding_box(), op.bounding_box()), (pp.bounding_square(), op.bounding_square())):
        assert (a.center.x, a.center.y, a.half_width, a.half_height) == \
               (b.center.x, b.center.y, b.half_width, b.half_height)
    assert [((a.x, a.y), (b.x, b.y)) for a, b in pp.edges()] == \
           [((a.x, a.y), (b.x, b.y)) for a, b in op.edges()]
    rng = random.Random(5)
    for _ in range(3000):
        x, y = rng.uniform(-1, 31), rng.uniform(-1, 11)
        assert pp.contains_point(pm.Point(x, y)) == op.contains_point(om.Point(x, y))
        hw, hh = rng.uniform(0, 3), rng.uniform(0, 3)
        pb = pm.AABB(pm.Point(x, y), hw, hh)
        ob = om.AABB(om.Point(x, y), hw, hh)
        assert pp.edges_intersect_aabb(pb) == op.edges_intersect_aabb(ob)
        assert pp.intersects_aabb(pb) == op.intersects_aabb(ob)


def test_segment_predicates_match_oracle():
    pm, om = _product(), _oracle()
    rng = random.Random(9)
    grid = [0.0, 0.5, 1.0, -1.0, 2.0]
    for k in range(4000):
        if k % 2:   # exact grid points: collinear / touching cases
            c = [rng.choice(grid) for _ in range(8)]
        else:
            c = [rng.uniform(-2, 2) for _ in range(8)]
        P, O = [pm.Point(c[2 * i], c[2 * i + 1]) for i in range(4)], \
               [om.Point(c[2 * i], c[2 * i + 1]) for i in range(4)]
        assert pm.do_intersect(*P) == om.do_intersect(*O)
        a, b = pm.line_segment_intersection(*P), om.line_segment_intersection(*O)
        assert (a is None) == (b is None)
        if a is not None:
            assert (a.x, a.y) == (b.x, b.y)
        hw, hh = abs(c[6]) + 0.25, abs(c[7]) + 0.25
        r1 = pm.intersect_quad_edge(P[0], hw, hh, P[1], P[2])
        r2 = om.intersect_quad_edge(om.quad_new_rect(O[0], hw, hh), O[1], O[2])
        assert [(p.x, p.y) for p in r1] == [(p.x, p.y) for p in r2]


def test_bad_inputs_fail_loudly():
    qm = _product()
    from cfdamd import CfdError
    with pytest.raises(CfdError):
        qm.Polygon.new([qm.Point(0, 0), qm.Point(1, 0), qm.Point(0, 1)], [0, 1, 7])
    with pytest.raises(CfdError):
        qm.tesselate(qm.Polygon.new_rect(0, 0, 1, 1), 0.0, 0.0)
