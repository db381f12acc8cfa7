"""GPU: Mesh::from_quad_tree (mesh.rs:51-227) built by the HIP kernels
(csrc/cfd_mesh.hip) against the oracle restatement (oracle/quad_mesh_ref.py),
bit for bit in f64: the kept cells and their order, all four neighbour lists
(ranges and indices, ascending), the cell/edge intersection points, and
full_bounding_box."""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _both(build):
    from cfdamd import quad_mesh as qm
    import quad_mesh_ref as qr
    return build(qm), build(qr)


def _default(m):
    return m.default_polygon()


def _octagon(m):
    P = m.Point
    vb = [P(5.0 + 4.0 * math.cos(i * (2 * math.pi) / 8), 5.0 + 4.0 * math.sin(i * (2 * math.pi) / 8))
          for i in range(8)]
    return m.Polygon.new(vb, list(range(8)))


def _concave(m):
    P = m.Point
    return m.Polygon.new([P(0.0, 0.0), P(4.0, 0.0), P(4.0, 3.0), P(2.0, 1.0), P(0.0, 3.0)],
                         [0, 1, 2, 3, 4])


def _two_holes(m):
    poly = m.Polygon.new_rect(0.0, 0.0, 12.0, 6.0)
    poly.add_hole(m.Polygon.new_rect(2.0, 2.0, 2.0, 2.0))
    poly.add_hole(m.Polygon.new_polygon(m.Point(8.0, 3.0), 1.5, 6, 0.3))
    return poly


CASES = {
    "default_0.1_0.5": (_default, 0.1, 0.5),     # views/mesh_view.rs defaults
    "default_0.3_1.0": (_default, 0.3, 1.0),
    "octagon_0.5_5.0": (_octagon, 0.5, 5.0),     # quad_tree.rs:119-136
    "concave_0.1_0.5": (_concave, 0.1, 0.5),
    "two_holes_0.15_0.6": (_two_holes, 0.15, 0.6),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_mesh_matches_oracle(name):
    from cfdamd import quad_mesh as qm
    import quad_mesh_ref as qr
    build, f, mx = CASES[name]
    pp, op = build(qm), build(qr)
    mesh = qm.Mesh.from_quad_tree(qm.tesselate(pp, f, mx), pp)
    ref = qr.Mesh(qr.tesselate(op, f, mx), op)
    assert mesh.num_cells == ref.cell_centers_x.size > 0
    for a in ("cell_centers_x", "cell_centers_y", "cell_half_width", "cell_half_height"):
        assert np.array_equal(getattr(mesh, a).view(np.uint64), getattr(ref, a).view(np.uint64)), a
    for face in ("east", "west", "north", "south"):
        for a in (f"neighbors_{face}_range", f"neighbors_{face}_indexes"):
            assert np.array_equal(getattr(mesh, a), getattr(ref, a)), a
        assert getattr(mesh, f"neighbors_{face}_indexes").size > 0
    assert np.array_equal(mesh.cell_intersections_range, ref.cell_intersections_range)
    assert np.array_equal(mesh.cell_intersections_points.view(np.uint64),
                          ref.cell_intersections_points.view(np.uint64))
    b, rb = mesh.full_bounding_box(), ref.full_bounding_box()
    assert (b.center.x, b.center.y, b.half_width, b.half_height) == \
           (rb.center.x, rb.center.y, rb.half_width, rb.half_height)
    # visit_cell hands out the same slices
    seen = []
    mesh.visit_cell(0, lambda c: seen.append(c))
    assert seen[0].east.size == int(ref.neighbors_east_range[0][1] - ref.neighbors_east_range[0][0])


def test_mesh_of_empty_filter_and_errors():
    """A polygon far from every leaf centre still keeps the cells that touch
    it; a hole with its own hole is refused loudly on the device path."""
    from cfdamd import CfdError
    from cfdamd import quad_mesh as qm
    poly = qm.Polygon.new_rect(0.0, 0.0, 4.0, 4.0)
    hole = qm.Polygon.new_rect(1.0, 1.0, 2.0, 2.0)
    hole.add_hole(qm.Polygon.new_rect(1.5, 1.5, 1.0, 1.0))
    poly.add_hole(hole)
    with pytest.raises(CfdError):
        qm.Mesh.from_quad_tree(qm.tesselate(poly, 0.5, 1.0), poly)
