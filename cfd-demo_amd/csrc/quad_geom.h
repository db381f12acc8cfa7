// quad_geom.h — the geometry predicates of the reference's mesher
// (/root/reference/src/utils/intersection.rs, src/quad_mesh/*.rs), shared by
// the host code (tesselation) and the device kernels (mesh construction) of
// cfd_mesh.hip, so both evaluate the same f64 expressions.  Rust f64
// semantics: IEEE double, no contraction (built with -ffp-contract=off),
// f64::min/max ignore a NaN operand like fmin/fmax, EPSILON = DBL_EPSILON.
#pragma once
#include <hip/hip_runtime.h>

#include <float.h>
#include <math.h>

#include "../../include/cfd.h"

namespace qm {

#define QM_HD __host__ __device__ __forceinline__

constexpr double kEps = DBL_EPSILON;   // std::f64::EPSILON

// orientation (intersection.rs:3-13): 0 collinear, 1 clockwise, 2 counter-clockwise
QM_HD int orientation(const cfd_point &p, const cfd_point &q, const cfd_point &r) {
    const double val = (q.y - p.y) * (r.x - q.x) - (q.x - p.x) * (r.y - q.y);
    if (fabs(val) < kEps) return 0;
    return val > 0.0 ? 1 : 2;
}

// on_segment (intersection.rs:15-18): q within the bounding box of p-r (+-eps)
QM_HD bool on_segment(const cfd_point &p, const cfd_point &q, const cfd_point &r) {
    return (q.x <= fmax(p.x, r.x) + kEps && q.x >= fmin(p.x, r.x) - kEps) &&
           (q.y <= fmax(p.y, r.y) + kEps && q.y >= fmin(p.y, r.y) - kEps);
}

// do_intersect (intersection.rs:20-38)
QM_HD bool do_intersect(const cfd_point &p, const cfd_point &q, const cfd_point &a,
                        const cfd_point &b) {
    const int o1 = orientation(p, q, a);
    const int o2 = orientation(p, q, b);
    const int o3 = orientation(a, b, p);
    const int o4 = orientation(a, b, q);
    if (o1 != o2 && o3 != o4) return true;
    if (o1 == 0 && on_segment(p, a, q)) return true;
    if (o2 == 0 && on_segment(p, b, q)) return true;
    if (o3 == 0 && on_segment(a, p, b)) return true;
    if (o4 == 0 && on_segment(a, q, b)) return true;
    return false;
}

// line_segment_intersection (intersection.rs:41-63): false for None
QM_HD bool segment_intersection(const cfd_point &p, const cfd_point &q, const cfd_point &a,
                                const cfd_point &b, cfd_point *out) {
    if (!do_intersect(p, q, a, b)) return false;
    const double a1 = q.y - p.y;
    const double b1 = p.x - q.x;
    const double c1 = a1 * p.x + b1 * p.y;
    const double a2 = b.y - a.y;
    const double b2 = a.x - b.x;
    const double c2 = a2 * a.x + b2 * a.y;
    const double det = a1 * b2 - a2 * b1;
    if (fabs(det) < kEps) return false;
    out->x = (b2 * c1 - b1 * c2) / det;
    out->y = (a1 * c2 - a2 * c1) / det;
    return true;
}

QM_HD bool seen(const cfd_point *pts, int n, const cfd_point &x) {
    for (int k = 0; k < n; ++k)
        if (fabs(pts[k].x - x.x) < kEps && fabs(pts[k].y - x.y) < kEps) return true;
    return false;
}

// intersect_quad_edge (intersection.rs:68-129) for the axis-aligned quad of
// Quad::new_rect (quad.rs:24-35): vertices bottom-left, bottom-right,
// top-right, top-left.  Writes at most 8 points into out, returns the count.
QM_HD int intersect_quad_edge(const cfd_point &center, double hw, double hh, const cfd_point &p1,
                              const cfd_point &p2, cfd_point *out) {
    const double left = center.x - hw, right = center.x + hw;
    const double bottom = center.y - hh, top = center.y + hh;
    const cfd_point v[4] = {{left, bottom}, {right, bottom}, {right, top}, {left, top}};
    int n = 0;
    for (int i = 0; i < 4; ++i) {
        const cfd_point &v1 = v[i];
        const cfd_point &v2 = v[(i + 1) % 4];
        if (orientation(p1, p2, v1) == 0 && orientation(p1, p2, v2) == 0) {
            const double d_x = p2.x - p1.x;
            const double d_y = p2.y - p1.y;
            const double norm = d_x * d_x + d_y * d_y;
            if (fabs(norm) < kEps) continue;
            const double t_v1 = ((v1.x - p1.x) * d_x + (v1.y - p1.y) * d_y) / norm;
            const double t_v2 = ((v2.x - p1.x) * d_x + (v2.y - p1.y) * d_y) / norm;
            const double t_start = fmax(fmin(t_v1, t_v2), 0.0);
            const double t_end = fmin(fmax(t_v1, t_v2), 1.0);
            if (t_start <= t_end + kEps) {
                const cfd_point s = {p1.x + t_start * d_x, p1.y + t_start * d_y};
                const cfd_point e = {p1.x + t_end * d_x, p1.y + t_end * d_y};
                if (!seen(out, n, s)) out[n++] = s;
                if (!seen(out, n, e)) out[n++] = e;
                continue;
            }
        }
        cfd_point x;
        if (segment_intersection(p1, p2, v1, v2, &x) && !seen(out, n, x)) out[n++] = x;
    }
    return n;
}

// Ray casting of one ring (polygon.rs:76-88): pts[0..n) in polygon order.
QM_HD bool ring_contains(const cfd_point *pts, int n, const cfd_point &p) {
    int count = 0;
    for (int i = 0; i < n; ++i) {
        const int j = (i + 1) % n;
        const cfd_point &a = pts[i];
        const cfd_point &b = pts[j];
        if ((a.y > p.y) != (b.y > p.y)) {
            const double x_intersect = a.x + (p.y - a.y) * (b.x - a.x) / (b.y - a.y);
            if (p.x < x_intersect) count += 1;
        }
    }
    return count % 2 == 1;
}

}  // namespace qm
