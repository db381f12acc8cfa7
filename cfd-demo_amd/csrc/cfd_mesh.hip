// cfd_mesh.hip — the reference's adaptive quadtree mesher (src/quad_mesh,
// src/utils/intersection.rs) behind include/cfd.h: polygons with holes, the
// recursive tesselation (host: a depth-first recursion over a handful of
// polygon edges), and Mesh::from_quad_tree (mesh.rs:51-227) on the GPU.
//
// Mesh::from_quad_tree is the data-parallel part.  The reference filters the
// leaves by polygon membership, then runs an O(n^2) double loop comparing
// every cell's bounds with every other cell's to find face neighbours
// (mesh.rs:131-154), then intersects every cell's quad with every polygon
// edge (mesh.rs:186-210).  Here each of those is a count kernel, a device
// prefix sum (hipcub) and a fill kernel that repeats the same test in the
// same order, so every neighbour list comes out in ascending cell order
// exactly as the reference's push loop builds it.  The pair loop streams the
// other cells' bounds through LDS tiles (256 cells x 4 doubles) shared by a
// workgroup.  All arithmetic is the reference's f64 (quad_geom.h).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/cfd.h"
#include "quad_geom.h"

extern "C" void cfdrt_set_error(const char *msg);

using qm::kEps;

namespace {

int err(int code, const char *msg) {
    cfdrt_set_error(msg);
    return code;
}

#define MESH_HIP(expr)                                                                     \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess) {                                                            \
            cfdrt_set_error((std::string(#expr) + ": " + hipGetErrorString(e_)).c_str());  \
            return CFD_EHIP;                                                               \
        }                                                                                  \
    } while (0)

// polygon_is_self_intersecting (polygon.rs:208-231)
bool self_intersecting(const std::vector<cfd_point> &pts) {
    const size_t n = pts.size();
    if (n < 4) return false;
    for (size_t i = 0; i < n; ++i) {
        const cfd_point &p1 = pts[i], &q1 = pts[(i + 1) % n];
        for (size_t j = i + 1; j < n; ++j) {
            if (j == i || (j + 1) % n == i || (i + 1) % n == j) continue;
            if (qm::do_intersect(p1, q1, pts[j], pts[(j + 1) % n])) return true;
        }
    }
    return false;
}

cfd_point tl(const cfd_aabb &b) { return {b.center.x - b.half_width, b.center.y - b.half_height}; }
cfd_point tr(const cfd_aabb &b) { return {b.center.x + b.half_width, b.center.y - b.half_height}; }
cfd_point bl(const cfd_aabb &b) { return {b.center.x - b.half_width, b.center.y + b.half_height}; }
cfd_point br(const cfd_aabb &b) { return {b.center.x + b.half_width, b.center.y + b.half_height}; }

// AABB::intersects_segment (aabb.rs:78-89)
bool aabb_intersects_segment(const cfd_aabb &box, const cfd_point &a, const cfd_point &b) {
    const cfd_point t_l = tl(box), t_r = tr(box), b_l = bl(box), b_r = br(box);
    return qm::do_intersect(a, b, t_l, t_r) || qm::do_intersect(a, b, t_r, b_r) ||
           qm::do_intersect(a, b, b_r, b_l) || qm::do_intersect(a, b, b_l, t_l);
}

}  // namespace

struct cfd_polygon {
    std::vector<cfd_point> vb;      // vertex_buffer
    std::vector<uint64_t> verts;    // vertices (indices into vb)
    std::vector<cfd_polygon *> holes;
    ~cfd_polygon() {
        for (cfd_polygon *h : holes) delete h;
    }
    std::vector<cfd_point> ring() const {
        std::vector<cfd_point> r(verts.size());
        for (size_t k = 0; k < verts.size(); ++k) r[k] = vb[verts[k]];
        return r;
    }
    // contains_point (polygon.rs:81-103)
    bool contains(const cfd_point &p) const {
        const std::vector<cfd_point> r = ring();
        if (!qm::ring_contains(r.data(), (int)r.size(), p)) return false;
        for (const cfd_polygon *h : holes)
            if (h->contains(p)) return false;
        return true;
    }
    // edges (polygon.rs:186-196): the reference pairs vertex_buffer[i] with
    // vertex_buffer[(i + 1) % vertices.len()] for each vertex index i
    std::vector<cfd_point> edges() const {
        std::vector<cfd_point> e;
        const size_t n = verts.size();
        for (uint64_t i : verts) {
            e.push_back(vb[i]);
            e.push_back(vb[(i + 1) % n]);
        }
        return e;
    }
    // edges_intersect_aabb (polygon.rs:119-133)
    bool edges_intersect(const cfd_aabb &box) const {
        const std::vector<cfd_point> e = edges();
        for (size_t k = 0; k + 1 < e.size(); k += 2)
            if (aabb_intersects_segment(box, e[k], e[k + 1])) return true;
        for (const cfd_polygon *h : holes)
            if (h->edges_intersect(box)) return true;
        return false;
    }
    // bounding_box (polygon.rs:150-178): over the whole vertex buffer
    cfd_aabb bbox() const {
        double min_x = INFINITY, max_x = -INFINITY, min_y = INFINITY, max_y = -INFINITY;
        for (const cfd_point &p : vb) {
            min_x = std::fmin(min_x, p.x);
            max_x = std::fmax(max_x, p.x);
            min_y = std::fmin(min_y, p.y);
            max_y = std::fmax(max_y, p.y);
        }
        cfd_aabb b;
        b.center = {(min_x + max_x) / 2.0, (min_y + max_y) / 2.0};
        b.half_width = (max_x - min_x) / 2.0;
        b.half_height = (max_y - min_y) / 2.0;
        return b;
    }
};

struct cfd_quadtree {
    std::vector<cfd_aabb> boxes;
    std::vector<int64_t> children;   // 4 per node, -1 for leaves
    uint64_t leaves = 0;
};

struct cfd_mesh {
    std::vector<double> cx, cy, hw, hh;
    std::vector<uint64_t> nb_range[4], nb_index[4];
    std::vector<uint64_t> x_range;
    std::vector<cfd_point> x_points;
    double build_ms = 0.0;
};

namespace {

// Every edge edges_intersect_aabb visits (polygon.rs:119-133: own edges, then
// each hole's, recursively), flattened once per tesselation: the predicate
// is an OR over them, so the order is immaterial.
void all_edges(const cfd_polygon &p, std::vector<cfd_point> *out) {
    const std::vector<cfd_point> e = p.edges();
    out->insert(out->end(), e.begin(), e.end());
    for (const cfd_polygon *h : p.holes) all_edges(*h, out);
}

// tesselate_impl (quad_tree.rs:22-100), depth-first pre-order
int tesselate_node(const std::vector<cfd_point> &edges, const cfd_aabb &b, double feature,
                   double max_cell, int depth, cfd_quadtree *t) {
    if (depth > 64) return err(CFD_EINVAL, "tesselate: no termination (feature_size <= 0?)");
    const double cell_size = std::fmin(2.0 * b.half_width, 2.0 * b.half_height);
    bool intersects_edges = false;
    for (size_t k = 0; k + 1 < edges.size() && !intersects_edges; k += 2)
        intersects_edges = aabb_intersects_segment(b, edges[k], edges[k + 1]);
    const int64_t me = (int64_t)t->boxes.size();
    t->boxes.push_back(b);
    t->children.insert(t->children.end(), {-1, -1, -1, -1});
    if ((cell_size <= feature || !intersects_edges) && cell_size <= max_cell) {
        t->leaves++;
        return 0;
    }
    const double nhw = b.half_width / 2.0, nhh = b.half_height / 2.0;
    const double cx = b.center.x, cy = b.center.y;
    const cfd_aabb q[4] = {{{cx - nhw, cy - nhh}, nhw, nhh},
                           {{cx + nhw, cy - nhh}, nhw, nhh},
                           {{cx - nhw, cy + nhh}, nhw, nhh},
                           {{cx + nhw, cy + nhh}, nhw, nhh}};
    for (int k = 0; k < 4; ++k) {
        t->children[me * 4 + k] = (int64_t)t->boxes.size();
        int rc = tesselate_node(edges, q[k], feature, max_cell, depth + 1, t);
        if (rc) return rc;
    }
    return 0;
}

// ------------------------------------------------------------------ kernels

struct Rings {
    const cfd_point *pts;   // outer ring, then each hole's ring
    const int *off;         // ring k = pts[off[k] .. off[k+1])
    int n_rings;            // 1 + holes
};

// contains_point with one level of holes (holes without holes of their own)
__device__ bool dev_contains(const Rings &R, const cfd_point &p) {
    if (!qm::ring_contains(R.pts + R.off[0], R.off[1] - R.off[0], p)) return false;
    for (int k = 1; k < R.n_rings; ++k)
        if (qm::ring_contains(R.pts + R.off[k], R.off[k + 1] - R.off[k], p)) return false;
    return true;
}

// mesh.rs:57-78: keep a leaf when its centre or a vertex is inside.
__global__ void k_mesh_filter(const double *cx, const double *cy, const double *hw,
                              const double *hh, long n, Rings R, int *keep) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const cfd_point c = {cx[i], cy[i]};
    const bool center_inside = dev_contains(R, c);
    const double left = cx[i] - hw[i], right = cx[i] + hw[i];
    const double bottom = cy[i] - hh[i], top = cy[i] + hh[i];
    const bool vertex_inside = dev_contains(R, {left, bottom}) || dev_contains(R, {left, top}) ||
                               dev_contains(R, {right, bottom}) || dev_contains(R, {right, top});
    keep[i] = (center_inside || vertex_inside) ? 1 : 0;
}

// compaction + the bounds of mesh.rs:101-110
__global__ void k_mesh_compact(const double *cx, const double *cy, const double *hw,
                               const double *hh, long n, const int *keep, const int *pos,
                               double *ocx, double *ocy, double *ohw, double *ohh, double4 *bounds) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !keep[i]) return;
    const int k = pos[i];
    ocx[k] = cx[i];
    ocy[k] = cy[i];
    ohw[k] = hw[i];
    ohh[k] = hh[i];
    bounds[k] = make_double4(cx[i] - hw[i], cx[i] + hw[i], cy[i] - hh[i], cy[i] + hh[i]);
}

constexpr int kTile = 256;

// mesh.rs:120-154.  FILL 0: count per face; FILL 1: write the indices at the
// scanned offsets, j ascending.
template <int FILL>
__global__ __launch_bounds__(kTile) void k_mesh_neighbors(const double4 *bounds, int n,
                                                          int *counts, const int *starts,
                                                          int *indexes) {
    __shared__ double4 tile[kTile];
    const int i = (int)blockIdx.x * kTile + (int)threadIdx.x;
    const bool live = i < n;
    const double4 me = live ? bounds[i] : make_double4(0, 0, 0, 0);   // (xmin, xmax, ymin, ymax)
    const double eps = 1e-6;
    int c[4] = {0, 0, 0, 0};
    int w[4] = {0, 0, 0, 0};
    if (FILL && live)
        for (int d = 0; d < 4; ++d) w[d] = starts[d * n + i];
    for (int t0 = 0; t0 < n; t0 += kTile) {
        __syncthreads();
        if (t0 + (int)threadIdx.x < n) tile[threadIdx.x] = bounds[t0 + threadIdx.x];
        __syncthreads();
        if (!live) continue;
        const int m = min(kTile, n - t0);
        for (int q = 0; q < m; ++q) {
            const int j = t0 + q;
            if (j == i) continue;
            const double4 o = tile[q];
            const bool y_overlap = me.z < o.w && me.w > o.z;
            const bool x_overlap = me.x < o.y && me.y > o.x;
            const bool e = fabs(o.x - me.y) < eps && y_overlap;   // east
            const bool wst = fabs(o.y - me.x) < eps && y_overlap; // west
            const bool nth = fabs(o.z - me.w) < eps && x_overlap; // north
            const bool sth = fabs(o.w - me.z) < eps && x_overlap; // south
            if (FILL) {
                if (e) indexes[w[0]++] = j;
                if (wst) indexes[w[1]++] = j;
                if (nth) indexes[w[2]++] = j;
                if (sth) indexes[w[3]++] = j;
            } else {
                c[0] += e;
                c[1] += wst;
                c[2] += nth;
                c[3] += sth;
            }
        }
    }
    if (!FILL && live)
        for (int d = 0; d < 4; ++d) counts[d * n + i] = c[d];
}

// mesh.rs:186-210: every cell's quad against every polygon edge, outer
// polygon first, then each hole, in edge order.
template <int FILL>
__global__ void k_mesh_intersections(const double *cx, const double *cy, const double *hw,
                                     const double *hh, int n, const cfd_point *edges, int n_edges,
                                     int *counts, const int *starts, cfd_point *points) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= n) return;
    const cfd_point c = {cx[i], cy[i]};
    int total = 0, w = FILL ? starts[i] : 0;
    cfd_point buf[8];
    for (int e = 0; e < n_edges; ++e) {
        const int k = qm::intersect_quad_edge(c, hw[i], hh[i], edges[2 * e], edges[2 * e + 1], buf);
        if (FILL)
            for (int q = 0; q < k; ++q) points[w++] = buf[q];
        total += k;
    }
    if (!FILL) counts[i] = total;
}

// exclusive prefix sum of n ints into out (device), total into *sum (host)
int exclusive_scan(const int *in, int *out, int n, long *sum, hipStream_t s) {
    if (n == 0) {
        *sum = 0;
        return 0;
    }
    size_t bytes = 0;
    MESH_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in, out, n, s));
    void *tmp = nullptr;
    MESH_HIP(hipMalloc(&tmp, bytes + 16));
    MESH_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, bytes, in, out, n, s));
    int last_in = 0, last_out = 0;
    MESH_HIP(hipMemcpyAsync(&last_in, in + n - 1, 4, hipMemcpyDeviceToHost, s));
    MESH_HIP(hipMemcpyAsync(&last_out, out + n - 1, 4, hipMemcpyDeviceToHost, s));
    MESH_HIP(hipStreamSynchronize(s));
    MESH_HIP(hipFree(tmp));
    *sum = (long)last_in + (long)last_out;
    return 0;
}

struct DevBuf {
    std::vector<void *> ptrs;
    ~DevBuf() {
        for (void *p : ptrs) (void)hipFree(p);
    }
    template <class T> int alloc(T **p, size_t n) {
        void *q = nullptr;
        hipError_t e = hipMalloc(&q, n * sizeof(T) + 64);
        if (e != hipSuccess) return err(CFD_EHIP, "hipMalloc failed (mesh)");
        ptrs.push_back(q);
        *p = (T *)q;
        return 0;
    }
};

int build_mesh(const cfd_quadtree &t, const cfd_polygon &poly, int device, cfd_mesh *out) {
    for (const cfd_polygon *h : poly.holes)
        if (!h->holes.empty()) return err(CFD_EINVAL, "mesh: holes with holes are not supported");
    MESH_HIP(hipSetDevice(device));
    // gather_leaves (mesh.rs:352-370): pre-order leaves
    std::vector<double> lcx, lcy, lhw, lhh;
    for (size_t k = 0; k < t.boxes.size(); ++k)
        if (t.children[4 * k] < 0) {
            lcx.push_back(t.boxes[k].center.x);
            lcy.push_back(t.boxes[k].center.y);
            lhw.push_back(t.boxes[k].half_width);
            lhh.push_back(t.boxes[k].half_height);
        }
    const long nl = (long)lcx.size();
    if (nl >= (1L << 30)) return err(CFD_EINVAL, "mesh: too many leaves");
    // polygon rings and edges (outer first, then holes in order)
    std::vector<cfd_point> pts = poly.ring();
    std::vector<int> off{0, (int)pts.size()};
    std::vector<cfd_point> edges = poly.edges();
    for (const cfd_polygon *h : poly.holes) {
        const std::vector<cfd_point> r = h->ring();
        pts.insert(pts.end(), r.begin(), r.end());
        off.push_back((int)pts.size());
        const std::vector<cfd_point> e = h->edges();
        edges.insert(edges.end(), e.begin(), e.end());
    }
    hipStream_t s;
    MESH_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    struct StreamGuard {
        hipStream_t s;
        ~StreamGuard() { (void)hipStreamDestroy(s); }
    } sg{s};
    hipEvent_t e0, e1;
    MESH_HIP(hipEventCreate(&e0));
    MESH_HIP(hipEventCreate(&e1));
    DevBuf db;
    double *dcx, *dcy, *dhw, *dhh, *ocx, *ocy, *ohw, *ohh;
    double4 *bounds;
    int *keep, *pos, *dpoff;
    cfd_point *dpts, *dedges;
    int rc;
    const size_t L = (size_t)std::max<long>(nl, 1);
    if ((rc = db.alloc(&dcx, L)) || (rc = db.alloc(&dcy, L)) || (rc = db.alloc(&dhw, L)) ||
        (rc = db.alloc(&dhh, L)) || (rc = db.alloc(&ocx, L)) || (rc = db.alloc(&ocy, L)) ||
        (rc = db.alloc(&ohw, L)) || (rc = db.alloc(&ohh, L)) || (rc = db.alloc(&bounds, L)) ||
        (rc = db.alloc(&keep, L)) || (rc = db.alloc(&pos, L)) ||
        (rc = db.alloc(&dpts, pts.size())) || (rc = db.alloc(&dpoff, off.size())) ||
        (rc = db.alloc(&dedges, std::max<size_t>(edges.size(), 1))))
        return rc;
    MESH_HIP(hipMemcpyAsync(dcx, lcx.data(), nl * 8, hipMemcpyHostToDevice, s));
    MESH_HIP(hipMemcpyAsync(dcy, lcy.data(), nl * 8, hipMemcpyHostToDevice, s));
    MESH_HIP(hipMemcpyAsync(dhw, lhw.data(), nl * 8, hipMemcpyHostToDevice, s));
    MESH_HIP(hipMemcpyAsync(dhh, lhh.data(), nl * 8, hipMemcpyHostToDevice, s));
    MESH_HIP(hipMemcpyAsync(dpts, pts.data(), pts.size() * sizeof(cfd_point), hipMemcpyHostToDevice, s));
    MESH_HIP(hipMemcpyAsync(dpoff, off.data(), off.size() * 4, hipMemcpyHostToDevice, s));
    if (!edges.empty())
        MESH_HIP(hipMemcpyAsync(dedges, edges.data(), edges.size() * sizeof(cfd_point),
                                hipMemcpyHostToDevice, s));
    MESH_HIP(hipEventRecord(e0, s));
    const int B = 256;
    Rings R{dpts, dpoff, (int)off.size() - 1};
    long n = 0;
    if (nl > 0) {
        hipLaunchKernelGGL(k_mesh_filter, dim3((unsigned)((nl + B - 1) / B)), dim3(B), 0, s, dcx, dcy,
                           dhw, dhh, nl, R, keep);
        if ((rc = exclusive_scan(keep, pos, (int)nl, &n, s))) return rc;
        hipLaunchKernelGGL(k_mesh_compact, dim3((unsigned)((nl + B - 1) / B)), dim3(B), 0, s, dcx,
                           dcy, dhw, dhh, nl, keep, pos, ocx, ocy, ohw, ohh, bounds);
    }
    const int nc = (int)n;
    const size_t NC = (size_t)std::max(nc, 1);
    int *counts, *starts, *xc, *xs;
    if ((rc = db.alloc(&counts, 4 * NC)) || (rc = db.alloc(&starts, 4 * NC)) ||
        (rc = db.alloc(&xc, NC)) || (rc = db.alloc(&xs, NC)))
        return rc;
    long tot[4] = {0, 0, 0, 0}, xtot = 0;
    int *idx[4] = {nullptr, nullptr, nullptr, nullptr};
    cfd_point *xpts = nullptr;
    if (nc > 0) {
        const dim3 g((unsigned)((nc + kTile - 1) / kTile));
        hipLaunchKernelGGL(k_mesh_neighbors<0>, g, dim3(kTile), 0, s, bounds, nc, counts,
                           (const int *)nullptr, (int *)nullptr);
        for (int d = 0; d < 4; ++d)
            if ((rc = exclusive_scan(counts + (size_t)d * nc, starts + (size_t)d * nc, nc, &tot[d], s)))
                return rc;
        // the four faces' lists live in one array, face after face
        int *all = nullptr;
        const long sum = tot[0] + tot[1] + tot[2] + tot[3];
        if ((rc = db.alloc(&all, (size_t)std::max<long>(sum, 1)))) return rc;
        // offset the per-face starts into one concatenated index array
        std::vector<int> hstarts(4 * (size_t)nc);
        MESH_HIP(hipMemcpyAsync(hstarts.data(), starts, 4 * (size_t)nc * 4, hipMemcpyDeviceToHost, s));
        MESH_HIP(hipStreamSynchronize(s));
        long base = 0;
        for (int d = 0; d < 4; ++d) {
            for (int k = 0; k < nc; ++k) hstarts[(size_t)d * nc + k] += (int)base;
            base += tot[d];
        }
        MESH_HIP(hipMemcpyAsync(starts, hstarts.data(), 4 * (size_t)nc * 4, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_mesh_neighbors<1>, g, dim3(kTile), 0, s, bounds, nc, (int *)nullptr,
                           (const int *)starts, all);
        base = 0;
        for (int d = 0; d < 4; ++d) {
            idx[d] = all + base;
            base += tot[d];
        }
        // cell / polygon-edge intersections
        const int ne = (int)(edges.size() / 2);
        const dim3 gx((unsigned)((nc + B - 1) / B));
        hipLaunchKernelGGL(k_mesh_intersections<0>, gx, dim3(B), 0, s, ocx, ocy, ohw, ohh, nc,
                           dedges, ne, xc, (const int *)nullptr, (cfd_point *)nullptr);
        if ((rc = exclusive_scan(xc, xs, nc, &xtot, s))) return rc;
        if ((rc = db.alloc(&xpts, (size_t)std::max<long>(xtot, 1)))) return rc;
        hipLaunchKernelGGL(k_mesh_intersections<1>, gx, dim3(B), 0, s, ocx, ocy, ohw, ohh, nc,
                           dedges, ne, (int *)nullptr, (const int *)xs, xpts);
    }
    MESH_HIP(hipGetLastError());
    MESH_HIP(hipEventRecord(e1, s));
    MESH_HIP(hipStreamSynchronize(s));
    float ms = 0.f;
    MESH_HIP(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    out->build_ms = ms;
    // results to the host SoA mesh
    out->cx.resize(nc);
    out->cy.resize(nc);
    out->hw.resize(nc);
    out->hh.resize(nc);
    if (nc > 0) {
        MESH_HIP(hipMemcpy(out->cx.data(), ocx, (size_t)nc * 8, hipMemcpyDeviceToHost));
        MESH_HIP(hipMemcpy(out->cy.data(), ocy, (size_t)nc * 8, hipMemcpyDeviceToHost));
        MESH_HIP(hipMemcpy(out->hw.data(), ohw, (size_t)nc * 8, hipMemcpyDeviceToHost));
        MESH_HIP(hipMemcpy(out->hh.data(), ohh, (size_t)nc * 8, hipMemcpyDeviceToHost));
    }
    std::vector<int> hc(4 * (size_t)nc), hs(4 * (size_t)nc);
    if (nc > 0) {
        MESH_HIP(hipMemcpy(hc.data(), counts, hc.size() * 4, hipMemcpyDeviceToHost));
        MESH_HIP(hipMemcpy(hs.data(), starts, hs.size() * 4, hipMemcpyDeviceToHost));
    }
    long base = 0;
    for (int d = 0; d < 4; ++d) {
        std::vector<int> li((size_t)tot[d]);
        if (tot[d] > 0)
            MESH_HIP(hipMemcpy(li.data(), idx[d], (size_t)tot[d] * 4, hipMemcpyDeviceToHost));
        out->nb_index[d].assign(li.begin(), li.end());
        out->nb_range[d].resize(2 * (size_t)nc);
        for (int k = 0; k < nc; ++k) {
            const uint64_t st = (uint64_t)(hs[(size_t)d * nc + k] - base);
            out->nb_range[d][2 * k] = st;
            out->nb_range[d][2 * k + 1] = st + (uint64_t)hc[(size_t)d * nc + k];
        }
        base += tot[d];
    }
    std::vector<int> hxc((size_t)nc), hxs((size_t)nc);
    if (nc > 0) {
        MESH_HIP(hipMemcpy(hxc.data(), xc, (size_t)nc * 4, hipMemcpyDeviceToHost));
        MESH_HIP(hipMemcpy(hxs.data(), xs, (size_t)nc * 4, hipMemcpyDeviceToHost));
    }
    out->x_points.resize((size_t)xtot);
    if (xtot > 0)
        MESH_HIP(hipMemcpy(out->x_points.data(), xpts, (size_t)xtot * sizeof(cfd_point),
                           hipMemcpyDeviceToHost));
    out->x_range.resize(2 * (size_t)nc);
    for (int k = 0; k < nc; ++k) {
        out->x_range[2 * k] = (uint64_t)hxs[k];
        out->x_range[2 * k + 1] = (uint64_t)(hxs[k] + hxc[k]);
    }
    return 0;
}

int check_ptr(const void *p) { return p ? 0 : err(CFD_EINVAL, "null argument"); }

}  // namespace

// =============================================================== C ABI

extern "C" {

int cfd_polygon_new(const cfd_point *vertex_buffer, size_t n_points, const uint64_t *vertices,
                    size_t n_vertices, cfd_polygon **out, int *poly_error) {
    if (!out || !poly_error || (n_points && !vertex_buffer) || (n_vertices && !vertices))
        return err(CFD_EINVAL, "null argument");
    *out = nullptr;
    *poly_error = CFD_POLY_OK;
    if (n_vertices < 3) {   // polygon.rs:21-24
        *poly_error = CFD_POLY_NOT_ENOUGH_VERTICES;
        return 0;
    }
    for (size_t k = 0; k < n_vertices; ++k)
        if (vertices[k] >= n_points) return err(CFD_EINVAL, "vertex index out of range (reference panics)");
    cfd_polygon *p = new cfd_polygon();
    p->vb.assign(vertex_buffer, vertex_buffer + n_points);
    p->verts.assign(vertices, vertices + n_vertices);
    if (self_intersecting(p->ring())) {   // polygon.rs:29-32
        delete p;
        *poly_error = CFD_POLY_SELF_INTERSECTING;
        return 0;
    }
    *out = p;
    return 0;
}

int cfd_polygon_new_rect(double x, double y, double w, double h, cfd_polygon **out) {
    const cfd_point vb[4] = {{x, y}, {x + w, y}, {x + w, y + h}, {x, y + h}};
    const uint64_t v[4] = {0, 1, 2, 3};
    int pe = 0;
    int rc = cfd_polygon_new(vb, 4, v, 4, out, &pe);
    if (rc) return rc;
    if (pe) return err(CFD_EINVAL, "new_rect: degenerate rectangle (the reference unwrap panics)");
    return 0;
}

int cfd_polygon_new_regular(cfd_point center, double radius, size_t n, double start_angle,
                            cfd_polygon **out) {
    std::vector<cfd_point> vb;
    std::vector<uint64_t> v;
    const double tau = 6.283185307179586;   // std::f64::consts::TAU
    for (size_t i = 0; i < n; ++i) {
        const double theta = (double)i * tau / (double)n + start_angle;
        vb.push_back({center.x + radius * std::cos(theta), center.y + radius * std::sin(theta)});
        v.push_back(i);
    }
    int pe = 0;
    int rc = cfd_polygon_new(vb.data(), vb.size(), v.data(), v.size(), out, &pe);
    if (rc) return rc;
    if (pe) return err(CFD_EINVAL, "new_polygon: invalid polygon (the reference unwrap panics)");
    return 0;
}

int cfd_polygon_add_hole(cfd_polygon *p, cfd_polygon *hole, int *poly_error) {
    if (!p || !hole || !poly_error) return err(CFD_EINVAL, "null argument");
    *poly_error = CFD_POLY_OK;
    for (uint64_t idx : hole->verts)   // polygon.rs:71-76
        if (!p->contains(hole->vb[idx])) {
            *poly_error = CFD_POLY_INVALID_HOLE;
            return 0;
        }
    p->holes.push_back(hole);
    return 0;
}

int cfd_polygon_contains_point(const cfd_polygon *p, cfd_point pt, int *result) {
    if (check_ptr(p) || check_ptr(result)) return CFD_EINVAL;
    *result = p->contains(pt) ? 1 : 0;
    return 0;
}

int cfd_polygon_intersects_aabb(const cfd_polygon *p, const cfd_aabb *b, int *result) {
    if (check_ptr(p) || check_ptr(b) || check_ptr(result)) return CFD_EINVAL;
    *result = (p->contains(tl(*b)) || p->contains(tr(*b)) || p->contains(bl(*b)) ||
               p->contains(br(*b)) || p->contains(b->center))
                  ? 1
                  : 0;
    return 0;
}

int cfd_polygon_edges_intersect_aabb(const cfd_polygon *p, const cfd_aabb *b, int *result) {
    if (check_ptr(p) || check_ptr(b) || check_ptr(result)) return CFD_EINVAL;
    *result = p->edges_intersect(*b) ? 1 : 0;
    return 0;
}

int cfd_polygon_bounding_box(const cfd_polygon *p, cfd_aabb *out) {
    if (check_ptr(p) || check_ptr(out)) return CFD_EINVAL;
    *out = p->bbox();
    return 0;
}

int cfd_polygon_bounding_square(const cfd_polygon *p, cfd_aabb *out) {
    if (check_ptr(p) || check_ptr(out)) return CFD_EINVAL;
    const cfd_aabb b = p->bbox();
    const double max_dim = std::fmax(2.0 * b.half_width, 2.0 * b.half_height);
    out->center = b.center;
    out->half_width = max_dim / 2.0;
    out->half_height = max_dim / 2.0;
    return 0;
}

int cfd_polygon_edges(const cfd_polygon *p, cfd_point *out, size_t max_edges, size_t *n_edges) {
    if (check_ptr(p) || check_ptr(n_edges)) return CFD_EINVAL;
    const std::vector<cfd_point> e = p->edges();
    *n_edges = e.size() / 2;
    if (out)
        for (size_t k = 0; k < std::min(max_edges * 2, e.size()); ++k) out[k] = e[k];
    return 0;
}

void cfd_polygon_destroy(cfd_polygon *p) { delete p; }

int cfd_geom_do_intersect(cfd_point p, cfd_point q, cfd_point a, cfd_point b, int *result) {
    if (check_ptr(result)) return CFD_EINVAL;
    *result = qm::do_intersect(p, q, a, b) ? 1 : 0;
    return 0;
}

int cfd_geom_segment_intersection(cfd_point p, cfd_point q, cfd_point a, cfd_point b,
                                  cfd_point *out, int *found) {
    if (check_ptr(out) || check_ptr(found)) return CFD_EINVAL;
    *found = qm::segment_intersection(p, q, a, b, out) ? 1 : 0;
    return 0;
}

int cfd_geom_intersect_quad_edge(cfd_point center, double hw, double hh, cfd_point p1,
                                 cfd_point p2, cfd_point *out8, int *n) {
    if (check_ptr(out8) || check_ptr(n)) return CFD_EINVAL;
    *n = qm::intersect_quad_edge(center, hw, hh, p1, p2, out8);
    return 0;
}

int cfd_tesselate(const cfd_polygon *p, double feature_size, double max_cell_size,
                  cfd_quadtree **out) {
    if (check_ptr(p) || check_ptr(out)) return CFD_EINVAL;
    *out = nullptr;
    cfd_quadtree *t = new cfd_quadtree();
    cfd_aabb root;
    cfd_polygon_bounding_square(p, &root);   // quad_tree.rs:18-20
    std::vector<cfd_point> edges;
    all_edges(*p, &edges);
    int rc = tesselate_node(edges, root, feature_size, max_cell_size, 0, t);
    if (rc) {
        delete t;
        return rc;
    }
    *out = t;
    return 0;
}

int cfd_quadtree_size(const cfd_quadtree *t, uint64_t *n_nodes, uint64_t *n_leaves) {
    if (check_ptr(t)) return CFD_EINVAL;
    if (n_nodes) *n_nodes = t->boxes.size();
    if (n_leaves) *n_leaves = t->leaves;
    return 0;
}

int cfd_quadtree_nodes(const cfd_quadtree *t, cfd_aabb *boxes, int64_t *children4) {
    if (check_ptr(t)) return CFD_EINVAL;
    if (boxes) std::memcpy(boxes, t->boxes.data(), t->boxes.size() * sizeof(cfd_aabb));
    if (children4) std::memcpy(children4, t->children.data(), t->children.size() * 8);
    return 0;
}

void cfd_quadtree_destroy(cfd_quadtree *t) { delete t; }

int cfd_mesh_from_quadtree(const cfd_quadtree *t, const cfd_polygon *p, int device,
                           cfd_mesh **out) {
    if (check_ptr(t) || check_ptr(p) || check_ptr(out)) return CFD_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return err(CFD_EHIP, "no HIP device available");
    if (device < 0 || device >= ndev) return err(CFD_EINVAL, "device ordinal out of range");
    cfd_mesh *m = new cfd_mesh();
    int rc = build_mesh(*t, *p, device, m);
    if (rc) {
        delete m;
        return rc;
    }
    *out = m;
    return 0;
}

int cfd_mesh_sizes(const cfd_mesh *m, uint64_t *s) {
    if (check_ptr(m) || check_ptr(s)) return CFD_EINVAL;
    s[0] = m->cx.size();
    for (int d = 0; d < 4; ++d) s[1 + d] = m->nb_index[d].size();
    s[5] = m->x_points.size();
    return 0;
}

int cfd_mesh_cells(const cfd_mesh *m, double *cx, double *cy, double *hw, double *hh) {
    if (check_ptr(m)) return CFD_EINVAL;
    const size_t n = m->cx.size() * 8;
    if (cx) std::memcpy(cx, m->cx.data(), n);
    if (cy) std::memcpy(cy, m->cy.data(), n);
    if (hw) std::memcpy(hw, m->hw.data(), n);
    if (hh) std::memcpy(hh, m->hh.data(), n);
    return 0;
}

int cfd_mesh_neighbors(const cfd_mesh *m, int face, uint64_t *ranges, uint64_t *indexes) {
    if (check_ptr(m)) return CFD_EINVAL;
    if (face < 0 || face > 3) return err(CFD_EINVAL, "face must be 0..3");
    if (ranges) std::memcpy(ranges, m->nb_range[face].data(), m->nb_range[face].size() * 8);
    if (indexes) std::memcpy(indexes, m->nb_index[face].data(), m->nb_index[face].size() * 8);
    return 0;
}

int cfd_mesh_intersections(const cfd_mesh *m, uint64_t *ranges, cfd_point *points) {
    if (check_ptr(m)) return CFD_EINVAL;
    if (ranges) std::memcpy(ranges, m->x_range.data(), m->x_range.size() * 8);
    if (points) std::memcpy(points, m->x_points.data(), m->x_points.size() * sizeof(cfd_point));
    return 0;
}

// full_bounding_box (mesh.rs:294-338)
int cfd_mesh_full_bounding_box(const cfd_mesh *m, cfd_aabb *out) {
    if (check_ptr(m) || check_ptr(out)) return CFD_EINVAL;
    if (m->cx.empty()) {
        *out = cfd_aabb{{0.0, 0.0}, 0.0, 0.0};
        return 0;
    }
    double min_x = INFINITY, max_x = -INFINITY, min_y = INFINITY, max_y = -INFINITY;
    for (size_t i = 0; i < m->cx.size(); ++i) {
        const double l = m->cx[i] - m->hw[i], r = m->cx[i] + m->hw[i];
        const double b = m->cy[i] - m->hh[i], t = m->cy[i] + m->hh[i];
        // the quad's vertices folded with f64::min / max (bl, br, tr, tl)
        const double cmin_x = std::fmin(std::fmin(std::fmin(std::fmin(INFINITY, l), r), r), l);
        const double cmax_x = std::fmax(std::fmax(std::fmax(std::fmax(-INFINITY, l), r), r), l);
        const double cmin_y = std::fmin(std::fmin(std::fmin(std::fmin(INFINITY, b), b), t), t);
        const double cmax_y = std::fmax(std::fmax(std::fmax(std::fmax(-INFINITY, b), b), t), t);
        if (cmin_x < min_x) min_x = cmin_x;
        if (cmax_x > max_x) max_x = cmax_x;
        if (cmin_y < min_y) min_y = cmin_y;
        if (cmax_y > max_y) max_y = cmax_y;
    }
    out->center = {0.5 * (min_x + max_x), 0.5 * (min_y + max_y)};
    out->half_width = 0.5 * (max_x - min_x);
    out->half_height = 0.5 * (max_y - min_y);
    return 0;
}

int cfd_mesh_build_ms(const cfd_mesh *m, double *ms) {
    if (check_ptr(m) || check_ptr(ms)) return CFD_EINVAL;
    *ms = m->build_ms;
    return 0;
}

void cfd_mesh_destroy(cfd_mesh *m) { delete m; }

}  // extern "C"
