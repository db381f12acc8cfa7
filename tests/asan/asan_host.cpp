// asan_host.cpp — the host-side C++ of the product under AddressSanitizer +
// UndefinedBehaviorSanitizer, on the CPU (no GPU needed):
//   * slab_plan.h: every plan over a sweep of grid heights, rank counts,
//     halo depths and sweep indices, with the invariants the runtime relies on
//     (contiguous cover of the rows, ghost rows inside their allocations,
//     sweep bands inside the deep-halo allocation);
//   * cfd_runtime.cpp: the Model::run worker driven from several threads at
//     once (commands, snapshots, residual drains, a rejected SetParams, a
//     failing step) over stub_model.cpp;
//   * cfd_mesh.hip's host code: polygons with holes, the segment / box
//     predicates and the quadtree tesselation of the reference's default mesh.
// Exit status 0 and no sanitizer report = pass (tests/test_asan_host.py).
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "../../include/cfd.h"
#include "../../cfd-demo_amd/csrc/slab_plan.h"

extern "C" cfd_model *stub_model_create(uint64_t nx, uint64_t ny, int fail_after);
extern "C" void stub_model_destroy(cfd_model *m);

static int g_fail = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                         \
        }                                                                     \
    } while (0)

static void test_slab_plan() {
    for (uint64_t ny = 4; ny <= 300; ny += 7) {
        for (int n = 1; n <= 8; ++n) {
            if (ny / (uint64_t)n < 4) continue;
            uint64_t next = 0;
            for (int r = 0; r < n; ++r) {
                uint64_t j0, j1;
                cfd::plan_slab(ny, n, r, &j0, &j1);
                CHECK(j0 == next && j1 > j0);
                next = j1;
                const int nyl = (int)(j1 - j0);
                for (int hg = 1; hg <= std::min(32, nyl - 2); hg += 3) {
                    int h[6];
                    cfd::plan_halo(cfd::HALO_PP, nyl, hg, r, n, h);
                    for (int side = 0; side < 2; ++side) {
                        const int rows = h[3 * side + 2];
                        if (!rows) continue;
                        CHECK(h[3 * side] >= 0 && h[3 * side] + rows <= nyl);      // sent rows owned
                        CHECK(h[3 * side + 1] >= -hg && h[3 * side + 1] + rows <= nyl + hg);
                    }
                    for (int kind : {cfd::HALO_U, cfd::HALO_V}) {
                        cfd::plan_halo(kind, nyl, 2, r, n, h);
                        for (int side = 0; side < 2; ++side)
                            if (h[3 * side + 2]) CHECK(h[3 * side + 1] >= -2 && h[3 * side + 1] + 2 <= nyl + 3);
                    }
                    const int iters = 37;
                    for (int it = 0; it < iters; ++it) {
                        int lo, hi, ex;
                        cfd::plan_sweep((int)j0, nyl, (int)ny, hg, it, iters, &lo, &hi, &ex);
                        CHECK(lo >= -hg && hi <= nyl + hg);
                    }
                    for (int tmax = 1; tmax <= 8; ++tmax) {
                        int it = 0, exch = 0;
                        while (it < iters) {
                            int T, lo, hi, ex;
                            cfd::plan_block((int)j0, nyl, (int)ny, n > 1 ? hg : 0, it, tmax, iters, &T,
                                            &lo, &hi, &ex);
                            CHECK(T >= 1 && T <= tmax && it + T <= iters);
                            CHECK(lo >= -hg && hi <= nyl + hg);
                            it += T;
                            exch += ex;
                        }
                        CHECK(n == 1 || exch >= 1);
                    }
                }
            }
            CHECK(next == ny);
        }
    }
}

static void test_runtime() {
    for (int round = 0; round < 3; ++round) {
        cfd_model *m = stub_model_create(64, 48, round == 2 ? 25 : -1);
        cfd_runner *r = nullptr;
        CHECK(cfd_run_start(m, &r) == 0 && r);
        std::atomic<bool> done{false};
        std::vector<std::thread> ts;
        ts.emplace_back([&] {   // commands
            cfd_params p;
            cfd_default_params(&p);
            for (int k = 0; k < 200 && !done; ++k) {
                cfd_run_request_snapshot(r);
                if (k % 17 == 0) cfd_run_pause(r);
                if (k % 17 == 3) cfd_run_resume(r);
                p.jacobi_iters = 10 + k % 40;
                CHECK(cfd_run_set_params(r, &p) == 0);
                std::this_thread::sleep_for(std::chrono::microseconds(300));
            }
            p.jacobi_iters = 1 << 20;   // rejected synchronously
            CHECK(cfd_run_set_params(r, &p) == CFD_EINVAL);
            cfd_run_resume(r);
        });
        ts.emplace_back([&] {   // snapshots
            std::vector<float> u(65 * 48), v(64 * 49), pp(64 * 48);
            for (int k = 0; k < 300 && !done; ++k) {
                float dt;
                int paused, avail;
                CHECK(cfd_run_last_snapshot(r, u.data(), v.data(), pp.data(), &dt, &paused, &avail) == 0);
                std::this_thread::sleep_for(std::chrono::microseconds(200));
            }
        });
        ts.emplace_back([&] {   // residual log
            cfd_residuals buf[16];
            for (int k = 0; k < 300 && !done; ++k) {
                int n = 0;
                CHECK(cfd_run_new_residuals(r, buf, 16, &n) == 0 && n >= 0 && n <= 16);
                char msg[64];
                (void)cfd_run_status(r, msg, sizeof msg);
                (void)cfd_run_steps(r);
                std::this_thread::sleep_for(std::chrono::microseconds(150));
            }
        });
        for (auto &t : ts) t.join();
        done = true;
        char msg[128];
        const int st = cfd_run_status(r, msg, sizeof msg);
        CHECK(round == 2 ? st == CFD_EHIP : st == 0);
        CHECK(cfd_run_stop(r) == 0);
        stub_model_destroy(m);
    }
}

static void test_mesher() {
    cfd_polygon *rect = nullptr, *hole = nullptr, *bad = nullptr;
    int perr = 0;
    CHECK(cfd_polygon_new_rect(0, 0, 30, 10, &rect) == 0);
    CHECK(cfd_polygon_new_regular(cfd_point{5, 5}, 1.0, 4, 6.283185307179586 / 8.0, &hole) == 0);
    CHECK(cfd_polygon_add_hole(rect, hole, &perr) == 0 && perr == 0);
    const cfd_point bow[4] = {{0, 0}, {1, 1}, {1, 0}, {0, 1}};
    const uint64_t idx[4] = {0, 1, 2, 3};
    CHECK(cfd_polygon_new(bow, 4, idx, 4, &bad, &perr) == 0 && perr == CFD_POLY_SELF_INTERSECTING && !bad);
    CHECK(cfd_polygon_new(bow, 4, idx, 2, &bad, &perr) == 0 && perr == CFD_POLY_NOT_ENOUGH_VERTICES);
    int res = -1;
    CHECK(cfd_polygon_contains_point(rect, cfd_point{5, 5}, &res) == 0 && res == 0);
    CHECK(cfd_polygon_contains_point(rect, cfd_point{15, 5}, &res) == 0 && res == 1);
    const cfd_aabb box{{5, 5}, 0.5, 0.5};
    CHECK(cfd_polygon_intersects_aabb(rect, &box, &res) == 0);
    CHECK(cfd_polygon_edges_intersect_aabb(rect, &box, &res) == 0);
    cfd_aabb bb;
    CHECK(cfd_polygon_bounding_box(rect, &bb) == 0 && bb.half_width == 15.0);
    CHECK(cfd_polygon_bounding_square(rect, &bb) == 0);
    cfd_point edges[64];
    size_t ne = 0;
    CHECK(cfd_polygon_edges(rect, edges, 32, &ne) == 0 && ne == 4);   // outer ring (polygon.rs:186-196)
    cfd_point one[2];
    CHECK(cfd_polygon_edges(rect, one, 1, &ne) == 0 && ne == 4);      // copy truncated, count whole
    cfd_point out8[8];
    int n = 0;
    CHECK(cfd_geom_intersect_quad_edge(cfd_point{0, 0}, 1, 1, cfd_point{-2, 0}, cfd_point{2, 0}, out8, &n) == 0 &&
          n >= 2);
    cfd_point ip;
    int found = 0;
    CHECK(cfd_geom_segment_intersection(cfd_point{0, 0}, cfd_point{1, 1}, cfd_point{0, 1}, cfd_point{1, 0}, &ip,
                                        &found) == 0 && found == 1);
    for (double feature : {0.5, 0.1, 0.05}) {
        cfd_quadtree *t = nullptr;
        CHECK(cfd_tesselate(rect, feature, 0.5, &t) == 0 && t);
        uint64_t nn = 0, nl = 0;
        CHECK(cfd_quadtree_size(t, &nn, &nl) == 0 && nl > 0 && nn >= nl);
        std::vector<cfd_aabb> boxes(nn);
        std::vector<int64_t> kids(4 * nn);
        CHECK(cfd_quadtree_nodes(t, boxes.data(), kids.data()) == 0);
        for (uint64_t k = 0; k < 4 * nn; ++k) CHECK(kids[k] >= -1 && kids[k] < (int64_t)nn);
        cfd_quadtree_destroy(t);
    }
    cfd_polygon_destroy(rect);
}

int main() {
    test_slab_plan();
    test_runtime();
    test_mesher();
    if (g_fail) {
        std::fprintf(stderr, "%d check(s) failed\n", g_fail);
        return 1;
    }
    std::printf("asan_host ok\n");
    return 0;
}
