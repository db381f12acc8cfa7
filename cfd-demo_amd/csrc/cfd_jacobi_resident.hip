// cfd_jacobi_resident.hip — the whole tolerance-mode Jacobi solve of a small
// grid in ONE launch (r4): jacobi_pressure (model.rs:734-824) with the
// reference's early exit (model.rs:816) decided on the device, sweep by sweep.
//
// Why.  The reference's default design point (default_grid(), 800 x 264,
// SimulationParams::default(): <= 50 sweeps, early exit 1e-4, <= 20 corrector
// passes) runs ~1,050 sweeps per step on 211 K cells.  The row-march launches
// (k_jacobi_lds, MODE 2) are latency-bound there: 8 wave columns x 33
// segments = 264 waves on 1,024 SIMDs, each marching its rows through T
// stages of IEEE divisions — 43 us per 7-sweep launch, plus a check launch and
// a launch boundary per launch (7.97 ms per step, profiles/r4/prof_r4h).
//
// What.  The grid is cut into 2D tiles (BR rows x BC columns, output cells);
// each of G <= #CUs workgroups loops over its tiles.  Per block of T sweeps a
// tile loads its cells plus a T-cell halo of p' (and rhs) into LDS, runs the T
// sweeps there on a box that shrinks by one cell per sweep (the halo cone), the
// boundary rows / columns recomputed in place by the reference's rules
// (model.rs:807-815) so no tile needs a neighbour mid-block, and stores its
// output cells; every sweep's residual max over the tile's residual cells
// (rows 1..ny-2, columns 1..simd_end-1: model.rs:755-772's SIMD chunks,
// NaN-ignoring) goes to Ctl::err[sweep] by atomic max.  Then a grid barrier;
// every workgroup reads the block's T residuals and takes the same decision:
// the first sweep below p_tol ends the solve, and unless it is the block's last
// sweep the tiles re-run the block from its source buffer (untouched: the block
// wrote the other one) with exactly that many sweeps into the same
// destination — the speculative scheme of the per-launch path, with a barrier
// instead of a launch boundary plus a check launch.  Ctl::spec_launches gets
// the blocks run, so k_finalize_solve (exact_flips = 2) flips the buffer and
// counts the sweeps exactly as after the per-launch path.
//
// Residency.  The barrier needs all G workgroups resident at once: G <= the
// CU count and the launch is taken only where the occupancy query admits two
// such workgroups per CU (two models' resident solves fit side by side);
// in-process launches of different models are ordered by the persistent-launch
// gate.  Every wait is bounded by wall time (s_memrealtime): past the deadline
// the waiter raises the abort word (Fields::persist[1]) and the zero-copy host
// word, every workgroup leaves, and the model reports CFD_ETIMEOUT (as
// k_jacobi_persist).
//
// Hand-off (MI355X_MICROARCH.md, Consumer, always): p' outputs are stored
// write-through (relaxed agent-scope atomic stores: sc1), every wave drains
// them (vmcnt(0)) before the workgroup barrier, then one lane adds to the
// barrier counter (agent scope); the waiting lane polls it (relaxed agent
// loads, s_sleep), then one agent acquire + vmcnt(0) + the workgroup barrier
// before any p' load.  The counters and an exit ticket live in
// Fields::persist's head lines (2: top / single counter, 4: exit ticket, 5-12:
// group counters, 13-20: group generations); the workgroup that draws the
// last exit ticket zeroes them, so every launch starts from 0.
#include <cstring>
#include <map>
#include <mutex>

#include "cfd_device.h"

namespace cfd {
namespace {

// sweeps per block between grid barriers: 10 since r6 (the reference
// default's 50-sweep solves as 5 blocks instead of 6 + a 2-sweep tail:
// 3.216 -> 3.050 ms per step; 9: 3.073, 13: 3.202; profiles/r6/prof_r6v,
// prof_r6w)
#ifndef CFD_RES_T
#define CFD_RES_T 10
#endif
constexpr int kResMaxT = CFD_RES_T;

// CFD_RES_STAMP (diagnostic builds only): thread 0 of workgroups 0..255
// records s_memrealtime (100 MHz) at the phase boundaries of every block --
// load start, load done, sweeps done, stores issued, stores drained, barrier
// passed, residuals read -- in g_res_stamp (vector stores), read back by
// cfd_diag_res_stamps (tools/res_stamps.py).  Off in the product build.
#ifndef CFD_RES_STAMP
#define CFD_RES_STAMP 0
#endif
constexpr int kResStampWG = 256, kResStampN = 64;
#if CFD_RES_STAMP
__device__ unsigned long long g_res_stamp[kResStampWG * kResStampN];
#endif

// WAVES: 8 (512 threads) or 16; ROWS: rows of one column a thread updates
// per step of its loop (their LDS loads in flight together).  fin: the last workgroup out runs the solve's
// finalize (k_finalize_solve's body, exact_flips = 2) instead of a launch.
template <int FAST, int WAVES, int ROWS>
__global__ __launch_bounds__(WAVES * 64) void k_jacobi_resident(
    Geom g, Fields f, int pass, int iters, int T, int BR, int BC, int tiles_x, int ntiles,
    int res_hi, uint32_t deadline, int late, int fin, int check_break) {
    constexpr int kResWaves = WAVES;
    extern __shared__ float lds_dyn[];
    __shared__ float red_s[kResWaves][kResMaxT];
    __shared__ int flag_s;   // abort (1) after the barrier; last workgroup out at the end
    __shared__ uint32_t err_s[kResMaxT];
    Ctl *const ctl = f.ctl;
    float *const p0 = f.pp[0], *const p1 = f.pp[1];
    const float *__restrict__ rhs = f.rhs;
    uint32_t *const persist = f.persist;
    uint32_t *const host_fail = f.host_nonfinite ? f.host_nonfinite + 2 : nullptr;
    if (pass_off(ctl, pass)) {
        // the pass does not run: its finalize still closes the corrector loop
        // (go[pass + 1] = 0)
        if (fin && blockIdx.x == 0) solve_finalize_body(g, f, pass, iters, check_break, 0, 2);
        return;
    }
    uint32_t *const abortw = persist + 1;
    uint32_t *const bar = persist + 2 * kPersistFlagStride;
    uint32_t *const ticket = persist + 4 * kPersistFlagStride;
    if (__hip_atomic_load(abortw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;

    const int nx = g.nx, ny = g.ny;
    const int G = (int)gridDim.x, wg = (int)blockIdx.x;
    const int wave = (int)threadIdx.x >> 6, lane = (int)threadIdx.x & 63;
    const int HW = (BR + 2 * T) * (BC + 2 * T);
    float *const LA = lds_dyn, *const LB = lds_dyn + HW, *const LR = lds_dyn + 2 * HW;
    const float dx_sq = g.dx_sq, dy_sq = g.dy_sq, denom = g.denom;
    const float r_dx_sq = g.r_dx_sq, r_dy_sq = g.r_dy_sq, r_denom = g.r_denom;
    const float omega = 0.75f;
    const float om1 = 1.0f - omega;
    const int cur0 = ctl->cur;
    [[maybe_unused]] int nstamp = 0;
    auto stamp = [&]() {
#if CFD_RES_STAMP
        if (threadIdx.x == 0 && wg < kResStampWG && nstamp < kResStampN)
            g_res_stamp[wg * kResStampN + nstamp] = __builtin_amdgcn_s_memrealtime();
        ++nstamp;
#endif
    };
    stamp();

    // The tile's LDS region is its output cells plus a T-cell halo (clamped
    // to the grid), the same for every block, so with one tile per workgroup
    // the rhs region is loaded once per solve (rhs is constant in a solve).
    const bool keep_rhs = ntiles <= G;
    bool rhs_in = false;
    constexpr int NT = kResWaves * 64;
    // Tb sweeps of every tile of this workgroup from `src` into `dst`;
    // publish: fold each sweep's residual into red_s[wave][s]
    auto run_tiles = [&](const float *__restrict__ src, float *__restrict__ dst, int Tb,
                         bool publish) {
        for (int t = wg; t < ntiles; t += G) {
            const int ty = t / tiles_x, tx = t - ty * tiles_x;
            const int r0 = ty * BR, r1 = min(ny, r0 + BR);
            const int c0 = tx * BC, c1 = min(nx, c0 + BC);
            const int R0 = max(0, r0 - T), R1 = min(ny, r1 + T);
            const int C0 = max(0, c0 - T), C1 = min(nx, c1 + T);
            const int W = C1 - C0, H = R1 - R0;
            const bool ld_rhs = !(keep_rhs && rhs_in);
            rhs_in = true;
            __syncthreads();   // the previous tile's LDS reads are done
            stamp();
            {
                // flat over the region, 4 loads in flight per thread before
                // their LDS stores; row = idx / W by a float reciprocal (exact
                // for these sizes: idx < 2^13)
                const float rW = 1.0f / (float)W;
                const int n = H * W;
                for (int i0 = (int)threadIdx.x; i0 < n; i0 += 4 * NT) {
                    float pv[4], rv[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int i = i0 + u * NT;
                        const int rr = (int)(((float)i + 0.5f) * rW);
                        const size_t gi = (size_t)(R0 + rr) * nx + (C0 + i - rr * W);
                        pv[u] = i < n ? src[gi] : 0.0f;
                        rv[u] = (i < n && ld_rhs) ? rhs[gi] : 0.0f;
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int i = i0 + u * NT;
                        if (i < n) {
                            LA[i] = pv[u];
                            if (ld_rhs) LR[i] = rv[u];
                        }
                    }
                }
            }
            __syncthreads();
            stamp();
            float *A = LA, *B = LB;
            const bool edge = r0 - T <= 0 || r1 + T >= ny || c0 - T <= 0 || c1 + T >= nx;
            for (int s = 0; s < Tb; ++s) {
                const int e = Tb - 1 - s;   // the box this sweep must cover: outputs + e
                const int br0 = max(0, r0 - e), br1 = min(ny, r1 + e);
                const int bc0 = max(0, c0 - e), bc1 = min(nx, c1 + e);
                // interior cells (model.rs:775-793, operation for operation),
                // ROWS consecutive rows of one column per thread: their loads
                // issue together (rows past the region clamp to its last row;
                // those values feed no stored cell)
                const int ir0 = max(br0, 1), ir1 = min(br1, ny - 1);
                const int ic0 = max(bc0, 1), ic1 = min(bc1, nx - 1);
                float ms = 0.0f;
                const int nrg = (ir1 - ir0 + ROWS - 1) / ROWS;
                for (int q = wave; q < nrg; q += kResWaves) {
                    const int rb = ir0 + q * ROWS;
                    for (int c = ic0 + lane; c < ic1; c += 64) {
                        const int cc = c - C0;
                        float col[ROWS + 2], lf[ROWS], rt[ROWS], rh[ROWS];
#pragma unroll
                        for (int k = 0; k < ROWS + 2; ++k)
                            col[k] = A[(min(rb - 1 + k, R1 - 1) - R0) * W + cc];
#pragma unroll
                        for (int k = 0; k < ROWS; ++k) {
                            const int i = (min(rb + k, R1 - 1) - R0) * W + cc;
                            lf[k] = A[i - 1];
                            rt[k] = A[i + 1];
                            rh[k] = LR[i];
                        }
#pragma unroll
                        for (int k = 0; k < ROWS; ++k) {
                            const int r = rb + k;
                            if (r < ir1) {
                                const float center = col[k + 1];
                                const float horizontal = fdiv<FAST>(rt[k] + lf[k], dx_sq, r_dx_sq);
                                const float vertical = fdiv<FAST>(col[k + 2] + col[k], dy_sq, r_dy_sq);
                                const float p_update =
                                    fdiv<FAST>(horizontal + vertical - rh[k], denom, r_denom);
                                const float nv = omega * p_update + om1 * center;
                                B[(r - R0) * W + cc] = nv;
                                if (publish && r >= r0 && r < r1 && c >= c0 && c < c1 && c < res_hi) {
                                    const float d = fabsf(nv - center);
                                    ms = d > ms ? d : ms;   // NaN-ignoring, like reduce_max
                                }
                            }
                        }
                    }
                }
                if (edge) {
                    // p' boundary conditions (model.rs:807-815) on the box's
                    // boundary cells, from this sweep's interior values: row
                    // copies, then column 0 = column 1, column nx-1 = 0
                    __syncthreads();
                    auto at = [&](int r, int c) { return B[(r - R0) * W + (c - C0)]; };
                    auto bc_value = [&](int r, int c) -> float {
                        if (c == nx - 1) return 0.0f;
                        if (c == 0) return at(r == 0 ? 1 : (r == ny - 1 ? ny - 2 : r), 1);
                        return at(r == 0 ? 1 : ny - 2, c);
                    };
                    if (wave < 2) {   // rows 0 and ny-1, whole box width
                        const int r = wave == 0 ? 0 : ny - 1;
                        if (r >= br0 && r < br1)
                            for (int c = bc0 + lane; c < bc1; c += 64)
                                B[(r - R0) * W + (c - C0)] = bc_value(r, c);
                    } else if (wave < 4) {   // columns 0 and nx-1, interior rows
                        const int c = wave == 2 ? 0 : nx - 1;
                        if (c >= bc0 && c < bc1)
                            for (int r = ir0 + lane; r < ir1; r += 64)
                                B[(r - R0) * W + (c - C0)] = bc_value(r, c);
                    }
                }
                if (publish) {
                    const float wm = wave_max(ms);
                    if (lane == 0) red_s[wave][s] = fmaxf(red_s[wave][s], wm);
                }
                __syncthreads();
                float *tmp = A;
                A = B;
                B = tmp;
            }
            stamp();
            // the tile's outputs, written through (sc1) for the other workgroups
            for (int r = r0 + wave; r < r1; r += kResWaves)
                for (int c = c0 + lane; c < c1; c += 64)
                    __hip_atomic_store(reinterpret_cast<uint32_t *>(dst + (size_t)r * nx + c),
                                       __float_as_uint(A[(r - R0) * W + (c - C0)]), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
        }
    };

    int it = 0, k = 0, blocks = 0;
    bool aborted = false;
    for (;;) {
        const int Tb = min(T, iters - it);
        const bool last = it + Tb >= iters;
        const float *src = ((cur0 + k) & 1) ? p1 : p0;
        float *dst = ((cur0 + k) & 1) ? p0 : p1;
        // every sweep's residual with the tolerance on; a fixed-count solve
        // needs only its last sweep's (k_finalize_solve folds err[iters-1])
        const bool publish = g.tol_enabled || last;
        if (threadIdx.x < kResWaves * kResMaxT) red_s[threadIdx.x / kResMaxT][threadIdx.x % kResMaxT] = 0.0f;
        __syncthreads();
        run_tiles(src, dst, Tb, publish);
        stamp();
        __syncthreads();
        if (publish && (int)threadIdx.x < Tb && (g.tol_enabled || (int)threadIdx.x == Tb - 1)) {
            float m = 0.0f;
#pragma unroll
            for (int w = 0; w < kResWaves; ++w) m = fmaxf(m, red_s[w][threadIdx.x]);
            if (m > 0.0f)
                __hip_atomic_fetch_max(&ctl->err[it + (int)threadIdx.x], __float_as_uint(m),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        blocks = k + 1;
        if (!g.tol_enabled && last) break;   // fixed count: the kernel boundary publishes
        if (late > 0 && k == 0 && wg % late == 1 && threadIdx.x == 0) {
            // test knob (CFD_PERSIST_LATE=k): these workgroups arrive 2 ms late
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (__builtin_amdgcn_s_memrealtime() - t0 < 200000u) __builtin_amdgcn_s_sleep(127);
        }
        // ---- grid barrier: outputs and residual atomics drained, one arrival ----
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        stamp();
        if (threadIdx.x == 0) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            int fail = 0;
            // wait until *w >= want (relaxed agent polls, bounded)
            auto wait_ge = [&](uint32_t *w, uint32_t want) {
                for (;;) {
                    if (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want) return;
                    if (__hip_atomic_load(abortw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u ||
                        __builtin_amdgcn_s_memrealtime() - t0 > (uint64_t)deadline) {
                        fail = 1;
                        return;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            };
            {
                // two levels (MI355X_MICROARCH.md barrier-xcd; one counter with
                // G pollers measured 3.99 vs 3.59 ms per step, r4): workgroup w
                // arrives on group counter w % 8 (round-robin dispatch puts a
                // group on one XCD: speed only, never correctness); the
                // group's last arriver (told by its returning add) arrives on
                // the top counter, waits for all groups and raises the group's
                // generation word, which the group's other workgroups poll
                const int grp = wg & 7, ngrp = G < 8 ? G : 8;
                const uint32_t gsize = (uint32_t)(G / 8 + (grp < G % 8 ? 1 : 0));
                uint32_t *gc = persist + (5 + grp) * kPersistFlagStride;
                uint32_t *gg = persist + (13 + grp) * kPersistFlagStride;
                const uint32_t v = __hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (v + 1u == gsize * (uint32_t)(k + 1)) {
                    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    wait_ge(bar, (uint32_t)ngrp * (uint32_t)(k + 1));
                    __hip_atomic_store(gg, (uint32_t)(k + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } else {
                    wait_ge(gg, (uint32_t)(k + 1));
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (fail) {
                __hip_atomic_store(abortw, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (host_fail)   // zero-copy host word: cfd_* calls report CFD_ETIMEOUT
                    __hip_atomic_store(host_fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            flag_s = fail;
        }
        __syncthreads();
        stamp();
        if (flag_s) {
            aborted = true;
            break;
        }
        // the block's residuals, final once every arrival is in (agent-scope
        // loads: performed where the atomics were)
        if (g.tol_enabled && (int)threadIdx.x < Tb)
            err_s[threadIdx.x] = __hip_atomic_load(&ctl->err[it + (int)threadIdx.x], __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        stamp();
        // the first sweep of the block below p_tol ends the solve (model.rs:816)
        int j = Tb;
        if (g.tol_enabled) {
            j = 0;
            while (j < Tb && !(__uint_as_float(err_s[j]) < g.p_tol)) ++j;
        }
        if (j < Tb) {
            if (j + 1 < Tb) run_tiles(src, dst, j + 1, false);   // exactly j + 1 sweeps
            break;
        }
        if (last) break;
        it += Tb;
        ++k;
    }
    if (aborted) return;
    if (!fin && wg == 0 && threadIdx.x == 0) ctl->spec_launches = blocks;   // k_finalize_solve's flips
    // the last workgroup out: every arrival is in; zero the counters for the
    // next launch and (fin) finalize the solve
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const bool lastwg =
            __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)G - 1u;
        if (lastwg) {
            __hip_atomic_store(bar, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (int q = 0; q < 8; ++q) {
                __hip_atomic_store(persist + (5 + q) * kPersistFlagStride, 0u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(persist + (13 + q) * kPersistFlagStride, 0u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
            __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (fin) {
                ctl->spec_launches = blocks;   // every workgroup ran the same blocks
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // every err[] atomic is in
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        }
        flag_s = lastwg;
    }
    __syncthreads();
    if (fin && flag_s) solve_finalize_body(g, f, pass, iters, check_break, 0, 2);
}

struct ResidentPlan {
    int BR, BC, tiles_x, ntiles, G, lds;
};

inline int resident_lds_bytes(int BR, int BC, int T) { return 3 * (BR + 2 * T) * (BC + 2 * T) * 4; }

// The launched instantiation: 8 waves (512 threads; the occupancy query admits
// two per CU, the residency rule above) and one row per thread step (r6: the
// reference default 3.60 -> 3.23 ms per step at 18 x 48 tiles against 3.33
// with 2 rows; 16-wave workgroups -1.5 %, not taken: profiles/r6/prof_r6j,
// prof_r6m).
// build-time (r6 A/B at T = 10, profiles/r6/prof_r6aj: 8 waves 1 row 3.031,
// 2 rows 3.081 ms; 16 waves do not fit two workgroups per CU with this LDS
// and fall back to the per-launch path, 7.32 ms)
#ifndef CFD_RES_WAVES
#define CFD_RES_WAVES 8
#endif
#ifndef CFD_RES_ROWS
#define CFD_RES_ROWS 1
#endif
constexpr int kResLaunchWaves = CFD_RES_WAVES, kResLaunchRows = CFD_RES_ROWS;

// Workgroups of the launched instantiation per CU with `lds` bytes of dynamic
// LDS; cached per lds -- the plan is consulted on every tolerance-mode solve
template <int FAST>
int resident_blocks_per_cu(int lds) {
    static std::mutex mu;
    static std::map<int, int> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(lds);
    if (it != cache.end()) return it->second;
    const void *k =
        reinterpret_cast<const void *>(&k_jacobi_resident<FAST, kResLaunchWaves, kResLaunchRows>);
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, kResLaunchWaves * 64, lds) != hipSuccess)
        n = 0;
    cache[lds] = n;
    return n;
}

// Tile shape: the candidate with the least sweep work per workgroup
// (ceil(tiles / G) x the lane slots of its T boxes), every candidate admitting 2 workgroups per CU
// (one per CU in the grid, a margin of one).  Single domain only (rows
// 0..ny-1 owned; the fields' ghost rows unused).  The occupancy queries are
// cached; the rest is a few integer operations.
bool resident_plan(const Geom &g, int T, ResidentPlan *p) {
    if (g.nx < 4 || g.ny < 4 || g.j0 != 0 || g.nyl != g.ny) return false;
    // box widths BC + 2e (e = 0..T-1) fill 64-lane passes: BC = 48 -> 48..62
    // columns in one pass, 112 -> 112..126 in two.  r6: rows 18-24 too -- the
    // reference default (800 x 264) took 32 x 48 (153 tiles, box 48 x 64);
    // 18 x 48 (255 tiles, box 34 x 64) runs the step 3.60 -> 3.23 ms
    // (profiles/r6/prof_r6i, prof_r6j)
    // r6, T = 10: BC = 46 keeps every sweep's box (BC + 2e, e < T) in one
    // 64-lane pass (48 needs two for e = 9)
    static const int cand[][2] = {{8, 48},  {16, 48}, {18, 48}, {20, 48}, {24, 48},
                                  {32, 48}, {19, 46}, {20, 46}, {22, 46}, {24, 46},
                                  {16, 112}, {32, 112}};
    long best = -1;
    for (const auto &cd : cand) {
        const int BR = cd[0], BC = cd[1];
        const int lds = resident_lds_bytes(BR, BC, T);
        const int occ = g.res_div == 1   ? resident_blocks_per_cu<1>(lds)
                        : g.res_div == 2 ? resident_blocks_per_cu<2>(lds)
                        : g.res_div == 3 ? resident_blocks_per_cu<3>(lds)
                                         : resident_blocks_per_cu<0>(lds);
        if (occ < 2) continue;
        const int tx = cdiv(g.nx, BC), ty = cdiv(g.ny, BR);
        const long nt = (long)tx * ty;
        const int G = (int)std::min<long>(nt, (long)g.n_cu);
        // lane slots a workgroup's sweeps occupy: rows x 64-lane passes of
        // each sweep's box
        long slots = 0;
        for (int e = 0; e < T; ++e) slots += (long)(BR + 2 * e) * 64 * cdiv(BC + 2 * e, 64);
        const long work = (long)cdiv(nt, G) * slots;
        if (best < 0 || work < best) {
            best = work;
            *p = ResidentPlan{BR, BC, tx, (int)nt, G, lds};
        }
    }
    return best >= 0;
}

}  // namespace

// residual columns [1, simd_end): model.rs:755-772's 8-lane chunks
static int resident_simd_end(int nx) {
    int e = 1;
    while (e + 8 <= nx - 1) e += 8;
    return e;
}

bool launch_jacobi_resident(const Geom &g, const Fields &f, int pass, int iters, int fin,
                            int check_break, hipStream_t s) {
    if (iters <= 0) return false;
    constexpr int T = kResMaxT;   // sweeps per block between grid barriers
    ResidentPlan p;
    if (!resident_plan(g, T, &p)) return false;
    const char *de = getenv("CFD_PERSIST_DEADLINE_US");
    const double dl_us = de ? std::max(0.0, atof(de)) : 10e6;
    const uint32_t deadline = (uint32_t)std::min(4.0e9, dl_us * 100.0);
    const char *le = getenv("CFD_PERSIST_LATE");
    const int late = le ? std::max(0, atoi(le)) : 0;
#define CFD_RES_LAUNCH(FASTV)                                                                       \
    hipLaunchKernelGGL((k_jacobi_resident<FASTV, kResLaunchWaves, kResLaunchRows>), dim3(p.G),      \
                       dim3(kResLaunchWaves * 64), p.lds, s, g, f, pass, iters, T, p.BR, p.BC,     \
                       p.tiles_x, p.ntiles, resident_simd_end(g.nx), deadline, late, fin, check_break)
    if (g.res_div == 1)
        CFD_RES_LAUNCH(1);
    else if (g.res_div == 2)
        CFD_RES_LAUNCH(2);
    else if (g.res_div == 3)
        CFD_RES_LAUNCH(3);
    else
        CFD_RES_LAUNCH(0);
#undef CFD_RES_LAUNCH
    return true;
}

#if CFD_RES_STAMP
extern "C" int cfd_diag_res_stamps(unsigned long long *host, int n) {
    if (n > kResStampWG * kResStampN) n = kResStampWG * kResStampN;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_res_stamp), (size_t)n * 8, 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? n : -1;
}
#endif

bool jacobi_resident_geometry(const Geom &g, int *br, int *bc, int *tiles, int *wgs) {
    // (the tile plan the launch would take; false: none fits)
    ResidentPlan p;
    if (!resident_plan(g, kResMaxT, &p)) return false;
    *br = p.BR;
    *bc = p.BC;
    *tiles = p.ntiles;
    *wgs = p.G;
    return true;
}

}  // namespace cfd
