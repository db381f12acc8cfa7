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
// before any p' load.  The counter and an exit ticket live in Fields::persist's
// head lines 2 and 4; the workgroup that draws the last exit ticket zeroes
// both, so every launch starts from 0.
#include "cfd_device.h"

namespace cfd {
namespace {

constexpr int kResWaves = 8;   // 512-thread workgroups: 2 waves per SIMD at 1 workgroup per CU
constexpr int kResMaxT = 8;

template <int FAST>
__global__ __launch_bounds__(kResWaves * 64) void k_jacobi_resident(
    Geom g, float *__restrict__ p0, float *__restrict__ p1, const float *__restrict__ rhs, Ctl *ctl,
    uint32_t *persist, uint32_t *host_fail, int pass, int iters, int T, int BR, int BC, int tiles_x,
    int ntiles, int res_hi, uint32_t deadline, int late) {
    extern __shared__ float lds_dyn[];
    __shared__ float red_s[kResWaves][kResMaxT];
    __shared__ int flag_s;   // abort (1) after the barrier
    __shared__ uint32_t err_s[kResMaxT];
    if (pass_off(ctl, pass)) return;
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

    // Tb sweeps of every tile of this workgroup from `src` into `dst`;
    // publish: fold each sweep's residual into red_s[wave][s]
    auto run_tiles = [&](const float *__restrict__ src, float *__restrict__ dst, int Tb,
                         bool publish) {
        for (int t = wg; t < ntiles; t += G) {
            const int ty = t / tiles_x, tx = t - ty * tiles_x;
            const int r0 = ty * BR, r1 = min(ny, r0 + BR);
            const int c0 = tx * BC, c1 = min(nx, c0 + BC);
            const int R0 = max(0, r0 - Tb), R1 = min(ny, r1 + Tb);
            const int C0 = max(0, c0 - Tb), C1 = min(nx, c1 + Tb);
            const int W = C1 - C0;
            __syncthreads();   // the previous tile's LDS reads are done
            for (int r = R0 + wave; r < R1; r += kResWaves)
                for (int c = C0 + lane; c < C1; c += 64) {
                    const int i = (r - R0) * W + (c - C0);
                    LA[i] = src[(size_t)r * nx + c];
                    LR[i] = rhs[(size_t)r * nx + c];
                }
            __syncthreads();
            float *A = LA, *B = LB;
            const bool edge = r0 - Tb <= 0 || r1 + Tb >= ny || c0 - Tb <= 0 || c1 + Tb >= nx;
            for (int s = 0; s < Tb; ++s) {
                const int e = Tb - 1 - s;   // the box this sweep must cover: outputs + e
                const int br0 = max(0, r0 - e), br1 = min(ny, r1 + e);
                const int bc0 = max(0, c0 - e), bc1 = min(nx, c1 + e);
                // interior cells (model.rs:775-793, operation for operation)
                const int ir0 = max(br0, 1), ir1 = min(br1, ny - 1);
                const int ic0 = max(bc0, 1), ic1 = min(bc1, nx - 1);
                float ms = 0.0f;
                for (int r = ir0 + wave; r < ir1; r += kResWaves) {
                    const bool own_r = publish && r >= r0 && r < r1;
                    for (int c = ic0 + lane; c < ic1; c += 64) {
                        const int i = (r - R0) * W + (c - C0);
                        const float center = A[i];
                        const float horizontal = fdiv<FAST>(A[i + 1] + A[i - 1], dx_sq, r_dx_sq);
                        const float vertical = fdiv<FAST>(A[i + W] + A[i - W], dy_sq, r_dy_sq);
                        const float p_update =
                            fdiv<FAST>(horizontal + vertical - LR[i], denom, r_denom);
                        const float nv = omega * p_update + om1 * center;
                        B[i] = nv;
                        if (own_r && c >= c0 && c < c1 && c < res_hi) {
                            const float d = fabsf(nv - center);
                            ms = d > ms ? d : ms;   // NaN-ignoring, like reduce_max
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
        if (threadIdx.x == 0) {
            __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t want = (uint32_t)G * (uint32_t)(k + 1);
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            int fail = 0;
            for (;;) {
                if (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want) break;
                if (__hip_atomic_load(abortw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u ||
                    __builtin_amdgcn_s_memrealtime() - t0 > (uint64_t)deadline) {
                    fail = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
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
    if (threadIdx.x == 0) {
        if (wg == 0 && !aborted) ctl->spec_launches = blocks;   // k_finalize_solve's buffer flips
        if (!aborted &&
            __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                (uint32_t)G - 1u) {
            // the last workgroup out: every arrival is in, zero for the next launch
            __hip_atomic_store(bar, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

struct ResidentPlan {
    int BR, BC, tiles_x, ntiles, G, lds;
};

inline int resident_lds_bytes(int BR, int BC, int T) { return 3 * (BR + 2 * T) * (BC + 2 * T) * 4; }

template <int FAST>
int resident_blocks_per_cu(int lds) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &n, reinterpret_cast<const void *>(&k_jacobi_resident<FAST>), kResWaves * 64, lds) !=
        hipSuccess)
        return 0;
    return n;
}

// Tile shape: the candidate with the least LDS-box work per workgroup
// (ceil(tiles / G) x box cells), every candidate admitting 2 workgroups per CU.
bool resident_plan(const Geom &g, int T, ResidentPlan *p) {
    static const int cand[][2] = {{8, 64}, {16, 64}, {16, 128}, {32, 96}};
    long best = -1;
    for (const auto &cd : cand) {
        const int BR = cd[0], BC = cd[1];
        const int lds = resident_lds_bytes(BR, BC, T);
        const int occ = g.fastdiv == 1   ? resident_blocks_per_cu<1>(lds)
                        : g.fastdiv == 2 ? resident_blocks_per_cu<2>(lds)
                                         : resident_blocks_per_cu<0>(lds);
        if (occ < 2) continue;
        const int tx = cdiv(g.nx, BC), ty = cdiv(g.ny, BR);
        const long nt = (long)tx * ty;
        const int G = (int)std::min<long>(nt, g.n_cu);
        const long work = (long)cdiv(nt, G) * (BR + 2 * T) * (BC + 2 * T);
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

bool launch_jacobi_resident(const Geom &g, const Fields &f, int pass, int iters, hipStream_t s) {
    if (iters <= 0 || g.nx < 4 || g.ny < 4 || g.hg != 0 || g.j0 != 0 || g.nyl != g.ny) return false;
    const int T = kResMaxT;
    ResidentPlan p;
    if (!resident_plan(g, T, &p)) return false;
    const char *de = getenv("CFD_PERSIST_DEADLINE_US");
    const double dl_us = de ? std::max(0.0, atof(de)) : 10e6;
    const uint32_t deadline = (uint32_t)std::min(4.0e9, dl_us * 100.0);
    uint32_t *hf = f.host_nonfinite ? f.host_nonfinite + 2 : nullptr;
    const char *le = getenv("CFD_PERSIST_LATE");
    const int late = le ? std::max(0, atoi(le)) : 0;
#define CFD_RES_LAUNCH(FASTV)                                                                      \
    hipLaunchKernelGGL((k_jacobi_resident<FASTV>), dim3(p.G), dim3(kResWaves * 64), p.lds, s, g,   \
                       f.pp[0], f.pp[1], f.rhs, f.ctl, f.persist, hf, pass, iters, T, p.BR, p.BC,     \
                       p.tiles_x, p.ntiles, resident_simd_end(g.nx), deadline, late)
    if (g.fastdiv == 1)
        CFD_RES_LAUNCH(1);
    else if (g.fastdiv == 2)
        CFD_RES_LAUNCH(2);
    else
        CFD_RES_LAUNCH(0);
#undef CFD_RES_LAUNCH
    return true;
}

bool jacobi_resident_geometry(const Geom &g, int *br, int *bc, int *tiles, int *wgs) {
    ResidentPlan p;
    if (!resident_plan(g, kResMaxT, &p)) return false;
    *br = p.BR;
    *bc = p.BC;
    *tiles = p.ntiles;
    *wgs = p.G;
    return true;
}

}  // namespace cfd
