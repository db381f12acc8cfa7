// cfd_jacobi_lds.h — kind 5: the temporally blocked Jacobi march
// (model.rs:748-815, T sweeps per launch) with its rhs window in LDS.
// Included by three translation units that instantiate it for disjoint sets
// of T (cfd_jacobi_lds.hip: T <= 4 and the dispatch, cfd_jacobi_lds567.hip,
// cfd_jacobi_lds8.hip), so the kind's compile runs in parallel.
//
// Same schedule as the prefetch-pipelined march (cfd_jacobi_pipe.h): a wave
// owns 64 lanes x 2 columns of a row segment and marches along it; stage s
// (1..T) of slot v computes row k-s (k = k_first + v) from stage s-1's rows
// k-s-1..k-s+1, so every stage is one sweep of the reference, bit for bit.
// What changes is where each value lives between its load and its last use:
//   PQ[v % PD]  p' input row k+PD, loaded PD slots ahead       (registers)
//   RQ[v % PD]  rhs row k+PD, loaded PD slots ahead            (registers)
//   ring[v % D] rhs row k, written at slot v, read by stage s  (LDS, D >= T+1)
//               at slot v+s
//   W[s][v % 3] the newest row of stage s                      (registers)
// The march kind 4 keeps all T+PD rhs rows a slot needs in registers: ~130
// VGPRs at T = 8, 3 waves per SIMD.  Here the rhs window costs one
// ds_write_b64 and T ds_read_b64 per slot instead, and the kernel fits 8 waves
// per SIMD (~60 VGPRs, 4.5 KB of LDS per wave at T = 8).  The slot loop is
// unrolled by U = D (a multiple of 3 and of PD), so every ring index — W, PQ,
// RQ and the LDS slot, an immediate offset — is a compile-time constant.
//
// The horizontal neighbour sums are written as two scalar adds whose second
// operand is a DPP lane shift (wave_shr:1 / wave_shl:1): the backend folds
// each shift into its add (v_add_f32_dpp), one VALU instruction per sum.  This
// translation unit is built with -fno-slp-vectorize so the two adds are not
// packed back into a v_pk_add_f32 (VOP3P cannot take DPP); the rest of the
// update is explicit packed f32 arithmetic on column pairs.
#pragma once
#include <cmath>
#include <type_traits>

#include "cfd_device.h"

namespace cfd {
namespace {

constexpr int kLdsWaves = 4;   // waves per workgroup (256 threads)
#ifndef CFD_LDS_SB
#define CFD_LDS_SB 0   // scheduling barriers: 1 between slots, 2 also between stages
#endif                 // (bound live ranges; measured no faster, r2 ab_lds_R*.log)
#ifndef CFD_LDS_PD
#define CFD_LDS_PD 3   // prefetch distance (slots) of the p' and rhs rows
#endif
// CFD_LDS_DIAG (timing diagnostics only, WRONG results), bits: 1 = no global
// loads (rows are a lane constant), 2 = no LDS ring (stage s reads the
// register prefetch of another row), 4 = no p' stores.  At 4096^2 (r6,
// profiles/r6/prof_r6q/abvar_diag.log): 5.03 us per sweep; without stores
// 4.46, without loads 4.15, without both 4.06.  gfx950 counts a wave's loads
// and stores in ONE vmcnt, in issue order, so each wait for a prefetched row
// also waits for the p' stores issued before it: the stores cost through that
// coupling.  A fifth "store wave" per workgroup draining LDS rings of the
// output rows measured slower (5.79; 5.22 even with its stores and ring waits
// compiled out -- the 96-VGPR cap that 5 waves per SIMD need, and the fifth
// wave shares wave 0's SIMD: profiles/r6/prof_r6t, prof_r6s/wave_place.log).
#ifndef CFD_LDS_DIAG
#define CFD_LDS_DIAG 0
#endif
#ifndef CFD_LDS_WPE
#define CFD_LDS_WPE 0  // > 0: minimum waves per SIMD for the register allocation
#endif
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
// CFD_LDS_STAMP (diagnostic builds only): every wave of a RES=false launch
// records its start and end (s_memrealtime, 100 MHz), its shader-clock span
// (s_memtime) and its HW_ID / XCC_ID in g_lds_stamp (vector stores), read back
// by cfd_diag_lds_stamps.  Off in the product build.
#ifndef CFD_LDS_PRIO
#define CFD_LDS_PRIO 1  // progress-ordered issue priority (LdsMarch::set_prio)
#endif
#ifndef CFD_LDS_COMPACT
#define CFD_LDS_COMPACT 0  // 1: warm-up and tail share one run-time-guarded slot group
#endif
#ifndef CFD_LDS_STAMP
#define CFD_LDS_STAMP 0
#endif
#if CFD_LDS_STAMP
constexpr int kStampWaves = 1 << 15;
__device__ unsigned long long g_lds_stamp[kStampWaves * 4];
#endif

#ifndef CFD_LDS_ST_AUX
#define CFD_LDS_ST_AUX 16  // p' stores write-through (sc1): 5.07 vs 5.13 us/sweep plain, nt 5.78 (r3 ab_staux.log)
#endif

#ifndef CFD_LDS_LD_AUX
#define CFD_LDS_LD_AUX 0  // cache-policy bits of the p' loads (16 = sc1: bypass L1)
#endif

#ifndef CFD_LDS_HOIST
#define CFD_LDS_HOIST 0  // 1: read a slot's T rhs rows from the LDS ring at its start (r2: 5.09 vs 5.00 us/sweep, off)
#endif

#ifndef CFD_LDS_SPLIT
#define CFD_LDS_SPLIT 1  // independent stage groups per slot (see LdsMarch)
#endif
constexpr int lds_gcd(int a, int b) { return b == 0 ? a : lds_gcd(b, a % b); }
// Slots of lag accumulated before stage s when the T stages form G groups,
// each group one slot behind the one before it.
constexpr int lds_off(int s, int T, int G) { return s <= 0 ? 0 : ((s - 1) * G) / T; }
// register window rows per stage: 3, or 4 when a stage reads its
// predecessor's rows one slot late
constexpr int lds_nw(int G) { return G > 1 ? 4 : 3; }
// rhs ring depth: the smallest multiple of lcm(NW, PD) holding the T + off(T)
// + 1 rows between the newest load and the last stage's read
constexpr int ring_depth(int T, int PD, int G) {
    const int nw = lds_nw(G);
    const int q = nw / lds_gcd(nw, PD) * PD;
    const int need = T + lds_off(T, T, G) + 1;
    return ((need + q - 1) / q) * q;
}

// MODE: 0 plain launch; 1 (RES) the solve's last launch, publishes the last
// stage's residual; 2 (SPEC) the speculative tolerance-mode launch: every
// stage's residual goes to its own sweep's slot set, and the launch is skipped
// once an earlier launch of the solve converged (Ctl::spec_stop); 3 (REDO)
// re-runs the converged launch from its untouched source buffer with the
// run-time stage count Ctl::spec_redo < T (stores only the segment's rows).
// SUMS (persistent launches only, FAST == 1 with dx^2 == dy^2 a power of two,
// r4): the update forms (h + v) * (1/dx^2) instead of h * (1/dx^2) +
// v * (1/dy^2) -- one packed multiply per column pair and stage fewer (10
// VALU instructions instead of 11).  Bitwise the same whenever |h|, |v| <
// 2^104: both products are then exact scalings by a power of two, and
// RN(R h + R v) = R RN(h + v) for R = 2^k (scaling commutes with rounding,
// overflow included; a subnormal h + v is exact).  k_jacobi_persist proves
// that bound per task before it picks SUMS (its guard); otherwise, and for
// every other launch, the reference's form runs.
// (r5's optimistic per-wave SUMS form for per-launch solves and r4's
// whole-solve guard lost their A/B against the reference's form and were
// removed in r6: every per-launch march runs the reference's form.)
template <int T, int FAST, int MODE, bool SUMS = false>
struct LdsMarch {
    static constexpr bool RES = MODE == 1 || MODE == 5, SPEC = MODE == 2, REDO = MODE == 3;
    // MODE 4 (PERSIST): a block of k_jacobi_persist; p' moves between
    // workgroups inside the launch, so its loads bypass L1 and its stores
    // write through (sc1 both ways, MI355X_MICROARCH.md visibility rules).
    // MODE 5: its last block, which also publishes the residual (RES)
    static constexpr bool PERSIST = MODE == 4 || MODE == 5;
    // persistent blocks in the reference's form track what the SUMS guard
    // needs: max |p'| of the rows the wave loads (imax) and of the rhs rows it
    // uses (rmax); every persistent block tracks max |p'| of the rows it
    // stores (omax), which are its neighbours' inputs in the next block
#ifndef CFD_PROBE_NOTRACK
#define CFD_PROBE_NOTRACK 0   // (diagnostic builds: no guard tracking)
#endif
    static constexpr bool TRACK_IN = PERSIST && !SUMS && !CFD_PROBE_NOTRACK;
    static constexpr bool TRACK_OUT = PERSIST && !CFD_PROBE_NOTRACK;
    static_assert(!SUMS || FAST == 1, "SUMS: reciprocal multiply");
    static constexpr int PLD_AUX = PERSIST ? 16 : CFD_LDS_LD_AUX;
    static constexpr int PST_AUX = PERSIST ? 16 : CFD_LDS_ST_AUX;
    // Stage s of slot v computes row k - s - off(s).  With G = 1 (off = 0)
    // this is the plain pipeline: stage s reads stage s-1's row of the SAME
    // slot, one serial chain of T dependent updates per slot.  With G > 1 the
    // stages form G groups and each group runs one slot behind the previous
    // one: a group's first stage reads rows its predecessor finished in an
    // EARLIER slot, so a slot holds G independent chains of T/G updates (ILP
    // that hides the packed-f32 result latency), for one more window row per
    // stage (NW = 4) and off(T) more warm-up and ring rows.  The set of
    // (stage, row) updates is the same, and so is every value.
    static constexpr int G = CFD_LDS_SPLIT;
    static constexpr int NW = lds_nw(G);            // register window rows per stage
    static constexpr int PD = CFD_LDS_PD;           // prefetch distance (slots) of p' and rhs
    static constexpr int OFFT = lds_off(T, T, G);
    static constexpr int D = ring_depth(T, PD, G);  // rhs ring depth; PD and NW divide it
    static constexpr int U = D;                     // slot unroll: every ring index compile-time
    static constexpr int WARM = 2 * T + OFFT;       // stage s starts at slot 2s + off(s)
    static constexpr int H = (T + 1) / 2;           // halo lanes per side (2 columns per lane)
    static constexpr int OUTL = 64 - 2 * H;         // lanes whose columns are stored
    static constexpr int off(int s) { return lds_off(s, T, G); }
    static constexpr int start(int s) { return 2 * s + off(s); }
    static_assert(D % PD == 0 && D % NW == 0 && D >= T + OFFT + 1, "ring geometry");
    static_assert(G >= 1 && G <= T, "stage groups");

    f2 W[T][NW];
    f2 PQ[PD];
    f2 RQ[PD];
    // this wave's D x 64 slots (LDS).  Typed as the packed pair itself: a
    // float2-struct ring made the compiler split every read into a b32 and a
    // b64 load plus a v_mov per stage
    f2 *ring;
    int lane;
    int k_first, S, lo_clamp, hi_clamp, nch, g_first, g_last, g_top, g_zero, row_bytes;
    int wbase;   // first row of the wave's buffer window (descriptors start there)
    int ch, vo_ld, vo_st, abase, dir;
    bool e0, e1;         // residual columns (kCol slots)
    // the Jacobi divisors and their reciprocals (uniform values, not a pointer
    // to the kernel argument: a pointer escaping into the block function made
    // the compiler copy the argument to scratch)
    float dx_sq, r_dx_sq, dy_sq, r_dy_sq, denom, r_denom;
    __amdgpu_buffer_rsrc_t rs_p, rs_r, rs_d;
    float m;
    float omax, imax, rmax;   // PERSIST: the guard's maxima (above)
    float mm[SPEC ? T : 1];   // SPEC: stage s's residual (segment rows only)
    int r0v, r1v;             // the segment's output rows (march order)
    int nst;                  // REDO: stages to run (< T)
    int nyl_;

    LdsMarch() = default;

    __device__ __forceinline__ int act(int vrow) const { return abase + dir * vrow; }

    // Row `vrow` (virtual, march order) of p' or rhs.  Rows outside the
    // allocation lie beyond the global boundary and rows past the segment's
    // last input row are never needed: both are clamped to a row that exists
    // (their values only reach halo rows that the boundary patch overwrites).
    template <int AUX = 0>
    __device__ __forceinline__ f2 ld(__amdgpu_buffer_rsrc_t rs, int vrow) const {
        if (CFD_LDS_DIAG & 1) return (f2){__int_as_float(vo_ld + vrow), 1.0f};
        vrow = vrow < k_first + S ? vrow : k_first + S - 1;
        int row = act(vrow);
        row = row < lo_clamp ? lo_clamp : (row > hi_clamp ? hi_clamp : row);
        const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, vo_ld, (row - wbase) * row_bytes, AUX);
        return (f2){__uint_as_float(v.x), __uint_as_float(v.y)};
    }
    __device__ __forceinline__ void st(const f2 &x, int row) const {
        if (CFD_LDS_DIAG & 4) {   // keep the value live without storing it
            asm volatile("" ::"v"(x.x), "v"(x.y));
            return;
        }
        const u32x2 v = {__float_as_uint(x.x), __float_as_uint(x.y)};
        __builtin_amdgcn_raw_buffer_store_b64(v, rs_d, vo_st, (row - wbase) * row_bytes, PST_AUX);
    }

    // One reference update (model.rs:775-793) of the lane's column pair.
    __device__ __forceinline__ f2 update(const f2 &B, const f2 &C, const f2 &Tp, const f2 &Rh) const {
        // horizontal: P(i+1) + P(i-1); the neighbour columns come from the
        // adjacent lanes (left lane's second column, right lane's first)
        const float hx = C.y + from_left(C.y);
        const float hy = C.x + from_right(C.x);
        const f2 h = {hx, hy};
        const f2 v = Tp + B;
        f2 s;
        if constexpr (SUMS) {
            s = (h + v) * r_dx_sq;   // == h * r_dx_sq + v * r_dy_sq under the guard
        } else {
            const f2 hz = fdiv2<FAST>(h, dx_sq, r_dx_sq);
            const f2 vt = fdiv2<FAST>(v, dy_sq, r_dy_sq);
            s = hz + vt;
        }
        const f2 pu = fdiv2<FAST>(s - Rh, denom, r_denom);
        const float omega = 0.75f;
        const float om1 = 1.0f - omega;
        return omega * pu + om1 * C;
    }

    // E: which boundary logic a slot carries.  kCol: the global column
    // patches and the residual's column range (waves at the left/right
    // boundary); kRow: the global row patches and boundary-row stores (waves
    // whose rows reach a global boundary row).
    static constexpr int kCol = 1, kRow = 2;

    template <int E>
    __device__ __forceinline__ f2 stage(const f2 &B, const f2 &C, const f2 &Tp, const f2 &Rh) const {
        f2 o = update(B, C, Tp, Rh);
        if (E & kCol) {
            if (ch == 0) o.x = o.y;             // P(0,j) = P(1,j)
            if (ch == nch - 1) o.y = 0.0f;      // P(nx-1,j) = 0
        }
        return o;
    }

    // Slot v (k = k_first + v), V_ == v (mod U).  GUARD 0: warm-up (V_ == v,
    // stage s runs from slot start(s) on); GUARD 2: the final partial group;
    // GUARD 3: both, decided at run time (CFD_LDS_COMPACT).
    template <int V_, int GUARD, int E>
    __device__ __forceinline__ void slot(int v) {
        if ((GUARD == 2 || GUARD == 3) && v >= S) return;
        if (CFD_LDS_SB >= 1) __builtin_amdgcn_sched_barrier(0);
        const int k = k_first + v;
        W[0][V_ % NW] = PQ[V_ % PD];                                 // input row k
        PQ[V_ % PD] = ld<PLD_AUX>(rs_p, k + PD);
        if (!(CFD_LDS_DIAG & 2))
            ring[(V_ % D) * 64 + lane] = RQ[V_ % PD];                 // rhs row k
        RQ[V_ % PD] = ld(rs_r, k + PD);
        // the slot's T ring reads issued together (the ring rows of earlier
        // slots; this slot's write went to another entry): one LDS latency
        // per slot instead of one per stage
        f2 rhv[T];
        if (CFD_LDS_HOIST && !(CFD_LDS_DIAG & 2)) {
#pragma unroll
            for (int s = 1; s <= T; ++s) rhv[s - 1] = ring[((V_ - s - off(s) + 8 * D) % D) * 64 + lane];
        }
#pragma unroll
        for (int s = 1; s <= T; ++s) {
            if (GUARD == 0 && V_ < start(s)) continue;               // compile-time
            if (GUARD == 3 && v < start(s)) continue;                // wave-uniform
            if (CFD_LDS_SB >= 2 && s > 1) __builtin_amdgcn_sched_barrier(0);
            const int r = k - s - off(s);
            const f2 rh = (CFD_LDS_DIAG & 2) ? RQ[(V_ + s) % PD]
                                             : (CFD_LDS_HOIST ? rhv[s - 1]
                                                              : ring[((V_ - s - off(s) + 8 * D) % D) * 64 + lane]);
            // stage s-1 finished row r+1 in slot v - dl (dl = 0 inside a
            // group, 1 at a group's first stage), row r one slot earlier, ...
            constexpr int kW = 4 * NW;
            const int dl = off(s) - off(s - 1);
            const f2 &B = W[s - 1][(V_ - dl - 2 + kW) % NW];         // stage s-1, row r-1
            const f2 &C = W[s - 1][(V_ - dl - 1 + kW) % NW];         //            row r
            const f2 &Tp = W[s - 1][(V_ - dl + kW) % NW];            //            row r+1
            if (REDO && s > nst) continue;                            // wave-uniform
            if constexpr (TRACK_IN) {
                // stage 1 reads every input row (as Tp, once) and every rhs row
                if (s == 1) {
                    imax = fmaxf(fmaxf(imax, fabsf(Tp.x)), fabsf(Tp.y));
                    rmax = fmaxf(fmaxf(rmax, fabsf(rh.x)), fabsf(rh.y));
                }
            }
            f2 n = stage<E>(B, C, Tp, rh);
            if constexpr (SPEC) {
                // every stage is one reference sweep: its max |new - old|.
                // Waves whose rows reach no global boundary row take every
                // row they compute, branch-free: a row outside the segment
                // [r0v, r1v) (warm-up and run-out cone) holds the exact
                // sweep value of an interior row — its inputs are all loaded
                // rows, k_first = r0v - T — which the segment owning it also
                // counts, and a max is unchanged by a repeated element.  The
                // row-edge waves count only their own rows: with k_first =
                // r0v - T, r - r0v = v - s - T (compile-time in the warm-up).
                bool in_seg;
                if constexpr (!(E & kRow))
                    in_seg = true;
                else if constexpr (GUARD == 0)
                    in_seg = V_ - s - T >= 0 && v - s - T < r1v - r0v;
                else
                    in_seg = v - s - T >= 0 && v - s - T < r1v - r0v;
                if (in_seg) {
                    const f2 d = n - C;
                    if (!(E & kCol)) {
                        mm[s - 1] = fmaxf(fmaxf(mm[s - 1], fabsf(d.x)), fabsf(d.y));
                    } else {
                        if (e0) mm[s - 1] = fmaxf(mm[s - 1], fabsf(d.x));
                        if (e1) mm[s - 1] = fmaxf(mm[s - 1], fabsf(d.y));
                    }
                }
            }
            if (REDO && s == nst) {
                // the stored stage: only rows of this segment (the march
                // computes the T-stage window, wider than nst stages need)
                if (r >= r0v && r < r1v) {
                    const int ra = act(r);
                    st(n, ra);
                    if ((E & kRow) && r == g_first) st(n, g_zero);
                    if ((E & kRow) && r == g_last) st(n, g_top);
                }
            } else if (s < T) {
                // stage s's row r-1 is its previous slot's row
                if ((E & kRow) && r == g_top) n = W[s][(V_ - 1 + kW) % NW]; // P(i,ny-1) = P(i,ny-2)
                W[s][V_ % NW] = n;
                if ((E & kRow) && r == g_first) W[s][(V_ - 1 + kW) % NW] = n; // P(i,0) = P(i,1)
            } else {
                const int ra = act(r);
                if (RES && ra >= 0 && ra < nyl_) {
                    const f2 d = n - C;
                    if (!(E & kCol)) {
                        m = fmaxf(fmaxf(m, fabsf(d.x)), fabsf(d.y));
                    } else {
                        if (e0) m = fmaxf(m, fabsf(d.x));
                        if (e1) m = fmaxf(m, fabsf(d.y));
                    }
                }
                st(n, ra);
                if ((E & kRow) && r == g_first) st(n, g_zero);
                if ((E & kRow) && r == g_last) st(n, g_top);
#ifndef CFD_PROBE_NOOMAX
#define CFD_PROBE_NOOMAX 0
#endif
                if constexpr (TRACK_OUT && !CFD_PROBE_NOOMAX)
                    omax = fmaxf(fmaxf(omax, fabsf(n.x)), fabsf(n.y));
            }
        }
    }

    template <int V_, int E>
    __device__ __forceinline__ void warmup() {
        if constexpr (V_ < WARM) {
            slot<V_, 0, E>(V_);
            warmup<V_ + 1, E>();
        }
    }

    // U slots from `base`; OFF == base (mod U)
    template <int J, int GUARD, int E, int OFF = WARM>
    __device__ __forceinline__ void group(int base) {
        if constexpr (J < U) {
            slot<OFF + J, GUARD, E>(base + J);
            group<J + 1, GUARD, E, OFF>(base);
        }
    }

    // Issue priority from progress.  The SIMD arbiter issues from the oldest
    // ready wave, so of the ~4 equal marches sharing a SIMD the first-launched
    // finishes first and the last one runs its final third nearly alone, at
    // the latency of its own dependent chain (r2 wave timeline: ends at 21 /
    // 25 / 32 / 39 us for one 40-row launch).  A wave lowers its priority as
    // it passes each quarter of its march, so the waves behind catch up and
    // the SIMD keeps four waves to issue from until close to the end.
    __device__ __forceinline__ void set_prio(int done) const {
        if (!CFD_LDS_PRIO) return;
        const int rows = S - WARM, d4 = 4 * done;   // wave-uniform
        if (d4 >= 3 * rows)
            __builtin_amdgcn_s_setprio(0);
        else if (d4 >= 2 * rows)
            __builtin_amdgcn_s_setprio(1);
        else if (d4 >= rows)
            __builtin_amdgcn_s_setprio(2);
        else
            __builtin_amdgcn_s_setprio(3);
    }

    // E: 0 (interior waves), kCol (waves at the left/right boundary), or
    // kCol|kRow (waves whose rows reach a global boundary row; the column
    // patches are no-ops on interior columns).  Chosen once per wave: a
    // per-group switch between paths costs ~15 VGPRs of phi copies.
    template <int E>
    __device__ __forceinline__ void run() {
        if (CFD_LDS_COMPACT) {
            // warm-up and tail through one run-time-guarded group: half the
            // code of the unrolled warm-up + guarded tail (2U >= WARM)
            static_assert(2 * U >= WARM, "warm-up fits two groups");
            set_prio(0);
            group<0, 3, E, 0>(0);
            group<0, 3, E, 0>(U);
            int base = 2 * U;
            for (; base + U <= S; base += U) {
                set_prio(base - WARM);
                group<0, 1, E, 0>(base);
            }
            set_prio(base - WARM);
            if (base < S) group<0, 3, E, 0>(base);
            return;
        }
        set_prio(0);
        warmup<0, E>();
        int base = WARM;
        const int full_end = WARM + ((S - WARM) / U) * U;
        for (; base < full_end; base += U) {
            set_prio(base - WARM);
            group<0, 1, E>(base);
        }
        set_prio(base - WARM);
        if (base < S) group<0, 2, E>(base);
    }
};

// One T-sweep block of one workgroup's four wave tiles (the body of
// k_jacobi_lds; k_jacobi_persist runs it once per block).  `bid`: the
// workgroup's (XCD-renumbered) index.  Returns without touching memory for
// waves with no rows.
// trk (persistent blocks): per wave, trk[3 w .. 3 w + 2] = max |p'| of the
// rows it stored, of the p' rows it loaded and of the rhs rows it used (the
// last two only in the reference's form; 0 where not tracked or no rows).
template <int T, int FAST, int MODE, bool SUMS = false>
__device__ __forceinline__ void lds_block(const Geom &g, float *__restrict__ pa,
                                          float *__restrict__ pb, const float *__restrict__ rhs,
                                          Ctl *ctl, uint32_t *res_slots, int par, int out_lo,
                                          int out_hi, int nwc, int nseg, int wlo, int whi, f2 *lds,
                                          int nst, int bid, float *trk = nullptr) {
    using M = LdsMarch<T, FAST, MODE, SUMS>;
    constexpr bool RES = M::RES;
    M w;
    w.nst = nst;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int lane = (int)threadIdx.x & 63;
    if (M::PERSIST && trk && lane == 0) trk[3 * wave] = trk[3 * wave + 1] = trk[3 * wave + 2] = 0.0f;
    const int wc = bid % nwc;
    const int seg = (bid / nwc) * kLdsWaves + wave;
    const int nrows = out_hi - out_lo;
    if (seg >= nseg) return;
    // rows split in proportion to weights: 16 per segment, wlo / whi for the
    // first / last one (lighter where that segment runs the boundary-row path)
    const long total = nseg == 1 ? 16 : wlo + whi + 16L * (nseg - 2);
    auto cum = [&](int i) -> long { return i <= 0 ? 0 : (i >= nseg ? total : wlo + 16L * (i - 1)); };
    const int r0 = out_lo + (int)(cum(seg) * nrows / total);
    const int r1 = out_lo + (int)(cum(seg + 1) * nrows / total);
    if (r0 >= r1) return;
    const int nx = g.nx;
    w.ring = lds + wave * M::D * 64;
    w.lane = lane;
    w.nch = nx / 2;
    w.nyl_ = g.nyl;
    w.lo_clamp = -g.hg;
    w.hi_clamp = g.nyl + g.hg - 1;
    w.ch = wc * M::OUTL - M::H + lane;
    const bool in_dom = w.ch >= 0 && w.ch < w.nch;
    const bool out_lane = in_dom && lane >= M::H && lane < 64 - M::H;
    const int col = 2 * w.ch;
    w.row_bytes = nx * 4;
    constexpr int kFar = 0x7FFF0000;   // voffset of a lane that must not touch memory
    w.vo_ld = in_dom ? col * 4 : kFar;
    w.vo_st = out_lane ? col * 4 : kFar;
    // buffers ping-pong once per LAUNCH: par = launches since the solve began
    const int si = (ctl->cur + par) & 1;
    float *src_alloc = si ? pb : pa;
    float *dst_alloc = si ? pa : pb;
    // buffer descriptors over the rows this wave can touch, [r0 - T, r1 + T)
    // clamped to the allocation, with a row of margin: offsets stay small at
    // any field size, so a parked lane's voffset (kFar) plus the row offset
    // never wraps 2^32 and always lands past the window (fields of any size,
    // not just up to 1 GiB)
    const int wb = max(w.lo_clamp, r0 - T - 1), wt = min(w.hi_clamp, r1 + T);
    w.wbase = wb;
    const long woff = (long)(wb - w.lo_clamp) * nx;
    const int wbytes = (wt - wb + 1) * nx * 4;
    w.rs_p = __builtin_amdgcn_make_buffer_rsrc(src_alloc + woff, 0, wbytes, 0x00020000);
    w.rs_d = __builtin_amdgcn_make_buffer_rsrc(dst_alloc + woff, 0, wbytes, 0x00020000);
    w.rs_r = __builtin_amdgcn_make_buffer_rsrc((void *)(rhs - (long)g.hg * nx + woff), 0, wbytes,
                                               0x00020000);
    w.dx_sq = g.dx_sq;
    w.r_dx_sq = g.r_dx_sq;
    w.dy_sq = g.dy_sq;
    w.r_dy_sq = g.r_dy_sq;
    w.denom = g.denom;
    w.r_denom = g.r_denom;
    // residual columns 1..=nx-8 (the reference's full 8-lane chunks, Q6)
    w.e0 = out_lane && col >= 1 && col <= nx - 8;
    w.e1 = out_lane && col + 1 >= 1 && col + 1 <= nx - 8;
    w.g_first = 1 - g.j0;
    w.g_last = g.ny - 2 - g.j0;
    w.g_top = g.ny - 1 - g.j0;
    w.g_zero = -g.j0;
    w.m = 0.0f;
    w.omax = w.imax = w.rmax = 0.0f;
#pragma unroll
    for (int s = 0; s < (M::SPEC ? T : 1); ++s) w.mm[s] = 0.0f;
    w.r0v = r0;
    w.r1v = r1;
    w.k_first = r0 - T;
    w.S = (r1 - r0) + M::WARM;
    w.abase = 0;
    w.dir = 1;
    const f2 z = {0.0f, 0.0f};
#pragma unroll
    for (int s = 0; s < T; ++s)
#pragma unroll
        for (int q = 0; q < M::NW; ++q) w.W[s][q] = z;
    // edge waves: a lane stores column 0 or a column outside the residual
    // range, or a stage touches a global boundary row; interior waves skip
    // all boundary logic
    const int ch_lo = wc * M::OUTL - M::H, ch_hi = ch_lo + 63;
    const bool col_edge = ch_lo <= 0 || 2 * (ch_hi + 1) > nx - 8;
    const int lo_row = w.k_first - 2, hi_row = r1 + T + M::OFFT + 2;   // every row a stage computes
    auto hits = [&](int r) { return r >= lo_row && r <= hi_row; };
    const bool row_edge = hits(w.g_zero) || hits(w.g_first) || hits(w.g_last) || hits(w.g_top);
    const bool edge = col_edge || row_edge;
    // odd interior segments march downward through the mirrored rows (the
    // stencil is symmetric and f32 addition commutative: same bits), so
    // neighbouring segments read their shared rows at the same time
    if (!edge && (seg & 1)) {
        w.abase = r0 + r1 - 1;
        w.dir = -1;
    }
#pragma unroll
    for (int q = 0; q < M::PD; ++q) {
        w.PQ[q] = w.template ld<M::PLD_AUX>(w.rs_p, w.k_first + q);
        w.RQ[q] = w.ld(w.rs_r, w.k_first + q);
    }
    // the march and what the launch publishes
    if (row_edge)
        w.template run<M::kCol | M::kRow>();
    else if (col_edge)
        w.template run<M::kCol>();
    else
        w.template run<0>();
    if (M::PERSIST && trk) {
        const float o = wave_max(out_lane ? w.omax : 0.0f);
        const float im = M::TRACK_IN ? wave_max(w.imax) : 0.0f;
        const float rm = M::TRACK_IN ? wave_max(w.rmax) : 0.0f;
        if (lane == 0) {
            trk[3 * wave] = o;
            trk[3 * wave + 1] = im;
            trk[3 * wave + 2] = rm;
        }
    }
    if (M::SPEC) {
#pragma unroll
        for (int s = 0; s < T; ++s) {
            const float ms = wave_max(out_lane ? w.mm[s] : 0.0f);
            if (lane == 0 && ms > 0.0f)
                atomicMax(res_slots + (size_t)s * kResSlots * kResStride +
                              ((bid * kLdsWaves + wave) & (kResSlots - 1)) * kResStride,
                          __float_as_uint(ms));
        }
    }
    if (!RES) return;
    const float m = wave_max(out_lane ? w.m : 0.0f);
    if (lane == 0) publish_max(res_slots, bid * kLdsWaves + wave, m);
}

// Minimum waves per SIMD the register allocation must allow (the SPEC
// launch holds T residual maxima on top of the plain march: 99 VGPRs, 4
// waves; pinned to 5 it spills).
#ifndef CFD_LDS_SPEC_WPE
#define CFD_LDS_SPEC_WPE 5
#endif
constexpr int lds_min_waves(int mode) {
    return mode == 2 ? CFD_LDS_SPEC_WPE : (CFD_LDS_WPE > 0 ? CFD_LDS_WPE : 1);
}
// The lagged early-exit check (r5, single-domain speculative solves; replaces
// the one-workgroup k_spec_check launch after every speculative launch): each
// workgroup of the NEXT launch folds the T residual slot sets of launch lpar
// itself (sweeps [it0, it0 + T), published a launch boundary earlier, never
// reset during the solve -- the finalize folds and clears them) and finds the
// first sweep below p_tol (model.rs:816).  Every workgroup computes the same
// value; workgroup 0 publishes it (the launches that ran and, with `stop`, the
// stop / re-run fields k_spec_check would set).  Returns that sweep's index,
// T when none converged.  Called by every thread of the workgroup.
__device__ __forceinline__ int spec_lag_first(const Geom &g, Ctl *ctl, const uint32_t *set0, int it0,
                                              int T, int lpar, bool stop = true) {
    __shared__ float e_s[kMaxTemporal];
    const int wv = (int)threadIdx.x >> 6;
    for (int s = wv; s < T; s += kLdsWaves) {
        const float v = read_max(set0 + (size_t)s * kResSlots * kResStride, ctl->err[it0 + s]);
        if ((threadIdx.x & 63) == 0) e_s[s] = v;
    }
    __syncthreads();
    int j = 0;
    while (j < T && !(e_s[j] < g.p_tol)) ++j;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        ctl->spec_launches = lpar + 1;
        if (stop && j < T) {
            ctl->spec_stop = 1;
            ctl->spec_launch = lpar;
            ctl->spec_redo = j + 1 < T ? j + 1 : 0;
        }
    }
    return j;
}

template <int T, int FAST, int MODE>
__global__ __launch_bounds__(kLdsWaves * 64, lds_min_waves(MODE)) void k_jacobi_lds(
    Geom g, float *__restrict__ pa, float *__restrict__ pb, const float *__restrict__ rhs,
    Ctl *ctl, uint32_t *res_slots, int pass, int par, int out_lo, int out_hi, int nwc, int nseg,
    int wlo, int whi, int it, int lag) {
    using M = LdsMarch<T, FAST, MODE>;
    [[maybe_unused]] constexpr bool RES = M::RES;   // the stamp guard's
    __shared__ f2 lds[kLdsWaves * M::D * 64];
#if CFD_LDS_STAMP
    const unsigned long long st_rt0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long st_t0 = __builtin_amdgcn_s_memtime();
    struct StampOnExit {
        unsigned long long rt0, t0;
        unsigned long long bid;   // the XCD-renumbered block (tile: bid % nwc, row group bid / nwc)
        __device__ ~StampOnExit() {
            if (RES) return;
            const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            // hwreg(id, 0, 32): HW_ID = 4, XCC_ID = 20
            const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));
            const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11));
            const int idx = (int)blockIdx.x * kLdsWaves + ((int)threadIdx.x >> 6);
            if ((threadIdx.x & 63) == 0 && idx < kStampWaves) {
                g_lds_stamp[idx * 4 + 0] = rt0;
                g_lds_stamp[idx * 4 + 1] = rt1;
                g_lds_stamp[idx * 4 + 2] = (bid << 40) | ((t1 - t0) & 0xFFFFFFFFFFull);
                g_lds_stamp[idx * 4 + 3] = ((unsigned long long)xcc << 32) | hw;
            }
        }
    } stamp_guard{st_rt0, st_t0, (unsigned long long)xcd_block(g)};
#endif
    if (pass_off(ctl, pass)) return;
    int nst = 0;
    if constexpr (M::SPEC) {
        if (lag > 0) {
            // the previous launch's check (k_spec_check's, a launch boundary
            // after its residuals were published).  spec_stop is read once
            // per workgroup: workgroup 0 of THIS launch may set it meanwhile,
            // and the workgroup's waves must take one path (barriers below)
            __shared__ int stop_s;
            if (threadIdx.x == 0) stop_s = ctl->spec_stop;
            __syncthreads();
            if (stop_s) return;
            if (spec_lag_first(g, ctl, res_slots - (size_t)lag * kResSlots * kResStride, it - lag, lag,
                               par - 1) < lag)
                return;   // it converged: this launch and every later one skip
        } else if (ctl->spec_stop) {
            return;   // an earlier launch of the solve converged
        }
    }
    if constexpr (M::REDO) {
        if (lag > 0 && !ctl->spec_stop) {
            // the solve's last launch (par, sweeps [it, it + lag)) is checked
            // here; only the count of launches that ran is published (the
            // other workgroups read spec_stop / spec_redo / spec_launch)
            const int j = spec_lag_first(g, ctl, res_slots, it, lag, par, false);
            nst = j + 1 < lag ? j + 1 : 0;
        } else {
            nst = ctl->spec_redo;
            par = ctl->spec_launch;   // re-run that launch: same source, same destination
        }
        if (nst <= 0) return;
    }
    lds_block<T, FAST, MODE>(g, pa, pb, rhs, ctl, res_slots, par, out_lo, out_hi, nwc, nseg, wlo,
                             whi, lds, nst, xcd_block(g));
}

// Persistent fixed-count solve: ONE launch runs nblk blocks of T sweeps
// (par0.. launches of the per-launch form) over ntiles tiles (tile = the four
// wave segments of one workgroup of the per-launch form).  Task (t, b), block
// b of tile t, reads the rows that t and its 3 x 3 neighbours (adjacent wave
// columns hold the halo lanes' columns, adjacent row groups the T-row input
// bands) wrote in block b-1, and overwrites the buffer they read in block
// b-1, so it starts once all nine have finished block b-1 — no launch
// boundary, no grid-wide drain, and a slow tile holds back only its
// neighbours.
//
// Ownership with stealing.  Workgroup w owns tile w (XCD-renumbered, as the
// per-launch form maps it) and runs its blocks in order, so on a GPU that
// holds every workgroup at once each one keeps its tile (and its rows' L2) for
// the whole solve.  A block is CLAIMED before it runs: tile t's line holds a
// claim counter beside its done flag, advanced by compare-and-swap, so every
// task runs exactly once.  An owner claims all its tile's unclaimed blocks
// with one CAS when it starts (no atomic per block on the fast path).  A
// workgroup that has waited more than `steal` ticks for a
// neighbour's block b-1 that nobody has claimed — its owner is not resident
// (a co-tenant kernel, another model's launch, RCCL kernels, a grid larger
// than the GPU holds) — claims that block itself, runs it when ready and then
// returns to its own task (a small stack of claimed tasks in LDS).
// Deadlock-free by construction: a wait is on a block that is either claimed
// by a running workgroup or stealable; the owner's own task sits at the
// bottom of its stack and a thief takes only a block below the one it waits
// to run (one CAS from the value it read, never "the next one"), so blocks
// fall strictly up every stack, no task depends on one below it, and waits
// never form a cycle.  The launch completes with any number of its workgroups resident.
// (The r3 form needed all of them resident at once: a co-tenant could strand
// it until its spin limit, with p' left invalid; a ticketed form that took
// tasks in block order measured 7.6 us per sweep against 4.7: a workgroup
// then waits for an arbitrary tile's neighbourhood, in effect a grid barrier
// per block.)
//
// Hand-off (MI355X_MICROARCH.md "Valid forms", Consumer, always): p' stores
// write through (sc1) and every wave drains them (s_waitcnt vmcnt(0)) before
// the workgroup's barrier, then ONE lane stores the tile's flag (agent scope);
// a waiting workgroup's wave 0 polls the nine flags (relaxed agent loads,
// s_sleep), then ONE agent acquire (buffer_inv sc1) + vmcnt(0) + the
// workgroup barrier before any p' load.  The launch runs several workgroups
// per CU, outside the table under which sc1 loads alone may replace the
// acquire, so the acquire stays (acq = 1).  Flags and claim counters hold epoch * 2^kPersistBlockBits
// + blocks done / claimed (a solve has at most kMaxSweeps / 8 = 512 blocks);
// the host gives every persistent launch a new epoch (never under graph
// capture: arguments would freeze), so a value below the epoch's base reads
// as 0 and nothing needs clearing between launches.  Waits are bounded by
// wall time (s_memrealtime, `deadline` ticks of 10 ns): past it the waiter
// sets the abort word persist[1], every workgroup leaves at its next poll or
// at entry, and a zero-copy host word makes the model's next cfd_* call report
// CFD_ETIMEOUT (a fault: residency no longer causes one).
//
// SUMS guard (r4; sums != 0 when the grid allows the form at all, LdsMarch):
// task (t, b) of the owner runs the SUMS form when every p' value it reads is
// below plim = 2^124 / R and every rhs value below rlim = 2^124, which keeps
// every value its 8 sweeps form below 2^126 / R (a sweep adds at most
// 0.1875 |rhs| / R to max |p'|: |hz + vt| <= 4 R max|p'| = denom max|p'|), so
// R |h|, R |v| < 2^127.  What a task reads: rows its 3 x 3 neighbours stored in
// block b-1 -- each wave publishes max |p'| of its stores with the tile's
// flag, in the tile's line (words 2-5 / 6-9 by block parity) -- and rows no
// tile of this launch writes (a slab's rows beyond its band), constant during
// the launch but different in the two p' buffers: blocks 0 and 1 run the
// reference's form and measure the tile's inputs in each buffer (and its rhs
// rows); a stolen task runs the reference's form.  max is NaN-ignoring: a NaN
// propagates through either form as the same operand.
constexpr int kStealDepth = 16;
#ifndef CFD_PERSIST_WPE
#define CFD_PERSIST_WPE 3   // the padded launch's 3 waves per SIMD: at most 168 VGPRs
#endif
template <int T, int FAST>
__global__ __launch_bounds__(kLdsWaves * 64, CFD_PERSIST_WPE) void k_jacobi_persist(
    Geom g, float *__restrict__ pa, float *__restrict__ pb, const float *__restrict__ rhs,
    Ctl *ctl, uint32_t *persist, uint32_t *host_fail, uint32_t *res_slots, uint32_t epoch, int pass,
    int par0, int nblk, int out_lo, int out_hi, int nwc, int nseg, int wlo, int whi, int ngrp,
    int acq, uint32_t deadline, uint32_t steal, int late, int sums, float plim, float rlim) {
    using M = LdsMarch<T, FAST, 4>;
    __shared__ f2 lds[kLdsWaves * M::D * 64];
    // control (wave 0 writes, everyone reads after a barrier): the task to
    // run, the claimed-task stack, the owner's next claimed block
    // (-2: claim it now, -1: none left)
    __shared__ int run_tile_s, run_blk_s, abort_s, own_next_s, sp_s, fast_s;
    __shared__ int stk_tile[kStealDepth], stk_blk[kStealDepth];
    // the SUMS guard: per-wave maxima of the block just run (lds_block trk),
    // the own tile's input maxima per p' buffer and its rhs maximum
    __shared__ float trk_s[3 * kLdsWaves], own_im_s[2], own_rm_s;
    __shared__ int own_ok_s[2], nfast_s;
    if (pass_off(ctl, pass)) return;
    const int ntiles = ngrp * nwc;
    const int own = xcd_block(g);
    if (own >= ntiles) return;   // a grid larger than the tiles: nothing owned
    const unsigned base = epoch << kPersistBlockBits;
    uint32_t *lines = persist + kPersistHeadLines * kPersistFlagStride;   // per tile: [0] done, [1] claimed
    const int lane = (int)threadIdx.x & 63;
    // blocks claimed of a tile from its claim word (values of older epochs read 0)
    auto count = [&](unsigned v) -> int { return v < base ? 0 : (int)(v - base); };
    // claim blocks of tile t by CAS from `v` (a read or guess of its claim
    // word): the first block claimed, or -1 when every block is claimed or
    // (thief) the word was not `v`.  all = true (the owner, once, when it
    // starts): every block not yet claimed, retrying from the word's actual
    // value -- a resident owner thus holds its whole tile and no thief ever
    // touches it, with no atomic per block.  A thief (all = false) takes
    // exactly the one block it saw unclaimed, or nothing: a later block of
    // that tile could depend on a task the thief holds below it on its stack
    // (a cycle).
    auto claim = [&](int t, unsigned v, bool all) -> int {
        uint32_t *w = lines + (size_t)t * kPersistFlagStride + 1;
        for (;;) {
            const int c = count(v);
            if (c >= nblk) return -1;
            unsigned exp = v;
            if (__hip_atomic_compare_exchange_strong(w, &exp, base + (unsigned)(all ? nblk : c + 1),
                                                     __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT))
                return c;
            if (!all) return -1;
            v = exp;   // the word as it was: retry from it
        }
    };
    if (threadIdx.x == 0) {
        sp_s = 0;
        own_next_s = -2;
        own_ok_s[0] = own_ok_s[1] = 0;
        own_im_s[0] = own_im_s[1] = own_rm_s = 0.0f;
        nfast_s = 0;
        // fail fast after an abort (every later launch of the model too)
        abort_s = __hip_atomic_load(persist + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
        if (late > 0 && own % late == 1) {   // test knob: this owner starts late (not resident)
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (__builtin_amdgcn_s_memrealtime() - t0 < 200000u) __builtin_amdgcn_s_sleep(127);
        }
    }
    __syncthreads();
    if (abort_s) return;
    for (;;) {
        if (threadIdx.x < 64) {
            // ---- wave 0: the next task that is ready (claiming / stealing) ----
            int sp = sp_s, run_t = -1, run_b = -1;
            bool fail = false, fast = false;
            if (sp == 0) {
                int nb = own_next_s;
                if (nb == -2) {
                    int c = -1;
                    if (lane == 0) c = claim(own, 0u, true);
                    nb = __builtin_amdgcn_readfirstlane(c);
                }
                if (nb >= 0) {
                    if (lane == 0) {
                        stk_tile[0] = own;
                        stk_blk[0] = nb;
                    }
                    sp = 1;
                }
                own_next_s = -1;
            }
            while (sp > 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // stack writes before reads
                const int tt = stk_tile[sp - 1], bb = stk_blk[sp - 1];
                if (bb == 0) {
                    run_t = tt, run_b = bb;
                    --sp;
                    break;
                }
                // lanes 0..8 watch the task's tile and its neighbours, lane 9 the abort word
                const int wc = tt % nwc, gi = tt / nwc;
                const int c = wc + lane % 3 - 1, r = gi + lane / 3 - 1;
                const bool nbr = lane < 9 && c >= 0 && c < nwc && r >= 0 && r < ngrp;
                const int nt = nbr ? r * nwc + c : -1;
                const uint32_t *w = nbr ? lines + (size_t)nt * kPersistFlagStride
                                        : (lane == 9 ? persist + 1 : nullptr);
                const unsigned want = base + (unsigned)bb;
                const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                bool ready = false, pushed = false;
                for (;;) {
                    const unsigned v = w ? __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                         : 0u;
                    const bool ok = lane < 9 ? (!nbr || v >= want) : v == 0u;
                    if (__all(ok)) {
                        ready = true;
                        break;
                    }
                    const uint64_t el = __builtin_amdgcn_s_memrealtime() - t0;
                    if (__any(lane == 9 && v != 0u) || el > (uint64_t)deadline) {
                        fail = true;
                        break;
                    }
                    if (el > (uint64_t)steal && sp < kStealDepth) {
                        // a neighbour block this task needs that nobody has claimed
                        const unsigned cw = nbr && v < want
                                                ? __hip_atomic_load(w + 1, __ATOMIC_RELAXED,
                                                                    __HIP_MEMORY_SCOPE_AGENT)
                                                : 0u;
                        const bool cand = nbr && v < want && count(cw) < bb;
                        const uint64_t m = __ballot(cand);
                        if (m) {
                            const int l = __builtin_ctzll(m);
                            const int st = __shfl(nt, l, 64);
                            const unsigned sv = __shfl(cw, l, 64);
                            int got = -1;
                            if (lane == 0) {
                                got = claim(st, sv, false);
                                if (got >= 0)   // steals counted for diagnostics (cfd_get_persist_steals)
                                    __hip_atomic_fetch_add(persist + 2, 1u, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT);
                            }
                            got = __builtin_amdgcn_readfirstlane(got);
                            if (got >= 0) {   // run it first, then come back to this task
                                if (lane == 0) {
                                    stk_tile[sp] = st;
                                    stk_blk[sp] = got;
                                }
                                ++sp;
                                pushed = true;
                                break;
                            }
                        }
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                if (fail) break;
                if (pushed) continue;
                if (ready) {
                    run_t = tt, run_b = bb;
                    --sp;
                    if (acq) {
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    } else {
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keeps loads below the poll
                    }
                    if (sums && tt == own && bb >= 2 && own_ok_s[bb & 1] && own_rm_s < rlim &&
                        own_im_s[bb & 1] < plim) {
                        // the neighbours' stores of block bb-1 (published with their flags)
                        float mo = 0.0f;
                        if (nbr) {
                            const uint32_t *q = w + 2 + 4 * ((bb - 1) & 1);
#pragma unroll
                            for (int k = 0; k < kLdsWaves; ++k)
                                mo = fmaxf(mo, __uint_as_float(__hip_atomic_load(
                                                   q + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
                        }
                        fast = wave_max(mo) < plim;
                    }
                    break;
                }
            }
            if (lane == 0) {
                sp_s = sp;
                run_tile_s = run_t;
                run_blk_s = run_b;
                fast_s = fast;
                abort_s = fail;
                if (fail) {
                    __hip_atomic_store(persist + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (host_fail)   // zero-copy host word: cfd_* calls report CFD_ETIMEOUT
                        __hip_atomic_store(host_fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
        }
        __syncthreads();
        const int tile = run_tile_s, b = run_blk_s;
        if (abort_s || tile < 0) {   // workgroup-uniform
            if (threadIdx.x == 0 && nfast_s)   // diagnostics: blocks run in the SUMS form
                __hip_atomic_fetch_add(persist + 3, (uint32_t)nfast_s, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        const bool fast = fast_s;
        const bool res = res_slots && b == nblk - 1;   // the solve's last block: its residual too
#ifndef CFD_PROBE_NOSUMS
#define CFD_PROBE_NOSUMS 0   // (diagnostic builds: the reference's form only)
#endif
        if constexpr (FAST == 1 && !CFD_PROBE_NOSUMS) {
            if (fast) {
                if (res)
                    lds_block<T, FAST, 5, true>(g, pa, pb, rhs, ctl, res_slots, par0 + b, out_lo, out_hi,
                                                nwc, nseg, wlo, whi, lds, 0, tile, trk_s);
                else
                    lds_block<T, FAST, 4, true>(g, pa, pb, rhs, ctl, nullptr, par0 + b, out_lo, out_hi,
                                                nwc, nseg, wlo, whi, lds, 0, tile, trk_s);
            }
        }
        if (!fast) {
            if (res)
                lds_block<T, FAST, 5>(g, pa, pb, rhs, ctl, res_slots, par0 + b, out_lo, out_hi, nwc,
                                      nseg, wlo, whi, lds, 0, tile, trk_s);
            else
                lds_block<T, FAST, 4>(g, pa, pb, rhs, ctl, nullptr, par0 + b, out_lo, out_hi, nwc,
                                      nseg, wlo, whi, lds, 0, tile, trk_s);
        }
        // every wave's max |p'| stored, with (before) the flag: the next
        // block's guard of the neighbours (written through, drained below)
        if (sums && lane == 0) {
            const int wv = (int)threadIdx.x >> 6;
            __hip_atomic_store(lines + (size_t)tile * kPersistFlagStride + 2 + 4 * (b & 1) + wv,
                               __float_as_uint(trk_s[3 * wv]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // publish: every wave's write-through stores drained, then one flag
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            // the owner's next block (it claimed all of them when it started)
            if (tile == own) {
                own_next_s = b + 1 < nblk ? b + 1 : -1;
                if (fast) {
                    ++nfast_s;
                } else {
                    // the tile's inputs in the buffer block b read, and its rhs
                    float im = 0.0f, rm = 0.0f;
#pragma unroll
                    for (int k = 0; k < kLdsWaves; ++k) {
                        im = fmaxf(im, trk_s[3 * k + 1]);
                        rm = fmaxf(rm, trk_s[3 * k + 2]);
                    }
                    own_im_s[b & 1] = fmaxf(own_im_s[b & 1], im);
                    own_ok_s[b & 1] = 1;
                    own_rm_s = fmaxf(own_rm_s, rm);
                }
            }
            __hip_atomic_store(lines + (size_t)tile * kPersistFlagStride, base + (unsigned)b + 1u,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Workgroups of k_jacobi_lds<T, FAST, RES> one CU holds at once (occupancy
// API, cached per instantiation).
// Dynamic LDS added to a launch (bytes) to cap the workgroups the hardware
// places on one CU, so a round of resident waves is spread evenly at a chosen
// occupancy.  Default: 24 KiB on fixed-count launches (MODE 0/1) whose p'
// pair + rhs fit the 256 MiB Infinity Cache: 18 + 24 KiB per 4-wave
// workgroup admits 3 per CU (3 waves per SIMD) where the registers allow 5,
// and the round's 3/5 of the waves each march a 5/3 longer segment (less
// warm-up recompute) on a launch that is VALU- not memory-bound: developed
// 4096^2 cavity 5.60 -> 5.28 us/sweep (profiles/r3/ab_pad3.log).  None on
// HBM-streaming slabs, where more waves in flight pay (8192^2: 23.8 vs 24.5
// us/sweep padded), nor on the speculative launches (ab_pad_parity.log).
// CFD_LDS_PAD=<bytes> forces one value on every launch.
// The test is on the OWNED rows (r4): every slab of the weak-scaling series
// (4096^2, 8192x2048 and 16384x1024, 16.78 M cells, 201 MB) runs the same
// geometry; with the hg ghost rows counted, the 16384x1024 slab (32 ghost rows
// each side, 214 MB) fell past the threshold and ran unpadded while the
// others were padded.  The ghost rows (6 % at C5) still fit the 256 MiB cache.
inline int lds_pad_bytes(const Geom &g, int mode) {
    static const int forced = [] {
        const char *e = getenv("CFD_LDS_PAD");
        return e ? std::max(0, std::min(64 * 1024, atoi(e))) : -1;
    }();
    if (forced >= 0) return forced;
    constexpr uint64_t kMallResident = 200ull << 20;
    const uint64_t ws = 3ull * (uint64_t)g.nyl * (uint64_t)g.nx * 4u;
    return mode <= 1 && ws <= kMallResident ? 24 * 1024 : 0;
}
template <int T, int FAST, int MODE>
int lds_blocks_per_cu(int pad) {
    static int cache[2] = {0, 0};   // unpadded, padded (one pad value per process)
    int &nb = cache[pad > 0 ? 1 : 0];
    if (nb == 0) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &n, reinterpret_cast<const void *>(&k_jacobi_lds<T, FAST, MODE>), kLdsWaves * 64, pad) !=
                hipSuccess ||
            n < 1)
            n = 1;
        nb = n;
    }
    return nb;
}

// Segments per wave column.  g.tb_rows > 0: fixed rows per segment.  0
// (default): as many segments as ONE round of resident waves holds — every
// SIMD gets its waves at once and the same march length, so no CU waits for a
// second, partial round — or whole multiples of a round when a round would
// make segments longer than kMaxRows.
// occ_override > 0: size the round for that many workgroups per CU (the
// persistent kernel's own occupancy)
template <int T, int FAST, int MODE>
int lds_segments(const Geom &g, int nrows, int nwc, int pad, int occ_override = 0) {
    if (g.tb_rows > 0) return cdiv(nrows, g.tb_rows);
    constexpr int kMaxRows = 160, kMinRows = 8;
    const int bpc = occ_override > 0 ? occ_override : lds_blocks_per_cu<T, FAST, MODE>(pad);
    const int wgs_per_col = std::max(1, g.n_cu * bpc / nwc);
    const int per_round = kLdsWaves * wgs_per_col;
    // the persistent launch (occ_override) keeps ONE round whatever the
    // segment length: a tile per resident workgroup, so no tile waits for an
    // owner that is not resident (8192^2: two rounds made half the tiles run
    // by stealing, 274 vs 170 us per block, profiles/r4/prof_r4a)
    const int rounds =
        occ_override > 0 ? 1 : std::max(1, cdiv(nrows, (long)per_round * kMaxRows));
    return std::max(1, std::min(per_round * rounds, nrows / kMinRows));
}

template <int T, int MODE>
void launch_lds_t(const Geom &g, const Fields &f, int pass, int par, int it, int out_lo, int out_hi,
                  uint32_t *rs, hipStream_t s, int lag = 0) {
    const int nch = g.nx / 2;
    const int nwc = cdiv(nch, LdsMarch<T, 1, MODE>::OUTL);
    const int nrows = out_hi - out_lo;
    const int pad = lds_pad_bytes(g, MODE);
    const int nseg = g.fastdiv == 1   ? lds_segments<T, 1, MODE>(g, nrows, nwc, pad)
                     : g.fastdiv == 2 ? lds_segments<T, 2, MODE>(g, nrows, nwc, pad)
                                      : lds_segments<T, 0, MODE>(g, nrows, nwc, pad);
    const dim3 grid(nwc * cdiv(nseg, kLdsWaves)), block(kLdsWaves * 64);
    float *pa = f.pp[0] - (long)g.hg * g.nx, *pb = f.pp[1] - (long)g.hg * g.nx;
    // a segment whose rows reach a global boundary row runs the kCol|kRow
    // path, ~1.45x the VALU work per row of an interior one (r2 wave
    // timeline): it gets ~1/1.45 of the rows
    constexpr int kEdgeWeight = 11;
    const int reach = T + 2;
    const int wlo = out_lo - reach <= 1 - g.j0 ? kEdgeWeight : 16;
    const int whi = out_hi + reach >= g.ny - 2 - g.j0 ? kEdgeWeight : 16;
#define CFD_LDS_LAUNCH(FASTV)                                                                      \
    hipLaunchKernelGGL((k_jacobi_lds<T, FASTV, MODE>), grid, block, pad, s, g, pa, pb, f.rhs, f.ctl, \
                       rs, pass, par, out_lo, out_hi, nwc, nseg, wlo, whi, it, lag)
    if (g.fastdiv == 1)
        CFD_LDS_LAUNCH(1);
    else if (g.fastdiv == 2)
        CFD_LDS_LAUNCH(2);
    else
        CFD_LDS_LAUNCH(0);
#undef CFD_LDS_LAUNCH
}

// T sweeps per launch: mode 0 / 1 (plain / last-stage residual, chosen by
// rs != nullptr), 2 (SPEC, rs = the first stage's slot set), 3 (REDO, T = 8).
template <int T>
void launch_lds_T(const Geom &g, const Fields &f, int pass, int par, int it, int out_lo, int out_hi,
                  uint32_t *rs, int mode, hipStream_t s, int lag = 0) {
    if (mode == 2) {
        launch_lds_t<T, 2>(g, f, pass, par, it, out_lo, out_hi, rs, s, lag);
        return;
    }
    if constexpr (T == 8) {
        if (mode == 3) {
            launch_lds_t<8, 3>(g, f, pass, par, it, out_lo, out_hi, rs, s, lag);
            return;
        }
    }
    if (rs)
        launch_lds_t<T, 1>(g, f, pass, par, it, out_lo, out_hi, rs, s);
    else
        launch_lds_t<T, 0>(g, f, pass, par, it, out_lo, out_hi, rs, s);
}

// Workgroups of k_jacobi_persist<T, FAST> one CU holds at once with `pad`
// bytes of dynamic LDS: the occupancy API on the launched kernel itself,
// capped by the SGPR rule of MI355X_MICROARCH.md (Residency): at 97-112 SGPRs
// the hardware admits 6 four-wave workgroups where the API may say 7.  Used to
// size the tiles so one round of workgroups covers them; residency is no
// longer a correctness condition (claims and stealing, k_jacobi_persist).
template <int T, int FAST>
int persist_blocks_per_cu(int pad) {
    static int cache[2] = {0, 0};
    int &nb = cache[pad > 0 ? 1 : 0];
    if (nb == 0) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &n, reinterpret_cast<const void *>(&k_jacobi_persist<T, FAST>), kLdsWaves * 64, pad) !=
                hipSuccess ||
            n < 1)
            n = 1;
        nb = std::min(n, 6);
    }
    return nb;
}

// The persistent form of launch_lds_t<T, 0> over nblk blocks: the same tile
// geometry (pad, segments, weights), its round sized by the persistent
// kernel's own occupancy; one workgroup per tile.  false (nothing launched):
// more tiles than kPersistMaxGroups lines, or row groups shorter than two
// T-row bands.
template <int T>
bool launch_lds_persist_t(const Geom &g, const Fields &f, int pass, int par0, int nblk, int out_lo,
                          int out_hi, uint32_t epoch, uint32_t *rs, hipStream_t s) {
    const int nch = g.nx / 2;
    const int nwc = cdiv(nch, LdsMarch<T, 1, 0>::OUTL);
    const int nrows = out_hi - out_lo;
    const int pad = lds_pad_bytes(g, 0);
    const int occ = g.fastdiv == 1   ? persist_blocks_per_cu<T, 1>(pad)
                    : g.fastdiv == 2 ? persist_blocks_per_cu<T, 2>(pad)
                                     : persist_blocks_per_cu<T, 0>(pad);
    const int nseg = g.fastdiv == 1   ? lds_segments<T, 1, 0>(g, nrows, nwc, pad, occ)
                     : g.fastdiv == 2 ? lds_segments<T, 2, 0>(g, nrows, nwc, pad, occ)
                                      : lds_segments<T, 0, 0>(g, nrows, nwc, pad, occ);
    const int ngrp = cdiv(nseg, kLdsWaves);
    // rows for a T-row band per group: a task's input rows lie in its 3 x 3
    // neighbourhood
    if (ngrp * nwc > kPersistMaxGroups || nrows < ngrp * 2 * T) return false;
    // one workgroup per tile (each owns one); CFD_PERSIST_GRID=<n> launches
    // n >= tiles (the surplus owns nothing and leaves).  Knobs are read per
    // launch (one getenv each per solve) so tests can change them.
    const char *ge = getenv("CFD_PERSIST_GRID");
    const int nwg = std::max(ngrp * nwc, ge ? atoi(ge) : 0);
    const dim3 grid(nwg), block(kLdsWaves * 64);
    float *pa = f.pp[0] - (long)g.hg * g.nx, *pb = f.pp[1] - (long)g.hg * g.nx;
    constexpr int kEdgeWeight = 11;
    const int reach = T + 2;
    const int wlo = out_lo - reach <= 1 - g.j0 ? kEdgeWeight : 16;
    const int whi = out_hi + reach >= g.ny - 2 - g.j0 ? kEdgeWeight : 16;
    const int acq = 1;   // the agent acquire after each poll (MI355X_MICROARCH.md)
    // wait deadline in s_memrealtime ticks (100 MHz): CFD_PERSIST_DEADLINE_US,
    // default 10 s (a wait that long is a fault; time-sliced GPUs stay far
    // below it)
    const char *de = getenv("CFD_PERSIST_DEADLINE_US");
    const double dl_us = de ? std::max(0.0, atof(de)) : 10e6;
    const uint32_t deadline = (uint32_t)std::min(4.0e9, dl_us * 100.0);
    // a neighbour block unclaimed after this long is stolen
    // (CFD_PERSIST_STEAL_US, default 50 us: a block takes ~40 us at 4096^2)
    const char *se = getenv("CFD_PERSIST_STEAL_US");
    const double st_us = se ? std::max(0.0, atof(se)) : 50.0;
    const uint32_t steal = (uint32_t)std::min(4.0e9, st_us * 100.0);
    // test knob: owners of tiles w % k == 1 start 2 ms late (CFD_PERSIST_LATE=k)
    const char *le = getenv("CFD_PERSIST_LATE");
    const int late = le ? std::max(0, atoi(le)) : 0;
    // the SUMS form (LdsMarch): reciprocal multiply, dx^2 == dy^2 with a
    // power-of-two reciprocal R >= 1 (h * R, v * R exact below overflow);
    // CFD_JACOBI_SUMS=0 keeps the reference's form everywhere
    const char *ue = getenv("CFD_JACOBI_SUMS");
    int exp2 = 0;
    const float R = g.r_dx_sq;
    const bool pow2 = R >= 1.0f && std::frexp(R, &exp2) == 0.5f;
    const int sums = !(ue && atoi(ue) == 0) && g.fastdiv == 1 && g.dx_sq == g.dy_sq &&
                     g.r_dx_sq == g.r_dy_sq && pow2;
    const float plim = sums ? std::ldexp(1.0f, 124) / R : 0.0f, rlim = std::ldexp(1.0f, 124);
#define CFD_LDS_PLAUNCH(FASTV)                                                                     \
    hipLaunchKernelGGL((k_jacobi_persist<T, FASTV>), grid, block, pad, s, g, pa, pb, f.rhs, f.ctl, \
                       f.persist, f.host_nonfinite ? f.host_nonfinite + 2 : nullptr, rs, epoch, pass, \
                       par0, nblk, out_lo, out_hi, nwc, nseg, wlo, whi, ngrp, acq, deadline, steal,  \
                       late, sums, plim, rlim)
    if (g.fastdiv == 1)
        CFD_LDS_PLAUNCH(1);
    else if (g.fastdiv == 2)
        CFD_LDS_PLAUNCH(2);
    else
        CFD_LDS_PLAUNCH(0);
#undef CFD_LDS_PLAUNCH
    return true;
}

}  // namespace

// per-translation-unit entry points (cfd_jacobi_lds*.hip)
void launch_lds_t567(const Geom &g, const Fields &f, int T, int pass, int par, int it, int out_lo,
                     int out_hi, uint32_t *rs, int mode, hipStream_t s, int lag);
void launch_lds_t8(const Geom &g, const Fields &f, int pass, int par, int it, int out_lo, int out_hi,
                   uint32_t *rs, int mode, hipStream_t s, int lag);
bool launch_lds_persist8(const Geom &g, const Fields &f, int pass, int par0, int nblk, int out_lo,
                         int out_hi, uint32_t epoch, uint32_t *rs, hipStream_t s);

}  // namespace cfd
