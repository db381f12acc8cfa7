// cfd_jacobi_chain.hip — kind 5's 8-sweep march with the four wave segments
// of a workgroup CHAINED (r5, model.rs:748-815 bit for bit).
//
// The per-launch march (cfd_jacobi_lds.h) gives every wave its own row
// segment.  Stage s of a segment needs stage s-1 of the rows on either side
// of it, so each wave also computes a "cone" of rows its neighbours own: T-s
// rows below its first row (warm-up) and T-1-s above its last (run-out), 56
// stage-rows per wave at T = 8 — 14 % of the work of a 51-row segment.
//
// Here a workgroup's four waves take four consecutive segments of one wave
// column and alternate direction (up, down, up, down), so every internal
// boundary is a MEETING of two marches at the same moment:
//   W0 up   [A, A+L0)          warm-up cone below A (the group's outer edge)
//   W1 down [A+L0, A+L0+D)     starts at its top, meeting W2's start
//   W2 up   [A+L0+D, A+L0+2D)  starts at its bottom, meeting W1's start
//   W3 down [A+L0+2D, B)       warm-up cone above B
// and W0/W1 (W2/W3) reach their shared boundary at the END of their marches.
// At a meeting the two waves hand each other the one boundary row each stage
// needs from the other side, through LDS, one row per slot for T-1 slots,
// instead of recomputing the other's rows: the workgroup keeps 2 of the 8
// half-cones (56 stage-rows instead of 224 per 4 segments, -9 % VALU work at
// 4096^2).  In virtual row numbers (v = the march's own order) every wave
// loads from row 0 and owns rows f..D (f = T after a warm-up, 1 after a
// meeting start); stage s computes row v - s at slot v:
//   start meeting: stage s runs from slot s+1 (its first row needs the
//     partner's stage s-1 value of the partner's first row, sent at slot s);
//   end meeting: stage s ends at slot D+s with row D, whose upper neighbour
//     is the partner's stage s-1 value of ITS last row (sent at slot D+s-1).
// Every wave of the group has the same slot count D+T+1.  A hand-off is one
// LDS row per (wave, meeting, stage) and a per-(wave, meeting) flag holding
// the last stage published: the producer never waits (every row has its own
// entry), the consumer polls the flag only when it needs the row, one slot
// after the partner produced it (workgroup barriers at every hand-off slot
// measured 5.88 vs 4.99 us per sweep: each forced the group's four SIMDs
// into lockstep).  Each value is the reference's: a stage reads exactly the
// neighbours the reference's sweep reads, computed by exactly the
// reference's expression.
//
// The first and last row group of every wave column (whose rows reach the
// global boundary rows, or are too few for a chain) run the per-launch march
// unchanged (lds_block with explicit rows).
//
// SUMS (optimistic, r5): chain groups run the form (h + v) * R (LdsMarch's
// SUMS, one packed multiply fewer per column pair and stage) and track max
// |p'| of every input row they load and max |rhs|; the group checks the
// bound that makes the form bitwise for every value its sweeps form (inputs
// below 2^124 / R, rhs below 2^124, drift T * 0.1875 * max|rhs| / R, the
// guard of k_jacobi_persist) and, where it fails, re-runs the group in the
// reference's form from the untouched source buffer (the destination rows it
// stored are rewritten; nothing reads them inside the launch).
#include "cfd_jacobi_lds.h"

namespace cfd {
namespace {

constexpr int kChainStages = 8;   // hand-off rows per (wave, meeting): stages 1..T-1, T <= 8

// CFD_CHAIN_STAMP (diagnostic builds only, tools/chain_stamps.py): every wave
// records s_memrealtime at its start, the end of its opening, the end of its
// steady slots, the end of its march and its exit, plus its HW_ID / XCC_ID,
// role and row group (vector stores into g_chain_stamp)
#ifndef CFD_CHAIN_STAMP
#define CFD_CHAIN_STAMP 0
#endif
#if CFD_CHAIN_STAMP
constexpr int kChainStampWaves = 1 << 15;
__device__ unsigned long long g_chain_stamp[kChainStampWaves * 8];
__device__ __forceinline__ unsigned long long chain_now() { return __builtin_amdgcn_s_memrealtime(); }
#endif

template <int T, int FAST, bool RES, bool SUMS, bool WARM, int E>
struct ChainMarch {
    static_assert(T <= kChainStages, "hand-off rows");
    static constexpr int NW = 3;
    static constexpr int PD = CFD_LDS_PD;
    static constexpr int DR = ring_depth(T, PD, 1);   // rhs ring rows (9 at T = 8)
    static constexpr int U = DR;                      // slot unroll
    static constexpr int H = (T + 1) / 2;             // halo lanes per side
    static constexpr int OUTL = 64 - 2 * H;
    static constexpr int kCol = 1;
    static constexpr int PLD_AUX = CFD_LDS_LD_AUX, PST_AUX = CFD_LDS_ST_AUX;
    // first slot of stage s; the opening runs slots [0, P0): through stage
    // T's first slot (after a meeting start, that slot still takes a hand-off)
    static constexpr int st0(int s) { return WARM ? 2 * s : s + 1; }
    static constexpr int P0 = st0(T) + (WARM ? 0 : 1);
    static_assert(DR % NW == 0 && DR % PD == 0 && DR >= T + 1, "ring geometry");

    f2 W[T][NW];   // W[s][v % NW]: stage s's row of slot v
    f2 PQ[PD], RQ[PD];
    f2 *ring;      // this wave's rhs ring (LDS)
    f2 *xb;        // the group's hand-off rows: [wave][meeting][stage][64 lanes]
    uint32_t *xf;  // [wave][meeting]: the last stage published
    int lane, wave, ps, pe;   // partner wave of the start / end meeting
    int Dd, S, abase, dir, ch, nch, vo_ld, vo_st, row_bytes, wbase, lo_clamp, hi_clamp, nyl_;
    bool e0, e1;
    float dx_sq, r_dx_sq, dy_sq, r_dy_sq, denom, r_denom;
    __amdgpu_buffer_rsrc_t rs_p, rs_r, rs_d;
    float m, imax, rmax;
    unsigned long long t_open = 0, t_steady = 0, t_march = 0;   // CFD_CHAIN_STAMP

    __device__ __forceinline__ int act(int vrow) const { return abase + dir * vrow; }

    template <int AUX = 0>
    __device__ __forceinline__ f2 ld(__amdgpu_buffer_rsrc_t rs, int vrow) const {
        vrow = vrow <= Dd + 1 ? vrow : Dd + 1;   // prefetch past the last input row
        int row = act(vrow);
        row = row < lo_clamp ? lo_clamp : (row > hi_clamp ? hi_clamp : row);
        const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, vo_ld, (row - wbase) * row_bytes, AUX);
        return (f2){__uint_as_float(v.x), __uint_as_float(v.y)};
    }
    __device__ __forceinline__ void st(const f2 &x, int row) const {
        const u32x2 v = {__float_as_uint(x.x), __float_as_uint(x.y)};
        __builtin_amdgcn_raw_buffer_store_b64(v, rs_d, vo_st, (row - wbase) * row_bytes, PST_AUX);
    }

    // model.rs:775-793 on the lane's column pair (LdsMarch::update)
    __device__ __forceinline__ f2 update(const f2 &B, const f2 &C, const f2 &Tp, const f2 &Rh) const {
        const float hx = C.y + from_left(C.y);
        const float hy = C.x + from_right(C.x);
        const f2 h = {hx, hy};
        const f2 v = Tp + B;
        f2 s;
        if constexpr (SUMS) {
            s = (h + v) * r_dx_sq;
        } else {
            const f2 hz = fdiv2<FAST>(h, dx_sq, r_dx_sq);
            const f2 vt = fdiv2<FAST>(v, dy_sq, r_dy_sq);
            s = hz + vt;
        }
        const f2 pu = fdiv2<FAST>(s - Rh, denom, r_denom);
        const float omega = 0.75f;
        const float om1 = 1.0f - omega;
        f2 o = omega * pu + om1 * C;
        if (E & kCol) {
            if (ch == 0) o.x = o.y;             // P(0,j) = P(1,j)
            if (ch == nch - 1) o.y = 0.0f;      // P(nx-1,j) = 0
        }
        return o;
    }

    // stage s's row for the partner: the row, then the flag (workgroup-scope
    // release: the row's LDS write has completed; no wait on global loads)
    __device__ __forceinline__ void send(const f2 &n, int ph, int s) const {
        xb[((wave * 2 + ph) * kChainStages + s) * 64 + lane] = n;
        __hip_atomic_store(&xf[wave * 2 + ph], (uint32_t)s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    // the partner's stage s row, once its flag says it is there (the partner
    // is in this workgroup and produces it without waiting on us; the poll is
    // bounded all the same)
    __device__ __forceinline__ f2 recv(int partner, int ph, int s) const {
#pragma unroll 1
        for (int k = 0; k < (1 << 22); ++k) {
            const uint32_t fl = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(&xf[partner * 2 + ph], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
            if ((int)fl >= s) break;
            __builtin_amdgcn_s_sleep(1);
        }
        return xb[((partner * 2 + ph) * kChainStages + s) * 64 + lane];
    }

    // Slot v (V_ == v mod U).  PH 0: the opening slots (V_ == v, compile-time
    // stage ramp and start hand-offs); 1: steady (every stage, no hand-off);
    // 3: steady, skipped past slot Dd (the remainder before the closing).
    template <int V_, int PH>
    __device__ __forceinline__ void slot(int v) {
        if (PH == 3 && v > Dd) return;
        const int k = v;
        W[0][V_ % NW] = PQ[V_ % PD];
        PQ[V_ % PD] = ld<PLD_AUX>(rs_p, k + PD);
        ring[(V_ % DR) * 64 + lane] = RQ[V_ % PD];
        RQ[V_ % PD] = ld(rs_r, k + PD);
        constexpr int kW = 4 * NW;
#pragma unroll
        for (int s = 1; s <= T; ++s) {
            if (PH == 0 && V_ < st0(s)) continue;   // compile-time
            if constexpr (PH == 0 && !WARM) {
                // the first row's lower neighbour: the partner's stage s-1
                // value of its own first row
                if (s >= 2 && V_ == st0(s)) W[s - 1][(V_ - 2 + kW) % NW] = recv(ps, 0, s - 1);
            }
            const f2 rh = ring[((V_ - s + 8 * DR) % DR) * 64 + lane];
            const f2 n = stage_at(s, W[s - 1][(V_ - 2 + kW) % NW], W[s - 1][(V_ - 1 + kW) % NW],
                                  W[s - 1][V_ % NW], rh, PH == 0 && V_ == st0(1));
            if (s < T)
                W[s][V_ % NW] = n;
            else
                store_row(n, W[s - 1][(V_ - 1 + kW) % NW], act(v - T));
            if constexpr (PH == 0 && !WARM) {
                if (s <= T - 1 && V_ == st0(s)) send(n, 0, s);
            }
        }
    }

    // stage s's update with the SUMS form's input tracking (stage 1 sees
    // every input row once as Tp, its first slot the first two as B and C)
    __device__ __forceinline__ f2 stage_at(int s, const f2 &B, const f2 &C, const f2 &Tp, const f2 &rh,
                                           bool first) {
        if constexpr (SUMS) {
            if (s == 1) {
                imax = fmaxf(fmaxf(imax, fabsf(Tp.x)), fabsf(Tp.y));
                rmax = fmaxf(fmaxf(rmax, fabsf(rh.x)), fabsf(rh.y));
                if (first)
                    imax = fmaxf(fmaxf(imax, fmaxf(fabsf(B.x), fabsf(B.y))),
                                 fmaxf(fabsf(C.x), fabsf(C.y)));
            }
        }
        return update(B, C, Tp, rh);
    }
    // stage T's row: the residual (RES) and the store
    __device__ __forceinline__ void store_row(const f2 &n, const f2 &C, int ra) {
        if (RES) {
            const f2 d = n - C;
            if (!(E & kCol)) {
                m = fmaxf(fmaxf(m, fabsf(d.x)), fabsf(d.y));
            } else {
                if (e0) m = fmaxf(m, fabsf(d.x));
                if (e1) m = fmaxf(m, fabsf(d.y));
            }
        }
        st(n, ra);
    }

    // The closing: slots Dd+1 .. Dd+T, compile-time.  Slot Dd+J runs stages
    // J..T; stage J makes row Dd (the last) from the partner's stage J-1 row
    // and hands its own on.  No loads: the last input row (Dd+1) was
    // prefetched, and every rhs row a closing stage reads is in the ring.
    // The register rings are first rotated so that slot Dd+1 sits at index 0
    // (a 3-way switch, once per wave); the LDS ring is addressed at run time.
    template <int R>
    __device__ __forceinline__ void rotate() {
        // new[i] = old[(i + R) % 3]
        if constexpr (R != 0) {
#pragma unroll
            for (int q = 0; q < T; ++q) {
                const f2 a0 = W[q][R % NW], a1 = W[q][(1 + R) % NW], a2 = W[q][(2 + R) % NW];
                W[q][0] = a0, W[q][1] = a1, W[q][2] = a2;
            }
            const f2 p0 = PQ[R % PD], p1 = PQ[(1 + R) % PD], p2 = PQ[(2 + R) % PD];
            PQ[0] = p0, PQ[1] = p1, PQ[2] = p2;
        }
    }
    template <int J>
    __device__ __forceinline__ void closing_slot(int r9) {
        // W index of slot Dd+J after the rotation: (J-1) % NW
        constexpr int I0 = (J - 1) % NW, Im1 = (J - 2 + NW) % NW, Im2 = (J - 3 + 2 * NW) % NW;
        if (J == 1) W[0][I0] = PQ[0];   // input row Dd+1
#pragma unroll
        for (int s = J; s <= T; ++s) {
            if (s >= 2 && s == J) W[s - 1][I0] = recv(pe, 1, s - 1);   // the last row's upper neighbour
            // rhs row Dd+J-s sits in ring slot (Dd+J-s) mod DR, r9 = (Dd+1) mod DR
            int q = r9 + J - 1 - s;   // in [r9 - T, r9 - 1]
            q = q < 0 ? q + DR : q;
            const f2 rh = ring[q * 64 + lane];
            const f2 n = stage_at(s, W[s - 1][Im2], W[s - 1][Im1], W[s - 1][I0], rh, false);
            if (s < T)
                W[s][I0] = n;
            else
                store_row(n, W[s - 1][Im1], act(Dd + J - T));
            if (s == J && s <= T - 1) send(n, 1, s);
        }
    }
    template <int J>
    __device__ __forceinline__ void closing(int r9) {
        if constexpr (J <= T) {
            closing_slot<J>(r9);
            closing<J + 1>(r9);
        }
    }
    __device__ __forceinline__ void close_march() {
        // slot Dd+1's register-ring index before the rotation
        const int phi = (Dd + 1) % NW;
        if (phi == 1)
            rotate<1>();
        else if (phi == 2)
            rotate<2>();
        closing<1>((Dd + 1) % DR);
    }

    template <int V_>
    __device__ __forceinline__ void opening() {
        if constexpr (V_ < P0) {
            slot<V_, 0>(V_);
            opening<V_ + 1>();
        }
    }
    template <int J, int PH>
    __device__ __forceinline__ void group(int base) {
        if constexpr (J < U) {
            slot<P0 + J, PH>(base + J);
            group<J + 1, PH>(base);
        }
    }
    // progress-ordered issue priority (LdsMarch::set_prio)
    __device__ __forceinline__ void set_prio(int done) const {
        if (!CFD_LDS_PRIO) return;
        const int rows = S - P0, d4 = 4 * done;
        if (d4 >= 3 * rows)
            __builtin_amdgcn_s_setprio(0);
        else if (d4 >= 2 * rows)
            __builtin_amdgcn_s_setprio(1);
        else if (d4 >= rows)
            __builtin_amdgcn_s_setprio(2);
        else
            __builtin_amdgcn_s_setprio(3);
    }
    __device__ __forceinline__ void run() {
        set_prio(0);
        opening<0>();
#if CFD_CHAIN_STAMP
        t_open = chain_now();
#endif
        int base = P0;
        for (; base + U <= Dd + 1; base += U) {   // every slot of the group <= Dd
            set_prio(base - P0);
            group<0, 1>(base);
        }
#if CFD_CHAIN_STAMP
        t_steady = chain_now();
#endif
        set_prio(base - P0);
        group<0, 3>(base);   // the steady slots left before the closing (< U)
        close_march();
#if CFD_CHAIN_STAMP
        t_march = chain_now();
#endif
    }
};

// A chain wave's march in form SUMS; returns its (wave-max) guard maxima.
template <int T, int FAST, bool RES, bool SUMS, bool WARM, int E>
__device__ __forceinline__ void chain_run(const Geom &g, float *src_alloc, float *dst_alloc,
                                          const float *rhs, f2 *lds, uint32_t *xflags, int wave, int lane,
                                          int wc, int Dd, int abase, int dir, int ps, int pe, float *im,
                                          float *rm, float *mres) {
    using M = ChainMarch<T, FAST, RES, SUMS, WARM, E>;
    M w;
    w.lane = lane;
    w.wave = wave;
    w.ps = ps;
    w.pe = pe;
    w.Dd = Dd;
    w.S = Dd + T + 1;
    w.abase = abase;
    w.dir = dir;
    w.ring = lds + wave * M::DR * 64;
    w.xb = lds + kLdsWaves * M::DR * 64;
    w.xf = xflags;
    const int nx = g.nx;
    w.nch = nx / 2;
    w.nyl_ = g.nyl;
    w.lo_clamp = -g.hg;
    w.hi_clamp = g.nyl + g.hg - 1;
    w.ch = wc * M::OUTL - M::H + lane;
    const bool in_dom = w.ch >= 0 && w.ch < w.nch;
    const bool out_lane = in_dom && lane >= M::H && lane < 64 - M::H;
    const int col = 2 * w.ch;
    w.row_bytes = nx * 4;
    constexpr int kFar = 0x7FFF0000;
    w.vo_ld = in_dom ? col * 4 : kFar;
    w.vo_st = out_lane ? col * 4 : kFar;
    // buffer window: every row the wave loads or stores, with a row of margin
    const int ra0 = w.act(0), ra1 = w.act(Dd + 1);
    const int wb = max(w.lo_clamp, min(ra0, ra1) - 1), wt = min(w.hi_clamp, max(ra0, ra1) + 1);
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
    w.e0 = out_lane && col >= 1 && col <= nx - 8;
    w.e1 = out_lane && col + 1 >= 1 && col + 1 <= nx - 8;
    w.m = w.imax = w.rmax = 0.0f;
    const f2 z = {0.0f, 0.0f};
#pragma unroll
    for (int s = 0; s < T; ++s)
#pragma unroll
        for (int q = 0; q < M::NW; ++q) w.W[s][q] = z;
#pragma unroll
    for (int q = 0; q < M::PD; ++q) {
        w.PQ[q] = w.template ld<M::PLD_AUX>(w.rs_p, q);
        w.RQ[q] = w.ld(w.rs_r, q);
    }
    w.run();
#if CFD_CHAIN_STAMP
    if (!RES && lane == 0 && (int)blockIdx.x * kLdsWaves + wave < kChainStampWaves) {
        unsigned long long *p = g_chain_stamp + ((size_t)blockIdx.x * kLdsWaves + wave) * 8;
        p[1] = w.t_open;
        p[2] = w.t_steady;
        p[3] = w.t_march;
    }
#endif
    *im = wave_max(in_dom ? w.imax : 0.0f);
    *rm = wave_max(in_dom ? w.rmax : 0.0f);
    *mres = wave_max(out_lane ? w.m : 0.0f);
}

template <int T, int FAST, bool RES, bool SUMS, int E>
__device__ __forceinline__ void chain_role(const Geom &g, float *src, float *dst, const float *rhs, f2 *lds,
                                           uint32_t *xflags, int wave, int lane, int wc, int Dd, int abase, int dir, int ps,
                                           int pe, float *im, float *rm, float *mres) {
    if (wave == 0 || wave == kLdsWaves - 1)
        chain_run<T, FAST, RES, SUMS, true, E>(g, src, dst, rhs, lds, xflags, wave, lane, wc, Dd, abase, dir, ps,
                                               pe, im, rm, mres);
    else
        chain_run<T, FAST, RES, SUMS, false, E>(g, src, dst, rhs, lds, xflags, wave, lane, wc, Dd, abase, dir, ps,
                                                pe, im, rm, mres);
}

template <int T, int FAST, bool RES, bool SUMS>
__device__ __forceinline__ void chain_form(const Geom &g, float *src, float *dst, const float *rhs, f2 *lds,
                                           uint32_t *xflags, int wave, int lane, int wc, bool col_edge, int Dd, int abase,
                                           int dir, int ps, int pe, float *im, float *rm, float *mres) {
    if (col_edge)
        chain_role<T, FAST, RES, SUMS, 1>(g, src, dst, rhs, lds, xflags, wave, lane, wc, Dd, abase, dir, ps, pe,
                                          im, rm, mres);
    else
        chain_role<T, FAST, RES, SUMS, 0>(g, src, dst, rhs, lds, xflags, wave, lane, wc, Dd, abase, dir, ps, pe,
                                          im, rm, mres);
}

// One launch of T = 8 sweeps over rows [out_lo, out_hi) (single domain):
// row group 0 and ngrp-1 of every wave column per launch as lds_block, the
// groups between as chains.  Group k (1..ngrp-2) has D = d0 + (k-1 < nhi),
// 4D + 2 - 2T rows; group 0 has elo rows, group ngrp-1 the rest.
template <int T, int FAST, int MODE>
__global__ __launch_bounds__(kLdsWaves * 64, 1) void k_jacobi_chain(
    Geom g, float *__restrict__ pa, float *__restrict__ pb, const float *__restrict__ rhs, Ctl *ctl,
    uint32_t *res_slots, int pass, int par, int out_lo, int out_hi, int nwc, int ngrp, int d0, int nhi,
    int elo, int wlo, int whi, int sums, float plim, float rlim, uint32_t *cstat) {
    using MC = ChainMarch<T, FAST, MODE == 1, false, false, 0>;
    constexpr bool RES = MODE == 1;
    // per wave: its rhs ring (DR rows), then every wave's hand-off rows
    // (2 meetings x kChainStages), then the hand-off flags
    __shared__ f2 lds[kLdsWaves * (MC::DR + 2 * kChainStages) * 64];
    __shared__ uint32_t xflags[2 * kLdsWaves];
    __shared__ float gm[2 * kLdsWaves];
    __shared__ int redo_s;
    if (pass_off(ctl, pass)) return;
#if CFD_CHAIN_STAMP
    struct StampOnExit {
        unsigned long long t0;
        int role;
        __device__ ~StampOnExit() {
            const int idx = (int)blockIdx.x * kLdsWaves + ((int)threadIdx.x >> 6);
            if (MODE == 0 && (threadIdx.x & 63) == 0 && idx < kChainStampWaves) {
                unsigned long long *p = g_chain_stamp + (size_t)idx * 8;
                const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));
                const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11));
                p[0] = t0;
                p[4] = chain_now();
                p[5] = ((unsigned long long)xcc << 32) | hw;
                p[6] = (unsigned long long)role;
            }
        }
    } stamp_guard{chain_now(), 0};
#endif
    const int bid = xcd_block(g);
    // diagnostics (cfd_get_chain_stats): chain launches, groups re-run in the
    // reference's form
    if (blockIdx.x == 0 && threadIdx.x == 0 && cstat) atomicAdd(cstat + 1, 1u);
    const int wc = bid % nwc, grp = bid / nwc;
    if (grp >= ngrp) return;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
#if CFD_CHAIN_STAMP
    // role: 0..3 chain waves, 4 edge group; the row group above it
    stamp_guard.role = ((grp == 0 || grp == ngrp - 1) ? 4 : wave) | (grp << 8);
#endif
    const int lane = (int)threadIdx.x & 63;
    const int M = ngrp - 2;
    const int r4_0 = 4 * d0 + 2 - 2 * T;   // rows of a chain group with D = d0
    // first row of group k (k >= 1)
    auto gstart = [&](int k) { return out_lo + elo + (k - 1) * r4_0 + 4 * min(k - 1, nhi); };
    if (grp == 0 || grp == ngrp - 1) {
        // an edge group: the per-launch march on explicit rows, split over the
        // four waves with the boundary-row segment lighter (launch_lds_t)
        const int a = grp == 0 ? out_lo : gstart(ngrp - 1);
        const int b = grp == 0 ? out_lo + elo : out_hi;
        const int w0 = grp == 0 ? wlo : 16, w3 = grp == 0 ? 16 : whi;
        const int tot = w0 + 32 + w3;
        auto cum = [&](int i) { return i <= 0 ? 0 : (i >= 4 ? tot : w0 + 16 * (i - 1)); };
        const int r0 = a + cum(wave) * (b - a) / tot, r1 = a + cum(wave + 1) * (b - a) / tot;
        if (r0 >= r1) return;
        lds_block<T, FAST, MODE>(g, pa, pb, rhs, ctl, res_slots, par, out_lo, out_hi, nwc, 4 * ngrp, wlo,
                                 whi, lds, 0, bid, 0, nullptr, nullptr, nullptr, nullptr, 0.0f, 0.0f, r0, r1);
        return;
    }
    (void)M;
    const int Dd = d0 + (grp - 1 < nhi ? 1 : 0);
    const int A = gstart(grp);
    const int L0 = Dd - T + 1;
    // the four roles (virtual row 0 = the first row each wave loads)
    int abase, dir, ps = 0, pe;
    if (wave == 0) {
        abase = A - T, dir = 1, pe = 1;
    } else if (wave == 1) {
        abase = A + L0 + Dd, dir = -1, ps = 2, pe = 0;
    } else if (wave == 2) {
        abase = A + L0 + Dd - 1, dir = 1, ps = 1, pe = 3;
    } else {
        abase = A + L0 + 2 * Dd + L0 - 1 + T, dir = -1, pe = 2;
    }
    const int si = (ctl->cur + par) & 1;   // buffers ping-pong once per launch
    float *src = si ? pb : pa, *dst = si ? pa : pb;
    constexpr int H = MC::H, OUTL = MC::OUTL;
    const int ch_lo = wc * OUTL - H, ch_hi = ch_lo + 63;
    const bool col_edge = ch_lo <= 0 || 2 * (ch_hi + 1) > g.nx - 8;
    float im = 0.0f, rm = 0.0f, mres = 0.0f;
    bool done = false;
    // the hand-off flags start at 0 (LDS is not cleared between workgroups)
    if (threadIdx.x < 2 * kLdsWaves) xflags[threadIdx.x] = 0u;
    __syncthreads();
    if (FAST == 1 && sums) {
        chain_form<T, FAST, RES, (FAST == 1)>(g, src, dst, rhs, lds, xflags, wave, lane, wc, col_edge, Dd, abase,
                                             dir, ps, pe, &im, &rm, &mres);
        if (lane == 0) {
            gm[wave] = im;
            gm[kLdsWaves + wave] = rm;
        }
        __syncthreads();
        float gi = 0.0f, gr = 0.0f;
#pragma unroll
        for (int q = 0; q < kLdsWaves; ++q) {
            gi = fmaxf(gi, gm[q]);
            gr = fmaxf(gr, gm[kLdsWaves + q]);
        }
        // bound on every value the group's T sweeps form: inputs + T drifts
        // of 0.1875 max|rhs| / R (dx^2 == 1 / R exactly under FAST == 1)
        const float drift = 0.1875f * (float)T * gr * g.dx_sq;
        done = gi < 0.5f * plim && gr < rlim && drift < 0.5f * plim;
        if (threadIdx.x == 0) redo_s = done ? 0 : 1;
        __syncthreads();
        done = redo_s == 0;
        if (!done) {
            if (threadIdx.x == 0 && cstat) atomicAdd(cstat + 2, 1u);
            if (threadIdx.x < 2 * kLdsWaves) xflags[threadIdx.x] = 0u;   // the re-run's hand-offs
            __syncthreads();
        }
    }
    if (!done)
        chain_form<T, FAST, RES, false>(g, src, dst, rhs, lds, xflags, wave, lane, wc, col_edge, Dd, abase, dir,
                                        ps, pe, &im, &rm, &mres);
    if (RES && lane == 0) publish_max(res_slots, bid * kLdsWaves + wave, mres);
}

// Workgroups of k_jacobi_chain<T, FAST, MODE> per CU with `pad` bytes of
// dynamic LDS (occupancy API, cached per pad value).
template <int T, int FAST, int MODE>
int chain_blocks_per_cu(int pad) {
    static int cache[2] = {0, 0};
    int &nb = cache[pad > 0 ? 1 : 0];
    if (nb == 0) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &n, reinterpret_cast<const void *>(&k_jacobi_chain<T, FAST, MODE>), kLdsWaves * 64, pad) !=
                hipSuccess ||
            n < 1)
            n = 1;
        nb = std::min(n, 6);
    }
    return nb;
}

}  // namespace

// The chain plan of one launch (host): row groups per wave column, the chain
// groups' D (d0, the first nhi of them d0 + 1) and the first edge group's
// rows.  false: no chain fits (too few rows), the caller runs launch_lds.
bool chain_plan(const Geom &g, int out_lo, int out_hi, int occ, int *nwc_o, int *ngrp_o, int *d0_o,
                int *nhi_o, int *elo_o) {
    constexpr int T = 8;
    using MC = ChainMarch<T, 1, false, false, false, 0>;
    const int nch = g.nx / 2;
    const int nwc = cdiv(nch, MC::OUTL);
    const int nrows = out_hi - out_lo;
    // one round of resident workgroups per launch (lds_segments)
    int ngrp = std::max(1, g.n_cu * occ / nwc);
    ngrp = std::min(ngrp, nrows / 32);
    for (; ngrp >= 3; --ngrp) {
        const int M = ngrp - 2;
        // chain group: 4D + 2 - 2T rows in D + T + 1 slots; edge group: 4 waves
        // of D + 1 - T rows in the same slots
        const long num = (long)nrows - (long)M * (2 - 2 * T) - 8L * (1 - T);
        const int d0 = (int)(num / (4L * ngrp));
        if (d0 < 2 * T - 1) continue;   // the opening and closing slots must not overlap
        const long mid = (long)M * (4L * d0 + 2 - 2 * T);
        const long rest = (long)nrows - mid - 8L * (d0 + 1 - T);
        int nhi = (int)std::max(0L, std::min((long)M, rest * M / (4L * ngrp)));
        const long etot = (long)nrows - mid - 4L * nhi;
        const int elo = (int)(etot / 2), ehi = (int)(etot - elo);
        // edge groups: >= 8 rows per wave, and the chain groups' cones never
        // reach a global boundary row (they carry no row patches)
        const int reach_lo = out_lo + elo - T - 1, reach_hi = out_hi - ehi + T;
        if (elo < 32 || ehi < 32 || reach_lo <= 1 - g.j0 || reach_hi >= g.ny - 2 - g.j0) continue;
        *nwc_o = nwc;
        *ngrp_o = ngrp;
        *d0_o = d0;
        *nhi_o = nhi;
        *elo_o = elo;
        return true;
    }
    return false;
}

namespace {
// workgroups per CU the chain launch's round is sized for
int chain_occ(const Geom &g, int mode) {
    constexpr int T = 8;
    // no occupancy pad: the kernel's own LDS (rhs rings + hand-off rows,
    // ~51 KB) and its ~130 VGPRs already hold it to 3 workgroups per CU
    const int pad = 0;
    (void)mode;
    int occ = 0;
#define CFD_CHAIN_OCC(FV, MV) occ = chain_blocks_per_cu<T, FV, MV>(pad)
    if (g.fastdiv == 1) {
        if (mode) CFD_CHAIN_OCC(1, 1); else CFD_CHAIN_OCC(1, 0);
    } else if (g.fastdiv == 2) {
        if (mode) CFD_CHAIN_OCC(2, 1); else CFD_CHAIN_OCC(2, 0);
    } else {
        if (mode) CFD_CHAIN_OCC(0, 1); else CFD_CHAIN_OCC(0, 0);
    }
#undef CFD_CHAIN_OCC
    return occ;
}
bool chain_geom_ok(const Geom &g) {
    // single domain only (a slab's bands reach into ghost rows); every
    // division form the per-launch march has
    return g.fastdiv >= 0 && g.fastdiv <= 2 && g.j0 == 0 && g.nyl == g.ny && g.tb_kind == 5;
}
}  // namespace

bool chain_applies(const Geom &g, int out_lo, int out_hi) {
    int nwc, ngrp, d0, nhi, elo;
    return chain_enabled() && chain_geom_ok(g) &&
           chain_plan(g, out_lo, out_hi, chain_occ(g, 0), &nwc, &ngrp, &d0, &nhi, &elo);
}

// k_jacobi_chain for an 8-sweep block (mode 0 / 1 = residual on the last
// stage); false: not applicable (the caller launches the per-launch march).
bool launch_lds_chain8(const Geom &g, const Fields &f, int pass, int par, int out_lo, int out_hi,
                       uint32_t *rs, hipStream_t s) {
    constexpr int T = 8;
    if (!chain_geom_ok(g)) return false;
    const int mode = rs ? 1 : 0;
    // no occupancy pad: the kernel's own LDS (rhs rings + hand-off rows,
    // ~51 KB) and its ~130 VGPRs already hold it to 3 workgroups per CU
    const int pad = 0;
    (void)mode;
    const int occ = chain_occ(g, mode);
    int nwc, ngrp, d0, nhi, elo;
    if (!chain_plan(g, out_lo, out_hi, occ, &nwc, &ngrp, &d0, &nhi, &elo)) return false;
    constexpr int kEdgeWeight = 11;
    const int reach = T + 2;
    const int wlo = out_lo - reach <= 1 - g.j0 ? kEdgeWeight : 16;
    const int whi = out_hi + reach >= g.ny - 2 - g.j0 ? kEdgeWeight : 16;
    // the optimistic SUMS form: reciprocal multiply, dx^2 == dy^2 with a
    // power-of-two reciprocal R >= 1 (CFD_JACOBI_SUMS=0: never)
    const char *se = getenv("CFD_JACOBI_SUMS");   // per launch: tests switch it
    const int sums_env = se ? atoi(se) : -1;
    int e2 = 0;
    const float R = g.r_dx_sq;
    const int sums = sums_env != 0 && g.fastdiv == 1 && g.dx_sq == g.dy_sq && g.r_dx_sq == g.r_dy_sq &&
                     R >= 1.0f && std::frexp(R, &e2) == 0.5f;
    const float plim = sums ? std::ldexp(1.0f, 124) / R : 0.0f, rlim = std::ldexp(1.0f, 124);
    const dim3 grid(nwc * ngrp), block(kLdsWaves * 64);
    float *pa = f.pp[0] - (long)g.hg * g.nx, *pb = f.pp[1] - (long)g.hg * g.nx;
#define CFD_CHAIN_LAUNCH(FV, MV)                                                                      \
    hipLaunchKernelGGL((k_jacobi_chain<T, FV, MV>), grid, block, pad, s, g, pa, pb, f.rhs, f.ctl, rs, \
                       pass, par, out_lo, out_hi, nwc, ngrp, d0, nhi, elo, wlo, whi, sums, plim, rlim, \
                       f.guard_slots ? f.guard_slots + (size_t)kGuardSets * kResSlots * kResStride : nullptr)
    if (g.fastdiv == 1) {
        if (mode) CFD_CHAIN_LAUNCH(1, 1); else CFD_CHAIN_LAUNCH(1, 0);
    } else if (g.fastdiv == 2) {
        if (mode) CFD_CHAIN_LAUNCH(2, 1); else CFD_CHAIN_LAUNCH(2, 0);
    } else {
        if (mode) CFD_CHAIN_LAUNCH(0, 1); else CFD_CHAIN_LAUNCH(0, 0);
    }
#undef CFD_CHAIN_LAUNCH
    return true;
}

#if CFD_CHAIN_STAMP
extern "C" int cfd_diag_chain_stamps(unsigned long long *host, int nwaves) {
    if (nwaves > kChainStampWaves) nwaves = kChainStampWaves;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_chain_stamp), (size_t)nwaves * 64, 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? nwaves : -1;
}
#endif

}  // namespace cfd
