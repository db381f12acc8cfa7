// cfd_jacobi_lds.hip — kind 5: the temporally blocked Jacobi march
// (model.rs:748-815, T sweeps per launch) with its rhs window in LDS.
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
#ifndef CFD_LDS_WPE
#define CFD_LDS_WPE 0  // > 0: minimum waves per SIMD for the register allocation
#endif
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int lds_gcd(int a, int b) { return b == 0 ? a : lds_gcd(b, a % b); }
// rhs ring depth: the smallest multiple of lcm(3, PD) that holds T+1 rows
constexpr int ring_depth(int T, int PD) {
    const int q = 3 / lds_gcd(3, PD) * PD;
    return ((T + 1 + q - 1) / q) * q;
}

template <int T, int FAST, bool RES>
struct LdsMarch {
    static constexpr int PD = CFD_LDS_PD;       // prefetch distance (slots) of p' and rhs
    static constexpr int D = ring_depth(T, PD); // rhs ring depth (rows); PD and 3 divide it
    static constexpr int U = D;                 // slot unroll: every ring index compile-time
    static constexpr int H = (T + 1) / 2;       // halo lanes per side (2 columns per lane)
    static constexpr int OUTL = 64 - 2 * H;     // lanes whose columns are stored
    static_assert(D % PD == 0 && D % 3 == 0 && D >= T + 1, "ring geometry");

    f2 W[T][3];
    f2 PQ[PD];
    f2 RQ[PD];
    float2 *ring;        // this wave's D x 64 slots (LDS)
    int lane;
    int k_first, S, lo_clamp, hi_clamp, nch, g_first, g_last, g_top, g_zero, row_bytes;
    int ch, vo_ld, vo_st, abase, dir;
    bool e0, e1;         // residual columns (EDGE waves)
    const Geom *g;       // the kernel argument: divisors and their reciprocals
    __amdgpu_buffer_rsrc_t rs_p, rs_r, rs_d;
    float m;

    __device__ __forceinline__ int act(int vrow) const { return abase + dir * vrow; }

    // Row `vrow` (virtual, march order) of p' or rhs.  Rows outside the
    // allocation lie beyond the global boundary and rows past the segment's
    // last input row are never needed: both are clamped to a row that exists
    // (their values only reach halo rows that the boundary patch overwrites).
    __device__ __forceinline__ f2 ld(__amdgpu_buffer_rsrc_t rs, int vrow) const {
        vrow = vrow < k_first + S ? vrow : k_first + S - 1;
        int row = act(vrow);
        row = row < lo_clamp ? lo_clamp : (row > hi_clamp ? hi_clamp : row);
        const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, vo_ld, (row - lo_clamp) * row_bytes, 0);
        return (f2){__uint_as_float(v.x), __uint_as_float(v.y)};
    }
    __device__ __forceinline__ void st(const f2 &x, int row) const {
        const u32x2 v = {__float_as_uint(x.x), __float_as_uint(x.y)};
        __builtin_amdgcn_raw_buffer_store_b64(v, rs_d, vo_st, (row - lo_clamp) * row_bytes, 0);
    }

    // One reference update (model.rs:775-793) of the lane's column pair.
    __device__ __forceinline__ f2 update(const f2 &B, const f2 &C, const f2 &Tp, const f2 &Rh) const {
        // horizontal: P(i+1) + P(i-1); the neighbour columns come from the
        // adjacent lanes (left lane's second column, right lane's first)
        const float hx = C.y + from_left(C.y);
        const float hy = C.x + from_right(C.x);
        const f2 h = {hx, hy};
        const f2 v = Tp + B;
        const f2 hz = fdiv2<FAST>(h, g->dx_sq, g->r_dx_sq);
        const f2 vt = fdiv2<FAST>(v, g->dy_sq, g->r_dy_sq);
        const f2 pu = fdiv2<FAST>(hz + vt - Rh, g->denom, g->r_denom);
        const float omega = 0.75f;
        const float om1 = 1.0f - omega;
        return omega * pu + om1 * C;
    }

    template <bool EDGE>
    __device__ __forceinline__ f2 stage(const f2 &B, const f2 &C, const f2 &Tp, const f2 &Rh) const {
        f2 o = update(B, C, Tp, Rh);
        if (EDGE) {
            if (ch == 0) o.x = o.y;             // P(0,j) = P(1,j)
            if (ch == nch - 1) o.y = 0.0f;      // P(nx-1,j) = 0
        }
        return o;
    }

    // Slot v (k = k_first + v), V_ == v (mod U).  GUARD 0: warm-up (V_ == v,
    // stage s runs from slot 2s on); GUARD 2: the final partial group.
    template <int V_, int GUARD, bool EDGE>
    __device__ __forceinline__ void slot(int v) {
        if (GUARD == 2 && v >= S) return;
        if (CFD_LDS_SB >= 1) __builtin_amdgcn_sched_barrier(0);
        const int k = k_first + v;
        W[0][V_ % 3] = PQ[V_ % PD];                                  // input row k
        PQ[V_ % PD] = ld(rs_p, k + PD);
        ring[(V_ % D) * 64 + lane] = make_float2(RQ[V_ % PD].x, RQ[V_ % PD].y);   // rhs row k
        RQ[V_ % PD] = ld(rs_r, k + PD);
#pragma unroll
        for (int s = 1; s <= T; ++s) {
            if (GUARD == 0 && V_ < 2 * s) continue;                  // compile-time
            if (CFD_LDS_SB >= 2 && s > 1) __builtin_amdgcn_sched_barrier(0);
            const int r = k - s;
            const float2 rh = ring[((V_ - s + 8 * D) % D) * 64 + lane];
            const f2 &B = W[s - 1][(V_ + 1) % 3];                    // stage s-1, row r-1
            const f2 &C = W[s - 1][(V_ + 2) % 3];                    //            row r
            const f2 &Tp = W[s - 1][V_ % 3];                         //            row r+1
            f2 n = stage<EDGE>(B, C, Tp, (f2){rh.x, rh.y});
            if (s < T) {
                if (EDGE && r == g_top) n = W[s][(V_ + 2) % 3];      // P(i,ny-1) = P(i,ny-2)
                W[s][V_ % 3] = n;
                if (EDGE && r == g_first) W[s][(V_ + 2) % 3] = n;    // P(i,0) = P(i,1)
            } else {
                const int ra = act(r);
                if (RES && ra >= 0 && ra < nyl_) {
                    const f2 d = n - C;
                    if (!EDGE) {
                        m = fmaxf(fmaxf(m, fabsf(d.x)), fabsf(d.y));
                    } else {
                        if (e0) m = fmaxf(m, fabsf(d.x));
                        if (e1) m = fmaxf(m, fabsf(d.y));
                    }
                }
                st(n, ra);
                if (EDGE && r == g_first) st(n, g_zero);
                if (EDGE && r == g_last) st(n, g_top);
            }
        }
    }
    int nyl_;

    template <int V_, bool EDGE>
    __device__ __forceinline__ void warmup() {
        if constexpr (V_ < 2 * T) {
            slot<V_, 0, EDGE>(V_);
            warmup<V_ + 1, EDGE>();
        }
    }

    template <int J, int GUARD, bool EDGE>
    __device__ __forceinline__ void group(int base) {
        if constexpr (J < U) {
            slot<2 * T + J, GUARD, EDGE>(base + J);
            group<J + 1, GUARD, EDGE>(base);
        }
    }

    template <bool EDGE>
    __device__ __forceinline__ void run() {
        warmup<0, EDGE>();
        int base = 2 * T;
        const int full_end = 2 * T + ((S - 2 * T) / U) * U;
        for (; base < full_end; base += U) group<0, 1, EDGE>(base);
        if (base < S) group<0, 2, EDGE>(base);
    }
};

#if CFD_LDS_WPE > 0
#define CFD_LDS_BOUNDS __launch_bounds__(kLdsWaves * 64, CFD_LDS_WPE)
#else
#define CFD_LDS_BOUNDS __launch_bounds__(kLdsWaves * 64)
#endif
template <int T, int FAST, bool RES>
__global__ CFD_LDS_BOUNDS void k_jacobi_lds(
    Geom g, float *__restrict__ pa, float *__restrict__ pb, const float *__restrict__ rhs,
    Ctl *ctl, uint32_t *res_slots, int pass, int par, int out_lo, int out_hi, int nwc, int nseg) {
    using M = LdsMarch<T, FAST, RES>;
    __shared__ float2 lds[kLdsWaves * M::D * 64];
    if (pass_off(ctl, pass)) return;
    M w;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int lane = (int)threadIdx.x & 63;
    const int bid = xcd_block(g);
    const int wc = bid % nwc;
    const int seg = (bid / nwc) * kLdsWaves + wave;
    const int nrows = out_hi - out_lo;
    if (seg >= nseg) return;
    const int r0 = out_lo + (int)(((long)seg * nrows) / nseg);
    const int r1 = out_lo + (int)(((long)(seg + 1) * nrows) / nseg);
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
    const int pbytes = (g.nyl + 2 * g.hg) * nx * 4;
    w.rs_p = __builtin_amdgcn_make_buffer_rsrc(src_alloc, 0, pbytes, 0x00020000);
    w.rs_d = __builtin_amdgcn_make_buffer_rsrc(dst_alloc, 0, pbytes, 0x00020000);
    w.rs_r = __builtin_amdgcn_make_buffer_rsrc((void *)(rhs - (long)g.hg * nx), 0, pbytes,
                                               0x00020000);
    w.g = &g;
    // residual columns 1..=nx-8 (the reference's full 8-lane chunks, Q6)
    w.e0 = out_lane && col >= 1 && col <= nx - 8;
    w.e1 = out_lane && col + 1 >= 1 && col + 1 <= nx - 8;
    w.g_first = 1 - g.j0;
    w.g_last = g.ny - 2 - g.j0;
    w.g_top = g.ny - 1 - g.j0;
    w.g_zero = -g.j0;
    w.m = 0.0f;
    w.k_first = r0 - T;
    w.S = (r1 - r0) + 2 * T;
    w.abase = 0;
    w.dir = 1;
    const f2 z = {0.0f, 0.0f};
#pragma unroll
    for (int s = 0; s < T; ++s) w.W[s][0] = w.W[s][1] = w.W[s][2] = z;
    // EDGE waves: a lane stores column 0 or a column outside the residual
    // range, or a stage touches a global boundary row; interior waves skip
    // all boundary logic
    const int ch_lo = wc * M::OUTL - M::H, ch_hi = ch_lo + 63;
    const bool col_edge = ch_lo <= 0 || 2 * (ch_hi + 1) > nx - 8;
    const int lo_row = w.k_first - 2, hi_row = r1 + T + 2;
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
        w.PQ[q] = w.ld(w.rs_p, w.k_first + q);
        w.RQ[q] = w.ld(w.rs_r, w.k_first + q);
    }
    if (edge)
        w.template run<true>();
    else
        w.template run<false>();
    if (!RES) return;
    const float m = wave_max(out_lane ? w.m : 0.0f);
    if (lane == 0) publish_max(res_slots, bid * kLdsWaves + wave, m);
}

template <int T, bool RES>
void launch_lds_t(const Geom &g, const Fields &f, int pass, int par, int out_lo, int out_hi,
                  uint32_t *rs, hipStream_t s) {
    const int nch = g.nx / 2;
    const int nwc = cdiv(nch, LdsMarch<T, 1, RES>::OUTL);
    const int rows = g.tb_rows > 0 ? g.tb_rows : 24;
    const int nseg = cdiv(out_hi - out_lo, rows);
    const dim3 grid(nwc * cdiv(nseg, kLdsWaves)), block(kLdsWaves * 64);
    float *pa = f.pp[0] - (long)g.hg * g.nx, *pb = f.pp[1] - (long)g.hg * g.nx;
#define CFD_LDS_LAUNCH(FASTV)                                                                      \
    hipLaunchKernelGGL((k_jacobi_lds<T, FASTV, RES>), grid, block, 0, s, g, pa, pb, f.rhs, f.ctl, \
                       rs, pass, par, out_lo, out_hi, nwc, nseg)
    if (g.fastdiv == 1)
        CFD_LDS_LAUNCH(1);
    else if (g.fastdiv == 2)
        CFD_LDS_LAUNCH(2);
    else
        CFD_LDS_LAUNCH(0);
#undef CFD_LDS_LAUNCH
}

template <bool RES>
void launch_lds_res(const Geom &g, const Fields &f, int T, int pass, int par, int out_lo,
                    int out_hi, uint32_t *rs, hipStream_t s) {
    switch (T) {
    case 1: launch_lds_t<1, RES>(g, f, pass, par, out_lo, out_hi, rs, s); break;
    case 2: launch_lds_t<2, RES>(g, f, pass, par, out_lo, out_hi, rs, s); break;
    case 3: launch_lds_t<3, RES>(g, f, pass, par, out_lo, out_hi, rs, s); break;
    case 4: launch_lds_t<4, RES>(g, f, pass, par, out_lo, out_hi, rs, s); break;
    case 5: launch_lds_t<5, RES>(g, f, pass, par, out_lo, out_hi, rs, s); break;
    case 6: launch_lds_t<6, RES>(g, f, pass, par, out_lo, out_hi, rs, s); break;
    case 7: launch_lds_t<7, RES>(g, f, pass, par, out_lo, out_hi, rs, s); break;
    default: launch_lds_t<8, RES>(g, f, pass, par, out_lo, out_hi, rs, s); break;
    }
}

}  // namespace

void launch_lds(const Geom &g, const Fields &f, int T, int pass, int it, int par, int out_lo,
                int out_hi, uint32_t *rs, hipStream_t s) {
    (void)it;
    if (rs)
        launch_lds_res<true>(g, f, T, pass, par, out_lo, out_hi, rs, s);
    else
        launch_lds_res<false>(g, f, T, pass, par, out_lo, out_hi, rs, s);
}

}  // namespace cfd
