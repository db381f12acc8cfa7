// cfd_jacobi_pipe.h — the prefetch-pipelined temporally blocked Jacobi march
// (kinds 3 and 4), generic in the columns per lane (VEC 4: float4 chunks,
// VEC 2: float2 chunks), instantiated by cfd_jacobi_pipe4.hip / _pipe2.hip.
//
// T weighted-Jacobi sweeps (model.rs:748-815) per launch.  A wave owns 64
// lanes x VEC columns of a row segment and marches up (or down) it; stage s
// (1..T) of slot k computes row k-s from stage s-1's rows k-s-1..k-s+1, so
// every stage is one sweep of the reference and p'/rhs come from HBM once per
// launch.  Edge values go stale one column per sweep from the wave's sides
// inward, so H = ceil(T/VEC) halo lanes on each side are computed but not
// stored.  Every HBM load is issued PD slots before its first use:
//   PQ[v % PD]   p' input row k_first+v, loaded PD slots ahead
//   W[s][v % 3]  newest row of stage s (stage 0 = input)
//   RH[q % NR]   rhs row k_first+q; stage s at slot v reads q = v-s, the load
//                at slot v fetches q = v-1+PD (NR = T+PD rows live)
// and the slot loop is unrolled by U = lcm(3, PD, NR), so every ring index is
// a compile-time constant.  Row offsets travel in the scalar soffset of the
// buffer instructions; the per-lane voffset is fixed (out of range for lanes
// that must not load or store), so no memory operation needs an exec mask.
#pragma once
#include "cfd_device.h"

namespace cfd {
namespace {

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int cgcd(int a, int b) { return b == 0 ? a : cgcd(b, a % b); }
constexpr int clcm(int a, int b) { return a / cgcd(a, b) * b; }
constexpr int kFarOffset = 0x7FFF0000;   // voffset of a lane that must not touch memory

// cache-policy bits of the march's buffer instructions (gfx950 CPol: 1 SC0,
// 2 NT, 16 SC1): p' input loads, rhs loads, p'_new stores
#ifndef CFD_CPOL_PLD
#define CFD_CPOL_PLD 0
#endif
#ifndef CFD_CPOL_RLD
#define CFD_CPOL_RLD 0
#endif
#ifndef CFD_CPOL_ST
#define CFD_CPOL_ST 0
#endif
// CFD_TRIM 1: skip the prefetches past the segment's last input row (they
// would fetch rows the neighbouring segment owns); CFD_PIPE_WAVES: waves per
// workgroup; CFD_PD4: prefetch distance at T = 4
#ifndef CFD_TRIM
#define CFD_TRIM 1
#endif
#ifndef CFD_PIPE_WAVES
#define CFD_PIPE_WAVES kJacWavesPerBlock
#endif
#ifndef CFD_PD4
#define CFD_PD4 2
#endif
#ifndef CFD_PD8
#define CFD_PD8 4
#endif
// CFD_PIPE_WPE > 0: minimum waves per SIMD the register allocation must allow
#ifndef CFD_PIPE_WPE
#define CFD_PIPE_WPE 0
#endif
// CFD_FORCE_EDGE 1 (diagnostic): every wave takes the boundary-condition path
#ifndef CFD_FORCE_EDGE
#define CFD_FORCE_EDGE 0
#endif
constexpr int kPipeWaves = CFD_PIPE_WAVES;

// prefetch distance per T: deep enough to cover HBM latency with a short
// unroll period U = lcm(3, PD, T+PD)
template <int T> struct PipeDepth { static constexpr int PD = 4; };   // T 2: U 12
template <> struct PipeDepth<8> { static constexpr int PD = CFD_PD8; };  // PD 4: U 12
template <> struct PipeDepth<1> { static constexpr int PD = 2; };     // U 6
template <> struct PipeDepth<3> { static constexpr int PD = 3; };     // U 6
template <> struct PipeDepth<4> { static constexpr int PD = CFD_PD4; };  // PD 2: U 6
template <> struct PipeDepth<5> { static constexpr int PD = 3; };     // U 24
template <> struct PipeDepth<6> { static constexpr int PD = 3; };     // U 9
template <> struct PipeDepth<7> { static constexpr int PD = 2; };     // U 18

// One reference Jacobi update (model.rs:775-793) of the 2 consecutive columns
// a lane holds: horizontal sums as swap(C) + (L, R), the swap folded into the
// packed add's op_sel; otherwise as jacobi_row4.
template <int FAST>
__device__ __forceinline__ float2 jacobi_row2(const float2 &B, const float2 &C, const float2 &T,
                                              const float2 &Rh, float L, float R, float dx_sq,
                                              float dy_sq, float denom, float r_dx_sq,
                                              float r_dy_sq, float r_denom) {
    const f2 c = {C.x, C.y};
    const f2 h = __builtin_shufflevector(c, c, 1, 0) + (f2){L, R};
    const f2 v = (f2){T.x, T.y} + (f2){B.x, B.y};
    const f2 hz = fdiv2<FAST>(h, dx_sq, r_dx_sq);
    const f2 vt = fdiv2<FAST>(v, dy_sq, r_dy_sq);
    const f2 pu = fdiv2<FAST>(hz + vt - (f2){Rh.x, Rh.y}, denom, r_denom);
    const float omega = 0.75f;
    const float om1 = 1.0f - omega;
    const f2 n = omega * pu + om1 * c;
    return make_float2(n.x, n.y);
}

template <int VEC> struct Lane;

template <> struct Lane<4> {
    using V = float4;
    template <int CP>
    static __device__ __forceinline__ V load(__amdgpu_buffer_rsrc_t rs, int vo, int so) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, so, CP);
        return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                           __uint_as_float(v.w));
    }
    static __device__ __forceinline__ void store(const V &x, __amdgpu_buffer_rsrc_t rs, int vo,
                                                 int so) {
        const u32x4 v = {__float_as_uint(x.x), __float_as_uint(x.y), __float_as_uint(x.z),
                         __float_as_uint(x.w)};
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, vo, so, CFD_CPOL_ST);
    }
    template <int FAST>
    static __device__ __forceinline__ V row(const V &B, const V &C, const V &T, const V &Rh,
                                            float dx_sq, float dy_sq, float denom, float r_dx_sq,
                                            float r_dy_sq, float r_denom) {
        return jacobi_row4<FAST>(B, C, T, Rh, from_left(C.w), from_right(C.x), dx_sq, dy_sq,
                                 denom, r_dx_sq, r_dy_sq, r_denom);
    }
    // P(0,j) = P(1,j) / P(nx-1,j) = 0 on the lane holding column 0 / nx-1
    static __device__ __forceinline__ void bc_first(V &o) { o.x = o.y; }
    static __device__ __forceinline__ void bc_last(V &o) { o.w = 0.0f; }
    static __device__ __forceinline__ float absdiff_max(float m, const V &n, const V &c) {
        return fmaxf(fmaxf(fmaxf(fmaxf(m, fabsf(n.x - c.x)), fabsf(n.y - c.y)), fabsf(n.z - c.z)),
                     fabsf(n.w - c.w));
    }
    static __device__ __forceinline__ float absdiff_max_masked(float m, const V &n, const V &c,
                                                               const bool *e) {
        if (e[0]) m = fmaxf(m, fabsf(n.x - c.x));
        if (e[1]) m = fmaxf(m, fabsf(n.y - c.y));
        if (e[2]) m = fmaxf(m, fabsf(n.z - c.z));
        if (e[3]) m = fmaxf(m, fabsf(n.w - c.w));
        return m;
    }
    static __device__ __forceinline__ V zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
};

template <> struct Lane<2> {
    using V = float2;
    template <int CP>
    static __device__ __forceinline__ V load(__amdgpu_buffer_rsrc_t rs, int vo, int so) {
        const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, vo, so, CP);
        return make_float2(__uint_as_float(v.x), __uint_as_float(v.y));
    }
    static __device__ __forceinline__ void store(const V &x, __amdgpu_buffer_rsrc_t rs, int vo,
                                                 int so) {
        const u32x2 v = {__float_as_uint(x.x), __float_as_uint(x.y)};
        __builtin_amdgcn_raw_buffer_store_b64(v, rs, vo, so, CFD_CPOL_ST);
    }
    template <int FAST>
    static __device__ __forceinline__ V row(const V &B, const V &C, const V &T, const V &Rh,
                                            float dx_sq, float dy_sq, float denom, float r_dx_sq,
                                            float r_dy_sq, float r_denom) {
        return jacobi_row2<FAST>(B, C, T, Rh, from_left(C.y), from_right(C.x), dx_sq, dy_sq,
                                 denom, r_dx_sq, r_dy_sq, r_denom);
    }
    static __device__ __forceinline__ void bc_first(V &o) { o.x = o.y; }
    static __device__ __forceinline__ void bc_last(V &o) { o.y = 0.0f; }
    static __device__ __forceinline__ float absdiff_max(float m, const V &n, const V &c) {
        return fmaxf(fmaxf(m, fabsf(n.x - c.x)), fabsf(n.y - c.y));
    }
    static __device__ __forceinline__ float absdiff_max_masked(float m, const V &n, const V &c,
                                                               const bool *e) {
        if (e[0]) m = fmaxf(m, fabsf(n.x - c.x));
        if (e[1]) m = fmaxf(m, fabsf(n.y - c.y));
        return m;
    }
    static __device__ __forceinline__ V zero() { return make_float2(0.f, 0.f); }
};

template <int T, int FAST, int VEC>
struct Pipe {
    using L = Lane<VEC>;
    using V = typename L::V;
    static constexpr int PD = PipeDepth<T>::PD;
    static constexpr int NR = T + PD;
    static constexpr int U = clcm(clcm(3, PD), NR);
    static constexpr int H = (T + VEC - 1) / VEC;
    static constexpr int OUTL = 64 - 2 * H;
    V W[T][3];
    V RH[NR];
    V PQ[PD];
    int k_first, S, nyl, nch, hg, g_first, g_last, g_top, g_zero, row_bytes;
    int ch, vo_ld, vo_st;
    int abase, dir;      // actual row = abase + dir * virtual row (dir -1: downward march)
    bool e[VEC];
    float dx_sq, dy_sq, denom, r_dx_sq, r_dy_sq, r_denom;
    __amdgpu_buffer_rsrc_t rs_p, rs_r, rs_d, rs_null;
    float m;

    __device__ __forceinline__ int act(int row) const { return abase + dir * row; }

    template <int CP>
    __device__ __forceinline__ V ld(__amdgpu_buffer_rsrc_t rs, int vrow) const {
        const int row = act(vrow);
        // uniform: scalar descriptor select
        const bool ok = row >= -hg && row < nyl + hg && (!CFD_TRIM || vrow < k_first + S);
        return L::template load<CP>(ok ? rs : rs_null, vo_ld, ok ? (row + hg) * row_bytes : 0);
    }
    __device__ __forceinline__ void st(const V &x, int row) const {
        L::store(x, rs_d, vo_st, (row + hg) * row_bytes);
    }

    template <bool EDGE>
    __device__ __forceinline__ V stage(const V &B, const V &C, const V &Tp, const V &Rh) const {
        V o = L::template row<FAST>(B, C, Tp, Rh, dx_sq, dy_sq, denom, r_dx_sq, r_dy_sq, r_denom);
        if (EDGE) {
            if (ch == 0) L::bc_first(o);
            if (ch == nch - 1) L::bc_last(o);
        }
        return o;
    }

    // Slot v (k = k_first + v).  V_ == v (mod U) fixes every ring index; in the
    // warm-up (GUARD 0) V_ == v and stage s only runs from slot 2s on; GUARD 2
    // is the final partial group (slots past the segment end return).
    template <int V_, int GUARD, bool EDGE>
    __device__ __forceinline__ void slot(int v) {
        if (GUARD == 2 && v >= S) return;
        const int k = k_first + v;
        W[0][V_ % 3] = PQ[V_ % PD];                             // input row k
        PQ[V_ % PD] = ld<CFD_CPOL_PLD>(rs_p, k + PD);
#pragma unroll
        for (int s = 1; s <= T; ++s) {
            if (GUARD == 0 && V_ < 2 * s) continue;              // compile-time
            const int r = k - s;
            const V &B = W[s - 1][(V_ + 1) % 3];                 // stage s-1, row r-1
            const V &C = W[s - 1][(V_ + 2) % 3];                 //              row r
            const V &Tp = W[s - 1][V_ % 3];                      //              row r+1
            V n = stage<EDGE>(B, C, Tp, RH[(V_ - s + NR * 8) % NR]);
            if (s < T) {
                if (EDGE && r == g_top) n = W[s][(V_ + 2) % 3];  // P(i,ny-1) = P(i,ny-2)
                W[s][V_ % 3] = n;
                if (EDGE && r == g_first) W[s][(V_ + 2) % 3] = n;   // P(i,0) = P(i,1)
            } else {
                const int ra = act(r);
                if (ra < nyl && ra >= 0)
                    m = EDGE ? L::absdiff_max_masked(m, n, C, e) : L::absdiff_max(m, n, C);
                st(n, ra);
                if (EDGE && r == g_first) st(n, g_zero);
                if (EDGE && r == g_last) st(n, g_top);
            }
        }
        RH[(V_ - 1 + PD + NR) % NR] = ld<CFD_CPOL_RLD>(rs_r, k - 1 + PD);     // rhs row k-1+PD
    }

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

#if CFD_PIPE_WPE > 0
#define CFD_PIPE_BOUNDS __launch_bounds__(kPipeWaves * 64, CFD_PIPE_WPE)
#else
#define CFD_PIPE_BOUNDS __launch_bounds__(kPipeWaves * 64)
#endif
template <int T, int FAST, int VEC>
__global__ CFD_PIPE_BOUNDS void k_jacobi_pipe(
    Geom g, float *__restrict__ pa, float *__restrict__ pb, const float *__restrict__ rhs,
    Ctl *ctl, uint32_t *res_slots, int pass, int it, int par, int out_lo, int out_hi, int nwc,
    int nseg) {
    if (pass_off(ctl, pass)) return;
    using Wv = Pipe<T, FAST, VEC>;
    using L = typename Wv::L;
    Wv w;
    // the wave index is uniform; readfirstlane lets the compiler see it, so
    // every row/slot condition below is a scalar branch
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int lane = (int)threadIdx.x & 63;
    const int bid = xcd_block(g);
    const int wc = bid % nwc;
    const int seg = (bid / nwc) * kPipeWaves + wave;
    const int nrows = out_hi - out_lo;
    if (seg >= nseg) return;
    // balanced segments: nseg row ranges differing by at most one row
    const int r0 = out_lo + (int)(((long)seg * nrows) / nseg);
    const int r1 = out_lo + (int)(((long)(seg + 1) * nrows) / nseg);
    if (r0 >= r1) return;
    const int nx = g.nx;
    w.nch = nx / VEC;
    w.hg = g.hg;
    w.nyl = g.nyl;
    w.ch = wc * Wv::OUTL - Wv::H + lane;
    const bool in_dom = w.ch >= 0 && w.ch < w.nch;
    const bool out_lane = in_dom && lane >= Wv::H && lane < 64 - Wv::H;
    const int col = VEC * w.ch;
    w.row_bytes = nx * 4;
    w.vo_ld = in_dom ? col * 4 : kFarOffset;
    w.vo_st = out_lane ? col * 4 : kFarOffset;
    // buffers ping-pong once per LAUNCH: par = launches since the solve began
    const int si = (ctl->cur + par) & 1;
    float *src_alloc = si ? pb : pa;
    float *dst_alloc = si ? pa : pb;
    const int pbytes = (w.nyl + 2 * w.hg) * nx * 4;
    w.rs_p = __builtin_amdgcn_make_buffer_rsrc(src_alloc, 0, pbytes, 0x00020000);
    w.rs_d = __builtin_amdgcn_make_buffer_rsrc(dst_alloc, 0, pbytes, 0x00020000);
    w.rs_r = __builtin_amdgcn_make_buffer_rsrc((void *)(rhs - (long)w.hg * nx), 0, pbytes,
                                               0x00020000);
    w.rs_null = __builtin_amdgcn_make_buffer_rsrc(src_alloc, 0, 0, 0x00020000);
    w.dx_sq = g.dx_sq;
    w.dy_sq = g.dy_sq;
    w.denom = g.denom;
    w.r_dx_sq = g.r_dx_sq;
    w.r_dy_sq = g.r_dy_sq;
    w.r_denom = g.r_denom;
    // residual columns 1..=nx-8 (the reference's full 8-lane chunks, Q2)
#pragma unroll
    for (int q = 0; q < VEC; ++q) w.e[q] = out_lane && col + q >= 1 && col + q <= nx - 8;
    w.g_first = 1 - g.j0;
    w.g_last = g.ny - 2 - g.j0;
    w.g_top = g.ny - 1 - g.j0;
    w.g_zero = -g.j0;
    w.m = 0.0f;
    w.k_first = r0 - T;
    w.S = (r1 - r0) + 2 * T;
    w.abase = 0;
    w.dir = 1;
    const typename Wv::V z = L::zero();
#pragma unroll
    for (int s = 0; s < T; ++s) w.W[s][0] = w.W[s][1] = w.W[s][2] = z;
    // EDGE waves: a lane of theirs stores column 0 or a column whose residual
    // is not counted (chunks nch-2.. for VEC 4), or a stage touches a global
    // boundary row; interior waves skip all boundary logic
    const int ch_lo = wc * Wv::OUTL - Wv::H, ch_hi = ch_lo + 63;
    const bool col_edge = ch_lo <= 0 || VEC * (ch_hi + 1) > nx - 8;
    // every row any stage touches, in either march direction (one spare each side)
    const int lo_row = w.k_first - 2, hi_row = r1 + T + 2;
    auto hits = [&](int r) { return r >= lo_row && r <= hi_row; };
    const bool row_edge = hits(w.g_zero) || hits(w.g_first) || hits(w.g_last) || hits(w.g_top);
    const bool edge = CFD_FORCE_EDGE || col_edge || row_edge;
    // Interior segments alternate their march direction (odd ones run downward
    // through the mirrored row space — the stencil is symmetric and f32
    // addition commutative, so the bits are the same): neighbouring segments
    // then read the rows they share at the same time, from L2, instead of one
    // at its start and the other at its end.
    if (!edge && (seg & 1)) {
        w.abase = r0 + r1 - 1;
        w.dir = -1;
    }
    // prologue: p' rows k_first .. k_first+PD-1, rhs rows k_first .. k_first+PD-2
#pragma unroll
    for (int q = 0; q < Wv::PD; ++q) w.PQ[q] = w.template ld<CFD_CPOL_PLD>(w.rs_p, w.k_first + q);
#pragma unroll
    for (int q = 0; q < Wv::NR; ++q) w.RH[q] = q < Wv::PD - 1 ? w.template ld<CFD_CPOL_RLD>(w.rs_r, w.k_first + q) : z;
    if (edge)
        w.template run<true>();
    else
        w.template run<false>();
    if (!res_slots) return;
    const float m = wave_max(out_lane ? w.m : 0.0f);
    if (lane == 0) publish_max(res_slots, bid * kPipeWaves + wave, m);
}

template <int VEC, int T>
void launch_pipe_t(const Geom &g, const Fields &f, int pass, int it, int par, int out_lo,
                   int out_hi, uint32_t *rs, hipStream_t s) {
    const int nch = g.nx / VEC;
    const int nwc = cdiv(nch, Pipe<T, 1, VEC>::OUTL);
    int nseg;
    if (g.tb_rows > 0) {
        nseg = cdiv(out_hi - out_lo, g.tb_rows);
    } else {
        const int blocks_per_strip = cdiv((long)g.tb_bpc * g.n_cu, nwc);
        nseg = blocks_per_strip * kPipeWaves;
        const int max_seg = (out_hi - out_lo) / 8;     // keep >= 8 rows per segment
        if (nseg > max_seg) nseg = std::max(1, max_seg);
    }
    const dim3 grid(nwc * cdiv(nseg, kPipeWaves)), block(kPipeWaves * 64);
    float *pa = f.pp[0] - (long)g.hg * g.nx, *pb = f.pp[1] - (long)g.hg * g.nx;
    if (g.fastdiv == 1)
        hipLaunchKernelGGL((k_jacobi_pipe<T, 1, VEC>), grid, block, 0, s, g, pa, pb, f.rhs, f.ctl,
                           rs, pass, it, par, out_lo, out_hi, nwc, nseg);
    else if (g.fastdiv == 2)
        hipLaunchKernelGGL((k_jacobi_pipe<T, 2, VEC>), grid, block, 0, s, g, pa, pb, f.rhs, f.ctl,
                           rs, pass, it, par, out_lo, out_hi, nwc, nseg);
    else
        hipLaunchKernelGGL((k_jacobi_pipe<T, 0, VEC>), grid, block, 0, s, g, pa, pb, f.rhs, f.ctl,
                           rs, pass, it, par, out_lo, out_hi, nwc, nseg);
}

template <int VEC>
void launch_pipe(const Geom &g, const Fields &f, int T, int pass, int it, int par, int out_lo,
                 int out_hi, uint32_t *rs, hipStream_t s) {
    switch (T) {
    case 1: launch_pipe_t<VEC, 1>(g, f, pass, it, par, out_lo, out_hi, rs, s); break;
    case 2: launch_pipe_t<VEC, 2>(g, f, pass, it, par, out_lo, out_hi, rs, s); break;
    case 3: launch_pipe_t<VEC, 3>(g, f, pass, it, par, out_lo, out_hi, rs, s); break;
    case 4: launch_pipe_t<VEC, 4>(g, f, pass, it, par, out_lo, out_hi, rs, s); break;
    case 5: launch_pipe_t<VEC, 5>(g, f, pass, it, par, out_lo, out_hi, rs, s); break;
    case 6: launch_pipe_t<VEC, 6>(g, f, pass, it, par, out_lo, out_hi, rs, s); break;
    case 7: launch_pipe_t<VEC, 7>(g, f, pass, it, par, out_lo, out_hi, rs, s); break;
    default: launch_pipe_t<VEC, 8>(g, f, pass, it, par, out_lo, out_hi, rs, s); break;
    }
}

}  // namespace
}  // namespace cfd
