// cfd_jacobi_tb1.hip — k_jacobi_tb: T <= 4 weighted-Jacobi sweeps per launch
// (model.rs:734-824) by a register march, one halo lane per wave side.
#include "cfd_device.h"

namespace cfd {
namespace {

// T weighted-Jacobi sweeps in one launch (temporal blocking; fixed-count
// solves only — the tolerance test needs every sweep's residual).
//
// A wave owns 64 float4 column chunks; lanes 0 and 63 are halo lanes whose
// values go stale one element per sweep from the outside in, so for T <= 4
// lanes 1..62 (248 columns) stay exact and are the only ones stored; wave
// columns overlap by two chunks.  The wave marches a segment of R output rows
// through T pipelined stages: at row slot k it loads input row k and stage s
// (1..T) computes row k-s from stage s-1's window of rows k-s-1..k-s+1, so
// every stage is one sweep of the reference, at R + 2T row slots per segment.
// p' and rhs come from HBM once per launch (12 B per T cell-updates).
//
// Per stage the p' boundary conditions of model.rs:807-815 are applied to the
// window itself: column 0 takes column 1, column nx-1 is 0, global row ny-1
// copies row ny-2, and global row 0 is patched with row 1 as soon as row 1 is
// computed (before the next stage reads it).  Only the final stage is stored,
// with the same fused boundary stores as k_jacobi.
// Per-wave state of k_jacobi_tb.  Register rings are indexed by the slot
// number v (0-based within the segment) modulo their period, so with the slot
// loop unrolled by 6 (= lcm of the periods 2, 3 and 6) every index is a
// compile-time constant and no window ever moves between registers:
//   PF[v % 2]        p' input row k_first+v, loaded two slots ahead
//   W[s][v % 3]      newest row of stage s (stage 0 = input)
//   RH[(q-k_first+1) % 6]  rhs row q (rows k-4 .. k+1 live at slot k)
template <int T, int FAST>
struct TbWave {
    float4 W[T][3];
    float4 RH[6];
    float4 PF[2];
    // geometry (wave-uniform scalars unless noted)
    int k_first, S, r0, r1, nyl, nch, nx, hg, g_first, g_last, g_top, g_zero, row_bytes;
    int ch, col, lane, off0;    // per lane
    bool out_lane, e0, e1, e2, e3;
    float dx_sq, dy_sq, denom, r_dx_sq, r_dy_sq, r_denom;
    __amdgpu_buffer_rsrc_t rs_p, rs_r;
    float *dst;
    float m;

    __device__ __forceinline__ float4 ld4(const __amdgpu_buffer_rsrc_t &rs, int row) const {
        constexpr int kOOB = -16;
        const int o = (off0 < 0 || row < -hg || row >= nyl + hg) ? kOOB : off0 + row * row_bytes;
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0);
        return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                           __uint_as_float(v.w));
    }

    // one reference sweep of one row (model.rs:775-793 + BCs :807-815 per column)
    template <bool EDGE>
    __device__ __forceinline__ float4 stage(const float4 &B, const float4 &Cc, const float4 &Tp,
                                            const float4 &Rh) const {
        const float L0 = from_left(Cc.w);
        const float R3 = from_right(Cc.x);
        float4 o = jacobi_row4<FAST>(B, Cc, Tp, Rh, L0, R3, dx_sq, dy_sq, denom, r_dx_sq,
                                     r_dy_sq, r_denom);
        if (EDGE) {
            if (ch == 0) o.x = o.y;
            if (ch == nch - 1) o.w = 0.0f;
        }
        return o;
    }

    // Slot v of the segment.  V is a compile-time value with V == v (mod 6)
    // that fixes every ring index; in the warm-up (GUARD == 0, V == v
    // exactly) it also decides at compile time which stages already have
    // rows to compute (stage s starts at slot 2s).  GUARD == 2 is the final
    // partial group: slots past the segment end return (uniform branch).
    template <int V, int GUARD, bool EDGE>
    __device__ __forceinline__ void slot(int v) {
        if (GUARD == 2 && v >= S) return;
        const int k = k_first + v;
        W[0][V % 3] = PF[V % 2];                             // input row k
        PF[V % 2] = ld4(rs_p, k + 2);                        // two slots ahead
#pragma unroll
        for (int s = 1; s <= T; ++s) {
            if (GUARD == 0 && V < 2 * s) continue;            // compile-time
            const int r = k - s;
            const float4 &B = W[s - 1][(V + 1) % 3];          // stage s-1, row r-1
            const float4 &C = W[s - 1][(V + 2) % 3];          //              row r
            const float4 &Tp = W[s - 1][V % 3];               //              row r+1
            const float4 &Rh = RH[(V - s + 1 + 6) % 6];       // rhs row r
            float4 n = stage<EDGE>(B, C, Tp, Rh);
            if (s < T) {
                if (EDGE && r == g_top) n = W[s][(V + 2) % 3];   // P(i,ny-1) = P(i,ny-2)
                W[s][V % 3] = n;
                if (EDGE && r == g_first) W[s][(V + 2) % 3] = n; // P(i,0) = P(i,1)
            } else {
                // final stage, rows r0 <= r < r1 (v >= 2T, v < S)
                if (r < nyl && r >= 0) {
                    if (EDGE) {
                        if (out_lane) {
                            if (e0) m = fmaxf(m, fabsf(n.x - C.x));
                            if (e1) m = fmaxf(m, fabsf(n.y - C.y));
                            if (e2) m = fmaxf(m, fabsf(n.z - C.z));
                            if (e3) m = fmaxf(m, fabsf(n.w - C.w));
                        }
                    } else {
                        // interior wave: every column of an output lane is a
                        // residual column; halo lanes are cleared at the end
                        m = fmaxf(fmaxf(fmaxf(fmaxf(m, fabsf(n.x - C.x)), fabsf(n.y - C.y)),
                                        fabsf(n.z - C.z)),
                                  fabsf(n.w - C.w));
                    }
                }
                if (out_lane) {
                    *reinterpret_cast<float4 *>(dst + (long)r * nx + col) = n;
                    if (EDGE && r == g_first)
                        *reinterpret_cast<float4 *>(dst + (long)g_zero * nx + col) = n;
                    if (EDGE && r == g_last)
                        *reinterpret_cast<float4 *>(dst + (long)g_top * nx + col) = n;
                }
            }
        }
        RH[(V + 2) % 6] = ld4(rs_r, k + 1);                   // rhs row k+1
    }

    template <int V, bool EDGE>
    __device__ __forceinline__ void warmup() {
        if constexpr (V < 2 * T) {
            slot<V, 0, EDGE>(V);
            warmup<V + 1, EDGE>();
        }
    }

    // steady-state group of 6 slots starting at v = base (base == 2T mod 6)
    template <int GUARD, bool EDGE>
    __device__ __forceinline__ void group(int base) {
        slot<2 * T + 0, GUARD, EDGE>(base + 0);
        slot<2 * T + 1, GUARD, EDGE>(base + 1);
        slot<2 * T + 2, GUARD, EDGE>(base + 2);
        slot<2 * T + 3, GUARD, EDGE>(base + 3);
        slot<2 * T + 4, GUARD, EDGE>(base + 4);
        slot<2 * T + 5, GUARD, EDGE>(base + 5);
    }

    // the whole segment; EDGE = the wave touches a domain boundary (column 0
    // or nx-1, or a global row 0/1/ny-2/ny-1 in any stage) and needs the
    // boundary-condition logic; interior waves skip it entirely
    template <bool EDGE>
    __device__ __forceinline__ void run() {
        warmup<0, EDGE>();                              // slots 0 .. 2T-1
        int base = 2 * T;
        const int full_end = 2 * T + ((S - 2 * T) / 6) * 6;
        for (; base < full_end; base += 6) group<1, EDGE>(base);
        if (base < S) group<2, EDGE>(base);             // final partial group
    }
};

// T weighted-Jacobi sweeps in one launch (temporal blocking; fixed-count
// solves only — the tolerance test needs every sweep's residual).
//
// A wave owns 64 float4 column chunks; lanes 0 and 63 are halo lanes whose
// values go stale one element per sweep from the outside in, so for T <= 4
// lanes 1..62 (248 columns) stay exact and are the only ones stored; wave
// columns overlap by two chunks.  The wave marches a segment of R output rows
// through T pipelined stages: at row slot k it loads input row k and stage s
// (1..T) computes row k-s from stage s-1's window of rows k-s-1..k-s+1, so
// every stage is one sweep of the reference, at R + 2T row slots per segment.
// p' and rhs come from HBM once per launch (12 B per T cell-updates).
//
// Per stage the p' boundary conditions of model.rs:807-815 are applied to the
// window itself: column 0 takes column 1, column nx-1 is 0, global row ny-1
// copies row ny-2, and global row 0 is patched with row 1 as soon as row 1 is
// computed (before the next stage reads it).  Only the final stage is stored,
// with the same fused boundary stores as k_jacobi.
template <int T, int FAST>
__global__ __launch_bounds__(kJacWavesPerBlock * 64) void k_jacobi_tb(
    Geom g, float *__restrict__ pa, float *__restrict__ pb, const float *__restrict__ rhs,
    Ctl *ctl, uint32_t *res_slots, int pass, int it, int par, int out_lo, int out_hi, int nwc,
    int nseg) {
    if (pass_off(ctl, pass)) return;
    TbWave<T, FAST> w;
    // the wave index is uniform; readfirstlane lets the compiler see it, so
    // every row/slot condition below becomes a scalar branch
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    w.lane = (int)threadIdx.x & 63;
    const int bid = xcd_block(g);
    const int wc = bid % nwc;
    const int seg = (bid / nwc) * kJacWavesPerBlock + wave;
    // balanced segments: nseg row ranges differing by at most one row
    const int nrows = out_hi - out_lo;
    if (seg >= nseg) return;
    w.r0 = out_lo + (int)(((long)seg * nrows) / nseg);
    w.r1 = out_lo + (int)(((long)(seg + 1) * nrows) / nseg);
    if (w.r0 >= w.r1) return;
    w.nx = g.nx;
    w.nch = g.nx >> 2;
    w.hg = g.hg;
    w.nyl = g.nyl;
    w.ch = wc * 62 - 1 + w.lane;
    const bool in_dom = w.ch >= 0 && w.ch < w.nch;
    w.out_lane = in_dom && w.lane >= 1 && w.lane <= 62;

    // buffers ping-pong once per LAUNCH: par = launches since the solve began
    const int si = (ctl->cur + par) & 1;
    float *src_alloc = si ? pb : pa;
    float *dst_alloc = si ? pa : pb;
    const int pbytes = (w.nyl + 2 * w.hg) * w.nx * 4;
    w.rs_p = __builtin_amdgcn_make_buffer_rsrc(src_alloc, 0, pbytes, 0x00020000);
    w.rs_r = __builtin_amdgcn_make_buffer_rsrc((void *)(rhs - (long)w.hg * w.nx), 0, pbytes,
                                               0x00020000);
    w.dst = dst_alloc + (long)w.hg * w.nx;
    w.dx_sq = g.dx_sq;
    w.dy_sq = g.dy_sq;
    w.denom = g.denom;
    w.r_dx_sq = g.r_dx_sq;
    w.r_dy_sq = g.r_dy_sq;
    w.r_denom = g.r_denom;
    w.col = 4 * w.ch;
    w.row_bytes = w.nx * 4;
    w.off0 = in_dom ? (w.hg * w.nx + w.col) * 4 : -16;
    w.e0 = (w.col >= 1) && (w.col <= w.nx - 8);
    w.e1 = (w.col + 1 <= w.nx - 8);
    w.e2 = (w.col + 2 <= w.nx - 8);
    w.e3 = (w.col + 3 <= w.nx - 8);
    w.g_first = 1 - g.j0;
    w.g_last = g.ny - 2 - g.j0;
    w.g_top = g.ny - 1 - g.j0;
    w.g_zero = -g.j0;
    w.m = 0.0f;
    w.k_first = w.r0 - T;
    w.S = (w.r1 - w.r0) + 2 * T;

    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int s = 0; s < T; ++s) w.W[s][0] = w.W[s][1] = w.W[s][2] = z4;
    // prologue loads: input rows k_first, k_first+1; rhs rows k_first-1, k_first
    w.PF[0] = w.ld4(w.rs_p, w.k_first);
    w.PF[1] = w.ld4(w.rs_p, w.k_first + 1);
    w.RH[0] = w.ld4(w.rs_r, w.k_first - 1);
    w.RH[1] = w.ld4(w.rs_r, w.k_first);
#pragma unroll
    for (int q = 2; q < 6; ++q) w.RH[q] = z4;
    // interior waves store chunks 1 .. nch-3 only (all residual columns)
    const bool col_edge = wc == 0 || (wc * 62 + 63 >= w.nch - 2);
    const int lo_row = w.k_first - 1, hi_row = w.r1 + T + 1;   // every row any stage touches
    auto hits = [&](int r) { return r >= lo_row && r <= hi_row; };
    const bool row_edge = hits(w.g_zero) || hits(w.g_first) || hits(w.g_last) || hits(w.g_top);
    if (col_edge || row_edge)
        w.template run<true>();
    else
        w.template run<false>();
    if (!res_slots) return;
    const float m = wave_max(w.out_lane ? w.m : 0.0f);
    if (w.lane == 0) publish_max(res_slots, (int)blockIdx.x * kJacWavesPerBlock + wave, m);
}

template <int T>
void launch_t(const Geom &g, const Fields &f, int pass, int it, int par, int out_lo, int out_hi,
              uint32_t *rs, hipStream_t s) {
    const int nch = g.nx / 4;
    const int nwc = cdiv(nch, 62);
    int nseg;
    if (g.tb_rows > 0) {
        nseg = cdiv(out_hi - out_lo, g.tb_rows);
    } else {
        const int blocks_per_strip = cdiv((long)g.tb_bpc * g.n_cu, nwc);
        nseg = blocks_per_strip * kJacWavesPerBlock;
        const int max_seg = (out_hi - out_lo) / 8;     // keep >= 8 rows per segment
        if (nseg > max_seg) nseg = std::max(1, max_seg);
    }
    const dim3 grid(nwc * cdiv(nseg, kJacWavesPerBlock)), block(kJacWavesPerBlock * 64);
    float *pa = f.pp[0] - (long)g.hg * g.nx, *pb = f.pp[1] - (long)g.hg * g.nx;
    if (g.fastdiv == 1)
        hipLaunchKernelGGL((k_jacobi_tb<T, 1>), grid, block, 0, s, g, pa, pb, f.rhs, f.ctl, rs,
                           pass, it, par, out_lo, out_hi, nwc, nseg);
    else if (g.fastdiv == 2)
        hipLaunchKernelGGL((k_jacobi_tb<T, 2>), grid, block, 0, s, g, pa, pb, f.rhs, f.ctl, rs,
                           pass, it, par, out_lo, out_hi, nwc, nseg);
    else
        hipLaunchKernelGGL((k_jacobi_tb<T, 0>), grid, block, 0, s, g, pa, pb, f.rhs, f.ctl, rs,
                           pass, it, par, out_lo, out_hi, nwc, nseg);
}

}  // namespace

void launch_tb1(const Geom &g, const Fields &f, int T, int pass, int it, int par, int out_lo,
                int out_hi, uint32_t *rs, hipStream_t s) {
    switch (T) {
    case 1: launch_t<1>(g, f, pass, it, par, out_lo, out_hi, rs, s); break;
    case 2: launch_t<2>(g, f, pass, it, par, out_lo, out_hi, rs, s); break;
    case 3: launch_t<3>(g, f, pass, it, par, out_lo, out_hi, rs, s); break;
    default: launch_t<4>(g, f, pass, it, par, out_lo, out_hi, rs, s); break;
    }
}

}  // namespace cfd
