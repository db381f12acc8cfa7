// cfd_predict_march.hip — both velocity predictors and the divergence in one
// row march, first- and second-order upwind (piso_step K1-K3: model.rs:538-670
// with compute_ustar / compute_vstar :381-521 and the face helpers :891-1248,
// then divergence :1406-1440).
//
// Mapping: a lane owns 4 columns (chunk c, i0 = 4c) and a wave 64 consecutive
// chunks; a wave marches up a segment of rows [r0, r1).  At step k it holds u
// rows k-2..k+2 and v rows k-1..k+3 in register rings (the second-order
// stencil's reach; the first-order one uses the middle of it) and
//   v*(k+1)  from v rows k-1..k+3 and u row k+1,
//   u*(k)    from u rows k-2..k+2 and v rows k, k+1,
//   rhs(k)   from u*(k), the east face u*(k, i0+4) of the lane on the right,
//            v*(k) (carried from the previous step) and v*(k+1),
// so every u / v value is loaded once per segment and u*, v* never return
// from memory for the divergence.  Rows are prefetched PD steps ahead.
//
// Horizontal neighbours (two columns each side for the second-order faces)
// come from the adjacent lanes by DPP lane shifts.  Waves step 62 chunks:
// lanes 0 and 63 only feed their neighbours (lane 63's u* of its first face is
// exact — that face reads nothing right of the lane — and is lane 62's east
// face).  Loads are flat: the chunk past the last column (c = nx/4) loads
// u faces nx..nx+3 and v columns nx..nx+3 of each row, i.e. the next row's
// first values, which is exactly what the reference's flat-indexed wrap reads
// (U(nx+1, j) == U(0, j+1), V(nx, j) == V(0, j+1): Q1-Q3); that lane stores u
// face nx, the one face of its chunk that exists.
//
// The face arithmetic is u_pred_val / v_pred_val (cfd_predict.h) over a
// register accessor and the divergence is k_divergence's expression, so the
// results are the unfused kernels', bit for bit.  Faces the reference does not
// predict (face 0, v column 0, rows outside glo..u_hi / v_hi) are read from
// memory, as k_divergence reads them.
#include "cfd_device.h"
#include "cfd_predict.h"

namespace cfd {
namespace {

#ifndef CFD_PM_WPE
#define CFD_PM_WPE 3  // minimum waves per SIMD (caps VGPRs at 168)
#endif
#ifndef CFD_PM_USTORE
#define CFD_PM_USTORE 0    // u* store: 0 one dword-aligned dwordx4 (75.1 us), 1 four dwords (75.7 us)
#endif
#ifndef CFD_PM_ROWS_FO
#define CFD_PM_ROWS_FO 8   // first-order march segment rows (r2: 8 rows 75.0 us, 16 rows 80.4 us)
#endif
#ifndef CFD_PM_PD
#define CFD_PM_PD 1   // prefetch distance (steps) of the u / v rows (1: 88.6 vs 90.3 us SO, r2 pm)
#endif

typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));

// Stencil accessor over the step's windows: u / v row k - 2 + r in x[r],
// columns i0-2..i0+5 at index 2 + column - i0; C = window row of the face.
template <int C>
struct MAcc {
    const float (&u)[6][8];
    const float (&v)[6][8];
    int q;
    __device__ __forceinline__ float U(int di, int dj) const { return u[C + dj][q + 2 + di]; }
    __device__ __forceinline__ float V(int di, int dj) const { return v[C + dj][q + 2 + di]; }
};

template <int SCHEME, int SP, bool MASK, int R>
struct PredMarch {
    static constexpr int PD = CFD_PM_PD;
    static constexpr int D = PD + 5;   // ring depth: 5 stencil rows + PD in flight

    float UQ[D][4];   // u row kb - 2 + t in slot t % D (t >= 0)
    float VQ[D][4];   // v row kb - 1 + t in slot t % D
    // u* face 0 / v* column 0 of the same rows (never predicted: the chunk-0
    // lane's divergence reads them), prefetched with the rings — a load whose
    // value is needed at once would wait for every row load in flight
    float UB[D], VB[D];
    float vs[4];      // v*(k), carried from the previous step
    const Geom *g;
    Fields f;
    __amdgpu_buffer_rsrc_t rs_u, rs_v, rs_us, rs_vs;
    int vo;                 // lane's byte offset in a row (far when outside the grid)
    int i0, c, nch;         // first column, chunk, chunks per row (nx / 4)
    bool st_lane;           // lanes 1..62: store what they compute
    int kb, r0, r1, glo, u_hi, v_hi, W;
    float dt;

    __device__ __forceinline__ void ld_u(float (&d)[4], int row) const {
        row = row < -kGhostUV ? -kGhostUV : (row > g->nyl + kGhostUV - 1 ? g->nyl + kGhostUV - 1 : row);
        const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs_u, vo, (row + kGhostUV) * W * 4, 0);
        d[0] = __uint_as_float(x.x); d[1] = __uint_as_float(x.y);
        d[2] = __uint_as_float(x.z); d[3] = __uint_as_float(x.w);
    }
    __device__ __forceinline__ void ld_v(float (&d)[4], int row) const {
        row = row < -kGhostUV ? -kGhostUV : (row > g->nyl + kGhostUV ? g->nyl + kGhostUV : row);
        const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs_v, vo, (row + kGhostUV) * g->nx * 4, 0);
        d[0] = __uint_as_float(x.x); d[1] = __uint_as_float(x.y);
        d[2] = __uint_as_float(x.z); d[3] = __uint_as_float(x.w);
    }

    __device__ __forceinline__ float ld_b(__amdgpu_buffer_rsrc_t rs, int row, int pitch, int hi) const {
        row = row < -kGhostUV ? -kGhostUV : (row > hi ? hi : row);
        return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, 0, (row + kGhostUV) * pitch * 4, 0));
    }
    __device__ __forceinline__ void ld_rows(int t, int slot) {
        ld_u(UQ[slot], kb - 2 + t);
        ld_v(VQ[slot], kb - 1 + t);
        UB[slot] = ld_b(rs_us, kb - 2 + t, W, g->nyl + kGhostUV - 1);
        VB[slot] = ld_b(rs_vs, kb - 1 + t, g->nx, g->nyl + kGhostUV);
    }

    // Step t (k = kb + t), T_ == t (mod D).  t == 0 only forms v*(r0).
    // GEN: the general step (first two and last steps of a segment: rows the
    // reference does not predict, read from memory, and the segment end).
    // The steady state (GEN false) has no load under a branch, so the
    // compiler's wait counts never drain the rows in flight.
    // INT: the wave's columns and the steady steps' rows are interior
    // (u_pred_val / v_pred_val skip their column and row tests)
    template <int T_, bool GEN, bool INT>
    __device__ __forceinline__ void step(int t) {
        constexpr bool I = INT && !GEN;
        const int k = kb + t;
        const int nx = g->nx;
        Fields ff = f;
        if (!MASK) ff.any_pmask = 0;   // obstacle-free slab: no mask loads
        float ux[6][8], vx[6][8];
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
            for (int x = 0; x < 8; ++x) ux[r][x] = vx[r][x] = 0.0f;
#pragma unroll
        for (int r = 0; r < 5; ++r)     // u rows k-2..k+2: slot (t + r) % D
#pragma unroll
            for (int x = 0; x < 4; ++x) ux[r][2 + x] = UQ[(T_ + r) % D][x];
#pragma unroll
        for (int r = 1; r < 6; ++r)     // v rows k-1..k+3: slot (t + r - 1) % D
#pragma unroll
            for (int x = 0; x < 4; ++x) vx[r][2 + x] = VQ[(T_ + r - 1) % D][x];
        // neighbour columns the faces read: u row k (+-2), u row k+1 (+1),
        // v row k (-1), v row k+1 (+-2)
        ux[2][0] = from_left(ux[2][4]);
        ux[2][1] = from_left(ux[2][5]);
        ux[2][6] = from_right(ux[2][2]);
        ux[2][7] = from_right(ux[2][3]);
        ux[3][6] = from_right(ux[3][2]);
        vx[2][1] = from_left(vx[2][5]);
        vx[3][0] = from_left(vx[3][4]);
        vx[3][1] = from_left(vx[3][5]);
        vx[3][6] = from_right(vx[3][2]);
        vx[3][7] = from_right(vx[3][3]);
        const float ub = UB[(T_ + 2) % D], vb = VB[(T_ + 2) % D];   // u* face 0 row k, v* col 0 row k+1
        // the rows leave the ring: u row k-2 and v row k-1 make room for the
        // rows D ahead
        ld_rows(t + D, T_ % D);

        // v*(k+1)
        const int rv = k + 1;
        float vn[4];
        if (!GEN || (rv >= glo && rv <= v_hi)) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                vn[q] = v_pred_val<SCHEME, SP, I>(*g, ff, dt, min(i0 + q, nx - 1), rv,
                                               MAcc<3>{ux, vx, q});
            if (c == 0) vn[0] = vb;   // column 0 is not predicted
            if (st_lane && c < nch && (!GEN || t > 0 || r0 == 0))
                *reinterpret_cast<float4 *>(f.v_star + (long)rv * nx + i0) =
                    make_float4(vn[0], vn[1], vn[2], vn[3]);
        } else {
            const float4 a = c < nch ? *reinterpret_cast<const float4 *>(f.v_star + (long)rv * nx + i0)
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
            vn[0] = a.x; vn[1] = a.y; vn[2] = a.z; vn[3] = a.w;
        }
        if (!GEN || t > 0) {
            // u*(k)
            float us[4];
            const long ku = (long)k * W + i0;
            const bool upred = !GEN || (k >= glo && k <= u_hi);
            if (upred) {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    us[q] = u_pred_val<SCHEME, SP, I>(*g, ff, dt, min(i0 + q, nx), k, MAcc<2>{ux, vx, q});
                if (c == 0) us[0] = ub;   // face 0 is not predicted
            } else if (c <= nch) {
                const f4u a = *reinterpret_cast<const f4u *>(f.u_star + ku);
                us[0] = a.x; us[1] = a.y; us[2] = a.z; us[3] = a.w;
            } else {
                us[0] = us[1] = us[2] = us[3] = 0.0f;
            }
            const float east = from_right(us[0]);
            if (st_lane) {
                if (c < nch) {
                    if (upred) {
                        if (CFD_PM_USTORE == 0) {   // one dword-aligned 16-byte store
                            *reinterpret_cast<f4u *>(f.u_star + ku) = (f4u){us[0], us[1], us[2], us[3]};
                        } else {                    // four dword stores
                            f.u_star[ku] = us[0];
                            f.u_star[ku + 1] = us[1];
                            f.u_star[ku + 2] = us[2];
                            f.u_star[ku + 3] = us[3];
                        }
                    }
                    const float rdx = g->r_dx, rdy = g->r_dy, dx = g->dx, dy = g->dy;
                    float4 rh;
                    rh.x = (sdiv<SP>(us[1] - us[0], dx, rdx) + sdiv<SP>(vn[0] - vs[0], dy, rdy)) / dt;
                    rh.y = (sdiv<SP>(us[2] - us[1], dx, rdx) + sdiv<SP>(vn[1] - vs[1], dy, rdy)) / dt;
                    rh.z = (sdiv<SP>(us[3] - us[2], dx, rdx) + sdiv<SP>(vn[2] - vs[2], dy, rdy)) / dt;
                    rh.w = (sdiv<SP>(east - us[3], dx, rdx) + sdiv<SP>(vn[3] - vs[3], dy, rdy)) / dt;
                    *reinterpret_cast<float4 *>(f.rhs + (long)k * nx + i0) = rh;
                } else if (c == nch && upred) {
                    f.u_star[ku] = us[0];   // face nx
                }
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) vs[q] = vn[q];
    }

    // D steps from t = base, base == OFF (mod D)
    template <int J, bool GEN, int OFF>
    __device__ __forceinline__ void group(int base) {
        if constexpr (J < D) {
            step<(OFF + J) % D, GEN>(base + J);
            group<J + 1, GEN, OFF>(base);
        }
    }

    // the segment's R + 1 steps, fully unrolled (every ring index and step
    // kind compile-time, no loop back edge whose register copies would wait
    // for the rows in flight): t = 0, 1 and R general, the rest steady
    template <int T, bool INT>
    __device__ __forceinline__ void steps() {
        if constexpr (T <= R) {
            step<T % D, (T < 2 || T == R), INT>(T);
            steps<T + 1, INT>();
        }
    }
    template <bool INT>
    __device__ __forceinline__ void run() {
#pragma unroll
        for (int t = 0; t < D; ++t) ld_rows(t, t);
        steps<0, INT>();
    }
};

template <int SCHEME, int SP, bool MASK, int R>
__global__ __launch_bounds__(kBlock, CFD_PM_WPE) void k_predict_march(Geom g, Fields f, float dt_override,
                                                          int glo, int u_hi, int v_hi, int nwc,
                                                          int nseg, int set_inlet, int row_lo,
                                                          int row_hi) {
    if (set_inlet && blockIdx.x == 0 && threadIdx.x == 0) {
        // k_step_begin's work when it copies nothing: the inlet ramp
        // (simulation_step as f32 / ramp_up_steps as f32) * target (model.rs:311-316),
        // read by the corrector finish at the end of the step
        Ctl *c = f.ctl;
        const uint32_t st = c->step;
        c->inlet = st < 100u ? ((float)st / 100.0f) * g.target_inlet : g.target_inlet;
        c->go[0] = 1;
    }
    PredMarch<SCHEME, SP, MASK, R> m;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int lane = (int)threadIdx.x & 63;
    const int bid = xcd_block(g);
    const int wc = bid % nwc;
    const int seg = (bid / nwc) * (kBlock / 64) + wave;
    if (seg >= nseg) return;   // wave-uniform
    const int nx = g.nx;
    // R rows per segment of the launch's rows [row_lo, row_hi); the last one
    // ends at row_hi and overlaps its neighbour (both store the same values;
    // no segment reads what another stores)
    m.r0 = row_lo + min(seg * R, row_hi - row_lo - R);
    m.r1 = m.r0 + R;
    m.g = &g;
    m.f = f;
    m.W = nx + 1;
    m.nch = nx / 4;
    m.c = wc * 62 - 1 + lane;
    const bool in_dom = m.c >= 0 && m.c <= m.nch;
    m.i0 = in_dom ? 4 * m.c : 0;
    m.st_lane = in_dom && lane >= 1 && lane <= 62;
    m.vo = in_dom ? 4 * m.i0 : 0x7FFF0000;
    m.rs_u = __builtin_amdgcn_make_buffer_rsrc(f.u_alloc_base, 0, (int)(f.u_alloc * 4), 0x00020000);
    m.rs_v = __builtin_amdgcn_make_buffer_rsrc(f.v_alloc_base, 0, (int)(f.v_alloc * 4), 0x00020000);
    m.rs_us = __builtin_amdgcn_make_buffer_rsrc(f.u_star_base, 0, (int)(f.u_alloc * 4), 0x00020000);
    m.rs_vs = __builtin_amdgcn_make_buffer_rsrc(f.v_star_base, 0, (int)(f.v_alloc * 4), 0x00020000);
    m.glo = glo;
    m.u_hi = u_hi;
    m.v_hi = v_hi;
    m.kb = m.r0 - 1;
    m.dt = dt_of(f.ctl, dt_override);
#pragma unroll
    for (int q = 0; q < 4; ++q) m.vs[q] = 0.0f;
    // interior wave: every chunk it touches has columns in [3, nx-3] (so the
    // last chunk nch is not among them), and the steady steps' faces (u row
    // k, v row k+1, k = r0+1 .. r1-2) lie on global rows [2, ny-3] / [2, ny-2]
    const int c_lo = wc * 62 - 1, c_hi = wc * 62 + 62;
    const bool interior = 4 * c_lo >= 3 && 4 * c_hi + 3 <= nx - 3 &&
                          g.j0 + m.r0 + 1 >= 2 && g.j0 + m.r1 - 2 <= g.ny - 3;
    // the interior form only where it changes the code (second order)
    if (SCHEME == 1 && interior)
        m.template run<true>();
    else
        m.template run<false>();
}

}  // namespace

bool predict_march_ok(const Geom &g, const Fields &f) {
    auto a16 = [](const void *p) { return ((uintptr_t)p & 15u) == 0; };
    return g.pred_div == 2 && g.nx % 4 == 0 && g.nx >= 8 && g.nyl >= 4 && a16(f.v) && a16(f.v_star) &&
           a16(f.rhs) && (uint64_t)f.u_alloc * 4u < (1ull << 31) &&
           (uint64_t)f.v_alloc * 4u < (1ull << 31);
}

void launch_predict_march(const Geom &g, const Fields &f, float dt_override, hipStream_t s,
                          bool set_inlet, int row_lo, int row_hi) {
    if (row_hi < 0) row_hi = g.nyl;
    const int glo = (g.j0 > 1 ? g.j0 : 1) - g.j0;
    const int u_hi = ((g.j0 + g.nyl - 1) < (g.ny - 2) ? (g.j0 + g.nyl - 1) : (g.ny - 2)) - g.j0;
    const int v_hi = ((g.j0 + g.nyl) < (g.ny - 1) ? (g.j0 + g.nyl) : (g.ny - 1)) - g.j0;
    // rows per segment: 8 (two rounds of ~3-4 waves per SIMD at 4096^2 with
    // 17 wave columns; 16-row segments measured equal for the first-order
    // scheme and 17 % slower for the second-order one, whose unrolled march
    // then outgrows the instruction cache), 4 on slabs under 8 rows
    // first order: CFD_PM_ROWS_FO rows per segment (compile-time knob, 8)
    const int big = g.scheme == 0 ? CFD_PM_ROWS_FO : 8;
    const int span = row_hi - row_lo;
    const int rows = span >= big ? big : (span >= 8 ? 8 : 4);
    const int nwc = cdiv(g.nx / 4 + 1, 62);
    const int nseg = cdiv(row_hi - row_lo, rows);
    const dim3 grid(nwc * cdiv(nseg, kBlock / 64));
#define CFD_LAUNCH_PM(SC, SPV, MK, R)                                                              \
    hipLaunchKernelGGL((k_predict_march<SC, SPV, MK, R>), grid, dim3(kBlock), 0, s, g, f, dt_override, \
                       glo, u_hi, v_hi, nwc, nseg, set_inlet ? 1 : 0, row_lo, row_hi)
#define CFD_LAUNCH_PM3(SC, SPV, MK)                                         \
    if (CFD_PM_ROWS_FO != 8 && SC == 0 && rows == CFD_PM_ROWS_FO)           \
        CFD_LAUNCH_PM(SC, SPV, MK, (SC == 0 ? CFD_PM_ROWS_FO : 8));          \
    else if (rows == 8) CFD_LAUNCH_PM(SC, SPV, MK, 8); else CFD_LAUNCH_PM(SC, SPV, MK, 4)
#define CFD_LAUNCH_PM2(SC, SPV) \
    if (f.any_pmask) { CFD_LAUNCH_PM3(SC, SPV, true); } else { CFD_LAUNCH_PM3(SC, SPV, false); }
    if (g.scheme == 0) {
        if (g.sp_pow2) { CFD_LAUNCH_PM2(0, 1); } else { CFD_LAUNCH_PM2(0, 0); }
    } else {
        if (g.sp_pow2) { CFD_LAUNCH_PM2(1, 1); } else { CFD_LAUNCH_PM2(1, 0); }
    }
#undef CFD_LAUNCH_PM3
#undef CFD_LAUNCH_PM2
#undef CFD_LAUNCH_PM
}

}  // namespace cfd
