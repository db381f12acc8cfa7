// cfd_kernels.hip — CDNA4 (gfx950) kernels for cfd-demo's Model::update hot path.
//
// Every kernel reproduces the reference's f32 arithmetic bit for bit: the
// file is compiled with -ffp-contract=off (Rust never fuses a*b+c), `/` is
// HIP's default correctly-rounded f32 division, denormals are kept, and each
// expression keeps the reference's evaluation order.  Maxima are exact and
// order-independent, so the reductions (wave shuffles + one atomicMax on the
// f32 bit pattern of a non-negative value) are deterministic.
//
// Citations are /root/reference/src/model.rs line numbers.
#include "cfd_device.h"
#include "cfd_predict.h"

namespace cfd {

// 16 bytes at a 4-byte aligned address (the u rows' pitch nx + 1): one
// global_load/store_dwordx4 (unaligned access mode) instead of four dwords
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));

namespace {
// Exhaustive proof of the fast forms for one divisor c (r = RN(1/c)):
// counts inputs x where x*r (mode 1) or the corrected form (mode 2) differs
// from IEEE x/c; NaN results compare equal to NaN.
__global__ __launch_bounds__(kBlock) void k_verify_division(float c, float r,
                                                            unsigned long long *counts) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t stride = gridDim.x * blockDim.x;
    uint32_t bad1 = 0, bad2 = 0, bad3 = 0;
    for (uint64_t k = tid; k < (1ull << 32); k += stride) {
        const float x = __uint_as_float((uint32_t)k);
        const float ref = x / c;
        const float m1 = fdiv<1>(x, c, r);
        const float m2 = fdiv<2>(x, c, r);
        const float m3 = fdiv<3>(x, c, r);
        const bool rn = ref != ref;
        bad1 += (rn ? (m1 == m1) : (__float_as_uint(m1) != __float_as_uint(ref))) ? 1u : 0u;
        bad2 += (rn ? (m2 == m2) : (__float_as_uint(m2) != __float_as_uint(ref))) ? 1u : 0u;
        bad3 += (rn ? (m3 == m3) : (__float_as_uint(m3) != __float_as_uint(ref))) ? 1u : 0u;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        bad1 += __shfl_xor(bad1, o, 64);
        bad2 += __shfl_xor(bad2, o, 64);
        bad3 += __shfl_xor(bad3, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        if (bad1) atomicAdd(&counts[0], (unsigned long long)bad1);
        if (bad2) atomicAdd(&counts[1], (unsigned long long)bad2);
        if (bad3) atomicAdd(&counts[2], (unsigned long long)bad3);
    }
}

// ------------------------------------------------------------- copies (K0/K5b)

__device__ __forceinline__ void copy4(float *__restrict__ dst, const float *__restrict__ src,
                                      size_t n4, size_t tid, size_t stride) {
    const float4 *s = reinterpret_cast<const float4 *>(src);
    float4 *d = reinterpret_cast<float4 *>(dst);
    for (size_t k = tid; k < n4; k += stride) d[k] = s[k];
}

// update() prologue (model.rs:307-316): u_old <- u, v_old <- v, inlet ramp.
// With `copy` 0 (the fused corrector computes the residuals from the values it
// overwrites) only the control words are touched.
__global__ __launch_bounds__(kBlock) void k_step_begin(Geom g, Fields f, int copy) {
    const size_t tid = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    if (copy) {
        copy4(f.u_old_base, f.u_alloc_base, f.u_alloc / 4, tid, stride);
        copy4(f.v_old_base, f.v_alloc_base, f.v_alloc / 4, tid, stride);
    }
    if (tid == 0) {
        Ctl *c = f.ctl;
        const uint32_t st = c->step;
        // (simulation_step as f32 / ramp_up_steps as f32) * target (model.rs:311-316)
        c->inlet = st < 100u ? ((float)st / 100.0f) * g.target_inlet : g.target_inlet;
        c->go[0] = 1;
    }
}

// u_star <- u, v_star <- v before each extra correction pass (model.rs:698-699).
__global__ __launch_bounds__(kBlock) void k_copy_star(Fields f, int pass) {
    if (pass_off(f.ctl, pass)) return;
    const size_t tid = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    copy4(f.u_star_base, f.u_alloc_base, f.u_alloc / 4, tid, stride);
    copy4(f.v_star_base, f.v_alloc_base, f.v_alloc / 4, tid, stride);
}

// Predictor face arithmetic (u_pred_val / v_pred_val) and GAcc: cfd_predict.h.


template <int SCHEME, int SP>
__global__ __launch_bounds__(kBlock) void k_u_predictor(Geom g, Fields f, float dt_override,
                                                        int row_lo, int nbx) {
    const int bid = xcd_block(g);
    const int i = 1 + (bid % nbx) * kBlock + (int)threadIdx.x;
    const int lj = row_lo + bid / nbx;
    if (i > g.nx) return;
    const GAcc a{f.u, f.v, (long)lj * (g.nx + 1) + i, (long)lj * g.nx + i, g.nx + 1, g.nx};
    f.u_star[(long)lj * (g.nx + 1) + i] = u_pred_val<SCHEME, SP>(g, f, dt_of(f.ctl, dt_override), i, lj, a);
}


template <int SCHEME, int SP>
__global__ __launch_bounds__(kBlock) void k_v_predictor(Geom g, Fields f, float dt_override,
                                                        int row_lo, int nbx) {
    const int bid = xcd_block(g);
    const int i = 1 + (bid % nbx) * kBlock + (int)threadIdx.x;
    const int lj = row_lo + bid / nbx;
    if (i > g.nx - 1) return;
    const GAcc a{f.u, f.v, (long)lj * (g.nx + 1) + i, (long)lj * g.nx + i, g.nx + 1, g.nx};
    f.v_star[(long)lj * g.nx + i] = v_pred_val<SCHEME, SP>(g, f, dt_of(f.ctl, dt_override), i, lj, a);
}

// Both predictors in one pass (piso_step's K1 + K2): each thread computes the
// u face and the v face at (i, lj), sharing the u / v loads through L1; u rows
// run to u_hi, v rows to v_hi (v also covers the slab's top face row).  Same
// values as the two single kernels (one launch and one pass over u, v less).
// Measured alternatives on the bench workload (r1): 4 columns per thread
// with strided scalar loads 185 us, an LDS-staged 256 x 16 tile 147 us,
// this form 113 us.
template <int SCHEME, int SP>
__global__ __launch_bounds__(kBlock) void k_predict(Geom g, Fields f, float dt_override, int row_lo,
                                                    int u_hi, int v_hi, int nbx) {
    const int bid = xcd_block(g);
    const int i = 1 + (bid % nbx) * kBlock + (int)threadIdx.x;
    const int lj = row_lo + bid / nbx;
    const GAcc a{f.u, f.v, (long)lj * (g.nx + 1) + i, (long)lj * g.nx + i, g.nx + 1, g.nx};
    if (lj <= u_hi && i <= g.nx)
        f.u_star[(long)lj * (g.nx + 1) + i] = u_pred_val<SCHEME, SP>(g, f, dt_of(f.ctl, dt_override), i, lj, a);
    if (lj <= v_hi && i <= g.nx - 1)
        f.v_star[(long)lj * g.nx + i] = v_pred_val<SCHEME, SP>(g, f, dt_of(f.ctl, dt_override), i, lj, a);
}

// Both first-order predictors with four columns per thread (i0 = 4t): the
// pitch-nx v rows move as float4 (v row lj-1, lj, lj+1 and the v* store), the
// pitch-(nx+1) u rows as scalars, and each value is loaded once for the eight
// faces it feeds (u_pred_val / v_pred_val over an RAccN, so the arithmetic is
// the single-face kernel's, bit for bit).  Face 0 and column 0 are not
// predicted (model.rs:538, :586); the thread owning columns nx-4..nx-1 also
// predicts u face nx, through the flat-indexed GAcc (its east and north
// neighbours wrap to the next row, Q1-Q3).  Requires 16-byte aligned v and
// v* rows (checked by the launcher).
// Each thread takes RPT = 2 consecutive rows (96 vs 104 us for one row and
// 107 for four, r1): the window of u and v rows
// lj-1 .. lj+RPT is loaded up front (every load in flight at once, and the
// rows shared by neighbouring output rows loaded once), then the 8 x RPT
// faces are computed with the same u_pred_val / v_pred_val arithmetic.
// Rows past the last row a predictor needs are clamped to it (their values
// are never used), so no load leaves the allocation.
struct RAccN {
    const float (*ur)[6];
    const float (*vr)[6];
    int q;
    __device__ __forceinline__ float U(int di, int dj) const { return ur[dj + 1][q + 1 + di]; }
    __device__ __forceinline__ float V(int di, int dj) const { return vr[dj + 1][q + 1 + di]; }
};

template <int SP, int RPT>
__global__ __launch_bounds__(kBlock) void k_predict4r(Geom g, Fields f, float dt_override,
                                                      int row_lo, int u_hi, int v_hi, int nbx) {
    const int bid = xcd_block(g);
    const int i0 = 4 * ((bid % nbx) * kBlock + (int)threadIdx.x);
    const int lj0 = row_lo + (bid / nbx) * RPT;
    const int nx = g.nx, W = nx + 1;
    if (i0 >= nx) return;
    const float dtv = dt_of(f.ctl, dt_override);   // once: a per-face reload waits on every load
    const float *__restrict__ u = f.u;
    const float *__restrict__ v = f.v;
    const int u_cap = u_hi + 1 > v_hi ? u_hi + 1 : v_hi;   // last u row any face reads
    const int v_cap = v_hi + 1;                            // last v row any face reads
    float ur[RPT + 2][6], vr[RPT + 2][6];
#pragma unroll
    for (int r = 0; r < RPT + 2; ++r) {
        const int ru = min(lj0 - 1 + r, u_cap), rv = min(lj0 - 1 + r, v_cap);
        const long ku = (long)ru * W + i0, kv = (long)rv * nx + i0;
        const bool mid = r >= 1 && r <= RPT;   // output rows: their east/west neighbours too
        ur[r][0] = (mid && i0 > 0) ? u[ku - 1] : 0.0f;
#pragma unroll
        for (int c = 0; c < 4; ++c) ur[r][c + 1] = u[ku + c];
        ur[r][5] = mid ? u[ku + 4] : 0.0f;
        const float4 a = *reinterpret_cast<const float4 *>(v + kv);
        vr[r][1] = a.x; vr[r][2] = a.y; vr[r][3] = a.z; vr[r][4] = a.w;
        vr[r][0] = (mid && i0 > 0) ? v[kv - 1] : 0.0f;
        vr[r][5] = mid ? v[kv + 4] : 0.0f;   // column nx wraps to the next row's column 0
    }
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
        const int lj = lj0 + r;
        const long ku = (long)lj * W + i0, kv = (long)lj * nx + i0;
        if (lj <= u_hi) {
            float o[4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                o[q] = u_pred_val<0, SP>(g, f, dtv, i0 + q, lj, RAccN{ur + r, vr + r, q});
            float *__restrict__ us = f.u_star + ku;
            if (i0 > 0) us[0] = o[0];
            us[1] = o[1];
            us[2] = o[2];
            us[3] = o[3];
            if (i0 + 4 == nx) {
                const GAcc a{f.u, f.v, ku + 4, kv + 4, W, nx};
                us[4] = u_pred_val<0, SP>(g, f, dtv, nx, lj, a);
            }
        }
        if (lj <= v_hi) {
            float o[4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                o[q] = v_pred_val<0, SP>(g, f, dtv, i0 + q, lj, RAccN{ur + r, vr + r, q});
            float *__restrict__ vs = f.v_star + kv;
            if (i0 > 0) {
                *reinterpret_cast<float4 *>(vs) = make_float4(o[0], o[1], o[2], o[3]);
            } else {
                vs[1] = o[1];
                vs[2] = o[2];
                vs[3] = o[3];
            }
        }
    }
}

// ------------------------------------------------------------ divergence (K3)

// rhs = div(u*, v*) / dt on every owned pressure cell (model.rs:1406-1440).
// A thread owns 4 consecutive cells: v* rows and the rhs row are 16-byte
// aligned (pitch nx, nx % 8 == 0) and move as float4; the u* row (pitch nx+1)
// is read as 5 scalars.  One float per thread capped this stream at ~3 TB/s.
template <int SP>
__global__ __launch_bounds__(kBlock) void k_divergence(Geom g, Fields f, int pass,
                                                       float dt_override, int nbx) {
    if (pass_off(f.ctl, pass)) return;
    const int bid = xcd_block(g);
    const int i0 = 4 * ((bid % nbx) * kBlock + (int)threadIdx.x);
    const int lj = bid / nbx;
    const int nx = g.nx, W = nx + 1;
    if (i0 >= nx) return;
    const float dt = dt_of(f.ctl, dt_override);
    const float *__restrict__ us = f.u_star + (long)lj * W + i0;
    const float4 vs = *reinterpret_cast<const float4 *>(f.v_star + (long)lj * nx + i0);
    const float4 vn = *reinterpret_cast<const float4 *>(f.v_star + (long)(lj + 1) * nx + i0);
    const float u0 = us[0], u1 = us[1], u2 = us[2], u3 = us[3], u4 = us[4];
    const float rdx = g.r_dx, rdy = g.r_dy, dx = g.dx, dy = g.dy;
    float4 r;
    r.x = (sdiv<SP>(u1 - u0, dx, rdx) + sdiv<SP>(vn.x - vs.x, dy, rdy)) / dt;
    r.y = (sdiv<SP>(u2 - u1, dx, rdx) + sdiv<SP>(vn.y - vs.y, dy, rdy)) / dt;
    r.z = (sdiv<SP>(u3 - u2, dx, rdx) + sdiv<SP>(vn.z - vs.z, dy, rdy)) / dt;
    r.w = (sdiv<SP>(u4 - u3, dx, rdx) + sdiv<SP>(vn.w - vs.w, dy, rdy)) / dt;
    *reinterpret_cast<float4 *>(f.rhs + (long)lj * nx + i0) = r;
}

// The head of a corrector-loop pass (model.rs:698-704): u* <- u, v* <- v and
// rhs = div(u*, v*) / dt in one pass.  The divergence is formed from the u
// and v values the copy has just read (they are the new u*, v*), so u* and v*
// are not read back: 20 B per cell instead of the 28 of k_copy_star +
// k_divergence, and one launch.  A thread owns 4 cells of one allocation row;
// ghost rows are copied too (k_copy_star copies whole allocations), owned rows
// also get rhs, with k_divergence's arithmetic bit for bit.
template <int SP>
__global__ __launch_bounds__(kBlock) void k_copy_star_div(Geom g, Fields f, int pass,
                                                          float dt_override, int nbx) {
    if (pass_off(f.ctl, pass)) return;
    const int bid = xcd_block(g);
    const int i0 = 4 * ((bid % nbx) * kBlock + (int)threadIdx.x);
    const int lr = bid / nbx - kGhostUV;   // local row: v rows -G..nyl+G, u rows -G..nyl+G-1
    const int nx = g.nx, W = nx + 1;
    if (i0 >= nx) return;
    const float4 vs = *reinterpret_cast<const float4 *>(f.v + (long)lr * nx + i0);
    *reinterpret_cast<float4 *>(f.v_star + (long)lr * nx + i0) = vs;
    if (lr >= g.nyl + kGhostUV) return;   // v's extra face row
    const float *__restrict__ ur = f.u + (long)lr * W + i0;
    float *__restrict__ us = f.u_star + (long)lr * W + i0;
    const float u0 = ur[0], u1 = ur[1], u2 = ur[2], u3 = ur[3], u4 = ur[4];
    us[0] = u0;
    us[1] = u1;
    us[2] = u2;
    us[3] = u3;
    if (i0 + 4 == nx) us[4] = u4;   // face nx
    if (lr < 0 || lr >= g.nyl) return;
    const float4 vn = *reinterpret_cast<const float4 *>(f.v + (long)(lr + 1) * nx + i0);
    const float dt = dt_of(f.ctl, dt_override);
    const float rdx = g.r_dx, rdy = g.r_dy, dx = g.dx, dy = g.dy;
    float4 r;
    r.x = (sdiv<SP>(u1 - u0, dx, rdx) + sdiv<SP>(vn.x - vs.x, dy, rdy)) / dt;
    r.y = (sdiv<SP>(u2 - u1, dx, rdx) + sdiv<SP>(vn.y - vs.y, dy, rdy)) / dt;
    r.z = (sdiv<SP>(u3 - u2, dx, rdx) + sdiv<SP>(vn.z - vs.z, dy, rdy)) / dt;
    r.w = (sdiv<SP>(u4 - u3, dx, rdx) + sdiv<SP>(vn.w - vs.w, dy, rdy)) / dt;
    *reinterpret_cast<float4 *>(f.rhs + (long)lr * nx + i0) = r;
}

// ------------------------------------------- predict + divergence (K1-K3)

// Both first-order predictors and the divergence in one pass (piso_step
// K1-K3: model.rs:538-670 and :1406-1440), over k_predict4r's tile: a lane
// owns 4 columns (i0 = 4c) and RPT rows lj0..lj0+RPT-1.  Besides u* and v* of
// those rows it predicts v* of row lj0 (the tile below owns it) and takes the
// east face u*(r, i0+4) from the lane on its right (DPP lane shift), so rhs
// of its own cells needs no u* / v* from memory: the divergence's re-read of
// u*, v* (8 B per cell) and a launch go, for one more v row in the window
// (RPT+3 rows of v, RPT+2 of u) and 1/RPT more v* arithmetic.  Lane 63 only
// feeds lane 62's east face, so waves step 63 chunks.  Faces the reference
// does not predict (face 0, column 0 of v, rows outside glo..u_hi / v_hi) take
// u* / v* from memory, as k_divergence reads them.  The arithmetic is
// u_pred_val / v_pred_val and k_divergence's, bit for bit.
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));

struct RAcc3 {   // stencil rows dj = -1, 0, +1 of u and of v, column q of four
    const float *u0, *u1, *u2, *v0, *v1, *v2;
    int q;
    __device__ __forceinline__ float U(int di, int dj) const {
        return (dj < 0 ? u0 : (dj == 0 ? u1 : u2))[q + 1 + di];
    }
    __device__ __forceinline__ float V(int di, int dj) const {
        return (dj < 0 ? v0 : (dj == 0 ? v1 : v2))[q + 1 + di];
    }
};

template <int SP, int RPT>
__global__ __launch_bounds__(kBlock) void k_predict_div(Geom g, Fields f, float dt_override,
                                                        int glo, int u_hi, int v_hi, int nwc,
                                                        int ntile) {
    const int nx = g.nx, W = nx + 1;
    const int bid = xcd_block(g);
    const int lane = (int)threadIdx.x & 63;
    const int wc = bid % nwc;
    const int tile = (bid / nwc) * (kBlock / 64) + ((int)threadIdx.x >> 6);
    if (tile >= ntile) return;   // wave-uniform
    const int lj0 = tile * RPT;
    const int c = wc * 63 + lane;
    const bool live = 4 * c < nx;
    const bool out = live && lane < 63;     // lanes that store
    const int i0 = live ? 4 * c : nx - 4;   // dead lanes compute on safe columns
    const int u_cap = u_hi + 1 > v_hi ? u_hi + 1 : v_hi;   // last u row any face reads
    const int v_cap = v_hi + 1;                            // last v row any face reads
    const float dt = dt_of(f.ctl, dt_override);
    const float rdx = g.r_dx, rdy = g.r_dy, dx = g.dx, dy = g.dy;
    // ur[k] = u row lj0-1+k, vr[k] = v row lj0-1+k; columns i0-1..i0+4
    float ur[RPT + 2][6], vr[RPT + 3][6];
#pragma unroll
    for (int k = 0; k < RPT + 2; ++k) {
        const int r = min(max(lj0 - 1 + k, glo - 1), u_cap);
        const float *p = f.u + (long)r * W + i0;
        ur[k][0] = i0 > 0 ? p[-1] : 0.0f;
        const f4u a = *reinterpret_cast<const f4u *>(p);
        ur[k][1] = a.x; ur[k][2] = a.y; ur[k][3] = a.z; ur[k][4] = a.w;
        ur[k][5] = p[4];
    }
#pragma unroll
    for (int k = 0; k < RPT + 3; ++k) {
        const int r = min(max(lj0 - 1 + k, glo - 1), v_cap);
        const float *p = f.v + (long)r * nx + i0;
        vr[k][0] = i0 > 0 ? p[-1] : 0.0f;
        const float4 a = *reinterpret_cast<const float4 *>(p);
        vr[k][1] = a.x; vr[k][2] = a.y; vr[k][3] = a.z; vr[k][4] = a.w;
        // column nx wraps to the next row's column 0 (flat index): only the
        // stencil's middle row (<= v_hi) needs it, and row v_hi + 1 exists
        vr[k][5] = (i0 + 4 < nx || r <= v_hi) ? p[4] : 0.0f;
    }
    const int r_end = min(lj0 + RPT, g.nyl);   // rhs rows lj0..r_end-1
    // v* rows lj0..lj0+RPT
    float vs[RPT + 1][4];
#pragma unroll
    for (int k = 0; k <= RPT; ++k) {
        const int rr = lj0 + k;
        if (rr >= glo && rr <= v_hi) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                vs[k][q] = v_pred_val<0, SP>(g, f, dt, i0 + q, rr,
                                             RAcc3{ur[k + 1], ur[k + 1], ur[k + 1], vr[k], vr[k + 1],
                                                   vr[k + 2], q});
            if (i0 == 0) vs[k][0] = f.v_star[(long)rr * nx];   // column 0 is not predicted
            // own rows lj0+1..r_end, and row lj0 of the lowest tile
            if (out && (k > 0 || lj0 == 0) && rr <= r_end) {
                float *d = f.v_star + (long)rr * nx + i0;
                if (i0 > 0) {
                    *reinterpret_cast<float4 *>(d) = make_float4(vs[k][0], vs[k][1], vs[k][2], vs[k][3]);
                } else {
                    d[1] = vs[k][1];
                    d[2] = vs[k][2];
                    d[3] = vs[k][3];
                }
            }
        } else if (rr <= r_end) {
            const float4 a = *reinterpret_cast<const float4 *>(f.v_star + (long)rr * nx + i0);
            vs[k][0] = a.x; vs[k][1] = a.y; vs[k][2] = a.z; vs[k][3] = a.w;
        }
    }
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const int r = lj0 + k;
        if (r >= r_end) break;   // wave-uniform
        float us[4];
        const bool upred = r >= glo && r <= u_hi;
        const long ku = (long)r * W + i0;
        if (upred) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                us[q] = u_pred_val<0, SP>(g, f, dt, i0 + q, r,
                                          RAcc3{ur[k], ur[k + 1], ur[k + 2], vr[k], vr[k + 1],
                                                vr[k + 2], q});
            if (i0 == 0) us[0] = f.u_star[ku];   // face 0 is not predicted
        } else {
            const f4u a = *reinterpret_cast<const f4u *>(f.u_star + ku);
            us[0] = a.x; us[1] = a.y; us[2] = a.z; us[3] = a.w;
        }
        float east = from_right(us[0]);
        if (i0 + 4 == nx) {
            if (upred) {
                const GAcc a{f.u, f.v, ku + 4, (long)r * nx + i0 + 4, W, nx};
                east = u_pred_val<0, SP>(g, f, dt, nx, r, a);
            } else {
                east = f.u_star[ku + 4];
            }
        }
        if (out) {
            if (upred) {
                float *d = f.u_star + ku;
                if (i0 > 0) d[0] = us[0];
                d[1] = us[1];
                d[2] = us[2];
                d[3] = us[3];
                if (i0 + 4 == nx) d[4] = east;
            }
            float4 rh;
            rh.x = (sdiv<SP>(us[1] - us[0], dx, rdx) + sdiv<SP>(vs[k + 1][0] - vs[k][0], dy, rdy)) / dt;
            rh.y = (sdiv<SP>(us[2] - us[1], dx, rdx) + sdiv<SP>(vs[k + 1][1] - vs[k][1], dy, rdy)) / dt;
            rh.z = (sdiv<SP>(us[3] - us[2], dx, rdx) + sdiv<SP>(vs[k + 1][2] - vs[k][2], dy, rdy)) / dt;
            rh.w = (sdiv<SP>(east - us[3], dx, rdx) + sdiv<SP>(vs[k + 1][3] - vs[k][3], dy, rdy)) / dt;
            *reinterpret_cast<float4 *>(f.rhs + (long)r * nx + i0) = rh;
        }
    }
}

// ---------------------------------------------------------------- Jacobi (K4)

// One weighted-Jacobi sweep (omega 0.75) with the p' boundary conditions
// fused into the stores (model.rs:748-815).
//
// Mapping: a wave owns 64 float4 column chunks (256 columns) of one row
// segment of R rows and marches up the segment, keeping rows j-1, j, j+1 in
// registers: p' and rhs are each read from HBM once per sweep, p'_new written
// once (12 B per cell-update), and horizontal neighbours come from adjacent
// lanes (__shfl) instead of re-reads.  Rows are processed 4 at a time with all
// 8 row loads of a group issued before any arithmetic.
//
// Boundary conditions, as stores (model.rs:807-815 applied after the swap):
// the reference's final values are P(0,j) = N(1,j), P(nx-1,j) = 0,
// P(i,0) = N(i,1), P(i,ny-1) = N(i,ny-2) for the freshly computed interior
// N — so column 0 takes column 1's value, column nx-1 stores 0, and the
// threads computing global rows 1 and ny-2 also store rows 0 and ny-1.
// Column nx-1's own update (which reads the wrapped P(0,j+1), Q5) is never
// stored, exactly as the reference overwrites it.
//
// Residual: max |N - P| over columns 1..=nx-8 only (the reference's full
// 8-lane chunks; the scalar tail :755-772 never updates max_error), owned
// rows only, NaN-ignoring like reduce_max.  One atomicMax per wave, into the
// sweep's spread slot set (only when `res`: a fixed-count solve needs the last
// sweep's residual alone).
template <int R, int FAST>
__global__ __launch_bounds__(kJacWavesPerBlock * 64) void k_jacobi(
    Geom g, float *__restrict__ pa, float *__restrict__ pb, const float *__restrict__ rhs,
    Ctl *ctl, uint32_t *slots, int pass, int it, int row_lo, int row_hi, int nbx, int res) {
    if (pass_off(ctl, pass)) return;
    // early exit of the previous sweep (model.rs:816): a skipped sweep leaves
    // its slots at 0 so every later sweep of the solve skips too.
    if (g.tol_enabled && it > 0 &&
        read_max(slots + (size_t)(it - 1) * kResSlots * kResStride, ctl->err[it - 1]) < g.p_tol)
        return;

    const int nx = g.nx, nch = nx >> 2, hg = g.hg, nyl = g.nyl;
    const int wave = (int)threadIdx.x >> 6, lane = (int)threadIdx.x & 63;
    const int bid = xcd_block(g);
    const int bx = bid % nbx, seg = bid / nbx;
    const int wcol = bx * kJacWavesPerBlock + wave;
    if (wcol * 64 >= nch) return;                         // wave-uniform
    const int ch = wcol * 64 + lane;
    const bool valid = ch < nch;
    const int r0 = row_lo + seg * R;
    const int r1 = min(r0 + R, row_hi);
    if (r0 >= r1) return;

    // pa/pb: the two p' allocations (first ghost row); (cur + it) picks the
    // source.  Loads go through buffer descriptors: a lane with nothing to
    // load gets an out-of-range offset and reads 0 without a branch.
    const int si = (ctl->cur + it) & 1;
    float *src_alloc = si ? pb : pa;
    float *dst_alloc = si ? pa : pb;
    const int pbytes = (nyl + 2 * hg) * nx * 4;
    const __amdgpu_buffer_rsrc_t rs_p =
        __builtin_amdgcn_make_buffer_rsrc(src_alloc, 0, pbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rs_r =
        __builtin_amdgcn_make_buffer_rsrc((void *)(rhs - (long)hg * nx), 0, pbytes, 0x00020000);
    float *__restrict__ dst = dst_alloc + (long)hg * nx;

    const float dx_sq = g.dx_sq, dy_sq = g.dy_sq, denom = g.denom;
    const float r_dx_sq = g.r_dx_sq, r_dy_sq = g.r_dy_sq, r_denom = g.r_denom;
    const float omega = 0.75f;
    const float om1 = 1.0f - omega;

    constexpr int kOOB = -16;   // >= num_records as unsigned: reads 0
    const int col = 4 * ch;
    const int row_bytes = nx * 4;
    // byte offsets at local row 0 (p' offsets include the hg ghost rows)
    const int off_p = valid ? (hg * nx + col) * 4 : kOOB;
    const int off_r = valid ? (hg * nx + col) * 4 : kOOB;
    const int off_l = (lane == 0 && ch > 0 && valid) ? (hg * nx + col - 1) * 4 : kOOB;
    const int off_rt = (lane == 63 && ch + 1 < nch) ? (hg * nx + col + 4) * 4 : kOOB;
    const bool e0 = (col >= 1) && (col <= nx - 8);   // residual columns 1..=nx-8
    const bool e1 = (col + 1 <= nx - 8);
    const bool e2 = (col + 2 <= nx - 8);
    const bool e3 = (col + 3 <= nx - 8);
    const int gj_first = 1 - g.j0, gj_last = g.ny - 2 - g.j0;   // local rows of global 1, ny-2

    auto ld4 = [&](const __amdgpu_buffer_rsrc_t &rs, int off, int row) -> float4 {
        const int o = off < 0 ? off : off + row * row_bytes;
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0);
        return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                           __uint_as_float(v.w));
    };
    auto ld1 = [&](int off, int row) -> float {
        const int o = off < 0 ? off : off + row * row_bytes;
        return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_p, o, 0, 0));
    };

    float m = 0.0f;
    // sliding window: w0..w5 = p' rows j-1 .. j+4 of the current 4-row group;
    // rows past r1 are clamped to r1 (always inside the allocation, unused)
    float4 w0 = ld4(rs_p, off_p, r0 - 1);
    float4 w1 = ld4(rs_p, off_p, r0);
    for (int j = r0; j < r1; j += 4) {
        const bool l1 = j + 1 < r1, l2 = j + 2 < r1, l3 = j + 3 < r1;
        const int j1c = l1 ? j + 1 : j, j2c = l2 ? j + 2 : j, j3c = l3 ? j + 3 : j;
        // issue every load of the group before any arithmetic
        const float4 w2 = ld4(rs_p, off_p, j + 1);
        const float4 w3 = ld4(rs_p, off_p, j1c + 1);
        const float4 w4 = ld4(rs_p, off_p, j2c + 1);
        const float4 w5 = ld4(rs_p, off_p, j3c + 1);
        const float4 h0 = ld4(rs_r, off_r, j);
        const float4 h1 = ld4(rs_r, off_r, j1c);
        const float4 h2 = ld4(rs_r, off_r, j2c);
        const float4 h3 = ld4(rs_r, off_r, j3c);
        const float lf0 = ld1(off_l, j), lf1 = ld1(off_l, j1c), lf2 = ld1(off_l, j2c),
                    lf3 = ld1(off_l, j3c);
        const float rt0 = ld1(off_rt, j), rt1 = ld1(off_rt, j1c), rt2 = ld1(off_rt, j2c),
                    rt3 = ld1(off_rt, j3c);

        auto row_update = [&](int row, const float4 &B, const float4 &C, const float4 &T,
                              const float4 &Rh, float lf, float rt) {
            const float horiz_l = __shfl_up(C.w, 1, 64);
            const float horiz_r = __shfl_down(C.x, 1, 64);
            const float L0 = (lane == 0) ? lf : horiz_l;
            const float R3 = (lane == 63) ? rt : horiz_r;
            const float cc[4] = {C.x, C.y, C.z, C.w};
            const float rr[4] = {C.y, C.z, C.w, R3};
            const float ll[4] = {L0, C.x, C.y, C.z};
            const float tt[4] = {T.x, T.y, T.z, T.w};
            const float bb[4] = {B.x, B.y, B.z, B.w};
            const float hh[4] = {Rh.x, Rh.y, Rh.z, Rh.w};
            float n[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float horizontal = fdiv<FAST>(rr[k] + ll[k], dx_sq, r_dx_sq);
                const float vertical = fdiv<FAST>(tt[k] + bb[k], dy_sq, r_dy_sq);
                const float p_update = fdiv<FAST>(horizontal + vertical - hh[k], denom, r_denom);
                n[k] = omega * p_update + om1 * cc[k];
            }
            if (row >= 0 && row < nyl) {
                if (e0) m = fmaxf(m, fabsf(n[0] - cc[0]));
                if (e1) m = fmaxf(m, fabsf(n[1] - cc[1]));
                if (e2) m = fmaxf(m, fabsf(n[2] - cc[2]));
                if (e3) m = fmaxf(m, fabsf(n[3] - cc[3]));
            }
            float4 o = make_float4(n[0], n[1], n[2], n[3]);
            if (ch == 0) o.x = n[1];          // P(0,j) = P(1,j)
            if (ch == nch - 1) o.w = 0.0f;    // P(nx-1,j) = 0
            if (valid) {
                *reinterpret_cast<float4 *>(dst + (long)row * nx + col) = o;
                if (row == gj_first)          // P(i,0) = P(i,1)
                    *reinterpret_cast<float4 *>(dst + (long)(row - 1) * nx + col) = o;
                if (row == gj_last)           // P(i,ny-1) = P(i,ny-2)
                    *reinterpret_cast<float4 *>(dst + (long)(row + 1) * nx + col) = o;
            }
        };
        row_update(j, w0, w1, w2, h0, lf0, rt0);
        if (l1) row_update(j + 1, w1, w2, w3, h1, lf1, rt1);
        if (l2) row_update(j + 2, w2, w3, w4, h2, lf2, rt2);
        if (l3) row_update(j + 3, w3, w4, w5, h3, lf3, rt3);
        w0 = w4;
        w1 = w5;
    }
    if (!res) return;
    m = wave_max(m);
    if (lane == 0) publish_max(slots + (size_t)it * kResSlots * kResStride, bid * kJacWavesPerBlock + wave, m);
}

// (solve_finalize_body: cfd_device.h, shared with the resident solve).
// r6: 1,024 threads -- a tolerance-mode solve's finalize folds and clears
// every sweep's 32 residual slots (50 sets), one set per wave at a time: 16
// waves take 4 rounds of slot reads instead of 13 (C3 in the reference's
// control flow spent 12.9 us per solve here, 21 solves per step).
constexpr int kFinThreads = 1024;
__global__ __launch_bounds__(kFinThreads) void k_finalize_solve(Geom g, Fields f, int pass, int iters,
                                                           int check_break, int flips,
                                                           int exact_flips) {
    solve_finalize_body(g, f, pass, iters, check_break, flips, exact_flips);
}

// After the speculative launch covering sweeps [it, it+T) (launch_jacobi_spec):
// fold its T residual slot sets into Ctl::err, and find the first of its
// sweeps whose residual is below p_tol (model.rs:816).  That sweep ends the
// solve: later launches skip (spec_stop), and unless it is the launch's last
// sweep the launch is re-run with exactly that many sweeps (spec_redo).
__global__ __launch_bounds__(kBlock) void k_spec_check(Geom g, Fields f, int pass, int it, int T,
                                                       int par) {
    Ctl *c = f.ctl;
    if (pass_off(c, pass) || c->spec_stop) return;
    const int wv = (int)threadIdx.x >> 6, nw = (int)blockDim.x >> 6;
    for (int k = it + wv; k < it + T; k += nw) {
        uint32_t *set = f.err_slots + (size_t)k * kResSlots * kResStride;
        const float v = read_max(set, c->err[k]);
        if ((threadIdx.x & 63) < kResSlots) set[(threadIdx.x & 63) * kResStride] = 0u;
        if ((threadIdx.x & 63) == 0) c->err[k] = __float_as_uint(v);
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    int j = 0;
    while (j < T && !(__uint_as_float(c->err[it + j]) < g.p_tol)) ++j;
    c->spec_launches = par + 1;
    if (j < T) {
        c->spec_stop = 1;
        c->spec_launch = par;
        c->spec_redo = j + 1 < T ? j + 1 : 0;
    }
}

// The speculative solve on slabs (r5): the host counts every launch of the
// solve as a buffer flip (it must know which buffer's ghost rows to exchange
// before each launch), so when a launch L < n-1 converged and its re-run
// left the result in buffer cur + L + 1 of the other parity, that buffer's
// owned rows are copied to buffer cur + n (the ghost rows are re-exchanged
// before they are read again).
__global__ __launch_bounds__(kBlock) void k_spec_align(Geom g, Fields f, int pass, int n) {
    const Ctl *c = f.ctl;
    if (pass_off(c, pass) || !c->spec_stop) return;
    const int L = c->spec_launch;
    if (((n - (L + 1)) & 1) == 0) return;
    const float4 *src = reinterpret_cast<const float4 *>(f.pp[(c->cur + L + 1) & 1]);
    float4 *dst = reinterpret_cast<float4 *>(f.pp[(c->cur + n) & 1]);
    const size_t n4 = (size_t)g.nyl * g.nx / 4;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

// dst[q] = max(dst[q], slots of set q), then zero the slots (q < n).
__global__ void k_fold_slots(uint32_t *dst, uint32_t *slots, int n) {
    const int q = (int)threadIdx.x;
    if (q >= n) return;
    uint32_t *set = slots + (size_t)q * kResSlots * kResStride;
    uint32_t v = dst[q];
    for (int s = 0; s < kResSlots; ++s) {
        v = max(v, set[s * kResStride]);
        set[s * kResStride] = 0u;
    }
    dst[q] = v;
}

// ------------------------------------------------------------- corrector (K5)

// apply_corrector (model.rs:1334-1404).  u: all owned rows, faces 1..nx-1;
// faces nx-7..nx-1 are the scalar tail and associate (dt * dp) / dx (Q9).
// v: global rows 1..=ny-1 held by this slab (incl. the shared face row).
// p += p'.
template <int SP>
__global__ __launch_bounds__(kBlock) void k_corrector(Geom g, Fields f, int pass,
                                                      float dt_override, int nbx) {
    Ctl *c = f.ctl;
    if (pass_off(c, pass)) return;
    const int bid = xcd_block(g);
    const int i = (bid % nbx) * kBlock + (int)threadIdx.x;   // 0..nx
    const int lj = bid / nbx;                                // 0..nyl
    const int nx = g.nx, W = nx + 1;
    if (i > nx) return;
    const float dt = dt_of(c, dt_override);
    const float *__restrict__ pp = c->cur ? f.pp[1] : f.pp[0];
    const int j = g.j0 + lj;
    if (lj < g.nyl && i >= 1 && i <= nx - 1) {
        const float p_right = pp[(long)lj * nx + i];
        const float p_left = pp[(long)lj * nx + i - 1];
        const long k = (long)lj * W + i;
        if (i >= nx - 7)
            f.u[k] = f.u_star[k] - sdiv<SP>(dt * (p_right - p_left), g.dx, g.r_dx);
        else
            f.u[k] = f.u_star[k] - dt * sdiv<SP>(p_right - p_left, g.dx, g.r_dx);
    }
    if (i < nx && j >= 1 && j <= g.ny - 1) {
        const float p_top = pp[(long)lj * nx + i];
        const float p_bottom = pp[(long)(lj - 1) * nx + i];
        const long k = (long)lj * nx + i;
        f.v[k] = f.v_star[k] - dt * sdiv<SP>(p_top - p_bottom, g.dy, g.r_dy);
    }
    if (i < nx && lj < g.nyl) {
        const long k = (long)lj * nx + i;
        f.p[k] = f.p[k] + pp[k];
    }
}

// k_corrector with a thread per 4 consecutive cells of a row: the p', v, v*
// and p rows (pitch nx, 16-byte aligned) move as float4, the u / u* row
// (pitch nx+1) as scalars; the left neighbour p'(i0-1) of the first u face is
// one more scalar load.  The same expressions per face and cell as
// k_corrector (Q9 tail included), so the same bits; one float per thread held
// the corrector at ~4 TB/s.
template <int SP>
__global__ __launch_bounds__(kBlock) void k_corrector4(Geom g, Fields f, int pass,
                                                       float dt_override, int nbx) {
    Ctl *c = f.ctl;
    if (pass_off(c, pass)) return;
    const int bid = xcd_block(g);
    const int i0 = 4 * ((bid % nbx) * kBlock + (int)threadIdx.x);   // cells i0..i0+3
    const int lj = bid / nbx;                                       // 0..nyl
    const int nx = g.nx, W = nx + 1;
    if (i0 >= nx) return;
    const float dt = dt_of(c, dt_override);
    const float *__restrict__ pp = c->cur ? f.pp[1] : f.pp[0];
    const int j = g.j0 + lj;
    const long kc = (long)lj * nx + i0;
    float4 pc = {0.f, 0.f, 0.f, 0.f};
    if (lj < g.nyl) {
        pc = *reinterpret_cast<const float4 *>(pp + kc);
        const float pl = i0 > 0 ? pp[kc - 1] : 0.0f;
        const float pr[4] = {pc.x, pc.y, pc.z, pc.w};
        const float pw[4] = {pl, pc.x, pc.y, pc.z};
        const long ku = (long)lj * W + i0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = i0 + q;
            if (i < 1 || i > nx - 1) continue;
            if (i >= nx - 7)
                f.u[ku + q] = f.u_star[ku + q] - sdiv<SP>(dt * (pr[q] - pw[q]), g.dx, g.r_dx);
            else
                f.u[ku + q] = f.u_star[ku + q] - dt * sdiv<SP>(pr[q] - pw[q], g.dx, g.r_dx);
        }
    }
    if (j >= 1 && j <= g.ny - 1) {
        const float4 pt = lj < g.nyl ? pc : *reinterpret_cast<const float4 *>(pp + kc);
        const float4 pb = *reinterpret_cast<const float4 *>(pp + kc - nx);
        const float4 vs = *reinterpret_cast<const float4 *>(f.v_star + kc);
        float4 o;
        o.x = vs.x - dt * sdiv<SP>(pt.x - pb.x, g.dy, g.r_dy);
        o.y = vs.y - dt * sdiv<SP>(pt.y - pb.y, g.dy, g.r_dy);
        o.z = vs.z - dt * sdiv<SP>(pt.z - pb.z, g.dy, g.r_dy);
        o.w = vs.w - dt * sdiv<SP>(pt.w - pb.w, g.dy, g.r_dy);
        *reinterpret_cast<float4 *>(f.v + kc) = o;
    }
    if (lj < g.nyl) {
        float4 pv = *reinterpret_cast<const float4 *>(f.p + kc);
        pv.x = pv.x + pc.x;
        pv.y = pv.y + pc.y;
        pv.z = pv.z + pc.z;
        pv.w = pv.w + pc.w;
        *reinterpret_cast<float4 *>(f.p + kc) = pv;
    }
}

// The corrector of pass k fused with the head of pass k+1 (model.rs:693 +
// 698-704: apply_corrector, then u* <- u, v* <- v and rhs = div(u*, v*)/dt)
// when the device says pass k+1 runs (Ctl::go[pass+1], set by the solve's
// finalize before this launch); otherwise the plain corrector.  Single domain,
// one thread per 4 cells of an allocation row.
//
// The corrected velocities go straight into the next pass's u* / v*, and
// u / v get their final values only from the loop's last corrector: every
// pass's corrector overwrites every corrected face of u and v and leaves the
// others (u faces 0 and nx, v rows 0 and ny, ghost rows) as they are, which is
// also what the copies give u* / v* there.  The divergence of a row needs the
// corrected east face u(i0+4) of the next thread and v of the next row: both
// are recomputed here from the corrector's inputs with its own expressions
// (the same bits), so those inputs must not be overwritten by this launch --
// the passes alternate arrays.  Pass k reads its u* / v* from u_star / v_star
// when k is even and from u / v when k is odd, and writes the corrected values
// to the other pair:
//   head, k even: u_star -> u (u already holds u at the uncorrected places);
//   head, k odd:  u -> u_star (plus u* <- u at the uncorrected places, ghost
//                 rows included, as k_copy_star_div does);
//   last, k even: k_corrector4 (u <- u_star - corr);
//   last, k odd:  u_star <- u everywhere (the reference's u* of the last
//                 pass), then u <- u - corr in place (elementwise).
// p += p' in every pass.  32 B per cell (read u*, v*, p', p; write the other
// pair, p, rhs) against 48 for k_corrector4 + k_copy_star_div, and one launch
// per pass fewer.
template <int SP>
__device__ __forceinline__ float u_corr(const Geom &g, float us, float pr, float pw, float dt, int i) {
    // model.rs:1336-1362; faces nx-7..nx-1 are the scalar tail: (dt * dp) / dx (Q9)
    return i >= g.nx - 7 ? us - sdiv<SP>(dt * (pr - pw), g.dx, g.r_dx)
                         : us - dt * sdiv<SP>(pr - pw, g.dx, g.r_dx);
}

// ROWS allocation rows per thread (r6: a band march of kCfRows rows, as
// k_correct_finish4m): row lr's p' row, its v correction and the p' row below
// it come from row lr-1's iteration -- the v_row of row lr+1 that the
// divergence needs is the next row's vlo, the p' row lr+1 it loads the next
// row's pc -- instead of every row re-reading three p' rows and two v* rows
// and computing two v rows.  The same expressions on the same inputs: bitwise
// the one-row form (ROWS = 1).
template <int SP, int ROWS>
__global__ __launch_bounds__(kBlock) void k_correct_head4(Geom g, Fields f, int pass,
                                                          float dt_override, int nbx, int has_next) {
    Ctl *c = f.ctl;
    if (pass_off(c, pass)) return;
    // pass+1 exists (host) and runs (device: the early exit, model.rs:721)
    const bool head = has_next && c->go[pass + 1] != 0;
    const bool odd = pass & 1;
    const float *__restrict__ in_u = odd ? f.u : f.u_star;   // this pass's u*
    const float *__restrict__ in_v = odd ? f.v : f.v_star;
    float *__restrict__ out_u = odd ? f.u_star : f.u;        // the next pass's u*
    float *__restrict__ out_v = odd ? f.v_star : f.v;
    const int bid = xcd_block(g);
    const int i0 = 4 * ((bid % nbx) * kBlock + (int)threadIdx.x);
    const int nx = g.nx, W = nx + 1, nyl = g.nyl;
    if (i0 >= nx) return;
    const float dt = dt_of(c, dt_override);
    const float *__restrict__ pp = c->cur ? f.pp[1] : f.pp[0];
    auto v_row = [&](int r, const float4 &pt, bool *hit) -> float4 {
        const int jr = g.j0 + r;
        const long k = (long)r * nx + i0;
        *hit = jr >= 1 && jr <= g.ny - 1;   // model.rs:1366: rows 1..ny-1
        if (!*hit) return *reinterpret_cast<const float4 *>(f.v + k);
        const float4 pb = *reinterpret_cast<const float4 *>(pp + k - nx);
        const float4 vs = *reinterpret_cast<const float4 *>(in_v + k);
        float4 o;
        o.x = vs.x - dt * sdiv<SP>(pt.x - pb.x, g.dy, g.r_dy);
        o.y = vs.y - dt * sdiv<SP>(pt.y - pb.y, g.dy, g.r_dy);
        o.z = vs.z - dt * sdiv<SP>(pt.z - pb.z, g.dy, g.r_dy);
        o.w = vs.w - dt * sdiv<SP>(pt.w - pb.w, g.dy, g.r_dy);
        return o;
    };
    // allocation rows: v rows -G..nyl+G, u rows -G..nyl+G-1
    const int lr0 = (bid / nbx) * ROWS - kGhostUV, lr1 = min(lr0 + ROWS, nyl + 1 + kGhostUV);
    bool carry = false;          // p' row lr and v row lr from row lr-1's iteration
    float4 p_next = {0.f, 0.f, 0.f, 0.f}, v_next = {0.f, 0.f, 0.f, 0.f};
    // an owned head row's loads: p' row r, its west / east neighbours (clamped
    // in-row addresses, the edge lanes' values selected by the caller), u* row
    // r, p' row r+1, v* row r+1 (v where row r+1 is not corrected), p row r
    struct HRow {
        float4 pld, pt, vsn, pv;
        f4u iu;
        float iu4, plv, p4v;
    };
    HRow cur, nxt;
    bool have = false;   // cur holds row lr's loads
    auto load_hrow = [&](int r, HRow &h) {
        const long kc = (long)r * nx + i0, ku = (long)r * W + i0;
        h.pld = *reinterpret_cast<const float4 *>(pp + kc);
        h.plv = pp[kc - (i0 > 0 ? 1 : 0)];
        h.p4v = pp[kc + (i0 + 4 < nx ? 4 : 3)];
        h.iu = *reinterpret_cast<const f4u *>(in_u + ku);   // dword-aligned (pitch nx + 1)
        h.iu4 = in_u[ku + 4];
        h.pt = *reinterpret_cast<const float4 *>(pp + kc + nx);
        const int jr = g.j0 + r + 1;   // model.rs:1366: v rows 1..ny-1 are corrected
        h.vsn = *reinterpret_cast<const float4 *>((jr >= 1 && jr <= g.ny - 1 ? in_v : f.v) + kc + nx);
        h.pv = *reinterpret_cast<const float4 *>(f.p + kc);
    };
    for (int lr = lr0; lr < lr1; ++lr) {
        const long kc = (long)lr * nx + i0, ku = (long)lr * W + i0;
        const bool owned = lr >= 0 && lr < nyl;
        // u* <- u and v* <- v of the whole row (the next pass's u* at places no
        // corrector writes, or the last odd pass's u*): only when u* is out of date
        if (odd && (!head || !owned)) {
            *reinterpret_cast<float4 *>(f.v_star + kc) = *reinterpret_cast<const float4 *>(f.v + kc);
            if (lr < nyl + kGhostUV) {   // not v's extra face row
                const float *__restrict__ ur = f.u + ku;
                float *__restrict__ us = f.u_star + ku;
                *reinterpret_cast<f4u *>(us) = *reinterpret_cast<const f4u *>(ur);
                if (i0 + 4 == nx) us[4] = ur[4];   // face nx
            }
        }
        if (!owned && (head || lr != nyl)) {
            carry = false;
            have = false;
            continue;
        }
        if (!head) {
            // the loop's last corrector: u, v, p final (rows 0..nyl; v's row nyl)
            float4 pc = {0.f, 0.f, 0.f, 0.f};
            if (owned) {
                pc = *reinterpret_cast<const float4 *>(pp + kc);
                const float pl = i0 > 0 ? pp[kc - 1] : 0.0f;
                const float pr[4] = {pc.x, pc.y, pc.z, pc.w};
                const float pw[4] = {pl, pc.x, pc.y, pc.z};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int i = i0 + q;
                    if (i < 1 || i > nx - 1) continue;
                    f.u[ku + q] = u_corr<SP>(g, in_u[ku + q], pr[q], pw[q], dt, i);
                }
            }
            bool hit;
            const float4 o = v_row(lr, owned ? pc : *reinterpret_cast<const float4 *>(pp + kc), &hit);
            if (hit) *reinterpret_cast<float4 *>(f.v + kc) = o;
            if (owned) {
                float4 pv = *reinterpret_cast<const float4 *>(f.p + kc);
                pv.x = pv.x + pc.x;
                pv.y = pv.y + pc.y;
                pv.z = pv.z + pc.z;
                pv.w = pv.w + pc.w;
                *reinterpret_cast<float4 *>(f.p + kc) = pv;
            }
            carry = false;
            have = false;
            continue;
        }
        // ---- an owned row: corrector k, then pass k+1's copy and divergence
        // Row lr's loads were issued during row lr-1 (cur) unless this is the
        // band's first owned row; row lr+1's go out now, before row lr's
        // stores (no array this row stores is one the next row loads at the
        // same place), so each row's loads overlap the previous row's work.
        if (!have) load_hrow(lr, cur);
        const bool pf = ROWS > 1 && lr + 1 < lr1 && lr + 1 < nyl;   // the next row is owned too
        if (pf) load_hrow(lr + 1, nxt);
        // p' row lr: loaded every row and the carried copy selected, so no
        // branch guards the load; the edge lanes' values selected likewise
        const float4 pc = carry ? p_next : cur.pld;
        const float pl = i0 > 0 ? cur.plv : 0.0f;
        const float p4 = i0 + 4 < nx ? cur.p4v : 0.0f;   // for the east face i0+4
        const float pr[5] = {pc.x, pc.y, pc.z, pc.w, p4};
        const float pw[5] = {pl, pc.x, pc.y, pc.z, pc.w};
        float un[5];
        const float iuq[5] = {cur.iu.x, cur.iu.y, cur.iu.z, cur.iu.w, cur.iu4};
#pragma unroll
        for (int q = 0; q < 5; ++q) un[q] = u_corr<SP>(g, iuq[q], pr[q], pw[q], dt, i0 + q);
        // faces 0 and nx keep u (the only lanes whose i0 + q leaves 1..nx-1)
        if (i0 == 0) un[0] = f.u[ku];
        if (i0 + 4 == nx) un[4] = f.u[ku + 4];
        *reinterpret_cast<f4u *>(out_u + ku) = (f4u){un[0], un[1], un[2], un[3]};
        if (i0 + 4 == nx) out_u[ku + 4] = un[4];
        bool hit;
        const float4 vlo = carry ? v_next : v_row(lr, pc, &hit);
        const float4 pt = cur.pt;
        // v row lr+1 (v_row's expression; its p' row below is pc)
        float4 vhi = cur.vsn;
        {
            const int jr = g.j0 + lr + 1;
            if (jr >= 1 && jr <= g.ny - 1) {
                vhi.x = cur.vsn.x - dt * sdiv<SP>(pt.x - pc.x, g.dy, g.r_dy);
                vhi.y = cur.vsn.y - dt * sdiv<SP>(pt.y - pc.y, g.dy, g.r_dy);
                vhi.z = cur.vsn.z - dt * sdiv<SP>(pt.z - pc.z, g.dy, g.r_dy);
                vhi.w = cur.vsn.w - dt * sdiv<SP>(pt.w - pc.w, g.dy, g.r_dy);
            }
        }
        *reinterpret_cast<float4 *>(out_v + kc) = vlo;
        float4 pv = cur.pv;
        pv.x = pv.x + pc.x;
        pv.y = pv.y + pc.y;
        pv.z = pv.z + pc.z;
        pv.w = pv.w + pc.w;
        *reinterpret_cast<float4 *>(f.p + kc) = pv;
        const float rdx = g.r_dx, rdy = g.r_dy, dx = g.dx, dy = g.dy;
        float4 r;   // k_divergence's expression on the new u*, v*
        r.x = (sdiv<SP>(un[1] - un[0], dx, rdx) + sdiv<SP>(vhi.x - vlo.x, dy, rdy)) / dt;
        r.y = (sdiv<SP>(un[2] - un[1], dx, rdx) + sdiv<SP>(vhi.y - vlo.y, dy, rdy)) / dt;
        r.z = (sdiv<SP>(un[3] - un[2], dx, rdx) + sdiv<SP>(vhi.z - vlo.z, dy, rdy)) / dt;
        r.w = (sdiv<SP>(un[4] - un[3], dx, rdx) + sdiv<SP>(vhi.w - vlo.w, dy, rdy)) / dt;
        *reinterpret_cast<float4 *>(f.rhs + kc) = r;
        if (pf) cur = nxt;
        have = pf;
        carry = ROWS > 1;
        p_next = pt;
        v_next = vhi;
    }
}

// ------------------------------------------------- velocity boundaries (K6)

// Inlet face value of row j (model.rs:830-846): uniform or parabolic, >= 0.
__device__ __forceinline__ float inlet_value(const Geom &g, float inlet, int j) {
    if (g.profile == 0) return inlet;
    const float y = ((float)j + 0.5f) * g.dy;
    const float center = g.ly / 2.0f;
    const float radius = g.ly / 2.0f;
    const float q = (y - center) / radius;
    const float pv = inlet * (1.0f - q * q);
    return pv < 0.0f ? 0.0f : pv;
}

// apply_boundary_conditions (model.rs:826-875), in the reference's order; a
// single workgroup with barriers between the phases that touch the same
// faces.  bc_kind 1 = build-defined lid-driven cavity.
__global__ __launch_bounds__(1024) void k_boundary(Geom g, Fields f) {
    const int nx = g.nx, W = nx + 1, nyl = g.nyl;
    const float inlet = f.ctl->inlet;
    float *__restrict__ u = f.u;
    float *__restrict__ v = f.v;
    const int t = threadIdx.x, nt = blockDim.x;
    for (int lj = t; lj < nyl; lj += nt) {
        const int j = g.j0 + lj;
        if (g.bc_kind == 0) {
            u[(long)lj * W] = inlet_value(g, inlet, j);
            u[(long)lj * W + nx] = u[(long)lj * W + nx - 1];
        } else {
            u[(long)lj * W] = 0.0f;
            u[(long)lj * W + nx] = 0.0f;
        }
    }
    __syncthreads();
    const bool has_bottom = g.j0 == 0;
    const bool has_top = g.j0 + nyl == g.ny;
    for (int i = t; i <= nx; i += nt) {
        if (has_bottom) u[i] = 0.0f;
        if (has_top) {
            const float lid = (g.bc_kind == 1 && i > 0 && i < nx) ? inlet : 0.0f;
            u[(long)(nyl - 1) * W + i] = lid;
        }
    }
    for (int i = t; i < nx; i += nt) {
        if (has_bottom) v[i] = 0.0f;
        if (has_top) v[(long)nyl * nx + i] = 0.0f;
    }
    __syncthreads();
    for (int k = t; k < f.n_obs; k += nt) {
        const int oi = f.obs[2 * k], oj = f.obs[2 * k + 1];
        const int lj = oj - g.j0;
        if (lj >= 0 && lj < nyl) u[(long)lj * W + oi] = 0.0f;
        if (lj >= 0 && lj <= nyl) v[(long)lj * nx + oi] = 0.0f;
    }
}

// ------------------------------- fused corrector + boundaries + reductions (K5')

// update() with no extra corrector passes (model.rs:707-730 with
// corrector_passes 0): the one corrector pass (apply_corrector :1334-1404),
// the velocity boundaries (apply_boundary_conditions :827-875) and the step
// residuals/CFL maxima (:333-344, :879-880) in a single pass over the fields.
// Each thread writes the FINAL value of its u face and v face — the value the
// reference holds after the boundary routine has run in its order (columns,
// then rows over the corners, then obstacle faces) — and, because u/v are not
// touched between step start and here, the value it overwrites IS u_old/v_old:
// |new - old| needs no copy of the old fields and no second read.  Obstacle
// faces are bit 1 of the device masks.  Same grid as k_corrector.
template <int SP>
__global__ __launch_bounds__(kBlock) void k_correct_finish(Geom g, Fields f, float dt_override,
                                                           int nbx) {
    Ctl *c = f.ctl;
    const int nx = g.nx, W = nx + 1;
    float du = 0.f, dv = 0.f, mu = 0.f, mv = 0.f;
    bool bad = false;
    // each block walks a contiguous run of (row, 256-column) tiles, so the
    // residual maxima leave the block as 4 atomics, not 4 per wave per tile
    const long ntiles = (long)nbx * (g.nyl + 1);
    const int bid = xcd_block(g), G = (int)gridDim.x;
    const long t_lo = ntiles * bid / G, t_hi = ntiles * (bid + 1) / G;
    for (long t = t_lo; t < t_hi; ++t) {
        const int i = (int)(t % nbx) * kBlock + (int)threadIdx.x;   // 0..nx
        const int lj = (int)(t / nbx);                               // 0..nyl
        if (i <= nx) {
            const float dt = dt_of(c, dt_override);
            const float *__restrict__ pp = c->cur ? f.pp[1] : f.pp[0];
            const int j = g.j0 + lj;
            const long rp = (long)lj * nx;
            if (lj < g.nyl) {
                const long k = (long)lj * W + i;
                float nw;
                if (j == 0) {
                    nw = 0.0f;
                } else if (j == g.ny - 1) {
                    nw = (g.bc_kind == 1 && i > 0 && i < nx) ? c->inlet : 0.0f;
                } else if (i == 0) {
                    nw = g.bc_kind == 0 ? inlet_value(g, c->inlet, j) : 0.0f;
                } else if (i == nx) {
                    // outflow copies the corrected face nx-1 (scalar tail association, Q9)
                    nw = g.bc_kind == 0
                             ? f.u_star[k - 1] - sdiv<SP>(dt * (pp[rp + nx - 1] - pp[rp + nx - 2]),
                                                          g.dx, g.r_dx)
                             : 0.0f;
                } else {
                    const float p_right = pp[rp + i];
                    const float p_left = pp[rp + i - 1];
                    nw = (i >= nx - 7) ? f.u_star[k] - sdiv<SP>(dt * (p_right - p_left), g.dx, g.r_dx)
                                       : f.u_star[k] - dt * sdiv<SP>(p_right - p_left, g.dx, g.r_dx);
                }
                if (f.n_obs > 0 && (f.mask_u[k] & 2)) nw = 0.0f;
                const float old = f.u[k];
                f.u[k] = nw;
                du = fmaxf(du, fabsf(nw - old));
                mu = fmaxf(mu, fabsf(nw));
                bad |= nonfinite(nw);
            }
            if (i < nx) {
                const long k = rp + i;
                float nw;
                if (j == 0 || j == g.ny) {
                    nw = 0.0f;
                } else {
                    const float p_top = pp[k];
                    const float p_bottom = pp[k - nx];
                    nw = f.v_star[k] - dt * sdiv<SP>(p_top - p_bottom, g.dy, g.r_dy);
                }
                if (f.n_obs > 0 && (f.mask_v[k] & 2)) nw = 0.0f;
                const float old = f.v[k];
                f.v[k] = nw;
                dv = fmaxf(dv, fabsf(nw - old));
                mv = fmaxf(mv, fabsf(nw));
                bad |= nonfinite(nw);
                if (lj < g.nyl) f.p[k] = f.p[k] + pp[k];
            }
        }
    }
    flag_nonfinite(c, bad);
    __shared__ float red[kBlock / 64][4];
    du = wave_max(du);
    dv = wave_max(dv);
    mu = wave_max(mu);
    mv = wave_max(mv);
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[wv][0] = du;
        red[wv][1] = dv;
        red[wv][2] = mu;
        red[wv][3] = mv;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        float r = 0.f;
#pragma unroll
        for (int w = 0; w < kBlock / 64; ++w) r = fmaxf(r, red[w][threadIdx.x]);
        publish_max(f.red_slots + (size_t)threadIdx.x * kResSlots * kResStride, bid, r);
    }
}

// Final u face value at (i, j) of k_correct_finish, from its operands:
// ustar = u_star at the face (u_star of face nx-1 for the outflow face nx),
// p_right / p_left = the p' cells either side (p'(nx-1), p'(nx-2) for face nx).
template <int SP>
__device__ __forceinline__ float cf_u_face(const Geom &g, float inlet, float dt, int i, int j,
                                           float ustar, float p_right, float p_left) {
    const int nx = g.nx;
    if (j == 0) return 0.0f;
    if (j == g.ny - 1) return (g.bc_kind == 1 && i > 0 && i < nx) ? inlet : 0.0f;
    if (i == 0) return g.bc_kind == 0 ? inlet_value(g, inlet, j) : 0.0f;
    if (i == nx)
        return g.bc_kind == 0 ? ustar - sdiv<SP>(dt * (p_right - p_left), g.dx, g.r_dx) : 0.0f;
    return (i >= nx - 7) ? ustar - sdiv<SP>(dt * (p_right - p_left), g.dx, g.r_dx)
                         : ustar - dt * sdiv<SP>(p_right - p_left, g.dx, g.r_dx);
}

// k_correct_finish with four columns per thread: the pitch-nx streams (p', p,
// v*, v) move as float4, the pitch-(nx+1) u streams as four consecutive
// scalars, and the thread owning columns nx-4..nx-1 also finishes u face nx.
// Same values and maxima as k_correct_finish (one float per thread held the
// kernel near 4.7 TB/s, like the divergence before it went to float4).
// Requires 16-byte aligned p', p, v*, v (checked by the launcher).
// k_step_finalize's work (model.rs:333-377, :877-889) for one workgroup (its
// own launch: the maxima the previous launches published are visible).
__device__ __forceinline__ void step_finalize_body(const Geom &g, const Fields &f) {
    auto ld_ctl = [](const uint32_t *p) { return *p; };
    Ctl *c = f.ctl;
    if (threadIdx.x < 4) {   // fold the spread step maxima (sharded: already folded)
        uint32_t *set = f.red_slots + (size_t)threadIdx.x * kResSlots * kResStride;
        uint32_t v = ld_ctl(&c->red[threadIdx.x]);
        for (int s = 0; s < kResSlots; ++s) {
            v = max(v, ld_ctl(&set[s * kResStride]));
            set[s * kResStride] = 0u;
        }
        c->red[threadIdx.x] = v;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    // failure detection: red[4] is this step's non-finite flag
    // (all-reduced across slabs with the maxima); the first such step sticks
    if (ld_ctl(&c->red[4]) && !c->nonfinite_step) {
        c->nonfinite_step = c->step + 1u;
        if (f.host_nonfinite) *f.host_nonfinite = c->step + 1u;   // zero-copy host mirror
    }
    c->res_u = __uint_as_float(c->red[0]);
    c->res_v = __uint_as_float(c->red[1]);
    const float max_vel = fmaxf(__uint_as_float(c->red[2]), __uint_as_float(c->red[3]));
    c->step += 1u;
    if (f.host_progress) *f.host_progress = c->step;   // watchdog progress (zero-copy)
    c->time = c->time + c->dt;
    const float previous_dt = c->dt;
    float new_dt;
    if (max_vel == 0.0f) {
        new_dt = c->dt;
    } else {
        const float cfl = 0.2f;
        const float dt_cfl = cfl * fminf(g.dx, g.dy) / max_vel;
        new_dt = fminf(dt_cfl, c->dt);
    }
    c->dt = (new_dt > previous_dt) ? fminf(new_dt, previous_dt * 1.1f) : new_dt;
    // the step's last solve residual: all-reduced across slabs with the
    // maxima (a sharded fixed-count step skips the solve's own all-reduce)
    c->last_p = __uint_as_float(ld_ctl(&c->red[5]));
    c->red[0] = c->red[1] = c->red[2] = c->red[3] = c->red[4] = c->red[5] = 0u;
    // a persistent solve on some slab timed out this step (all-reduced,
    // launch_abort_to_red): every rank's host sees CFD_ETIMEOUT at its next
    // synchronisation and all of them re-run from their checkpoints
    // (cfd_model::recover); later persistent launches of this rank leave at once
    if (ld_ctl(&c->red[6])) {
        if (f.persist) __hip_atomic_store(f.persist + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (f.host_nonfinite)
            __hip_atomic_store(f.host_nonfinite + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ void k_abort_to_red(Fields f) {
    if (threadIdx.x == 0 && f.persist)
        f.ctl->red[6] = __hip_atomic_load(f.persist + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ? 1u : 0u;
}

// The all-reduced abort word back into this rank's abort flag and host word
// (k_step_finalize's part of it, for the entry points with no step finalize:
// cfd_piso_step, cfd_pressure_solve).
__global__ void k_abort_from_red(Fields f) {
    if (threadIdx.x != 0 || !f.ctl->red[6]) return;
    if (f.persist) __hip_atomic_store(f.persist + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (f.host_nonfinite)
        __hip_atomic_store(f.host_nonfinite + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_step_finalize(Geom g, Fields f) { step_finalize_body(g, f); }

// One row of k_correct_finish4m's work for the 4 columns i0..i0+3 of local
// row lj: pc = p' row lj, pb = p' row lj-1 (loaded by the caller), the step
// maxima and the non-finite flag accumulate into du..bad.
template <int SP>
__device__ __forceinline__ void cf4_row(const Geom &g, const Fields &f, const float *__restrict__ pp,
                                        float inlet, float dt, int i0, int lj, const float4 &pc,
                                        const float4 &pb, float &du, float &dv, float &mu,
                                        float &mv, bool &bad) {
    const int nx = g.nx, W = nx + 1;
    const int j = g.j0 + lj;
    const long rp = (long)lj * nx + i0;
    const bool vrow = (j != 0 && j != g.ny);
    if (lj < g.nyl) {
        const long k = (long)lj * W + i0;
        const float pl = (i0 > 0) ? pp[rp - 1] : 0.0f;
        // u rows have pitch nx + 1: their 4-column groups are dword-aligned
        // only, and move as one 16-byte access each (f4u)
        const f4u su = *reinterpret_cast<const f4u *>(f.u_star + k);
        const float s0 = su.x, s1 = su.y, s2 = su.z, s3 = su.w;
        float n0 = cf_u_face<SP>(g, inlet, dt, i0, j, s0, pc.x, pl);
        float n1 = cf_u_face<SP>(g, inlet, dt, i0 + 1, j, s1, pc.y, pc.x);
        float n2 = cf_u_face<SP>(g, inlet, dt, i0 + 2, j, s2, pc.z, pc.y);
        float n3 = cf_u_face<SP>(g, inlet, dt, i0 + 3, j, s3, pc.w, pc.z);
        if (f.n_obs > 0) {
            if (f.mask_u[k] & 2) n0 = 0.0f;
            if (f.mask_u[k + 1] & 2) n1 = 0.0f;
            if (f.mask_u[k + 2] & 2) n2 = 0.0f;
            if (f.mask_u[k + 3] & 2) n3 = 0.0f;
        }
        const f4u uo = *reinterpret_cast<const f4u *>(f.u + k);
        const float o0 = uo.x, o1 = uo.y, o2 = uo.z, o3 = uo.w;
        *reinterpret_cast<f4u *>(f.u + k) = (f4u){n0, n1, n2, n3};
        du = fmaxf(fmaxf(fmaxf(du, fabsf(n0 - o0)), fmaxf(fabsf(n1 - o1), fabsf(n2 - o2))),
                   fabsf(n3 - o3));
        mu = fmaxf(fmaxf(fmaxf(mu, fabsf(n0)), fmaxf(fabsf(n1), fabsf(n2))), fabsf(n3));
        bad |= nonfinite(n0) || nonfinite(n1) || nonfinite(n2) || nonfinite(n3);
        if (i0 + 4 == nx) {   // outflow face nx copies the corrected face nx-1 (Q9)
            float n4 = cf_u_face<SP>(g, inlet, dt, nx, j, s3, pc.w, pc.z);
            if (f.n_obs > 0 && (f.mask_u[k + 4] & 2)) n4 = 0.0f;
            const float o4 = f.u[k + 4];
            f.u[k + 4] = n4;
            du = fmaxf(du, fabsf(n4 - o4));
            mu = fmaxf(mu, fabsf(n4));
            bad |= nonfinite(n4);
        }
    }
    float4 nv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (vrow) {
        const float4 vs = *reinterpret_cast<const float4 *>(f.v_star + rp);
        nv.x = vs.x - dt * sdiv<SP>(pc.x - pb.x, g.dy, g.r_dy);
        nv.y = vs.y - dt * sdiv<SP>(pc.y - pb.y, g.dy, g.r_dy);
        nv.z = vs.z - dt * sdiv<SP>(pc.z - pb.z, g.dy, g.r_dy);
        nv.w = vs.w - dt * sdiv<SP>(pc.w - pb.w, g.dy, g.r_dy);
    }
    if (f.n_obs > 0) {
        if (f.mask_v[rp] & 2) nv.x = 0.0f;
        if (f.mask_v[rp + 1] & 2) nv.y = 0.0f;
        if (f.mask_v[rp + 2] & 2) nv.z = 0.0f;
        if (f.mask_v[rp + 3] & 2) nv.w = 0.0f;
    }
    const float4 ov = *reinterpret_cast<const float4 *>(f.v + rp);
    *reinterpret_cast<float4 *>(f.v + rp) = nv;
    dv = fmaxf(fmaxf(fmaxf(dv, fabsf(nv.x - ov.x)), fmaxf(fabsf(nv.y - ov.y), fabsf(nv.z - ov.z))),
               fabsf(nv.w - ov.w));
    mv = fmaxf(fmaxf(fmaxf(mv, fabsf(nv.x)), fmaxf(fabsf(nv.y), fabsf(nv.z))), fabsf(nv.w));
    bad |= nonfinite(nv.x) || nonfinite(nv.y) || nonfinite(nv.z) || nonfinite(nv.w);
    if (lj < g.nyl) {
        float4 p = *reinterpret_cast<const float4 *>(f.p + rp);
        p.x = p.x + pc.x;
        p.y = p.y + pc.y;
        p.z = p.z + pc.z;
        p.w = p.w + pc.w;
        *reinterpret_cast<float4 *>(f.p + rp) = p;
    }
}

// The corrector finish (model.rs:825-850's corrections, the boundary rows and
// the step maxima) for 4 columns per thread, each thread marching down a band
// of kCfRows rows: p' row lj, loaded for row lj, is row lj+1's lower neighbour
// (the v correction's p'(j-1)), so every p' row crosses HBM once instead of
// twice.
// ROWS: the band (kCfRows, or 1 where the bands would leave the chip idle:
// cf_rows).
#ifndef CFD_CF_ROWS   // build-time (r6 A/B, profiles/r6/prof_r6ag: C3 16 / 8 / 4 rows
#define CFD_CF_ROWS 16  // 10.04 / 10.36 / 10.18 ms per step)
#endif
constexpr int kCfRows = CFD_CF_ROWS;
template <int SP, int ROWS>
__global__ __launch_bounds__(kBlock) void k_correct_finish4m(Geom g, Fields f, float dt_override,
                                                             int nbx) {
    Ctl *c = f.ctl;
    const int nx = g.nx;
    float du = 0.f, dv = 0.f, mu = 0.f, mv = 0.f;
    bool bad = false;
    const int bid = xcd_block(g);
    const int i0 = 4 * ((bid % nbx) * kBlock + (int)threadIdx.x);
    const int l0 = (bid / nbx) * ROWS, l1 = min(l0 + ROWS, g.nyl + 1);
    const float dt = dt_of(c, dt_override);
    const float inlet = c->inlet;
    const float *__restrict__ pp = c->cur ? f.pp[1] : f.pp[0];
    if (i0 < nx) {
        float4 pb = make_float4(0.f, 0.f, 0.f, 0.f);
        {
            const int j = g.j0 + l0;
            if (j != 0 && j != g.ny) pb = *reinterpret_cast<const float4 *>(pp + (long)(l0 - 1) * nx + i0);
        }
        for (int lj = l0; lj < l1; ++lj) {
            const int j = g.j0 + lj;
            const bool vrow = (j != 0 && j != g.ny);
            float4 pc = make_float4(0.f, 0.f, 0.f, 0.f);
            if (lj < g.nyl || vrow) pc = *reinterpret_cast<const float4 *>(pp + (long)lj * nx + i0);
            cf4_row<SP>(g, f, pp, inlet, dt, i0, lj, pc, vrow ? pb : make_float4(0.f, 0.f, 0.f, 0.f),
                        du, dv, mu, mv, bad);
            pb = pc;
        }
    }
    flag_nonfinite(c, bad);
    __shared__ float red[kBlock / 64][4];
    du = wave_max(du);
    dv = wave_max(dv);
    mu = wave_max(mu);
    mv = wave_max(mv);
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[wv][0] = du;
        red[wv][1] = dv;
        red[wv][2] = mu;
        red[wv][3] = mv;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        float r = 0.f;
#pragma unroll
        for (int w = 0; w < kBlock / 64; ++w) r = fmaxf(r, red[w][threadIdx.x]);
        publish_max(f.red_slots + (size_t)threadIdx.x * kResSlots * kResStride, bid, r);
    }
}

// ------------------------------------------------- step reductions (K7)

// max |u - u_old|, max |v - v_old| (model.rs:333-344) and max |u|, max |v|
// (compute_automatic_time_step :879-880) over the owned rows; f32::max
// ignores NaN, as fmaxf does.
__global__ __launch_bounds__(kBlock) void k_step_reduce(Geom g, Fields f) {
    const size_t tid = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const size_t nu = (size_t)g.nyl * (g.nx + 1), nv = (size_t)(g.nyl + 1) * g.nx;
    float du = 0.f, dv = 0.f, mu = 0.f, mv = 0.f;
    bool bad = false;
    for (size_t k = tid; k < nu; k += stride) {
        const float a = f.u[k];
        du = fmaxf(du, fabsf(a - f.u_old[k]));
        mu = fmaxf(mu, fabsf(a));
        bad |= nonfinite(a);
    }
    for (size_t k = tid; k < nv; k += stride) {
        const float a = f.v[k];
        dv = fmaxf(dv, fabsf(a - f.v_old[k]));
        mv = fmaxf(mv, fabsf(a));
        bad |= nonfinite(a);
    }
    flag_nonfinite(f.ctl, bad);
    du = wave_max(du);
    dv = wave_max(dv);
    mu = wave_max(mu);
    mv = wave_max(mv);
    if ((threadIdx.x & 63) == 0) {
        const int key = (int)(tid >> 6);
        constexpr size_t S = (size_t)kResSlots * kResStride;
        publish_max(f.red_slots, key, du);
        publish_max(f.red_slots + S, key, dv);
        publish_max(f.red_slots + 2 * S, key, mu);
        publish_max(f.red_slots + 3 * S, key, mv);
    }
}

// update() epilogue (model.rs:347-377): residuals, step/time, CFL dt.


inline int copy_grid(size_t n4) {
    long b = cdiv((long)n4, kBlock);
    return (int)(b < 2048 ? (b < 1 ? 1 : b) : 2048);
}

}  // namespace

// ------------------------------------------------------------------ launchers

void launch_step_begin(const Geom &g, const Fields &f, int copy, hipStream_t s) {
    size_t n4 = f.u_alloc > f.v_alloc ? f.u_alloc / 4 : f.v_alloc / 4;
    hipLaunchKernelGGL(k_step_begin, dim3(copy ? copy_grid(n4) : 1), dim3(kBlock), 0, s, g, f,
                       copy);
}

void launch_copy_star(const Geom &g, const Fields &f, int pass, hipStream_t s) {
    size_t n4 = f.u_alloc > f.v_alloc ? f.u_alloc / 4 : f.v_alloc / 4;
    hipLaunchKernelGGL(k_copy_star, dim3(copy_grid(n4)), dim3(kBlock), 0, s, f, pass);
}

void launch_u_predictor(const Geom &g, const Fields &f, float dt_override, hipStream_t s) {
    const int glo = g.j0 > 1 ? g.j0 : 1;
    const int ghi = (g.j0 + g.nyl - 1) < (g.ny - 2) ? (g.j0 + g.nyl - 1) : (g.ny - 2);
    if (ghi < glo) return;
    const int nbx = cdiv(g.nx, kBlock);
    const dim3 grid(nbx * (ghi - glo + 1));
#define CFD_LAUNCH_U(SC, SPV) hipLaunchKernelGGL((k_u_predictor<SC, SPV>), grid, dim3(kBlock), 0, s, \
                                                 g, f, dt_override, glo - g.j0, nbx)
    if (g.scheme == 0) {
        if (g.sp_pow2) CFD_LAUNCH_U(0, 1); else CFD_LAUNCH_U(0, 0);
    } else {
        if (g.sp_pow2) CFD_LAUNCH_U(1, 1); else CFD_LAUNCH_U(1, 0);
    }
#undef CFD_LAUNCH_U
}

void launch_v_predictor(const Geom &g, const Fields &f, float dt_override, hipStream_t s) {
    const int glo = g.j0 > 1 ? g.j0 : 1;
    const int ghi = (g.j0 + g.nyl) < (g.ny - 1) ? (g.j0 + g.nyl) : (g.ny - 1);
    if (ghi < glo) return;
    const int nbx = cdiv(g.nx - 1, kBlock);
    const dim3 grid(nbx * (ghi - glo + 1));
#define CFD_LAUNCH_V(SC, SPV) hipLaunchKernelGGL((k_v_predictor<SC, SPV>), grid, dim3(kBlock), 0, s, \
                                                 g, f, dt_override, glo - g.j0, nbx)
    if (g.scheme == 0) {
        if (g.sp_pow2) CFD_LAUNCH_V(0, 1); else CFD_LAUNCH_V(0, 0);
    } else {
        if (g.sp_pow2) CFD_LAUNCH_V(1, 1); else CFD_LAUNCH_V(1, 0);
    }
#undef CFD_LAUNCH_V
}

void launch_predict(const Geom &g, const Fields &f, float dt_override, hipStream_t s) {
    const int glo = g.j0 > 1 ? g.j0 : 1;
    const int u_hi = (g.j0 + g.nyl - 1) < (g.ny - 2) ? (g.j0 + g.nyl - 1) : (g.ny - 2);
    const int v_hi = (g.j0 + g.nyl) < (g.ny - 1) ? (g.j0 + g.nyl) : (g.ny - 1);
    const int ghi = u_hi > v_hi ? u_hi : v_hi;
    if (ghi < glo) return;
    static const int vec = [] {
        const char *e = getenv("CFD_PRED_VEC");
        return e ? atoi(e) : 1;
    }();
    auto a16 = [](const void *p) { return ((uintptr_t)p & 15u) == 0; };
    if (vec && g.scheme == 0 && g.nx % 4 == 0 && a16(f.v) && a16(f.v_star)) {
        const int nbx4 = cdiv(g.nx / 4, kBlock);
        const dim3 gr(nbx4 * cdiv(ghi - glo + 1, 2));
        if (g.sp_pow2)
            hipLaunchKernelGGL((k_predict4r<1, 2>), gr, dim3(kBlock), 0, s, g, f, dt_override,
                               glo - g.j0, u_hi - g.j0, v_hi - g.j0, nbx4);
        else
            hipLaunchKernelGGL((k_predict4r<0, 2>), gr, dim3(kBlock), 0, s, g, f, dt_override,
                               glo - g.j0, u_hi - g.j0, v_hi - g.j0, nbx4);
        return;
    }
    const int nbx = cdiv(g.nx, kBlock);
    const dim3 grid(nbx * (ghi - glo + 1));
#define CFD_LAUNCH_P(SC, SPV) hipLaunchKernelGGL((k_predict<SC, SPV>), grid, dim3(kBlock), 0, s, g, f, \
                                                 dt_override, glo - g.j0, u_hi - g.j0, v_hi - g.j0, nbx)
    if (g.scheme == 0) {
        if (g.sp_pow2) CFD_LAUNCH_P(0, 1); else CFD_LAUNCH_P(0, 0);
    } else {
        if (g.sp_pow2) CFD_LAUNCH_P(1, 1); else CFD_LAUNCH_P(1, 0);
    }
#undef CFD_LAUNCH_P
}

bool predict_div_fused(const Geom &g, const Fields &f) {
    auto a16 = [](const void *p) { return ((uintptr_t)p & 15u) == 0; };
    return g.pred_div == 1 && g.scheme == 0 && g.nx % 4 == 0 && g.nx >= 8 && a16(f.v) && a16(f.v_star) &&
           a16(f.rhs);
}

void launch_predict_div(const Geom &g, const Fields &f, float dt_override, hipStream_t s) {
    const int glo = (g.j0 > 1 ? g.j0 : 1) - g.j0;
    const int u_hi = ((g.j0 + g.nyl - 1) < (g.ny - 2) ? (g.j0 + g.nyl - 1) : (g.ny - 2)) - g.j0;
    const int v_hi = ((g.j0 + g.nyl) < (g.ny - 1) ? (g.j0 + g.nyl) : (g.ny - 1)) - g.j0;
    constexpr int rpt = 2;   // rows per thread
    const int nwc = cdiv(g.nx / 4, 63);
    const int ntile = cdiv(g.nyl, rpt);
    const dim3 grid(nwc * cdiv(ntile, kBlock / 64));
#define CFD_LAUNCH_PD(SPV, R)                                                                    \
    hipLaunchKernelGGL((k_predict_div<SPV, R>), grid, dim3(kBlock), 0, s, g, f, dt_override, glo, \
                       u_hi, v_hi, nwc, ntile)
    if (g.sp_pow2) CFD_LAUNCH_PD(1, 2); else CFD_LAUNCH_PD(0, 2);
#undef CFD_LAUNCH_PD
}

void launch_copy_star_div(const Geom &g, const Fields &f, int pass, float dt_override,
                          hipStream_t s) {
    const int nbx = cdiv(g.nx / 4, kBlock);
    const dim3 grid(nbx * (g.nyl + 1 + 2 * kGhostUV));
    if (g.sp_pow2)
        hipLaunchKernelGGL(k_copy_star_div<1>, grid, dim3(kBlock), 0, s, g, f, pass, dt_override, nbx);
    else
        hipLaunchKernelGGL(k_copy_star_div<0>, grid, dim3(kBlock), 0, s, g, f, pass, dt_override, nbx);
}

void launch_divergence(const Geom &g, const Fields &f, int pass, float dt_override,
                       hipStream_t s) {
    const int nbx = cdiv(g.nx / 4, kBlock);
    if (g.sp_pow2)
        hipLaunchKernelGGL(k_divergence<1>, dim3(nbx * g.nyl), dim3(kBlock), 0, s, g, f, pass,
                           dt_override, nbx);
    else
        hipLaunchKernelGGL(k_divergence<0>, dim3(nbx * g.nyl), dim3(kBlock), 0, s, g, f, pass,
                           dt_override, nbx);
}

void launch_jacobi_sweep(const Geom &g, const Fields &f, int pass, int it, int row_lo,
                         int row_hi, int res, hipStream_t s) {
    if (row_hi <= row_lo) return;
    const int nch = g.nx / 4;
    const int nwc = cdiv(nch, 64);
    const int nbx = cdiv(nwc, kJacWavesPerBlock);
    const int nseg = cdiv(row_hi - row_lo, kJacRowsPerWave);
    float *pa = f.pp[0] - (long)g.hg * g.nx, *pb = f.pp[1] - (long)g.hg * g.nx;
    const dim3 grid(nbx * nseg), block(kJacWavesPerBlock * 64);
    if (g.fastdiv == 1)
        hipLaunchKernelGGL((k_jacobi<kJacRowsPerWave, 1>), grid, block, 0, s, g, pa, pb, f.rhs,
                           f.ctl, f.err_slots, pass, it, row_lo, row_hi, nbx, res);
    else if (g.fastdiv == 2)
        hipLaunchKernelGGL((k_jacobi<kJacRowsPerWave, 2>), grid, block, 0, s, g, pa, pb, f.rhs,
                           f.ctl, f.err_slots, pass, it, row_lo, row_hi, nbx, res);
    else
        hipLaunchKernelGGL((k_jacobi<kJacRowsPerWave, 0>), grid, block, 0, s, g, pa, pb, f.rhs,
                           f.ctl, f.err_slots, pass, it, row_lo, row_hi, nbx, res);
}

void launch_jacobi_block(const Geom &g, const Fields &f, int pass, int it, int par, int T,
                         int out_lo, int out_hi, int res, hipStream_t s) {
    if (out_hi <= out_lo) return;
    uint32_t *rs = res ? f.err_slots + (size_t)(it + T - 1) * kResSlots * kResStride : nullptr;
    if (g.tb_kind == 3)
        launch_pipe4(g, f, T, pass, it, par, out_lo, out_hi, rs, s);
    else if (g.tb_kind == 4)
        launch_pipe2(g, f, T, pass, it, par, out_lo, out_hi, rs, s);
    else if (g.tb_kind == 5)
        launch_lds(g, f, T, pass, it, par, out_lo, out_hi, rs, s);
    else
        launch_tb1(g, f, T, pass, it, par, out_lo, out_hi, rs, s);
}

bool launch_jacobi_persist(const Geom &g, const Fields &f, int pass, int par0, int nblk,
                           int out_lo, int out_hi, uint32_t epoch, int res_it, hipStream_t s) {
    if (out_hi <= out_lo || nblk < 1 || g.tb_kind != 5 || !f.persist) return false;
    uint32_t *rs = res_it >= 0 ? f.err_slots + (size_t)res_it * kResSlots * kResStride : nullptr;
    return launch_lds_persist8(g, f, pass, par0, nblk, out_lo, out_hi, epoch, rs, s);
}

void launch_jacobi_spec(const Geom &g, const Fields &f, int pass, int it, int par, int T,
                        int out_lo, int out_hi, hipStream_t s, int lag) {
    if (out_hi <= out_lo) return;
    launch_lds(g, f, T, pass, it, par, out_lo, out_hi,
               f.err_slots + (size_t)it * kResSlots * kResStride, s, 2, lag);
}

void launch_spec_check(const Geom &g, const Fields &f, int pass, int it, int T, int par,
                       hipStream_t s) {
    hipLaunchKernelGGL(k_spec_check, dim3(1), dim3(kBlock), 0, s, g, f, pass, it, T, par);
}

void launch_jacobi_redo(const Geom &g, const Fields &f, int pass, int out_lo, int out_hi,
                        hipStream_t s, int last_it, int last_par, int last_T) {
    if (out_hi <= out_lo) return;
    launch_lds(g, f, kMaxTemporal, pass, last_it, last_par, out_lo, out_hi,
               last_T > 0 ? f.err_slots + (size_t)last_it * kResSlots * kResStride : nullptr, s, 3,
               last_T);
}

void launch_spec_align(const Geom &g, const Fields &f, int pass, int n, hipStream_t s) {
    hipLaunchKernelGGL(k_spec_align, dim3(256), dim3(kBlock), 0, s, g, f, pass, n);
}

void launch_fold_slots(uint32_t *dst, uint32_t *slots, int n, hipStream_t s) {
    hipLaunchKernelGGL(k_fold_slots, dim3(1), dim3(64), 0, s, dst, slots, n);
}

void launch_verify_division(float c, float r, unsigned long long *dev_counts, hipStream_t s) {
    hipLaunchKernelGGL(k_verify_division, dim3(8192), dim3(kBlock), 0, s, c, r, dev_counts);
}

void launch_finalize_solve(const Geom &g, const Fields &f, int pass, int iters, int check_break,
                           int flips, hipStream_t s, int exact_flips) {
    hipLaunchKernelGGL(k_finalize_solve, dim3(1), dim3(kFinThreads), 0, s, g, f, pass, iters,
                       check_break, flips, exact_flips);
}

void launch_corrector(const Geom &g, const Fields &f, int pass, float dt_override,
                      hipStream_t s) {
    auto a16 = [](const void *p) { return ((uintptr_t)p & 15u) == 0; };
    const char *ve = getenv("CFD_CORR_VEC");   // 0: the one-float-per-thread kernel
    const bool vec_env = !(ve && atoi(ve) == 0);
    if (vec_env && g.nx % 4 == 0 && a16(f.v) && a16(f.v_star) && a16(f.p) && a16(f.pp[0]) &&
        a16(f.pp[1])) {
        const int nbx4 = cdiv(g.nx / 4, kBlock);
        if (g.sp_pow2)
            hipLaunchKernelGGL(k_corrector4<1>, dim3(nbx4 * (g.nyl + 1)), dim3(kBlock), 0, s, g, f,
                               pass, dt_override, nbx4);
        else
            hipLaunchKernelGGL(k_corrector4<0>, dim3(nbx4 * (g.nyl + 1)), dim3(kBlock), 0, s, g, f,
                               pass, dt_override, nbx4);
        return;
    }
    const int nbx = cdiv(g.nx + 1, kBlock);
    if (g.sp_pow2)
        hipLaunchKernelGGL(k_corrector<1>, dim3(nbx * (g.nyl + 1)), dim3(kBlock), 0, s, g, f, pass,
                           dt_override, nbx);
    else
        hipLaunchKernelGGL(k_corrector<0>, dim3(nbx * (g.nyl + 1)), dim3(kBlock), 0, s, g, f, pass,
                           dt_override, nbx);
}

bool correct_head_ok(const Geom &g, const Fields &f) {
    auto a16 = [](const void *p) { return ((uintptr_t)p & 15u) == 0; };
    const char *e = getenv("CFD_CORR_HEAD");   // 0: corrector + separate pass head
    return !(e && atoi(e) == 0) && g.nx % 4 == 0 && a16(f.v) && a16(f.v_star) && a16(f.p) &&
           a16(f.pp[0]) && a16(f.pp[1]) && a16(f.rhs);
}

// Rows per thread of the corrector bands: kCfRows where that still gives
// every CU two workgroups, else 1 (the 800 x 264 reference default: 17
// workgroups of 16-row bands ran k_correct_head4 in 34.6 us against 5.9 us for
// 270 one-row workgroups, profiles/r6/prof_r6u vs prof_r6l)
static int cf_rows(const Geom &g, int nbx, int nrows) {
    return (long)nbx * cdiv(nrows, kCfRows) >= 2L * g.n_cu ? kCfRows : 1;
}

void launch_correct_head(const Geom &g, const Fields &f, int pass, float dt_override, bool has_next,
                         hipStream_t s) {
    const int nbx4 = cdiv(g.nx / 4, kBlock);
    const int hn = has_next ? 1 : 0;
    // the band march, kCfRows rows per thread, where it still fills the chip
    // (r6: C3 in the reference's control flow 10.37 -> 10.26 ms per step
    // against one row per thread, best of 3; profiles/r6/prof_r6p/ab_corrhead.log);
    // on small grids one row per thread (cf_rows)
    const int nrows = g.nyl + 1 + 2 * kGhostUV;
    const int rows = cf_rows(g, nbx4, nrows);
    const dim3 grid(nbx4 * cdiv(nrows, rows));
#define CFD_LAUNCH_CH(SPV, RW)                                                                    \
    hipLaunchKernelGGL((k_correct_head4<SPV, RW>), grid, dim3(kBlock), 0, s, g, f, pass, dt_override, \
                       nbx4, hn)
    if (rows == kCfRows) {
        if (g.sp_pow2) CFD_LAUNCH_CH(1, kCfRows); else CFD_LAUNCH_CH(0, kCfRows);
    } else {
        if (g.sp_pow2) CFD_LAUNCH_CH(1, 1); else CFD_LAUNCH_CH(0, 1);
    }
#undef CFD_LAUNCH_CH
}

void launch_correct_finish(const Geom &g, const Fields &f, float dt_override, hipStream_t s) {
    auto a16 = [](const void *p) { return ((uintptr_t)p & 15u) == 0; };
    if (g.nx % 4 == 0 && a16(f.pp[0]) && a16(f.pp[1]) && a16(f.p) && a16(f.v) && a16(f.v_star)) {
        const int nbx = cdiv(g.nx / 4, kBlock);
        const int rows = cf_rows(g, nbx, g.nyl + 1);
        const dim3 grid(nbx * cdiv(g.nyl + 1, rows));
#define CFD_LAUNCH_CF(SPV, RW)                                                                     \
    hipLaunchKernelGGL((k_correct_finish4m<SPV, RW>), grid, dim3(kBlock), 0, s, g, f, dt_override, nbx)
        if (rows == kCfRows) {
            if (g.sp_pow2) CFD_LAUNCH_CF(1, kCfRows); else CFD_LAUNCH_CF(0, kCfRows);
        } else {
            if (g.sp_pow2) CFD_LAUNCH_CF(1, 1); else CFD_LAUNCH_CF(0, 1);
        }
#undef CFD_LAUNCH_CF
        return;
    }
    const int nbx = cdiv(g.nx + 1, kBlock);
    const long ntiles = (long)nbx * (g.nyl + 1);
    const int blocks = (int)std::min<long>(ntiles, 8L * g.n_cu);
    if (g.sp_pow2)
        hipLaunchKernelGGL(k_correct_finish<1>, dim3(blocks), dim3(kBlock), 0, s, g, f, dt_override, nbx);
    else
        hipLaunchKernelGGL(k_correct_finish<0>, dim3(blocks), dim3(kBlock), 0, s, g, f, dt_override, nbx);
}

void launch_boundary(const Geom &g, const Fields &f, hipStream_t s) {
    hipLaunchKernelGGL(k_boundary, dim3(1), dim3(1024), 0, s, g, f);
}

void launch_step_reduce(const Geom &g, const Fields &f, hipStream_t s) {
    const size_t n = (size_t)(g.nyl + 1) * (g.nx + 1);
    hipLaunchKernelGGL(k_step_reduce, dim3(copy_grid(n / 4 + 1)), dim3(kBlock), 0, s, g, f);
}

void launch_abort_to_red(const Fields &f, hipStream_t s) {
    hipLaunchKernelGGL(k_abort_to_red, dim3(1), dim3(64), 0, s, f);
}

void launch_abort_from_red(const Fields &f, hipStream_t s) {
    hipLaunchKernelGGL(k_abort_from_red, dim3(1), dim3(64), 0, s, f);
}

void launch_step_finalize(const Geom &g, const Fields &f, hipStream_t s) {
    hipLaunchKernelGGL(k_step_finalize, dim3(1), dim3(64), 0, s, g, f);
}

}  // namespace cfd
