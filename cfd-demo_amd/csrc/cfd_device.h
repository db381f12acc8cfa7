// cfd_device.h — device helpers shared by the kernel translation units
// (cfd_kernels.hip, cfd_jacobi_tb1.hip, cfd_jacobi_pipe*.hip).  Everything is
// internal to each translation unit (anonymous namespace).
#pragma once
#include "cfd_internal.h"

#include <algorithm>

namespace cfd {
namespace {

inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }


constexpr int kBlock = 256;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float dt_of(const Ctl *c, float dt_override) {
    return __builtin_isnan(dt_override) ? c->dt : dt_override;
}

__device__ __forceinline__ bool pass_off(const Ctl *c, int pass) {
    return pass >= 0 && c->go[pass] == 0;
}

__device__ __forceinline__ float wave_max(float m) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    return m;
}

// Publish a non-negative maximum into slot `key` of a spread set (cfd_internal.h).
__device__ __forceinline__ void publish_max(uint32_t *set, int key, float m) {
    if (m > 0.0f) atomicMax(&set[(key & (kResSlots - 1)) * kResStride], __float_as_uint(m));
}

// NaN or +-Inf (the step's failure check, SURVEY.md §5: the reference itself
// has none and keeps stepping on a blown-up field).
__device__ __forceinline__ bool nonfinite(float x) { return !(fabsf(x) <= 3.40282347e38f); }
// Raise the step's non-finite flag (Ctl::red[4]); only lanes that saw one store.
__device__ __forceinline__ void flag_nonfinite(Ctl *c, bool bad) {
    if (bad) atomicOr(&c->red[4], 1u);
}

// max(base, every slot of a set); called by all 64 lanes of a wave, uniform result.
__device__ __forceinline__ float read_max(const uint32_t *set, uint32_t base) {
    const int lane = (int)threadIdx.x & 63;
    const float v = lane < kResSlots ? __uint_as_float(set[lane * kResStride]) : 0.0f;
    return fmaxf(wave_max(v), __uint_as_float(base));
}

// XCD-aware block order.  The dispatcher deals workgroups to the 8 XCDs
// round-robin (block b -> XCD b % 8), and each XCD has its own L2; renumber
// so XCD x works on one contiguous range of tiles (rows), keeping the rows
// neighbouring tiles share (stencil rows, segment overlaps) in one L2.  The
// last G % 8 blocks keep their own index.
__device__ __forceinline__ int xcd_block(const Geom &g) {
    const int b = (int)blockIdx.x, G = (int)gridDim.x;
    if (!g.xcd_remap) return b;
    const int per = G >> 3;
    if (b >= (per << 3)) return b;
    return (b & 7) * per + (b >> 3);
}

// Lane shifts on the VALU (DPP wave_shr:1 / wave_shl:1, gfx9 family) instead
// of the LDS crossbar: lane l receives lane l-1 (from_left) or l+1
// (from_right); the wave's end lanes receive 0 (bound_ctrl: no register
// initialisation needed; they are halo lanes).
__device__ __forceinline__ float from_left(float x) {
    return __builtin_bit_cast(
        float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float from_right(float x) {
    return __builtin_bit_cast(
        float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x130, 0xf, 0xf, true));
}

// x / c with the reference's IEEE rounding.  FAST 1 and 2 are used only for
// divisors whose result equals IEEE `/` for every one of the 2^32 inputs,
// proven on the device at model creation (verify_division, cfd_model.hip).
// FAST 3 (r4): the FMA-corrected form for |x| >= 2^-96 and IEEE `/` below
// (where the correction's residual underflows: every mismatch of form 2 on
// the reference's default-grid divisors lies at |x| < 2^-104), proven for all
// 2^32 inputs per divisor like the others; NaN takes the IEEE branch, +-0 the
// product (r6).
constexpr float kDivGuardMin = 0x1p-96f;
template <int FAST>
__device__ __forceinline__ float fdiv(float x, float c, float r) {
    if (FAST == 1) return x * r;
    if (FAST == 2) {
        const float q0 = x * r;
        const float q = __builtin_fmaf(__builtin_fmaf(-q0, c, x), r, q0);
        return __builtin_isfinite(q0) ? q : q0;
    }
    if (FAST == 3) {
        // (r6) a zero dividend takes the product too: x * r is +-0 with x's
        // sign, as x / c -- exact zeros (a cold or Dirichlet region) no longer
        // need the IEEE division; and the guard is ONE wave-uniform branch:
        // the corrected product for every lane, the IEEE quotient only when
        // some lane of the wave needs it (no per-lane exec-mask juggling per
        // division).  Each lane's value is the same function of x as before,
        // so the exhaustive per-divisor proof (k_verify_division) covers it.
        const float q0 = x * r;
        const float qc = __builtin_fmaf(__builtin_fmaf(-q0, c, x), r, q0);
        float q = __builtin_isfinite(q0) && x != 0.0f ? qc : q0;
        const bool ok = __builtin_fabsf(x) >= kDivGuardMin || x == 0.0f;   // NaN: not ok
        if (__builtin_expect(!__all(ok), 0)) q = ok ? q : x / c;
        return q;
    }
    return x / c;
}

// x / c for a grid spacing c (dx, dy, dx*dx, dy*dy).  SP: every spacing is an
// exact power of two with a normal reciprocal (Geom::sp_pow2, checked on the
// host), so x * (1/c) is the correctly rounded value of the same real number
// as x / c — bit-identical for every x, including subnormals, infinities and NaN.
template <int SP>
__device__ __forceinline__ float sdiv(float x, float c, float r) {
    return SP ? x * r : x / c;
}

typedef float f2 __attribute__((ext_vector_type(2)));

template <int FAST>
__device__ __forceinline__ f2 fdiv2(f2 x, float c, float r) {
    if (FAST == 1) return x * r;                        // v_pk_mul_f32
    return (f2){fdiv<FAST>(x.x, c, r), fdiv<FAST>(x.y, c, r)};
}

// End of a pressure solve: how many sweeps ran, which buffer is current, the
// returned residual (model.rs:816-823), and whether the corrector loop goes on
// (model.rs:721-723).  Resets the per-sweep slots for the next solve.
// k_finalize_solve's work (one workgroup of kBlock threads): fold the solve's
// residual slots into Ctl::err, count the sweeps that ran, flip the current
// p' buffer, set the next corrector pass's go flag, clear err[].
__device__ __forceinline__ void solve_finalize_body(const Geom &g, const Fields &f, int pass,
                                                    int iters, int check_break, int flips,
                                                    int exact_flips) {
    Ctl *c = f.ctl;
    __shared__ int go_s;
    // fold the spread residual slots into err[]: every sweep's with the
    // tolerance on, only the last one's for a fixed-count solve (the only
    // sweep that publishes); one wave per sweep, one lane per slot
    const int k_lo = g.tol_enabled ? 0 : (iters > 0 ? iters - 1 : 0);
    const int wv = (int)threadIdx.x >> 6, nw = (int)blockDim.x >> 6;
    for (int k = k_lo + wv; k < iters; k += nw) {
        uint32_t *set = f.err_slots + (size_t)k * kResSlots * kResStride;
        const float v = read_max(set, c->err[k]);
        if ((threadIdx.x & 63) < kResSlots) set[(threadIdx.x & 63) * kResStride] = 0u;
        if ((threadIdx.x & 63) == 0) c->err[k] = __float_as_uint(v);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const int go = pass < 0 ? 1 : c->go[pass];
        if (go) {
            int n = iters;
            if (g.tol_enabled && iters > 0) {
                n = 1;
                // model.rs:816: only `max_error < tolerance` exits (a NaN
                // residual runs on, as every sweep kernel's check does)
                while (n < iters && !(__uint_as_float(c->err[n - 1]) < g.p_tol)) ++n;
            }
            const float res = n > 0 ? __uint_as_float(c->err[n - 1]) : 0.0f;
            // one buffer flip per launch: per sweep with the tolerance on,
            // `flips` (host-known launch count) for fixed-count solves
            // 3 (r5, the speculative solve on slabs): `flips` launches, the
            // converged launch's result aligned to that buffer (k_spec_align)
            c->cur = (c->cur + (exact_flips == 2 ? c->spec_launches
                                : (g.tol_enabled && !exact_flips) ? n : flips)) & 1;
            c->last_p = res;
            c->red[5] = __float_as_uint(res);   // the step-end all-reduce carries it (slabs)
            c->n_exec_last = (uint32_t)n;
            c->sweeps_total += (uint64_t)n;
        }
        if (pass >= 0 && pass + 1 <= kMaxPasses)
            c->go[pass + 1] = (go && !(check_break && g.tol_enabled && c->last_p < g.p_tol)) ? 1 : 0;
        if (exact_flips >= 2) c->spec_stop = c->spec_redo = c->spec_launch = c->spec_launches = 0;
        go_s = go;
    }
    __syncthreads();
    if (go_s)
        for (int k = threadIdx.x; k < iters; k += blockDim.x) c->err[k] = 0u;
}

// One reference Jacobi update (model.rs:775-793) of the 4 consecutive
// columns a lane holds, C = row j, B = row j-1, T = row j+1, Rh = rhs row j,
// L0 / R3 = the columns left / right of the chunk.  The arithmetic is the
// reference's, operation for operation, on column pairs: each pair is one
// packed VOP3P instruction, and the horizontal sums are formed as
// swap(C01) + (L0, C.z) and swap(C23) + (C.y, R3), so the swap folds into
// op_sel and only two register moves remain per 4 columns (f32 addition is
// commutative bit for bit).
template <int FAST>
__device__ __forceinline__ float4 jacobi_row4(const float4 &B, const float4 &C, const float4 &T,
                                              const float4 &Rh, float L0, float R3, float dx_sq,
                                              float dy_sq, float denom, float r_dx_sq,
                                              float r_dy_sq, float r_denom) {
    const f2 c01 = {C.x, C.y}, c23 = {C.z, C.w};
    const f2 h01 = __builtin_shufflevector(c01, c01, 1, 0) + (f2){L0, C.z};
    const f2 h23 = __builtin_shufflevector(c23, c23, 1, 0) + (f2){C.y, R3};
    const f2 v01 = (f2){T.x, T.y} + (f2){B.x, B.y};
    const f2 v23 = (f2){T.z, T.w} + (f2){B.z, B.w};
    const f2 hz01 = fdiv2<FAST>(h01, dx_sq, r_dx_sq), hz23 = fdiv2<FAST>(h23, dx_sq, r_dx_sq);
    const f2 vt01 = fdiv2<FAST>(v01, dy_sq, r_dy_sq), vt23 = fdiv2<FAST>(v23, dy_sq, r_dy_sq);
    const f2 pu01 = fdiv2<FAST>(hz01 + vt01 - (f2){Rh.x, Rh.y}, denom, r_denom);
    const f2 pu23 = fdiv2<FAST>(hz23 + vt23 - (f2){Rh.z, Rh.w}, denom, r_denom);
    const float omega = 0.75f;
    const float om1 = 1.0f - omega;
    const f2 n01 = omega * pu01 + om1 * c01;
    const f2 n23 = omega * pu23 + om1 * c23;
    return make_float4(n01.x, n01.y, n23.x, n23.y);
}

}  // namespace
}  // namespace cfd
