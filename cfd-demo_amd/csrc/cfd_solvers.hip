// cfd_solvers.hip — the alternative pressure solvers of the reference's
// JavaScript variant on gfx950, selected by cfd_params.pressure_solver:
//   1: SOR (index.html:741-774), swept red-black;
//   2: multigrid V-cycles (index.html:775-795, 1344-1470).
//
// Arithmetic: the script computes in IEEE double and stores into
// Float32Array; these kernels do the same (f64 VALU, f32 fields in HBM), so
// each stored word equals the script's — the multigrid path is checked bit for
// bit against the script itself run under node (tests/golden/js_mg_*.npz).
// Divisions by a grid constant c become x * (1/c) only when c is a power of
// two: then 1/c is exact and both forms are the correctly rounded value of the
// same real number, for every x (MgLevel::fast / SorConst::fast, decided on
// the host).
//
// Multigrid mapping: levels whose grid exceeds a threshold (CFD_MG_TAIL,
// default 64 x 64 cells) run as one grid-wide launch per pass (smooth,
// residual, restrict, prolong-add: every pass is a stencil over L2/HBM, one
// f32 written per cell); all coarser levels, down to the coarsest and back up,
// run inside ONE single-workgroup launch (k_mg_tail) with workgroup barriers
// between passes, so the ~100 tiny passes of the bottom of the V-cycle cost
// one launch instead of a hundred.
#include "cfd_device.h"

namespace cfd {
namespace {

__device__ __forceinline__ double ddiv(double x, double c, double r, int fast) {
    return fast ? x * r : x / c;
}

// ------------------------------------------------------------------- SOR

// One color of red-black SOR over the interior i = 1..nx-2, j = 1..ny-2
// (index.html:749-760: omega 1.7, p_update and the relaxation in double,
// stored as f32; |new - old| feeds the residual).  A thread owns a column
// pair (2q, 2q+1) of one row, i.e. one cell of each color.  The black pass
// also applies the p' boundary conditions of :761-770 as stores: it holds the
// pair's final values, so column 0 takes column 1, column nx-1 stores 0, and
// the threads of rows 1 and ny-2 also store rows 0 and ny-1 — exactly the
// script's result after its row loop then its column loop.  Every cell that
// reads a boundary value (column 0 / nx-1, row 0 / ny-1) is updated by the
// same thread that later stores that boundary value.
__global__ __launch_bounds__(kBlock) void k_sor_color(float *__restrict__ pp,
                                                      const float *__restrict__ rhs, int nx, int ny,
                                                      SorConst k, int color, Ctl *ctl,
                                                      uint32_t *err_slots, int pass, int it,
                                                      int tol, float p_tol, int res, int nbx) {
    if (pass_off(ctl, pass)) return;
    // early exit of the previous iteration (index.html:772)
    if (tol && it > 0 &&
        read_max(err_slots + (size_t)(it - 1) * kResSlots * kResStride, ctl->err[it - 1]) < p_tol)
        return;
    const int bid = (int)blockIdx.x;
    const int q = (bid % nbx) * kBlock + (int)threadIdx.x;
    const int j = bid / nbx + 1;
    const int i0 = 2 * q;
    float m = 0.0f;
    if (i0 < nx) {
        const long row = (long)j * nx;
        float2 c = *reinterpret_cast<const float2 *>(pp + row + i0);
        const int i = i0 + ((i0 + j + color) & 1);   // this color's cell of the pair
        if (i >= 1 && i <= nx - 2) {
            const long idx = row + i;
            const double p_old = (double)(i == i0 ? c.x : c.y);
            const double h = ddiv((double)pp[idx + 1] + (double)pp[idx - 1], k.dx2, k.r_dx2, k.fast);
            const double v = ddiv((double)pp[idx + nx] + (double)pp[idx - nx], k.dy2, k.r_dy2, k.fast);
            const double p_update = ddiv(h + v - (double)rhs[idx], k.denom, k.r_denom, k.fast);
            const double omega = 1.7;
            const float nv = (float)((1.0 - omega) * p_old + omega * p_update);
            m = (float)fabs((double)nv - p_old);
            if (i == i0) c.x = nv; else c.y = nv;
            if (color == 0) pp[idx] = nv;
        }
        if (color == 1) {
            if (i0 == 0) c.x = c.y;            // P(0,j) = P(1,j)
            if (i0 + 1 == nx - 1) c.y = 0.0f;  // P(nx-1,j) = 0
            *reinterpret_cast<float2 *>(pp + row + i0) = c;
            if (j == 1) *reinterpret_cast<float2 *>(pp + i0) = c;                               // row 0
            if (j == ny - 2) *reinterpret_cast<float2 *>(pp + (long)(ny - 1) * nx + i0) = c;   // row ny-1
        }
    }
    if (!res) return;
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0)
        publish_max(err_slots + (size_t)it * kResSlots * kResStride,
                    bid * (kBlock / 64) + ((int)threadIdx.x >> 6), m);
}

// p' = 0 at the start of a solve (index.html:743, :777), gated by the
// corrector loop like every solve kernel.
__global__ __launch_bounds__(kBlock) void k_fill_zero(float4 *p, long n4, const Ctl *ctl, int pass) {
    if (pass_off(ctl, pass)) return;
    for (long k = (long)blockIdx.x * kBlock + threadIdx.x; k < n4; k += (long)gridDim.x * kBlock)
        p[k] = make_float4(0.f, 0.f, 0.f, 0.f);
}

// ------------------------------------------------------------- multigrid

// mgSmooth (index.html:1351-1359), one sweep: interior cells get the Jacobi
// value, boundary cells are copied (the script leaves them in place; here the
// sweep ping-pongs between two buffers).
__device__ __forceinline__ void mg_smooth_cell(const MgLevel &L, const float *__restrict__ src,
                                               float *__restrict__ dst, int i, int j) {
    const int nx = L.nx;
    const long idx = (long)j * nx + i;
    if (i == 0 || j == 0 || i == nx - 1 || j == L.ny - 1) {
        dst[idx] = src[idx];
        return;
    }
    const double p_e = src[idx + 1], p_w = src[idx - 1];
    const double p_n = src[idx + nx], p_s = src[idx - nx];
    const double h = ddiv(p_e + p_w, L.dx2, L.r_dx2, L.fast);
    const double v = ddiv(p_n + p_s, L.dy2, L.r_dy2, L.fast);
    dst[idx] = (float)ddiv(h + v - (double)L.rhs[idx], L.denom, L.r_denom, L.fast);
}

// r = rhs - A p on the interior, 0 on the boundary (index.html:1430-1441).
__device__ __forceinline__ void mg_residual_cell(const MgLevel &L, const float *__restrict__ p,
                                                 int i, int j) {
    const int nx = L.nx;
    const long idx = (long)j * nx + i;
    if (i == 0 || j == 0 || i == nx - 1 || j == L.ny - 1) {
        L.r[idx] = 0.0f;
        return;
    }
    const double p_e = p[idx + 1], p_w = p[idx - 1], p_n = p[idx + nx], p_s = p[idx - nx];
    const double ap = ddiv(p_e + p_w, L.dx2, L.r_dx2, L.fast) +
                      ddiv(p_n + p_s, L.dy2, L.r_dy2, L.fast) - L.denom * (double)p[idx];
    L.r[idx] = (float)((double)L.rhs[idx] - ap);
}

// mgRestrict (index.html:1372-1395) of F.r into C.rhs, and C's first buffer
// zeroed (the coarse error's initial value, :1455).  Corner cells follow the
// script's order: the column injection overwrites the row injection.
__device__ __forceinline__ void mg_restrict_cell(const MgLevel &F, const MgLevel &Cl, int i, int j) {
    const int nxf = F.nx, nxc = Cl.nx, nyc = Cl.ny;
    const float *__restrict__ fine = F.r;
    float v;
    if (i == 0) {
        v = fine[(long)(2 * j) * nxf];
    } else if (i == nxc - 1) {
        v = fine[(long)(nxf - 1) + (long)(2 * j) * nxf];
    } else if (j == 0) {
        v = fine[2 * i];
    } else if (j == nyc - 1) {
        v = fine[2 * (long)i + (long)(F.ny - 1) * nxf];
    } else {
        const long c = (long)(2 * j) * nxf + 2 * i;
        const double sum = (double)fine[c] +
                           0.5 * ((double)fine[c - 1] + (double)fine[c + 1] +
                                  (double)fine[c - nxf] + (double)fine[c + nxf]) +
                           0.25 * ((double)fine[c - nxf - 1] + (double)fine[c + nxf - 1] +
                                   (double)fine[c - nxf + 1] + (double)fine[c + nxf + 1]);
        v = (float)(sum / 4.0);
    }
    const long k = (long)j * nxc + i;
    Cl.rhs[k] = v;
    Cl.a[k] = 0.0f;
}

// mgProlongate (index.html:1398-1421) of the coarse error e, added to p
// (:1464-1466): p = f32(p + f32(bilinear)).
__device__ __forceinline__ void mg_prolong_add_cell(const MgLevel &Cl, const float *__restrict__ e,
                                                    const MgLevel &F, float *__restrict__ p, int i,
                                                    int j) {
    const int nxc = Cl.nx, nyc = Cl.ny;
    const int j0 = j >> 1, i0 = i >> 1;
    const int j1 = min(j0 + 1, nyc - 1), i1 = min(i0 + 1, nxc - 1);
    const double b = (j & 1) ? 0.5 : 0.0, a = (i & 1) ? 0.5 : 0.0;
    const double val = (1 - a) * (1 - b) * (double)e[(long)j0 * nxc + i0] +
                       a * (1 - b) * (double)e[(long)j0 * nxc + i1] +
                       (1 - a) * b * (double)e[(long)j1 * nxc + i0] +
                       a * b * (double)e[(long)j1 * nxc + i1];
    const long idx = (long)j * F.nx + i;
    p[idx] = (float)((double)p[idx] + (double)(float)val);
}

// Grid-wide passes: one cell per thread, nbx blocks per row.
__global__ __launch_bounds__(kBlock) void k_mg_smooth(MgLevel L, const float *src, float *dst,
                                                      const Ctl *ctl, int pass, int nbx) {
    if (pass_off(ctl, pass)) return;
    const int i = ((int)blockIdx.x % nbx) * kBlock + (int)threadIdx.x, j = (int)blockIdx.x / nbx;
    if (i < L.nx) mg_smooth_cell(L, src, dst, i, j);
}

__global__ __launch_bounds__(kBlock) void k_mg_residual(MgLevel L, const float *p, const Ctl *ctl,
                                                        int pass, int nbx) {
    if (pass_off(ctl, pass)) return;
    const int i = ((int)blockIdx.x % nbx) * kBlock + (int)threadIdx.x, j = (int)blockIdx.x / nbx;
    if (i < L.nx) mg_residual_cell(L, p, i, j);
}

__global__ __launch_bounds__(kBlock) void k_mg_restrict(MgLevel F, MgLevel Cl, const Ctl *ctl,
                                                        int pass, int nbx) {
    if (pass_off(ctl, pass)) return;
    const int i = ((int)blockIdx.x % nbx) * kBlock + (int)threadIdx.x, j = (int)blockIdx.x / nbx;
    if (i < Cl.nx) mg_restrict_cell(F, Cl, i, j);
}

__global__ __launch_bounds__(kBlock) void k_mg_prolong_add(MgLevel Cl, const float *e, MgLevel F,
                                                           float *p, const Ctl *ctl, int pass,
                                                           int nbx) {
    if (pass_off(ctl, pass)) return;
    const int i = ((int)blockIdx.x % nbx) * kBlock + (int)threadIdx.x, j = (int)blockIdx.x / nbx;
    if (i < F.nx) mg_prolong_add_cell(Cl, e, F, p, i, j);
}

// The bottom of the V-cycle, levels s..Lc (Lc = coarsest), in one workgroup:
// down  {5 smooths a->b..->b, residual, restrict into l+1} for l = s..Lc-1,
// 15 smooths at Lc (mgVcycle's pre-smooth + the coarse "solve", :1444-1447),
// up    {prolong-add into b, 5 smooths b->..->a} for l = Lc-1..s.
// Level s starts in a and ends in a; Lc ends in b.  a0/b0 override level 0's
// buffers (the model's current / other p' buffer).
constexpr int kTailThreads = 1024;

__global__ __launch_bounds__(kTailThreads) void k_mg_tail(const MgLevel *__restrict__ lv, int s,
                                                          int lc, float *a0, float *b0,
                                                          const Ctl *ctl, int pass) {
    if (pass_off(ctl, pass)) return;
    const int tid = (int)threadIdx.x;
    auto A = [&](int l) { return l == 0 ? a0 : lv[l].a; };
    auto B = [&](int l) { return l == 0 ? b0 : lv[l].b; };
    auto level = [&](int l) {
        MgLevel L = lv[l];
        L.a = A(l);
        L.b = B(l);
        return L;
    };
    auto smooth_n = [&](const MgLevel &L, float *x, float *y, int n) {
        const int cells = L.nx * L.ny;
        for (int t = 0; t < n; ++t) {
            for (int k = tid; k < cells; k += kTailThreads) mg_smooth_cell(L, x, y, k % L.nx, k / L.nx);
            __syncthreads();
            float *tmp = x;
            x = y;
            y = tmp;
        }
    };
    for (int l = s; l < lc; ++l) {
        const MgLevel L = level(l), Cl = level(l + 1);
        smooth_n(L, L.a, L.b, 5);
        for (int k = tid; k < L.nx * L.ny; k += kTailThreads) mg_residual_cell(L, L.b, k % L.nx, k / L.nx);
        __syncthreads();
        for (int k = tid; k < Cl.nx * Cl.ny; k += kTailThreads) mg_restrict_cell(L, Cl, k % Cl.nx, k / Cl.nx);
        __syncthreads();
    }
    {
        const MgLevel L = level(lc);
        smooth_n(L, L.a, L.b, 15);
        if (lc == 0) {   // the whole hierarchy is one level: the caller expects p' in a
            for (int k = tid; k < L.nx * L.ny; k += kTailThreads) L.a[k] = L.b[k];
        }
    }
    for (int l = lc - 1; l >= s; --l) {
        const MgLevel L = level(l), Cl = level(l + 1);
        const float *e = (l + 1 == lc) ? Cl.b : Cl.a;
        for (int k = tid; k < L.nx * L.ny; k += kTailThreads)
            mg_prolong_add_cell(Cl, e, L, L.b, k % L.nx, k / L.nx);
        __syncthreads();
        smooth_n(L, L.b, L.a, 5);
    }
}

// Final residual of the multigrid branch (index.html:783-795): max |A p - rhs|
// over the interior, NaN ignored, published as f32 into a spread slot set.
__global__ __launch_bounds__(kBlock) void k_mg_final_residual(MgLevel L, const float *p,
                                                              uint32_t *slots, const Ctl *ctl,
                                                              int pass, int nbx) {
    if (pass_off(ctl, pass)) return;
    const int i = ((int)blockIdx.x % nbx) * kBlock + (int)threadIdx.x, j = (int)blockIdx.x / nbx;
    const int nx = L.nx;
    float m = 0.0f;
    if (i >= 1 && i <= nx - 2 && j >= 1 && j <= L.ny - 2) {
        const long idx = (long)j * nx + i;
        const double r = ddiv((double)p[idx + 1] + (double)p[idx - 1], L.dx2, L.r_dx2, L.fast) +
                         ddiv((double)p[idx + nx] + (double)p[idx - nx], L.dy2, L.r_dy2, L.fast) -
                         L.denom * (double)p[idx] - (double)L.rhs[idx];
        m = (float)fabs(r);
    }
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) publish_max(slots, (int)blockIdx.x * (kBlock / 64) + ((int)threadIdx.x >> 6), m);
}

inline int grid_of(int nx, int ny, int *nbx) {
    *nbx = cdiv(nx, kBlock);
    return *nbx * ny;
}

}  // namespace

// ------------------------------------------------------------------ launchers

void launch_sor_color(float *pp, const float *rhs, int nx, int ny, const SorConst &k, int color,
                      Ctl *ctl, uint32_t *err_slots, int pass, int it, int tol, float p_tol, int res,
                      hipStream_t s) {
    if (ny < 3) return;
    const int nbx = cdiv(nx / 2, kBlock);
    hipLaunchKernelGGL(k_sor_color, dim3(nbx * (ny - 2)), dim3(kBlock), 0, s, pp, rhs, nx, ny, k,
                       color, ctl, err_slots, pass, it, tol, p_tol, res, nbx);
}

void launch_fill_zero(float *p, size_t n, const Ctl *ctl, int pass, hipStream_t s) {
    const long n4 = (long)(n / 4);
    const int blocks = (int)std::min<long>(std::max<long>(cdiv(n4, kBlock), 1), 4096);
    hipLaunchKernelGGL(k_fill_zero, dim3(blocks), dim3(kBlock), 0, s, (float4 *)p, n4, ctl, pass);
}

void launch_mg_smooth(const MgLevel &L, const float *src, float *dst, const Ctl *ctl, int pass,
                      hipStream_t s) {
    int nbx;
    const int g = grid_of(L.nx, L.ny, &nbx);
    hipLaunchKernelGGL(k_mg_smooth, dim3(g), dim3(kBlock), 0, s, L, src, dst, ctl, pass, nbx);
}

void launch_mg_residual(const MgLevel &L, const float *p, const Ctl *ctl, int pass, hipStream_t s) {
    int nbx;
    const int g = grid_of(L.nx, L.ny, &nbx);
    hipLaunchKernelGGL(k_mg_residual, dim3(g), dim3(kBlock), 0, s, L, p, ctl, pass, nbx);
}

void launch_mg_restrict(const MgLevel &F, const MgLevel &Cl, const Ctl *ctl, int pass, hipStream_t s) {
    int nbx;
    const int g = grid_of(Cl.nx, Cl.ny, &nbx);
    hipLaunchKernelGGL(k_mg_restrict, dim3(g), dim3(kBlock), 0, s, F, Cl, ctl, pass, nbx);
}

void launch_mg_prolong_add(const MgLevel &Cl, const float *e, const MgLevel &F, float *p,
                           const Ctl *ctl, int pass, hipStream_t s) {
    int nbx;
    const int g = grid_of(F.nx, F.ny, &nbx);
    hipLaunchKernelGGL(k_mg_prolong_add, dim3(g), dim3(kBlock), 0, s, Cl, e, F, p, ctl, pass, nbx);
}

void launch_mg_tail(const MgLevel *dev_levels, int s_level, int coarsest, float *a0, float *b0,
                    const Ctl *ctl, int pass, hipStream_t s) {
    hipLaunchKernelGGL(k_mg_tail, dim3(1), dim3(kTailThreads), 0, s, dev_levels, s_level, coarsest,
                       a0, b0, ctl, pass);
}

void launch_mg_final_residual(const MgLevel &L, const float *p, uint32_t *slots, const Ctl *ctl,
                              int pass, hipStream_t s) {
    int nbx;
    const int g = grid_of(L.nx, L.ny, &nbx);
    hipLaunchKernelGGL(k_mg_final_residual, dim3(g), dim3(kBlock), 0, s, L, p, slots, ctl, pass, nbx);
}

}  // namespace cfd
