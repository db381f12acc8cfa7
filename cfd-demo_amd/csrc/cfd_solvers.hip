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

// x / c in the script's double arithmetic.  FAST is a template parameter:
// with a runtime flag the compiler if-converts and evaluates the ~30-instruction
// IEEE f64 division sequence on both paths.
template <int FAST>
__device__ __forceinline__ double ddiv(double x, double c, double r) {
    if (FAST) return x * r;
    return x / c;
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
template <int FAST>
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
            const double h = ddiv<FAST>((double)pp[idx + 1] + (double)pp[idx - 1], k.dx2, k.r_dx2);
            const double v = ddiv<FAST>((double)pp[idx + nx] + (double)pp[idx - nx], k.dy2, k.r_dy2);
            const double p_update = ddiv<FAST>(h + v - (double)rhs[idx], k.denom, k.r_denom);
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

// One whole red-black SOR iteration in one launch (both colors), p' read from
// `src` and written to the other buffer, so p' and rhs cross HBM once per
// iteration (12 B per cell-update) instead of once per color.  A wave owns 64
// lanes x one column pair (one red and one black cell per row) and a segment
// of R interior rows [r0, r0+R) (local rows of the model's slab; a sharded
// slab needs 2 ghost rows of p' and 1 of rhs); all rows it needs — p' rows
// r0-2..r0+R+1 and rhs rows r0-1..r0+R — are read once, then
//   red  rows r0-1..r0+R   from the old black neighbours (src),
//   black rows r0..r0+R-1  from the new red ones (registers),
// exactly the two color passes of k_sor_color over the same values: a red
// update reads only old black cells and boundary cells, a black update only
// new red cells (its vertical and horizontal neighbours have the other
// parity) and boundary cells, which no pass of the iteration changes.  The
// boundary conditions are stored as k_sor_color's black pass stores them.
// Horizontal neighbours come from the adjacent lanes (DPP); lanes 0 and 63
// only feed them, so waves step 62 pairs.  Iteration 0 reads no source: the
// solve starts from p' = 0 (index.html:743).  The last segment of a column
// ends at row_hi and overlaps its neighbour (identical stores).
// As a row march (r2; it replaced a form that loaded all of a segment's rows
// up front, ~80 VGPRs of rows against ~30): the p' and rhs rows stream
// through register rings (prefetched PD steps ahead), so more waves share
// each SIMD.  Step t (0..R+1) forms the
// red cells of row r0-1+t from p' rows r0-2+t..r0+t, then (t >= 2) the black
// cells of row r0-2+t from the red rows of steps t-2..t and stores that row.
template <int FAST, int R, int PD>
struct SorMarch {
    static constexpr int DA = 3 + PD;   // p' ring: rows a = t..t+2 in use, PD in flight
    static constexpr int DB = 2 + PD;   // rhs ring: rows b = t-1, t in use
    float2 AQ[DA], BQ[DB];
    float red[3];                       // red cells of rows r0-1+t-2 .. r0-1+t (slot t % 3)
    const float *src, *rhs;
    float *dst;
    int nx, ny, i0, r0, j0, lo_clamp, hi_clamp, it;
    bool in_dom, out;
    SorConst k;
    float m;

    __device__ __forceinline__ float2 ld(const float *p, int row, bool src_row) const {
        row = min(max(row, lo_clamp), hi_clamp);
        return (in_dom && (!src_row || it > 0)) ? *reinterpret_cast<const float2 *>(p + (long)row * nx + i0)
                                                : make_float2(0.0f, 0.0f);
    }
    __device__ __forceinline__ float relax(float p_old_f, float pe, float pw, float pn, float ps,
                                           float rh, bool upd, bool count) {
        if (!upd) return p_old_f;
        const double p_old = (double)p_old_f;
        const double h = ddiv<FAST>((double)pe + (double)pw, k.dx2, k.r_dx2);
        const double v = ddiv<FAST>((double)pn + (double)ps, k.dy2, k.r_dy2);
        const double p_update = ddiv<FAST>(h + v - (double)rh, k.denom, k.r_denom);
        const double omega = 1.7;
        const float nv = (float)((1.0 - omega) * p_old + omega * p_update);
        if (count) m = fmaxf(m, (float)fabs((double)nv - p_old));
        return nv;
    }
    template <int T>
    __device__ __forceinline__ void step() {
        // red cells of row rr = r0-1+T (p' rows a = T..T+2, rhs row b = T)
        {
            const int rr = r0 - 1 + T;
            const float2 dn = AQ[T % DA], a = AQ[(T + 1) % DA], up = AQ[(T + 2) % DA];
            const float2 rh = BQ[T % DB];
            const bool row_in = j0 + rr >= 1 && j0 + rr <= ny - 2;
            const bool count = out && T >= 1 && T <= R;
            if (((j0 + rr) & 1) == 0) {   // red at x (column i0)
                const int i = i0;
                red[T % 3] = relax(a.x, a.y, from_left(a.y), up.x, dn.x, rh.x,
                                   row_in && i >= 1 && i <= nx - 2, count);
            } else {                      // red at y (column i0 + 1)
                const int i = i0 + 1;
                red[T % 3] = relax(a.y, from_right(a.x), a.x, up.y, dn.y, rh.y,
                                   row_in && i >= 1 && i <= nx - 2, count);
            }
        }
        if constexpr (T >= 2) {
            // black cells of row rb = r0-2+T: own old value p' row a = T, rhs b = T-1
            const int rb = r0 - 2 + T;
            const float2 a = AQ[T % DA];
            const float2 rh = BQ[(T - 1) % DB];
            const float rd = red[(T - 1) % 3], rdn = red[(T - 2) % 3], rup = red[T % 3];
            float2 o;
            if (((j0 + rb) & 1) == 0) {   // red at x, black at y (column i0 + 1)
                const int i = i0 + 1;
                o.x = rd;
                o.y = relax(a.y, from_right(rd), rd, rup, rdn, rh.y, i >= 1 && i <= nx - 2, out);
            } else {                      // black at x (column i0), red at y
                const int i = i0;
                o.y = rd;
                o.x = relax(a.x, rd, from_left(rd), rup, rdn, rh.x, i >= 1 && i <= nx - 2, out);
            }
            if (i0 == 0) o.x = o.y;            // P(0,j) = P(1,j)
            if (i0 + 1 == nx - 1) o.y = 0.0f;  // P(nx-1,j) = 0
            if (out) {
                *reinterpret_cast<float2 *>(dst + (long)rb * nx + i0) = o;
                if (j0 + rb == 1) *reinterpret_cast<float2 *>(dst + (long)(rb - 1) * nx + i0) = o;       // row 0
                if (j0 + rb == ny - 2) *reinterpret_cast<float2 *>(dst + (long)(rb + 1) * nx + i0) = o;  // row ny-1
            }
        }
        // the ring slots the step is done with take the rows DA / DB ahead
        AQ[T % DA] = ld(src, r0 - 2 + T + DA, true);
        if constexpr (T >= 1) BQ[(T - 1) % DB] = ld(rhs, r0 - 1 + T - 1 + DB, false);
    }
    template <int T>
    __device__ __forceinline__ void steps() {
        if constexpr (T <= R + 1) {
            step<T>();
            steps<T + 1>();
        }
    }
    __device__ __forceinline__ void run() {
#pragma unroll
        for (int a = 0; a < DA; ++a) AQ[a] = ld(src, r0 - 2 + a, true);
#pragma unroll
        for (int b = 0; b < DB; ++b) BQ[b] = ld(rhs, r0 - 1 + b, false);
        steps<0>();
    }
};

template <int FAST, int R>
__global__ __launch_bounds__(kBlock) void k_sor_march(const float *__restrict__ pa,
                                                      const float *__restrict__ pb,
                                                      float *__restrict__ qa, float *__restrict__ qb,
                                                      const float *__restrict__ rhs, int nx, int ny,
                                                      SorConst k, Ctl *ctl, uint32_t *err_slots,
                                                      int pass, int it, int tol, float p_tol,
                                                      int res, int nwc, int nseg, int row_lo,
                                                      int row_hi, int j0, int lo_clamp,
                                                      int hi_clamp) {
    if (pass_off(ctl, pass)) return;
    if (tol && it > 0 &&
        read_max(err_slots + (size_t)(it - 1) * kResSlots * kResStride, ctl->err[it - 1]) < p_tol)
        return;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int lane = (int)threadIdx.x & 63;
    const int bid = (int)blockIdx.x;
    const int wc = bid % nwc;
    const int seg = (bid / nwc) * (kBlock / 64) + wave;
    if (seg >= nseg) return;   // wave-uniform
    SorMarch<FAST, R, 2> w;
    const int si = (ctl->cur + it) & 1;
    w.src = si ? pb : pa;
    w.dst = si ? qa : qb;
    w.rhs = rhs;
    w.nx = nx;
    w.ny = ny;
    w.r0 = row_lo + min(seg * R, row_hi - row_lo - R);
    w.j0 = j0;
    w.lo_clamp = lo_clamp;
    w.hi_clamp = hi_clamp;
    w.it = it;
    const int c = wc * 62 - 1 + lane;
    w.in_dom = c >= 0 && 2 * c < nx;
    w.out = w.in_dom && lane >= 1 && lane <= 62;
    w.i0 = 2 * c;
    w.k = k;
    w.m = 0.0f;
    w.run();
    if (!res) return;
    const float m = wave_max(w.out ? w.m : 0.0f);
    if (lane == 0) publish_max(err_slots + (size_t)it * kResSlots * kResStride, bid * (kBlock / 64) + wave, m);
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
template <int FAST>
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
    const double h = ddiv<FAST>(p_e + p_w, L.dx2, L.r_dx2);
    const double v = ddiv<FAST>(p_n + p_s, L.dy2, L.r_dy2);
    dst[idx] = (float)ddiv<FAST>(h + v - (double)L.rhs[idx], L.denom, L.r_denom);
}

// r = rhs - A p on the interior, 0 on the boundary (index.html:1430-1441).
template <int FAST>
__device__ __forceinline__ void mg_residual_cell(const MgLevel &L, const float *__restrict__ p,
                                                 int i, int j) {
    const int nx = L.nx;
    const long idx = (long)j * nx + i;
    if (i == 0 || j == 0 || i == nx - 1 || j == L.ny - 1) {
        L.r[idx] = 0.0f;
        return;
    }
    const double p_e = p[idx + 1], p_w = p[idx - 1], p_n = p[idx + nx], p_s = p[idx - nx];
    const double ap = ddiv<FAST>(p_e + p_w, L.dx2, L.r_dx2) +
                      ddiv<FAST>(p_n + p_s, L.dy2, L.r_dy2) - L.denom * (double)p[idx];
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
// the four coarse values of fine cell (i, j)'s bilinear stencil
struct ProlongIn {
    float e00, e01, e10, e11;
};
__device__ __forceinline__ ProlongIn mg_prolong_load(const MgLevel &Cl, const float *__restrict__ e,
                                                     int i, int j) {
    const int nxc = Cl.nx, nyc = Cl.ny;
    const int j0 = j >> 1, i0 = i >> 1;
    const int j1 = min(j0 + 1, nyc - 1), i1 = min(i0 + 1, nxc - 1);
    return {e[(long)j0 * nxc + i0], e[(long)j0 * nxc + i1], e[(long)j1 * nxc + i0],
            e[(long)j1 * nxc + i1]};
}
__device__ __forceinline__ float mg_prolong_combine(const ProlongIn &q, float p_old, int i, int j) {
    const double b = (j & 1) ? 0.5 : 0.0, a = (i & 1) ? 0.5 : 0.0;
    const double val = (1 - a) * (1 - b) * (double)q.e00 + a * (1 - b) * (double)q.e01 +
                       (1 - a) * b * (double)q.e10 + a * b * (double)q.e11;
    return (float)((double)p_old + (double)(float)val);
}
__device__ __forceinline__ float mg_prolong_add_val(const MgLevel &Cl, const float *__restrict__ e,
                                                    float p_old, int i, int j) {
    return mg_prolong_combine(mg_prolong_load(Cl, e, i, j), p_old, i, j);
}

__device__ __forceinline__ void mg_prolong_add_cell(const MgLevel &Cl, const float *__restrict__ e,
                                                    const MgLevel &F, float *__restrict__ p, int i,
                                                    int j) {
    const long idx = (long)j * F.nx + i;
    p[idx] = mg_prolong_add_val(Cl, e, p[idx], i, j);
}

// Five mgSmooth sweeps in one launch (temporal blocking): a block owns a
// window of kSmW columns x kSmH rows of p and rhs — its kSmW - 2T output
// columns by kSmTH output rows plus T halo cells on every side — and runs the
// T sweeps on it on-chip, storing the output tile once, so p and rhs cross HBM
// once per T sweeps instead of T times.  Each thread owns one window column
// in registers (p, rhs; vertical neighbours are register neighbours, the
// unrolled row loop keeps every index static); only the column exchange with
// the neighbouring threads goes through LDS (ping-pong, one barrier per
// sweep).  Cells whose dependency cone leaves the window compute garbage that
// no valid cell reads: after sweep s the window minus s cells on each side is
// exact, so the output tile is exact after T.  Every sweep is the
// single-sweep arithmetic of mg_smooth_cell, so results are identical.
constexpr int kSmT = 5;                    // sweeps per launch (mgVcycle pre/post-smooth, :1427, :1469)
constexpr int kSmW = 256;                  // window columns = threads per block
constexpr int kSmOW = kSmW - 2 * kSmT;     // output columns per block
// output rows per block: tall tiles (less halo recompute) on big levels,
// short ones (shorter serial row march per block) on small levels
#ifndef CFD_MG_TH_BIG
#define CFD_MG_TH_BIG 30
#endif
constexpr int kSmTHBig = CFD_MG_TH_BIG, kSmTHSmall = 14;

template <int FAST, int kSmTH>
__global__ __launch_bounds__(kSmW) void k_mg_smooth5(MgLevel L, const float *__restrict__ src,
                                                     float *__restrict__ dst, const Ctl *ctl,
                                                     int pass, int nbx) {
    constexpr int kSmH = kSmTH + 2 * kSmT;     // window rows
    if (pass_off(ctl, pass)) return;
    __shared__ float xch[2][kSmH][kSmW];
    const int x = (int)threadIdx.x;
    const int gx0 = ((int)blockIdx.x % nbx) * kSmOW - kSmT;   // window origin (global)
    const int gy0 = ((int)blockIdx.x / nbx) * kSmTH - kSmT;
    const int nx = L.nx, ny = L.ny;
    const int gx = gx0 + x;
    const bool col_in = gx >= 0 && gx < nx;
    const bool bcol = gx == 0 || gx == nx - 1;
    const int xl = x > 0 ? x - 1 : 0, xr = x < kSmW - 1 ? x + 1 : kSmW - 1;
    float c[kSmH];
    double rh[kSmH];
#pragma unroll
    for (int y = 0; y < kSmH; ++y) {
        const int gy = gy0 + y;
        const bool in = col_in && gy >= 0 && gy < ny;
        const long k = (long)gy * nx + gx;
        c[y] = in ? src[k] : 0.0f;
        rh[y] = in ? (double)L.rhs[k] : 0.0;
        xch[0][y][x] = c[y];
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < kSmT; ++s) {
        const int cur = s & 1;
        // rows top-down in place: `below` keeps the old value of row y-1
        double below = (double)c[0];
#pragma unroll
        for (int y = 1; y < kSmH - 1; ++y) {
            const int gy = gy0 + y;
            const double here = (double)c[y];
            if (!(bcol || gy <= 0 || gy >= ny - 1)) {
                const double h = ddiv<FAST>((double)xch[cur][y][xr] + (double)xch[cur][y][xl],
                                            L.dx2, L.r_dx2);
                const double vt = ddiv<FAST>((double)c[y + 1] + below, L.dy2, L.r_dy2);
                c[y] = (float)ddiv<FAST>(h + vt - rh[y], L.denom, L.r_denom);
            }
            below = here;
            if (s + 1 < kSmT) xch[cur ^ 1][y][x] = c[y];
        }
        if (s + 1 < kSmT) __syncthreads();
    }
    if (col_in && x >= kSmT && x < kSmW - kSmT) {
#pragma unroll
        for (int y = kSmT; y < kSmH - kSmT; ++y) {
            const int gy = gy0 + y;
            if (gy < ny) dst[(long)gy * nx + gx] = c[y];
        }
    }
}

// The same five sweeps with one WAVE per window (64 columns x kTH + 10 rows)
// and no LDS: a lane owns one window column in registers (p as f32, rhs as
// f32 — its widening to double is exact), and the old values of the
// horizontal neighbours come from the adjacent lanes by DPP: the wave reads
// them in the same instruction stream before any lane writes the row, which
// is exactly the LDS copy of the previous sweep's row.  The 80 KB LDS
// exchange of the block form held occupancy to 2 workgroups per CU; here
// registers alone bound it.  Output: lanes kSmT..63-kSmT of the window.
// PRO: the up-leg's prolong-add (index.html:1464-1466) is applied to the
// window as it is loaded — src + prolongate(e) exactly as
// mg_prolong_add_cell forms it — so the added field is never stored: one
// grid-wide pass (read src and e, write src) less per level and cycle.
// RES: the down-leg's residual r = rhs - A p (index.html:1430-1441) of the
// smoothed field is formed in the same launch: the window keeps one more
// halo cell per side (kSmT + 1), so the smoothed values the residual reads
// around the output tile are exact too, and the residual pass (read p and
// rhs again, write r) goes.
template <int FAST, int kTH, bool PRO, bool RES = false>
__global__ __launch_bounds__(kBlock) void k_mg_smooth5w(MgLevel L, const float *__restrict__ src,
                                                        float *__restrict__ dst, const Ctl *ctl,
                                                        int pass, int nwx, int nwin, MgLevel Cl,
                                                        const float *__restrict__ e) {
    constexpr int kHL = kSmT + (RES ? 1 : 0);   // window halo
    constexpr int kH = kTH + 2 * kHL;           // window rows
    constexpr int kOW = 64 - 2 * kHL;           // output columns per window
    if (pass_off(ctl, pass)) return;
    const int lane = (int)threadIdx.x & 63;
    const int win = (int)blockIdx.x * (kBlock / 64) + __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    if (win >= nwin) return;   // wave-uniform
    const int nx = L.nx, ny = L.ny;
    const int gx = (win % nwx) * kOW - kHL + lane;
    const int gy0 = L.lo + (win / nwx) * kTH - kHL;   // windows tile output rows [lo, hi)
    const bool col_in = gx >= 0 && gx < nx;
    const bool bcol = gx == 0 || gx == nx - 1;
    float c[kH], rh[kH];
#pragma unroll
    for (int y = 0; y < kH; ++y) {
        const int gy = gy0 + y;
        const bool in = col_in && gy >= L.ys && gy < L.ye;
        const long k = (long)gy * nx + gx;
        c[y] = in ? (PRO ? mg_prolong_add_val(Cl, e, src[k], gx, gy) : src[k]) : 0.0f;
        rh[y] = in ? L.rhs[k] : 0.0f;
    }
#pragma unroll 1
    for (int s = 0; s < kSmT; ++s) {
        // rows top-down in place: `below` keeps the old value of row y-1
        double below = (double)c[0];
#pragma unroll
        for (int y = 1; y < kH - 1; ++y) {
            const int gy = gy0 + y;
            const double here = (double)c[y];
            const float left = from_left(c[y]), right = from_right(c[y]);
            if (!(bcol || gy <= 0 || gy >= ny - 1)) {
                const double h = ddiv<FAST>((double)right + (double)left, L.dx2, L.r_dx2);
                const double vt = ddiv<FAST>((double)c[y + 1] + below, L.dy2, L.r_dy2);
                c[y] = (float)ddiv<FAST>(h + vt - (double)rh[y], L.denom, L.r_denom);
            }
            below = here;
        }
    }
    if (RES) {
        // r of the output tile (mg_residual_cell's expression)
        const bool out = col_in && lane >= kHL && lane < 64 - kHL;
#pragma unroll
        for (int y = kHL; y < kH - kHL; ++y) {
            const int gy = gy0 + y;
            const float left = from_left(c[y]), right = from_right(c[y]);
            float r = 0.0f;
            if (!(bcol || gy <= 0 || gy >= ny - 1)) {
                const double ap = ddiv<FAST>((double)right + (double)left, L.dx2, L.r_dx2) +
                                  ddiv<FAST>((double)c[y + 1] + (double)c[y - 1], L.dy2, L.r_dy2) -
                                  L.denom * (double)c[y];
                r = (float)((double)rh[y] - ap);
            }
            if (out && gy < L.hi) L.r[(long)gy * nx + gx] = r;
        }
    }
    if (col_in && lane >= kHL && lane < 64 - kHL) {
#pragma unroll
        for (int y = kHL; y < kH - kHL; ++y) {
            const int gy = gy0 + y;
            if (gy < L.hi) dst[(long)gy * nx + gx] = c[y];
        }
    }
}

// The same five sweeps (and the PRO / RES fusions) as a register-ring row
// march: a wave owns a 64-column strip and kMgSlots consecutive input rows;
// stage s (1..5) of slot t computes row t - 2s of sweep s from the rows sweep
// s-1 finished in the three earlier slots (lag 2: the five updates of a slot
// are independent, so one wave has five-way ILP).  A row of each sweep is
// computed once per strip instead of once per overlapping window, so the
// vertical halo recompute of k_mg_smooth5w (10 rows per 30) shrinks to the
// march's warm-up (15-17 slots per 128).  Every update is mg_smooth_cell's
// expression and every stored value is computed from exact inputs: stage s
// of row u is exact for u >= s (the rows below are the real field, clamped
// loads only past the grid), the halo columns as in k_mg_smooth5w.
#ifndef CFD_MG_SLOTS
#define CFD_MG_SLOTS 128
#endif
constexpr int kMgSlots = CFD_MG_SLOTS;   // slots per wave (multiple of kMgU)
constexpr int kMgU = 16;         // slot unroll: W rings of 4, rhs ring of 16
constexpr int kMgPD = 4;         // prefetch distance of p and rhs rows
template <bool RES>
constexpr int mg_march_rows() { return kMgSlots - (RES ? 17 : 15); }

template <int FAST, bool PRO, bool RES>
__global__ __launch_bounds__(kBlock) void k_mg_smooth5m(MgLevel L, const float *__restrict__ src,
                                                        float *__restrict__ dst, const Ctl *ctl,
                                                        int pass, int nwx, int nwin, MgLevel Cl,
                                                        const float *__restrict__ e) {
    constexpr int kHL = kSmT + (RES ? 1 : 0);
    constexpr int kOW = 64 - 2 * kHL;
    constexpr int R = mg_march_rows<RES>();
    constexpr int NS = kSmT + 1;                 // stage rings (0 = input)
    if (pass_off(ctl, pass)) return;
    const int lane = (int)threadIdx.x & 63;
    const int win = (int)blockIdx.x * (kBlock / 64) + __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    if (win >= nwin) return;   // wave-uniform
    const int nx = L.nx, ny = L.ny;
    const int gx = (win % nwx) * kOW - kHL + lane;
    const int r0 = L.lo + (win / nwx) * R;       // first output row
    const int ra = r0 - kHL;                     // row of slot 0
    const bool col_in = gx >= 0 && gx < nx;
    const bool bcol = gx == 0 || gx == nx - 1;
    const bool out = col_in && lane >= kHL && lane < 64 - kHL;
    const int gxc = min(max(gx, 0), nx - 1);
    const float *__restrict__ ps = src + gxc;
    const float *__restrict__ prh = L.rhs + gxc;
    // the warm-up slots read ring rows from before slot 0; their values reach
    // only rows that are never stored, but they must not be uninitialised
    float W[NS][4];
#pragma unroll
    for (int a = 0; a < NS; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) W[a][b] = 0.0f;
    float RH[kMgU];
    float PQ[4];
    ProlongIn EQ[4];
    // loads stay in the stored rows (past the grid or the slab's ghosts: clamped)
    auto rowc = [&](int u) { return min(max(ra + u, L.ys), L.ye - 1); };
#pragma unroll
    for (int u = 0; u < kMgPD; ++u) {
        const int gy = rowc(u);
        PQ[u] = ps[(long)gy * nx];
        if (PRO) EQ[u] = mg_prolong_load(Cl, e, gxc, gy);
        RH[u] = prh[(long)gy * nx];
    }
    for (int base = 0; base < kMgSlots; base += kMgU) {
#pragma unroll
        for (int j = 0; j < kMgU; ++j) {
            const int t = base + j;
            // input row t (stage 0), then the prefetch of row t + kMgPD
            {
                const int gy = rowc(t);
                W[0][j % 4] = PRO ? mg_prolong_combine(EQ[j % 4], PQ[j % 4], gxc, gy) : PQ[j % 4];
                const int gp = rowc(t + kMgPD);
                PQ[j % 4] = ps[(long)gp * nx];
                if (PRO) EQ[j % 4] = mg_prolong_load(Cl, e, gxc, gp);
                RH[(j + kMgPD) % kMgU] = prh[(long)gp * nx];
            }
#pragma unroll
            for (int st = 1; st <= kSmT; ++st) {
                const int u = t - 2 * st;            // row of this stage
                const int x = ra + u;
                const float up = W[st - 1][(j - 2 * st + 1 + 64) % 4];
                const float c = W[st - 1][(j - 2 * st + 64) % 4];
                const float dn = W[st - 1][(j - 2 * st - 1 + 64) % 4];
                const float left = from_left(c), right = from_right(c);
                const double h = ddiv<FAST>((double)right + (double)left, L.dx2, L.r_dx2);
                const double vt = ddiv<FAST>((double)up + (double)dn, L.dy2, L.r_dy2);
                const float nv = (float)ddiv<FAST>(h + vt - (double)RH[(j - 2 * st + 64) % kMgU],
                                                  L.denom, L.r_denom);
                W[st][(j - 2 * st + 64) % 4] = (bcol || x <= 0 || x >= ny - 1) ? c : nv;
            }
            {
                // sweep 5 of row t - 10 is final
                const int u = t - 2 * kSmT, x = ra + u;
                if (out && u >= kHL && u < kHL + R && x < L.hi)
                    dst[(long)x * nx + gx] = W[kSmT][(j - 2 * kSmT + 64) % 4];
            }
            if (RES) {
                // residual of row t - 11 from sweep 5's rows t - 12 .. t - 10
                const int u = t - 2 * kSmT - 1, x = ra + u;
                const float c = W[kSmT][(j - 2 * kSmT - 1 + 64) % 4];
                const float up = W[kSmT][(j - 2 * kSmT + 64) % 4];
                const float dn = W[kSmT][(j - 2 * kSmT - 2 + 64) % 4];
                const float left = from_left(c), right = from_right(c);
                const double ap = ddiv<FAST>((double)right + (double)left, L.dx2, L.r_dx2) +
                                  ddiv<FAST>((double)up + (double)dn, L.dy2, L.r_dy2) -
                                  L.denom * (double)c;
                const float r = (bcol || x <= 0 || x >= ny - 1)
                                    ? 0.0f
                                    : (float)((double)RH[(j - 2 * kSmT - 1 + 64) % kMgU] - ap);
                if (out && u >= kHL && u < kHL + R && x < L.hi) L.r[(long)x * nx + gx] = r;
            }
        }
    }
}

// Grid-wide passes: one cell per thread, nbx blocks per row.
template <int FAST>
__global__ __launch_bounds__(kBlock) void k_mg_smooth(MgLevel L, const float *src, float *dst,
                                                      const Ctl *ctl, int pass, int nbx) {
    if (pass_off(ctl, pass)) return;
    const int i = ((int)blockIdx.x % nbx) * kBlock + (int)threadIdx.x, j = (int)blockIdx.x / nbx;
    if (i < L.nx) mg_smooth_cell<FAST>(L, src, dst, i, j);
}

template <int FAST>
__global__ __launch_bounds__(kBlock) void k_mg_residual(MgLevel L, const float *p, const Ctl *ctl,
                                                        int pass, int nbx) {
    if (pass_off(ctl, pass)) return;
    const int i = ((int)blockIdx.x % nbx) * kBlock + (int)threadIdx.x, j = (int)blockIdx.x / nbx;
    if (i < L.nx) mg_residual_cell<FAST>(L, p, i, j);
}

__global__ __launch_bounds__(kBlock) void k_mg_restrict(MgLevel F, MgLevel Cl, const Ctl *ctl,
                                                        int pass, int nbx) {
    if (pass_off(ctl, pass)) return;
    const int i = ((int)blockIdx.x % nbx) * kBlock + (int)threadIdx.x;
    const int j = Cl.lo + (int)blockIdx.x / nbx;   // coarse rows [lo, hi)
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

template <int FAST>
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
            for (int k = tid; k < cells; k += kTailThreads) mg_smooth_cell<FAST>(L, x, y, k % L.nx, k / L.nx);
            __syncthreads();
            float *tmp = x;
            x = y;
            y = tmp;
        }
    };
    for (int l = s; l < lc; ++l) {
        const MgLevel L = level(l), Cl = level(l + 1);
        smooth_n(L, L.a, L.b, 5);
        for (int k = tid; k < L.nx * L.ny; k += kTailThreads) mg_residual_cell<FAST>(L, L.b, k % L.nx, k / L.nx);
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
// A block walks a band of `rows` rows (one column per thread) and publishes
// one maximum: per-wave atomics over a 4096^2 grid would serialise.
template <int FAST>
__global__ __launch_bounds__(kBlock) void k_mg_final_residual(MgLevel L, const float *p,
                                                              uint32_t *slots, const Ctl *ctl,
                                                              int pass, int nbx, int rows) {
    if (pass_off(ctl, pass)) return;
    __shared__ float wmax[kBlock / 64];
    const int i = ((int)blockIdx.x % nbx) * kBlock + (int)threadIdx.x;
    const int jb = L.lo + ((int)blockIdx.x / nbx) * rows;   // rows [lo, hi)
    const int nx = L.nx;
    float m = 0.0f;
    if (i >= 1 && i <= nx - 2) {
        const int j1 = min(jb + rows, min(L.hi, L.ny - 1));
        for (int j = max(jb, 1); j < j1; ++j) {
            const long idx = (long)j * nx + i;
            const double r = ddiv<FAST>((double)p[idx + 1] + (double)p[idx - 1], L.dx2, L.r_dx2) +
                             ddiv<FAST>((double)p[idx + nx] + (double)p[idx - nx], L.dy2, L.r_dy2) -
                             L.denom * (double)p[idx] - (double)L.rhs[idx];
            m = fmaxf(m, (float)fabs(r));
        }
    }
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float b = wmax[0];
        for (int w = 1; w < kBlock / 64; ++w) b = fmaxf(b, wmax[w]);
        publish_max(slots, (int)blockIdx.x, b);
    }
}

// interior rows per k_sor_march segment: 32 where the slab has
// them (4096^2, 200 iterations: 9.02 ms; 8 rows 9.60, 16 rows 9.94, 64 rows
// 13.45), else 16 (the minimum: sor_fused_ok)
constexpr int kSorRows = 16, kSorRowsBig = 32;

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
    if (k.fast)
        hipLaunchKernelGGL(k_sor_color<1>, dim3(nbx * (ny - 2)), dim3(kBlock), 0, s, pp, rhs, nx, ny,
                           k, color, ctl, err_slots, pass, it, tol, p_tol, res, nbx);
    else
        hipLaunchKernelGGL(k_sor_color<0>, dim3(nbx * (ny - 2)), dim3(kBlock), 0, s, pp, rhs, nx, ny,
                           k, color, ctl, err_slots, pass, it, tol, p_tol, res, nbx);
}

bool sor_fused_ok(int nx, int nrows) { return nx % 2 == 0 && nx >= 4 && nrows >= kSorRows; }

void launch_sor_fused(float *pa, float *pb, const float *rhs, int nx, int ny, const SorConst &k,
                      Ctl *ctl, uint32_t *err_slots, int pass, int it, int tol, float p_tol, int res,
                      int row_lo, int row_hi, int j0, int lo_clamp, int hi_clamp, hipStream_t s) {
    const int nwc = cdiv(nx / 2, 62);
    const bool big = row_hi - row_lo >= kSorRowsBig;
    const int nseg = cdiv(row_hi - row_lo, big ? kSorRowsBig : kSorRows);
    const dim3 grid(nwc * cdiv(nseg, kBlock / 64));
#define CFD_LAUNCH_SOR(KER, FASTV, RR)                                                              \
    hipLaunchKernelGGL((KER<FASTV, RR>), grid, dim3(kBlock), 0, s, pa, pb, pa, pb, rhs,              \
                       nx, ny, k, ctl, err_slots, pass, it, tol, p_tol, res, nwc, nseg, row_lo,      \
                       row_hi, j0, lo_clamp, hi_clamp)
    if (k.fast && big)
        CFD_LAUNCH_SOR(k_sor_march, 1, kSorRowsBig);
    else if (k.fast)
        CFD_LAUNCH_SOR(k_sor_march, 1, kSorRows);
    else if (big)
        CFD_LAUNCH_SOR(k_sor_march, 0, kSorRowsBig);
    else
        CFD_LAUNCH_SOR(k_sor_march, 0, kSorRows);
#undef CFD_LAUNCH_SOR
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
    if (L.fast)
        hipLaunchKernelGGL(k_mg_smooth<1>, dim3(g), dim3(kBlock), 0, s, L, src, dst, ctl, pass, nbx);
    else
        hipLaunchKernelGGL(k_mg_smooth<0>, dim3(g), dim3(kBlock), 0, s, L, src, dst, ctl, pass, nbx);
}

static int mg_smooth_mode() {
    // CFD_MG_SMOOTH: 1 the LDS block form, 2 the row march on every level,
    // 3 the wave windows on every level, 4 the march on levels of at least
    // 2^22 cells and the windows below; default
    // (0): as 4 (4096^2 solve: windows 2.21, march everywhere 1.96, march
    // from 2^23 1.90, from 2^22 1.70, from 2^21 1.71 ms;
    // profiles/r2/mg/mgm2.log, mg_min_ab.log)
    // read per launch (a few per V-cycle level) so tests can switch forms
    const char *e = getenv("CFD_MG_SMOOTH");
    return e ? atoi(e) : 0;
}

bool mg_smooth_wave_form() { return mg_smooth_mode() != 1; }

// the row march for this level?
static bool mg_use_march(const MgLevel &L) {
    const int m = mg_smooth_mode();
    if (m == 2) return true;
    constexpr int lg = 22;   // log2 cells of the smallest march level
    return (m == 0 || m == 4) && (long)L.nx * L.ny >= (1L << lg);
}

template <bool PRO, bool RES>
static void launch_mg_march(const MgLevel &L, const float *src, float *dst, const Ctl *ctl, int pass,
                            const MgLevel &Cl, const float *e, hipStream_t s) {
    constexpr int kHL = kSmT + (RES ? 1 : 0);
    const int nwx = cdiv(L.nx, 64 - 2 * kHL);
    const int nwin = nwx * cdiv(L.hi - L.lo, mg_march_rows<RES>());
    const dim3 grid(cdiv(nwin, kBlock / 64)), block(kBlock);
    if (L.fast)
        hipLaunchKernelGGL((k_mg_smooth5m<1, PRO, RES>), grid, block, 0, s, L, src, dst, ctl, pass, nwx, nwin, Cl, e);
    else
        hipLaunchKernelGGL((k_mg_smooth5m<0, PRO, RES>), grid, block, 0, s, L, src, dst, ctl, pass, nwx, nwin, Cl, e);
}

void launch_mg_prolong_smooth5(const MgLevel &Cl, const float *e, const MgLevel &L, const float *src,
                               float *dst, const Ctl *ctl, int pass, hipStream_t s) {
    if (mg_use_march(L)) return launch_mg_march<true, false>(L, src, dst, ctl, pass, Cl, e, s);
    const bool big = (long)L.nx * L.ny >= (1L << 23);
    const int nwx = cdiv(L.nx, 64 - 2 * kSmT);
    const int nwin = nwx * cdiv(L.hi - L.lo, big ? kSmTHBig : kSmTHSmall);
    const dim3 grid(cdiv(nwin, kBlock / 64)), block(kBlock);
#define CFD_LAUNCH_PSM5W(FASTV, TH) \
    hipLaunchKernelGGL((k_mg_smooth5w<FASTV, TH, true>), grid, block, 0, s, L, src, dst, ctl, pass, nwx, nwin, Cl, e)
    if (L.fast && big)
        CFD_LAUNCH_PSM5W(1, kSmTHBig);
    else if (L.fast)
        CFD_LAUNCH_PSM5W(1, kSmTHSmall);
    else if (big)
        CFD_LAUNCH_PSM5W(0, kSmTHBig);
    else
        CFD_LAUNCH_PSM5W(0, kSmTHSmall);
#undef CFD_LAUNCH_PSM5W
}

void launch_mg_smooth5_residual(const MgLevel &L, const float *src, float *dst, const Ctl *ctl,
                                int pass, hipStream_t s) {
    if (mg_use_march(L)) return launch_mg_march<false, true>(L, src, dst, ctl, pass, L, nullptr, s);
    const bool big = (long)L.nx * L.ny >= (1L << 23);
    const int nwx = cdiv(L.nx, 64 - 2 * (kSmT + 1));
    const int nwin = nwx * cdiv(L.hi - L.lo, big ? kSmTHBig : kSmTHSmall);
    const dim3 grid(cdiv(nwin, kBlock / 64)), block(kBlock);
#define CFD_LAUNCH_RSM5W(FASTV, TH) \
    hipLaunchKernelGGL((k_mg_smooth5w<FASTV, TH, false, true>), grid, block, 0, s, L, src, dst, ctl, pass, nwx, nwin, L, nullptr)
    if (L.fast && big)
        CFD_LAUNCH_RSM5W(1, kSmTHBig);
    else if (L.fast)
        CFD_LAUNCH_RSM5W(1, kSmTHSmall);
    else if (big)
        CFD_LAUNCH_RSM5W(0, kSmTHBig);
    else
        CFD_LAUNCH_RSM5W(0, kSmTHSmall);
#undef CFD_LAUNCH_RSM5W
}

void launch_mg_smooth5(const MgLevel &L, const float *src, float *dst, const Ctl *ctl, int pass,
                       hipStream_t s) {
    if (mg_smooth_wave_form() && mg_use_march(L))
        return launch_mg_march<false, false>(L, src, dst, ctl, pass, L, nullptr, s);
    if (mg_smooth_wave_form()) {
        const bool big = (long)L.nx * L.ny >= (1L << 23);
        const int nwx = cdiv(L.nx, 64 - 2 * kSmT);
        const int nwin = nwx * cdiv(L.hi - L.lo, big ? kSmTHBig : kSmTHSmall);
        const dim3 grid(cdiv(nwin, kBlock / 64)), block(kBlock);
#define CFD_LAUNCH_SM5W(FASTV, TH) \
        hipLaunchKernelGGL((k_mg_smooth5w<FASTV, TH, false>), grid, block, 0, s, L, src, dst, ctl, pass, nwx, nwin, L, nullptr)
        if (L.fast && big)
            CFD_LAUNCH_SM5W(1, kSmTHBig);
        else if (L.fast)
            CFD_LAUNCH_SM5W(1, kSmTHSmall);
        else if (big)
            CFD_LAUNCH_SM5W(0, kSmTHBig);
        else
            CFD_LAUNCH_SM5W(0, kSmTHSmall);
#undef CFD_LAUNCH_SM5W
        return;
    }
    const int nbx = cdiv(L.nx, kSmOW);
    const bool big = (long)L.nx * L.ny >= (1L << 23);
    const int nby = cdiv(L.ny, big ? kSmTHBig : kSmTHSmall);
    const dim3 grid(nbx * nby), block(kSmW);
    if (L.fast && big)
        hipLaunchKernelGGL((k_mg_smooth5<1, kSmTHBig>), grid, block, 0, s, L, src, dst, ctl, pass, nbx);
    else if (L.fast)
        hipLaunchKernelGGL((k_mg_smooth5<1, kSmTHSmall>), grid, block, 0, s, L, src, dst, ctl, pass, nbx);
    else if (big)
        hipLaunchKernelGGL((k_mg_smooth5<0, kSmTHBig>), grid, block, 0, s, L, src, dst, ctl, pass, nbx);
    else
        hipLaunchKernelGGL((k_mg_smooth5<0, kSmTHSmall>), grid, block, 0, s, L, src, dst, ctl, pass, nbx);
}

void launch_mg_residual(const MgLevel &L, const float *p, const Ctl *ctl, int pass, hipStream_t s) {
    int nbx;
    const int g = grid_of(L.nx, L.ny, &nbx);
    if (L.fast)
        hipLaunchKernelGGL(k_mg_residual<1>, dim3(g), dim3(kBlock), 0, s, L, p, ctl, pass, nbx);
    else
        hipLaunchKernelGGL(k_mg_residual<0>, dim3(g), dim3(kBlock), 0, s, L, p, ctl, pass, nbx);
}

void launch_mg_restrict(const MgLevel &F, const MgLevel &Cl, const Ctl *ctl, int pass, hipStream_t s) {
    if (Cl.hi <= Cl.lo) return;
    int nbx;
    const int g = grid_of(Cl.nx, Cl.hi - Cl.lo, &nbx);
    hipLaunchKernelGGL(k_mg_restrict, dim3(g), dim3(kBlock), 0, s, F, Cl, ctl, pass, nbx);
}

void launch_mg_prolong_add(const MgLevel &Cl, const float *e, const MgLevel &F, float *p,
                           const Ctl *ctl, int pass, hipStream_t s) {
    int nbx;
    const int g = grid_of(F.nx, F.ny, &nbx);
    hipLaunchKernelGGL(k_mg_prolong_add, dim3(g), dim3(kBlock), 0, s, Cl, e, F, p, ctl, pass, nbx);
}

void launch_mg_tail(const MgLevel *dev_levels, int s_level, int coarsest, float *a0, float *b0,
                    int fast, const Ctl *ctl, int pass, hipStream_t s) {
    if (fast)
        hipLaunchKernelGGL(k_mg_tail<1>, dim3(1), dim3(kTailThreads), 0, s, dev_levels, s_level,
                           coarsest, a0, b0, ctl, pass);
    else
        hipLaunchKernelGGL(k_mg_tail<0>, dim3(1), dim3(kTailThreads), 0, s, dev_levels, s_level,
                           coarsest, a0, b0, ctl, pass);
}

void launch_mg_final_residual(const MgLevel &L, const float *p, uint32_t *slots, const Ctl *ctl,
                              int pass, hipStream_t s) {
    const int nbx = cdiv(L.nx, kBlock);
    const int rows = 32;
    const dim3 grid(nbx * std::max(1, cdiv(L.hi - L.lo, rows)));
    if (L.fast)
        hipLaunchKernelGGL(k_mg_final_residual<1>, grid, dim3(kBlock), 0, s, L, p, slots, ctl, pass,
                           nbx, rows);
    else
        hipLaunchKernelGGL(k_mg_final_residual<0>, grid, dim3(kBlock), 0, s, L, p, slots, ctl, pass,
                           nbx, rows);
}

}  // namespace cfd
