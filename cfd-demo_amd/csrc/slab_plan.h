// slab_plan.h — host-only 1D row-slab decomposition plan.
//
// Pure integer logic shared by the HIP runtime (cfd_model.hip) and, through
// the C ABI (cfd_plan_*), by the multi-rank CPU tests: which global rows a
// rank owns, which rows each Jacobi sweep recomputes (deep halos), when p'
// ghost rows are exchanged, and which local rows go to / come from each
// neighbour for every field.  Local row lj = global row - j0.
#pragma once
#include <algorithm>
#include <cstdint>

namespace cfd {

// Even split of ny pressure rows; the first ny % n ranks get one extra row.
inline void plan_slab(uint64_t ny, int n_ranks, int rank, uint64_t *j0, uint64_t *j1) {
    const uint64_t base = ny / (uint64_t)n_ranks, rem = ny % (uint64_t)n_ranks;
    const uint64_t r = (uint64_t)rank;
    *j0 = r * base + (r < rem ? r : rem);
    *j1 = *j0 + base + (r < rem ? 1 : 0);
}

// Sweep `it` of a fixed-count solve with halo depth hg: local rows [lo, hi)
// to recompute (owned rows plus a band of ghost rows that shrinks by one
// per sweep since the last exchange, clipped to global rows 1..ny-2), and
// whether hg rows of the freshly written p' buffer are exchanged after it.
// Invariant: after an exchange the hg ghost rows on each side are exact;
// sweep s (0-based since the exchange) reads rows up to hg - s deep.
inline void plan_sweep(int j0, int nyl, int ny, int hg, int it, int iters, int *lo, int *hi,
                       int *exchange) {
    const int s = it % hg;
    const int ext = hg - 1 - s;
    const int lo_g = 1 - j0, hi_g = ny - 1 - j0;
    *lo = std::max(-ext, lo_g);
    *hi = std::min(nyl + ext, hi_g);
    *exchange = (s == hg - 1 || it == iters - 1) ? 1 : 0;
}

// Temporally blocked form: the block of sweeps starting at `it` runs
// *T = min(t_max, sweeps left before the next exchange, sweeps left in the
// solve) sweeps in one launch and stores its final sweep on local rows
// [out_lo, out_hi) (= what plan_sweep gives for the block's last sweep);
// *exchange as in plan_sweep.  hg <= 0 means unsharded (no exchanges): then
// the solve's ceil(iters / t_max) launches share its sweeps evenly.
inline void plan_block(int j0, int nyl, int ny, int hg, int it, int t_max, int iters, int *T,
                       int *out_lo, int *out_hi, int *exchange) {
    const int lo_g = 1 - j0, hi_g = ny - 1 - j0;
    if (hg <= 0) {
        // the same number of launches as t_max-sized blocks, the sweeps
        // spread evenly over them (50 = 8 + 6 x 7, not 6 x 8 + 2): a short
        // tail launch costs a whole pass over p' and rhs for few sweeps
        const int rem = iters - it, t = std::max(1, t_max);
        const int nl = (rem + t - 1) / t;
        *T = nl > 0 ? (rem + nl - 1) / nl : 0;
        *out_lo = lo_g;
        *out_hi = hi_g;
        *exchange = 0;
        return;
    }
    const int s = it % hg;
    *T = std::min(std::min(t_max, hg - s), iters - it);
    int ex;
    plan_sweep(j0, nyl, ny, hg, it + *T - 1, iters, out_lo, out_hi, &ex);
    *exchange = ex;
}

// Overlapped exchange block (SURVEY.md §8(e) overlap plan): the block that
// ends with a p' exchange is split into the bands the exchange sends — rows
// [0, hg) to rank-1 and [nyl-hg, nyl) to rank+1, computed first, then
// exchanged while the rest runs — and the interior rows.  Ghost rows of the
// block's range [lo, hi) are not computed: the exchange replaces them.
// out6 = {band_lo[0], band_hi[0], band_lo[1], band_hi[1], in_lo, in_hi}, an
// empty band (lo == hi) where there is no neighbour; returns 0 when the slab
// is too thin to split (then the block runs whole, exchange after it).
inline int plan_overlap(int nyl, int hg, int rank, int n_ranks, int lo, int hi, int out6[6]) {
    const bool below = rank > 0, above = rank < n_ranks - 1;
    out6[0] = 0;
    out6[1] = below ? hg : 0;
    out6[2] = above ? nyl - hg : nyl;
    out6[3] = nyl;
    out6[4] = below ? hg : lo;
    out6[5] = above ? nyl - hg : hi;
    return out6[5] > out6[4] ? 1 : 0;
}

// Halo geometry for one field, in local rows:
//   out[0..2] = {send_start, recv_start, rows} with the rank below (rank-1)
//   out[3..5] = {send_start, recv_start, rows} with the rank above (rank+1)
// rows = 0 where there is no neighbour.
//   kind 0 = u (pressure rows, G = 2 ghosts each side)
//   kind 1 = v (face rows; row nyl is the face shared with the rank above and
//            is computed by both ranks, so only rows beyond it travel)
//   kind 2 = p' (pressure rows, depth `depth`)
enum { HALO_U = 0, HALO_V = 1, HALO_PP = 2 };
inline void plan_halo(int kind, int nyl, int depth, int rank, int n_ranks, int out[6]) {
    int below[3] = {0, 0, 0}, above[3] = {0, 0, 0};
    if (kind == HALO_U) {
        below[0] = 0; below[1] = -2; below[2] = 2;
        above[0] = nyl - 2; above[1] = nyl; above[2] = 2;
    } else if (kind == HALO_V) {
        below[0] = 1; below[1] = -2; below[2] = 2;
        above[0] = nyl - 2; above[1] = nyl + 1; above[2] = 2;
    } else {
        below[0] = 0; below[1] = -depth; below[2] = depth;
        above[0] = nyl - depth; above[1] = nyl; above[2] = depth;
    }
    if (rank == 0) below[2] = 0;
    if (rank == n_ranks - 1) above[2] = 0;
    for (int k = 0; k < 3; ++k) {
        out[k] = below[k];
        out[3 + k] = above[k];
    }
}

}  // namespace cfd
