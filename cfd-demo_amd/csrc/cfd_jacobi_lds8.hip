// cfd_jacobi_lds8.hip — kind 5 (cfd_jacobi_lds.h) for T = 8, the default
// launch of the solve, and the wave-timeline readback of stamp builds.
#include "cfd_jacobi_lds.h"

namespace cfd {

void launch_lds_t8(const Geom &g, const Fields &f, int pass, int par, int it, int out_lo, int out_hi,
                   uint32_t *rs, int mode, hipStream_t s, int lag) {
    launch_lds_T<8>(g, f, pass, par, it, out_lo, out_hi, rs, mode, s, lag);
}

bool launch_lds_persist8(const Geom &g, const Fields &f, int pass, int par0, int nblk, int out_lo,
                         int out_hi, uint32_t epoch, uint32_t *rs, hipStream_t s) {
    return launch_lds_persist_t<8>(g, f, pass, par0, nblk, out_lo, out_hi, epoch, rs, s);
}

void lds_geometry8(const Geom &g, int out_lo, int out_hi, bool persist, int *pad, int *occ, int *nwc,
                   int *nseg) {
    constexpr int T = 8;
    const int nc = cdiv(g.nx / 2, LdsMarch<T, 1, 0>::OUTL);
    const int pd = lds_pad_bytes(g, 0);
    int o = 0;
    if (persist)
        o = g.fastdiv == 1 ? persist_blocks_per_cu<T, 1>(pd)
            : g.fastdiv == 2 ? persist_blocks_per_cu<T, 2>(pd) : persist_blocks_per_cu<T, 0>(pd);
    else
        o = g.fastdiv == 1 ? lds_blocks_per_cu<T, 1, 0>(pd)
            : g.fastdiv == 2 ? lds_blocks_per_cu<T, 2, 0>(pd) : lds_blocks_per_cu<T, 0, 0>(pd);
    const int nrows = out_hi - out_lo;
    const int ns = g.fastdiv == 1   ? lds_segments<T, 1, 0>(g, nrows, nc, pd, persist ? o : 0)
                   : g.fastdiv == 2 ? lds_segments<T, 2, 0>(g, nrows, nc, pd, persist ? o : 0)
                                    : lds_segments<T, 0, 0>(g, nrows, nc, pd, persist ? o : 0);
    if (pad) *pad = pd;
    if (occ) *occ = o;
    if (nwc) *nwc = nc;
    if (nseg) *nseg = ns;
}

#if CFD_LDS_STAMP
extern "C" int cfd_diag_lds_stamps(unsigned long long *host, int nwaves) {
    if (nwaves > kStampWaves) nwaves = kStampWaves;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_lds_stamp), (size_t)nwaves * 32, 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? nwaves : -1;
}
#endif

}  // namespace cfd
