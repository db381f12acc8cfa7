// cfd_jacobi_lds8.hip — kind 5 (cfd_jacobi_lds.h) for T = 8, the default
// launch of the solve, and the wave-timeline readback of stamp builds.
#include "cfd_jacobi_lds.h"

namespace cfd {

void launch_lds_t8(const Geom &g, const Fields &f, int pass, int par, int out_lo, int out_hi,
                   uint32_t *rs, int mode, hipStream_t s) {
    launch_lds_T<8>(g, f, pass, par, out_lo, out_hi, rs, mode, s);
}

bool launch_lds_persist8(const Geom &g, const Fields &f, int pass, int par0, int nblk, int out_lo,
                         int out_hi, uint32_t epoch, uint32_t *rs, hipStream_t s) {
    return launch_lds_persist_t<8>(g, f, pass, par0, nblk, out_lo, out_hi, epoch, rs, s);
}

#if CFD_LDS_STAMP
extern "C" int cfd_diag_lds_stamps(unsigned long long *host, int nwaves) {
    if (nwaves > kStampWaves) nwaves = kStampWaves;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_lds_stamp), (size_t)nwaves * 32, 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? nwaves : -1;
}
#endif

}  // namespace cfd
