// cfd_jacobi_lds.hip — kind 5 (cfd_jacobi_lds.h) for T = 1..4, and the
// dispatch over T (launch_lds, cfd_internal.h).
#include "cfd_jacobi_lds.h"

namespace cfd {

void launch_lds(const Geom &g, const Fields &f, int T, int pass, int it, int par, int out_lo,
                int out_hi, uint32_t *rs, hipStream_t s, int mode, int lag) {
    switch (T) {
    case 1: launch_lds_T<1>(g, f, pass, par, it, out_lo, out_hi, rs, mode, s, lag); break;
    case 2: launch_lds_T<2>(g, f, pass, par, it, out_lo, out_hi, rs, mode, s, lag); break;
    case 3: launch_lds_T<3>(g, f, pass, par, it, out_lo, out_hi, rs, mode, s, lag); break;
    case 4: launch_lds_T<4>(g, f, pass, par, it, out_lo, out_hi, rs, mode, s, lag); break;
    case 5:
    case 6:
    case 7: launch_lds_t567(g, f, T, pass, par, it, out_lo, out_hi, rs, mode, s, lag); break;
    default: launch_lds_t8(g, f, pass, par, it, out_lo, out_hi, rs, mode, s, lag); break;
    }
}

}  // namespace cfd
