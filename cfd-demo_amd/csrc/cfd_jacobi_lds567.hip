// cfd_jacobi_lds567.hip — kind 5 (cfd_jacobi_lds.h) for T = 5..7.
#include "cfd_jacobi_lds.h"

namespace cfd {

void launch_lds_t567(const Geom &g, const Fields &f, int T, int pass, int par, int it, int out_lo,
                     int out_hi, uint32_t *rs, int mode, hipStream_t s, int lag) {
    if (T == 5)
        launch_lds_T<5>(g, f, pass, par, it, out_lo, out_hi, rs, mode, s, lag);
    else if (T == 6)
        launch_lds_T<6>(g, f, pass, par, it, out_lo, out_hi, rs, mode, s, lag);
    else
        launch_lds_T<7>(g, f, pass, par, it, out_lo, out_hi, rs, mode, s, lag);
}

}  // namespace cfd
