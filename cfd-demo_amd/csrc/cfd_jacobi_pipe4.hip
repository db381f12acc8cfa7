// cfd_jacobi_pipe4.hip — kind 3: the pipelined Jacobi march, 4 columns per lane.
#include "cfd_jacobi_pipe.h"

namespace cfd {
void launch_pipe4(const Geom &g, const Fields &f, int T, int pass, int it, int par, int out_lo,
                  int out_hi, uint32_t *rs, hipStream_t s) {
    launch_pipe<4>(g, f, T, pass, it, par, out_lo, out_hi, rs, s);
}
}  // namespace cfd
