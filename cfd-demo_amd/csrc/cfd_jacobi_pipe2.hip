// cfd_jacobi_pipe2.hip — kind 4: the pipelined Jacobi march, 2 columns per lane
// (half the registers of kind 3 per wave, twice the waves per row segment).
#include "cfd_jacobi_pipe.h"

namespace cfd {
void launch_pipe2(const Geom &g, const Fields &f, int T, int pass, int it, int par, int out_lo,
                  int out_hi, uint32_t *rs, hipStream_t s) {
    launch_pipe<2>(g, f, T, pass, it, par, out_lo, out_hi, rs, s);
}
}  // namespace cfd
