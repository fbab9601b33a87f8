// k_v5.hip -- the v5 integer-adder model on the matrix core (gemm_v5mx.h) and its B pre-pass, in
// their own translation unit.  Launcher: fp8approx_launch.h.
#define FP8A_OWN_V5 1
#include "fp8approx_launch.h"
#include "gemm_f8mx.h"
#include "gemm_v5mx.h"

namespace fp8a {

void launch_v5mx(const GemmArgs &a, hipStream_t s) {
    const dim3 gv((unsigned)(((a.M + V5_BMT - 1) / V5_BMT) * ((a.N + V5_BNT - 1) / V5_BNT) * a.splits));
    const bool uf = a.flags & F_UF, of = a.flags & F_OF;
    if (uf && of) gemm_v5mx_kernel<true, true><<<gv, 256, 0, s>>>(a);
    else if (uf) gemm_v5mx_kernel<true, false><<<gv, 256, 0, s>>>(a);
    else if (of) gemm_v5mx_kernel<false, true><<<gv, 256, 0, s>>>(a);
    else gemm_v5mx_kernel<false, false><<<gv, 256, 0, s>>>(a);
}

}  // namespace fp8a
