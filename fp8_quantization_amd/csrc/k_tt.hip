// k_tt.hip -- the E3M4 / E2M5 tile-table kernels (gemm_tt.h, gemm_tt16.h) and their B pre-pass,
// in their own translation unit.  Launchers: fp8approx_launch.h.
#define FP8A_OWN_TT 1
#include "fp8approx_launch.h"
#include "gemm_f8mx.h"
#include "gemm_tt.h"
#include "gemm_tt16.h"

namespace fp8a {

void launch_tt(const GemmArgs &a, dim3 grid, hipStream_t s) {
    if (a.wfmt == 2) {  // E3M4: the packed-f16 tile-table kernel (run_gemm)
        const int bm = a.ttf7 ? Tt16Cfg<true>::BMR : Tt16Cfg<false>::BMR;
        const dim3 g16((unsigned)(((a.M + bm - 1) / bm) * ((a.N + BN - 1) / BN) * a.splits));
        a.ttf7 ? gemm_tt16_kernel<true><<<g16, NT, 0, s>>>(a) : gemm_tt16_kernel<false><<<g16, NT, 0, s>>>(a);
        // gated: reruns the launch in the f32 form when a tile left the f16 window (flag bits 1-4)
        a.ttf7 ? gemm_tt_kernel<4, true, true><<<grid, NT, 0, s>>>(a) : gemm_tt_kernel<4, false, true><<<grid, NT, 0, s>>>(a);
        return;
    }
    if (a.Mw == 4) {  // the tile-table kernel on pre-decoded operands
        a.ttf7 ? gemm_tt_kernel<4, true, false><<<grid, NT, 0, s>>>(a) : gemm_tt_kernel<4, false, false><<<grid, NT, 0, s>>>(a);
    } else {  // 128-row tiles on 8-wave workgroups
        static_assert(tt_rh<5>() == 2 && tt_rh<4>() == 1, "gemm_tt_kernel launch shapes");
        const dim3 g5((unsigned)(((a.M + 127) / 128) * ((a.N + BN - 1) / BN) * a.splits));
        gemm_tt_kernel<5, false, false><<<g5, 2 * NT, 0, s>>>(a);
    }
}

int tt_rerun_stats(unsigned long long *v, bool reset) {
    if (hipMemcpyFromSymbol(v, HIP_SYMBOL(g_tt_reruns), sizeof(unsigned long long)) != hipSuccess) return -1;
    if (reset) {
        const unsigned long long z = 0;
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_tt_reruns), &z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}

}  // namespace fp8a
