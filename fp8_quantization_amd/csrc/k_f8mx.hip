// k_f8mx.hip -- gemm_f8mx_kernel (gemm_f8mx.h), one translation unit per result-grid form XF
// (-DFP8A_XF_PART=0 / 1 / 2, compiled in parallel by build_native.py); part 0 also holds the
// operand pre-passes xm_decode_a / xm_decode_b.  Launchers: fp8approx_launch.h.
#ifndef FP8A_XF_PART
#error "k_f8mx.hip is compiled once per part: -DFP8A_XF_PART=0..2"
#endif
#define FP8A_OWN_F8MX 1
#define FP8A_OWN_F8MX_DECODE (FP8A_XF_PART == 0)
#include "fp8approx_launch.h"
#include "gemm_f8mx.h"

namespace fp8a {

template <int NCG, int RB, int XF>
static void launch_shape(const GemmArgs &a, hipStream_t s) {
    using Cf = XmCfg<NCG, RB>;
    const int64_t xt = ((a.M + Cf::BMT - 1) / Cf::BMT) * ((a.N + Cf::BNT - 1) / Cf::BNT);
    const dim3 g((unsigned)(xt * a.splits));
    // (the emitting instances only where this launch writes the next convolution's word image
    // from its own store: unsplit, fp8a_conv2d_chain)
    const bool emit = a.em.w != nullptr && a.splits == 1;
    if (a.af32) {
        if (emit) gemm_f8mx_kernel<NCG, RB, true, XF, true><<<g, Cf::NT, 0, s>>>(a);
        else gemm_f8mx_kernel<NCG, RB, true, XF, false><<<g, Cf::NT, 0, s>>>(a);
    } else {
        if (emit) gemm_f8mx_kernel<NCG, RB, false, XF, true><<<g, Cf::NT, 0, s>>>(a);
        else gemm_f8mx_kernel<NCG, RB, false, XF, false><<<g, Cf::NT, 0, s>>>(a);
    }
}

template <int XF>
static void launch_xf(const GemmArgs &a, hipStream_t s) {
    if (a.xncg == 1) {
        launch_shape<1, 4, XF>(a, s);
    } else if constexpr (XF == 2) {
        launch_shape<2, 4, XF>(a, s);  // (the halved-block form: at most 32 columns, gemm_f8mx.h)
    } else {
        if (a.xncg == 2) launch_shape<2, 4, XF>(a, s);
        else launch_shape<4, 8, XF>(a, s);
    }
}

static int clock_read(unsigned long long *v, bool reset) {
    if (hipMemcpyFromSymbol(v, HIP_SYMBOL(g_clk), 3 * sizeof(unsigned long long)) != hipSuccess) return -1;
    if (reset) {
        const unsigned long long z[3] = {0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_clk), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}

#if FP8A_XF_PART == 0
void launch_f8mx_xf0(const GemmArgs &a, hipStream_t s) { launch_xf<0>(a, s); }
int f8mx_clock_xf0(unsigned long long *v, bool reset) { return clock_read(v, reset); }
#elif FP8A_XF_PART == 1
void launch_f8mx_xf1(const GemmArgs &a, hipStream_t s) { launch_xf<1>(a, s); }
int f8mx_clock_xf1(unsigned long long *v, bool reset) { return clock_read(v, reset); }
#else
void launch_f8mx_xf2(const GemmArgs &a, hipStream_t s) { launch_xf<2>(a, s); }
int f8mx_clock_xf2(unsigned long long *v, bool reset) { return clock_read(v, reset); }
#endif

}  // namespace fp8a
