// k_fast.hip -- gemm_fast_kernel (gemm_fast.h), one translation unit per part P = 2 * S2N + QBMA
// (build_native.py compiles it four times with -DFP8A_FAST_PART=P, in parallel).  Launchers:
// fp8approx_launch.h.
#define FP8A_OWN_FAST 1
#include "fp8approx_launch.h"
#include "gemm_f8mx.h"
#include "gemm_fast.h"

#ifndef FP8A_FAST_PART
#error "k_fast.hip is compiled once per part: -DFP8A_FAST_PART=0..3"
#endif

namespace fp8a {

template <bool S2N, bool QBMA, bool GCLIP>
static void launch_table_modes(int mode, const GemmArgs &a, dim3 grid, hipStream_t s) {
    switch (mode) {
        case TM_NONE: gemm_fast_kernel<S2N, QBMA, GCLIP, TM_NONE><<<grid, NT, 0, s>>>(a); break;
        case TM_W1U: gemm_fast_kernel<S2N, QBMA, GCLIP, TM_W1U><<<grid, NT, 0, s>>>(a); break;
        case TM_W2S1: gemm_fast_kernel<S2N, QBMA, GCLIP, TM_W2S1><<<grid, NT, 0, s>>>(a); break;
        case TM_W2U1: gemm_fast_kernel<S2N, QBMA, GCLIP, TM_W2U1><<<grid, NT, 0, s>>>(a); break;
        case TM_W2S2: gemm_fast_kernel<S2N, QBMA, GCLIP, TM_W2S2><<<grid, NT, 0, s>>>(a); break;
        case TM_W2U2: gemm_fast_kernel<S2N, QBMA, GCLIP, TM_W2U2><<<grid, NT, 0, s>>>(a); break;
        default: gemm_fast_kernel<S2N, QBMA, GCLIP, TM_LUT><<<grid, NT, 0, s>>>(a); break;
    }
}

#if FP8A_FAST_PART == 0
void launch_fast_p0(int mode, bool gclip, const GemmArgs &a, dim3 grid, hipStream_t s) {
    if (mode == TM_QAMAA) gemm_fast_kernel<false, false, false, TM_QAMAA><<<grid, NT, 0, s>>>(a);
    else if (mode == TM_V5) gemm_fast_kernel<false, false, false, TM_V5><<<grid, NT, 0, s>>>(a);
    else if (gclip) launch_table_modes<false, false, true>(mode, a, grid, s);
    else launch_table_modes<false, false, false>(mode, a, grid, s);
}
#elif FP8A_FAST_PART == 1
void launch_fast_p1(int mode, bool gclip, const GemmArgs &a, dim3 grid, hipStream_t s) {
    if (gclip) launch_table_modes<false, true, true>(mode, a, grid, s);
    else launch_table_modes<false, true, false>(mode, a, grid, s);
}
#elif FP8A_FAST_PART == 2
void launch_fast_p2(int mode, bool gclip, const GemmArgs &a, dim3 grid, hipStream_t s) {
    if (gclip) launch_table_modes<true, false, true>(mode, a, grid, s);
    else launch_table_modes<true, false, false>(mode, a, grid, s);
}
#else
void launch_fast_p3(int mode, bool gclip, const GemmArgs &a, dim3 grid, hipStream_t s) {
    if (mode == TM_F8) gemm_fast_kernel<true, true, false, TM_F8><<<grid, NT, 0, s>>>(a);
    else if (gclip) launch_table_modes<true, true, true>(mode, a, grid, s);
    else launch_table_modes<true, true, false>(mode, a, grid, s);
}
#endif

}  // namespace fp8a
