// fp8approx_launch.h -- launchers of the GEMM kernel families that live in their own translation
// units (build_native.py compiles them in parallel and links one libfp8approx.so).  A template
// kernel is instantiated and launched only inside its own unit; the host dispatch in
// fp8approx.hip calls these functions.  Non-template kernels of those units (xm_decode_a,
// xm_decode_b, tt_decode_b, v5mx_decode_b) are declared by their headers and launched directly.
#pragma once
#include "fp8approx_common.h"

namespace fp8a {

// k_fast.hip, part P = 2 * S2N + QBMA: gemm_fast_kernel<S2N, QBMA, gclip, mode> for the table
// modes TM_NONE .. TM_LUT; part 0 also runs TM_QAMAA and TM_V5 (no s2n / qbma / golden-clip
// variants), part 3 the E4M3 TM_F8 form (s2n + qbma, no golden clip).
void launch_fast_p0(int mode, bool gclip, const GemmArgs &a, dim3 grid, hipStream_t s);
void launch_fast_p1(int mode, bool gclip, const GemmArgs &a, dim3 grid, hipStream_t s);
void launch_fast_p2(int mode, bool gclip, const GemmArgs &a, dim3 grid, hipStream_t s);
void launch_fast_p3(int mode, bool gclip, const GemmArgs &a, dim3 grid, hipStream_t s);

// k_f8mx.hip, one part per result-grid form XF of gemm_f8mx_kernel (0 = E4M3, 1 = E5M2 plain,
// 2 = E5M2 halved-block); the tile shape is a.xncg, the A staging a.af32, the word-image emission
// a.em.w (unsplit launches only).
void launch_f8mx_xf0(const GemmArgs &a, hipStream_t s);
void launch_f8mx_xf1(const GemmArgs &a, hipStream_t s);
void launch_f8mx_xf2(const GemmArgs &a, hipStream_t s);
// The in-kernel clock sums of a -DFP8A_CLOCK_STAMP=1 build (memtime, realtime, workgroups), per part.
int f8mx_clock_xf0(unsigned long long *v, bool reset);
int f8mx_clock_xf1(unsigned long long *v, bool reset);
int f8mx_clock_xf2(unsigned long long *v, bool reset);

// k_tt.hip: the tile-table kernels on pre-decoded operands (a.wfmt 1: gemm_tt_kernel, 2:
// gemm_tt16_kernel + the gated f32 rerun); grid = gemm_fast_kernel's 64 x 64 tile grid.
void launch_tt(const GemmArgs &a, dim3 grid, hipStream_t s);
// launches rerun in gemm_tt_kernel's f32 form (fp8a_fallback_stats [2])
int tt_rerun_stats(unsigned long long *v, bool reset);

// k_v5.hip: the v5 matrix-core form (a.wfmt 4), per OF / UF switch pair.
void launch_v5mx(const GemmArgs &a, hipStream_t s);

}  // namespace fp8a
