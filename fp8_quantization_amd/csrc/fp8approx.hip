// fp8approx.hip -- the C-ABI (include/fp8approx.h) of the MI355X (gfx950) approx-FP8 matmul/conv
// engine: argument checks, table packing, workspace layout, the host dispatch of the GEMM paths
// (run_gemm), the convolution / linear entry points, and the small kernels (split-K reduce, gated
// exact kernel, tensor-bias depthwise forms, fake quantizer, pooling, the exact product of
// gemm_dense.h).  The approx GEMM kernel families are compiled in their own units (k_*.hip,
// fp8approx_launch.h).  Hot path: approx_v9 (revollllt/FP8_quantization,
// approx/approx_matmul_whole_v9.py:10-169); DESIGN.md has the derivations and the exactness argument.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/fp8approx.h"
#include "fp8approx_common.h"
#include "fp8approx_launch.h"
#include "gemm_f8mx.h"
#include "gemm_v5mx.h"
#include "gemm_tt.h"
#include "gemm_tt16.h"
#include "gemm_dense.h"
#include "conv_tbx.h"

// (defined with C linkage below; run_gemm launches it too)
extern "C" __global__ void fq_bias_kernel(fp8a::FqIn fq, float *bias_out, int32_t *ibias_out);

namespace fp8a {

// ------------------------------------------------------------------------- error handling
static thread_local std::string g_err;

static int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

static int hip_check(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(FP8A_EHIP, std::string(what) + ": " + hipGetErrorString(e));
    return FP8A_OK;
}

static int pack_table(const int32_t *table, int M, bool approx, TablePack &tp, int &mode) {
    memset(&tp, 0, sizeof(tp));
    mode = TM_NONE;
    if (!approx || table == nullptr) return FP8A_OK;
    const int n = 1 << M;
    if (n * n > 1024) return fail(FP8A_EFORMAT, "error table larger than 32x32 (mant_width > 5)");
    int lo = 0, hi = 0;
    for (int i = 0; i < n * n; ++i) {
        if (table[i] < -128 || table[i] > 127) return fail(FP8A_EINVAL, "error table entry out of int8 range");
        tp.raw[i] = (int8_t)table[i];
        lo = std::min(lo, table[i]);
        hi = std::max(hi, table[i]);
    }
    if (lo == 0 && hi == 0) return FP8A_OK;
    const int words2 = (n * 2 + 31) / 32;
    if (lo >= 0 && hi <= 1 && n <= 32) {
        mode = TM_W1U;
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j)
                if (table[i * n + j]) tp.rows[i][0] |= 1u << j;
    } else if (lo >= -2 && hi <= 1 && words2 <= 2) {
        mode = words2 == 1 ? TM_W2S1 : TM_W2S2;
    } else if (lo >= 0 && hi <= 3 && words2 <= 2) {
        mode = words2 == 1 ? TM_W2U1 : TM_W2U2;
    } else {
        mode = TM_LUT;
    }
    if (mode >= TM_W2S1 && mode <= TM_W2U2) {
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) {
                const uint32_t code = (uint32_t)table[i * n + j] & 3u;
                const int bit = j * 2;
                tp.rows[i][bit >> 5] |= code << (bit & 31);
            }
    }
    return FP8A_OK;
}

// Fallback statistics since load (or the last reset): [0] launches whose gated exact kernel
// ran, [1] 64 x 64 output units it recomputed, [2] launches rerun in gemm_tt_kernel's f32 form
// (gemm_tt16_kernel's f16 window left), [3] tensor-bias launches recomputed by
// conv_tb_direct_kernel.  Read with fp8a_fallback_stats (include/fp8approx.h).
__device__ unsigned long long g_fallback[4];

// Sums the split-K partials in split order (deterministic) and writes the output mapping.
// Partial layout: row-major [M][N] (rowmajor output) or [img][N][hw] (NCHW output).
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const GemmArgs p) {
    const int64_t MN = p.M * p.N;
    const float pb = post_bias(p);
    const EmitCtx ec = emit_ctx(p);
    uint32_t sehi = 0;
    const int S = p.splits;
    const bool vec = p.nchw ? ((p.hw & 3) == 0) : ((p.N & 3) == 0 && (p.ldc & 3) == 0);
    const bool aligned = ((((uintptr_t)p.C) & 15) == 0) && ((((uintptr_t)p.part) & 15) == 0) && ((MN & 3) == 0) &&
                         ((((uintptr_t)p.res) & 15) == 0);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    if (vec && aligned) {
        for (int64_t q4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q4 < MN / 4; q4 += stride) {
            const int64_t q = q4 * 4;
            float4 acc = *reinterpret_cast<const float4 *>(p.part + q);
            for (int sp = 1; sp < S; ++sp) {
                const float4 v = *reinterpret_cast<const float4 *>(p.part + sp * MN + q);
                acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
            }
            int64_t o;
            if (p.nchw) {
                const int64_t img = q / (p.N * p.hw), rem = q - img * p.N * p.hw, n = rem / p.hw, pix = rem - n * p.hw;
                o = (img * p.ctot + p.coff + n) * p.hw + pix;
                if (p.ep) {  // the 4 values share channel coff + n (hw % 4 == 0)
                    const int64_t ch = p.coff + n;
                    acc.x = epi(p.ep, p.ep_act, p.ep_lo, p.ep_hi, ch, acc.x);
                    acc.y = epi(p.ep, p.ep_act, p.ep_lo, p.ep_hi, ch, acc.y);
                    acc.z = epi(p.ep, p.ep_act, p.ep_lo, p.ep_hi, ch, acc.z);
                    acc.w = epi(p.ep, p.ep_act, p.ep_lo, p.ep_hi, ch, acc.w);
                }
            } else {
                const int64_t m = q / p.N, n = q - m * p.N;
                o = m * p.ldc + n;
                if (p.ep) {
                    acc.x = epi(p.ep, p.ep_act, p.ep_lo, p.ep_hi, p.coff + n, acc.x);
                    acc.y = epi(p.ep, p.ep_act, p.ep_lo, p.ep_hi, p.coff + n + 1, acc.y);
                    acc.z = epi(p.ep, p.ep_act, p.ep_lo, p.ep_hi, p.coff + n + 2, acc.z);
                    acc.w = epi(p.ep, p.ep_act, p.ep_lo, p.ep_hi, p.coff + n + 3, acc.w);
                }
            }
            const float4 r = post4(p, o, acc, pb);
            *reinterpret_cast<float4 *>(p.C + o) = r;
            if (p.em.w) emit4(p, ec, o, r, sehi);
        }
        if (p.em.w) wave_max_atomic(p.em.invalid + 5, sehi);
        return;
    }
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < MN; q += stride) {
        float acc = p.part[q];
        for (int sp = 1; sp < S; ++sp) acc += p.part[sp * MN + q];
        int64_t o, ch;
        if (p.nchw) {
            const int64_t img = q / (p.N * p.hw), rem = q - img * p.N * p.hw, n = rem / p.hw, pix = rem - n * p.hw;
            o = (img * p.ctot + p.coff + n) * p.hw + pix;
            ch = p.coff + n;
        } else {
            const int64_t m = q / p.N, n = q - m * p.N;
            o = m * p.ldc + n;
            ch = p.coff + n;
        }
        const float r = post1(p, o, epi(p.ep, p.ep_act, p.ep_lo, p.ep_hi, ch, acc), pb);
        p.C[o] = r;
        if (p.em.w) emit1(p, ec, o, r, sehi);
    }
    if (p.em.w) wave_max_atomic(p.em.invalid + 5, sehi);
}

// A(m, k) for the exact kernels: matrix or implicit im2col (through the fused input quantizer
// when there is one).
__device__ __forceinline__ float load_A(const GemmArgs &p, int64_t m, int64_t k) {
    if (!p.conv) {
        const float v = p.A[m * p.lda + k];
        if (p.fqin.mx == nullptr) return v;
        const float mx = *p.fqin.mx;
        return fq_apply(v, mx, fq_bias(mx, p.fqin.E, p.fqin.M), p.fqin.M, p.fqin.S);
    }
    const int64_t hw = p.Ho * p.Wo, img = m / hw, pix = m - img * hw;
    const int64_t ho = pix / p.Wo, wo = pix - ho * p.Wo;
    const int64_t taps = (int64_t)p.kh * p.kw, c = k / taps, t = k - c * taps, ky = t / p.kw, kx = t - ky * p.kw;
    const int64_t hi = ho * p.sh - p.ph + ky * p.dh, wi = wo * p.sw - p.pw + kx * p.dw;
    if (hi < 0 || hi >= p.H || wi < 0 || wi >= p.W) return 0.0f;
    const float v = p.X[((img * p.Cin + p.cbase + c) * p.H + hi) * p.W + wi];
    if (p.fqin.mx == nullptr) return v;
    const float mx = *p.fqin.mx;
    return fq_apply(v, mx, fq_bias(mx, p.fqin.E, p.fqin.M), p.fqin.M, p.fqin.S);
}

__device__ __forceinline__ void gemm_exact_units(const GemmArgs &p, uint32_t f, const DFmt &fA, const DFmt &fR, bool tb);

__global__ __launch_bounds__(256) void gemm_exact_kernel(const GemmArgs p) {
    const bool tb = p.flags & F_TB;
    if (p.post_bout != nullptr && blockIdx.x == 0 && threadIdx.x == 0) {  // the output quantizer's bias
        const float b = fq_bias(*p.post_fq.mx, p.post_fq.E, p.post_fq.M);
        *p.post_bout = b;
        *p.post_ibout = (int32_t)b;
    }
    const DFmt fA = dfmt(p.E, p.Mw, *p.bA, tb), fR = dfmt(p.E, p.Mw, *p.bR, tb);
    if (p.flag == nullptr) {  // the tensor-bias path: the exact kernel is the product itself
        for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < p.M * p.N;
             idx += (int64_t)gridDim.x * blockDim.x) {
            const int64_t m = idx % p.M, n = idx / p.M;
            const DFmt fB = dfmt(p.E, p.Mw, p.bB[n * p.bBs], tb);
            float s = 0.0f, part = 0.0f;
            for (int64_t k = 0; k < p.K; ++k) {
                part += exact_term(load_A(p, m, k), p.B[k * p.sbk + n * p.sbn], fA, fB, fR, p.tab.raw, p.flags);
                if ((k & 15) == 15) {
                    s += part;
                    part = 0.0f;
                }
            }
            s += part;
            const int64_t o = out_index(p, m, n);
            const float r = post1(p, o, epi(p.ep, p.ep_act, p.ep_lo, p.ep_hi, p.coff + n, s), post_bias(p));
            p.C[o] = r;
            if (p.em.w) {
                uint32_t sh = 0;
                emit1(p, emit_ctx(p), o, r, sh);
                if (sh) atomicMax(p.em.invalid + 5, sh);
            }
        }
        return;
    }
    // Gated after a fast launch: nothing to do unless it flagged (uniform per grid; the grid is
    // capped, so the no-op case costs one small launch); then only the marked 64 x 64 units
    // (every unit with FB_ALL), one unit per block step: thread = (row, 16 columns).  The kernel
    // ends the launch: it reports the flag word to the caller (flag_out) and zeroes the flag
    // arena's other slot (arena_clear: the previous launch's words)
    arena_clear(p.arena_clr, p.arena_clr16);
    const uint32_t f = __hip_atomic_load(p.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (p.flag_out && blockIdx.x == 0 && threadIdx.x == 0) *p.flag_out = f;
    if (f & FB_ANY) gemm_exact_units(p, f, fA, fR, tb);
}

// The marked units of a flagged launch (gemm_exact_kernel); every thread returns here.
__device__ __forceinline__ void gemm_exact_units(const GemmArgs &p, uint32_t f, const DFmt &fA, const DFmt &fR, bool tb) {
    const bool all = (f & FB_ALL) != 0u || p.urow == nullptr;
    const int64_t nur = (p.M + 63) >> 6, nuc = (p.N + 63) >> 6;
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&g_fallback[0], 1ull);
    const float pb = post_bias(p);
    const EmitCtx ec = emit_ctx(p);
    for (int64_t u = blockIdx.x; u < nur * nuc; u += gridDim.x) {
        const int64_t ur = u / nuc, uc = u - ur * nuc;
        if (!all && !p.urow[ur] && !p.ucol[uc] && !(p.utile[u] & UT_EXACT)) continue;  // (block-uniform)
        if (threadIdx.x == 0) atomicAdd(&g_fallback[1], 1ull);
        const int64_t m = 64 * ur + (threadIdx.x & 63), nb = 64 * uc + 16 * (threadIdx.x >> 6);
        if (m >= p.M) continue;
        float s[16], part[16];
        DFmt fB[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            s[j] = part[j] = 0.0f;
            fB[j] = dfmt(p.E, p.Mw, p.bB[min(nb + j, p.N - 1) * p.bBs], tb);
        }
        for (int64_t k = 0; k < p.K; ++k) {
            const float a = load_A(p, m, k);
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int64_t n = min(nb + j, p.N - 1);
                part[j] += exact_term(a, p.B[k * p.sbk + n * p.sbn], fA, fB[j], fR, p.tab.raw, p.flags);
                if ((k & 15) == 15) {
                    s[j] += part[j];
                    part[j] = 0.0f;
                }
            }
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int64_t n = nb + j;
            if (n >= p.N) break;
            const int64_t o = out_index(p, m, n);
            const float r = post1(p, o, epi(p.ep, p.ep_act, p.ep_lo, p.ep_hi, p.coff + n, s[j] + part[j]), pb);
            p.C[o] = r;
            if (p.em.w) {
                uint32_t sh = 0;
                emit1(p, ec, o, r, sh);
                if (sh) atomicMax(p.em.invalid + 5, sh);
            }
        }
    }
}

__global__ __launch_bounds__(256) void terms_kernel(const GemmArgs p, float *T) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= p.M * p.K * p.N) return;
    const int64_t n = idx % p.N, k = (idx / p.N) % p.K, m = idx / (p.N * p.K);
    const bool tb = p.flags & F_TB;
    const DFmt fA = dfmt(p.E, p.Mw, *p.bA, tb), fR = dfmt(p.E, p.Mw, *p.bR, tb);
    const DFmt fB = dfmt(p.E, p.Mw, p.bB[n * p.bBs], tb);
    T[idx] = exact_term(p.A[m * p.lda + k], p.B[k * p.sbk + n * p.sbn], fA, fB, fR, p.tab.raw, p.flags);
}

__global__ __launch_bounds__(256) void decompose_kernel(const float *x, int64_t rows, int64_t cols, int64_t ld,
                                                        int E, int M, const int32_t *bias, int64_t bs,
                                                        uint32_t flags, int32_t *expo, int32_t *mant) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= rows * cols) return;
    const int64_t r = idx / cols, c = idx - r * cols;
    const DFmt f = dfmt(E, M, bias[r * bs], flags & F_TB);
    int e, m;
    exact_dec(x[r * ld + c], f, flags & F_GCLIP, e, m);
    expo[idx] = e;
    mant[idx] = m;
}

__global__ __launch_bounds__(256) void quant_kernel(const float *x, int64_t n, int E, int M, const int32_t *bias,
                                                    uint32_t flags, float *out) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n) return;
    const DFmt f = dfmt(E, M, *bias, flags & F_TB);
    out[idx] = exact_q(x[idx], f, flags & F_GCLIP);
}

// im2col, K ordered (c, ky, kx) like approx_calculation.py:738-745.
__global__ __launch_bounds__(256) void im2col_kernel(const float *x, float *out, int64_t Bn, int64_t C, int64_t H,
                                                     int64_t W, int kh, int kw, int sh, int sw, int ph, int pw,
                                                     int dh, int dw, int64_t Ho, int64_t Wo) {
    const int64_t K = C * kh * kw;
    const int64_t total = Bn * Ho * Wo * K;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = idx % K, m = idx / K;
        const int64_t kx = k % kw, ky = (k / kw) % kh, c = k / (kw * kh);
        const int64_t wo = m % Wo, ho = (m / Wo) % Ho, b = m / (Wo * Ho);
        const int64_t hi = ho * sh - ph + ky * dh, wi = wo * sw - pw + kx * dw;
        float v = 0.0f;
        if (hi >= 0 && hi < H && wi >= 0 && wi < W) v = x[((b * C + c) * H + hi) * W + wi];
        out[idx] = v;
    }
}

// Single-output-channel groups (depthwise): tensor-bias semantics, direct from NCHW x.
// TB = false: the same literal restatement with int-bias semantics -- the v5 model's depthwise
// convolutions (v5 has no tensor-bias path: its products are the GEMM path's, with a zero
// operand's NONZERO term at every padded position, as the reference's im2col supplies them).
template <bool TB>
__global__ __launch_bounds__(256) void conv_tb_direct_kernel(const float *x, const float *w, float *y, int64_t Bn,
                                                             int64_t Cin, int64_t H, int64_t W, int64_t Cout,
                                                             int kh, int kw, int sh, int sw, int ph, int pw, int dh,
                                                             int dw, int groups, int64_t Ho, int64_t Wo, int E,
                                                             int Mw, const int32_t *bA, const int32_t *bW,
                                                             const int32_t *bR, TablePack tab, uint32_t flags,
                                                             const uint32_t *gate, uint32_t *gate_out, uint4 *clr,
                                                             uint32_t clr16, const float2 *ep, int ep_act,
                                                             float ep_lo, float ep_hi, FqIn fq) {
    // after conv_tb_fast_kernel: run only if it flagged inputs outside its exactness window.  The
    // gate word is a slot of the stream's flag arena (flag_arena): this kernel reports it to the
    // caller's workspace word (gate_out) and zeroes the arena's other slot (arena_clear)
    arena_clear(clr, clr16);
    const uint32_t gv = gate != nullptr ? __hip_atomic_load(gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 1u;
    if (gate_out != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *gate_out = gv;
    if (gv == 0u) return;
    if (gate != nullptr && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&g_fallback[3], 1ull);
    const int64_t total = Bn * Cout * Ho * Wo;
    const int64_t cpg = Cin / groups;   // input channels per group
    const DFmt fA = dfmt(E, Mw, *bA, TB), fR = dfmt(E, Mw, *bR, TB);
    const float fmx = fq.mx ? *fq.mx : 0.0f, fbias = fq.mx ? fq_bias(fmx, fq.E, fq.M) : 0.0f;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t wo = idx % Wo, ho = (idx / Wo) % Ho, co = (idx / (Wo * Ho)) % Cout, b = idx / (Wo * Ho * Cout);
        const int64_t g = co / (Cout / groups);
        const DFmt fB = dfmt(E, Mw, bW[co], TB);
        float s = 0.0f, part = 0.0f;
        int cnt = 0;
        for (int64_t c = 0; c < cpg; ++c)
            for (int ky = 0; ky < kh; ++ky)
                for (int kx = 0; kx < kw; ++kx) {
                    const int64_t hi = ho * sh - ph + ky * dh, wi = wo * sw - pw + kx * dw;
                    float a = (hi >= 0 && hi < H && wi >= 0 && wi < W)
                                  ? x[((b * Cin + g * cpg + c) * H + hi) * W + wi] : 0.0f;
                    if (fq.mx) a = fq_apply(a, fmx, fbias, fq.M, fq.S);
                    const float bv = w[((co * cpg + c) * kh + ky) * kw + kx];
                    part += exact_term(a, bv, fA, fB, fR, tab.raw, TB ? (flags | F_TB) : flags);
                    if (++cnt == 16) {
                        s += part;
                        part = 0.0f;
                        cnt = 0;
                    }
                }
        y[idx] = epi(ep, ep_act, ep_lo, ep_hi, co, s + part);
    }
}

// Single-output-channel groups (depthwise) with the tensor-bias semantics, fast form.
// With int32-tensor biases >= 2 the reference's param_prepare yields min_norm = 0 (quirk F5):
// no operand or result is subnormal, every nonzero value decodes at its own binade.  For
// exactly representable operands (M-bit mantissa at their binade, |x| in [2^-62, 2^50]) and
// with_s2nn2s_opt on, golden_clip_OF off, the term is then
//   v0 = a*b - T[mA][mB] * cA * cB * 2^-M                         (exact, as in the GEMM)
//   sign quirk F7: Q_R(g) is 0 only in the binade 2^-bR (expo 0, mantissa rounding to 0), where
//                  a negative g gives the term |v0|
//   Q_R, tb form: round at the value's own binade with the F6 clamp, except in the binade
//                  [2^-bR, 2^(1-bR)) (expo field 0), whose decode is 2^(1-bR) * m / 2^M, i.e.
//                  2 * (Q(x) - sign * 2^-bR)
// Anything else sets the gate word and conv_tb_direct_kernel recomputes the launch exactly.
// One thread per output pixel; grid (pixel chunks, Cout, Bn); the channel's decoded weights and
// the error table live in LDS.
constexpr int TBF_MAXK = 512;

__global__ __launch_bounds__(256) void conv_tb_fast_kernel(const float *x, const float *w, float *y, int64_t Cin,
                                                           int64_t H, int64_t W, int64_t Cout, int kh, int kw,
                                                           int sh, int sw, int ph, int pw, int dh, int dw, int groups,
                                                           int64_t Ho, int64_t Wo, int Mw, const int32_t *bA,
                                                           const int32_t *bW, const int32_t *bR, TablePack tab,
                                                           uint32_t flags, uint32_t *gate, const float2 *ep,
                                                           int ep_act, float ep_lo, float ep_hi) {
    __shared__ float sw_v[TBF_MAXK], sw_c[TBF_MAXK];
    __shared__ int32_t sw_m[TBF_MAXK];
    __shared__ float sT[1024];
    const int64_t co = blockIdx.y, img = blockIdx.z;
    const int64_t cpg = Cin / groups, g = co / (Cout / groups);
    const int K = (int)(cpg * kh * kw), M = Mw, n = 1 << M;
    const int a_b = *bA, r_b = *bR, w_b = bW[co];
    const bool approx = flags & F_APPROX, qbma = flags & F_QBMA;
    bool bad = !(a_b >= 2 && w_b >= 2 && r_b >= 2 && a_b <= 120 && w_b <= 120 && r_b <= 120 && K <= TBF_MAXK);
    const uint32_t offgrid = (1u << (23 - M)) - 1u;
    for (int i = threadIdx.x; i < n * n; i += blockDim.x) sT[i] = approx ? (float)tab.raw[i] : 0.0f;
    for (int k = threadIdx.x; k < K && k < TBF_MAXK; k += blockDim.x) {
        const float v = w[co * K + k];
        const uint32_t ua = __float_as_uint(v) & 0x7FFFFFFFu;
        bad |= (ua != 0u) && ((ua & offgrid) != 0u || ua < 0x20800000u || ua > 0x58800000u);
        sw_v[k] = v;
        sw_c[k] = __uint_as_float(__float_as_uint(v) & 0xFF800000u) * p2(-M);  // cB * 2^-M (0 for zeros)
        sw_m[k] = (int32_t)((ua >> (23 - M)) & (uint32_t)(n - 1));
    }
    __syncthreads();
    // Q_R constants (tb form: no subnormal floor)
    const float kb = 2.0f - p2(-M) - p2(-22), kc = 1.5f * p2(23 - M);
    const uint32_t q0exp = (uint32_t)(127 - r_b) << 23;             // exponent field of 2^-bR
    const float zlo = p2(-r_b), zhi = p2(-r_b) * (1.0f + p2(-M - 1));  // |g| where Q_R(g) == 0
    const int64_t pix = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = pix < Ho * Wo;
    const int64_t ho = live ? pix / Wo : 0, wo = live ? pix - ho * Wo : 0;
    float acc = 0.0f;
    int k = 0;
    for (int64_t c = 0; c < cpg; ++c) {
        const float *xc = x + ((img * Cin + g * cpg + c) * H) * W;
        for (int ky = 0; ky < kh; ++ky) {
            const int64_t hi = ho * sh - ph + (int64_t)ky * dh;
            for (int kx = 0; kx < kw; ++kx, ++k) {
                const int64_t wi = wo * sw - pw + (int64_t)kx * dw;
                const float a = (live && hi >= 0 && hi < H && wi >= 0 && wi < W) ? xc[hi * W + wi] : 0.0f;
                const uint32_t ua = __float_as_uint(a) & 0x7FFFFFFFu;
                bad |= (ua != 0u) && ((ua & offgrid) != 0u || ua < 0x20800000u || ua > 0x58800000u);
                const float cA = __uint_as_float(__float_as_uint(a) & 0xFF800000u);
                const int mA = (int)((ua >> (23 - M)) & (uint32_t)(n - 1));
                const float b = sw_v[k];
                const float gq = a * b;  // exact
                float v = __fmaf_rn(-sT[mA * n + sw_m[k]], cA * sw_c[k], gq);
                // F7: Q_R(g) == 0 (so the sign is +) only for |g| in [2^-bR, 2^-bR (1 + 2^-(M+1))]
                const float ag = fabsf(gq);
                if (gq < 0.0f && ag >= zlo && ag <= zhi) v = fabsf(v);
                if (qbma) {
                    const uint32_t pb = __float_as_uint(v) & 0x7F800000u;
                    const float pe = __uint_as_float(pb);
                    const float bd = pe * kb;
                    const float xs = __builtin_amdgcn_fmed3f(v, -bd, bd);
                    const float cc = pe * kc;
                    float r = (xs + cc) - cc;
                    if (pb == q0exp) r = 2.0f * (r - copysignf(pe, v));  // expo field 0: 2^(1-bR) m / 2^M
                    v = r;
                }
                acc += v;
            }
        }
    }
    const bool anybad = __syncthreads_or(bad ? 1 : 0);
    if (anybad) {
        if (threadIdx.x == 0) atomicOr(gate, 1u);
        return;
    }
    if (live) y[((img * Cout + co) * Ho + ho) * Wo + wo] = epi(ep, ep_act, ep_lo, ep_hi, co, acc);
}


// FP8 fake quantizer (fp8_quantizer.py:97-173), one sign bit.
__global__ __launch_bounds__(256) void fp8_quantize_kernel(const float *x, int64_t rows, int64_t inner,
                                                           const float *maxval, int per_row, int E, int M,
                                                           int sign_bits, float *out, float *bias_out,
                                                           int32_t *ibias_out) {
    const int64_t total = rows * inner;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = per_row ? idx / inner : 0;
        const float mx = maxval[r];
        const float bias = fq_bias(mx, E, M);
        out[idx] = fq_apply(x[idx], mx, bias, M, sign_bits);
        if ((idx % inner) == 0) {
            if (bias_out) bias_out[r] = bias;
            if (ibias_out) ibias_out[r] = (int32_t)bias;
        }
    }
}

// nn.MaxPool2d (dilation 1, floor mode) on NCHW fp32: the stem pooling between the first conv
// and layer1 of the ResNets (torchvision layout), one thread per output, NaN-propagating like
// ATen's max_pool2d.  Not an approx op: it sits on the benchmarked step (torch's kernel took
// 0.59 ms of a 38 ms ResNet-18 batch-256 step).
__global__ __launch_bounds__(256) void max_pool2d_kernel(const float *x, float *y, int64_t planes, int H, int W,
                                                         int Ho, int Wo, int kh, int kw, int sh, int sw, int ph,
                                                         int pw) {
    const int64_t total = planes * Ho * Wo;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int wo = (int)(idx % Wo);
        const int64_t t = idx / Wo;
        const int ho = (int)(t % Ho);
        const int64_t pl = t / Ho;
        const float *xp = x + pl * H * W;
        float m = -INFINITY;
        const int h0 = ho * sh - ph, w0 = wo * sw - pw;
        for (int ky = 0; ky < kh; ++ky) {
            const int hi = h0 + ky;
            if ((unsigned)hi >= (unsigned)H) continue;
            for (int kx = 0; kx < kw; ++kx) {
                const int wi = w0 + kx;
                if ((unsigned)wi >= (unsigned)W) continue;
                const float v = xp[(int64_t)hi * W + wi];
                m = (v > m || v != v) ? v : m;
            }
        }
        y[idx] = m;
    }
}

// The ResNet stem configuration (3x3 window, stride 2, padding 1) on rows of W % 8 == 0: each
// thread makes 4 consecutive outputs of one row from two aligned float4 loads + one scalar per
// input row (27 scalar loads before), one float4 store.  Same scan order (window row, then
// column) and NaN rule as max_pool2d_kernel, so the same bits.
// nn.AvgPool2d with one output per plane (fp8a_avg_pool2d_plane; MobileNetV2's head).  ATen's
// avg_pool2d sums the window in row-major order in fp32 and divides by kh kw once; so does this
// (the same bits).  ATen reads with one thread per plane (lanes a plane apart: 0.41 ms for the
// head at batch 512); here a workgroup stages PB consecutive planes through LDS with contiguous
// loads (plane stride padded odd: conflict-free per-thread sums), then thread = plane.
__global__ __launch_bounds__(128) void avg_pool_plane_kernel(const float *x, float *y, int64_t planes, int PB, int W,
                                                             int hw, int ps, int kh, int kw, float inv_hw) {
    extern __shared__ float ap_sm[];
    const int tid = threadIdx.x;
    const int64_t P0 = (int64_t)blockIdx.x * PB;
    const int npl = (int)min((int64_t)PB, planes - P0), n = npl * hw;
    const float *xb = x + P0 * hw;
    for (int d0 = tid; d0 < n; d0 += 4 * 128) {
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = d0 + 128 * u < n ? xb[d0 + 128 * u] : 0.0f;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int d = d0 + 128 * u;
            if (d < n) {
                const int pl = dw_div(d, hw, inv_hw);
                ap_sm[pl * ps + d - pl * hw] = v[u];
            }
        }
    }
    __syncthreads();
    for (int t = tid; t < npl; t += 128) {
        const float *s = ap_sm + t * ps;
        float acc = 0.0f;
        for (int r = 0; r < kh; ++r)
            for (int c = 0; c < kw; ++c) acc += s[r * W + c];
        y[P0 + t] = acc / (float)(kh * kw);
    }
}

__global__ __launch_bounds__(256) void max_pool2d_s2k3_kernel(const float *x, float *y, int64_t planes, int H, int W,
                                                             int Ho) {
    const int Wq = W / 8;  // 4-output groups per output row (Wo = W / 2)
    const int64_t total = planes * Ho * Wq;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int q = (int)(idx % Wq);
        const int64_t t = idx / Wq;
        const int ho = (int)(t % Ho);
        const int64_t pl = t / Ho;
        const float *xp = x + pl * H * W;
        float m[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
        const int c0 = 8 * q;  // input columns c0 - 1 .. c0 + 7
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
            const int hi = 2 * ho - 1 + ky;
            if ((unsigned)hi >= (unsigned)H) continue;
            const float *r = xp + (int64_t)hi * W + c0;
            const float4 a = *reinterpret_cast<const float4 *>(r), b = *reinterpret_cast<const float4 *>(r + 4);
            const float v[9] = {c0 > 0 ? r[-1] : -INFINITY, a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
            for (int o = 0; o < 4; ++o)
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) {
                    if (o == 0 && kx == 0 && c0 == 0) continue;  // left padding
                    const float u = v[2 * o + kx];
                    m[o] = (u > m[o] || u != u) ? u : m[o];
                }
        }
        *reinterpret_cast<float4 *>(y + (pl * Ho + ho) * (int64_t)(W / 2) + 4 * q) = make_float4(m[0], m[1], m[2], m[3]);
    }
}

// ------------------------------------------------------------------------- host dispatch
// The GEMM kernel families are instantiated and launched in their own translation units
// (fp8approx_launch.h): gemm_fast_kernel in k_fast.hip, gemm_f8mx_kernel in k_f8mx.hip, the
// tile-table kernels in k_tt.hip, the v5 form in k_v5.hip.
// E4M3 (XF 0) or E5M2 (mant_width 2) result grid; E5M2 launches both its kernels, the plain one
// (XF 1) over every tile and the halved-block one (XF 2), which recomputes only the tiles the plain
// one marked UT_HALF (the top binade, gemm_f8mx.h) and exits at once without FB_HALF
static void launch_f8mx(const GemmArgs &a, hipStream_t s) {
    if (a.Mw == 2) {
        launch_f8mx_xf1(a, s);
        launch_f8mx_xf2(a, s);
    } else {
        launch_f8mx_xf0(a, s);
    }
}

// gemm_f8mx_kernel's tile width: the fewest padded columns, ties to the wider tile (N = 16 -> 16,
// 24 / 32 / 96 / 160 -> 32, multiples of 64 -> 64).  Option "xm_ncg" / FP8A_XM_NCG=<1|2|4> forces it
// (0 = this choice; A/B runs and identity tests).
static int g_opt_xm_ncg = getenv("FP8A_XM_NCG") ? atoi(getenv("FP8A_XM_NCG")) : 0;  // option "xm_ncg"
static int xm_ncg(int64_t N) {
    const int forced = g_opt_xm_ncg;
    if (forced == 1 || forced == 2 || forced == 4) return forced;
    int best = 4;
    int64_t bp = (N + 63) / 64 * 64;
    for (int c : {2, 1}) {
        const int64_t pad = (N + 16 * c - 1) / (16 * c) * (16 * c);
        if (pad < bp) {
            bp = pad;
            best = c;
        }
    }
    return best;
}

static void launch_fast(int mode, const GemmArgs &a, hipStream_t s) {
    const int64_t tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
    const dim3 grid((unsigned)(tiles * a.splits));
    if (mode == TM_V5) {  // the v5 model has no s2n / qbma / golden-clip variants
        if (a.aw && a.wfmt == 4) launch_v5mx(a, s);  // the matrix-core form (gemm_v5mx.h)
        else launch_fast_p0(TM_V5, false, a, grid, s);
        return;
    }
    if (mode == TM_QAMAA) {
        launch_fast_p0(TM_QAMAA, false, a, grid, s);
        return;
    }
    if (a.aw && (a.wfmt == 1 || a.wfmt == 2)) {  // E3M4 / E2M5: the tile-table kernels (run_gemm)
        launch_tt(a, grid, s);
        return;
    }
    if (mode == TM_F8) {  // s2n + qbma, no golden clip (selected in run_gemm)
        // matrix-core accumulation on pre-decoded operands (gemm_f8mx.h) when run_gemm staged
        // them, else the VALU-accumulating form
        if (a.aw || a.af32) launch_f8mx(a, s);
        else launch_fast_p3(TM_F8, false, a, grid, s);
        return;
    }
    const bool s2n = a.flags & F_S2N, q = a.flags & F_QBMA, gc = a.flags & F_GCLIP;
    if (s2n) q ? launch_fast_p3(mode, gc, a, grid, s) : launch_fast_p2(mode, gc, a, grid, s);
    else q ? launch_fast_p1(mode, gc, a, grid, s) : launch_fast_p0(mode, gc, a, grid, s);
}

static int check_format(int E, int Mw) {
    if (E < 1 || Mw < 1 || Mw > 5 || E > 6 || E + Mw > 8)
        return fail(FP8A_EFORMAT, "Invalid combination of expo_width and mant_width");
    return FP8A_OK;
}

constexpr size_t FLAG_BYTES = 256;  // workspace prefix holding the off-grid flag word

// Launch paths taken by run_gemm since load (fp8a_path_stats): host-side counters.
enum { PATH_F8MX = 0, PATH_TT = 1, PATH_TT16 = 2, PATH_FAST = 3, PATH_EXACT = 4, PATH_DENSE = 5, PATH_V5MX = 6,
       PATH_N = 7 };
static std::atomic<uint64_t> g_paths[PATH_N];

// Kernel timing (fp8a_kernel_timing / fp8a_kernel_time): while on, run_gemm brackets the product
// kernel launch(es) of every GEMM (launch_fast: gemm_f8mx_kernel, gemm_tt*_kernel, gemm_v5mx_kernel
// or gemm_fast_kernel -- not the operand pre-passes, split-K reduce or gated exact kernel) with HIP
// events on the launching stream, so a benchmark can report the dominant kernel's own time next to
// the op's.  Host-side, single-threaded use (benchmarks); events come from a pool.
struct KernelEv {
    hipEvent_t a, b;
    int path, dispatches;
    double macs;
};
static bool g_ktime = false;
static std::vector<KernelEv> g_kev;
static std::vector<hipEvent_t> g_evpool;
static hipEvent_t pool_event() {
    if (!g_evpool.empty()) {
        hipEvent_t e = g_evpool.back();
        g_evpool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return e;
}
// Options (fp8a_set_option):
// "tbx_rw": output rows per thread of conv_tbx_kernel (1 or 2; 2 needs undilated rows).
// FP8A_TBX_RW=<n> sets it at load.
static int g_opt_tbx_rw = getenv("FP8A_TBX_RW") ? atoi(getenv("FP8A_TBX_RW")) : 2;
// "tbs": the table-form depthwise 3x3 on the LDS-DMA-staged conv_tbsg_kernel (2, default:
// MobileNetV2 E4M3 21.7k -> 22.8k, config 3 v9 19.6k -> 20.5k images/s), the register-staged
// conv_tbs_kernel (1), both with the word pre-pass fused, or on tbx_decode_a + conv_tbx_kernel (0);
// the same bits.  FP8A_TBS=<n>.
static int g_opt_tbs = getenv("FP8A_TBS") ? atoi(getenv("FP8A_TBS")) : 2;
// "dw3": the exact depthwise 3x3 on the LDS-DMA-staged, 4-outputs-per-thread dn_dw3g_kernel (2,
// default: config 1 26.1k -> 28.3k images/s), the register-staged dn_dw3_kernel (1) or the general
// dn_group_conv (0); the same bits.  FP8A_DW3=<n> sets it at load.
static int g_opt_dw3 = getenv("FP8A_DW3") ? atoi(getenv("FP8A_DW3")) : 2;
// "dn_direct": exact convolutions with K <= 32 and N <= 64 on dn_direct_kernel (1, default) or on
// the bf16 matrix-core GEMM (0).  FP8A_DN_DIRECT=<n> sets it at load.
static int g_opt_dn_direct = getenv("FP8A_DN_DIRECT") ? atoi(getenv("FP8A_DN_DIRECT")) : 1;
// "v5ds": the v5 depthwise 3 x 3 on the staged conv_v5ds_kernel (1, default) or on the word
// pre-passes + conv_v5dw_kernel (0); the same bits.  FP8A_V5DS=<n> sets it at load.
static int g_opt_v5ds = getenv("FP8A_V5DS") ? atoi(getenv("FP8A_V5DS")) : 1;
// "dw_target": outputs per workgroup the LDS-staged depthwise kernels aim at (plan_dw3 / plan_tbs;
// halved until the window fits dw_lds).  FP8A_DW_TARGET=<n>.
static int g_opt_dw_target = getenv("FP8A_DW_TARGET") ? atoi(getenv("FP8A_DW_TARGET")) : 4096;
// "dw_lds": the LDS bytes per workgroup those plans allow (FP8A_DW_LDS=<n>, at most 64 KB).
static int g_opt_dw_lds = getenv("FP8A_DW_LDS") ? atoi(getenv("FP8A_DW_LDS")) : 40960;

// Compute units of the current device (cached); 256 (MI355X) when no device is visible.
static int device_cus() {
    static int cache[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
        (void)hipGetLastError();
        return 256;
    }
    if (cache[dev] == 0) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) {
            (void)hipGetLastError();
            cus = 256;
        }
        cache[dev] = cus;
    }
    return cache[dev];
}

// Split-K factor for a fast launch, from a time model fitted on MI355X (ResNet-18 layers,
// FP8A_SPLITK = 1..6 sweeps).  The fast kernel holds 4 workgroups per CU (128 VGPRs), so a launch
// runs in rounds of 4*CUs tiles, each round lasting one tile's time (BM*BN*K products at about
// 4.4 G products/s per workgroup slot); a last, partly filled round costs min(1, 0.4 + 1.1*fill)
// of a full one (a half-filled round costs a full one, a 6 %-filled one 0.45).  Splitting K
// multiplies the tile count and divides the round length, and adds a pass that writes and
// re-reads S*M*N partial floats (charged at 2 TB/s).  Each split keeps at least 16 K-tiles.
// FP8A_SPLITK=<S> forces S (experiments).
static int choose_splits(int64_t M, int64_t N, int64_t K) {
    static int forced = -1;
    if (forced < 0) {
        const char *e = getenv("FP8A_SPLITK");
        forced = e ? std::max(0, atoi(e)) : 0;
    }
    const int64_t kt = (K + BK - 1) / BK;
    if (forced > 0) return (int)std::max<int64_t>(1, std::min<int64_t>(forced, kt));
    const int64_t tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    const double slots = 4.0 * device_cus();
    static double rate = 0.0;  // approx-MAC/s of one 64x64 workgroup at 4 per CU (FP8A_SPLITK_RATE overrides)
    if (rate == 0.0) {
        const char *e = getenv("FP8A_SPLITK_RATE");
        rate = e ? std::max(1e8, atof(e)) : 4.4e9;
    }
    const double t_round = (double)BM * BN * K / rate;                      // s
    const double t_split = 2.0 * (double)M * N * sizeof(float) / 2.0e12;   // s per split
    double best = 1e300;
    int bs = 1;
    for (int S = 1; S <= 8; ++S) {
        if (S > 1 && kt < 16 * S) break;
        const double q = (double)tiles * S / slots, fl = std::floor(q), fr = q - fl;
        const double rounds = fl + (fr > 1e-9 ? std::min(1.0, 0.4 + 1.1 * fr) : 0.0);
        const double t = rounds / S * t_round + (S > 1 ? S * t_split : 0.0);
        if (t < best * (1.0 - 1e-3)) {
            best = t;
            bs = S;
        }
    }
    return bs;
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Bytes of the pre-decoded operands of the matrix-core E4M3 kernel (gemm_f8mx.h): A words
// (a_words of them) + B column pairs [Kpad][Npad / 2] of 8 bytes.
// The B image: the E4M3 / E5M2 column pairs ([kpad][npad / 2] uint2) or the v5 form's four table
// words per column ([kpad][npad] uint2, gemm_v5mx.h) -- sized for the larger.
static size_t xm_b_bytes(int64_t kpad, int64_t npad) { return align256((size_t)(kpad * npad) * 8); }
static size_t xm_operand_bytes(int64_t N, int64_t K, int64_t a_words) {
    const int64_t kpad = (K + BK - 1) / BK * BK, npad = (N + BN - 1) / BN * BN;
    // + table image + the E5M2 B exponent ranges
    return align256((size_t)a_words * 4) + xm_b_bytes(kpad, npad) + 16384 + align256((size_t)(kpad * npad / 16) * 2);
}

// The per-unit fallback marks after the flag word: urow [nur], ucol [nuc], utile [nur * nuc] bytes.
static size_t unit_bytes(int64_t M, int64_t N) {
    const int64_t nur = (M + 63) / 64, nuc = (N + 63) / 64;
    return align256((size_t)(nur + nuc + nur * nuc));
}
static size_t head_bytes(int64_t M, int64_t N) { return FLAG_BYTES + unit_bytes(M, N); }

static size_t splitk_bytes(int64_t M, int64_t N, int64_t K) {
    const int S = choose_splits(M, N, K);
    return S > 1 ? align256((size_t)S * (size_t)M * (size_t)N * sizeof(float)) : 0;
}


// flag word + unit marks + split-K partials + the matrix-core kernels' pre-decoded operands
// (gemm_f8mx.h).  conv_words: the conv word image's element count, 0 for a matrix A.
static size_t gemm_workspace_bytes(int64_t M, int64_t N, int64_t K, int64_t conv_words) {
    const int64_t a_words = conv_words > 0 ? conv_words : M * ((K + BK - 1) / BK * BK);
    return head_bytes(M, N) + splitk_bytes(M, N, K) + xm_operand_bytes(N, K, a_words);
}

// The table + hardware-fp8 form applies (TM_F8; run_gemm then takes the matrix-core kernel when
// the workspace holds its pre-decoded operands): E4M3 (e4m3 conversion) or E5M2 (bf8 conversion,
// round 4), a {0,1} or zero table, s2n + qbma, no golden clip, int-bias semantics, not v5.
// (E5M2 has no VALU TM_F8 form: without the pre-decoded operands it keeps its table mode.)
// FP8A_NO_F8=1 keeps the arithmetic forms; FP8A_NO_F8_E5M2=1 only for E5M2 (A/B runs).
static bool f8_form(int E, int Mw, uint32_t flags, int table_mode) {
    static const bool no_f8 = getenv("FP8A_NO_F8") != nullptr;
    static const bool no_f8_e5 = getenv("FP8A_NO_F8_E5M2") != nullptr;
    const bool fmt = (E == 4 && Mw == 3) || (E == 5 && Mw == 2 && !no_f8_e5);
    return !no_f8 && !(flags & F_V5) && fmt && (table_mode == TM_NONE || table_mode == TM_W1U) &&
           (flags & F_S2N) && (flags & F_QBMA) && !(flags & F_GCLIP) && !(flags & F_TB);
}

// v5 (E5M2, adder wrap on): the matrix-core form of gemm_v5mx.h; FP8A_NO_V5MX=1 keeps
// gemm_fast_kernel<TM_V5> (A/B runs)
static bool v5mx_form(int Mw, uint32_t flags, int table_mode) {
    static const bool no_v5mx = getenv("FP8A_NO_V5MX") != nullptr;
    return table_mode == TM_V5 && Mw == 2 && (flags & F_OFUF) && !no_v5mx;
}

// The tile-table kernel (gemm_tt_kernel) applies: E3M4 / E2M5 (mantissa 4 or 5), any table mode
// of the int-bias path, s2n + qbma, no golden clip, not v5 (FP8A_NO_TT=1 keeps gemm_fast_kernel);
// not E2M5 with a signed table: its F7 form (two 32-row tables, one K-step per staged tile) was
// measured slower than gemm_fast_kernel.
static bool tt_form(int Mw, uint32_t flags, const TablePack &tab) {
    static const bool no_tt = getenv("FP8A_NO_TT") != nullptr;
    if (no_tt || (flags & F_V5) || !(Mw == 4 || Mw == 5) || !(flags & F_S2N) || !(flags & F_QBMA) ||
        (flags & F_GCLIP) || (flags & F_TB))
        return false;
    bool neg = false;
    for (int i = 0; i < (1 << (2 * Mw)); ++i) neg |= tab.raw[i] < 0;
    return Mw == 4 || !neg;
}

// E3M4 on the tile-table path runs the packed-f16 form (gemm_tt16_kernel) for signed tables (F7:
// +23 % on the ResNet-18 layer set) and for K >= 256 (+2-9 %); on short K its per-tile prologue
// (the frame shift's bias range, two barriers) outweighs the gain (MobileNetV2 E3M4 -3 %), and
// gemm_tt_kernel<4, F7> runs.  FP8A_NO_TT16=1 keeps gemm_tt_kernel everywhere.
// (option "tt16_mink": the smallest K of an unsigned-table launch on the f16 form; default 64 since
// round 5: ResNet-50 E3M4 2,045 -> 2,082 images/s with its K = 64 / 128 / 147 launches on the f16
// form, profiles/r05_tt16_mink/ -- round 3's tt16 lost 3 % there)
static int g_opt_tt16_mink = getenv("FP8A_TT16_MINK") ? std::max(0, atoi(getenv("FP8A_TT16_MINK"))) : 64;
// option "tt_band" (default 1; FP8A_TT_BAND): gemm_tt_kernel's band / zero wave-tile forms (gemm_tt.h)
static int g_opt_tt_band = getenv("FP8A_TT_BAND") ? atoi(getenv("FP8A_TT_BAND")) : 1;
static bool tt16_form(int Mw, bool f7, int64_t K) {
    static const bool no_tt16 = getenv("FP8A_NO_TT16") != nullptr;
    return !no_tt16 && Mw == 4 && (f7 || K >= g_opt_tt16_mink);
}

static bool no_mx() {
    static const bool v = getenv("FP8A_NO_MX") != nullptr;
    return v;
}

// The conv word image: every plane is the input plane inside a zero border at least as wide as
// the convolution's padding -- ph rows above and below; pw columns on the left, widened to 4 when
// W % 4 == 0 so that the interior rows start 16-B aligned, and the row length rounded up to a
// multiple of 4 (the pre-decode then moves the interior with 16-B loads and stores).
struct WordImage {
    int64_t H, W;    // image height / width (words)
    int ph, pw;      // top / left border
};
static WordImage word_image(int64_t H, int64_t W, int ph, int pw) {
    WordImage w;
    w.ph = ph;
    w.H = H + 2 * ph;
    if (pw > 0 && pw <= 4 && W % 4 == 0) {
        w.pw = 4;
        w.W = (W + 4 + pw + 3) / 4 * 4;
    } else {
        w.pw = pw;
        w.W = W + 2 * pw;
    }
    return w;
}

// Words of the pre-decoded A operand: conv, the group's word image [Bn][aw_c][awH][awW]; matrix,
// [M][Kpad].
static int64_t xm_a_words(const GemmArgs &a) {
    const int64_t kpad = (a.K + BK - 1) / BK * BK;
    if (!a.conv) return a.M * kpad;
    const WordImage w = word_image(a.H, a.W, a.ph, a.pw);
    return (a.M / (a.Ho * a.Wo)) * a.aw_c * w.H * w.W;
}

// gemm_f8mx_kernel reads A as fp32 and decodes it while staging (no xm_decode_a pass) for a 1x1
// unpadded conv or a matrix A whose source lies within 32-bit byte offsets, when the launch has at
// most FP8A_AF32_MAXCT column tiles (default 1; 0 = never): each column tile decodes its A
// elements again (~25 VALU operations each), against the pre-pass's 8 B of HBM traffic per element.
// Round 2 measured at most 0 / 2 / 4 tiles 4610 / 4613 / 4543 images/s on ResNet-50 E4M3 and chose
// 3; with round 5's pre-pass (4 loads in flight per thread) at most 1 tile wins everywhere:
// MobileNetV2 E4M3 23,877 -> 24,482, E5M2 v9 21,225 -> 21,561, ResNet-50 E4M3 4,790 -> 4,840
// (profiles/r05_af32/).
static int g_opt_af32_maxct = getenv("FP8A_AF32_MAXCT") ? std::max(0, atoi(getenv("FP8A_AF32_MAXCT"))) : 1;
// (a strided 1x1 conv's pre-pass decodes sh x sw input pixels per one the product reads, so the
// fp32 staging is allowed up to sh x sw times as many column tiles: ResNet-18's downsampling convs)
static int64_t af32_maxct(int sh, int sw) { return (int64_t)g_opt_af32_maxct * sh * sw; }
static bool xm_af32(const GemmArgs &a) {
    const int64_t bnt = 16 * a.xncg, ct = (a.N + bnt - 1) / bnt;
    if (ct > (a.conv ? af32_maxct(a.sh, a.sw) : g_opt_af32_maxct)) return false;  // option "af32_maxct"
    if (a.conv) {
        if (a.kh != 1 || a.kw != 1 || a.ph != 0 || a.pw != 0) return false;
        const int64_t bn = a.M / (a.Ho * a.Wo);
        return bn * a.Cin * a.H * a.W * 4 < (1ll << 32);
    }
    return a.A != nullptr && a.M * a.lda * 4 < (1ll << 32) && a.lda >= a.K;
}

// The fallback-flag arena of a (device, stream): two slots, used by the launches on the stream in
// turn, each holding one launch's flag word, the pre-passes' extremes and its per-unit marks.  A
// launch finds its slot zero; its last kernel (the gated exact / literal kernel) zeroes the other
// slot's words, which the previous launch used (arena_clear) -- so launches need no fill, and the
// clearing races nothing.  Zeroed once when (re)allocated; grows by reallocation after the stream
// drains.  A launch that stops before its last kernel (a launch error) leaves its successor a slot
// with stale words: that launch then reruns the marked units exactly -- the same bits, more time.
//
// Stream capture (a HIP graph being recorded on s): the arena's host-side rotation would be frozen
// into the graph -- a forward with an odd number of launches would start every replay after the
// first on a slot its own last launch left dirty, and the clear sizes would be those of capture
// time.  So a captured launch never touches the arena: its words live in the head of the caller's
// workspace (which the caller allocates per call; torch's allocator gives a graph its own pool),
// zeroed by a fill kernel at the start of the launch (dev_fill: not a memset node), and it clears nothing.  Every replay then
// starts from zero words whatever ran before it, eager launches keep their own rotation, and an
// eager launch that grows the arena afterwards cannot touch memory a graph references.  Growth never
// frees an arena (retired ones stay allocated: at most the size of the current one in total), so
// it needs no stream synchronisation either.
struct FlagArena {
    uint32_t *p = nullptr;
    size_t slot = 0;       // bytes per slot
    int cur = 0;           // the slot the next launch uses
    size_t dirty[2] = {0, 0};
};
struct ArenaLease {
    uint32_t *mine = nullptr;  // this launch's slot (zero)
    uint4 *clr = nullptr;      // the other slot, and its 16-byte words the last kernel zeroes
    uint32_t clr16 = 0;
};
// Is a graph being captured on s?  (-1: the query itself failed; the error is recorded)
// In-stream fills as kernels of our own, not hipMemsetAsync / hipMemset2DAsync: under stream capture
// a memset becomes a graph memset node, and on this ROCm such nodes did not refill their destination
// on replays after the first (measured: tools/dbg_capture2.py, DESIGN.md §3r -- a captured launch's
// flag words then held stale data).  A kernel node re-executes every replay like any other.
__global__ __launch_bounds__(256) void fill_u8_kernel(uint8_t *p, size_t n, uint32_t v8) {
    const uint32_t w = v8 * 0x01010101u;
    const size_t lead = std::min(n, (size_t)((16 - ((uintptr_t)p & 15)) & 15)), n16 = (n - lead) / 16;
    const size_t t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (size_t)gridDim.x * blockDim.x;
    uint4 *q = reinterpret_cast<uint4 *>(p + lead);
    for (size_t i = t0; i < n16; i += nt) q[i] = make_uint4(w, w, w, w);
    for (size_t i = t0; i < lead; i += nt) p[i] = (uint8_t)v8;  // (bytes before the first 16-B boundary)
    for (size_t i = lead + 16 * n16 + t0; i < n; i += nt) p[i] = (uint8_t)v8;  // (and after the last)
}
__global__ __launch_bounds__(256) void fill_rows_kernel(float *p, int64_t ld, int64_t w, int64_t h) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < w * h; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / w;
        p[r * ld + (i - r * w)] = 0.0f;
    }
}
static hipError_t dev_fill(void *p, int v, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    fill_u8_kernel<<<(unsigned)std::max<size_t>(1, std::min<size_t>((n / 16 + 255) / 256, 1024)), 256, 0, s>>>(
        (uint8_t *)p, n, (uint32_t)(v & 0xFF));
    return hipGetLastError();
}
static hipError_t dev_zero_rows(float *p, int64_t ld, int64_t w, int64_t h, hipStream_t s) {
    if (w <= 0 || h <= 0) return hipSuccess;
    fill_rows_kernel<<<(unsigned)std::min<int64_t>((w * h + 255) / 256, 8192), 256, 0, s>>>(p, ld, w, h);
    return hipGetLastError();
}
static int stream_capturing(hipStream_t s) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) != hipSuccess) return -1;
    static const bool dbg = getenv("FP8A_DEBUG_CAPTURE") != nullptr;  // diagnostics: the query per lease
    if (dbg) fprintf(stderr, "fp8a lease stream=%p capturing=%d\n", (void *)s, (int)st);
    return st == hipStreamCaptureStatusActive ? 1 : 0;
}
// The lease of a captured launch: `need` bytes at the head of its workspace, zeroed in-stream.
static bool capture_lease(hipStream_t s, void *ws, size_t ws_bytes, size_t need, ArenaLease &l) {
    if (ws == nullptr || ws_bytes < need) return false;
    static const bool dbg = getenv("FP8A_DEBUG_CAPTURE") != nullptr;
    if (dbg) fprintf(stderr, "fp8a capture lease ws=%p need=%zu ws_bytes=%zu\n", ws, need, ws_bytes);
    if (dev_fill(ws, 0, need, s) != hipSuccess) return false;
    l.mine = (uint32_t *)ws;
    l.clr = nullptr;
    l.clr16 = 0;
    return true;
}
static std::mutex g_arena_mu;
static std::map<std::pair<int, uintptr_t>, FlagArena> g_arenas;
static bool flag_arena(hipStream_t s, size_t need, ArenaLease &l) {
    static std::vector<void *> retired;  // grown-out-of arenas: never freed (in-flight launches may use them)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    need = (need + 255) & ~(size_t)255;
    std::lock_guard<std::mutex> lock(g_arena_mu);
    FlagArena &ar = g_arenas[{dev, (uintptr_t)s}];
    if (ar.slot < need) {
        const size_t slot = std::max(need, std::max(2 * ar.slot, (size_t)65536));
        void *p = nullptr;
        if (hipMalloc(&p, 2 * slot) != hipSuccess) return false;
        if (dev_fill(p, 0, 2 * slot, s) != hipSuccess) {
            (void)hipFree(p);
            return false;
        }
        if (ar.p) retired.push_back(ar.p);
        ar = FlagArena{};
        ar.p = (uint32_t *)p;
        ar.slot = slot;
    }
    const int other = 1 - ar.cur;
    l.mine = ar.p + (size_t)ar.cur * (ar.slot / 4);
    l.clr = reinterpret_cast<uint4 *>(ar.p + (size_t)other * (ar.slot / 4));
    l.clr16 = (uint32_t)(ar.dirty[other] / 16);
    ar.dirty[other] = 0;
    ar.dirty[ar.cur] = need;
    ar.cur = other;
    return true;
}
// A depthwise launch's gate word: the workspace head under capture, else an arena slot.
static bool dw_lease(hipStream_t s, void *ws, size_t ws_bytes, ArenaLease &l) {
    const int cap = stream_capturing(s);
    if (cap < 0) return false;
    return cap ? capture_lease(s, ws, ws_bytes, FLAG_BYTES, l) : flag_arena(s, FLAG_BYTES, l);
}
static int lease_error() {
    const int rc = hip_check("fp8a flag arena");
    return rc ? rc : fail(FP8A_EHIP, "fp8a flag arena: no room for the flag words (under stream capture they need "
                                     "the workspace head)");
}
// grid blocks of 256 threads that clear a lease's other slot in about four 16-byte stores each
static unsigned clear_blocks(const ArenaLease &l) { return (l.clr16 + 1023) / 1024; }

// Fast tiled kernel + gated exact kernel (int-bias path), or the exact kernel alone (tb path).
static int run_qamaa(GemmArgs &a, hipStream_t s);

static int run_gemm(GemmArgs &a, const int32_t *table, void *ws, size_t ws_bytes, hipStream_t s) {
    if (a.qmax) return run_qamaa(a, s);
    int rc = check_format(a.E, a.Mw);
    if (rc) return rc;
    if (a.M < 0 || a.N < 0 || a.K < 0) return fail(FP8A_EINVAL, "negative extent");
    if (a.post_bout && (a.M == 0 || a.N == 0 || a.K == 0)) {  // (no exact kernel below to write it)
        fq_bias_kernel<<<1, 1, 0, s>>>(a.post_fq, a.post_bout, a.post_ibout);
        const int rc0 = hip_check("fp8a output-quantizer bias");
        if (rc0) return rc0;
    }
    if (a.M == 0 || a.N == 0) return FP8A_OK;
    if (a.K == 0) {  // empty inner dimension: the reference's sum over an empty axis is 0
        if (a.nchw) return fail(FP8A_EINVAL, "empty convolution window");
        if (dev_zero_rows(a.C, a.ldc, a.N, a.M, s) != hipSuccess)
            return hip_check("fp8a zero fill");
        return FP8A_OK;
    }
    if ((!a.A && !a.conv) || (a.conv && !a.X) || !a.B || !a.C || !a.bA || !a.bB || !a.bR)
        return fail(FP8A_EINVAL, "null pointer");
    int mode;
    const bool v5 = a.flags & F_V5;
    if (v5 && (a.flags & F_TB)) return fail(FP8A_EINVAL, "the v5 model has no tensor-bias semantics");
    rc = pack_table(table, a.Mw, v5 || (a.flags & F_APPROX), a.tab, mode);
    if (rc) return rc;
    if (v5) mode = TM_V5;
    const int mode0 = mode;
    // E4M3 / E5M2 with a {0,1} (or no) table, s2n and per-product quantization: the LUT + hardware
    // fp8 / bf8 form (FP8A_NO_F8=1 keeps the arithmetic form, for comparison)
    if (f8_form(a.E, a.Mw, a.flags, mode)) mode = TM_F8;
    const int64_t total = a.M * a.N;
    const unsigned eblocks = (unsigned)std::min<int64_t>((total + 255) / 256, 4096);
    if (a.flags & F_TB) {
        a.flag = nullptr;
        ++g_paths[PATH_EXACT];
        gemm_exact_kernel<<<eblocks, 256, 0, s>>>(a);
        return hip_check("fp8a exact gemm launch");
    }
    if (ws == nullptr || ws_bytes < FLAG_BYTES) return fail(FP8A_EINVAL, "matmul workspace too small");
    // the flag word and the per-unit fallback marks live in the library's flag arena (zero on
    // entry, left zero by gemm_exact_kernel: no fill per launch); the workspace's first word
    // receives the final flag word, and its head stays reserved (the layout of the size queries)
    static const bool no_units = getenv("FP8A_NO_UNITS") != nullptr;  // diagnostics: whole-launch fallbacks
    const size_t head = ws_bytes >= head_bytes(a.M, a.N) ? head_bytes(a.M, a.N) : FLAG_BYTES;
    ArenaLease lease;
    const int cap = stream_capturing(s);  // (captured: the words live in the workspace head, flag_arena)
    if (cap < 0) return hip_check("fp8a stream capture query");
    if (cap ? !capture_lease(s, ws, ws_bytes, head, lease) : !flag_arena(s, head_bytes(a.M, a.N), lease))
        return lease_error();
    a.flag = lease.mine;
    a.flag_out = (uint32_t *)ws;
    a.arena_clr = lease.clr;
    a.arena_clr16 = lease.clr16;
    a.nur = (a.M + 63) / 64;
    a.nuc = (a.N + 63) / 64;
    a.urow = no_units || (cap && head < head_bytes(a.M, a.N)) ? nullptr : (uint8_t *)a.flag + FLAG_BYTES;
    a.ucol = no_units ? nullptr : a.urow + a.nur;
    a.utile = no_units ? nullptr : a.ucol + a.nuc;
    // split-K when the caller's workspace holds the partials (else one split)
    a.splits = choose_splits(a.M, a.N, a.K);
    if (a.splits > 1 && ws_bytes < head + splitk_bytes(a.M, a.N, a.K)) a.splits = 1;
    const int64_t kt = (a.K + BK - 1) / BK;
    a.kchunk = ((kt + a.splits - 1) / a.splits) * BK;
    a.part = a.splits > 1 ? (float *)((char *)ws + head) : nullptr;
    // the matrix-core E4M3 kernel and the tile-table kernel (E3M4 / E2M5) need their pre-decoded
    // operands in the workspace (else gemm_fast_kernel runs); FP8A_NO_MX=1 forces the latter
    a.aw = nullptr;
    const bool tt = mode != TM_F8 && tt_form(a.Mw, a.flags, a.tab);
    const bool v5mx = v5mx_form(a.Mw, a.flags, mode);
    if ((mode == TM_F8 || tt || v5mx) && !no_mx()) {
        const int64_t kpad = kt * BK, npad = (a.N + BN - 1) / BN * BN;
        const size_t off = head + (a.splits > 1 ? splitk_bytes(a.M, a.N, a.K) : 0);
        // gemm_f8mx_kernel reads its operands with 32-bit byte offsets
        const int64_t a_words = xm_a_words(a);
        const WordImage wi = word_image(a.H, a.W, a.ph, a.pw);
        a.awH = wi.H; a.awW = wi.W; a.awph = wi.ph; a.awpw = wi.pw;
        const bool fits32 = a_words < (1ll << 30) && kpad * npad * 4 < (1ll << 32);
        if (fits32 && ws_bytes >= off + xm_operand_bytes(a.N, a.K, a_words)) {
            char *base = (char *)ws + off;
            a.aw = (const uint32_t *)base;
            a.awld = kpad;
            a.bqw = (const uint2 *)(base + align256((size_t)a_words * 4));
            a.lutw = (const uint32_t *)(base + align256((size_t)a_words * 4) + xm_b_bytes(kpad, npad));
            a.ebr = (const uint16_t *)((const char *)a.lutw + 16384);
            a.xm_vmin = mode == TM_NONE ? 0 : -1;
            a.npad = npad;
            a.ttf7 = 0;
            for (int i = 0; tt && i < (1 << (2 * a.Mw)); ++i) a.ttf7 |= a.tab.raw[i] < 0;
            a.wfmt = v5mx ? 4 : tt ? (tt16_form(a.Mw, a.ttf7, a.K) ? 2 : 1) : 0;
            if (a.wfmt == 1 && !g_opt_tt_band) a.ebr = nullptr;  // (gemm_tt_kernel: no band test)
            a.xncg = tt ? 4 : xm_ncg(a.N);
            // the input's word image from the previous launch (fp8a_conv2d_chain): its words replace
            // the A pre-pass, which then runs gated (only to write the fused quantizer's bias, or to
            // re-decode x if the image arrived invalid)
            const bool use_img = a.in_img != nullptr && !tt && a.conv && a.fqin.mx != nullptr;
            if (use_img) a.aw = a.in_img + 64;
            a.af32 = !tt && !v5mx && !use_img && xm_af32(a) ? 1 : 0;
            const int64_t rows = a.conv ? a.M / (a.Ho * a.Wo) : a.M, cols = a_words / std::max<int64_t>(rows, 1);
            dim3 ga((unsigned)std::min<int64_t>((cols + 255) / 256, 64), (unsigned)std::min<int64_t>(rows, 1024));
            {  // the pre-pass's flattened 16-byte form (xm_decode_a: unbordered, rows and columns in
               // whole 16-byte chunks): a 1-D grid of about 4 chunks per thread
                const int64_t hw = a.H * a.W, lim0 = a.conv ? cols : a.K, istride = a.conv ? a.Cin * hw : a.lda;
                const float *in0 = a.conv ? a.X + a.cbase * hw : a.A;
                const bool flat = !(a.conv && (a.awph | a.awpw)) && lim0 % 4 == 0 && cols % 4 == 0 && istride % 4 == 0 &&
                                  ((uintptr_t)in0 & 15) == 0 && ((uintptr_t)a.aw & 15) == 0;
                if (flat) ga = dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((a_words / 4 + 1023) / 1024, 8192)), 1);
            }
            if (use_img) {
                a.gate = a.in_img;
                xm_decode_a<<<ga.y == 1 ? dim3(std::min(ga.x, 512u)) : dim3(std::min(ga.x, 8u), std::min(ga.y, 64u)), 256, 0,
                              s>>>(a);
                a.gate = nullptr;
            } else if (!a.af32) {
                xm_decode_a<<<ga, 256, 0, s>>>(a);
            }
            if (v5mx) {  // the four table words per (k, n), [Kpad][Npad]
                const unsigned gb = (unsigned)std::min<int64_t>((kpad * npad + 255) / 256, 4096);
                v5mx_decode_b<<<gb, 256, 0, s>>>(a, kpad);
            } else if (tt) {  // B words [Kpad][Npad] (the same bytes as the E4M3 pair grid) + the static image
                const unsigned gb = (unsigned)std::min<int64_t>((kpad * npad + 255) / 256, 4096);
                tt_decode_b<<<gb, 256, 0, s>>>(a, kpad);  // (+ gemm_tt16_kernel's f16 image when wfmt == 2)
            } else {
                const unsigned gb = (unsigned)std::min<int64_t>((kpad * npad / 2 + 255) / 256, 4096);
                xm_decode_b<<<gb, 256, 0, s>>>(a, kpad);
            }
            rc = hip_check("fp8a operand pre-decode launch");
            if (rc) return rc;
        }
    }
    if (a.fqin.mx && !a.aw)  // the caller (conv2d_impl) only fuses where the pre-decode runs
        return fail(FP8A_EINVAL, "internal: fused input quantization without the matrix-core path");
    if (mode == TM_F8 && a.Mw != 3 && !a.aw) mode = mode0;  // (gemm_fast_kernel's TM_F8 form is E4M3 only)
    ++g_paths[!a.aw ? PATH_FAST : a.wfmt == 0 ? PATH_F8MX : a.wfmt == 1 ? PATH_TT : a.wfmt == 4 ? PATH_V5MX : PATH_TT16];
    // word-image emission (fp8a_conv2d_chain): the E4M3 / E5M2 matrix-core kernel and the VALU
    // kernel emit the next convolution's words from their store; the tile-table and v5 matrix-core
    // kernels do not (store_tile<false>: the emission code cost gemm_tt16_kernel 32 SGPR spills and a
    // 38 % slower E3M4 layer set, round 4 -> 5), so their unsplit launch marks the image invalid
    // instead (emit_prep_kernel set the header valid before this launch) and the consumer's gated
    // pre-pass re-decodes its input from y (likewise under a GELU tail, which the emitting store
    // compiles out)
    if (a.em.w != nullptr && (a.em.form == 2 || (a.aw && a.wfmt != 0 && a.splits == 1) || a.post_act == 2)) {
        if (dev_fill(a.em.invalid, 1, sizeof(uint32_t), s) != hipSuccess) return hip_check("fp8a word image header");
        a.em.w = nullptr;
    }
    KernelEv kev{};
    if (g_ktime && !cap) {  // (no host-side events inside a captured graph)
        kev.a = pool_event();
        kev.b = pool_event();
        kev.path = !a.aw ? PATH_FAST : a.wfmt == 0 ? PATH_F8MX : a.wfmt == 1 ? PATH_TT : a.wfmt == 4 ? PATH_V5MX : PATH_TT16;
        // (E5M2: the plain and the halved-block form; E3M4 f16 form: + its gated f32 rerun)
        kev.dispatches = (a.aw && ((a.wfmt == 0 && a.Mw == 2) || a.wfmt == 2)) ? 2 : 1;
        kev.macs = (double)a.M * (double)a.N * (double)a.K;
        if (kev.a && kev.b) (void)hipEventRecord(kev.a, s);
    }
    launch_fast(mode, a, s);
    if (g_ktime && !cap && kev.a && kev.b) {
        (void)hipEventRecord(kev.b, s);
        g_kev.push_back(kev);
    }
    rc = hip_check("fp8a fast gemm launch");
    if (rc) return rc;
    if (a.splits > 1) {
        const int64_t q = a.M * a.N;
        const unsigned rb = (unsigned)std::min<int64_t>((q / 4 + 255) / 256 + 1, 8192);
        splitk_reduce_kernel<<<rb, 256, 0, s>>>(a);
        rc = hip_check("fp8a split-K reduce launch");
        if (rc) return rc;
    }
    // (at most 512 blocks: the kernel is a no-op but for the arena clearing unless the launch
    // flagged, and its 268 VGPRs hold it at one wave per SIMD -- 4096 blocks cost ~7.5 us of wave
    // launches per GEMM; a flagged launch loops its units over the blocks)
    const unsigned ublocks = std::max((unsigned)std::min<int64_t>(a.nur * a.nuc, 512), clear_blocks(lease));
    gemm_exact_kernel<<<ublocks, 256, 0, s>>>(a);
    rc = hip_check("fp8a gated exact gemm launch");
    static const bool dbg = getenv("FP8A_DEBUG_FLAGS") != nullptr;  // diagnostics: the flag word per launch
    if (!rc && dbg) {
        uint32_t f = 0;
        if (hipStreamSynchronize(s) == hipSuccess && hipMemcpy(&f, a.flag_out, sizeof(f), hipMemcpyDeviceToHost) == hipSuccess)
            fprintf(stderr, "fp8a flag M=%lld N=%lld K=%lld E=%d M=%d wfmt=%d flag=%u\n", (long long)a.M, (long long)a.N,
                    (long long)a.K, a.E, a.Mw, a.aw ? a.wfmt : -1, f);
    }
    return rc;
}

// qamaa: term = fq(a*b) (no operand decode: exact for any fp32 inputs), then fq(sum) in place.
static int run_qamaa(GemmArgs &a, hipStream_t s) {
    if (a.M < 0 || a.N < 0 || a.K < 0) return fail(FP8A_EINVAL, "negative extent");
    if (a.M == 0 || a.N == 0) return FP8A_OK;
    if (a.qM < 1 || a.qE < 1) return fail(FP8A_EFORMAT, "bad qamaa quantizer format");
    if (!a.nchw && a.ldc != a.N) return fail(FP8A_EINVAL, "qamaa output must be dense");
    if (a.K == 0) {
        if (dev_fill(a.C, 0, (size_t)a.M * a.N * sizeof(float), s) != hipSuccess) return hip_check("fill");
    } else {
        a.splits = 1;
        a.kchunk = a.K;
        launch_fast(TM_QAMAA, a, s);
        int rc = hip_check("fp8a qamaa gemm launch");
        if (rc) return rc;
    }
    return FP8A_OK;
}

// ------------------------------------------------------------------ the exact product (gemm_dense.h)
static inline int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }
static inline size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

static size_t dense_ws_bytes(int64_t M, int64_t N, int64_t K) {
    const int64_t mpad = round_up(std::max<int64_t>(M, 1), DN_T), npad = round_up(std::max<int64_t>(N, 1), DN_T);
    const int64_t kpad = round_up(std::max<int64_t>(K, 1), 32);
    // byte images at 2 B per element (the bf16 form; the fp8 forms use the first half)
    return al256(4 * (size_t)(mpad / DN_U + npad / DN_U) + 4) + al256((size_t)(2 * mpad * kpad)) +
           al256((size_t)(mpad * kpad / 32)) + al256((size_t)(2 * npad * kpad)) + al256((size_t)(npad * kpad / 32));
}

// A fresh, well-mixed nonzero mark tag per dense call (the dense path's marks are never cleared)
static uint32_t next_dense_gen() {
    static std::atomic<uint32_t> ctr{0};
    uint32_t g;
    do {
        g = (ctr.fetch_add(1) + 1) * 0x9E3779B1u;
        g ^= g >> 15;
    } while (g == 0u);
    return g;
}

static int run_dense(DenseArgs a, void *ws, size_t wsb, hipStream_t s) {
    if (a.M < 0 || a.N < 0 || a.K < 0) return fail(FP8A_EINVAL, "negative extent");
    if (a.fmt != FP8A_DENSE_E4M3 && a.fmt != FP8A_DENSE_E5M2 && a.fmt != FP8A_DENSE_BF16)
        return fail(FP8A_EINVAL, "unknown dense operand format");
    const bool qout = a.fz.qin.mx || a.fz.rq.mx || a.fz.oq.mx || a.fz.wq.mx;
    if (qout && (a.M == 0 || a.K == 0)) {  // no pack pass to leave the quantizers' biases
        dn_bias_kernel<<<(unsigned)std::max<int64_t>(1, (a.N + 255) / 256), 256, 0, s>>>(a.fz, a.N);
        const int rc = hip_check("fp8a dense quantizer biases");
        if (rc) return rc;
    }
    if (a.M == 0 || a.N == 0) return FP8A_OK;
    ++g_paths[PATH_DENSE];
    if (a.K == 0) {
        const hipError_t e = a.conv ? dev_fill(a.y, 0, (size_t)(a.M * a.N) * sizeof(float), s)
                                    : dev_zero_rows(a.y, a.ldc, a.N, a.M, s);
        return e == hipSuccess ? FP8A_OK : hip_check("fp8a dense fill");
    }
    // a small convolution (the stem: K = 27, N = 32) as direct fp32 FMAs (dn_direct_kernel; option
    // "dn_direct", default 1): a 128 x 128 MFMA tile would carry 32 live columns and 27 of 64 k
    if (g_opt_dn_direct && a.conv && a.K <= DD_K && a.N <= DD_N) {
        KernelEv kev{};
        if (g_ktime) {
            kev.a = pool_event();
            kev.b = pool_event();
            kev.path = PATH_DENSE;
            kev.dispatches = 1;
            kev.macs = 4.0 * ((double)a.M * a.K + (double)a.M * a.N) + 4.0 * (double)a.N * a.K;
            if (kev.a && kev.b) (void)hipEventRecord(kev.a, s);
        }
        const unsigned g = (unsigned)std::min<int64_t>((a.M + 255) / 256, 1 << 20);
        dn_direct_kernel<<<g, 256, 0, s>>>(a);
        if (g_ktime && kev.a && kev.b) {
            (void)hipEventRecord(kev.b, s);
            g_kev.push_back(kev);
        }
        return hip_check("fp8a dense direct launch");
    }
    a.mpad = round_up(a.M, DN_T);
    a.npad = round_up(a.N, DN_T);
    a.kpad = round_up(a.K, 32);
    if (a.kpad / 32 > 65535) return fail(FP8A_EINVAL, "K too large for the dense path (> 2097120)");
    if (ws == nullptr || wsb < dense_ws_bytes(a.M, a.N, a.K)) return fail(FP8A_EINVAL, "workspace too small");
    uint8_t *w = static_cast<uint8_t *>(ws);
    // the unit marks hold this call's tag, so no call clears them: a stale word matches the tag
    // only by chance (2^-32 per word), and then its unit is merely recomputed in fp32 by dn_fix
    const size_t nmark = 4 * (size_t)(a.mpad / DN_U + a.npad / DN_U) + 4;
    a.anymark = reinterpret_cast<uint32_t *>(w);
    a.urow = a.anymark + 1;
    a.ucol = a.urow + a.mpad / DN_U;
    a.gen = next_dense_gen();
    w += al256(nmark);
    a.qa = w;  w += al256((size_t)(2 * a.mpad * a.kpad));
    a.qas = w; w += al256((size_t)(a.mpad * a.kpad / 32));
    a.qb = w;  w += al256((size_t)(2 * a.npad * a.kpad));
    a.qbs = w;
    const dim3 ga((unsigned)((a.mpad + 255) / 256), (unsigned)(a.kpad / 32));
    const dim3 gb((unsigned)((a.npad + 255) / 256), (unsigned)(a.kpad / 32));
    const unsigned tiles = (unsigned)((a.mpad / DN_T) * (a.npad / DN_T));
    const unsigned units = (unsigned)((a.mpad / DN_U) * (a.npad / DN_U));
    // (kernel timing: the GEMM launch alone, its algorithmic bytes -- fp32 A read once, fp32 C
    // written once, the packed B image read once -- in the MAC slot)
    KernelEv kev{};
    auto kev_begin = [&]() {
        if (!g_ktime) return;
        kev.a = pool_event();
        kev.b = pool_event();
        kev.path = PATH_DENSE;
        kev.dispatches = 1;
        kev.macs = 4.0 * ((double)a.M * a.K + (double)a.M * a.N) +
                   (a.fmt == FP8A_DENSE_BF16 ? 2.0 : 1.0) * (double)a.npad * a.kpad;
        if (kev.a && kev.b) (void)hipEventRecord(kev.a, s);
    };
    auto kev_end = [&]() {
        if (g_ktime && kev.a && kev.b) {
            (void)hipEventRecord(kev.b, s);
            g_kev.push_back(kev);
        }
    };
    if (a.fmt == FP8A_DENSE_BF16) {  // (A straight from its fp32 source)
        dn_pack<true, 2><<<gb, 256, 0, s>>>(a);
        kev_begin();
        static const bool no_af = getenv("FP8A_NO_PW1") != nullptr;  // (A/B runs: the 64-bit indexing)
        const bool x32 = !no_af && a.conv && 4 * a.C * a.H * a.W * (a.M / (a.Ho * a.Wo)) < (1ll << 31);
        const bool pw1 = x32 && a.kh == 1 && a.kw == 1 && a.sh == 1 && a.sw == 1 && a.ph == 0 && a.pw == 0;
        if (pw1) dn_gemm_bf16<true, 1><<<tiles, 256, 0, s>>>(a);
        else if (x32) dn_gemm_bf16<true, 2><<<tiles, 256, 0, s>>>(a);
        else if (a.conv) dn_gemm_bf16<true><<<tiles, 256, 0, s>>>(a);
        else dn_gemm_bf16<false><<<tiles, 256, 0, s>>>(a);
    } else if (a.fmt == FP8A_DENSE_E4M3) {
        dn_pack<false, 0><<<ga, 256, 0, s>>>(a);
        dn_pack<true, 0><<<gb, 256, 0, s>>>(a);
        kev_begin();
        if (a.conv) dn_gemm<0, true><<<tiles, 256, 0, s>>>(a);
        else dn_gemm<0, false><<<tiles, 256, 0, s>>>(a);
    } else {
        dn_pack<false, 1><<<ga, 256, 0, s>>>(a);
        dn_pack<true, 1><<<gb, 256, 0, s>>>(a);
        kev_begin();
        if (a.conv) dn_gemm<1, true><<<tiles, 256, 0, s>>>(a);
        else dn_gemm<1, false><<<tiles, 256, 0, s>>>(a);
    }
    kev_end();
    dn_fix<<<std::min(units, 2048u), 256, 0, s>>>(a);
    return hip_check("fp8a dense launch");
}

static DenseArgs dense_args() {
    DenseArgs a;
    memset(&a, 0, sizeof(a));
    a.Ho = a.Wo = 1;
    a.kh = a.kw = a.sh = a.sw = a.dh = a.dw = 1;
    return a;
}

}  // namespace fp8a

using namespace fp8a;

template <typename I>
static void launch_group_conv(const GcArgs &a, hipStream_t s) {
    const unsigned g = (unsigned)std::min<int64_t>((a.total + 255) / 256, 65536);
    const bool d1 = a.dw == 1;
    if (d1 && a.kw == 3 && a.sw == 1) dn_group_conv<I, 3, 1><<<g, 256, 0, s>>>(a);
    else if (d1 && a.kw == 3 && a.sw == 2) dn_group_conv<I, 3, 2><<<g, 256, 0, s>>>(a);
    else if (d1 && a.kw == 5 && a.sw == 1) dn_group_conv<I, 5, 1><<<g, 256, 0, s>>>(a);
    else if (d1 && a.kw == 5 && a.sw == 2) dn_group_conv<I, 5, 2><<<g, 256, 0, s>>>(a);
    else dn_group_conv<I, 0, 1><<<g, 256, 0, s>>>(a);
}

// dn_dw3_kernel's block shape: about `target` outputs per workgroup (whole planes when a plane has
// fewer, else bands of rows of one plane), the staged window within dw_lds bytes of LDS (default
// 40 KB, four workgroups per CU: measured against 2 / 8 / 16 KB-windowed plans, §3l); false when even 256 outputs' window does not fit (very wide rows).
static bool plan_dw3(DwArgs &a, int S, size_t &lds, bool raw = false, int tap_bytes = 4) {
    const int64_t op = (int64_t)a.Ho * a.Wo;
    for (int target = std::max(256, g_opt_dw_target); target >= 256; target /= 2) {
        int PB, RB;
        if (op <= target) {
            RB = a.Ho;
            PB = (int)std::min<int64_t>(target / op, a.planes);
            if ((int64_t)a.H * a.W % 4 != 0 && PB >= 4) PB &= ~3;  // 16-byte aligned source ranges (dw_stage)
        } else {
            PB = 1;
            RB = std::max(1, target / a.Wo);
        }
        const int RS = (RB - 1) * S + 3,
                  WS = (std::max(a.W + DW_OX, DW_OX - a.pw + (a.Wo - 1) * S + 3) + 3) / 4 * 4;
        // raw (dn_dw3g_kernel): the unpadded source range from its 16-byte-aligned start
        const int64_t nsrc = RB == a.Ho ? (int64_t)PB * a.H * a.W : (int64_t)std::min(RS, a.H) * a.W;
        a.nimg = (int)(4 * ((nsrc + 6) / 4));
        const int64_t bytes = (raw ? (int64_t)a.nimg : (int64_t)PB * RS * WS) * 4 + (int64_t)PB * 9 * tap_bytes;
        if (bytes > std::min(65536, std::max(4096, g_opt_dw_lds))) continue;
        a.PB = PB; a.RB = RB; a.nb = (a.Ho + RB - 1) / RB; a.RS = RS; a.WS = WS;
        a.inv_c = 1.0f / a.C; a.inv_ws = 1.0f / WS; a.inv_pst = 1.0f / (RS * WS);
        a.inv_wo = 1.0f / a.Wo; a.inv_pout = 1.0f / (RB * a.Wo);
        a.inv_w = 1.0f / a.W; a.inv_hw = 1.0f / (a.H * a.W);
        a.inv_nqd = 1.0f / ((a.Wo + 3) / 4); a.inv_pq = 1.0f / (RB * ((a.Wo + 3) / 4));
        lds = (size_t)bytes;
        return ((a.planes + PB - 1) / PB) * a.nb < (1ll << 24);
    }
    return false;
}

// conv_tbs_kernel's block shape: dn_dw3_kernel's plan with quads of outputs and rows of staged
// words padded to a multiple of 4 (16-byte LDS reads).
static bool plan_tbs(TbsArgs &a, int S, int64_t planes, int64_t C, int64_t H, int64_t W, int64_t Ho, int64_t Wo,
                     int ph, int pw, size_t &lds) {
    if (H >= (1 << 20) || W >= (1 << 20) || C >= (1 << 20) || H * W >= (1ll << 22)) return false;  // (as plan_dw3's caller)
    a.planes = planes; a.C = (int)C; a.H = (int)H; a.W = (int)W; a.Ho = (int)Ho; a.Wo = (int)Wo; a.ph = ph; a.pw = pw;
    const int nq = (int)((Wo + TBX_TW - 1) / TBX_TW);
    const int WS = ((4 * nq - 1) * S + 3 + 3) / 4 * 4;
    const int64_t op = Ho * Wo;
    for (int target = std::max(256, g_opt_dw_target); target >= 256; target /= 2) {
        int PB, RB;
        if (op <= target) {
            RB = (int)Ho;
            PB = (int)std::min<int64_t>(target / op, planes);
            if (H * W % 4 != 0 && PB >= 4) PB &= ~3;  // 16-byte aligned source ranges (dw_stage)
        } else {
            PB = 1;
            RB = std::max(1, (int)(target / Wo));
        }
        const int RS = (RB - 1) * S + 3;
        const int64_t bytes = (int64_t)PB * RS * WS * 4 + 512 + (int64_t)PB * 9 * 8;
        if (bytes > std::min(65536, std::max(4096, g_opt_dw_lds))) continue;
        a.PB = PB; a.RB = RB; a.nb = (int)((Ho + RB - 1) / RB); a.RS = RS; a.WS = WS; a.nq = nq;
        a.inv_c = 1.0f / a.C; a.inv_ws = 1.0f / WS; a.inv_pst = 1.0f / (RS * WS);
        a.inv_nq = 1.0f / nq; a.inv_pq = 1.0f / (RB * nq);
        a.inv_w = 1.0f / a.W; a.inv_hw = 1.0f / (a.H * a.W);
        lds = (size_t)bytes;
        return ((planes + PB - 1) / PB) * a.nb < (1ll << 24);
    }
    return false;
}

extern "C" {

const char *fp8a_version(void) { return "fp8approx gfx950 r1"; }

const char *fp8a_last_error(void) { return g_err.c_str(); }

int fp8a_path_stats(uint64_t *out, int reset) {
    if (out == nullptr) return fail(FP8A_EINVAL, "null pointer");
    for (int i = 0; i < PATH_N; ++i) out[i] = reset ? g_paths[i].exchange(0) : g_paths[i].load();
    return FP8A_OK;
}

size_t fp8a_flag_arena_slot_bytes(fp8a_stream_t stream) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    std::lock_guard<std::mutex> lock(g_arena_mu);
    const auto it = g_arenas.find({dev, (uintptr_t)stream});
    return it == g_arenas.end() ? 0 : it->second.slot;
}

int fp8a_kernel_timing(int enable) {
    const int old = g_ktime ? 1 : 0;
    g_ktime = enable != 0;
    return old;
}

int fp8a_kernel_time(double *out, int reset) {
    if (out == nullptr) return fail(FP8A_EINVAL, "null pointer");
    for (int i = 0; i < 4 * PATH_N; ++i) out[i] = 0.0;
    for (const KernelEv &e : g_kev) {
        if (hipEventSynchronize(e.b) != hipSuccess) return hip_check("fp8a_kernel_time");
        float ms = 0.0f;
        if (hipEventElapsedTime(&ms, e.a, e.b) != hipSuccess) return hip_check("fp8a_kernel_time");
        out[4 * e.path] += ms;
        out[4 * e.path + 1] += 1.0;
        out[4 * e.path + 2] += e.dispatches;
        out[4 * e.path + 3] += e.macs;
    }
    if (reset) {
        for (const KernelEv &e : g_kev) {
            g_evpool.push_back(e.a);
            g_evpool.push_back(e.b);
        }
        g_kev.clear();
    }
    return FP8A_OK;
}

int fp8a_set_option(const char *name, int value) {
    if (name == nullptr) return fail(FP8A_EINVAL, "null pointer");
    if (strcmp(name, "xm_ncg") == 0) {
        const int old = g_opt_xm_ncg;
        g_opt_xm_ncg = value;
        return old;
    }
    if (strcmp(name, "af32_maxct") == 0) {
        const int old = g_opt_af32_maxct;
        g_opt_af32_maxct = std::max(0, value);
        return old;
    }
    if (strcmp(name, "tt_band") == 0) {
        const int old = g_opt_tt_band;
        g_opt_tt_band = value;
        return old;
    }
    if (strcmp(name, "tt16_mink") == 0) {
        const int old = g_opt_tt16_mink;
        g_opt_tt16_mink = std::max(0, value);
        return old;
    }
    if (strcmp(name, "tbx_rw") == 0) {
        const int old = g_opt_tbx_rw;
        g_opt_tbx_rw = value;
        return old;
    }
    if (strcmp(name, "tbs") == 0) {
        const int old = g_opt_tbs;
        g_opt_tbs = value;
        return old;
    }
    if (strcmp(name, "dw_lds") == 0) {
        const int old = g_opt_dw_lds;
        g_opt_dw_lds = std::min(65536, std::max(4096, value));
        return old;
    }
    if (strcmp(name, "dw_target") == 0) {
        const int old = g_opt_dw_target;
        g_opt_dw_target = std::max(256, value);
        return old;
    }
    if (strcmp(name, "dn_direct") == 0) {
        const int old = g_opt_dn_direct;
        g_opt_dn_direct = value;
        return old;
    }
    if (strcmp(name, "v5ds") == 0) {
        const int old = g_opt_v5ds;
        g_opt_v5ds = value;
        return old;
    }
    if (strcmp(name, "dw3") == 0) {
        const int old = g_opt_dw3;
        g_opt_dw3 = value;
        return old;
    }
    return fail(FP8A_EINVAL, std::string("unknown option ") + name);
}

int fp8a_fallback_stats(uint64_t *out, int reset) {
    if (out == nullptr) return fail(FP8A_EINVAL, "null pointer");
    unsigned long long v[4] = {0, 0, 0, 0}, tt = 0;
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpyFromSymbol(v, HIP_SYMBOL(g_fallback), sizeof(v)) != hipSuccess ||
        tt_rerun_stats(&tt, reset != 0) != 0)
        return hip_check("fp8a_fallback_stats");
    for (int i = 0; i < 4; ++i) out[i] = v[i];
    out[2] = tt;  // (gemm_tt_kernel's f32 reruns: k_tt.hip's counter)
    if (reset) {
        const unsigned long long z[4] = {0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_fallback), z, sizeof(z)) != hipSuccess) return hip_check("fp8a_fallback_stats");
    }
    return FP8A_OK;
}

size_t fp8a_dense_matmul_workspace_size(int64_t M, int64_t N, int64_t K) { return dense_ws_bytes(M, N, K); }

int fp8a_dense_matmul(const float *A, int64_t sam, int64_t sak, const float *B, int64_t sbk, int64_t sbn, float *C,
                      int64_t ldc, int64_t M, int64_t N, int64_t K, int fmt, void *workspace, size_t workspace_bytes,
                      fp8a_stream_t stream) {
    if (ldc < N) return fail(FP8A_EINVAL, "leading dimension smaller than extent");
    DenseArgs a = dense_args();
    a.x = A; a.sam = sam; a.sak = sak; a.w = B; a.sbk = sbk; a.sbn = sbn; a.y = C; a.ldc = ldc;
    a.M = M; a.N = N; a.K = K; a.fmt = fmt;
    return run_dense(a, workspace, workspace_bytes, (hipStream_t)stream);
}

size_t fp8a_dense_conv2d_workspace_size(int64_t Bn, int64_t Cin, int64_t H, int64_t W, int64_t Cout, int kh, int kw,
                                        int sh, int sw, int ph, int pw, int dh, int dw) {
    const int64_t Ho = (H + 2 * ph - dh * (kh - 1) - 1) / sh + 1;
    const int64_t Wo = (W + 2 * pw - dw * (kw - 1) - 1) / sw + 1;
    if (Ho <= 0 || Wo <= 0) return 0;
    return dense_ws_bytes(Bn * Ho * Wo, Cout, Cin * kh * kw);
}

int fp8a_dense_conv2d(const float *x, const float *w, float *y, int64_t Bn, int64_t Cin, int64_t H, int64_t W,
                      int64_t Cout, int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw, int fmt,
                      void *workspace, size_t workspace_bytes, fp8a_stream_t stream) {
    if (kh < 1 || kw < 1 || sh < 1 || sw < 1 || dh < 1 || dw < 1 || ph < 0 || pw < 0 || Bn < 0 || Cin < 0 || Cout < 0)
        return fail(FP8A_EINVAL, "bad convolution geometry");
    const int64_t Ho = (H + 2 * ph - dh * (kh - 1) - 1) / sh + 1;
    const int64_t Wo = (W + 2 * pw - dw * (kw - 1) - 1) / sw + 1;
    if (Ho <= 0 || Wo <= 0) return fail(FP8A_EINVAL, "empty convolution output");
    DenseArgs a = dense_args();
    a.x = x; a.w = w; a.y = y; a.conv = 1;
    a.C = Cin; a.H = H; a.W = W; a.Ho = Ho; a.Wo = Wo;
    a.kh = kh; a.kw = kw; a.sh = sh; a.sw = sw; a.ph = ph; a.pw = pw; a.dh = dh; a.dw = dw;
    a.M = Bn * Ho * Wo; a.N = Cout; a.K = Cin * kh * kw;
    a.sbk = 1; a.sbn = a.K;  // w [Cout][Cin][kh][kw]: B(k, n) = w[n * K + k]
    a.ldc = Cout; a.fmt = fmt;
    return run_dense(a, workspace, workspace_bytes, (hipStream_t)stream);
}

static int grouped_conv_impl(const float *x, const float *w, float *y, int64_t Bn, int64_t Cin, int64_t H, int64_t W,
                             int64_t Cout, int groups, int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw,
                             const DnFuse &fz, hipStream_t stream);

int fp8a_grouped_conv2d(const float *x, const float *w, float *y, int64_t Bn, int64_t Cin, int64_t H, int64_t W,
                        int64_t Cout, int groups, int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw,
                        fp8a_stream_t stream) {
    return grouped_conv_impl(x, w, y, Bn, Cin, H, W, Cout, groups, kh, kw, sh, sw, ph, pw, dh, dw, DnFuse{},
                             (hipStream_t)stream);
}

static int grouped_conv_impl(const float *x, const float *w, float *y, int64_t Bn, int64_t Cin, int64_t H, int64_t W,
                             int64_t Cout, int groups, int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw,
                             const DnFuse &fz, hipStream_t stream) {
    if (kh < 1 || kw < 1 || sh < 1 || sw < 1 || dh < 1 || dw < 1 || ph < 0 || pw < 0 || Bn < 0 || Cin < 0 || Cout < 0)
        return fail(FP8A_EINVAL, "bad convolution geometry");
    if (groups < 1 || Cin % groups != 0 || Cout % groups != 0) return fail(FP8A_EINVAL, "channels not divisible by groups");
    const int64_t Ho = (H + 2 * ph - dh * (kh - 1) - 1) / sh + 1;
    const int64_t Wo = (W + 2 * pw - dw * (kw - 1) - 1) / sw + 1;
    if (Ho <= 0 || Wo <= 0) return fail(FP8A_EINVAL, "empty convolution output");
    GcArgs a{};
    a.x = x; a.w = w; a.y = y;
    a.Cin = Cin; a.H = H; a.W = W; a.Cout = Cout; a.Ho = Ho; a.Wo = Wo;
    a.total = Bn * Cout * Ho * ((Wo + GC_OW - 1) / GC_OW);
    a.cig = (int)(Cin / groups); a.cog = (int)(Cout / groups);
    a.kh = kh; a.kw = kw; a.sh = sh; a.sw = sw; a.ph = ph; a.pw = pw; a.dh = dh; a.dw = dw;
    a.fz = fz;
    if (a.total == 0) {  // (no kernel to leave the fused quantizers' biases)
        if (fz.qin.mx || fz.rq.mx || fz.oq.mx || fz.wq.mx) {
            dn_bias_kernel<<<(unsigned)std::max<int64_t>(1, (Cout + 255) / 256), 256, 0, stream>>>(fz, Cout);
            return hip_check("fp8a grouped conv quantizer biases");
        }
        return FP8A_OK;
    }
    if (!x || !w || !y) return fail(FP8A_EINVAL, "null pointer");
    if (g_opt_dw3 && a.cig == 1 && a.cog == 1 && kh == 3 && kw == 3 && dh == 1 && dw == 1 && sh == sw && pw <= DW_OX &&
        (sh == 1 || sh == 2)) {
        DwArgs d{};
        d.x = x; d.w = w; d.y = y; d.fz = fz;
        d.planes = Bn * Cout; d.C = (int)Cout; d.H = (int)H; d.W = (int)W; d.Ho = (int)Ho; d.Wo = (int)Wo;
        d.ph = ph; d.pw = pw;
        size_t lds = 0;
        // (the staged kernels index a plane in 32-bit ints and divide by float reciprocals, dw_div:
        // planes of at most 2^22 values; larger ones take dn_group_conv)
        d.nx = Bn * Cin * H * W;
        const bool raw = g_opt_dw3 == 2;
        if (H < (1 << 20) && W < (1 << 20) && Cout < (1 << 20) && H * W < (1ll << 22) && plan_dw3(d, sh, lds, raw)) {
            const unsigned g = (unsigned)(((d.planes + d.PB - 1) / d.PB) * d.nb);
            if (raw && sh == 1) dn_dw3g_kernel<1><<<g, 256, lds, stream>>>(d);
            else if (raw) dn_dw3g_kernel<2><<<g, 256, lds, stream>>>(d);
            else if (sh == 1) dn_dw3_kernel<1><<<g, 256, lds, stream>>>(d);
            else dn_dw3_kernel<2><<<g, 256, lds, stream>>>(d);
            ++g_paths[PATH_DENSE];
            return hip_check("fp8a depthwise conv launch");
        }
    }
    if (a.total + 65536ll * 256 < (1ll << 31)) launch_group_conv<uint32_t>(a, stream);
    else launch_group_conv<int64_t>(a, stream);
    ++g_paths[PATH_DENSE];
    return hip_check("fp8a grouped conv launch");
}

int fp8a_clock_stats(uint64_t *out, int reset) {
    if (out == nullptr) return fail(FP8A_EINVAL, "null pointer");
    if (hipDeviceSynchronize() != hipSuccess) return hip_check("fp8a_clock_stats");
    unsigned long long v[3] = {0, 0, 0};
    int (*parts[3])(unsigned long long *, bool) = {f8mx_clock_xf0, f8mx_clock_xf1, f8mx_clock_xf2};
    for (auto f : parts) {
        unsigned long long w[3] = {0, 0, 0};
        if (f(w, reset != 0) != 0) return hip_check("fp8a_clock_stats");
        for (int i = 0; i < 3; ++i) v[i] += w[i];
    }
    for (int i = 0; i < 3; ++i) out[i] = v[i];
    return FP8A_OK;
}

int fp8a_dense_stats(uint64_t *out, int reset) {
    if (out == nullptr) return fail(FP8A_EINVAL, "null pointer");
    unsigned long long v[2] = {0, 0};
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpyFromSymbol(v, HIP_SYMBOL(g_dense), sizeof(v)) != hipSuccess)
        return hip_check("fp8a_dense_stats");
    out[0] = v[0];
    out[1] = v[1];
    if (reset) {
        const unsigned long long z[2] = {0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_dense), z, sizeof(z)) != hipSuccess) return hip_check("fp8a_dense_stats");
    }
    return FP8A_OK;
}

int fp8a_decompose(const float *x, int64_t rows, int64_t cols, int64_t ld, int E, int M, const int32_t *bias,
                   int64_t bias_stride, uint32_t flags, int32_t *expo, int32_t *mant, fp8a_stream_t stream) {
    int rc = check_format(E, M);
    if (rc) return rc;
    if (rows < 0 || cols < 0 || ld < cols) return fail(FP8A_EINVAL, "bad decompose extents");
    const int64_t total = rows * cols;
    if (total == 0) return FP8A_OK;
    decompose_kernel<<<(unsigned)((total + 255) / 256), 256, 0, (hipStream_t)stream>>>(
        x, rows, cols, ld, E, M, bias, bias_stride, flags, expo, mant);
    return hip_check("fp8a_decompose");
}

int fp8a_quant(const float *x, int64_t n, int E, int M, const int32_t *bias, uint32_t flags, float *out,
               fp8a_stream_t stream) {
    int rc = check_format(E, M);
    if (rc) return rc;
    if (n <= 0) return FP8A_OK;
    quant_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(x, n, E, M, bias, flags, out);
    return hip_check("fp8a_quant");
}

static GemmArgs make_args(const float *A, int64_t lda, const float *B, int64_t sbk, int64_t sbn, float *C,
                          int64_t ldc, int64_t M, int64_t N, int64_t K, int E, int Mw, const int32_t *bA,
                          const int32_t *bB, int64_t bBs, const int32_t *bR, uint32_t flags) {
    GemmArgs a;
    memset(&a, 0, sizeof(a));
    a.A = A; a.lda = lda; a.B = B; a.sbk = sbk; a.sbn = sbn; a.C = C; a.ldc = ldc;
    a.M = M; a.N = N; a.K = K; a.E = E; a.Mw = Mw; a.kexp = 0x7F800000u; a.kdc = (uint32_t)(23 - Mw) << 23;
    a.bA = bA; a.bB = bB; a.bBs = bBs; a.bR = bR;
    a.flags = flags; a.nchw = 0; a.hw = 1; a.ctot = N; a.coff = 0;
    a.splits = 1; a.kchunk = K; a.part = nullptr;
    return a;
}

size_t fp8a_matmul_workspace_size(void) { return FLAG_BYTES; }

size_t fp8a_matmul_workspace_size_mnk(int64_t M, int64_t N, int64_t K) {
    if (M <= 0 || N <= 0 || K <= 0) return FLAG_BYTES;
    return gemm_workspace_bytes(M, N, K, 0);
}

int fp8a_matmul(const float *A, int64_t lda, const float *B, int64_t sbk, int64_t sbn, float *C, int64_t ldc,
                int64_t M, int64_t N, int64_t K, int E, int Mw, const int32_t *bA, const int32_t *bB,
                int64_t bB_stride, const int32_t *bR, const int32_t *table, uint32_t flags, void *workspace,
                size_t workspace_bytes, fp8a_stream_t stream) {
    if (lda < K || ldc < N) return fail(FP8A_EINVAL, "leading dimension smaller than extent");
    GemmArgs a = make_args(A, lda, B, sbk, sbn, C, ldc, M, N, K, E, Mw, bA, bB, bB_stride, bR, flags);
    return run_gemm(a, table, workspace, workspace_bytes, (hipStream_t)stream);
}

int fp8a_terms(const float *A, int64_t lda, const float *B, int64_t sbk, int64_t sbn, float *T, int64_t M,
               int64_t N, int64_t K, int E, int Mw, const int32_t *bA, const int32_t *bB, int64_t bB_stride,
               const int32_t *bR, const int32_t *table, uint32_t flags, fp8a_stream_t stream) {
    int rc = check_format(E, Mw);
    if (rc) return rc;
    GemmArgs a = make_args(A, lda, B, sbk, sbn, nullptr, 0, M, N, K, E, Mw, bA, bB, bB_stride, bR, flags);
    int mode;
    rc = pack_table(table, Mw, (flags & (F_APPROX | F_V5)) != 0, a.tab, mode);
    if (rc) return rc;
    const int64_t total = M * N * K;
    if (total == 0) return FP8A_OK;
    terms_kernel<<<(unsigned)((total + 255) / 256), 256, 0, (hipStream_t)stream>>>(a, T);
    return hip_check("fp8a_terms");
}

int fp8a_im2col(const float *x, float *out, int64_t Bn, int64_t Cin, int64_t H, int64_t W, int kh, int kw, int sh,
                int sw, int ph, int pw, int dh, int dw, fp8a_stream_t stream) {
    const int64_t Ho = (H + 2 * ph - dh * (kh - 1) - 1) / sh + 1;
    const int64_t Wo = (W + 2 * pw - dw * (kw - 1) - 1) / sw + 1;
    if (Ho <= 0 || Wo <= 0) return fail(FP8A_EINVAL, "empty convolution output");
    const int64_t total = Bn * Ho * Wo * Cin * kh * kw;
    if (total == 0) return FP8A_OK;
    const int64_t blocks = std::min<int64_t>((total + 255) / 256, 65536);
    im2col_kernel<<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(x, out, Bn, Cin, H, W, kh, kw, sh, sw, ph, pw,
                                                                     dh, dw, Ho, Wo);
    return hip_check("fp8a_im2col");
}

size_t fp8a_conv2d_workspace_size(int64_t Bn, int64_t Cin, int64_t H, int64_t W, int64_t Cout, int kh, int kw,
                                  int sh, int sw, int ph, int pw, int dh, int dw, int groups) {
    if (groups <= 0 || Cout % groups != 0 || Cin % groups != 0) return 0;
    const int64_t Ho = (H + 2 * ph - dh * (kh - 1) - 1) / sh + 1;
    const int64_t Wo = (W + 2 * pw - dw * (kw - 1) - 1) / sw + 1;
    if (Ho <= 0 || Wo <= 0) return 0;
    // implicit GEMM (no im2col image): the off-grid flag word + split-K partials of one group
    const int64_t Mrows = Bn * Ho * Wo, cog = Cout / groups, Kg = (Cin / groups) * kh * kw;
    if (Mrows <= 0 || Kg <= 0) return FLAG_BYTES;
    // tensor-bias kernels: A words (+ the v5 depthwise form's B words)
    if (cog == 1) return FLAG_BYTES + align256((size_t)(Bn * Cin * H * W) * 4) + (size_t)(Cout * kh * kw) * 8;
    // A words: the zero-bordered word image of gemm_f8mx_kernel (xm_a_words)
    const WordImage wi = word_image(H, W, ph, pw);
    return gemm_workspace_bytes(Mrows, cog, Kg, Bn * (Cin / groups) * wi.H * wi.W);
}

int fp8a_conv2d(const float *x, const float *w, float *y, int64_t Bn, int64_t Cin, int64_t H, int64_t W,
                int64_t Cout, int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw, int groups, int E,
                int Mw, const int32_t *bA, const int32_t *bW, const int32_t *bR, const int32_t *table,
                uint32_t flags, void *workspace, size_t workspace_bytes, fp8a_stream_t stream) {
    return fp8a_conv2d_bn_act(x, w, y, Bn, Cin, H, W, Cout, kh, kw, sh, sw, ph, pw, dh, dw, groups, E, Mw, bA, bW, bR,
                              table, flags, nullptr, 0, 0.0f, 0.0f, workspace, workspace_bytes, stream);
}

// The convolution entry points.  fq.mx set: x is NOT yet quantized; the activation quantizer
// (fp8_quantizer.py:97-173, per tensor) is applied inside the matrix-core / tensor-bias-table
// pre-decodes (its bias written to fqb / fqi, which serve as bA), or -- for every other path --
// into xq (numel(x) floats) by one fake-quant pass first.

// A quantizer's bias (quantize_to_fp8_ste_MM's custom_bias) from its maxval, where no kernel of
// the launch family writes it.
__global__ void fq_bias_kernel(FqIn fq, float *bias_out, int32_t *ibias_out) {
    const float b = fq_bias(*fq.mx, fq.E, fq.M);
    *bias_out = b;
    *ibias_out = (int32_t)b;
}

static int conv2d_impl(const float *x, const float *w, float *y, int64_t Bn, int64_t Cin, int64_t H, int64_t W,
                       int64_t Cout, int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw, int groups,
                       int E, int Mw, const int32_t *bA, const int32_t *bW, const int32_t *bR, const int32_t *table,
                       uint32_t flags, const float *bn, int act, float act_lo, float act_hi, void *workspace,
                       size_t workspace_bytes, hipStream_t s, FqIn fq, float *fqb, int32_t *fqi, float *xq,
                       const float *res = nullptr, int post_act = 0, float post_lo = 0.0f, float post_hi = 0.0f,
                       FqIn post_fq = FqIn{}, const uint32_t *in_img = nullptr, const EmitW &em_in = EmitW{},
                       float *post_bout = nullptr, int32_t *post_ibout = nullptr) {
    const float2 *ep = reinterpret_cast<const float2 *>(bn);
    if (ep && (((uintptr_t)bn) & 7) != 0) return fail(FP8A_EINVAL, "bn parameters must be 8-byte aligned");
    int rc = check_format(E, Mw);
    if (rc) return rc;
    if (groups <= 0 || Cout % groups != 0 || Cin % groups != 0) return fail(FP8A_EINVAL, "bad groups");
    const int64_t Ho = (H + 2 * ph - dh * (kh - 1) - 1) / sh + 1;
    const int64_t Wo = (W + 2 * pw - dw * (kw - 1) - 1) / sw + 1;
    if (Ho <= 0 || Wo <= 0) return fail(FP8A_EINVAL, "empty convolution output");
    const int64_t cog = Cout / groups, cig = Cin / groups;
    const int64_t Mrows = Bn * Ho * Wo, Ktot = Cin * kh * kw, Kg = cig * kh * kw;
    if (Mrows == 0) {  // (the output quantizer's bias is still set, as its forward would)
        if (post_bout) fq_bias_kernel<<<1, 1, 0, s>>>(post_fq, post_bout, post_ibout);
        return post_bout ? hip_check("fp8a output-quantizer bias") : FP8A_OK;
    }
    // non-fused input quantization: one fake-quant pass into xq, then the plain path on it
    auto materialize = [&]() -> int {
        const int64_t nx = Bn * Cin * H * W;
        fp8_quantize_kernel<<<(unsigned)std::max<int64_t>(1, std::min<int64_t>((nx + 255) / 256, 65536)), 256, 0, s>>>(
            x, 1, nx, fq.mx, 0, fq.E, fq.M, fq.S, xq, fqb, fqi);
        x = xq;
        bA = fqi;
        fq.mx = nullptr;
        return hip_check("fp8a input fake-quant");
    };
    const bool post = res || post_act || post_fq.mx;
    // v5 words (form 2) come from the staged v5 depthwise kernel only: any other launch flags them invalid
    EmitW em = em_in;
    if (em.w && (em.form == 2) != ((flags & F_V5) && cog == 1 && !post && groups > 1)) {
        if (dev_fill(em.invalid, 1, sizeof(uint32_t), s) != hipSuccess) return hip_check("fp8a word image header");
        em = EmitW{};
    }
    if (res && (res == y || (((uintptr_t)res) & 15) != 0))
        return fail(FP8A_EINVAL, "the residual must be a 16-byte aligned tensor other than the output");
    if (cog == 1 && !(flags & F_V5)) {  // v5 never had tensor-bias semantics: it takes the GEMM path
        if (post) return fail(FP8A_EINVAL, "no block-output epilogue for single-output-channel groups");
        TablePack tp;
        int mode;
        rc = pack_table(table, Mw, flags & F_APPROX, tp, mode);
        if (rc) return rc;
        const int64_t total = Bn * Cout * Ho * Wo;
        uint32_t *gate = nullptr;
        ArenaLease lease;  // (gate: a slot of the stream's flag arena, flag_arena)
        bool emitted = false;  // (a requested word image: only the staged table-form kernel writes it)
        // fast form: needs s2n on and golden_clip_OF off (else every launch would fall back)
        const bool fast_ok = (flags & F_S2N) && !(flags & F_GCLIP) && workspace != nullptr &&
                             workspace_bytes >= FLAG_BYTES && Cout <= 65535 && Bn <= 65535;
        // E4M3 table form (conv_tbx.h): {0,1} / zero table, qbma, 3-wide kernel rows, stride 1 or 2
        const int64_t nwg = (Wo + TBX_TW - 1) / TBX_TW, items = Bn * Cout * Ho * nwg;
        static const bool no_tbx = getenv("FP8A_NO_TBX") != nullptr;
        const bool tbx_ok = fast_ok && !no_tbx && ((E == 4 && Mw == 3) || (E == 5 && Mw == 2)) &&
                            (mode == TM_NONE || mode == TM_W1U) &&
                            (flags & F_QBMA) && kw == 3 && dw == 1 && sh == sw && (sw == 1 || sw == 2) &&
                            items < (1ll << 31) && Ho * Wo < (1ll << 31) &&
                            workspace_bytes >= FLAG_BYTES + (size_t)(Bn * Cin * H * W) * 4;
        if (fq.mx && !tbx_ok) {
            rc = materialize();
            if (rc) return rc;
        }
        if (tbx_ok) {
            if (!dw_lease(s, workspace, workspace_bytes, lease)) return lease_error();
            gate = lease.mine;
            // the input's table-form words from the producing launch (fp8a_conv2d_chain, next_form 1:
            // header + [Bn][Cin][H][W] words of fq_in(x)); the pre-pass then runs gated on its header
            const bool use_img = in_img != nullptr && fq.mx != nullptr;
            uint32_t *aw = use_img ? const_cast<uint32_t *>(in_img) + 64 : (uint32_t *)((char *)workspace + FLAG_BYTES);
            TbsArgs tb{};
            size_t tlds = 0;
            // tbs = 2 (default): the LDS-DMA-staged conv_tbsg_kernel
            DwArgs dg{};
            size_t glds = 0;
            const bool tbsg = g_opt_tbs == 2 && !use_img && cig == 1 && kh == 3 && dh == 1 && H < (1 << 20) &&
                              W < (1 << 20) && Cout < (1 << 20) && H * W < (1ll << 22) && [&]() {
                                  dg.planes = Bn * Cout; dg.C = (int)Cout; dg.H = (int)H; dg.W = (int)W;
                                  dg.Ho = (int)Ho; dg.Wo = (int)Wo; dg.ph = ph; dg.pw = pw; dg.nx = Bn * Cin * H * W;
                                  if (!plan_dw3(dg, sw, glds, true, tbsg_tap_bytes())) return false;
                                  glds = tbsg_lds_bytes(dg.PB, dg.nimg);
                                  return glds <= 65536;
                              }();
            if (tbsg) {
                const unsigned gb = (unsigned)(((dg.planes + dg.PB - 1) / dg.PB) * dg.nb);
                // (it emits the next matrix-core convolution's words when fp8a_conv2d_chain asked, em.form 0)
                const EmitW emt = em.w && em.form == 0 ? em : EmitW{};
                emitted = emt.w != nullptr;
#define FP8A_TBSG(S_, M_) conv_tbsg_kernel<S_, M_><<<gb, 256, glds, s>>>(x, w, y, dg, fq, fqb, fqi, bA, bW, bR, tp, gate, ep, act, act_lo, act_hi, emt)
                if (Mw == 2) { if (sw == 1) FP8A_TBSG(1, 2); else FP8A_TBSG(2, 2); }
                else { if (sw == 1) FP8A_TBSG(1, 3); else FP8A_TBSG(2, 3); }
#undef FP8A_TBSG
                if (fq.mx) bA = fqi;
                rc = hip_check("fp8a_conv2d (tensor-bias groups, LDS-DMA staged table form)");
                if (rc) return rc;
            } else if (g_opt_tbs && !use_img && cig == 1 && kh == 3 && dh == 1 && plan_tbs(tb, sw, Bn * Cout, Cout, H, W, Ho, Wo,
                                                                                  ph, pw, tlds)) {
                const unsigned gb = (unsigned)(((tb.planes + tb.PB - 1) / tb.PB) * tb.nb);
#define FP8A_TBS(S_, M_) conv_tbs_kernel<S_, M_><<<gb, 256, tlds, s>>>(x, w, y, tb, fq, fqb, fqi, bA, bW, bR, tp, gate, ep, act, act_lo, act_hi)
                if (Mw == 2) { if (sw == 1) FP8A_TBS(1, 2); else FP8A_TBS(2, 2); }
                else { if (sw == 1) FP8A_TBS(1, 3); else FP8A_TBS(2, 3); }
#undef FP8A_TBS
                if (fq.mx) bA = fqi;
                rc = hip_check("fp8a_conv2d (tensor-bias groups, staged table form)");
                if (rc) return rc;
            } else {
            const int64_t nx = Bn * Cin * H * W;
            tbx_decode_a<<<(unsigned)std::min<int64_t>((nx + 255) / 256, use_img ? 1024 : 8192), 256, 0, s>>>(
                x, nx, aw, gate, fq, fqb, fqi, Mw, use_img ? in_img : nullptr);
            if (fq.mx) bA = fqi;
            TbxArgs ta;
            ta.Cin = Cin; ta.H = H; ta.W = W; ta.Cout = Cout; ta.Ho = Ho; ta.Wo = Wo;
            ta.kh = kh; ta.ph = ph; ta.pw = pw; ta.dh = dh; ta.cpg = (int)cig;
            ta.nwg = (uint32_t)nwg;
            const bool rw2 = g_opt_tbx_rw == 2 && dh == 1;
            ta.items = (uint32_t)(rw2 ? Bn * Cout * ((Ho + 1) / 2) * nwg : items);
            const unsigned gb = (unsigned)std::min<int64_t>((ta.items + 255) / 256, 8 * 1024);
#define FP8A_TBX(SW_, M_, RW_) conv_tbx_kernel<SW_, M_, RW_><<<gb, 256, 0, s>>>(aw, w, y, ta, bA, bW, bR, tp, gate, ep, act, act_lo, act_hi)
            if (Mw == 2) {
                if (sw == 1) { if (rw2) FP8A_TBX(1, 2, 2); else FP8A_TBX(1, 2, 1); }
                else { if (rw2) FP8A_TBX(2, 2, 2); else FP8A_TBX(2, 2, 1); }
            } else {
                if (sw == 1) { if (rw2) FP8A_TBX(1, 3, 2); else FP8A_TBX(1, 3, 1); }
                else { if (rw2) FP8A_TBX(2, 3, 2); else FP8A_TBX(2, 3, 1); }
            }
#undef FP8A_TBX
            rc = hip_check("fp8a_conv2d (tensor-bias groups, E4M3 / E5M2 table form)");
            if (rc) return rc;
            }
        } else if (fast_ok) {
            if (!dw_lease(s, workspace, workspace_bytes, lease)) return lease_error();
            gate = lease.mine;
            dim3 grid((unsigned)((Ho * Wo + 255) / 256), (unsigned)Cout, (unsigned)Bn);
            conv_tb_fast_kernel<<<grid, 256, 0, s>>>(x, w, y, Cin, H, W, Cout, kh, kw, sh, sw, ph, pw, dh, dw, groups,
                                                     Ho, Wo, Mw, bA, bW, bR, tp, flags | F_TB, gate, ep, act, act_lo,
                                                     act_hi);
            rc = hip_check("fp8a_conv2d (tensor-bias groups, fast)");
            if (rc) return rc;
        }
        // (gated: at most 1024 blocks -- a no-op launch unless the fast kernel flagged)
        const unsigned eb = (unsigned)(fast_ok ? std::min<int64_t>((total + 255) / 256, 1024) : (total + 255) / 256);
        if (fast_ok) {  // gated, grid-capped: a no-op launch unless the fast kernel flagged
            conv_tb_direct_kernel<true><<<std::max(eb, clear_blocks(lease)), 256, 0, s>>>(
                x, w, y, Bn, Cin, H, W, Cout, kh, kw, sh, sw, ph, pw, dh, dw, groups, Ho, Wo, E, Mw, bA, bW, bR, tp,
                flags | F_TB, gate, (uint32_t *)workspace, lease.clr, lease.clr16, ep, act, act_lo, act_hi, fq);
        } else {
            conv_tb_direct_kernel<true><<<eb, 256, 0, s>>>(x, w, y, Bn, Cin, H, W, Cout, kh, kw, sh, sw, ph, pw, dh, dw,
                                                     groups, Ho, Wo, E, Mw, bA, bW, bR, tp, flags | F_TB, nullptr,
                                                     nullptr, nullptr, 0u, ep, act, act_lo, act_hi, FqIn{});
        }
        if (em.w && !emitted && dev_fill(em.invalid, 1, sizeof(uint32_t), s) != hipSuccess)  // (no emission here)
            return hip_check("fp8a word image header");
        return hip_check("fp8a_conv2d (tensor-bias groups)");
    }
    // (a workspace below fp8a_conv2d_workspace_size but holding the flag word runs unsplit)
    if (workspace == nullptr || workspace_bytes < FLAG_BYTES) return fail(FP8A_EINVAL, "conv2d workspace too small");
    if (Kg >= (1ll << 31)) return fail(FP8A_EINVAL, "conv2d window too large");
    (void)Ktot;
    if (fq.mx) {  // fuse into the matrix-core pre-decode only where run_gemm will take that path
        TablePack tp;
        int mode;
        rc = pack_table(table, Mw, (flags & (F_APPROX | F_V5)) != 0, tp, mode);
        if (rc) return rc;
        if (flags & F_V5) mode = TM_V5;  // (as run_gemm)
        const WordImage wi = word_image(H, W, ph, pw);
        const int64_t a_words = Bn * cig * wi.H * wi.W;  // as xm_a_words / run_gemm
        const int64_t kpad = (Kg + BK - 1) / BK * BK, npad = (cog + BN - 1) / BN * BN;
        // (run_gemm's matrix-core forms: every one applies fq in its A pre-decode, xm_decode_a)
        const uint32_t gf = flags & ~F_TB;
        const bool form = f8_form(E, Mw, gf, mode) || tt_form(Mw, gf, tp) || v5mx_form(Mw, gf, mode);
        const bool fused = form && !no_mx() && a_words < (1ll << 30) &&
                           kpad * npad * 4 < (1ll << 32) &&
                           workspace_bytes >= gemm_workspace_bytes(Mrows, cog, Kg, a_words);
        if (!fused) {
            rc = materialize();
            if (rc) return rc;
        }
    }
    // v5 depthwise: one direct launch (a GEMM per single-column group would be `groups` launches of
    // N = 1 tiles: MobileNetV2 E5M2 v5 ran at ~500 images/s that way)
    if ((flags & F_V5) && cog == 1 && !post && groups > 1) {
        TablePack tp;
        int mode;
        rc = pack_table(table, Mw, true, tp, mode);
        if (rc) return rc;
        const int64_t total = Bn * Cout * Ho * Wo;
        // the word form (conv_v5dw_kernel, conv_tbx.h): E5M2 with the adder wrap, depthwise 3-wide
        // rows, stride 1 / 2; the literal kernel behind it runs only if its gate is raised
        const int64_t nx = Bn * Cin * H * W, nwg = (Wo + TBX_TW - 1) / TBX_TW, items = Bn * Cout * Ho * nwg;
        const size_t awb = align256((size_t)nx * 4);
        static const bool no_v5dw = getenv("FP8A_NO_V5DW") != nullptr;
        const bool v5dw_ok = !no_v5dw && Mw == 2 && (flags & F_OFUF) && cig == 1 && kw == 3 && kh <= 5 && dw == 1 &&
                             sh == sw && (sw == 1 || sw == 2) && items < (1ll << 31) && Ho * Wo < (1ll << 31) &&
                             workspace != nullptr && workspace_bytes >= FLAG_BYTES + awb + (size_t)(Cout * kh * kw) * 8;
        uint32_t *gate = nullptr;
        ArenaLease lease;  // (gate: a slot of the stream's flag arena, flag_arena)
        // the staged form (conv_v5ds_kernel: both pre-passes fused): depthwise 3 x 3, dilation 1
        DwArgs d{};
        size_t lds = 0;
        const bool v5ds = v5dw_ok && g_opt_v5ds && kh == 3 && kw == 3 && dh == 1 && H < (1 << 20) && W < (1 << 20) &&
                          Cout < (1 << 20) && H * W < (1ll << 22) && [&]() {
                              d.planes = Bn * Cout; d.C = (int)Cout; d.H = (int)H; d.W = (int)W;
                              d.Ho = (int)Ho; d.Wo = (int)Wo; d.ph = ph; d.pw = pw; d.nx = nx;
                              if (!plan_dw3(d, sh, lds, true)) return false;
                              lds = (size_t)d.nimg * 4 + (size_t)d.PB * 9 * 8;  // (tap words: 8 B)
                              return lds <= 65536;
                          }();
        if (v5ds) {
            if (!dw_lease(s, workspace, workspace_bytes, lease)) return lease_error();
            gate = lease.mine;
            const unsigned g = (unsigned)(((d.planes + d.PB - 1) / d.PB) * d.nb);
            // (it emits the next convolution's v5 words when fp8a_conv2d_chain asked for them, em.form 2)
            const EmitW emv = em.w && em.form == 2 ? em : EmitW{};
            if (sh == 1)
                conv_v5ds_kernel<1><<<g, 256, lds, s>>>(x, w, y, d, fq, fqb, fqi, bA, bW, bR, tp, flags, E, gate, ep,
                                                        act, act_lo, act_hi, emv);
            else
                conv_v5ds_kernel<2><<<g, 256, lds, s>>>(x, w, y, d, fq, fqb, fqi, bA, bW, bR, tp, flags, E, gate, ep,
                                                        act, act_lo, act_hi, emv);
            rc = hip_check("fp8a_conv2d (v5 depthwise, staged)");
            if (rc) return rc;
            if (fq.mx) bA = fqi;
            ++g_paths[PATH_FAST];
        } else if (v5dw_ok) {
            if (em.w && dev_fill(em.invalid, 1, sizeof(uint32_t), s) != hipSuccess)  // (no emission here)
                return hip_check("fp8a word image header");
            if (!dw_lease(s, workspace, workspace_bytes, lease)) return lease_error();
            gate = lease.mine;
            uint32_t *aw = (uint32_t *)((char *)workspace + FLAG_BYTES);
            uint2 *bwd = (uint2 *)((char *)workspace + FLAG_BYTES + awb);
            // (the input quantizer applied here, its bias written for the kernels after: bA = fqi)
            v5dw_decode_a<<<(unsigned)std::min<int64_t>((nx + 255) / 256, 8192), 256, 0, s>>>(x, nx, aw, E, Mw, bA, fq,
                                                                                               fqb, fqi);
            if (fq.mx) bA = fqi;
            const int64_t nb = Cout * kh * kw;
            v5dw_decode_b<<<(unsigned)std::min<int64_t>((nb + 255) / 256, 1024), 256, 0, s>>>(w, nb, kh * kw, bwd, E, Mw,
                                                                                               bA, bW, bR, tp);
            TbxArgs ta;
            ta.Cin = Cin; ta.H = H; ta.W = W; ta.Cout = Cout; ta.Ho = Ho; ta.Wo = Wo;
            ta.kh = kh; ta.ph = ph; ta.pw = pw; ta.dh = dh; ta.cpg = 1;
            ta.nwg = (uint32_t)nwg;
            ta.items = (uint32_t)items;
            const unsigned gb = (unsigned)std::min<int64_t>((items + 255) / 256, 8 * 1024);
            if (sw == 1)
                conv_v5dw_kernel<1><<<gb, 256, 0, s>>>(aw, bwd, y, ta, bR, flags, E, gate, ep, act, act_lo, act_hi);
            else
                conv_v5dw_kernel<2><<<gb, 256, 0, s>>>(aw, bwd, y, ta, bR, flags, E, gate, ep, act, act_lo, act_hi);
            rc = hip_check("fp8a_conv2d (v5 depthwise, word form)");
            if (rc) return rc;
            ++g_paths[PATH_FAST];
        } else {
            ++g_paths[PATH_EXACT];
            if (em.w && dev_fill(em.invalid, 1, sizeof(uint32_t), s) != hipSuccess)  // (no emission here)
                return hip_check("fp8a word image header");
            if (fq.mx) {
                fq_bias_kernel<<<1, 1, 0, s>>>(fq, fqb, fqi);
                bA = fqi;
            }
        }
        // (x unquantized when fq is set: the literal kernel applies fq to every loaded value)
        conv_tb_direct_kernel<false><<<std::max((unsigned)std::min<int64_t>((total + 255) / 256, 16384),
                                                clear_blocks(lease)), 256, 0, s>>>(
            x, w, y, Bn, Cin, H, W, Cout, kh, kw, sh, sw, ph, pw, dh, dw, groups, Ho, Wo, E, Mw, bA, bW, bR, tp, flags,
            gate, gate ? (uint32_t *)workspace : nullptr, lease.clr, lease.clr16, ep, act, act_lo, act_hi, fq);
        return hip_check("fp8a_conv2d (v5 depthwise, direct)");
    }
    for (int g = 0; g < groups; ++g) {
        GemmArgs a = make_args(nullptr, 0, w + g * cog * Kg, 1, Kg, y, 0, Mrows, cog, Kg, E, Mw, bA, bW + g * cog, 1,
                               bR, flags & ~F_TB);
        a.nchw = 1;
        a.hw = Ho * Wo;
        a.ctot = Cout;
        a.coff = g * cog;
        a.conv = 1;
        a.X = x;
        a.Cin = Cin; a.H = H; a.W = W; a.Ho = Ho; a.Wo = Wo; a.cbase = g * cig; a.aw_c = cig;
        a.kh = kh; a.kw = kw; a.sh = sh; a.sw = sw; a.ph = ph; a.pw = pw; a.dh = dh; a.dw = dw;
        fastdiv_params((uint32_t)(kh * kw), a.kk_mul, a.kk_shift);
        fastdiv_params((uint32_t)kw, a.kw_mul, a.kw_shift);
        a.ep = ep; a.ep_act = act; a.ep_lo = act_lo; a.ep_hi = act_hi;
        if (fq.mx) {
            a.fqin = fq;
            a.fq_bias = fqb;
            a.fq_ibias = fqi;
            a.bA = fqi;  // written by the A pre-decode before any kernel reads it
        }
        a.res = res; a.post_act = post_act; a.post_lo = post_lo; a.post_hi = post_hi; a.post_fq = post_fq;
        a.post_bout = post_bout; a.post_ibout = post_ibout;
        if (groups == 1) {  // (fp8a_conv2d_chain only asks for these on ungrouped convolutions)
            a.in_img = in_img;
            a.em = em;
        }
        rc = run_gemm(a, table, workspace, workspace_bytes, s);
        if (rc) return rc;
    }
    return FP8A_OK;
}

int fp8a_conv2d_bn_act(const float *x, const float *w, float *y, int64_t Bn, int64_t Cin, int64_t H, int64_t W,
                       int64_t Cout, int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw, int groups,
                       int E, int Mw, const int32_t *bA, const int32_t *bW, const int32_t *bR, const int32_t *table,
                       uint32_t flags, const float *bn, int act, float act_lo, float act_hi, void *workspace,
                       size_t workspace_bytes, fp8a_stream_t stream) {
    return conv2d_impl(x, w, y, Bn, Cin, H, W, Cout, kh, kw, sh, sw, ph, pw, dh, dw, groups, E, Mw, bA, bW, bR, table,
                       flags, bn, act, act_lo, act_hi, workspace, workspace_bytes, (hipStream_t)stream, FqIn{}, nullptr,
                       nullptr, nullptr);
}

size_t fp8a_conv2d_qin_workspace_size(int64_t Bn, int64_t Cin, int64_t H, int64_t W, int64_t Cout, int kh, int kw,
                                      int sh, int sw, int ph, int pw, int dh, int dw, int groups) {
    const size_t n = fp8a_conv2d_workspace_size(Bn, Cin, H, W, Cout, kh, kw, sh, sw, ph, pw, dh, dw, groups);
    return n == 0 ? 0 : align256(n) + align256((size_t)(Bn * Cin * H * W) * sizeof(float));
}

int fp8a_conv2d_qin(const float *x, const float *w, float *y, int64_t Bn, int64_t Cin, int64_t H, int64_t W,
                    int64_t Cout, int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw, int groups, int E,
                    int Mw, const int32_t *bW, const int32_t *bR, const int32_t *table, uint32_t flags,
                    const float *bn, int act, float act_lo, float act_hi, const float *in_maxval, int in_nbits,
                    int in_mbits, int in_sign_bits, float *in_bias_out, int32_t *in_ibias_out, void *workspace,
                    size_t workspace_bytes, fp8a_stream_t stream) {
    if (!in_maxval || !in_bias_out || !in_ibias_out) return fail(FP8A_EINVAL, "null pointer");
    const int qE = in_nbits - in_sign_bits - in_mbits;
    if (in_mbits < 1 || qE < 1) return fail(FP8A_EFORMAT, "bad FP8 quantizer format");
    const size_t xq_bytes = align256((size_t)(Bn * Cin * H * W) * sizeof(float));
    if (workspace == nullptr || workspace_bytes < FLAG_BYTES + xq_bytes)
        return fail(FP8A_EINVAL, "conv2d_qin workspace too small");
    // the fake-quant buffer of the non-fused paths sits at the workspace's end
    const size_t rest = (workspace_bytes - xq_bytes) & ~(size_t)255;
    float *xq = (float *)((char *)workspace + rest);
    return conv2d_impl(x, w, y, Bn, Cin, H, W, Cout, kh, kw, sh, sw, ph, pw, dh, dw, groups, E, Mw, nullptr, bW, bR,
                       table, flags, bn, act, act_lo, act_hi, workspace, rest, (hipStream_t)stream,
                       FqIn{in_maxval, qE, in_mbits, in_sign_bits}, in_bias_out, in_ibias_out, xq);
}


size_t fp8a_conv2d_block_workspace_size(int64_t Bn, int64_t Cin, int64_t H, int64_t W, int64_t Cout, int kh,
                                        int kw, int sh, int sw, int ph, int pw, int dh, int dw, int groups) {
    return fp8a_conv2d_qin_workspace_size(Bn, Cin, H, W, Cout, kh, kw, sh, sw, ph, pw, dh, dw, groups);
}

int fp8a_conv2d_block(const float *x, const float *w, float *y, int64_t Bn, int64_t Cin, int64_t H, int64_t W,
                      int64_t Cout, int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw, int groups, int E,
                      int Mw, const int32_t *bA, const int32_t *bW, const int32_t *bR, const int32_t *table,
                      uint32_t flags, const float *bn, int act, float act_lo, float act_hi, const float *in_maxval,
                      int in_nbits, int in_mbits, int in_sign_bits, float *in_bias_out, int32_t *in_ibias_out,
                      const float *res, int post_act, float post_lo, float post_hi, const float *out_maxval,
                      int out_nbits, int out_mbits, int out_sign_bits, float *out_bias_out, int32_t *out_ibias_out,
                      void *workspace, size_t workspace_bytes, fp8a_stream_t stream) {
    hipStream_t s = (hipStream_t)stream;
    if (post_act != 0 && post_act != 1) return fail(FP8A_EINVAL, "conv2d_block: post_act is 0 or 1");
    FqIn fin{}, fout{};
    if (in_maxval) {
        const int qE = in_nbits - in_sign_bits - in_mbits;
        if (in_mbits < 1 || qE < 1) return fail(FP8A_EFORMAT, "bad FP8 quantizer format");
        if (!in_bias_out || !in_ibias_out) return fail(FP8A_EINVAL, "null pointer");
        fin = FqIn{in_maxval, qE, in_mbits, in_sign_bits};
    } else if (!bA) {
        return fail(FP8A_EINVAL, "null pointer");
    }
    if (out_maxval) {
        const int qE = out_nbits - out_sign_bits - out_mbits;
        if (out_mbits < 1 || qE < 1) return fail(FP8A_EFORMAT, "bad FP8 quantizer format");
        if (!out_bias_out || !out_ibias_out) return fail(FP8A_EINVAL, "null pointer");
        fout = FqIn{out_maxval, qE, out_mbits, out_sign_bits};  // (its bias: written by the launch's gated exact kernel)
    }
    const size_t xq_bytes = fin.mx ? align256((size_t)(Bn * Cin * H * W) * sizeof(float)) : 0;
    if (workspace == nullptr || workspace_bytes < FLAG_BYTES + xq_bytes)
        return fail(FP8A_EINVAL, "conv2d_block workspace too small");
    const size_t rest = (workspace_bytes - xq_bytes) & ~(size_t)255;
    float *xq = fin.mx ? (float *)((char *)workspace + rest) : nullptr;
    return conv2d_impl(x, w, y, Bn, Cin, H, W, Cout, kh, kw, sh, sw, ph, pw, dh, dw, groups, E, Mw,
                       fin.mx ? nullptr : bA, bW, bR, table, flags, bn, act, act_lo, act_hi, workspace, rest, s, fin,
                       in_bias_out, in_ibias_out, xq, res, post_act, post_lo, post_hi, fout, nullptr, EmitW{},
                       fout.mx ? out_bias_out : nullptr, fout.mx ? out_ibias_out : nullptr);
}

// ----------------------------------------------------------------------------- word-image chain
// A convolution's input as the zero-bordered word image of gemm_f8mx_kernel (xm_decode_a's
// layout: [Bn][C][H + 2 ph][W'] with the left border widened for 16-B interior rows), behind a
// 256-B header whose first word is the "invalid" flag (fp8a_conv2d_chain).
size_t fp8a_word_image_bytes(int64_t Bn, int64_t C, int64_t H, int64_t W, int ph, int pw) {
    if (Bn <= 0 || C <= 0 || H <= 0 || W <= 0 || ph < 0 || pw < 0) return 0;
    const WordImage wi = word_image(H, W, ph, pw);
    return FLAG_BYTES + align256((size_t)(Bn * C * wi.H * wi.W) * 4);
}

// The emitting launch's header: [0] valid, [1] the next quantizer's maxval, [2] its float bias,
// [3] its 2^(1 - bias) bit pattern (the grid's min normal), [4] the next convolution's bR.
__global__ void emit_prep_kernel(uint32_t *hdr, FqIn fq, const int32_t *bR) {
    const float mx = *fq.mx, fb = fq_bias(mx, fq.E, fq.M);
    hdr[0] = 0u;
    hdr[1] = __float_as_uint(mx);
    hdr[2] = __float_as_uint(fb);
    hdr[3] = (uint32_t)(128 - (int)fb) << 23;
    hdr[4] = (uint32_t)*bR;
    hdr[5] = 0u;  // 255 - the smallest scale exponent of the emitted nonzero words (wave_max_atomic)
}

__global__ void word_image_fill_kernel(uint32_t *img, int64_t words) {
    if (blockIdx.x == 0 && threadIdx.x < 64) img[threadIdx.x] = 0u;  // header: valid
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (int64_t)gridDim.x * blockDim.x)
        img[64 + i] = XM_ZERO_WORD;  // the word of a zero (the border stays so)
}

int fp8a_word_image_init(void *image, int64_t Bn, int64_t C, int64_t H, int64_t W, int ph, int pw,
                         fp8a_stream_t stream) {
    if (image == nullptr || fp8a_word_image_bytes(Bn, C, H, W, ph, pw) == 0) return fail(FP8A_EINVAL, "word image");
    if (((uintptr_t)image & 255) != 0) return fail(FP8A_EINVAL, "word image must be 256-byte aligned");
    const WordImage wi = word_image(H, W, ph, pw);
    const int64_t words = Bn * C * wi.H * wi.W;
    word_image_fill_kernel<<<(unsigned)std::min<int64_t>((words + 255) / 256, 8192), 256, 0, (hipStream_t)stream>>>(
        (uint32_t *)image, words);
    return hip_check("fp8a word image init");
}

// Whether a convolution would read an in_image (fp8a_conv2d_chain): the matrix-core path with its A
// pre-pass (not the fp32-staging form of 1x1 convolutions with few column tiles, not the tile-table
// or VALU kernels), ungrouped, more than one output channel, a fused input quantizer.
int fp8a_conv2d_wants_image(int64_t Cout, int kh, int kw, int ph, int pw, int groups, int E, int Mw,
                            const int32_t *table, uint32_t flags, int sh, int sw, int dh, int dw) {
    if (Cout <= 1 || check_format(E, Mw) != FP8A_OK) return 0;
    TablePack tp;
    int mode;
    if (pack_table(table, Mw, (flags & F_APPROX) != 0, tp, mode) != FP8A_OK) return 0;
    if (groups > 1 && Cout == groups) {  // single-output-channel groups: the table form's words
        // opt-in (FP8A_CHAIN_TBX=1): measured on MobileNetV2 E4M3 the producers' emitting stores cost
        // 1.65 ms per forward for 0.85 ms of gated pre-passes saved (19708 -> 19036 images/s)
        static const bool no_tbx = getenv("FP8A_NO_TBX") != nullptr;
        static const bool chain_tbx = getenv("FP8A_CHAIN_TBX") != nullptr && atoi(getenv("FP8A_CHAIN_TBX")) != 0;
        const bool tbx = chain_tbx && !no_tbx && ((E == 4 && Mw == 3) || (E == 5 && Mw == 2)) &&
                         (mode == TM_NONE || mode == TM_W1U) && (flags & F_S2N) && (flags & F_QBMA) &&
                         !(flags & (F_GCLIP | F_V5)) && kw == 3 && dw == 1 && sh == sw && (sw == 1 || sw == 2);
        (void)kh; (void)dh;
        return tbx ? 2 : 0;
    }
    if (groups != 1 || no_mx()) return 0;
    // the v5 matrix-core form (gemm_v5mx_kernel): its words (v5_word_a) when unpadded (an image's
    // border holds the E4M3 / E5M2 form's zero word, fp8a_word_image_init); emitted by the staged
    // v5 depthwise kernel only (conv_v5ds_kernel) -- every other producer flags the image invalid
    if (flags & F_V5) return (v5mx_form(Mw, flags, TM_V5) && ph == 0 && pw == 0) ? 3 : 0;
    if (!f8_form(E, Mw, flags & ~F_TB, mode)) return 0;
    if (kh == 1 && kw == 1 && ph == 0 && pw == 0) {  // xm_af32: fp32 staging up to af32_maxct column tiles
        const int64_t bnt = 16 * xm_ncg(Cout), ct = (Cout + bnt - 1) / bnt;
        if (ct <= af32_maxct(sh, sw)) return 0;
    }
    return 1;
}

int fp8a_conv2d_chain(const float *x, const float *w, float *y, int64_t Bn, int64_t Cin, int64_t H, int64_t W,
                      int64_t Cout, int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw, int groups, int E,
                      int Mw, const int32_t *bA, const int32_t *bW, const int32_t *bR, const int32_t *table,
                      uint32_t flags, const float *bn, int act, float act_lo, float act_hi, const float *in_maxval,
                      int in_nbits, int in_mbits, int in_sign_bits, float *in_bias_out, int32_t *in_ibias_out,
                      const float *res, int post_act, float post_lo, float post_hi, const float *out_maxval,
                      int out_nbits, int out_mbits, int out_sign_bits, float *out_bias_out, int32_t *out_ibias_out,
                      void *in_image, void *out_image, int next_ph, int next_pw, const float *next_maxval,
                      int next_nbits, int next_mbits, int next_sign_bits, const int32_t *next_bR, int next_Mw,
                      int next_form, void *workspace, size_t workspace_bytes, fp8a_stream_t stream) {
    if (post_act != 0 && post_act != 1) return fail(FP8A_EINVAL, "conv2d_chain: post_act is 0 or 1");
    hipStream_t s = (hipStream_t)stream;
    if ((in_image && ((uintptr_t)in_image & 255)) || (out_image && ((uintptr_t)out_image & 255)))
        return fail(FP8A_EINVAL, "word images must be 256-byte aligned");
    FqIn fin{}, fout{};
    if (in_maxval) {
        const int qE = in_nbits - in_sign_bits - in_mbits;
        if (in_mbits < 1 || qE < 1) return fail(FP8A_EFORMAT, "bad FP8 quantizer format");
        if (!in_bias_out || !in_ibias_out) return fail(FP8A_EINVAL, "null pointer");
        fin = FqIn{in_maxval, qE, in_mbits, in_sign_bits};
    } else if (!bA) {
        return fail(FP8A_EINVAL, "null pointer");
    }
    if (out_maxval) {
        const int qE = out_nbits - out_sign_bits - out_mbits;
        if (out_mbits < 1 || qE < 1) return fail(FP8A_EFORMAT, "bad FP8 quantizer format");
        if (!out_bias_out || !out_ibias_out) return fail(FP8A_EINVAL, "null pointer");
        fout = FqIn{out_maxval, qE, out_mbits, out_sign_bits};  // (its bias: written by the launch's gated exact kernel)
    }
    EmitW em{};
    if (out_image) {
        const int64_t Ho = (H + 2 * ph - dh * (kh - 1) - 1) / sh + 1, Wo = (W + 2 * pw - dw * (kw - 1) - 1) / sw + 1;
        const int qE = next_nbits - next_sign_bits - next_mbits;
        if (!next_maxval || !next_bR || next_mbits < 1 || qE < 1 || !(next_Mw == 2 || next_Mw == 3) || next_ph < 0 ||
            next_pw < 0)
            return fail(FP8A_EINVAL, "bad next-convolution parameters for the word image");
        if (next_form < 0 || next_form > 2) return fail(FP8A_EINVAL, "bad word image form");
        // (the table form's words: the consumer's plain [Bn][C][Ho][Wo] layout, no border)
        const WordImage wi = next_form == 1 ? word_image(Ho, Wo, 0, 0) : word_image(Ho, Wo, next_ph, next_pw);
        // (form 2, v5 words: the staged v5 depthwise producer -- conv2d_impl flags the image invalid
        // where that kernel does not run; form 0 / 1: ungrouped producers)
        // (form 0 from a depthwise producer: the staged table-form kernel, round 6)
        const bool dwp = groups > 1 && Cin == groups && Cout == groups;
        const bool prod = next_form == 2 ? (flags & F_V5) && dwp
                                         : groups == 1 || (next_form == 0 && dwp && !(flags & F_V5));
        const bool can = prod && Cout > 1 && Ho > 0 && Wo > 0 && Bn * Cout * Ho * Wo < (1ll << 31) &&
                         Bn * Cout * wi.H * wi.W < (1ll << 30);
        // the header: valid (0) with the next quantizer's constants before this launch emits,
        // invalid (nonzero) when it cannot emit
        if (!can && dev_fill(out_image, 1, sizeof(uint32_t), s) != hipSuccess)
            return hip_check("fp8a word image header");
        if (can) {
            emit_prep_kernel<<<1, 1, 0, s>>>((uint32_t *)out_image, FqIn{next_maxval, qE, next_mbits, next_sign_bits},
                                             next_bR);
            em.w = (uint32_t *)out_image + 64;
            em.invalid = (uint32_t *)out_image;
            em.awH = (int)wi.H; em.awW = (int)wi.W; em.awph = wi.ph; em.awpw = wi.pw;
            em.Wo = (int)Wo;
            em.hw = (uint32_t)(Ho * Wo);
            fastdiv_params(em.hw, em.hw_mul, em.hw_shift);
            fastdiv_params((uint32_t)Wo, em.wo_mul, em.wo_shift);
            em.fq = FqIn{next_maxval, qE, next_mbits, next_sign_bits};
            em.bR = next_bR;
            em.Mw = next_Mw;
            em.form = next_form;
        }
    }
    const size_t xq_bytes = fin.mx ? align256((size_t)(Bn * Cin * H * W) * sizeof(float)) : 0;
    if (workspace == nullptr || workspace_bytes < FLAG_BYTES + xq_bytes)
        return fail(FP8A_EINVAL, "conv2d_chain workspace too small");
    const size_t rest = (workspace_bytes - xq_bytes) & ~(size_t)255;
    float *xq = fin.mx ? (float *)((char *)workspace + rest) : nullptr;
    return conv2d_impl(x, w, y, Bn, Cin, H, W, Cout, kh, kw, sh, sw, ph, pw, dh, dw, groups, E, Mw,
                       fin.mx ? nullptr : bA, bW, bR, table, flags, bn, act, act_lo, act_hi, workspace, rest, s, fin,
                       in_bias_out, in_ibias_out, xq, res, post_act, post_lo, post_hi, fout,
                       (const uint32_t *)in_image, em, fout.mx ? out_bias_out : nullptr, fout.mx ? out_ibias_out : nullptr);
}

size_t fp8a_matmul_block_workspace_size(int64_t M, int64_t N, int64_t K) {
    const size_t n = fp8a_matmul_workspace_size_mnk(M, N, K);
    return n == 0 ? 0 : align256(n) + align256((size_t)(M * K) * sizeof(float));
}

// A linear layer with its neighbours fused (QCustomLinearTorch.run_forward + the callers'
// elementwise tails, vit_quantized_approx.py:117-156): C = fq_out(clamp(bn_act(fq_in(A) @ B) + res)).
// Same contract as fp8a_conv2d_block with the row-major matrix operands of fp8a_matmul; with
// in_maxval, A must be dense (lda == K).
int fp8a_matmul_block(const float *A, int64_t lda, const float *B, int64_t sbk, int64_t sbn, float *C, int64_t ldc,
                      int64_t M, int64_t N, int64_t K, int E, int Mw, const int32_t *bA, const int32_t *bB,
                      int64_t bB_stride, const int32_t *bR, const int32_t *table, uint32_t flags, const float *bn,
                      int act, float act_lo, float act_hi, const float *in_maxval, int in_nbits, int in_mbits,
                      int in_sign_bits, float *in_bias_out, int32_t *in_ibias_out, const float *res, int post_act,
                      float post_lo, float post_hi, const float *out_maxval, int out_nbits, int out_mbits,
                      int out_sign_bits, float *out_bias_out, int32_t *out_ibias_out, void *workspace,
                      size_t workspace_bytes, fp8a_stream_t stream) {
    hipStream_t s = (hipStream_t)stream;
    if (lda < K || ldc < N) return fail(FP8A_EINVAL, "leading dimension smaller than extent");
    if (flags & (F_TB | F_V5)) return fail(FP8A_EINVAL, "matmul_block: int-bias v9 path only");
    if (post_act < 0 || post_act > 2) return fail(FP8A_EINVAL, "matmul_block: post_act is 0, 1 or 2");
    if (bn && (((uintptr_t)bn) & 7) != 0) return fail(FP8A_EINVAL, "bn parameters must be 8-byte aligned");
    if (res && (res == C || (((uintptr_t)res) & 15) != 0))
        return fail(FP8A_EINVAL, "the residual must be a 16-byte aligned tensor other than the output");
    FqIn fin{}, fout{};
    if (in_maxval) {
        const int qE = in_nbits - in_sign_bits - in_mbits;
        if (in_mbits < 1 || qE < 1) return fail(FP8A_EFORMAT, "bad FP8 quantizer format");
        if (!in_bias_out || !in_ibias_out) return fail(FP8A_EINVAL, "null pointer");
        if (lda != K) return fail(FP8A_EINVAL, "matmul_block: fused input quantization needs a dense A");
        fin = FqIn{in_maxval, qE, in_mbits, in_sign_bits};
    } else if (!bA) {
        return fail(FP8A_EINVAL, "null pointer");
    }
    if (out_maxval) {
        const int qE = out_nbits - out_sign_bits - out_mbits;
        if (out_mbits < 1 || qE < 1) return fail(FP8A_EFORMAT, "bad FP8 quantizer format");
        if (!out_bias_out || !out_ibias_out) return fail(FP8A_EINVAL, "null pointer");
        fout = FqIn{out_maxval, qE, out_mbits, out_sign_bits};  // (its bias: written by the launch's gated exact kernel)
    }
    const size_t xq_bytes = fin.mx ? align256((size_t)(M * K) * sizeof(float)) : 0;
    if (workspace == nullptr || workspace_bytes < FLAG_BYTES + xq_bytes)
        return fail(FP8A_EINVAL, "matmul_block workspace too small");
    const size_t rest = (workspace_bytes - xq_bytes) & ~(size_t)255;
    GemmArgs a = make_args(A, lda, B, sbk, sbn, C, ldc, M, N, K, E, Mw, fin.mx ? in_ibias_out : bA, bB, bB_stride, bR,
                           flags);
    a.ep = reinterpret_cast<const float2 *>(bn); a.ep_act = act; a.ep_lo = act_lo; a.ep_hi = act_hi;
    a.res = res; a.post_act = post_act; a.post_lo = post_lo; a.post_hi = post_hi; a.post_fq = fout;
    if (fout.mx) {
        a.post_bout = out_bias_out;
        a.post_ibout = out_ibias_out;
    }
    if (fin.mx && M > 0 && K > 0) {
        // fuse into the matrix-core pre-decode only where run_gemm will take that path (as conv2d_impl)
        TablePack tp;
        int mode;
        int rc = check_format(E, Mw);
        if (rc) return rc;
        rc = pack_table(table, Mw, (flags & F_APPROX) != 0, tp, mode);
        if (rc) return rc;
        const int64_t kpad = (K + BK - 1) / BK * BK, npad = (N + BN - 1) / BN * BN, a_words = M * kpad;
        const bool fused = f8_form(E, Mw, flags, mode) && !no_mx() && a_words < (1ll << 30) &&
                           kpad * npad * 4 < (1ll << 32) && rest >= gemm_workspace_bytes(M, N, K, 0);
        if (fused) {
            a.fqin = fin;
            a.fq_bias = in_bias_out;
            a.fq_ibias = in_ibias_out;  // written by the A pre-decode before any kernel reads it
        } else {  // one fake-quant pass into the workspace's end, then the plain path on it
            float *xq = (float *)((char *)workspace + rest);
            const int64_t nx = M * K;
            fp8_quantize_kernel<<<(unsigned)std::max<int64_t>(1, std::min<int64_t>((nx + 255) / 256, 65536)), 256, 0,
                                  s>>>(A, 1, nx, fin.mx, 0, fin.E, fin.M, fin.S, xq, in_bias_out, in_ibias_out);
            rc = hip_check("fp8a input fake-quant");
            if (rc) return rc;
            a.A = xq;
        }
    } else if (fin.mx) {  // empty product: the quantizer's bias is still set, as its forward would
        fq_bias_kernel<<<1, 1, 0, s>>>(fin, in_bias_out, in_ibias_out);
        int rc = hip_check("fp8a input-quantizer bias");
        if (rc) return rc;
    }
    return run_gemm(a, table, workspace, rest, s);
}

int fp8a_max_pool2d(const float *x, float *y, int64_t Bn, int64_t C, int64_t H, int64_t W, int kh, int kw, int sh,
                    int sw, int ph, int pw, fp8a_stream_t stream) {
    if (!x || !y) return fail(FP8A_EINVAL, "null pointer");
    if (kh < 1 || kw < 1 || sh < 1 || sw < 1 || ph < 0 || pw < 0 || 2 * ph > kh || 2 * pw > kw)
        return fail(FP8A_EINVAL, "bad pooling window");
    const int64_t Ho = (H + 2 * ph - kh) / sh + 1, Wo = (W + 2 * pw - kw) / sw + 1;
    if (Ho <= 0 || Wo <= 0) return fail(FP8A_EINVAL, "empty pooling output");
    const int64_t total = Bn * C * Ho * Wo;
    if (total == 0) return FP8A_OK;
    if (kh == 3 && kw == 3 && sh == 2 && sw == 2 && ph == 1 && pw == 1 && W % 8 == 0 && H * W < (1ll << 31) &&
        ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0) {
        const int64_t groups = Bn * C * Ho * (W / 8);
        max_pool2d_s2k3_kernel<<<(unsigned)std::min<int64_t>((groups + 255) / 256, 65536), 256, 0, (hipStream_t)stream>>>(
            x, y, Bn * C, (int)H, (int)W, (int)Ho);
        return hip_check("fp8a_max_pool2d");
    }
    max_pool2d_kernel<<<(unsigned)std::min<int64_t>((total + 255) / 256, 65536), 256, 0, (hipStream_t)stream>>>(
        x, y, Bn * C, (int)H, (int)W, (int)Ho, (int)Wo, kh, kw, sh, sw, ph, pw);
    return hip_check("fp8a_max_pool2d");
}

int fp8a_avg_pool2d_plane(const float *x, float *y, int64_t Bn, int64_t C, int64_t H, int64_t W, int kh, int kw,
                          int sh, int sw, fp8a_stream_t stream) {
    if (kh < 1 || kw < 1 || sh < 1 || sw < 1 || kh > H || kw > W || H - kh >= sh || W - kw >= sw)
        return fail(FP8A_EINVAL, "not a one-output-per-plane pooling window");
    if (H * W > 4096) return fail(FP8A_EINVAL, "plane over 4096 values");
    const int64_t planes = Bn * C;
    if (planes == 0) return FP8A_OK;
    if (!x || !y) return fail(FP8A_EINVAL, "null pointer");
    const int hw = (int)(H * W), ps = hw | 1, pb = std::min(128, 8192 / ps);
    avg_pool_plane_kernel<<<(unsigned)((planes + pb - 1) / pb), 128, (size_t)pb * ps * 4, (hipStream_t)stream>>>(
        x, y, planes, pb, (int)W, hw, ps, kh, kw, 1.0f / hw);
    return hip_check("fp8a_avg_pool2d_plane");
}

int fp8a_matmul_qamaa(const float *A, int64_t lda, const float *B, int64_t sbk, int64_t sbn, float *C, int64_t M,
                      int64_t N, int64_t K, const float *maxval, int n_bits, int Mbits, int sign_bits,
                      fp8a_stream_t stream) {
    if (lda < K) return fail(FP8A_EINVAL, "leading dimension smaller than extent");
    if (!A || !B || !C || !maxval) return fail(FP8A_EINVAL, "null pointer");
    GemmArgs a = make_args(A, lda, B, sbk, sbn, C, N, M, N, K, 1, 1, nullptr, nullptr, 0, nullptr, 0);
    a.qmax = maxval;
    a.qM = Mbits;
    a.qE = n_bits - sign_bits - Mbits;
    a.qsign = sign_bits;
    int rc = run_qamaa(a, (hipStream_t)stream);
    if (rc) return rc;
    return fp8a_fp8_quantize(C, 1, M * N, maxval, 0, n_bits, Mbits, sign_bits, C, nullptr, nullptr, stream);
}

int fp8a_conv2d_qamaa(const float *x, const float *w, float *y, int64_t Bn, int64_t Cin, int64_t H, int64_t W,
                      int64_t Cout, int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw, int groups,
                      const float *maxval, int n_bits, int Mbits, int sign_bits, fp8a_stream_t stream) {
    hipStream_t s = (hipStream_t)stream;
    if (groups <= 0 || Cout % groups != 0 || Cin % groups != 0) return fail(FP8A_EINVAL, "bad groups");
    if (Cout / groups == 1)
        return fail(FP8A_EINVAL, "single-output-channel groups take the exact product in the reference "
                                 "(approx_calculation.py:810-811): not a qamaa launch");
    const int64_t Ho = (H + 2 * ph - dh * (kh - 1) - 1) / sh + 1;
    const int64_t Wo = (W + 2 * pw - dw * (kw - 1) - 1) / sw + 1;
    if (Ho <= 0 || Wo <= 0) return fail(FP8A_EINVAL, "empty convolution output");
    const int64_t cog = Cout / groups, cig = Cin / groups, Kg = cig * kh * kw, Mrows = Bn * Ho * Wo;
    for (int g = 0; g < groups; ++g) {
        GemmArgs a = make_args(nullptr, 0, w + g * cog * Kg, 1, Kg, y, 0, Mrows, cog, Kg, 1, 1, nullptr, nullptr, 0,
                               nullptr, 0);
        a.nchw = 1; a.hw = Ho * Wo; a.ctot = Cout; a.coff = g * cog;
        a.conv = 1; a.X = x;
        a.Cin = Cin; a.H = H; a.W = W; a.Ho = Ho; a.Wo = Wo; a.cbase = g * cig;
        a.kh = kh; a.kw = kw; a.sh = sh; a.sw = sw; a.ph = ph; a.pw = pw; a.dh = dh; a.dw = dw;
        fastdiv_params((uint32_t)(kh * kw), a.kk_mul, a.kk_shift);
        fastdiv_params((uint32_t)kw, a.kw_mul, a.kw_shift);
        a.qmax = maxval; a.qM = Mbits; a.qE = n_bits - sign_bits - Mbits; a.qsign = sign_bits;
        int rc = run_qamaa(a, s);
        if (rc) return rc;
    }
    return fp8a_fp8_quantize(y, 1, Bn * Cout * Ho * Wo, maxval, 0, n_bits, Mbits, sign_bits, y, nullptr, nullptr,
                             stream);
}

int fp8a_fp8_quantize(const float *x, int64_t rows, int64_t inner, const float *maxval, int per_row, int n_bits,
                      int Mbits, int sign_bits, float *out, float *bias_out, int32_t *ibias_out,
                      fp8a_stream_t stream) {
    const int E = n_bits - sign_bits - Mbits;
    if (Mbits < 1 || E < 1) return fail(FP8A_EFORMAT, "bad FP8 quantizer format");
    const int64_t total = rows * inner;
    if (total <= 0) return FP8A_OK;
    const int64_t blocks = std::min<int64_t>((total + 255) / 256, 65536);
    fp8_quantize_kernel<<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(x, rows, inner, maxval, per_row, E,
                                                                           Mbits, sign_bits, out, bias_out, ibias_out);
    return hip_check("fp8a_fp8_quantize");
}

// The config-1 layer (approx_flag off) in one launch family: fq_in on the loaded input, the exact
// product (groups = 1: run_dense, the matrix core; groups > 1: dn_group_conv), and per output
// rq -> eval batch norm -> clamp -> fq_out in the store (gemm_dense.h DnFuse).  Each quantizer
// writes its bias (the reference quantizer's custom_bias) like fp8a_conv2d_qin.
static int fused_quantizer(const float *mx, int nbits, int mbits, int sign_bits, float *bias_out, int32_t *ibias_out,
                           FqIn &f) {
    f = FqIn{};
    if (!mx) return FP8A_OK;
    const int qE = nbits - sign_bits - mbits;
    if (mbits < 1 || qE < 1) return fail(FP8A_EFORMAT, "bad FP8 quantizer format");
    if (!bias_out || !ibias_out) return fail(FP8A_EINVAL, "null pointer");
    f = FqIn{mx, qE, mbits, sign_bits};
    return FP8A_OK;
}

int fp8a_dense_conv2d_fused(const float *x, const float *w, float *y, int64_t Bn, int64_t Cin, int64_t H, int64_t W,
                            int64_t Cout, int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw, int groups,
                            int fmt, const float *w_maxval, int w_per_channel, int w_nbits, int w_mbits,
                            int w_sign_bits, float *w_bias_out, int32_t *w_ibias_out, const float *in_maxval,
                            int in_nbits, int in_mbits, int in_sign_bits, float *in_bias_out, int32_t *in_ibias_out,
                            const float *res_maxval, int res_nbits, int res_mbits, int res_sign_bits,
                            float *res_bias_out, int32_t *res_ibias_out, const float *bn, int act, float act_lo,
                            float act_hi, const float *out_maxval, int out_nbits, int out_mbits, int out_sign_bits,
                            float *out_bias_out, int32_t *out_ibias_out, void *workspace, size_t workspace_bytes,
                            fp8a_stream_t stream) {
    hipStream_t s = (hipStream_t)stream;
    DnFuse fz{};
    int rc = fused_quantizer(w_maxval, w_nbits, w_mbits, w_sign_bits, w_bias_out, w_ibias_out, fz.wq);
    if (!rc) rc = fused_quantizer(in_maxval, in_nbits, in_mbits, in_sign_bits, in_bias_out, in_ibias_out, fz.qin);
    if (!rc) rc = fused_quantizer(res_maxval, res_nbits, res_mbits, res_sign_bits, res_bias_out, res_ibias_out, fz.rq);
    if (!rc) rc = fused_quantizer(out_maxval, out_nbits, out_mbits, out_sign_bits, out_bias_out, out_ibias_out, fz.oq);
    if (rc) return rc;
    fz.wq_row = w_maxval && w_per_channel ? 1 : 0;
    fz.bo[0] = in_bias_out; fz.ibo[0] = in_ibias_out;
    fz.bo[1] = res_bias_out; fz.ibo[1] = res_ibias_out;
    fz.bo[2] = out_bias_out; fz.ibo[2] = out_ibias_out;
    fz.bo[3] = w_bias_out; fz.ibo[3] = w_ibias_out;
    fz.ep = reinterpret_cast<const float2 *>(bn);
    fz.act = act;
    fz.lo = act_lo;
    fz.hi = act_hi;
    if (groups != 1)
        return grouped_conv_impl(x, w, y, Bn, Cin, H, W, Cout, groups, kh, kw, sh, sw, ph, pw, dh, dw, fz, s);
    if (kh < 1 || kw < 1 || sh < 1 || sw < 1 || dh < 1 || dw < 1 || ph < 0 || pw < 0 || Bn < 0 || Cin < 0 || Cout < 0)
        return fail(FP8A_EINVAL, "bad convolution geometry");
    const int64_t Ho = (H + 2 * ph - dh * (kh - 1) - 1) / sh + 1;
    const int64_t Wo = (W + 2 * pw - dw * (kw - 1) - 1) / sw + 1;
    if (Ho <= 0 || Wo <= 0) return fail(FP8A_EINVAL, "empty convolution output");
    DenseArgs a = dense_args();
    a.x = x; a.w = w; a.y = y; a.conv = 1;
    a.C = Cin; a.H = H; a.W = W; a.Ho = Ho; a.Wo = Wo;
    a.kh = kh; a.kw = kw; a.sh = sh; a.sw = sw; a.ph = ph; a.pw = pw; a.dh = dh; a.dw = dw;
    a.M = Bn * Ho * Wo; a.N = Cout; a.K = Cin * kh * kw;
    a.sbk = 1; a.sbn = a.K;
    a.ldc = Cout; a.fmt = fmt;
    a.fz = fz;
    return run_dense(a, workspace, workspace_bytes, s);
}

}  // extern "C"
