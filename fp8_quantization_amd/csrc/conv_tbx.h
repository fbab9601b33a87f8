// conv_tbx.h -- E4M3 depthwise (single-output-channel groups) with the tensor-bias semantics,
// table form.
//
// The reference takes single-column products down its tensor-bias path (approx_calculation.py:
// 800-809): with int32-tensor biases >= 2, param_prepare's integer powers make
// min_norm 0, so every nonzero value decodes at its own binade and Q_R rounds at the value's own
// binade (no subnormal floor).  Rounding is then scale-invariant, so for on-grid E4M3 operands
// with s2n, per-product quantization, no golden clip and a {0,1} (or zero) error table the term
// is a TABLE value times the operands' binades:
//     r = L(m_a, m_b) * c_a * c_b,   L = Q3c(sig_a sig_b - T[m_a][m_b] / 8)
// (Q3c: round to 3 mantissa bits at V's own binade with Q_R's saturating clamp, F6), followed by
// the two quirks the general kernel (conv_tb_fast_kernel) applies per term:
//   * the binade [2^-bR, 2^(1-bR)) has expo field 0 and decodes as 2^(1-bR) m / 8, i.e.
//     r -> 2 r - sign 2^(1-bR) there;
//   * F7: the sign comes from Q_R(g), g = a b, which is 0 only for |g| in [2^-bR, 2^-bR 17/16];
//     a negative such g gives |r|.  |g| = u |c_a c_b| with u = sig_a sig_b, so F7 fires only for
//     c_a c_b = -2^-bR with u <= 17/16 or c_a c_b = -2^(-1-bR) with u in [2, 17/8]: the table
//     carries that trigger value per (m_a, m_b) beside L.
// Per term that is an LDS read, two multiplies and two compare-selects (~13 VALU ops against
// ~30 for the general form).  A is pre-decoded once per launch into words (sign/exponent bits of
// a | m_a << 3, so the table byte offset is one v_and_or with m_b << 6); each thread computes 4
// consecutive outputs of one row and gathers the input words they share once.  Off-grid inputs,
// the exactness window and the bias window raise the gate word and conv_tb_direct_kernel
// recomputes the launch exactly (as behind conv_tb_fast_kernel).
#pragma once
#include "fp8approx_common.h"
#include "gemm_dense.h"
#include "gemm_f8mx.h"

namespace fp8a {
constexpr int TBX_TW = 4;  // outputs per thread along wo

struct TbxArgs {
    int64_t Cin, H, W, Cout, Ho, Wo;
    int kh, ph, pw, dh, cpg;
    uint32_t nwg, items;  // column groups per row, Bn * Cout * Ho * nwg
};

__device__ __forceinline__ uint32_t tbx_word(float v, const FqIn &fq, float fmx, float fbias, uint32_t lowm,
                                             uint32_t mmask, int M, bool &bad) {
    if (fq.mx) v = fq_apply(v, fmx, fbias, fq.M, fq.S);
    const uint32_t u = __float_as_uint(v), ua = u & 0x7FFFFFFFu;
    bad |= (ua != 0u) && ((ua & lowm) != 0u || ua < 0x20800000u || ua > 0x58800000u);
    return ua == 0u ? 0u : ((u & 0xFF800000u) | (((ua >> (23 - M)) & mmask) << 3));
}

// x (NCHW floats) -> words: (bits(x) & 0xFF800000) | (m << 3); 0 for zeros; gate on off-grid
// values / the exactness window (tensor-bias decode: every value at its own binade).
// With fused input quantization (fq.mx set) the values are fq(x) and the quantizer's bias is
// written to fq_bias / fq_ibias (the kernels' bA).
// img_hdr: the header of a word image the producing launch emitted into `out` (fp8a_conv2d_chain):
// nothing to decode unless it is flagged invalid (the quantizer's bias is still written).
__global__ __launch_bounds__(256) void tbx_decode_a(const float *x, int64_t n, uint32_t *out, uint32_t *gate,
                                                    FqIn fq, float *fq_bias_out, int32_t *fq_ibias_out, int M = 3,
                                                    const uint32_t *img_hdr = nullptr) {
    const uint32_t lowm = (1u << (23 - M)) - 1u, mmask = (1u << M) - 1u;  // below the grid's mantissa / its bits
    bool bad = false;
    const float fmx = fq.mx ? *fq.mx : 0.0f, fbias = fq.mx ? fq_bias(fmx, fq.E, fq.M) : 0.0f;
    if (fq.mx && blockIdx.x == 0 && threadIdx.x == 0) {
        *fq_bias_out = fbias;
        *fq_ibias_out = (int32_t)fbias;
    }
    if (img_hdr != nullptr && __hip_atomic_load(img_hdr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) return;
    auto word = [&](float v) { return tbx_word(v, fq, fmx, fbias, lowm, mmask, M, bad); };
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i0 = 0;
    if ((((uintptr_t)x | (uintptr_t)out) & 15) == 0) {  // 16-byte form over the n / 4 quads
        for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n / 4; q += stride) {
            const float4 v = reinterpret_cast<const float4 *>(x)[q];
            reinterpret_cast<uint4 *>(out)[q] = make_uint4(word(v.x), word(v.y), word(v.z), word(v.w));
        }
        i0 = n / 4 * 4;
    }
    for (int64_t i = i0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = word(x[i]);
    if (__syncthreads_or(bad ? 1 : 0) && threadIdx.x == 0) atomicOr(gate, 1u);
}

// The table entry (L, F7 trigger) for (m_b, m_a) = (i >> 3, i & 7) at result bias r_b (the
// derivation in the header; rows / columns past 2^M are unused).  Layout [m_b][m_a] (round 6; was
// [m_a][m_b]): a tap reads the 8 entries of its m_b, 8 B apart, so the lanes of a ds_read_b64
// group hit distinct banks (the [m_a][m_b] layout put m_a and m_a + 4 on one bank: 56 % of the
// kernel's LDS cycles were bank conflicts, profiles/r06_dw/).
template <int M>
__device__ __forceinline__ float2 tbx_lut_entry(int i, const TablePack &tab, int r_b) {
    constexpr float ULP = 1.0f / (1 << M);  // 2^-M
    const int mb = i >> 3, ma = i & 7;
    const int tv = (ma < (1 << M) && mb < (1 << M)) ? tab.raw[(ma << M) | mb] : 0;
    const float u = (1.0f + ULP * ma) * (1.0f + ULP * mb);  // exact
    const float v = __fmaf_rn(1.0f + ULP * ma, 1.0f + ULP * mb, -ULP * (float)tv);
    const float pe = __uint_as_float(__float_as_uint(v) & 0x7F800000u);
    const float xs = fminf(v, pe * (2.0f - ULP - p2(-22))), cc = pe * (float)(1 << (23 - M)) * 1.5f;
    const float L = (xs + cc) - cc;  // QMc(V'): RNE at V's binade after the saturating clamp
    uint32_t f7 = 0xFFFFFFFFu;       // never equal to a product of binades
    if (u <= 1.0f + 0.5f * ULP) f7 = 0x80000000u | ((uint32_t)(127 - r_b) << 23);
    else if (u >= 2.0f && u <= 2.0f + ULP) f7 = 0x80000000u | ((uint32_t)(126 - r_b) << 23);
    return make_float2(L, __uint_as_float(f7));
}

// One term of the table form: input word wa (m_a << 3 in its bits 3-5), the tap's c_b and m_b << 6,
// the table in LDS.
__device__ __forceinline__ float tbx_term(uint32_t wa, float cB, uint32_t mb64, const char *lut, uint32_t q0exp,
                                          float twoq) {
    // (mb64 masked: the offset is then provably small and the table's LDS base folds into the read's
    // offset field; the mask is per tap, the terms share it)
    const float2 e = *reinterpret_cast<const float2 *>(lut + ((wa & 0x38u) | (mb64 & 0x1C0u)));
    const float cab = __uint_as_float(wa & 0xFF800000u) * cB;  // exact
    float rv = e.x * cab;                                        // exact
    // expo field 0: 2 rv - sign 2^(1-bR), as sign x (2 |rv| - 2^(1-bR)) -- one fma with an abs
    // modifier and a bfi, where the signed form cost a bfi, an xor and the fma (round 6).  The same
    // value (RNE is odd-symmetric) but for |rv| = 2^-bR, rv < 0: -0 instead of +0, which no sum sees
    // (the accumulators start at +0 and are never -0)
    const float rs = copysignf(__fmaf_rn(2.0f, fabsf(rv), -twoq), rv);
    rv = ((__float_as_uint(rv) & 0x7F800000u) == q0exp) ? rs : rv;
    return (__float_as_uint(cab) == __float_as_uint(e.y)) ? fabsf(rv) : rv;  // F7
}

// M = 3 (E4M3) or 2 (E5M2, the same derivation with M-bit mantissas: L = QMc(sig_a sig_b - T / 2^M),
// saturating at 2 - 2^-M; F7 for u <= 1 + 2^-(M+1) or u in [2, 2 + 2^-M]); the table keeps the
// 8 x 8 layout (entry m_a * 8 + m_b) for both.
// RW = 2 (option "tbx_rw", the default for undilated rows): a thread computes the same 4 columns
// of two consecutive output rows; every input row of their union (kh + 1 rows at stride 1,
// kh + 2 at stride 2, against 2 kh for two threads) is gathered once and feeds both rows'
// accumulators, each still in (ky, kx) order -- bit-identical outputs, fewer and more independent
// loads per output (the one-row form waits on its loads 66 % of its cycles, §3f).
template <int SW, int M, int RW = 1>
__global__ __launch_bounds__(256) void conv_tbx_kernel(const uint32_t *aw, const float *w, float *y, TbxArgs t,
                                                       const int32_t *bA, const int32_t *bW, const int32_t *bR,
                                                       TablePack tab, uint32_t *gate, const float2 *ep, int ep_act,
                                                       float ep_lo, float ep_hi) {
    constexpr int KW = 3, NCOL = (TBX_TW - 1) * SW + KW;
    constexpr uint32_t LOWM = (1u << (23 - M)) - 1u, MMASK = (1u << M) - 1u;
    __shared__ float2 sL[64];
    const int a_b = *bA, r_b = *bR;
    bool bad = !(a_b >= 2 && a_b <= 120 && r_b >= 2 && r_b <= 120);
    if (threadIdx.x < 64) sL[threadIdx.x] = tbx_lut_entry<M>(threadIdx.x, tab, r_b);
    __syncthreads();
    const uint32_t q0exp = (uint32_t)(127 - r_b) << 23;
    const float twoq = __uint_as_float((uint32_t)(128 - r_b) << 23);
    const char *lut = reinterpret_cast<const char *>(sL);
    const int64_t HW = t.H * t.W;

    const uint32_t hog = ((uint32_t)t.Ho + RW - 1) / RW;  // row groups per plane
    for (uint32_t item = blockIdx.x * blockDim.x + threadIdx.x; item < t.items; item += gridDim.x * blockDim.x) {
        const uint32_t wg = item % t.nwg, r1 = item / t.nwg;
        const uint32_t ho0 = (r1 % hog) * RW, r2 = r1 / hog;
        const uint32_t co = r2 % (uint32_t)t.Cout, img = r2 / (uint32_t)t.Cout;
        const int wb = bW[co];
        bad |= !(wb >= 2 && wb <= 120);
        const int wo0 = (int)wg * TBX_TW, wi0 = wo0 * SW - t.pw;
        float acc[RW][TBX_TW];
#pragma unroll
        for (int j = 0; j < RW; ++j)
#pragma unroll
            for (int q = 0; q < TBX_TW; ++q) acc[j][q] = 0.0f;
        const int nr = RW == 1 ? t.kh : (RW - 1) * SW + t.kh;  // input rows (RW > 1: dh = 1)
        for (int c = 0; c < t.cpg; ++c) {
            const uint32_t *plane = aw + ((int64_t)img * t.Cin + (int64_t)co * t.cpg + c) * HW;
            const float *wk = w + ((int64_t)co * t.cpg + c) * t.kh * KW;
            for (int r = 0; r < nr; ++r) {
                const int hi = (int)ho0 * SW - t.ph + (RW == 1 ? r * t.dh : r);
                const bool rowok = (uint32_t)hi < (uint32_t)t.H;
                const uint32_t *row = plane + (int64_t)hi * t.W;
                uint32_t col[NCOL];
#pragma unroll
                for (int j = 0; j < NCOL; ++j) {
                    const int wi = wi0 + j;
                    col[j] = (rowok && (uint32_t)wi < (uint32_t)t.W) ? row[wi] : 0u;
                }
#pragma unroll
                for (int j = 0; j < RW; ++j) {
                    const int ky = r - j * SW;  // this input row's tap for output row ho0 + j
                    if (ky < 0 || ky >= t.kh) continue;
#pragma unroll
                    for (int kx = 0; kx < KW; ++kx) {
                        const uint32_t bw = __float_as_uint(wk[ky * KW + kx]), bwa = bw & 0x7FFFFFFFu;
                        bad |= (bwa != 0u) && ((bwa & LOWM) != 0u || bwa < 0x20800000u || bwa > 0x58800000u);
                        const float cB = __uint_as_float(bw & 0xFF800000u);
                        const uint32_t mb8 = ((bwa >> (23 - M)) & MMASK) << 6;  // (m_b << 6: the table row)
#pragma unroll
                        for (int q = 0; q < TBX_TW; ++q)
                            acc[j][q] += tbx_term(col[q * SW + kx], cB, mb8, lut, q0exp, twoq);
                    }
                }
            }
        }
#pragma unroll
        for (int j = 0; j < RW; ++j) {
            if (ho0 + j >= (uint32_t)t.Ho) break;
            float *yr = y + (((int64_t)img * t.Cout + co) * t.Ho + ho0 + j) * t.Wo;
#pragma unroll
            for (int q = 0; q < TBX_TW; ++q)
                if (wo0 + q < t.Wo) yr[wo0 + q] = epi(ep, ep_act, ep_lo, ep_hi, co, acc[j][q]);
        }
    }
    if (__syncthreads_or(bad ? 1 : 0) && threadIdx.x == 0) atomicOr(gate, 1u);
}

// conv_tbs_kernel: conv_tbx_kernel for the depthwise 3x3 (one input channel per output, dilation
// 1, stride S both ways) with tbx_decode_a fused in, staged through LDS (option "tbs", the
// default): the workgroup owns PB consecutive planes x RB output rows (as dn_dw3_kernel), loads
// the fp32 input window those rows read once with contiguous loads, applies the input quantizer
// and the word encoding into LDS (zero words for the padding), builds the table and the taps'
// (c_b, m_b) once, then thread = 4 consecutive outputs of a row: the window's words by 16-byte LDS
// reads (rows padded to a multiple of 4 words) and conv_tbx_kernel's terms in (ky, kx) order --
// the same bits, without the word image's write and read (8 B per input value) and the gathers'
// load latency.  The gate rules are the pre-pass's and the kernel's (values staged, taps, biases).
struct TbsArgs {
    int64_t planes;  // Bn x C
    int C, H, W, Ho, Wo, ph, pw;
    int PB, RB, nb, RS, WS, nq;  // planes / block, output rows / band, bands / plane, staged rows, row stride (words), quads / row
    float inv_c, inv_ws, inv_pst, inv_nq, inv_pq, inv_w, inv_hw;
};

template <int S, int M>
__global__ __launch_bounds__(256) void conv_tbs_kernel(const float *x, const float *w, float *y, const TbsArgs t, FqIn fq,
                                                       float *fq_bias_out, int32_t *fq_ibias_out, const int32_t *bA,
                                                       const int32_t *bW, const int32_t *bR, TablePack tab,
                                                       uint32_t *gate, const float2 *ep, int ep_act, float ep_lo,
                                                       float ep_hi) {
    constexpr int NCOL = (TBX_TW - 1) * S + 3;
    constexpr uint32_t LOWM = (1u << (23 - M)) - 1u, MMASK = (1u << M) - 1u;
    extern __shared__ uint4 tbs_sm[];
    uint32_t *sw = reinterpret_cast<uint32_t *>(tbs_sm);               // [PB][RS][WS] words
    float2 *sL = reinterpret_cast<float2 *>(sw + t.PB * t.RS * t.WS);  // the table
    uint2 *sB = reinterpret_cast<uint2 *>(sL + 64);                    // [PB][9] {c_b bits, m_b << 3}
    const int tid = threadIdx.x;
    const float fmx = fq.mx ? *fq.mx : 0.0f, fbias = fq.mx ? fq_bias(fmx, fq.E, fq.M) : 0.0f;
    if (fq.mx && blockIdx.x == 0 && tid == 0) {
        *fq_bias_out = fbias;
        *fq_ibias_out = (int32_t)fbias;
    }
    const int a_b = fq.mx ? (int32_t)fbias : *bA, r_b = *bR;
    bool bad = !(a_b >= 2 && a_b <= 120 && r_b >= 2 && r_b <= 120);
    if (tid < 64) sL[tid] = tbx_lut_entry<M>(tid, tab, r_b);
    const int band = (int)(blockIdx.x % (unsigned)t.nb);
    const int64_t P0 = (int64_t)(blockIdx.x / (unsigned)t.nb) * t.PB;
    const int npl = (int)min((int64_t)t.PB, t.planes - P0);
    const int oh0 = band * t.RB, nrow = min(t.RB, t.Ho - oh0), hi0 = oh0 * S - t.ph;
    const int pst = t.RS * t.WS, c0 = (int)(P0 % t.C);
    for (int d = tid; d < npl * 9; d += 256) {
        const int pl = d / 9;
        int c = c0 + pl;
        c -= dw_div(c, t.C, t.inv_c) * t.C;
        const int wb = bW[c];
        bad |= !(wb >= 2 && wb <= 120);
        const uint32_t bw = __float_as_uint(w[(int64_t)c * 9 + d - 9 * pl]), bwa = bw & 0x7FFFFFFFu;
        bad |= (bwa != 0u) && ((bwa & LOWM) != 0u || bwa < 0x20800000u || bwa > 0x58800000u);
        sB[d] = make_uint2(bw & 0xFF800000u, ((bwa >> (23 - M)) & MMASK) << 6);
    }
    dw_stage(x, P0, npl, t.H, t.W, hi0, t.pw, t.RS, t.WS, t.inv_w, t.inv_hw, t.RB == t.Ho, sw,
             [&](float v) { return tbx_word(v, fq, fmx, fbias, LOWM, MMASK, M, bad); });
    __syncthreads();
    const uint32_t q0exp = (uint32_t)(127 - r_b) << 23;
    const float twoq = __uint_as_float((uint32_t)(128 - r_b) << 23);
    const char *lut = reinterpret_cast<const char *>(sL);
    const int pq = t.RB * t.nq;
    for (int e = tid; e < npl * pq; e += 256) {
        const int pl = dw_div(e, pq, t.inv_pq), rem = e - pl * pq;
        const int orow = dw_div(rem, t.nq, t.inv_nq), q = rem - orow * t.nq;
        if (orow >= nrow) continue;
        const uint32_t *ws = sw + pl * pst + orow * S * t.WS + 4 * q * S;
        const uint2 *wb = sB + pl * 9;
        float acc[TBX_TW] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
            const uint32_t *wr = ws + ky * t.WS;
            uint32_t col[NCOL];
            const uint4 a0 = *reinterpret_cast<const uint4 *>(wr);
            col[0] = a0.x; col[1] = a0.y; col[2] = a0.z; col[3] = a0.w;
            if constexpr (S == 1) {
                const uint2 a1 = *reinterpret_cast<const uint2 *>(wr + 4);
                col[4] = a1.x; col[5] = a1.y;
            } else {
                const uint4 a1 = *reinterpret_cast<const uint4 *>(wr + 4);
                col[4] = a1.x; col[5] = a1.y; col[6] = a1.z; col[7] = a1.w;
                col[8] = wr[8];
            }
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
                const uint2 b = wb[3 * ky + kx];
                const float cB = __uint_as_float(b.x);
#pragma unroll
                for (int j = 0; j < TBX_TW; ++j) acc[j] += tbx_term(col[j * S + kx], cB, b.y, lut, q0exp, twoq);
            }
        }
        int co = c0 + pl;
        co -= dw_div(co, t.C, t.inv_c) * t.C;
        float *yr = y + ((P0 + pl) * t.Ho + oh0 + orow) * t.Wo;
#pragma unroll
        for (int j = 0; j < TBX_TW; ++j)
            if (4 * q + j < t.Wo) yr[4 * q + j] = epi(ep, ep_act, ep_lo, ep_hi, co, acc[j]);
    }
    if (__syncthreads_or(bad ? 1 : 0) && tid == 0) atomicOr(gate, 1u);
}

// conv_tbs_kernel with dn_dw3g_kernel's staging (option "tbs" = 2, the default): the source range
// copied raw into LDS by LDS-DMA (padding not stored: a tap outside the plane reads the zero word),
// each value turned into its table-form word in place (input quantizer, tbx_word and its window /
// grid checks), then 4 outputs per thread as conv_tbs_kernel: the same terms in the same order,
// the same bits, the same gate.
// The staged depthwise kernels' tap rows (ky) run as a loop, not unrolled (round 6): unrolled, the
// compiler hoisted every LDS read of the 36 terms and held the kernels at 116-126 VGPRs (4 waves /
// SIMD, 42 % of the wave cycles waiting); rolled, 41-56 VGPRs: MobileNetV2 E4M3 +3 %, E5M2 v9 +3.3 %,
// v5 +0.5 % (profiles/r06_dw/).  TBSG_WAVES: an occupancy floor for A/B builds (it spills).
#ifndef TBSG_WAVES
#define TBSG_WAVES 1
#endif
#ifndef TBSG_KYU
#define TBSG_KYU 1
#endif
#ifndef V5DS_KYU
#define V5DS_KYU 1
#endif
// Per-tap tables (round 6, option build TBSG_TAPT, off): each tap's 8 entries (m_a) with its c_b
// applied, L(m_a, m_b) c_b, and its F7 trigger divided by c_b -- a term is then one multiply by c_a
// (exact either way) and the trigger test is on c_a: the ky loop 160 -> 137 VALU instructions per 12
// terms, 576 B of LDS per plane more -- and MobileNetV2 1.1-1.4 % slower (the per-block table build
// and the smaller block plans it forces; profiles/r06_tapt/).  Bit-identical either way.
#ifndef TBSG_TAPT
#define TBSG_TAPT 0
#endif
// conv_tbsg_kernel's dynamic LDS: table (512 B), taps (72 B per plane), the per-tap tables (576 B
// per plane), the staged source from the next 16-byte boundary (nimg floats) -- in floats, and the
// launch's byte count; tbsg_tap_bytes: the per-plane bytes per tap for the block plan
__host__ __device__ constexpr int tbsg_img_off(int PB) { return (128 + 18 * PB + (TBSG_TAPT ? 144 * PB : 0) + 3) & ~3; }
__host__ __device__ constexpr size_t tbsg_lds_bytes(int PB, int nimg) { return 4 * ((size_t)tbsg_img_off(PB) + nimg); }
__host__ __device__ constexpr int tbsg_tap_bytes() { return TBSG_TAPT ? 72 : 8; }

// One term from a per-tap table (TBSG_TAPT): tap = the tap's 8 entries {L c_b, trigger / c_b}
__device__ __forceinline__ float tbx_term_t(uint32_t wa, const char *tap, uint32_t q0exp, float twoq) {
    const float2 e = *reinterpret_cast<const float2 *>(tap + (wa & 0x38u));
    const uint32_t cab = wa & 0xFF800000u;                 // c_a (0 for a zero word)
    float rv = e.x * __uint_as_float(cab);                  // exact: the same value as L (c_a c_b)
    const float rs = copysignf(__fmaf_rn(2.0f, fabsf(rv), -twoq), rv);  // expo field 0 (tbx_term)
    rv = ((__float_as_uint(rv) & 0x7F800000u) == q0exp) ? rs : rv;
    return (cab == __float_as_uint(e.y)) ? fabsf(rv) : rv;  // F7: c_a c_b == trigger <=> c_a == trigger / c_b
}
template <int S, int M>
__global__ __launch_bounds__(256, TBSG_WAVES) void conv_tbsg_kernel(const float *x, const float *w, float *y, const DwArgs p,
                                                        FqIn fq, float *fq_bias_out, int32_t *fq_ibias_out,
                                                        const int32_t *bA, const int32_t *bW, const int32_t *bR,
                                                        TablePack tab, uint32_t *gate, const float2 *ep, int ep_act,
                                                        float ep_lo, float ep_hi, EmitW em) {
    constexpr int NC = 3 * S + 3;
    constexpr uint32_t LOWM = (1u << (23 - M)) - 1u, MMASK = (1u << M) - 1u;
    extern __shared__ float dw_sm[];
    const int tid = threadIdx.x, wv = tid >> 6;
    const int band = (int)(blockIdx.x % (unsigned)p.nb);
    const int64_t P0 = (int64_t)(blockIdx.x / (unsigned)p.nb) * p.PB;
    const int npl = (int)min((int64_t)p.PB, p.planes - P0);
    const int oh0 = band * p.RB, nrow = min(p.RB, p.Ho - oh0), hi0 = oh0 * S - p.ph;
    const int hw = p.H * p.W;
    const bool plane_mode = p.RB == p.Ho;
    const int rlo = plane_mode ? 0 : max(hi0, 0), rhi = plane_mode ? p.H : min(hi0 + p.RS, p.H);
    const int n = plane_mode ? npl * hw : (rhi - rlo) * p.W;
    const int64_t g0 = P0 * hw + (int64_t)rlo * p.W, a0 = g0 & ~(int64_t)3;
    const int lead = (int)(g0 - a0), nq = (lead + n + 3) >> 2;
    // the table first (round 6): its LDS address is then a link-time constant, which the reads'
    // offset field carries (a per-term address add less); then the taps, then the staged source
    float2 *sL = reinterpret_cast<float2 *>(dw_sm);            // the table (64 entries)
    uint2 *sB = reinterpret_cast<uint2 *>(sL + 64);            // [PB][9] {c_b bits, m_b << 6}
    float2 *sT = reinterpret_cast<float2 *>(sB + 9 * p.PB);    // (TBSG_TAPT) [PB][9][8] per-tap tables
    float *img = dw_sm + tbsg_img_off(p.PB);
    const float *src = x + a0;
    for (int q0 = 0; q0 < nq; q0 += 256) {
        const int q = q0 + tid;
        if (q < nq) {
            if (a0 + 4 * (int64_t)q + 4 <= p.nx) {
                __builtin_amdgcn_global_load_lds(src + 4 * q, img + 4 * (q0 + 64 * wv), 16, 0, 0);
            } else {
                for (int e = 0; e < 4; ++e)
                    if (a0 + 4 * (int64_t)q + e < p.nx) img[4 * q + e] = src[4 * q + e];
            }
        }
    }
    const float fmx = fq.mx ? *fq.mx : 0.0f, fbias = fq.mx ? fq_bias(fmx, fq.E, fq.M) : 0.0f;
    if (fq.mx && blockIdx.x == 0 && tid == 0) {
        *fq_bias_out = fbias;
        *fq_ibias_out = (int32_t)fbias;
    }
    const int a_b = fq.mx ? (int32_t)fbias : *bA, r_b = *bR;
    bool bad = !(a_b >= 2 && a_b <= 120 && r_b >= 2 && r_b <= 120);
    if (tid < 64) sL[tid] = tbx_lut_entry<M>(tid, tab, r_b);
    const int c0 = (int)(P0 % p.C);
    for (int d = tid; d < npl * 9; d += 256) {
        const int pl = d / 9;
        int c = c0 + pl;
        c -= dw_div(c, p.C, p.inv_c) * p.C;
        const int wb = bW[c];
        bad |= !(wb >= 2 && wb <= 120);
        const uint32_t bw = __float_as_uint(w[(int64_t)c * 9 + d - 9 * pl]), bwa = bw & 0x7FFFFFFFu;
        bad |= (bwa != 0u) && ((bwa & LOWM) != 0u || bwa < 0x20800000u || bwa > 0x58800000u);
        sB[d] = make_uint2(bw & 0xFF800000u, ((bwa >> (23 - M)) & MMASK) << 6);
    }
    __syncthreads();  // (waits for the LDS-DMA)
    uint32_t *iw = reinterpret_cast<uint32_t *>(img);
    {  // in place: value -> its word (the source range only: the lead / tail words are never read)
        const int i0 = lead, i1 = lead + n;
        for (int i = i0 + tid; i < i1; i += 256) iw[i] = tbx_word(img[i], fq, fmx, fbias, LOWM, MMASK, M, bad);
    }
    if (TBSG_TAPT) {  // entry (tap d, m_a): {L(m_a, m_b) c_b, trigger / c_b} (never-matching for c_b = 0 or out of range)
        for (int e = tid; e < npl * 72; e += 256) {
            const uint2 b = sB[e >> 3];
            const float2 l = sL[(b.y >> 3) + (e & 7)];
            const uint32_t t = __float_as_uint(l.y), cb = b.x;
            // trigger -2^(Et - 127) / (+-2^(Eb - 127)) = -+2^(Et - Eb): exponent field Et - Eb + 127
            const int ef = (int)((t >> 23) & 0xFFu) - (int)((cb >> 23) & 0xFFu) + 127;
            const bool ok = t != 0xFFFFFFFFu && (cb & 0x7F800000u) != 0u && ef >= 1 && ef <= 254;
            const uint32_t tq = ok ? (((t ^ cb) & 0x80000000u) | ((uint32_t)ef << 23)) : 0xFFFFFFFFu;
            sT[e] = make_float2(l.x * __uint_as_float(cb), __uint_as_float(tq));
        }
    }
    __syncthreads();
    const uint32_t q0exp = (uint32_t)(127 - r_b) << 23;
    const float twoq = __uint_as_float((uint32_t)(128 - r_b) << 23);
    const char *lut = reinterpret_cast<const char *>(sL);
    const int nqd = (p.Wo + 3) >> 2, pq = p.RB * nqd;
    // word-image emission for the next (matrix-core) convolution, em.form 0 (round 6): the words
    // xm_decode_a would write from this launch's y -- fq_next(y) -> xm_word_a, the same floats, bit
    // for bit (emit_word) -- so the pointwise convolution after a depthwise one skips its pre-pass.
    // The next quantizer's constants from the image header (emit_prep_kernel), wave-uniform.
    float emx = 0.0f, efb = 0.0f;
    uint32_t eemn = 0u, sehi = 0u;
    int ebR = 0;
    bool eok = true;
    if (em.w) {
        emx = __uint_as_float(__builtin_amdgcn_readfirstlane((int)em.invalid[1]));
        efb = __uint_as_float(__builtin_amdgcn_readfirstlane((int)em.invalid[2]));
        eemn = __builtin_amdgcn_readfirstlane(em.invalid[3]);
        ebR = __builtin_amdgcn_readfirstlane((int)em.invalid[4]);
    }
    for (int e = tid; e < npl * pq; e += 256) {
        const int pl = dw_div(e, pq, p.inv_pq), rem = e - pl * pq;
        const int orow = dw_div(rem, nqd, p.inv_nqd), qd = rem - orow * nqd;
        if (orow >= nrow) continue;
        const int r0 = (oh0 + orow) * S - p.ph, cl = 4 * S * qd - p.pw;
        const uint32_t *xs = iw + lead + pl * hw + (r0 - rlo) * p.W + cl;
        const uint2 *wb = sB + pl * 9;
        bool cok[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) cok[c] = (unsigned)(cl + c) < (unsigned)p.W;
        float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll TBSG_KYU
        for (int ky = 0; ky < 3; ++ky) {
            const bool rok = (unsigned)(r0 + ky) < (unsigned)p.H;
            uint32_t col[NC];
#pragma unroll
            for (int c = 0; c < NC; ++c) col[c] = (rok && cok[c]) ? xs[ky * p.W + c] : 0u;
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
                if (TBSG_TAPT) {
                    const char *tap = reinterpret_cast<const char *>(sT + 8 * (9 * pl + 3 * ky + kx));
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[j] += tbx_term_t(col[j * S + kx], tap, q0exp, twoq);
                } else {
                    const uint2 b = wb[3 * ky + kx];
                    const float cB = __uint_as_float(b.x);
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[j] += tbx_term(col[j * S + kx], cB, b.y, lut, q0exp, twoq);
                }
            }
        }
        int co = c0 + pl;
        co -= dw_div(co, p.C, p.inv_c) * p.C;
        float *yo = y + ((P0 + pl) * p.Ho + oh0 + orow) * p.Wo + 4 * qd;
        uint32_t *wo = em.w ? em.w + ((uint32_t)(P0 + pl) * (uint32_t)em.awH + (uint32_t)(oh0 + orow + em.awph)) *
                                         (uint32_t)em.awW + (uint32_t)em.awpw + 4u * (uint32_t)qd
                            : nullptr;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (4 * qd + j < p.Wo) {
                const float o = epi(ep, ep_act, ep_lo, ep_hi, co, acc[j]);
                yo[j] = o;
                if (wo) {
                    const uint32_t wd = xm_word_a(fq_apply(o, emx, efb, em.fq.M, em.fq.S), em.Mw, xm_xbias(em.Mw), eemn,
                                                  ebR, eok);
                    wo[j] = wd;
                    sehi = max(sehi, word_sehi(wd));
                }
            }
    }
    if (em.w) wave_max_atomic(em.invalid + 5, sehi);  // (every lane: the loop above has ended for all)
    const bool ebad = em.w && !eok;
    if (__syncthreads_or(bad ? 1 : 0) && tid == 0) {
        atomicOr(gate, 1u);
        if (em.w) atomicOr(em.invalid, 1u);  // (the exact kernel rewrites y: the words are stale)
    }
    if (__syncthreads_or(ebad ? 1 : 0) && tid == 0) atomicOr(em.invalid, 1u);  // (a word off the window)
}

// (round 3's alternative depthwise forms conv_dwx_kernel -- band-staged in LDS -- and
// conv_dwg_kernel -- an fp32 gather -- measured slower than conv_tbx_kernel and were
// removed in round 4.)

// ---------------------------------------------------------------------------------------------
// conv_v5dw_kernel: the v5 integer-adder model's depthwise convolutions (BASELINE config 3 with
// approx_version 5, MobileNetV2 E5M2) -- the terms of exact_term_v5 (fp8approx_device.h; the
// reference's approx_mult_new, approx_matmul_whole_v5.py:155-182) in conv_tbx_kernel's layout.
// v5 decodes every operand exactly (clip_OF), so the A pre-pass (v5dw_decode_a) turns each input
// into a word and never gates; the weights' words come from v5dw_decode_b.  Per term:
//   r = c_a + c_b' + T[m_a][m_b]    (c_b' = B code - (bA + bB - bR) << M, a byte of the tap's row)
//   r = v5_ofuf(r)                   (adder wrap / OF / UF switches)
//   value: r in [0, 2^M): the subnormal band, r 2^(1-bR-M) (float(r) times a power of two);
//          else the normal binade (r >> M) - bR with mantissa r & (2^M - 1), whose float bits
//          are linear in r: (r << (23 - M)) + ((127 - bR) << 23) (also for r < 0 without the wrap)
//   signed with sign(a) sign(b), summed in k order (one channel, 3 taps x kh rows <= 16 terms, so
//   the chunked sum of conv_tb_direct_kernel<false> is the plain sequential sum).
// E5M2 with the adder wrap on (sim_hw_add_OFUF: r in [0, 2^(E+M)) after v5_ofuf, whatever the
// OF / UF switches) only -- 4 table bytes per tap row.  A result bias whose binades leave the
// normal float range raises the gate and conv_tb_direct_kernel<false> recomputes the launch.
//
// A word: sign(a) << 31 | (m_a * 8) << 16 | c_a (c_a < 2^7); the zero word (0) is the code of +0,
// which is also what the reference's im2col padding decodes to.
// fq.mx set: x is unquantized; the activation quantizer is applied to each value first and its
// bias (the decode's bA) written to fqb / fqi, as xm_decode_a does.
__global__ __launch_bounds__(256) void v5dw_decode_a(const float *x, int64_t n, uint32_t *out, int E, int M,
                                                     const int32_t *bA, FqIn fq, float *fqb, int32_t *fqi) {
    const float fmx = fq.mx ? *fq.mx : 0.0f, fbias = fq.mx ? fq_bias(fmx, fq.E, fq.M) : 0.0f;
    if (fq.mx && blockIdx.x == 0 && threadIdx.x == 0) {
        *fqb = fbias;
        *fqi = (int32_t)fbias;
    }
    const DFmt f = dfmt(E, M, fq.mx ? (int)fbias : *bA, false);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        float v = x[i];
        if (fq.mx) v = fq_apply(v, fmx, fbias, fq.M, fq.S);
        int e, m;
        exact_dec(v, f, true, e, m);
        out[i] = (v < 0.0f ? 0x80000000u : 0u) | ((uint32_t)(m * 8) << 16) | (uint32_t)(e * (1 << M) + m);
    }
}

// B words per (channel, tap): x = (c_b' << 1) | sign(b), y = the tap's table row T[m_a][m_b]
// for m_a = 0..3 as signed bytes.
__global__ __launch_bounds__(256) void v5dw_decode_b(const float *w, int64_t n, int taps, uint2 *out, int E, int M,
                                                     const int32_t *bA, const int32_t *bW, const int32_t *bR,
                                                     TablePack tab) {
    const int a_b = *bA, r_b = *bR;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t co = i / taps;
        const int b_b = bW[co];
        const float v = w[i];
        int e, m;
        exact_dec(v, dfmt(E, M, b_b, false), true, e, m);
        const int32_t cb = (e - (a_b + b_b - r_b)) * (1 << M) + m;
        uint32_t row = 0;
        for (int ma = 0; ma < 4; ++ma) row |= ((uint32_t)(uint8_t)tab.raw[(ma << M) | m]) << (8 * ma);
        out[i] = make_uint2(((uint32_t)cb << 1) | (v < 0.0f ? 1u : 0u), row);
    }
}

template <int SW>
__global__ __launch_bounds__(256) void conv_v5dw_kernel(const uint32_t *aw, const uint2 *bw, float *y, TbxArgs t,
                                                        const int32_t *bR, uint32_t flags, int E, uint32_t *gate,
                                                        const float2 *ep,
                                                        int ep_act, float ep_lo, float ep_hi) {
    constexpr int KW = 3, NCOL = (TBX_TW - 1) * SW + KW, M = 2;
    const int r_b = *bR;
    const int32_t maxi = ((1 << E) << M) - 1;
    bool bad = !(r_b >= -90 && r_b <= 120);
    const uint32_t lin0 = (uint32_t)(127 - r_b) << 23;          // float bits of r = 0 on the normal line
    const float csub = __uint_as_float((uint32_t)(126 - r_b) << 23);  // 2^(1 - bR - M), M = 2
    const int64_t HW = t.H * t.W;
    for (uint32_t item = blockIdx.x * blockDim.x + threadIdx.x; item < t.items; item += gridDim.x * blockDim.x) {
        const uint32_t wg = item % t.nwg, r1 = item / t.nwg;
        const uint32_t ho = r1 % (uint32_t)t.Ho, r2 = r1 / (uint32_t)t.Ho;
        const uint32_t co = r2 % (uint32_t)t.Cout, img = r2 / (uint32_t)t.Cout;
        const int wo0 = (int)wg * TBX_TW, wi0 = wo0 * SW - t.pw;
        float acc[TBX_TW] = {0.0f, 0.0f, 0.0f, 0.0f};
        const uint32_t *plane = aw + ((int64_t)img * t.Cin + (int64_t)co) * HW;
        const uint2 *wk = bw + (int64_t)co * t.kh * KW;
        for (int ky = 0; ky < t.kh; ++ky) {
            const int hi = (int)ho * SW - t.ph + ky * t.dh;
            const bool rowok = (uint32_t)hi < (uint32_t)t.H;
            const uint32_t *row = plane + (int64_t)hi * t.W;
            uint32_t col[NCOL];
#pragma unroll
            for (int j = 0; j < NCOL; ++j) {
                const int wi = wi0 + j;
                col[j] = (rowok && (uint32_t)wi < (uint32_t)t.W) ? row[wi] : 0u;
            }
#pragma unroll
            for (int kx = 0; kx < KW; ++kx) {
                const uint2 b = wk[ky * KW + kx];
                const int32_t cb = (int32_t)b.x >> 1;
                const uint32_t sb = b.x << 31;
#pragma unroll
                for (int q = 0; q < TBX_TW; ++q) {
                    const uint32_t wa = col[q * SW + kx];
                    const int32_t tv = __builtin_amdgcn_sbfe((int32_t)b.y, (wa >> 16) & 31u, 8);  // T[m_a][m_b]
                    int32_t r = (int32_t)(wa & 0xFFu) + cb + tv;
                    r = v5_ofuf(r, maxi, M, flags);
                    const float vn = __uint_as_float(((uint32_t)r << (23 - M)) + lin0);
                    const float vs = (float)r * csub;
                    const float v = ((uint32_t)r < (1u << M)) ? vs : vn;
                    acc[q] += __uint_as_float(__float_as_uint(v) ^ ((wa & 0x80000000u) ^ sb));
                }
            }
        }
        float *yr = y + (((int64_t)img * t.Cout + co) * t.Ho + ho) * t.Wo;
#pragma unroll
        for (int q = 0; q < TBX_TW; ++q)
            if (wo0 + q < t.Wo) yr[wo0 + q] = epi(ep, ep_act, ep_lo, ep_hi, co, acc[q]);
    }
    if (__syncthreads_or(bad ? 1 : 0) && threadIdx.x == 0) atomicOr(gate, 1u);
}

// conv_v5dw_kernel's terms with both pre-passes fused in (option "v5ds", the default): the
// workgroup's contiguous source range of x is copied raw into LDS by LDS-DMA (dn_dw3g_kernel's
// staging, padding not stored), each value is turned in place into its v5 word (the input
// quantizer first when fused -- v5dw_decode_a), the PB planes' 9 tap words are built from the
// weights (v5dw_decode_b), then thread = 4 consecutive outputs of a row, the window's words read
// once, the terms in (ky, kx) order from zero: the same bits as conv_v5dw_kernel without the word
// image's write and read (8 B per input value) and two launches.  Depthwise 3 x 3, stride S both
// ways, dilation 1.  The gate rule is conv_v5dw_kernel's (the result bias's range).
template <int S>
__global__ __launch_bounds__(256) void conv_v5ds_kernel(const float *x, const float *w, float *y, const DwArgs p,
                                                        FqIn fq, float *fqb, int32_t *fqi, const int32_t *bA,
                                                        const int32_t *bW, const int32_t *bR, TablePack tab,
                                                        uint32_t flags, int E, uint32_t *gate, const float2 *ep,
                                                        int ep_act, float ep_lo, float ep_hi, EmitW em) {
    constexpr int M = 2, NC = 3 * S + 3;
    extern __shared__ float dw_sm[];
    const int tid = threadIdx.x, wv = tid >> 6;
    const int band = (int)(blockIdx.x % (unsigned)p.nb);
    const int64_t P0 = (int64_t)(blockIdx.x / (unsigned)p.nb) * p.PB;
    const int npl = (int)min((int64_t)p.PB, p.planes - P0);
    const int oh0 = band * p.RB, nrow = min(p.RB, p.Ho - oh0), hi0 = oh0 * S - p.ph;
    const int hw = p.H * p.W;
    const bool plane_mode = p.RB == p.Ho;
    const int rlo = plane_mode ? 0 : max(hi0, 0), rhi = plane_mode ? p.H : min(hi0 + p.RS, p.H);
    const int n = plane_mode ? npl * hw : (rhi - rlo) * p.W;
    const int64_t g0 = P0 * hw + (int64_t)rlo * p.W, a0 = g0 & ~(int64_t)3;
    const int lead = (int)(g0 - a0), nq = (lead + n + 3) >> 2;
    float *img = dw_sm;
    uint2 *sB = reinterpret_cast<uint2 *>(dw_sm + p.nimg);  // [PB][9] tap words
    const float *src = x + a0;
    for (int q0 = 0; q0 < nq; q0 += 256) {
        const int q = q0 + tid;
        if (q < nq) {
            if (a0 + 4 * (int64_t)q + 4 <= p.nx) {
                __builtin_amdgcn_global_load_lds(src + 4 * q, img + 4 * (q0 + 64 * wv), 16, 0, 0);
            } else {
                for (int e = 0; e < 4; ++e)
                    if (a0 + 4 * (int64_t)q + e < p.nx) img[4 * q + e] = src[4 * q + e];
            }
        }
    }
    const float fmx = fq.mx ? *fq.mx : 0.0f, fbias = fq.mx ? fq_bias(fmx, fq.E, fq.M) : 0.0f;
    if (fq.mx && blockIdx.x == 0 && tid == 0) {
        *fqb = fbias;
        *fqi = (int32_t)fbias;
    }
    const int a_b = fq.mx ? (int)fbias : *bA, r_b = *bR;
    const int c0 = (int)(P0 % p.C);
    for (int d = tid; d < npl * 9; d += 256) {  // v5dw_decode_b for the block's planes
        const int pl = d / 9;
        int c = c0 + pl;
        c -= dw_div(c, p.C, p.inv_c) * p.C;
        const int b_b = bW[c];
        const float v = w[(int64_t)c * 9 + d - 9 * pl];
        int e, m;
        exact_dec(v, dfmt(E, M, b_b, false), true, e, m);
        const int32_t cb = (e - (a_b + b_b - r_b)) * (1 << M) + m;
        uint32_t row = 0;
        for (int ma = 0; ma < 4; ++ma) row |= ((uint32_t)(uint8_t)tab.raw[(ma << M) | m]) << (8 * ma);
        sB[d] = make_uint2(((uint32_t)cb << 1) | (v < 0.0f ? 1u : 0u), row);
    }
    __syncthreads();  // (waits for the LDS-DMA)
    {  // in place: value -> (input quantizer) -> v5 word (v5dw_decode_a)
        const DFmt f = dfmt(E, M, a_b, false);
        uint32_t *iw = reinterpret_cast<uint32_t *>(img);
        for (int i = tid; i < 4 * nq; i += 256) {
            float v = img[i];
            if (fq.mx) v = fq_apply(v, fmx, fbias, fq.M, fq.S);
            int e, m;
            exact_dec(v, f, true, e, m);
            iw[i] = (v < 0.0f ? 0x80000000u : 0u) | ((uint32_t)(m * 8) << 16) | (uint32_t)(e * (1 << M) + m);
        }
    }
    __syncthreads();
    const uint32_t *iw = reinterpret_cast<const uint32_t *>(img);
    const int32_t maxi = ((1 << E) << M) - 1;
    const bool bad = !(r_b >= -90 && r_b <= 120);
    const uint32_t lin0 = (uint32_t)(127 - r_b) << 23;
    const float csub = __uint_as_float((uint32_t)(126 - r_b) << 23);  // 2^(1 - bR - M), M = 2
    const int nqd = (p.Wo + 3) >> 2, pq = p.RB * nqd;
    // word-image emission for the next (v5 matrix-core, unpadded) convolution: v5_word_a of its input
    // quantizer's fq(y) at its own bias (the image header, emit_prep_kernel) -- xm_decode_a's words
    float emx = 0.0f, efb = 0.0f;
    if (em.w) {
        emx = __uint_as_float(__builtin_amdgcn_readfirstlane((int)em.invalid[1]));
        efb = __uint_as_float(__builtin_amdgcn_readfirstlane((int)em.invalid[2]));
    }
    const DFmt efmt = dfmt(em.Mw == 2 ? 5 : 4, em.Mw, (int)efb, false);
    for (int e = tid; e < npl * pq; e += 256) {
        const int pl = dw_div(e, pq, p.inv_pq), rem = e - pl * pq;
        const int orow = dw_div(rem, nqd, p.inv_nqd), qd = rem - orow * nqd;
        if (orow >= nrow) continue;
        const int r0 = (oh0 + orow) * S - p.ph, cl = 4 * S * qd - p.pw;
        const uint32_t *xs = iw + lead + pl * hw + (r0 - rlo) * p.W + cl;
        const uint2 *wb = sB + pl * 9;
        bool cok[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) cok[c] = (unsigned)(cl + c) < (unsigned)p.W;
        float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll V5DS_KYU
        for (int ky = 0; ky < 3; ++ky) {
            const bool rok = (unsigned)(r0 + ky) < (unsigned)p.H;
            uint32_t col[NC];
#pragma unroll
            for (int c = 0; c < NC; ++c) col[c] = (rok && cok[c]) ? xs[ky * p.W + c] : 0u;
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
                const uint2 b = wb[3 * ky + kx];
                const int32_t cb = (int32_t)b.x >> 1;
                const uint32_t sb = b.x << 31;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t wa = col[j * S + kx];
                    const int32_t tv = __builtin_amdgcn_sbfe((int32_t)b.y, (wa >> 16) & 31u, 8);  // T[m_a][m_b]
                    int32_t r = (int32_t)(wa & 0xFFu) + cb + tv;
                    r = v5_ofuf(r, maxi, M, flags);
                    const float vn = __uint_as_float(((uint32_t)r << (23 - M)) + lin0);
                    const float vs = (float)r * csub;
                    const float v = ((uint32_t)r < (1u << M)) ? vs : vn;
                    acc[j] += __uint_as_float(__float_as_uint(v) ^ ((wa & 0x80000000u) ^ sb));
                }
            }
        }
        int co = c0 + pl;
        co -= dw_div(co, p.C, p.inv_c) * p.C;
        float *yo = y + ((P0 + pl) * p.Ho + oh0 + orow) * p.Wo + 4 * qd;
        uint32_t *wo = em.w ? em.w + ((uint32_t)(P0 + pl) * (uint32_t)em.awH + (uint32_t)(oh0 + orow + em.awph)) *
                                         (uint32_t)em.awW + (uint32_t)em.awpw + 4u * (uint32_t)qd
                            : nullptr;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (4 * qd + j < p.Wo) {
                const float o = epi(ep, ep_act, ep_lo, ep_hi, co, acc[j]);
                yo[j] = o;
                if (wo) wo[j] = v5_word_a(fq_apply(o, emx, efb, em.fq.M, em.fq.S), efmt);
            }
    }
    if (__syncthreads_or(bad ? 1 : 0) && tid == 0) {
        atomicOr(gate, 1u);
        if (em.w) atomicOr(em.invalid, 1u);  // (the literal kernel rewrites y: the words are stale)
    }
}

}  // namespace fp8a
