// fp8approx_common.h -- definitions shared by the translation units of libfp8approx.so
// (fp8approx.hip: the C-ABI, the host dispatch and the small kernels; k_fast.hip, k_f8mx.hip,
// k_tt.hip, k_v5.hip: the GEMM kernel families, compiled in parallel by build_native.py).
// Launch arguments, operand decode, the shared epilogue (store_tile) and the word-image emission.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <string>

#include "../../include/fp8approx.h"
#include "fp8approx_device.h"

namespace fp8a {

// ------------------------------------------------------------------------- table packing
// The error table (get_error_table_NN, v9:555-592) is a host constant; it is analysed on the
// host and packed into the launch arguments so the hot loop reads one register per operand:
//   TM_W1U  : entries in {0,1}   -> 1 bit / entry, 2^M bits per row      (E4M3)
//   TM_W2S/U: entries in [-2,1] / [0,3] -> 2 bits / entry, R = 2^M*2/32 words per row
//   TM_LUT  : anything else -> float LUT in LDS (E2M5 no-comp: entries up to 5)
enum TMode : int { TM_NONE = 0, TM_W1U = 1, TM_W2S1 = 2, TM_W2U1 = 3, TM_W2S2 = 4, TM_W2U2 = 5, TM_LUT = 6,
                   TM_QAMAA = 7 /* quantize_after_mult_and_add: term = fq(a*b), no decode */,
                   TM_V5 = 8 /* v5 integer-adder model: code sum + compensation LUT, OF/UF wrap */,
                   TM_F8 = 9 /* E4M3 with s2n + qbma, table in {0,1}: LDS term LUT + hardware fp8 Q_R */ };

struct TablePack {
    uint32_t rows[64][2];  // packed rows for the bit modes (2^M <= 64)
    int8_t raw[1024];      // the full table (2^M x 2^M), row-major; exact path and LUT mode
};

// ------------------------------------------------------------------------- GEMM arguments
// FP8 fake quantizer of the activations (quantize_to_fp8_ste_MM, fp8_quantizer.py:97-173),
// per tensor: the bias from maxval, then clamp / binade step / round.  fp8_quantize_kernel and the
// fused input quantization of the approx ops (fp8a_conv2d_qin) share these, bit for bit.
struct FqIn {
    const float *mx;  // device maxval [1]; nullptr = the input is already quantized
    int E, M, S;      // exponent / mantissa / sign bits of the quantizer
};

__device__ __forceinline__ float fq_bias(float mx, int E, int M) {
    return rintf((float)(1 << E) - log2f(mx) + log2f(2.0f - p2(-M)) - 1.0f);
}

// quantize_to_fp8_ste_MM's forward (fp8_quantizer.py:97-173) on one value, bias = fq_bias(mx):
//   xc = clamp(v), ls = max(floor(log2 |xc|) + bias, 1) (1 for xc = 0), k = ls - M - bias,
//   q = rint(xc / 2^k) 2^k.
// (Round 5 measured a bit-level form -- RNE on the float's bits at or above the smallest normal
// binade -- against this one: 7 % slower on the fake-quant kernel, no faster in the depthwise
// stages or the dense GEMM, so the literal form stays.)
// rint(xc / 2^k) 2^k without the IEEE division: the quotient is exact (a power-of-two scaling) and
// is formed as xc 2^-k, in two exact steps when 2^-k itself overflows (k < -126: then |xc| <= maxval
// is tiny and xc 2^64 cannot overflow); 2^k = 0 (k < -149) leaves the division's (x / 0) * 0 = NaN,
// formed as (x inf) * 0.
__device__ __forceinline__ float fq_step(float xc, int k) {
    const float t = (k >= -126) ? xc * p2(-k) : (xc * 18446744073709551616.0f) * p2(-k - 64);
    const float r = rintf(t) * p2(k);
    return k < -149 ? rintf(xc * __builtin_huge_valf()) * p2(k) : r;  // (x / 0 = x inf: the same NaN)
}
__device__ __forceinline__ float fq_apply_lit(float xc, float bias, int M) {
    int e;
    frexpf(xc, &e);
    const float ls = (xc == 0.0f) ? 1.0f : fmaxf((float)(e - 1) + bias, 1.0f);
    return fq_step(xc, (int)(ls - (float)M - bias));
}
__device__ __forceinline__ float fq_apply(float v, float mx, float bias, int M, int sign_bits) {
    return fq_apply_lit(fminf(fmaxf(v, sign_bits ? -mx : 0.0f), mx), bias, M);
}

// Word-image hand-off (round 4, fp8a_conv2d_chain): a convolution's store also writes the NEXT
// convolution's pre-decoded A operand -- its zero-bordered word image (gemm_f8mx.h: the word of
// fq_next(y) for every output element y) -- so the next launch skips its xm_decode_a pass (which
// reads y back and writes the image: 8 B of HBM traffic per element).  Same words as that pass,
// bit for bit: the same fq_apply / xm_word_a on the same float.  An element outside the
// matrix-core window sets the image's header word, and the consumer's gated pre-pass then
// re-decodes its input from y (the fp32 output is always written).
struct EmitW {
    uint32_t *w;        // the image's words [Bn][C][awH][awW] (nullptr: no emission)
    uint32_t *invalid;  // the image's header word
    int awH, awW, awph, awpw;
    int Wo;
    uint32_t hw_mul, hw_shift, wo_mul, wo_shift;  // fastdiv by Ho * Wo and Wo (output index < 2^31)
    uint32_t hw;
    FqIn fq;            // the next convolution's input quantizer (per tensor)
    const int32_t *bR;  // its result bias
    int Mw;             // its mantissa width (3: e4m3 words, 2: e5m2)
    int form;           // 0: gemm_f8mx_kernel's words (zero-bordered image); 1: the tensor-bias table
                        // form's words (conv_tbx.h tbx_decode_a: a depthwise consumer, no border)
};

struct GemmArgs {
    const float *A;
    int64_t lda;
    const float *B;
    int64_t sbk, sbn;
    float *C;
    int64_t ldc;
    int64_t M, N, K;
    int E, Mw;
    uint32_t kexp, kdc;  // 0x7F800000 and (23 - Mw) << 23 as launch arguments: opaque SGPR operands
                         // keep q_fast at one v_and_or_b32 / one v_add_u32 (see make_qc)
    const int32_t *bA;
    const int32_t *bB;
    int64_t bBs;
    const int32_t *bR;
    uint32_t flags;
    // output mapping: rowmajor C[m*ldc + n], or NCHW C[(m/hw)*ctot*hw + (coff+n)*hw + m%hw]
    int nchw;
    int64_t hw, ctot, coff;
    uint32_t *flag;  // device word: set by the fast kernel when the exact kernel must run (FB_* bits);
                     // a slot of the library's flag arena (flag_arena, fp8approx.hip), zero on entry
    // per-unit fallback marks (64 x 64 output units): urow[row unit] / ucol[column unit] for an
    // operand outside the fast path's window, utile[row unit * nuc + column unit] for a tile whose
    // terms left it; the gated exact kernel recomputes only the marked units.  nullptr (a
    // workspace without room for them): any fallback recomputes the whole launch.
    uint8_t *urow, *ucol, *utile;
    int64_t nur, nuc;
    // split-K: block b works on tile b % tiles over k in [s*kchunk, (s+1)*kchunk), s = b / tiles;
    // with splits > 1 it writes its partial tile to part + s*M*N (the output layout with
    // ctot = N, coff = 0, ldc = N) and splitk_reduce_kernel sums the splits in order
    int splits;
    int64_t kchunk;
    float *part;
    // implicit-GEMM convolution: A(m, k) gathered from NCHW x (no im2col image), m = (b, ho, wo),
    // k = (c, ky, kx) within the group -- the reference's im2col order (approx_calculation.py:745)
    int conv;
    const float *X;
    int64_t Cin, H, W, Ho, Wo, cbase;
    int kh, kw, sh, sw, ph, pw, dh, dw;
    uint32_t kk_mul, kk_shift, kw_mul, kw_shift;  // fast division by kh*kw and by kw
    // qamaa: the res quantizer's FP8 fake quantizer (fp8_quantizer.py:97-173) per product
    const float *qmax;
    int qE, qM, qsign;
    // fused eval-mode BatchNorm + activation epilogue (BNFusedHijacker: F.batch_norm then ReLU /
    // ReLU6 / Hardtanh): per output channel {scale, shift}; ep_act clamps to [ep_lo, ep_hi]
    const float2 *ep;
    int ep_act;
    float ep_lo, ep_hi;
    // pre-decoded operands of the matrix-core E4M3 kernel (gemm_f8mx.h): A words (conv: the
    // group's [Bn][aw_c][H][W] slice; matrix: [M][awld]), B column pairs [Kpad][npad / 2]
    const uint32_t *aw;
    int64_t awld, aw_c;
    int64_t awH, awW;  // conv: the word image's height / width (H + 2 ph, W + 2 pw when zero-padded)
    int awph, awpw;    // conv: x's offset inside the word image (the zero border's width)
    int wfmt;          // pre-decoded operand format: 0 = gemm_f8mx_kernel's, 1 = gemm_tt_kernel's, 2 = gemm_tt16_kernel's,
                       // 4 = gemm_v5mx_kernel's
    int ttf7;          // gemm_tt_kernel: the table has negative entries (the F7 sign rule)
    int af32;          // gemm_f8mx_kernel reads A as fp32 and decodes it while staging (no A pre-pass)
    int xncg;          // gemm_f8mx_kernel's column groups per tile (4: 128 x 64, 2: 128 x 32, 1: 256 x 16)
    const uint2 *bqw;
    const uint32_t *lutw;  // the LDS table image (XM_LUT_WORDS words), written by xm_decode_b
    // E5M2 (gemm_f8mx_kernel XF = 1): per (K-step, 16-column group) the nonzero B elements' exponent
    // range, (max e_b + 128) | (min e_b + 128) << 8 ([kpad][npad / 16]; 0xFF00 when all are zero)
    const uint16_t *ebr;
    int xm_vmin;  // the smallest binade of the table value V' (0: V' >= 1, -1 with a {0,1} table)
    int64_t npad;
    // fused input quantization (fp8a_conv2d_qin): A = fq(X); the quantizer's bias is written to
    // fq_bias / fq_ibias by the A pre-decode, and bA points at fq_ibias
    FqIn fqin;
    float *fq_bias;
    int32_t *fq_ibias;
    // block-output epilogue (fp8a_conv2d_block): after BN / activation, y += res (same index as
    // y), then the post clamp (post_act 1) or GELU (post_act 2), then the block's output quantizer (post_fq)
    const float *res;
    int post_act;
    float post_lo, post_hi;
    FqIn post_fq;
    EmitW em;              // word-image emission for the next convolution (em.w nullptr: off)
    const uint32_t *gate;  // xm_decode_a: run only if *gate != 0 (the input image arrived invalid)
    const uint32_t *in_img; // the input's word image (header + words) a previous launch emitted, or nullptr
    TablePack tab;
    uint32_t *flag_out;  // the caller's workspace word that receives the launch's final flag word
    uint4 *arena_clr;    // the flag arena's other slot, and its 16-byte words to zero (arena_clear)
    uint32_t arena_clr16;
    float *post_bout;    // post_fq's bias outputs (its custom_bias), written by gemm_exact_kernel, or nullptr
    int32_t *post_ibout;
};

// Fallback flag word bits: FB_ANY = some output unit needs the exact kernel, FB_ALL = every
// unit does (a bias outside the exactness window, or no unit marks in the workspace).  (Bits
// 1-4 belong to gemm_tt16_kernel's f16 window, gemm_tt16.h.)
constexpr uint32_t FB_ANY = 1u, FB_ALL = 32u;
// FB_HALF: an E5M2 tile of gemm_f8mx_kernel's plain form met the result grid's top binade and
// asks the halved-block form (XF = 2) to recompute it; its unit marks carry UT_HALF.  Unit mark
// bits: UT_EXACT = recompute in the exact kernel, UT_HALF = recompute in the halved-block form
// (kept set by a halved-block tile that fails, so the tiles sharing the unit still see it).
constexpr uint32_t FB_HALF = 64u;
constexpr uint8_t UT_EXACT = 1u, UT_HALF = 2u;

// Fallback flag value of a block that found a bad operand: FB_ANY once the unit marks are
// written, FB_ALL too without them (or when `all`).
__device__ __forceinline__ uint32_t fb_bits(const GemmArgs &p, bool all = false) {
    return (all || p.urow == nullptr) ? (FB_ANY | FB_ALL) : FB_ANY;
}

// The flag arena (fp8approx.hip: flag_arena) has two slots per stream that launches use in turn:
// a launch finds its slot zero, and its last (gated) kernel zeroes the OTHER slot -- the words the
// previous launch left there, which nothing reads any more -- with every thread of its grid
// (16-byte stores; no fill launch, no counter, no ordering against the launch's own reads).
__device__ __forceinline__ void arena_clear(uint4 *clr, uint32_t n16) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += gridDim.x * blockDim.x)
        clr[i] = make_uint4(0u, 0u, 0u, 0u);
}

// Mark the row units of output rows [m_lo, m_hi) / the column unit of column n / the units of
// the output tile (m0 .. m0 + rows - 1, n0 .. n0 + 63) for the exact kernel (plain byte stores:
// every writer stores 1).  The caller raises the flag word (fb_bits).
__device__ __forceinline__ void fb_rows(const GemmArgs &p, int64_t m_lo, int64_t m_hi) {
    if (p.urow == nullptr || m_hi <= m_lo) return;
    for (int64_t u = m_lo >> 6; u <= (m_hi - 1) >> 6; ++u) p.urow[u] = 1;
}
__device__ __forceinline__ void fb_col(const GemmArgs &p, int64_t n) {
    if (p.ucol != nullptr) p.ucol[n >> 6] = 1;
}
__device__ __forceinline__ void fb_tile(const GemmArgs &p, int64_t m0, int64_t rows, int64_t n0,
                                        uint8_t mark = UT_EXACT) {
    if (p.utile == nullptr) return;
    const int64_t hi = min(m0 + rows, p.M);
    for (int64_t u = m0 >> 6; u <= (hi - 1) >> 6; ++u) p.utile[u * p.nuc + (n0 >> 6)] = mark;
}

// The block-output epilogue on one value / four values of the output at index o; pb = the post
// quantizer's bias (post_bias()).
__device__ __forceinline__ float post_bias(const GemmArgs &p) {
    return p.post_fq.mx ? fq_bias(*p.post_fq.mx, p.post_fq.E, p.post_fq.M) : 0.0f;
}

// nn.GELU() (approximate='none') in fp32 as ATen's GeluCUDAKernelImpl evaluates it:
// x * 0.5 * (1 + erf(x * M_SQRT1_2)), left to right, the same device erff (ocml)
__device__ __forceinline__ float gelu_erf(float x) {
    return x * 0.5f * (1.0f + erff(x * (float)M_SQRT1_2));
}

// GELU = false compiles the GELU tail out (the word-emitting store of gemm_f8mx_kernel, whose
// registers are at its occupancy budget; the host never pairs GELU with emission).
template <bool GELU = true>
__device__ __forceinline__ float post_tail(const GemmArgs &p, float v, float pb) {
    if (p.post_act == 1) v = fminf(fmaxf(v, p.post_lo), p.post_hi);
    else if (GELU && p.post_act == 2) v = gelu_erf(v);
    if (p.post_fq.mx) v = fq_apply(v, *p.post_fq.mx, pb, p.post_fq.M, p.post_fq.S);
    return v;
}

template <bool GELU = true>
__device__ __forceinline__ float post1(const GemmArgs &p, int64_t o, float v, float pb) {
    if (p.res) v += p.res[o];
    return post_tail<GELU>(p, v, pb);
}

template <bool GELU = true>
__device__ __forceinline__ float4 post4(const GemmArgs &p, int64_t o, float4 v, float pb) {
    if (p.res) {
        const float4 r = *reinterpret_cast<const float4 *>(p.res + o);
        v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
    }
    return make_float4(post_tail<GELU>(p, v.x, pb), post_tail<GELU>(p, v.y, pb), post_tail<GELU>(p, v.z, pb), post_tail<GELU>(p, v.w, pb));
}

// y = x * scale + shift with scale = gamma * invstd, shift = beta - mean * scale (ATen's eval
// batch-norm transform), then the activation clamp; c = output channel
__device__ __forceinline__ float epi(const float2 *ep, int act, float lo, float hi, int64_t c, float x) {
    if (ep == nullptr) return x;
    const float2 e = ep[c];
    const float v = __fmaf_rn(x, e.x, e.y);
    return act ? fminf(fmaxf(v, lo), hi) : v;
}

// n / d for 0 <= n < 2^31 via one mulhi: q = (mulhi(n, mul) + n) >> shift (Granlund-Montgomery).
static inline void fastdiv_params(uint32_t d, uint32_t &mul, uint32_t &shift) {
    uint32_t l = 0;
    while ((1ull << l) < d) ++l;
    shift = l;
    mul = (uint32_t)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
}

__device__ __forceinline__ uint32_t fastdiv(uint32_t n, uint32_t mul, uint32_t shift) {
    return (__umulhi(n, mul) + n) >> shift;
}

constexpr int BM = 64, BN = 64, BK = 16, TM = 4, TN = 4, NT = 256;
constexpr int AP = BM + 4, BP = BN + 4;

__device__ __forceinline__ uint32_t xm_word_a(float x, int M, int xb, uint32_t emnA, int bR, bool &ok);  // gemm_f8mx.h
__host__ __device__ constexpr int xm_xbias(int Mw);

// A = 0 as an A word of the matrix-core path (gemm_f8mx.h): cvt scale 2^126 (the code is 0), row 0.
// Nonzero words keep se <= 252, so a zero word is the one with se = 253, and the E5M2 halved form's
// se + 1 (254: 2^127) still flushes it to 0.
constexpr uint32_t XM_ZERO_WORD = 253u << 23;

// Word-image emission (EmitW): one word per final output value at NCHW output index o (< 2^31,
// the host checks).  The next quantizer's constants sit in the image's header (emit_prep_kernel:
// [1] maxval, [2] its float bias, [3] 2^(1 - bias) bits, [4] bR), made wave-uniform (SGPRs) once
// per epilogue: the matrix-core kernel runs at its 80-VGPR budget, and per-thread copies of them
// (or their recomputation from maxval) in VGPRs made it spill.
struct EmitCtx {
    float mx, fb;
    uint32_t emn;
    int bR;
};
__device__ __forceinline__ EmitCtx emit_ctx(const GemmArgs &p) {
    EmitCtx e{};
    if (p.em.w == nullptr) return e;
    const uint4 h = *reinterpret_cast<const uint4 *>(p.em.invalid);  // header words 0-3 (uniform: SGPRs)
    e.mx = __uint_as_float(__builtin_amdgcn_readfirstlane(h.y));
    e.fb = __uint_as_float(__builtin_amdgcn_readfirstlane(h.z));
    e.emn = __builtin_amdgcn_readfirstlane(h.w);
    e.bR = __builtin_amdgcn_readfirstlane((int)p.em.invalid[4]);
    return e;
}
__device__ __forceinline__ uint32_t emit_word(const GemmArgs &p, const EmitCtx &e, float v, bool &ok) {
    const float q = fq_apply(v, e.mx, e.fb, p.em.fq.M, p.em.fq.S);
    if (p.em.form) {  // tbx_decode_a's word of q (a value off the grid / outside the window: invalid)
        const uint32_t u = __float_as_uint(q), ua = u & 0x7FFFFFFFu, M = (uint32_t)p.em.Mw;
        ok = ok && (ua == 0u || ((ua & ((1u << (23 - M)) - 1u)) == 0u && ua >= 0x20800000u && ua <= 0x58800000u));
        return ua == 0u ? 0u : ((u & 0xFF800000u) | (((ua >> (23 - M)) & ((1u << M) - 1u)) << 3));
    }
    return xm_word_a(q, p.em.Mw, xm_xbias(p.em.Mw), e.emn, e.bR, ok);
}
// word index of NCHW output index o
__device__ __forceinline__ uint32_t emit_index(const GemmArgs &p, uint32_t uo, uint32_t &wo) {
    const uint32_t plane = fastdiv(uo, p.em.hw_mul, p.em.hw_shift), pix = uo - plane * p.em.hw;
    const uint32_t ho = fastdiv(pix, p.em.wo_mul, p.em.wo_shift);
    wo = pix - ho * (uint32_t)p.em.Wo;
    return (plane * (uint32_t)p.em.awH + ho + (uint32_t)p.em.awph) * (uint32_t)p.em.awW + wo + (uint32_t)p.em.awpw;
}
// Max of v over the wave, then one atomicMax into *dst (v >= 0; 0 records nothing) unless *dst
// already holds at least v -- every wave of a launch records into the same word, and the read
// first keeps the atomics (serialised on one L2 line) to the few waves that raise it.  Every lane
// of the wave must call it.
__device__ __forceinline__ void wave_max_atomic(uint32_t *dst, uint32_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off));
    if ((threadIdx.x & 63) == 0 && v != 0u && v > __hip_atomic_load(dst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        atomicMax(dst, v);
}
// 255 - the scale exponent of a nonzero word (the E5M2 halved-block decision reads the largest,
// gemm_f8mx.h xm_needs_halving; the header's word 5 collects it for the consumer)
__device__ __forceinline__ uint32_t word_sehi(uint32_t w) { return w == XM_ZERO_WORD ? 0u : 255u - (w >> 23); }

__device__ __forceinline__ void emit1(const GemmArgs &p, const EmitCtx &e, int64_t o, float v, uint32_t &sehi) {
    uint32_t wo;
    const uint32_t wi = emit_index(p, (uint32_t)o, wo);
    bool ok = true;
    const uint32_t w = emit_word(p, e, v, ok);
    p.em.w[wi] = w;
    sehi = max(sehi, word_sehi(w));
    if (!ok) atomicOr(p.em.invalid, 1u);
}
// four consecutive outputs (o % 4 == 0 in an NCHW plane of hw % 4 == 0): one 16-B store when
// they sit in one row of the image (Wo % 4 == 0: always; the interior rows start 16-B aligned)
__device__ __forceinline__ void emit4(const GemmArgs &p, const EmitCtx &e, int64_t o, float4 v, uint32_t &sehi) {
    uint32_t wo;
    const uint32_t wi = emit_index(p, (uint32_t)o, wo);
    bool ok0 = true, ok1 = true, ok2 = true, ok3 = true;
    const uint4 w = make_uint4(emit_word(p, e, v.x, ok0), emit_word(p, e, v.y, ok1), emit_word(p, e, v.z, ok2),
                               emit_word(p, e, v.w, ok3));
    sehi = max(max(sehi, max(word_sehi(w.x), word_sehi(w.y))), max(word_sehi(w.z), word_sehi(w.w)));
    if (wo + 3 < (uint32_t)p.em.Wo && (wi & 3u) == 0u) {
        *reinterpret_cast<uint4 *>(p.em.w + wi) = w;
    } else {
        p.em.w[wi] = w.x;
        uint32_t wo1;
        p.em.w[emit_index(p, (uint32_t)o + 1, wo1)] = w.y;
        p.em.w[emit_index(p, (uint32_t)o + 2, wo1)] = w.z;
        p.em.w[emit_index(p, (uint32_t)o + 3, wo1)] = w.w;
    }
    if (!(ok0 && ok1 && ok2 && ok3)) atomicOr(p.em.invalid, 1u);
}

__device__ __forceinline__ int64_t out_index(const GemmArgs &p, int64_t m, int64_t n) {
    if (!p.nchw) return m * p.ldc + n;
    const int64_t img = m / p.hw, pix = m - img * p.hw;
    return (img * p.ctot + p.coff + n) * p.hw + pix;
}

// Fast-path operand decode straight from the float32 bit pattern (int-bias semantics).
//   returns ok: x is exactly a value of the (M, b) grid (any exponent: A/B are decoded with
//               clip_OF=False, v9:58-59) and |x| is 0 or in [2^-62, 2^50] (exactness window:
//               every product and table term a normal float, every Q_R constant finite,
//               DESIGN.md §3).  Otherwise the launch is flagged and the exact kernel reruns it.
//   m        : the M-bit mantissa code = the top M bits of the fp32 mantissa (the s2n scale-up
//               by 2^M, v9:53, leaves the fp32 mantissa untouched)
//   c        : sign(x) * 2^floor(log2|x|): the scale of the error-table term.  Scale-up and
//               scale-back of s2n cancel in it; without s2n a subnormal operand fails the
//               reference's norm mask (v9:87), so c = 0 there, as for zeros.
__device__ __forceinline__ bool stage_decode(float x, int M, uint32_t emn, bool s2n, float &c, uint32_t &m) {
    const uint32_t u = __float_as_uint(x);
    const uint32_t ua = u & 0x7FFFFFFFu;
    const uint32_t ex = ua & 0x7F800000u;
    const bool sub = ua < emn;  // |x| < min_norm = 2^(1-b)
    const uint32_t sh = (uint32_t)(23 - M) + (sub ? ((emn - ex) >> 23) : 0u);
    const bool grid = (sh < 24u) ? ((ua & ((1u << sh) - 1u)) == 0u) : (ua == 0u);
    const bool win = (ua == 0u) || (ua >= 0x20800000u /*2^-62*/ && ua <= 0x58800000u /*2^50*/);
    m = (ua >> (23 - M)) & ((1u << M) - 1u);
    c = (ua == 0u || (!s2n && sub)) ? 0.0f : __uint_as_float(u & 0xFF800000u);
    return grid && win;
}

// Writes one thread's TM x TN outputs (rows m0 + ty*TM + i, columns n0 + tx*TN + j) to the
// output mapping, or to its split-K partial slice (same layout); applies the fused BN/activation
// epilogue when unsplit.
// EMIT = false compiles the word-image emission out (gemm_f8mx_kernel's non-emitting instances:
// the emission code alone pushed that kernel past its 80-VGPR budget).
// GELU = false: the GELU tail compiled out as well (gemm_f8mx_kernel's emitting instances).
template <bool EMIT = true, bool GELU = true>
__device__ __forceinline__ void store_tile(const GemmArgs &p, int64_t split, int64_t m0, int64_t n0, int ty, int tx,
                                           float (&acc)[TM][TN]) {
    const bool partial = p.splits > 1;
    float *const C = partial ? p.part + split * p.M * p.N : p.C;
    const int64_t ldc = partial ? p.N : p.ldc, ctot = partial ? p.N : p.ctot, coff = partial ? 0 : p.coff;
    const int64_t nb = n0 + tx * TN;
    if (!partial && p.ep != nullptr) {  // fused BN + activation (split-K applies it in the reduction)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int64_t ch = p.coff + min<int64_t>(nb + j, p.N - 1);
#pragma unroll
            for (int i = 0; i < TM; ++i) acc[i][j] = epi(p.ep, p.ep_act, p.ep_lo, p.ep_hi, ch, acc[i][j]);
        }
    }
    const float pb = partial ? 0.0f : post_bias(p);
    const GemmArgs &q = p;
    // word-image emission from each final value (the split-K reduction emits instead)
    const bool emit = EMIT && !partial && p.em.w != nullptr;
    const EmitCtx ec = EMIT ? emit_ctx(p) : EmitCtx{};
    uint32_t sehi = 0;
    auto fin1 = [&](int64_t o, float v) {
        if (partial) return v;
        v = post1<GELU>(q, o, v, pb);
        if (emit) emit1(q, ec, o, v, sehi);
        return v;
    };
    auto fin4 = [&](int64_t o, float4 v) {
        if (partial) return v;
        v = post4<GELU>(q, o, v, pb);
        if (emit) emit4(q, ec, o, v, sehi);
        return v;
    };
    if (!p.nchw) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int64_t m = m0 + ty * TM + i;
            if (m >= p.M) continue;
            if (nb + TN <= p.N && ((ldc & 3) == 0) && ((((uintptr_t)C) & 15) == 0)) {
                *reinterpret_cast<float4 *>(&C[m * ldc + nb]) =
                    fin4(m * ldc + nb, make_float4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]));
            } else {
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    if (nb + j < p.N) C[m * ldc + nb + j] = fin1(m * ldc + nb + j, acc[i][j]);
            }
        }
    } else {
        // NCHW: the thread's 4 rows are 4 consecutive pixels; when they lie in one image and
        // start 16-B aligned, each output channel gets one float4 store.
        const int64_t mb = m0 + ty * TM;
        const int64_t img = mb / p.hw, pix = mb - img * p.hw;
        const bool vec = (pix + TM <= p.hw) && (mb + TM <= p.M) && ((p.hw & 3) == 0) &&
                         ((((uintptr_t)C) & 15) == 0);
        if (vec) {
#pragma unroll
            for (int j = 0; j < TN; ++j)
                if (nb + j < p.N) {
                    const int64_t o = (img * ctot + coff + nb + j) * p.hw + pix;
                    *reinterpret_cast<float4 *>(&C[o]) = fin4(o, make_float4(acc[0][j], acc[1][j], acc[2][j], acc[3][j]));
                }
        } else {
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int64_t m = mb + i;
                if (m >= p.M) continue;
                const int64_t im = m / p.hw, px = m - im * p.hw;
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    if (nb + j < p.N) {
                        const int64_t o = (im * ctot + coff + nb + j) * p.hw + px;
                        C[o] = fin1(o, acc[i][j]);
                    }
            }
        }
    }
    if (emit) wave_max_atomic(p.em.invalid + 5, sehi);
}

}  // namespace fp8a
