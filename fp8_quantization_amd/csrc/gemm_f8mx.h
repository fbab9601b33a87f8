// gemm_f8mx.h -- the E4M3 fast path with matrix-core accumulation.  DESIGN.md §3a.
//
// Same arithmetic as gemm_fast_kernel<.., TM_F8>: for on-grid E4M3 operands with
// s2n and per-product quantization (v9:51-113), each term is
//     Q_R(V'(s_a, m_a, m_b) * c_b * |c_a|)  =  2^(7-bR) * e4m3(V' * c_b / scale_a),
// scale_a = 2^(7-bR) / |c_a|, where V' = min(sig_a sig_b - T[m_a][m_b] 2^-M, pre-clamp bound of
// its binade) is an LDS table value and e4m3() is gfx950's scaled fp8 conversion (RNE; the bR
// grid is the OCP e4m3 grid scaled by 2^(7-bR), subnormal band included).
//
// Summation on the matrix core: the fp8 codes are not decoded and added on the VALU; per 16-row
// block and staged tile one v_mfma_scale_f32_16x16x128_f8f6f4 multiplies the wave's 2048 codes
// (16 rows x 8 K-steps x 16 columns) by a constant 0/1 selection operand S, so that
//     D[m][n] += the 8 K-steps' codes of output (row m of the block, column n of the wave).
// Products with 1.0 and 0 are exact and D is fp32 in units of 2^(7-bR): the sum differs from an
// in-order fp32 sum only by accumulation order, inside the reference's own order freedom
// (v9:113, torch's sum) and the 1e-5 * sum|term| bar.
//
// The table holds bf16 PAIRS V'(row, code0), V'(row, code1): V' has at most 8 significant bits
// and the pre-clamp bound 1.8671875 x binade is bf16-exact (any bound in (1.8125, 1.875) x
// binade rounds like the reference's saturating mantissa, F6, and its subnormal top tie).  B
// codes are 0-7 = m_b and 8 = a zero B (entry +0).  c_b = s_b 2^e_b is applied as one packed
// 16-bit integer add on the pair (v_pk_add_u16 of (s_b << 15) + (e_b << 7) per half: exponent
// add and sign flip, no carry between the halves), and the pair goes straight into the bf16
// form of the scaled conversion.
//
// Tile table.  c_b depends only on the column, so the packed add is done ONCE per staged K-step
// and column pair for all 16 rows (8 s_a + m_a), not once per product: each staged tile builds
// tt[kk][tx][row][j] = V'(row, pair 2 tx + j) (+) c_b (2 KiB per K-step) from the static table,
// and the math loop reads, per A element, 4 columns per ds_read_b64 at (row offset | column
// block) + kk * stride: one v_and_or per A element (16 columns), one conversion per product
// pair, no packed add.  The build's stores are conflict-free because odd K-steps sit 16 banks
// over (stride 528 words); the math loop's reads are conflict-free because each 32-lane group
// holds an even and an odd K-step (64-bank ds_read_b64 banking).  The tile is 128 rows x 64
// columns, so each table build serves 128 rows (the VALU is the limit: per 8192 products a
// wave spends 64 conversions at ~2.7x an add, and the build's packed adds are the largest
// remaining share -- DESIGN.md §3a).
//
// Operands are decoded ONCE per launch by two pre-pass kernels (xm_decode_a / xm_decode_b):
// an A element becomes one 32-bit word (cvt scale exponent << 23 | table row offset; the
// conversion reads only the scale's exponent field), a B column pair one (addend pair, pair
// block offset) uint2.  The GEMM's staging is then a gather and stores (a 3x3 conv gathers
// each input element 9 times).  The pre-passes also carry the fallback checks (off-grid
// operand, exactness window, e4m3 scale range, bias window) into the launch's flag word.
//
// Static table layout [pair (code0 + 9 code1)][m_a] u32 for s_a = + (a negative A row is the same
// pair with the sign bits flipped, folded into the build's addend); zero A operands take scale
// 2^127 (the conversion returns 0), so their row is irrelevant.
//
// E5M2 (XF = 1, round 4) runs the same kernel: the E5M2 result grid of bias bR (binades from
// 2^(1-bR), 2 mantissa bits, subnormal step 2^(-1-bR)) is the OCP e5m2 (bf8) grid scaled by
// 2^(15-bR), so the conversion is v_cvt_scalef32_pk_bf8_bf16 with scale 2^(15-bR-e_a), the codes
// enter the MFMA as bf8 (cbsz = 1) against the same e4m3 selection operand, and the sums are in
// units of 2^(15-bR).  V' = sig_a sig_b - T 2^-2 has at most 6 significant bits (bf16-exact);
// its pre-clamp bound is 1.6875 x binade: any bound in (1.625, 1.75) rounds to the saturating
// mantissa 1.75 (F6) and keeps the subnormal band's top binade (x / step = 2 V') below the tie at
// 3.5 that the reference clamps to the largest subnormal 3.  Rows are 8 s_a + m_a with m_a < 4;
// B codes m_b < 4 and 8 = zero.  A term past the e5m2 range converts to inf / NaN and the tile
// falls back, as for E4M3.
#pragma once
#include "fp8approx_common.h"

namespace fp8a {

typedef int xm_v8i __attribute__((ext_vector_type(8)));
typedef float xm_v16f __attribute__((ext_vector_type(16)));
typedef float xm_v4f __attribute__((ext_vector_type(4)));
typedef short xm_s2 __attribute__((ext_vector_type(2)));
typedef unsigned short xm_u2 __attribute__((ext_vector_type(2)));
typedef __bf16 xm_b2 __attribute__((ext_vector_type(2)));

constexpr int XM_NPAIR = 81;
constexpr int XM_LUT_WORDS = XM_NPAIR * 8;  // [pair][m_a] u32 (s_a = +), 2.5 KiB
constexpr uint32_t XM_ROW_SHIFT = 3, XM_ROW_MASK = 0x78u;  // A word bits 3-6: row * 8 = byte offset in a column block
constexpr int XBK = 8;                         // K-steps per staged tile
constexpr int XM_TTK = 16 * 32 + 16;           // tile-table words per K-step: [tx 16][row 16][j 2] + bank shift
// (XM_ZERO_WORD, the word of A = 0: fp8approx.hip, next to the word-image emission)
constexpr int XM_CP = BN + 1;  // the 64-column epilogue slices of the other kernels: [64][BN + 1] floats

// Result-grid formats of the matrix-core path: XF 0 = E4M3 (OCP e4m3, bias 7), 1 = E5M2 (OCP e5m2 /
// bf8, bias 15), 2 = E5M2 with the halved-block form for the grid's top binade (below).
template <int XF>
struct XmFmt {
    static constexpr int M = XF ? 2 : 3;
    static constexpr int XB = XF ? 15 : 7;  // the OCP format's exponent bias
};
// E5M2: the launch needs the halved-block form when its largest A element times its largest B
// element can reach the result grid's top binade 31 - bR: e_a + e_b + 1 >= 31 - bR, i.e. the
// smallest A scale exponent se <= 112 + max e_b.  The pre-passes record both extremes in the
// workspace head (xm_decode_a: 255 - min se, xm_decode_b: max e_b + 128; 0 = none); without the A
// pre-pass (fp32 staging) the A grid's top binade (plus the one the quantizer's rounding can add)
// stands in.  The plain form runs every tile; a tile of it that met a NaN (a term past the e5m2
// range) goes to the halved-block form when the extremes allow the top binade (UT_HALF), else
// straight to the exact kernel.
__device__ __forceinline__ bool xm_needs_halving(const GemmArgs &p, bool af32, int bA, int bR) {
    const uint32_t a = __hip_atomic_load(p.flag + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t b = __hip_atomic_load(p.flag + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (b == 0u) return false;  // every B element is zero
    const int se_min = af32 ? 110 + bA - bR : (a == 0u ? 1000 : 255 - (int)a);
    return se_min <= 112 + (int)b - 128;
}
// The halved-block form's tile gate: the plain form raised FB_HALF and marked a unit of this tile
// UT_HALF (every tile without the unit marks)
__device__ __forceinline__ bool xm_half_gate(const GemmArgs &p, int64_t m0, int rows, int64_t n0, int cols) {
    if ((__hip_atomic_load(p.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & FB_HALF) == 0u) return false;
    if (p.utile == nullptr) return true;
    const int64_t r1 = (min(m0 + rows, p.M) - 1) >> 6, c1 = (min(n0 + cols, p.N) - 1) >> 6;
    bool any = false;
    for (int64_t r = m0 >> 6; r <= r1; ++r)
        for (int64_t c = n0 >> 6; c <= c1; ++c) any |= (p.utile[r * p.nuc + c] & UT_HALF) != 0;
    return any;
}
__host__ __device__ constexpr int xm_xbias(int Mw) { return Mw == 2 ? 15 : 7; }

// Tile shapes of gemm_f8mx_kernel<NCG, RB, AF32>: 4 waves; NCG column groups of 16 columns x
// (4 / NCG) row groups of RB 16-row blocks.  NCG = 4 (128 x 64) is the round-2 kernel; the narrow
// shapes (128 x 32, 256 x 16) serve layers with N = 16 / 24 / 32 / 96 / 160 (MobileNetV2's
// projections), where a 64-column tile converted up to 4x the products the layer has.
// A words in LDS: [kk / 2][row][kk % 2] -- one ds_write_b64 stores (and one ds_read_b64 reads) a
// row's words of a K-step pair; the pair arrays sit 32 banks apart, so the math loop's reads
// (lane groups of K-step pairs g, g + 1) and the staging's stores are conflict-free.
// B operand by LDS-DMA (option build, round 6; off): the staged tile's B pair words (XBK x TXN
// 16-byte chunks, each read by the 4 build units of its column block) go global -> LDS by
// global_load_lds_dwordx4 instead of through 8 prefetch VGPRs per thread.  The plain 128 x 64
// instance then fits 6 waves / SIMD (76 VGPRs, no spill) -- and ran 4 % slower: ResNet-18 12,175
// vs 12,673 images/s, ResNet-50 E4M3 4,671 vs 4,857 (profiles/r06_bdma/)
#ifndef XM_BDMA
#define XM_BDMA 0
#endif
template <int NCG, int RB>
struct XmCfg {
    static constexpr int NT = 256;
    static constexpr int BNT = 16 * NCG;          // tile columns
    static constexpr int RG = 4 / NCG;            // row groups
    static constexpr int BMT = 16 * RB * RG;      // tile rows
    static constexpr int TXN = 4 * NCG;           // 4-column blocks of the tile table
    // tile-table words per K-step: [tx][row 16][j 2] + a shift putting odd K-steps >= 16 banks over
    static constexpr int TTK = TXN * 32 + 16;
    static constexpr int AWQ = 2 * BMT + 32;
    static constexpr int APR = BMT / 64;          // A rows per staging thread
    static constexpr int NBU = 32 * TXN;          // table-build units per staged tile (8 K-steps x TXN x 4)
    static constexpr int BU = (NBU + NT - 1) / NT;
    static_assert(NT % (8 * TXN) == 0, "build units: one column block per thread");
    static constexpr int SR = 4096 / BNT;         // epilogue slab: SR rows x BNT columns = 16 outputs per thread
    static constexpr int CP = BNT + 1;
    struct Stage {
        uint32_t tt[XBK][TTK];  // c_b-applied pairs [kk][tx][row][j] (first: its byte offsets are the reads' immediates)
        uint32_t lut[XM_LUT_WORDS];
        uint32_t aw[XBK / 2][AWQ];  // A(m, k)'s word: cvt scale exponent << 23 | row << 3
#if XM_BDMA
        uint4 bw[XBK * TXN];        // the staged tile's B pair words [kk][column block], by LDS-DMA
#endif
    };
    union Smem {
        Stage st;
        float ct[SR * CP];  // epilogue transpose slab, aliased on the staging LDS
    };
    static_assert(NCG == 1 || NCG == 2 || NCG == 4, "column groups");
    static_assert(BMT % 64 == 0 && BMT % SR == 0, "tile rows");
    static_assert((TTK % 64) >= 16 && (TTK % 64) <= 48, "odd K-steps of the table build must not share banks");
};

// Exactness / range window shared by the pre-passes (as bias_ok in gemm_fast_kernel)
__device__ __forceinline__ bool xm_bias_ok(int b) { return b >= -100 && b <= 120; }

// Table word e of layout [pair][m_a]: the bf16 pair V'(m_a, code0), V'(m_a, code1), s_a = +, for
// M mantissa bits (3: E4M3, 2: E5M2; rows / codes >= 2^M are never addressed).
__device__ __forceinline__ uint32_t xm_lut_word(const TablePack &tab, int e, int M) {
    const int pr = e >> 3, ma = e & 7, n = 1 << M;
    const float ulp = M == 3 ? 0.125f : 0.25f;
    // Q_R's pre-clamp in bf16: any bound in (1.8125, 1.875) (M = 3) / (1.625, 1.75) (M = 2) x
    // binade rounds like the reference's saturating mantissa (and the subnormal top tie rounding down)
    const float bound = M == 3 ? 1.8671875f : 1.6875f;
    uint32_t w = 0;
    if (ma >= n) return 0u;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int cd = h ? (pr / 9) : (pr % 9);
        if (cd >= n) continue;  // zero B (code 8): +0
        const float t = (float)tab.raw[ma * n + cd];
        float v = __fmaf_rn(1.0f + ulp * ma, 1.0f + ulp * cd, -t * ulp);  // exact, <= 2M + 2 bits
        v = fminf(v, __uint_as_float(__float_as_uint(v) & 0x7F800000u) * bound);
        w |= (__float_as_uint(v) >> 16) << (16 * h);
    }
    return w;
}

// A element -> word: bits 23-30 the cvt scale exponent se (scale 2^(se-127) = 2^(xb-bR-e_a), xb the
// OCP format's bias: 7 e4m3, 15 e5m2), bits 3-6 the tile-table row (8 s_a + m_a); zeros
// XM_ZERO_WORD.  ok = on the (M, bA) grid, inside the exactness window and the scale range.
__device__ __forceinline__ uint32_t xm_word_a(float x, int M, int xb, uint32_t emnA, int bR, bool &ok) {
    float c;
    uint32_t mc;
    ok = stage_decode(x, M, emnA, true, c, mc);
    const uint32_t cb = __float_as_uint(c);
    const int se = 254 + xb - bR - (int)((cb >> 23) & 0xFFu);
    if ((cb & 0x7FFFFFFFu) == 0u) return XM_ZERO_WORD;
    ok = ok && se >= 1 && se <= 252;
    return ((uint32_t)min(max(se, 1), 252) << 23) | (((cb >> 31) * 8u + mc) << XM_ROW_SHIFT);
}

constexpr int TT_RS = 68;  // floats per m_a row of a K-step's table (64 columns + 4: conflict-free
                           // ds_read_b128 of 16 rows by a lane group)
constexpr uint32_t TT_EXP = 0xFF800000u;  // sign + exponent field of c (its mantissa is zero)
// gemm_tt_kernel's A word (gemm_tt.h): c_a's sign and exponent bits (mantissa field zero) |
// m_a x the table row stride; zeros 0.  ok = on the (M, bA) grid and inside the exactness window.
__device__ __forceinline__ uint32_t tt_word_a(float x, int M, uint32_t emnA, bool &ok) {
    float c;
    uint32_t mc;
    ok = stage_decode(x, M, emnA, true, c, mc);
    const uint32_t cb = __float_as_uint(c);
    if ((cb & 0x7FFFFFFFu) == 0u) return 0u;
    return (cb & TT_EXP) | (mc * (uint32_t)(4 * TT_RS));
}

// gemm_tt16_kernel's operand formats (gemm_tt16.h)
constexpr int TT16_XK = 4;                  // K-steps per staged tile (= the 4 lane groups)
constexpr int TT16_RS = 34;                 // u32 per m_a row of a K-step's table: 32 column pairs + 2
constexpr int TT16_KS = 16 * TT16_RS;       // u32 per K-step (2176 B)
constexpr uint32_t TT16_RSH = 2 * TT16_RS;  // the A word's row offset unit: 2 bytes
constexpr uint32_t TT16_EXP2 = 0xFC00FC00u; // sign + exponent fields of an f16 pair
constexpr int TT16_IMG = 2048;             // u32 offset of the f16 image in the table region (after gemm_tt_kernel's)

typedef _Float16 tt16_h2 __attribute__((ext_vector_type(2)));
typedef _Float16 tt16_h8 __attribute__((ext_vector_type(8)));
typedef float tt16_f4 __attribute__((ext_vector_type(4)));


// f16 bits of sign * 2^e (normal range)
__device__ __forceinline__ uint32_t tt16_pow2(int e, uint32_t sign) { return sign | ((uint32_t)(e + 15) << 10); }

// A word (wfmt 2): c_a' = c_a 2^(bA-1) in the sign / exponent fields of both f16 halves, m_a x
// TT16_RSH (the row's byte offset / 2) in the low half's mantissa field; zeros 0.  ok = on the
// (4, bA) grid; win is cleared by c_a' > 2^7 (a value more than one binade above the format's
// top one -- the quantizer's rint bias allows one -- is outside the f16 window).
__device__ __forceinline__ uint32_t tt16_word_a(float x, uint32_t emnA, int bA, bool &ok, bool &win) {
    float c;
    uint32_t mc;
    ok = stage_decode(x, 4, emnA, true, c, mc);
    const uint32_t cb = __float_as_uint(c);
    if ((cb & 0x7FFFFFFFu) == 0u) return 0u;
    const int e = (int)((cb >> 23) & 0xFFu) - 127 + bA - 1;  // c_a' = c_a 2^(bA-1): in [-4, 7] on the grid
    ok = ok && e >= -14 && e <= 15;
    win = win && e <= 7;
    const uint32_t h = tt16_pow2(min(max(e, -14), 15), (cb >> 16) & 0x8000u);
    return (h << 16) | h | (mc * TT16_RSH);
}

// A word of the v5 matrix-core form (xm_decode_a, wfmt 4; gemm_v5mx.h): (sign << 15 | code << 5) in both halves
__device__ __forceinline__ uint32_t v5_word_a(float v, const DFmt &f) {
    int e, m;
    exact_dec(v, f, true, e, m);
    const uint32_t h = (v < 0.0f ? 0x8000u : 0u) | ((uint32_t)(e * (1 << f.M) + m) << 5);
    return h * 0x10001u;
}

// xm_decode_a's record for xm_needs_halving: 255 - (the smallest se of its nonzero E5M2 words)
__device__ __forceinline__ void xm_record_se(const GemmArgs &p, uint32_t sehi) {
    if (p.Mw == 2 && p.wfmt == 0) wave_max_atomic(p.flag + 1, sehi);
}

// A pre-pass, one (image | row) per blockIdx.y step.  conv: the group's channel slice of x
// [Bn][Cin][H][W] (channels cbase..cbase+aw_c) -> words [Bn][aw_c][awH][awW], x at (awph, awpw)
// inside a border of zero words (the padding the convolution reads, so the wave-independent
// kernel gathers without bounds checks; no border for gemm_f8mx_kernel); matrix: A [M][lda] ->
// words [M][awld] (columns >= K zero words).
#if FP8A_OWN_F8MX_DECODE
__global__ __launch_bounds__(256) void xm_decode_a(const GemmArgs p) {
    // fused input quantization: A = fq(X) with the quantizer's own bias, which becomes bA
    const float fmx = p.fqin.mx ? *p.fqin.mx : 0.0f;
    const float fbias = p.fqin.mx ? fq_bias(fmx, p.fqin.E, p.fqin.M) : 0.0f;
    const int bA = p.fqin.mx ? (int)fbias : *p.bA, bR = *p.bR;
    if (p.fqin.mx && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
        *p.fq_bias = fbias;
        *p.fq_ibias = bA;
    }
    // gated (the input's word image was emitted by the previous launch, fp8a_conv2d_chain): the
    // words are already there unless an element left the window (the image's header word)
    if (p.gate != nullptr && __hip_atomic_load(p.gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
        // (the emitting launch recorded its words' smallest scale exponent in the image header)
        if (p.Mw == 2 && p.wfmt == 0 && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
            atomicMax(p.flag + 1, p.gate[5]);
        return;
    }
    const uint32_t emnA = (uint32_t)(128 - bA) << 23;
    const bool biasbad = !(xm_bias_ok(bA) && xm_bias_ok(bR));  // every output unit falls back
    bool bad = biasbad, win = true;
    // conv: a bad input element marks its image's output rows; matrix: its row
    const int64_t orows = p.conv ? p.Ho * p.Wo : 1;
    uint32_t *const out = const_cast<uint32_t *>(p.aw);
    const int64_t hw = p.H * p.W;
    const int64_t rows = p.conv ? p.M / (p.Ho * p.Wo) : p.M, cols = p.conv ? p.aw_c * p.awH * p.awW : p.awld;
    uint32_t sehi = 0;  // 255 - the smallest se of this thread's nonzero E5M2 words (xm_record_se)
    const DFmt fv5 = dfmt(p.E, p.Mw, bA, false);  // (wfmt 4: the v5 decode, clip_OF)
    auto word = [&](float v, bool &ok) {
        if (p.fqin.mx) v = fq_apply(v, fmx, fbias, p.fqin.M, p.fqin.S);
        if (p.wfmt == 4) return v5_word_a(v, fv5);
        if (p.wfmt == 2) return tt16_word_a(v, emnA, bA, ok, win);
        if (p.wfmt) return tt_word_a(v, p.Mw, emnA, ok);
        const uint32_t w = xm_word_a(v, p.Mw, xm_xbias(p.Mw), emnA, bR, ok);
        sehi = max(sehi, word_sehi(w));
        return w;
    };
    const uint32_t zw = p.wfmt ? 0u : XM_ZERO_WORD;  // the word of a zero (padding, columns >= K)
    auto st1 = [&](int64_t i, uint32_t w) { out[i] = w; };
    auto st4 = [&](int64_t i, uint4 w) { *reinterpret_cast<uint4 *>(out + i) = w; };  // i % 4 == 0
    if (p.conv && (p.awph | p.awpw)) {  // zero-bordered image (< 2^30 words, run_gemm): 32-bit index math
        // interior: four input elements per thread step along W, one 16-B load and one 16-B store
        // when W % 4 == 0 (run_gemm's word_image aligns the interior rows), else one element;
        // then the border words (zero) of every plane
        const uint32_t uW = (uint32_t)p.W, uH = (uint32_t)p.H, Wp = (uint32_t)p.awW, Hp = (uint32_t)p.awH;
        const uint32_t hwin = uH * uW, ph = (uint32_t)p.awph, pw = (uint32_t)p.awpw, pr = Wp - uW - pw;
        const uint32_t nin = (uint32_t)p.aw_c * hwin;
        const bool v4 = (uW % 4 == 0) && (Wp % 4 == 0) && (pw % 4 == 0) &&
                        (((uintptr_t)(p.X + p.cbase * hw) & 15) == 0) && ((p.Cin * hw) % 4 == 0) &&
                        (((uintptr_t)out & 15) == 0) && (cols % 4 == 0);
        const uint32_t per = v4 ? 4u : 1u, nb = 2 * ph * Wp + (pw + pr) * uH;  // border words per plane
        const uint32_t tstride = gridDim.x * blockDim.x, t0 = blockIdx.x * blockDim.x + threadIdx.x;
        for (int64_t r = blockIdx.y; r < rows; r += gridDim.y) {
            const float *in = p.X + (r * p.Cin + p.cbase) * hw;
            const int64_t o = r * cols;
            bool badr = false;
            for (uint32_t e = per * t0; e < nin; e += per * tstride) {
                const uint32_t c = e / hwin, t = e - c * hwin, hy = t / uW, wx = t - hy * uW;
                const int64_t d = o + (c * Hp + hy + ph) * Wp + pw + wx;
                if (v4) {
                    const float4 v = *reinterpret_cast<const float4 *>(in + e);
                    bool ok0 = true, ok1 = true, ok2 = true, ok3 = true;
                    st4(d, make_uint4(word(v.x, ok0), word(v.y, ok1), word(v.z, ok2), word(v.w, ok3)));
                    badr |= !(ok0 && ok1 && ok2 && ok3);
                } else {
                    bool ok = true;
                    st1(d, word(in[e], ok));
                    badr |= !ok;
                }
            }
            if (badr) fb_rows(p, r * orows, (r + 1) * orows);
            bad |= badr;
            for (uint32_t j = t0; j < (uint32_t)p.aw_c * nb; j += tstride) {
                const uint32_t c = j / nb, t = j - c * nb;
                uint32_t row, col;
                if (t < 2 * ph * Wp) {  // top / bottom rows
                    const uint32_t rr = t / Wp;
                    row = rr < ph ? rr : uH + rr;
                    col = t - rr * Wp;
                } else {  // left / right margins of the interior rows
                    const uint32_t u = t - 2 * ph * Wp, rr = u / (pw + pr), sc = u - rr * (pw + pr);
                    row = ph + rr;
                    col = sc < pw ? sc : uW + sc;
                }
                st1(o + (c * Hp + row) * Wp + col, zw);
            }
        }
        if (__syncthreads_or(bad ? 1 : 0) && threadIdx.x == 0) atomicOr(p.flag, fb_bits(p, biasbad));
        if (__syncthreads_or(win ? 0 : 1) && threadIdx.x == 0) atomicOr(p.flag, 4u);  // gemm_tt16_kernel's window (A)
        xm_record_se(p, sehi);
        return;
    }
    // 16-B form: every row start 16-B aligned and the valid columns a multiple of 4 (all the
    // conv images here; matrix rows when lda and K are)
    const int64_t lim0 = p.conv ? cols : p.K, istride = p.conv ? p.Cin * hw : p.lda;
    const float *in0 = p.conv ? p.X + p.cbase * hw : p.A;
    const bool vec = (lim0 % 4 == 0) && (cols % 4 == 0) && (istride % 4 == 0) && (((uintptr_t)in0 & 15) == 0) &&
                     (((uintptr_t)out & 15) == 0);
    if (vec) {
        // the (row, 4-column chunk) grid flattened over every thread of the launch (a row of a
        // matrix A is often shorter than the block's 1024 columns: ViT's 768); (row, chunk)
        // advanced by the thread count's quotient and remainder, so no division in the loop.
        // (< 2^30 words: run_gemm's fits32)
        const uint32_t c4n = (uint32_t)(cols / 4), lim4 = (uint32_t)(lim0 / 4), nq = (uint32_t)rows * c4n;
        const uint32_t nthr = gridDim.x * gridDim.y * blockDim.x;
        const uint32_t tid = (blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x;
        // XU chunks per thread step, their loads issued before any word is computed (a thread
        // with one chunk in flight left the pre-pass latency-bound: 1.5 TB/s on MobileNetV2's
        // expansion inputs)
        constexpr int XU = 4;
        const uint32_t dr = nthr / c4n, dc = nthr - dr * c4n;
        uint32_t r = tid / c4n, c = tid - r * c4n;
        for (uint32_t q = tid; q < nq; q += XU * nthr) {
            float4 v[XU];
            uint32_t rr[XU], cc[XU];
#pragma unroll
            for (int u = 0; u < XU; ++u) {
                rr[u] = r;
                cc[u] = c;
                if (q + u * nthr < nq && c < lim4)
                    v[u] = *reinterpret_cast<const float4 *>(in0 + (int64_t)r * istride + 4 * c);
                c += dc;
                r += dr;
                if (c >= c4n) {
                    c -= c4n;
                    ++r;
                }
            }
#pragma unroll
            for (int u = 0; u < XU; ++u) {
                if (q + u * nthr >= nq) break;
                uint4 w = make_uint4(zw, zw, zw, zw);
                if (cc[u] < lim4) {
                    bool ok0 = true, ok1 = true, ok2 = true, ok3 = true;
                    w = make_uint4(word(v[u].x, ok0), word(v[u].y, ok1), word(v[u].z, ok2), word(v[u].w, ok3));
                    if (!(ok0 && ok1 && ok2 && ok3)) {
                        fb_rows(p, (int64_t)rr[u] * orows, ((int64_t)rr[u] + 1) * orows);
                        bad = true;
                    }
                }
                st4((int64_t)rr[u] * cols + 4 * cc[u], w);
            }
        }
    } else {
        for (int64_t r = blockIdx.y; r < rows; r += gridDim.y) {
            const float *in = p.conv ? p.X + (r * p.Cin + p.cbase) * hw : p.A + r * p.lda;
            const int64_t lim = p.conv ? cols : p.K;
            const int64_t o = r * cols;
            bool badr = false;
            for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cols;
                 i += (int64_t)gridDim.x * blockDim.x) {
                bool ok = true;
                st1(o + i, (i < lim) ? word(in[i], ok) : zw);
                badr |= !ok;
            }
            if (badr) fb_rows(p, r * orows, (r + 1) * orows);
            bad |= badr;
        }
    }
    if (__syncthreads_or(bad ? 1 : 0) && threadIdx.x == 0) atomicOr(p.flag, fb_bits(p, biasbad));
    if (__syncthreads_or(win ? 0 : 1) && threadIdx.x == 0) atomicOr(p.flag, 4u);  // gemm_tt16_kernel's window (A)
    xm_record_se(p, sehi);
}
#else
__global__ void xm_decode_a(const GemmArgs p);
#endif  // FP8A_OWN_F8MX_DECODE

// B pre-pass: per (k, pair Q) of the padded [Kpad][npad / 2] pair grid, the addend pair
// ((s_b << 15) + (e_b << 7) per bf16 half, 0 for a zero B) and the pair's byte offset in the
// static table ((code0 + 9 code1) * 32); out-of-range elements are zeros.
#if FP8A_OWN_F8MX_DECODE
__global__ __launch_bounds__(256) void xm_decode_b(const GemmArgs p, int64_t kpad) {
    // (af32: A's bias -- maybe the fused input quantizer's, not written yet -- is checked by the GEMM)
    const int bA = p.af32 ? 0 : *p.bA, bR = *p.bR;
    const bool biasbad = !(xm_bias_ok(bA) && xm_bias_ok(bR));
    bool bad = biasbad;
    const int64_t hq = p.npad / 2, n = kpad * hq;
    uint2 *const bq = const_cast<uint2 *>(p.bqw);
    if (blockIdx.x == 0)  // the table image every GEMM workgroup copies into LDS
        for (int e = threadIdx.x; e < XM_LUT_WORDS; e += blockDim.x) const_cast<uint32_t *>(p.lutw)[e] = xm_lut_word(p.tab, e, p.Mw);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int64_t k = i / hq, q = i - k * hq;
        float c[2];
        uint32_t mc[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int64_t col = 2 * q + h;
            c[h] = 0.0f;
            mc[h] = 0;
            if (k < p.K && col < p.N) {
                const int bb = p.bB[col * p.bBs];
                const bool ok = stage_decode(p.B[k * p.sbk + col * p.sbn], p.Mw, (uint32_t)(128 - bb) << 23, true,
                                             c[h], mc[h]) && xm_bias_ok(bb);
                if (!ok) fb_col(p, col);
                bad |= !ok;
            }
        }
        uint32_t add = 0, code[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t cb = __float_as_uint(c[h]);
            if ((cb & 0x7FFFFFFFu) == 0u) {
                code[h] = 8u;
            } else {
                code[h] = mc[h];
                const uint32_t eb = ((cb >> 23) & 0xFFu) - 127u;  // mod 2^9 in the field below
                add |= ((((cb >> 31) << 15) + (eb << 7)) & 0xFFFFu) << (16 * h);
            }
        }
        bq[i] = make_uint2(add, (code[0] + 9u * code[1]) * 32u);
    }
    if (p.Mw == 2 && p.ebr != nullptr) {  // E5M2: each (K-step, 16-column group)'s exponent range
        const int64_t ng = p.npad / 16;
        uint32_t bmax = 0;
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < kpad * ng; i += stride) {
            const int64_t k = i / ng, g = i - k * ng;
            int emax = -128, emin = 127;
            for (int j = 0; j < 16 && k < p.K; ++j) {
                const int64_t col = 16 * g + j;
                if (col >= p.N) break;
                float c;
                uint32_t mc;
                stage_decode(p.B[k * p.sbk + col * p.sbn], p.Mw, (uint32_t)(128 - p.bB[col * p.bBs]) << 23, true, c, mc);
                const uint32_t cb = __float_as_uint(c);
                if ((cb & 0x7FFFFFFFu) == 0u) continue;
                const int e = (int)((cb >> 23) & 0xFFu) - 127;
                emax = max(emax, e);
                emin = min(emin, e);
            }
            const_cast<uint16_t *>(p.ebr)[i] = (uint16_t)((emax + 128) | ((emin + 128) << 8));
            bmax = max(bmax, (uint32_t)(emax + 128));
        }
        wave_max_atomic(p.flag + 2, bmax);  // for xm_needs_halving
    }
    if (__syncthreads_or(bad ? 1 : 0) && threadIdx.x == 0) atomicOr(p.flag, fb_bits(p, biasbad));
}
#else
__global__ void xm_decode_b(const GemmArgs p, int64_t kpad);
#endif  // FP8A_OWN_F8MX_DECODE

#if FP8A_OWN_F8MX
// In-kernel clock of gemm_f8mx_kernel (diagnostic build only: -DFP8A_CLOCK_STAMP=1, tools/clock_probe.py):
// thread 0 of every workgroup adds its s_memtime and s_memrealtime (100 MHz) deltas; the clock the
// chip held = sum dt / sum dr x 100 MHz (MI355X_MICROARCH.md, DVFS give-back item 6).  Nothing
// else reads g_clk; the product build compiles no stamp.
#ifndef FP8A_CLOCK_STAMP
#define FP8A_CLOCK_STAMP 0
#endif
__device__ unsigned long long g_clk[3];
#if FP8A_CLOCK_STAMP
#define FP8A_CLK_BEGIN const uint64_t clk_t0 = __builtin_amdgcn_s_memtime(), clk_r0 = __builtin_amdgcn_s_memrealtime();
#define FP8A_CLK_END                                                                                   \
    if (threadIdx.x == 0) {                                                                            \
        const uint64_t clk_t1 = __builtin_amdgcn_s_memtime(), clk_r1 = __builtin_amdgcn_s_memrealtime(); \
        atomicAdd(&g_clk[0], (unsigned long long)(clk_t1 - clk_t0));                                   \
        atomicAdd(&g_clk[1], (unsigned long long)(clk_r1 - clk_r0));                                   \
        atomicAdd(&g_clk[2], 1ull);                                                                    \
    }
#else
#define FP8A_CLK_BEGIN
#define FP8A_CLK_END
#endif
#ifndef XM_WAVES
// register bound: 5 waves / SIMD (<= 96 VGPRs; the 128 x 64 instance needs 82).  At 6 waves (80
// VGPRs) that instance spilled 4-30 VGPRs to scratch inside its K loop, and a scratch load's vmcnt
// wait also waited for the tile prefetch issued before it (in-order vmcnt): ResNet-18 layer set
// 28.7 -> 25.5 ms, bench 11835 -> 12454 images/s at 5 waves (round 5)
#define XM_WAVES 5
#endif
// the plain instance (staged words, no emission), with the B operand by LDS-DMA: 76 VGPRs, no spill
// at 6 waves (the emitting / fp32-staging instances spill 7-28 there and stay at XM_WAVES).  (The
// bound is a trait: a conditional expression in __launch_bounds__ works too, but the macro splits
// on a template argument list's comma)
#ifndef XM_WAVES_PLAIN
#define XM_WAVES_PLAIN (XM_BDMA ? 6 : XM_WAVES)
#endif
template <bool AF32, bool EMIT> struct XmWaves { static constexpr int value = XM_WAVES; };
template <> struct XmWaves<false, false> { static constexpr int value = XM_WAVES_PLAIN; };
// The GEMM.  Tile BMT x BNT (XmCfg), 4 waves; wave wv = column group wc = wv % NCG (the 16
// columns 16 wc .. 16 wc + 15, column blocks tx = 4 wc + c of the tile table) and row group
// wr = wv / NCG (16 RB rows).  Math mapping: lane = (row r16 of each of the wave's RB 16-row
// blocks, K-step pair g of the 8-step tile).  Per A element (row, K-step): ONE v_and_or_b32 (row
// offset | the wave's column base + the K-step's table offset; block c in the reads' immediates),
// four ds_read_b64 (16 columns), eight conversions; per 16-row block and tile one 16x16x128 MFMA
// sums the 4 lane groups' 2 K-steps.  Operands are read through buffer descriptors: uniform
// K-step offsets in SGPRs, 32-bit lane offsets (run_gemm keeps the images below 2^32 bytes); the
// conv word image carries the zero padding (xm_decode_a), so the gather has no bounds checks.
//
// AF32: A is read as fp32 straight from its source (a 1x1 / unpadded conv's x, or the matrix A)
// and turned into its word while it is staged -- the fused input quantizer, the on-grid / window
// checks and the fallback marks included -- instead of by the xm_decode_a pre-pass.  That pass
// writes and re-reads 8 B per A element through HBM; staging-time decoding costs ~25 VALU
// operations per element per column tile, the cheaper choice up to a few column tiles (run_gemm).
template <int NCG, int RB, bool AF32, int XF, bool EMIT>
__global__ __launch_bounds__(256, (XmWaves<AF32, EMIT>::value)) void gemm_f8mx_kernel(const GemmArgs p) {
    using Cf = XmCfg<NCG, RB>;
    constexpr int XM = XmFmt<XF>::M, XB = XmFmt<XF>::XB;
    constexpr int NT = Cf::NT, BMT = Cf::BMT, BNT = Cf::BNT, TTK = Cf::TTK, APR = Cf::APR;
    constexpr int BU = Cf::BU, NBU = Cf::NBU, TXN = Cf::TXN, SR = Cf::SR, CP = Cf::CP;
    __shared__ __attribute__((aligned(16))) typename Cf::Smem smu;
    auto &sm = smu.st;
    FP8A_CLK_BEGIN

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wvu = __builtin_amdgcn_readfirstlane(wv);
    const int wc = wvu % NCG, wr = wvu / NCG;  // the wave's column group and row group
    const int64_t num_mt = (p.M + BMT - 1) / BMT;
    const int64_t tiles = num_mt * ((p.N + BNT - 1) / BNT);
    const int64_t bid = (int64_t)blockIdx.x % tiles, split = (int64_t)blockIdx.x / tiles;
    const int64_t m0 = (bid % num_mt) * BMT;
    const int64_t n0 = (bid / num_mt) * BNT;
    if (XF == 2 && !xm_half_gate(p, m0, BMT, n0, BNT)) return;  // (a tile the plain form completed)
    const int kbeg = (int)(split * p.kchunk), kend = (int)min(p.K, (int64_t)kbeg + p.kchunk), K32 = (int)p.K;
    const int bR = *p.bR;
    // AF32: the A operand's bias (the fused input quantizer's, written once for the gated kernels)
    float fmx = 0.0f, fbias = 0.0f;
    int bA = 0;
    bool abad = false, biasbad = false;
    if (AF32) {
        fmx = p.fqin.mx ? *p.fqin.mx : 0.0f;
        fbias = p.fqin.mx ? fq_bias(fmx, p.fqin.E, p.fqin.M) : 0.0f;
        bA = p.fqin.mx ? (int)fbias : *p.bA;
        if (p.fqin.mx && blockIdx.x == 0 && tid == 0) {
            *p.fq_bias = fbias;
            *p.fq_ibias = bA;
        }
        biasbad = !(xm_bias_ok(bA) && xm_bias_ok(bR));  // every output unit falls back
    }
    const uint32_t emnA = (uint32_t)(128 - bA) << 23;

    // table: copied from the launch's pre-computed image (xm_decode_b), 16-B per thread and step
    for (int e = 4 * tid; e < XM_LUT_WORDS; e += 4 * NT)
        *reinterpret_cast<uint4 *>(&sm.lut[e]) = *reinterpret_cast<const uint4 *>(&p.lutw[e]);

    // tile-table build units e = tid + NT u (NBU per tile): (m_a pair q4, column block btx,
    // K-step bkk[u]); the 8 lanes of a ds_write_b128 group are 4 q4 x an even and an odd K-step
    // (>= 16 banks apart)
    const uint32_t hq8 = (uint32_t)(p.npad / 2) * 8u;  // bytes per K-step of the B pair grid
    // (NT is a multiple of 8 TXN, so the unit's column block is the same for every u)
    const int q4 = tid & 3, btx = (tid >> 3) % TXN;
    // unit u = the thread's unit 0 moved by u * NT: (NT a multiple of 8 TXN) the same column block,
    // K-step + u * BKU -- the per-unit offsets are uniform (soffset / immediates), one VGPR each
    constexpr int BKU = 2 * (NT / (8 * TXN));
    const int bkk0 = 2 * (tid / (8 * TXN)) + ((tid >> 2) & 1);
    const uint32_t boff0 = (uint32_t)(kbeg + bkk0) * hq8 + (uint32_t)(n0 / 2 + 2 * btx) * 8u;  // pair 2 btx: 16-B aligned
    const bool build = NBU % NT == 0 || tid < NBU;  // (NCG = 1: half the threads build)
#if XM_BDMA
    // this thread's DMA chunk (tid < XBK TXN): K-step kbeg + tid / TXN, pairs n0 / 2 + 2 (tid % TXN) + {0, 1}
    const float *bsrc = reinterpret_cast<const float *>(p.bqw) +
                        ((size_t)(kbeg + tid / TXN) * (hq8 / 4) + (size_t)(n0 / 2 + 2 * (tid % TXN)) * 2);
    (void)boff0;
#else
    const __amdgpu_buffer_rsrc_t brsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint2 *>(p.bqw), (short)0, -1, 0x00020000);
#endif

    // A staging: thread = (rows arow + 64 i, K-step pair akp), K-steps 2 akp + r.  conv: lane =
    // row (consecutive pixels), akp = the wave (wave-uniform: the k -> (c, ky, kx) split and the
    // word offset run on the scalar unit); matrix: four threads per row.  Rows past M re-read row
    // M - 1 (store_tile drops them).
    const int arow = p.conv ? lane : (tid >> 2), akp = p.conv ? wvu : (tid & 3);
    uint32_t aoff[APR];
    const uint32_t phw = AF32 ? (uint32_t)(p.H * p.W) : (uint32_t)(p.awH * p.awW), uW = (uint32_t)p.awW;
#pragma unroll
    for (int i = 0; i < APR; ++i) {
        const int64_t m = min(m0 + arow + 64 * i, p.M - 1);
        if (p.conv) {
            const int64_t hw = p.Ho * p.Wo, img = m / hw, pix = m - img * hw, ho = pix / p.Wo, wo = pix - ho * p.Wo;
            if (AF32)  // 1x1, unpadded: x[img][cbase + k][ho sh][wo sw]
                aoff[i] = (uint32_t)(4 * ((img * p.Cin + p.cbase) * (int64_t)phw + ho * p.sh * p.W + wo * p.sw));
            else
                aoff[i] = (uint32_t)(4 * (img * p.aw_c * (int64_t)phw + ho * p.sh * p.awW + wo * p.sw + (p.awpw - p.pw)));
        } else {
            aoff[i] = (uint32_t)(4 * (m * (AF32 ? p.lda : p.awld) + 2 * akp));
        }
    }
    const __amdgpu_buffer_rsrc_t arsrc =
        AF32 ? __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(p.conv ? p.X : p.A), (short)0, -1, 0x00020000)
             : __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(p.aw), (short)0, -1, 0x00020000);
    const int khw = p.kh * p.kw;
    uint32_t wa[APR][2];
#if !XM_BDMA
    uint4 wbq[BU];
#endif
    auto load_tile = [&](int k0) {
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            if (AF32 && !p.conv) {
                // matrix rows: k = k0 + 2 akp + r per lane, clamped to the row's last element (the
                // value is replaced at staging) so that no load leaves the row
                const uint32_t k = (uint32_t)min(k0 + 2 * akp + r, K32 - 1);
#pragma unroll
                for (int i = 0; i < APR; ++i)
                    wa[i][r] = __builtin_amdgcn_raw_buffer_load_b32(arsrc, (int)(aoff[i] - 8u * (uint32_t)akp + 4u * k), 0, 0);
                continue;
            }
            uint32_t ko;
            if (AF32) {
                ko = 4u * (uint32_t)min(k0 + 2 * akp + r, K32 - 1) * phw;  // channel plane (wave-uniform)
            } else if (p.conv) {
                // wave-uniform; past the group's last channel the address stays on channel K - 1 (the
                // word image ends there: the zero word at staging replaces the value)
                const int k = min(k0 + 2 * akp + r, K32 - 1);
                const uint32_t c = fastdiv((uint32_t)k, p.kk_mul, p.kk_shift);
                const uint32_t t = (uint32_t)k - c * (uint32_t)khw;
                const uint32_t ky = fastdiv(t, p.kw_mul, p.kw_shift);
                const uint32_t kx = t - ky * (uint32_t)p.kw;
                ko = 4u * (c * phw + ky * (uint32_t)p.dh * uW + kx * (uint32_t)p.dw);
            } else {
                ko = 4u * (uint32_t)(k0 + r);  // the matrix words are zero-padded to Kpad
            }
            ko = __builtin_amdgcn_readfirstlane(ko);
#pragma unroll
            for (int i = 0; i < APR; ++i) {
                // (K-steps past the group's last channel become zero words at staging: a select on the
                // loaded value here made the compiler wait for the prefetch right after issuing it)
                wa[i][r] = __builtin_amdgcn_raw_buffer_load_b32(arsrc, (int)aoff[i], (int)ko, 0);
            }
        }
#if XM_BDMA
        // chunk tid = (K-step tid / TXN, column block tid % TXN) -> bw[tid]; a wave's 64 chunks land
        // contiguously from its LDS base (the last, partial wave: lanes past the chunks stay off)
        if (tid < XBK * TXN)
            __builtin_amdgcn_global_load_lds(bsrc + (size_t)(k0 - kbeg) * (hq8 / 4), reinterpret_cast<float *>(&sm.bw[64 * wvu]), 16, 0, 0);  // (a uint4 * here: the host pass drops the kernel stubs)
#else
        if (build) {
            const uint32_t kb = __builtin_amdgcn_readfirstlane((uint32_t)(k0 - kbeg) * hq8);
#pragma unroll
            for (int u = 0; u < BU; ++u)  // (add0, off0, add1, off1) of pairs 2 btx, 2 btx + 1
                wbq[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                       brsrc, (int)boff0, (int)(kb + (uint32_t)(u * BKU) * hq8), 0));
        }
#endif
    };
    load_tile(kbeg);

    // the constant 0/1 selection operand of v_mfma_scale_f32_16x16x128_f8f6f4: lane (n + 16 g)
    // holds column n, K-block g; byte p is 1.0 (e4m3 0x38) where (p & 15) == n, i.e. where the same
    // byte of an A lane holds a code of output column n
    xm_v8i sel;
    {
        const int n = lane & 15;
#pragma unroll
        for (int v = 0; v < 8; ++v) {
            uint32_t w = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (((4 * v + b) & 15) == n) w |= 0x38u << (8 * b);
            sel[v] = (int)w;
        }
    }
    xm_v4f dq[RB];  // one 16x16 accumulator per 16-row block
#pragma unroll
    for (int b = 0; b < RB; ++b) dq[b] = (xm_v4f){0.0f, 0.0f, 0.0f, 0.0f};
    xm_v8i av = {0, 0, 0, 0, 0, 0, 0, 0};
    const char *lut = reinterpret_cast<const char *>(sm.lut);
    const uint32_t wvo = (uint32_t)wc * 512u;  // the wave's first column block (4 wc) in a K-step of the table
    typedef const volatile __attribute__((address_space(3))) uint64_t xm_lds_u64;
#if XM_BDMA
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's B chunks have landed (then the barrier: everyone's)
#endif
    __syncthreads();  // the static table is in LDS before the first build reads it

    for (int k0 = kbeg; k0 < kend; k0 += XBK) {
        if (AF32) {  // the staged values become words here (the loads above have landed)
#pragma unroll
            for (int i = 0; i < APR; ++i)
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    if (k0 + 2 * akp + r >= K32) {
                        wa[i][r] = XM_ZERO_WORD;
                    } else {
                        float v = __uint_as_float(wa[i][r]);
                        if (p.fqin.mx) v = fq_apply(v, fmx, fbias, p.fqin.M, p.fqin.S);
                        bool ok = true;
                        wa[i][r] = xm_word_a(v, XM, XB, emnA, bR, ok);
                        if (!ok) {  // the output row this A row feeds (1x1 conv / matrix), as the pre-pass marks it
                            const int64_t m = min(m0 + arow + 64 * i, p.M - 1);
                            fb_rows(p, m, m + 1);
                            abad = true;
                        }
                    }
                }
        }
        if (!AF32 && p.conv) {  // K-steps past the group's last channel (wave-uniform): zero words
#pragma unroll
            for (int r = 0; r < 2; ++r)
                if (k0 + 2 * akp + r >= K32)
#pragma unroll
                    for (int i = 0; i < APR; ++i) wa[i][r] = XM_ZERO_WORD;
        }
#pragma unroll
        for (int i = 0; i < APR; ++i)
            *reinterpret_cast<uint2 *>(&sm.aw[akp][2 * (arow + 64 * i)]) = make_uint2(wa[i][0], wa[i][1]);
        // build: rows 2 q4, 2 q4 + 1 of both signs for the unit's two column pairs
        if (build) {
#pragma unroll
            for (int u = 0; u < BU; ++u) {
#if XM_BDMA
                const uint4 b = sm.bw[(bkk0 + u * BKU) * TXN + btx];
#else
                const uint4 b = wbq[u];
#endif
                const uint2 s0 = *reinterpret_cast<const uint2 *>(lut + b.y + 8 * q4);
                const uint2 s1 = *reinterpret_cast<const uint2 *>(lut + b.w + 8 * q4);
                const xm_u2 a0 = __builtin_bit_cast(xm_u2, b.x), a1 = __builtin_bit_cast(xm_u2, b.z);
                const xm_u2 n0 = __builtin_bit_cast(xm_u2, b.x ^ 0x80008000u), n1 = __builtin_bit_cast(xm_u2, b.z ^ 0x80008000u);
                auto pk = [](uint32_t v, xm_u2 ad) { return __builtin_bit_cast(uint32_t, __builtin_bit_cast(xm_u2, v) + ad); };
                uint32_t *d = &sm.tt[bkk0 + u * BKU][btx * 32 + q4 * 4];
                *reinterpret_cast<uint4 *>(d) = make_uint4(pk(s0.x, a0), pk(s1.x, a1), pk(s0.y, a0), pk(s1.y, a1));
                *reinterpret_cast<uint4 *>(d + 16) = make_uint4(pk(s0.x, n0), pk(s1.x, n1), pk(s0.y, n0), pk(s1.y, n1));
            }
        }
        __syncthreads();
        if (k0 + XBK < kend) load_tile(k0 + XBK);  // next tile's loads fly during this tile's math

        // lane = (row r16 of each 16-row block, K-step pair g): per row block its A words of
        // K-steps 2 g, 2 g + 1 (one ds_read_b64), 16 columns each, one 16x16x128 MFMA summing the
        // block's 8 K-steps (4 lane groups x 2) -- half the matrix-pipe cycles of the 32x32 form
        {
            const int r16 = lane & 15, g = lane >> 4;
            const uint32_t base = wvo + (uint32_t)(2 * g) * (uint32_t)(TTK * 4);  // multiple of 128 B
            const char *tt0 = reinterpret_cast<const char *>(&sm.tt[0][0]);
            // E5M2: the result grid has one normal binade more than e5m2 (31 - bR, the OCP top
            // exponent being inf / NaN).  An A element whose products can reach it (se <= thi:
            // e_a + max e_b + 1 >= 31 - bR over its 16 columns) is converted one binade down (scale
            // exponent + 1, codes halved) and its MX block (the two A elements of lanes g, g ^ 1 at
            // the same h) scaled by 2 -- allowed when both elements' products stay at or above the
            // grid's second normal binade (se <= tok: e_a + min e_b + min binade(V') >= 2 - bR, a
            // zero element always), so the halved codes round exactly as the unhalved ones; else the
            // element stays unhalved, converts to inf and its tile falls back (as beyond the range).
            // thi / tok: the (K-step 2 g + h, this wave's 16 columns) thresholds on se, packed as
            // bytes (thi0, thi1, tok0, tok1).  (Branching around this per tile -- on whether any A
            // element of the launch could need it -- made the register allocator spill 50-250
            // VGPRs; as its own instance (XF = 2, the tiles the plain form marked UT_HALF), on
            // the 128 x 32 / 256 x 16 tiles, whose 60-70 VGPRs leave room for it: launch_f8mx.)
            uint32_t thr = 0u;
            if (XF == 2) {
                const int64_t ng = p.npad / 16, e0 = (int64_t)(k0 + 2 * g) * ng + (n0 / 16 + wc);
                const uint32_t r0 = p.ebr[e0], r1 = p.ebr[e0 + ng];
                const uint32_t thi0 = (uint32_t)max(112 + (int)(r0 & 0xFFu) - 128, 0);
                const uint32_t thi1 = (uint32_t)max(112 + (int)(r1 & 0xFFu) - 128, 0);
                const uint32_t tok0 = (uint32_t)min(max(140 + (int)(r0 >> 8) - 128 + p.xm_vmin, 0), 252);
                const uint32_t tok1 = (uint32_t)min(max(140 + (int)(r1 >> 8) - 128 + p.xm_vmin, 0), 252);
                thr = thi0 | (thi1 << 8) | (tok0 << 16) | (tok1 << 24);
            }
#pragma unroll
            for (int b = 0; b < RB; ++b) {
                const uint2 aw2 = *reinterpret_cast<const uint2 *>(&sm.aw[g][2 * (16 * (RB * wr + b) + r16)]);
                uint32_t awh[2] = {aw2.x, aw2.y};
                int sca = 127;  // this lane group's MX block scale (E8M0)
                if (XF == 2) {
                    // per element: need (se <= thi) and allow (se <= tok, or a zero: se 253), as
                    // sign bits of differences (se, thresholds < 256)
                    const uint32_t se0 = awh[0] >> 23, se1 = awh[1] >> 23;
                    const uint32_t n0b = (se0 - (thr & 0xFFu) - 1u) >> 31, n1b = (se1 - ((thr >> 8) & 0xFFu) - 1u) >> 31;
                    const uint32_t o0b = ((se0 - ((thr >> 16) & 0xFFu) - 1u) >> 31) | ((252u - se0) >> 31);
                    const uint32_t o1b = ((se1 - (thr >> 24) - 1u) >> 31) | ((252u - se1) >> 31);
                    const uint32_t bits = n0b | (n1b << 1) | (o0b << 2) | (o1b << 3);
                    const auto sw16 = __builtin_amdgcn_permlane16_swap(bits, bits, false, false);
                    const uint32_t pb = (g & 1) ? sw16[0] : sw16[1];  // lane ^ 16: the block partner
                    const uint32_t halve = (bits | pb) & ((bits & pb) >> 2) & 3u;
                    awh[0] += (halve & 1u) << 23;
                    awh[1] += (halve >> 1) << 23;
                    // block g's scale: blocks 0 / 2 (h = 0 / 1 of lane groups 0, 1), 1 / 3 (lane groups 2, 3)
                    const auto sw32 = __builtin_amdgcn_permlane32_swap(halve, halve, false, false);
                    const uint32_t ph = (g >= 2) ? sw32[0] : sw32[1];  // lane ^ 32
                    sca = 127 + (int)(((g == 1 || g == 2) ? ph : halve) >> (g >> 1) & 1u);
                }
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    uint32_t a;
                    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(a) : "v"(awh[h]), "s"(XM_ROW_MASK), "v"(base));
                    __builtin_assume((a & 7u) == 0u);
                    // (volatile: otherwise the two halves, used as different types, are split into
                    // two loads and re-merged into a ds_read2_b32 -- half the LDS rate of ds_read_b64)
                    xm_lds_u64 *ttk = (xm_lds_u64 *)(tt0 + h * TTK * 4);
                    uint2 v[4];
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const uint64_t w = ttk[(a >> 3) + 16 * c];
                        v[c] = make_uint2((uint32_t)w, (uint32_t)(w >> 32));
                    }
                    const float sc = __uint_as_float(awh[h]);
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        xm_s2 cv;
                        if (XF) {
                            asm("v_cvt_scalef32_pk_bf8_bf16 %0, %1, %2" : "=v"(cv) : "v"(v[c].x), "v"(sc));
                            cv = __builtin_amdgcn_cvt_scalef32_pk_bf8_bf16(cv, __builtin_bit_cast(xm_b2, v[c].y), sc, true);
                        } else {
                            asm("v_cvt_scalef32_pk_fp8_bf16 %0, %1, %2" : "=v"(cv) : "v"(v[c].x), "v"(sc));
                            cv = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(cv, __builtin_bit_cast(xm_b2, v[c].y), sc, true);
                        }
                        av[4 * h + c] = __builtin_bit_cast(int, cv);
                    }
                }
                // A codes e4m3 (cbsz 0) or bf8 (cbsz 1); the selection operand is e4m3 (blgp 0)
                dq[b] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, sel, dq[b], XF ? 1 : 0, 0, 0, sca, 0, 127);
            }
        }
#if XM_BDMA
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the next tile's B chunks (read by the next build)
#endif
        __syncthreads();
    }

    // a term beyond the e4m3 range came back NaN (and poisons its column): the exact kernel
    // recomputes the tile; (AF32) an A operand off the grid / outside the window marked its row
    // above, a bias outside the window every unit
    bool nan = false;
#pragma unroll
    for (int b = 0; b < RB; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) nan |= !__builtin_isfinite(dq[b][i]);
    const bool tnan = __syncthreads_or(nan ? 1 : 0) != 0;
    const bool tbad = AF32 && __syncthreads_or((abad || biasbad) ? 1 : 0) != 0;
    if ((tnan || tbad) && tid == 0) {
        // E5M2: a NaN of the plain form where the launch's extremes reach the top binade goes to
        // the halved-block form first (its own NaN -- beyond the range -- to the exact kernel)
        if (XF == 1 && tnan && xm_needs_halving(p, AF32, AF32 ? bA : 0, bR)) {
            fb_tile(p, m0, BMT, n0, UT_HALF);
            atomicOr(p.flag, FB_HALF);
            if (tbad) atomicOr(p.flag, fb_bits(p, biasbad));
        } else {
            if (tnan) fb_tile(p, m0, BMT, n0, XF == 2 ? (uint8_t)(UT_EXACT | UT_HALF) : UT_EXACT);
            atomicOr(p.flag, fb_bits(p, biasbad));
        }
    }

    // D (units of 2^(7-bR)) of row block b: lane l holds rows 4 (l >> 4) .. + 3, column l & 15
    // -> tile row 16 (RB wr + b) + 4 (l >> 4) + i, column 16 wc + (l & 15) -> an [SR][BNT] slab in
    // LDS per SR tile rows -> each thread's 4x4 block (64-row sub-slab sub, 4-column block cb),
    // epilogue mapping with consecutive lanes on consecutive pixels
    const float f8S = __uint_as_float((uint32_t)min(max(127 + XB - bR, 1), 254) << 23);
    float *ct = smu.ct;
    const int ety = tid & 15, etx = tid >> 4, cb = etx % (BNT / 4), sub = etx / (BNT / 4);
#pragma unroll
    for (int h = 0; h < BMT / SR; ++h) {
        if (h > 0) __syncthreads();  // the previous slab is read (the K loop's last barrier covers h = 0)
#pragma unroll
        for (int b = 0; b < RB; ++b) {
            const int rb = 16 * (RB * wr + b) - SR * h;  // the block's first row in the slab (wave-uniform)
            if (rb >= 0 && rb < SR) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    ct[(rb + 4 * (lane >> 4) + i) * CP + 16 * wc + (lane & 15)] = dq[b][i] * f8S;
            }
        }
        __syncthreads();
        float acc[TM][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = ct[(64 * sub + ety * TM + i) * CP + cb * TN + j];
        store_tile<EMIT, !EMIT>(p, split, m0 + SR * h + 64 * sub, n0, ety, cb, acc);  // (GELU tails: run_gemm never emits)
    }
    FP8A_CLK_END
}
#endif  // FP8A_OWN_F8MX

}  // namespace fp8a
