// gemm_dense.h -- the exact (non-approx) product on the matrix core.  DESIGN.md §3e.
//
// The reference's non-approx branch is a plain fp32 contraction of FP8-quantized operands:
// `x @ y` (approx_calculation.py:797, 811 -- the im2col form for convs; QuantizationHijacker
// with approx_flag off, BASELINE config 1).  Every value on an E4M3 / E5M2 grid has at most 4 / 3
// significant bits, so within one 32-k block it is EXACT in OCP e4m3 / e5m2 times a power-of-two
// block scale, and the block-scaled MFMA (v_mfma_scale_f32_16x16x128_f8f6f4) forms each product
// exactly and accumulates in fp32: the same sums up to summation order.
//
//   dn_pack<A|B>  -- one thread per (row, 32-k block): the block's largest magnitude picks the
//                    E8M0 scale (e4m3: largest binade 8 when the top value fits 448, else 7;
//                    e5m2: 15), the 32 values go to fp8 bytes, and each is converted back: a value
//                    that does not round-trip (off the FP8 grid, more than ~16 / ~31 binades below
//                    its block's largest, inf / NaN) marks its 64-row (A) / 64-column (B) unit.
//                    A is gathered straight from NCHW for convs (implicit im2col).
//   dn_gemm       -- 128 x 128 tiles, 4 waves of 64 x 64, per 128-k stage the byte images through
//                    LDS and 128 block-scaled MFMAs per wave, each over 16 k of one MX block with
//                    one value per 8-byte operand group (the matrix core's first summation stage
//                    is narrow: see dn_gemm).  NCHW stores use the transposed
//                    product (B as the MFMA's first operand) so consecutive lanes hold consecutive
//                    pixels.
//   dn_fix        -- the marked 64 x 64 units again in fp32 FMAs from the original operands (a
//                    no-op launch when nothing is marked; counted by fp8a_dense_stats).
#pragma once
#include "fp8approx_common.h"
#include "gemm_f8mx.h"

namespace fp8a {

constexpr int DN_T = 128;            // tile rows = tile columns
constexpr int DN_KC = 128;           // k per LDS stage (one MFMA K-step)
constexpr int DN_RS = DN_KC + 16;    // LDS row stride, bytes
constexpr int DN_U = 64;             // fallback unit edge

// The layer tail a config-1 (approx_flag off) BNFusedHijacker runs around its exact product,
// fused into the product's loads and stores (fp8a_dense_conv2d_fused; quantized_folded_bn.py:
// 30-83, hijacker.py:77-115): qin = the input's activation quantizer (quantize_input), applied
// to every A value as it is loaded; then per output value rq (the res quantizer,
// original_quantize_res), the eval batch norm as scale / shift of its channel, the clamp
// activation, and oq (the output's activation quantizer when the layer does not quantize its
// input).  Per-tensor FP8 quantizers (fp8_quantizer.py:97-173: fq_apply); any member off.
struct DnFuse {
    FqIn qin, rq, oq;
    FqIn wq;           // the weight quantizer, on every B (weight) value as it is loaded
    int wq_row;        // 1: wq.mx holds one maxval per output channel (per-channel weights)
    const float2 *ep;
    int act;
    float lo, hi;
    float *bo[4];      // the bias outputs (custom_bias) of qin, rq, oq, wq; int32 copies in ibo
    int32_t *ibo[4];
};
struct DnQv {  // the quantizers' maxval and bias, read once per thread
    float qmx, qb, rmx, rb, omx, ob;
};
__device__ __forceinline__ DnQv dn_qv(const DnFuse &f) {
    DnQv q{};
    if (f.qin.mx) { q.qmx = *f.qin.mx; q.qb = fq_bias(q.qmx, f.qin.E, f.qin.M); }
    if (f.rq.mx) { q.rmx = *f.rq.mx; q.rb = fq_bias(q.rmx, f.rq.E, f.rq.M); }
    if (f.oq.mx) { q.omx = *f.oq.mx; q.ob = fq_bias(q.omx, f.oq.E, f.oq.M); }
    return q;
}
// The weight quantizer of output channel n: maxval and bias
__device__ __forceinline__ float dn_wmx(const DnFuse &f, int64_t n) { return f.wq_row ? f.wq.mx[n] : *f.wq.mx; }
__device__ __forceinline__ float dn_wq(const DnFuse &f, float mx, float b, float v) {
    return f.wq.mx ? fq_apply(v, mx, b, f.wq.M, f.wq.S) : v;
}
__device__ __forceinline__ float dn_w(const DnFuse &f, int64_t n, float v) {
    if (!f.wq.mx) return v;
    const float mx = dn_wmx(f, n);
    return fq_apply(v, mx, fq_bias(mx, f.wq.E, f.wq.M), f.wq.M, f.wq.S);
}
__device__ __forceinline__ void dn_put_bias(const FqIn &q, const float *mx, float *bo, int32_t *ibo, int64_t i) {
    const float b = fq_bias(*mx, q.E, q.M);
    bo[i] = b;
    ibo[i] = (int32_t)b;
}
// The fused quantizers' bias outputs (what each reference quantizer's forward leaves in custom_bias),
// written by the first kernel of the layer: the per-tensor ones by channel 0's thread, a per-channel
// weight quantizer's by each channel's
__device__ __forceinline__ void dn_bias_out(const DnFuse &f, int64_t n, bool row = true) {
    if (n == 0) {
        if (f.qin.mx) dn_put_bias(f.qin, f.qin.mx, f.bo[0], f.ibo[0], 0);
        if (f.rq.mx) dn_put_bias(f.rq, f.rq.mx, f.bo[1], f.ibo[1], 0);
        if (f.oq.mx) dn_put_bias(f.oq, f.oq.mx, f.bo[2], f.ibo[2], 0);
    }
    if (f.wq.mx && (f.wq_row ? row : n == 0))
        dn_put_bias(f.wq, f.wq.mx + (f.wq_row ? n : 0), f.bo[3], f.ibo[3], f.wq_row ? n : 0);
}
// ... with no product to run (empty reduction or output): one thread per channel
__global__ __launch_bounds__(256) void dn_bias_kernel(const DnFuse f, int64_t N) {
    const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (n < N || n == 0) dn_bias_out(f, n, n < N);  // (no channel rows when N = 0)
}
__device__ __forceinline__ float dn_in(const DnFuse &f, const DnQv &q, float v) {
    return f.qin.mx ? fq_apply(v, q.qmx, q.qb, f.qin.M, f.qin.S) : v;
}
__device__ __forceinline__ float dn_out(const DnFuse &f, const DnQv &q, int64_t c, float v) {
    if (f.rq.mx) v = fq_apply(v, q.rmx, q.rb, f.rq.M, f.rq.S);
    if (f.ep) {
        const float2 e = f.ep[c];
        v = __fmaf_rn(v, e.x, e.y);
        if (f.act) v = fminf(fmaxf(v, f.lo), f.hi);
    }
    if (f.oq.mx) v = fq_apply(v, q.omx, q.ob, f.oq.M, f.oq.S);
    return v;
}

struct DenseArgs {
    const float *x;            // A: matmul element (m, k) at x[m * sam + k * sak]; conv: the NCHW input
    const float *w;            // B: element (k, n) at w[k * sbk + n * sbn]
    float *y;                  // C: y[m * ldc + n], or NCHW (conv)
    int64_t M, N, K, kpad, mpad, npad;
    int64_t sam, sak, sbk, sbn, ldc;
    int conv;
    int64_t C, H, W, Ho, Wo;
    int kh, kw, sh, sw, ph, pw, dh, dw;
    uint8_t *qa, *qas, *qb, *qbs;  // byte images [mpad|npad][kpad] and E8M0 scales [..][kpad / 32]
    uint32_t *urow, *ucol;         // unit marks [mpad / 64], [npad / 64]: == gen when marked
    uint32_t *anymark;             // gen once any unit is marked
    uint32_t gen;                  // this call's mark tag (run_dense: no clearing pass between calls)
    int fmt;                       // FP8A_DENSE_E4M3 / FP8A_DENSE_E5M2 / FP8A_DENSE_BF16
    DnFuse fz;                     // the fused layer tail (all off: the plain product)
};

__device__ unsigned long long g_dense[2];  // [0] launches with marked units, [1] units recomputed

__device__ __forceinline__ float dn_conv_elem(const DenseArgs &p, int64_t img, int64_t ho, int64_t wo, int64_t c,
                                              int i, int j) {
    const int64_t hi = ho * p.sh - p.ph + (int64_t)i * p.dh, wi = wo * p.sw - p.pw + (int64_t)j * p.dw;
    if (hi < 0 || hi >= p.H || wi < 0 || wi >= p.W) return 0.0f;
    return p.x[((img * p.C + c) * p.H + hi) * p.W + wi];
}

__device__ __forceinline__ float dn_a_raw(const DenseArgs &p, int64_t m, int64_t k) {
    if (!p.conv) return p.x[m * p.sam + k * p.sak];
    const int64_t hw = p.Ho * p.Wo, img = m / hw, pix = m - img * hw, ho = pix / p.Wo, wo = pix - ho * p.Wo;
    const int khw = p.kh * p.kw;
    const int64_t c = k / khw;
    const int t = (int)(k - c * khw), i = t / p.kw, j = t - i * p.kw;
    return dn_conv_elem(p, img, ho, wo, c, i, j);
}
// A(m, k) with the fused input quantizer (dn_pack / dn_fix: the rarely-run paths read its maxval
// per element)
__device__ __forceinline__ float dn_a(const DenseArgs &p, int64_t m, int64_t k) {
    const float v = dn_a_raw(p, m, k);
    if (!p.fz.qin.mx) return v;
    const float mx = *p.fz.qin.mx;
    return fq_apply(v, mx, fq_bias(mx, p.fz.qin.E, p.fz.qin.M), p.fz.qin.M, p.fz.qin.S);
}

// fp8 bytes of two floats (scale 1: the caller has applied the block scale) and back
template <int FMT>
__device__ __forceinline__ uint32_t dn_cvt2(float a, float b, bool &ok) {
    xm_s2 cv = {0, 0};
    float ra, rb;
    if constexpr (FMT == 0) {
        cv = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(cv, a, b, 1.0f, false);
        const uint32_t u = __builtin_bit_cast(uint32_t, cv);
        ra = __builtin_amdgcn_cvt_scalef32_f32_fp8((int)u, 1.0f, 0);
        rb = __builtin_amdgcn_cvt_scalef32_f32_fp8((int)u, 1.0f, 1);
    } else {
        cv = __builtin_amdgcn_cvt_scalef32_pk_bf8_f32(cv, a, b, 1.0f, false);
        const uint32_t u = __builtin_bit_cast(uint32_t, cv);
        ra = __builtin_amdgcn_cvt_scalef32_f32_bf8((int)u, 1.0f, 0);
        rb = __builtin_amdgcn_cvt_scalef32_f32_bf8((int)u, 1.0f, 1);
    }
    ok = ok && ra == a && rb == b;
    return __builtin_bit_cast(uint32_t, cv) & 0xFFFFu;
}

template <bool ISB, int FMT>
__global__ __launch_bounds__(256) void dn_pack(const DenseArgs p) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t rows = ISB ? p.N : p.M, rpad = ISB ? p.npad : p.mpad;
    if (r >= rpad) return;
    const int kb = blockIdx.y;
    const int64_t k0 = 32 * (int64_t)kb;
    float v[32];
#pragma unroll
    for (int e = 0; e < 32; ++e) v[e] = 0.0f;
    if (r < rows) {
        if (ISB) {
            float wmx = 0.0f, wb = 0.0f;
            if (p.fz.wq.mx) {
                wmx = dn_wmx(p.fz, r);
                wb = fq_bias(wmx, p.fz.wq.E, p.fz.wq.M);
            }
            if (kb == 0) dn_bias_out(p.fz, r);
#pragma unroll
            for (int e = 0; e < 32; ++e)
                if (k0 + e < p.K) v[e] = dn_wq(p.fz, wmx, wb, p.w[(k0 + e) * p.sbk + r * p.sbn]);
        } else if (p.conv) {
            const int64_t hw = p.Ho * p.Wo, img = r / hw, pix = r - img * hw, ho = pix / p.Wo, wo = pix - ho * p.Wo;
            const int khw = p.kh * p.kw;
            int64_t c = k0 / khw;
            int t = (int)(k0 - c * khw), i = t / p.kw, j = t - i * p.kw;
#pragma unroll
            for (int e = 0; e < 32; ++e) {
                if (k0 + e < p.K) v[e] = dn_conv_elem(p, img, ho, wo, c, i, j);
                if (++j == p.kw) {
                    j = 0;
                    if (++i == p.kh) { i = 0; ++c; }
                }
            }
        } else {
#pragma unroll
            for (int e = 0; e < 32; ++e)
                if (k0 + e < p.K) v[e] = p.x[r * p.sam + (k0 + e) * p.sak];
        }
    }
    if constexpr (FMT == 2) {  // bf16: exact iff the low 16 bits are zero (finite, normal or zero)
        bool ok = true;
        uint32_t wd[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const uint32_t u0 = __float_as_uint(v[2 * q]), u1 = __float_as_uint(v[2 * q + 1]);
            const uint32_t e0 = u0 & 0x7F800000u, e1 = u1 & 0x7F800000u;
            ok = ok && (u0 & 0xFFFFu) == 0u && (u1 & 0xFFFFu) == 0u && e0 != 0x7F800000u && e1 != 0x7F800000u &&
                 (e0 != 0u || (u0 & 0x7FFFFFFFu) == 0u) && (e1 != 0u || (u1 & 0x7FFFFFFFu) == 0u);
            wd[q] = (u0 >> 16) | (u1 & 0xFFFF0000u);
        }
        uint4 *q = reinterpret_cast<uint4 *>((ISB ? p.qb : p.qa) + 2 * (r * p.kpad + k0));
#pragma unroll
        for (int t = 0; t < 4; ++t) q[t] = make_uint4(wd[4 * t], wd[4 * t + 1], wd[4 * t + 2], wd[4 * t + 3]);
        if (!ok) {
            (ISB ? p.ucol : p.urow)[r / DN_U] = p.gen;
            *p.anymark = p.gen;
        }
        return;
    }
    float amax = 0.0f;
    bool ok = true;
#pragma unroll
    for (int e = 0; e < 32; ++e) {
        amax = fmaxf(amax, fabsf(v[e]));
        ok = ok && v[e] == v[e];  // NaN
    }
    int s = 0;
    if (amax > 0.0f) {
        if (!(amax <= 3.4028235e38f)) {
            ok = false;
        } else {
            int e;
            frexpf(amax, &e);
            --e;  // floor(log2 amax)
            s = FMT == 0 ? (ldexpf(amax, 8 - e) <= 448.0f ? e - 8 : e - 7) : e - 15;
            if (s < -127 || s > 127) { ok = false; s = 0; }
        }
    }
    uint32_t wd[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const uint32_t lo = dn_cvt2<FMT>(ldexpf(v[4 * q], -s), ldexpf(v[4 * q + 1], -s), ok);
        const uint32_t hi = dn_cvt2<FMT>(ldexpf(v[4 * q + 2], -s), ldexpf(v[4 * q + 3], -s), ok);
        wd[q] = lo | (hi << 16);
    }
    uint8_t *q = (ISB ? p.qb : p.qa) + r * p.kpad + k0;
    *reinterpret_cast<uint4 *>(q) = make_uint4(wd[0], wd[1], wd[2], wd[3]);
    *reinterpret_cast<uint4 *>(q + 16) = make_uint4(wd[4], wd[5], wd[6], wd[7]);
    (ISB ? p.qbs : p.qas)[r * (p.kpad / 32) + kb] = (uint8_t)(ok ? s + 127 : 127);
    if (!ok) {
        (ISB ? p.ucol : p.urow)[r / DN_U] = p.gen;
        *p.anymark = p.gen;
    }
}

struct DnSmem {
    uint8_t a[DN_T][DN_RS];
    uint8_t b[DN_T][DN_RS];
    uint32_t as[DN_T];  // the row's 4 block scales of the stage
    uint32_t bs[DN_T];
};

template <int FMT, bool NCHW>
__global__ __launch_bounds__(256, 2) void dn_gemm(const DenseArgs p) {
    __shared__ __attribute__((aligned(16))) DnSmem sm;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wr = __builtin_amdgcn_readfirstlane(wv >> 1), wc = __builtin_amdgcn_readfirstlane(wv & 1);
    const int64_t num_mt = p.mpad / DN_T;
    const int64_t m0 = ((int64_t)blockIdx.x % num_mt) * DN_T, n0 = ((int64_t)blockIdx.x / num_mt) * DN_T;
    const int64_t kpad = p.kpad, kb32 = kpad / 32;
    // staging: thread = (row, 4 of the stage's 8 16-byte granules); even threads also the scales
    const int srow = tid >> 1, sg0 = (tid & 1) * 4;
    const uint8_t *ga = p.qa + (m0 + srow) * kpad, *gb = p.qb + (n0 + srow) * kpad;
    const uint8_t *gas = p.qas + (m0 + srow) * kb32, *gbs = p.qbs + (n0 + srow) * kb32;
    uint4 ra[4], rb[4];
    uint32_t rsa = 0x7F7F7F7Fu, rsb = 0x7F7F7F7Fu;
    auto load = [&](int64_t k0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t kk = k0 + 16 * (sg0 + q);
            ra[q] = kk < kpad ? *reinterpret_cast<const uint4 *>(ga + kk) : make_uint4(0u, 0u, 0u, 0u);
            rb[q] = kk < kpad ? *reinterpret_cast<const uint4 *>(gb + kk) : make_uint4(0u, 0u, 0u, 0u);
        }
        if ((tid & 1) == 0) {
            rsa = rsb = 0u;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t b = k0 / 32 + q;
                rsa |= (uint32_t)(b < kb32 ? gas[b] : 127) << (8 * q);
                rsb |= (uint32_t)(b < kb32 ? gbs[b] : 127) << (8 * q);
            }
        }
    };
    xm_v4f acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (xm_v4f){0.0f, 0.0f, 0.0f, 0.0f};
    const int r16 = lane & 15, g = lane >> 4;
    load(0);
    for (int64_t k0 = 0; k0 < kpad; k0 += DN_KC) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            *reinterpret_cast<uint4 *>(&sm.a[srow][16 * (sg0 + q)]) = ra[q];
            *reinterpret_cast<uint4 *>(&sm.b[srow][16 * (sg0 + q)]) = rb[q];
        }
        if ((tid & 1) == 0) {
            sm.as[srow] = rsa;
            sm.bs[srow] = rsb;
        }
        __syncthreads();
        if (k0 + DN_KC < kpad) load(k0 + DN_KC);  // the next stage's loads fly during the MFMAs
        // One value per 8-byte group of the MFMA operand: the matrix core sums the products of each
        // 8-byte group in a narrow first stage that drops a product ~2^13 or more below its
        // neighbour (measured: tools/mfma_bf16_precision.hip, tools/debug_dense3.py),
        // and adds the groups exactly.  So each MFMA takes 16 real k -- half an MX block, its scale
        // in all four lane groups -- at slots 16 g, 16 g + 8, 64 + 16 g, 64 + 16 g + 8 of lane
        // group g (operand K layout measured, tools/mfma_scale_layout.hip: lane group g's bytes 0-15
        // are slots 16 g .., bytes 16-31 slots 64 + 16 g ..): k = 2 g, 2 g + 1, 8 + 2 g, 9 + 2 g.
#pragma unroll
        for (int ks = 0; ks < DN_KC / 16; ++ks) {
            xm_v8i af[4], bf[4];
            int sa[4], sb[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = 64 * wr + 16 * i + r16, col = 64 * wc + 16 * i + r16;
                const uint32_t a0 = *reinterpret_cast<const uint16_t *>(&sm.a[row][16 * ks + 2 * g]);
                const uint32_t a1 = *reinterpret_cast<const uint16_t *>(&sm.a[row][16 * ks + 8 + 2 * g]);
                const uint32_t b0 = *reinterpret_cast<const uint16_t *>(&sm.b[col][16 * ks + 2 * g]);
                const uint32_t b1 = *reinterpret_cast<const uint16_t *>(&sm.b[col][16 * ks + 8 + 2 * g]);
                af[i] = (xm_v8i){(int)(a0 & 0xFFu), 0, (int)(a0 >> 8), 0, (int)(a1 & 0xFFu), 0, (int)(a1 >> 8), 0};
                bf[i] = (xm_v8i){(int)(b0 & 0xFFu), 0, (int)(b0 >> 8), 0, (int)(b1 & 0xFFu), 0, (int)(b1 >> 8), 0};
                sa[i] = (int)((sm.as[row] >> (8 * (ks >> 1))) & 0xFFu);
                sb[i] = (int)((sm.bs[col] >> (8 * (ks >> 1))) & 0xFFu);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if constexpr (NCHW)  // D^T: rows = columns n, columns = rows m
                        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bf[j], af[i], acc[i][j], FMT, FMT,
                                                                                    0, sb[j], 0, sa[i]);
                    else
                        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bf[j], acc[i][j], FMT, FMT,
                                                                                    0, sa[i], 0, sb[j]);
                }
        }
        __syncthreads();
    }
    // lane (r16, g) holds D[4 g + r][r16] of each 16 x 16 block
    const int64_t hw = p.Ho * p.Wo;
    const DnQv qv = dn_qv(p.fz);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if constexpr (NCHW) {
                    const int64_t m = m0 + 64 * wr + 16 * i + r16, n = n0 + 64 * wc + 16 * j + 4 * g + r;
                    if (m < p.M && n < p.N) {
                        const int64_t img = m / hw, pix = m - img * hw;
                        p.y[(img * p.N + n) * hw + pix] = dn_out(p.fz, qv, n, acc[i][j][r]);
                    }
                } else {
                    const int64_t m = m0 + 64 * wr + 16 * i + 4 * g + r, n = n0 + 64 * wc + 16 * j + r16;
                    if (m < p.M && n < p.N) p.y[m * p.ldc + n] = dn_out(p.fz, qv, n, acc[i][j][r]);
                }
            }
}

// The bf16 form (fmt FP8A_DENSE_BF16, the default for the exact product): every value of an FP8 /
// E3M4 / E2M5 grid (<= 6 significant bits) is exact in bf16 at any exponent, so no block scales and
// no range limit; v_mfma_f32_16x16x32_bf16 forms the products exactly and adds them exactly down to
// fp32's last bit at every K position (measured: tools/mfma_bf16_precision.hip) -- 32 real k per
// MFMA, 4x the fp8 form's 16 at the same MFMA cycles.  A is read straight from the fp32 source
// (implicit im2col for convs: thread = row, 32 consecutive k per stage, lanes on consecutive rows,
// so every load instruction covers consecutive pixels) and truncated to bf16 in registers; a value
// that is not exact (low 16 bits set, inf / NaN, fp32 denormal) marks its row unit for dn_fix.  B
// comes from dn_pack's bf16 image.  128 x 128 tiles, 4 waves of 64 x 64, 64 k per LDS stage.
constexpr int DN_BK = 64;                 // k per LDS stage of the bf16 form
constexpr int DN_BRS = 2 * DN_BK + 16;    // bf16 LDS row stride, bytes
struct DnSmem16 {
    uint8_t a[DN_T][DN_BRS];
    uint8_t b[DN_T][DN_BRS];
};
typedef __bf16 dn_v8bf __attribute__((ext_vector_type(8)));

__device__ __forceinline__ bool dn_bf16_exact(uint32_t u) {
    const uint32_t e = u & 0x7F800000u;
    return (u & 0xFFFFu) == 0u && e != 0x7F800000u && (e != 0u || (u & 0x7FFFFFFFu) == 0u);
}

// AF (conv A addressing, x below 2^31 bytes, run_dense): 1 = a 1 x 1, stride-1, unpadded
// convolution (every MobileNetV2 / ResNet pointwise layer): A (m, k) = x[img][k][pixel], one pixel
// offset per row and a per-k channel-plane offset; 2 = any window: the (channel, ky, kx) of each k
// wave-uniform (scalar), per element two adds and the bounds test in 32 bits; 0 = 64-bit indexing
#ifndef FP8A_DN_BF16_WAVES
#define FP8A_DN_BF16_WAVES 3  // min waves per SIMD of the conv forms (2: 168-194 VGPRs; 3: config 1 30.1k -> 34.5k
                              // images/s; the matmul form stays at 2: it spills at 3)
#endif
template <bool CONV, int AF = 0>
__global__ __launch_bounds__(256, CONV ? FP8A_DN_BF16_WAVES : 2) void dn_gemm_bf16(const DenseArgs p) {
    __shared__ __attribute__((aligned(16))) DnSmem16 sm;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wr = __builtin_amdgcn_readfirstlane(wv >> 1), wc = __builtin_amdgcn_readfirstlane(wv & 1);
    const int64_t num_mt = p.mpad / DN_T;
    const int64_t m0 = ((int64_t)blockIdx.x % num_mt) * DN_T, n0 = ((int64_t)blockIdx.x / num_mt) * DN_T;
    const int64_t kpad = p.kpad;
    // A staging: thread = (row ar, k half ah): 32 consecutive k of the stage
    const int ar = tid & 127, ah = tid >> 7;
    const int64_t am = m0 + ar;
    const bool arow = am < p.M;
    int64_t img = 0, hi0 = 0, wi0 = 0;
    if (CONV && arow) {
        const int64_t hw = p.Ho * p.Wo, pix = am - (am / hw) * hw, ho = pix / p.Wo, wo = pix - ho * p.Wo;
        img = am / hw;
        hi0 = ho * p.sh - p.ph;
        wi0 = wo * p.sw - p.pw;
    }
    const float *xrow = CONV ? p.x + img * p.C * p.H * p.W : p.x + (arow ? am : 0) * p.sam;
    const int khw = p.kh * p.kw;
    const DnQv qv = dn_qv(p.fz);
    float ra[32];
    bool aok = true;
    // (AF 1: hi0 / wi0 are the pixel's own row / column.  x through a buffer resource of exactly its
    // bytes (< 2^31, run_dense): rows past M read 0; the k offset is wave-uniform (ah = tid / 128),
    // so each load is one VGPR offset (the pixel / image) + one SGPR offset (the channel plane))
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(p.x), (short)0, AF ? (int)(4 * p.C * p.H * p.W * (p.M / max(p.Ho * p.Wo, (int64_t)1))) : 0,
        0x00020000);
    const uint32_t voff = AF == 1 ? (uint32_t)(4 * (img * p.C * p.H * p.W + hi0 * p.W + wi0))
                                  : (uint32_t)(4 * img * p.C * p.H * p.W);
    const uint32_t pstride4 = (uint32_t)(4 * p.H * p.W);
    const int hi0i = (int)hi0, wi0i = (int)wi0, iH = (int)p.H, iW = (int)p.W;
    auto load_a = [&](int64_t k0) {
        const int64_t kb = k0 + 32 * ah;
        if (CONV && AF == 1) {
            const uint32_t kbu = (uint32_t)__builtin_amdgcn_readfirstlane((int)kb);
#pragma unroll
            for (int e = 0; e < 32; ++e)
                ra[e] = kbu + e < (uint32_t)p.K
                            ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, (int)voff, (int)((kbu + e) * pstride4), 0))
                            : 0.0f;
        } else if (CONV && AF == 2) {
            const int kbu = __builtin_amdgcn_readfirstlane((int)kb);
            int c = kbu / khw;
            int t = kbu - c * khw, i = t / p.kw, j = t - i * p.kw;
#pragma unroll
            for (int e = 0; e < 32; ++e) {
                const int hi = hi0i + i * p.dh, wi = wi0i + j * p.dw;
                const bool ok = arow && kbu + e < (int)p.K && (unsigned)hi < (unsigned)iH && (unsigned)wi < (unsigned)iW;
                ra[e] = ok ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, (int)(voff + 4u * (uint32_t)(hi * iW + wi)),
                                                                                  (int)((uint32_t)c * pstride4), 0))
                           : 0.0f;
                if (++j == p.kw) {
                    j = 0;
                    if (++i == p.kh) { i = 0; ++c; }
                }
            }
        } else if (CONV) {
            int64_t c = kb / khw;
            int t = (int)(kb - c * khw), i = t / p.kw, j = t - i * p.kw;
#pragma unroll
            for (int e = 0; e < 32; ++e) {
                const int64_t hi = hi0 + (int64_t)i * p.dh, wi = wi0 + (int64_t)j * p.dw;
                ra[e] = (arow && kb + e < p.K && hi >= 0 && hi < p.H && wi >= 0 && wi < p.W)
                            ? xrow[(c * p.H + hi) * p.W + wi] : 0.0f;
                if (++j == p.kw) {
                    j = 0;
                    if (++i == p.kh) { i = 0; ++c; }
                }
            }
        } else {
#pragma unroll
            for (int e = 0; e < 32; ++e) ra[e] = (arow && kb + e < p.K) ? xrow[(kb + e) * p.sak] : 0.0f;
        }
        if (p.fz.qin.mx) {  // the fused input quantizer (fq(0) = 0: padding unchanged)
#pragma unroll
            for (int e = 0; e < 32; ++e) ra[e] = dn_in(p.fz, qv, ra[e]);
        }
    };
    // B staging: thread = (column tid >> 1, 4 of the stage's 8 16-byte granules)
    const int bcol = tid >> 1, bg0 = (tid & 1) * 4;
    const uint8_t *gb = p.qb + 2 * (n0 + bcol) * kpad;
    uint4 rb[4];
    auto load_b = [&](int64_t k0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t kk = k0 + 8 * (bg0 + q);
            rb[q] = kk < kpad ? *reinterpret_cast<const uint4 *>(gb + 2 * kk) : make_uint4(0u, 0u, 0u, 0u);
        }
    };
    xm_v4f acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (xm_v4f){0.0f, 0.0f, 0.0f, 0.0f};
    const int r16 = lane & 15, g = lane >> 4;
    load_a(0);
    load_b(0);
    for (int64_t k0 = 0; k0 < kpad; k0 += DN_BK) {
        {
            uint32_t w[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const uint32_t u0 = __float_as_uint(ra[2 * q]), u1 = __float_as_uint(ra[2 * q + 1]);
                aok = aok && dn_bf16_exact(u0) && dn_bf16_exact(u1);
                w[q] = (u0 >> 16) | (u1 & 0xFFFF0000u);
            }
            uint4 *d = reinterpret_cast<uint4 *>(&sm.a[ar][64 * ah]);
#pragma unroll
            for (int t = 0; t < 4; ++t) d[t] = make_uint4(w[4 * t], w[4 * t + 1], w[4 * t + 2], w[4 * t + 3]);
#pragma unroll
            for (int q = 0; q < 4; ++q) *reinterpret_cast<uint4 *>(&sm.b[bcol][16 * (bg0 + q)]) = rb[q];
        }
        __syncthreads();
        if (k0 + DN_BK < kpad) {  // the next stage's loads fly during the MFMAs
            load_a(k0 + DN_BK);
            load_b(k0 + DN_BK);
        }
#pragma unroll
        for (int ks = 0; ks < DN_BK / 32; ++ks) {
            dn_v8bf af[4], bf[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {  // lane (r16, g): row / column r16, k 8 g .. 8 g + 7 of the step
                const int row = 64 * wr + 16 * i + r16, col = 64 * wc + 16 * i + r16;
                af[i] = __builtin_bit_cast(dn_v8bf, *reinterpret_cast<const uint4 *>(&sm.a[row][2 * (32 * ks + 8 * g)]));
                bf[i] = __builtin_bit_cast(dn_v8bf, *reinterpret_cast<const uint4 *>(&sm.b[col][2 * (32 * ks + 8 * g)]));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if constexpr (CONV)  // D^T: consecutive lanes on consecutive pixels for the NCHW store
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[i][j], 0, 0, 0);
                    else
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
                }
        }
        __syncthreads();
    }
    if (!aok) {
        p.urow[am / DN_U] = p.gen;
        *p.anymark = p.gen;
    }
    // epilogue through LDS, half the tile at a time (64 channels x 128 pixels for convs, 64 rows x
    // 128 columns for matmuls), so every store instruction writes 64 consecutive floats of one
    // output row / channel plane (full 128-B lines) instead of 16-float pieces
    static_assert(sizeof(DnSmem16) >= 64 * (DN_T + 1) * sizeof(float), "epilogue slice fits the stage buffers");
    float *ct = reinterpret_cast<float *>(&sm);
    constexpr int CP = DN_T + 1;
    const int64_t hw = p.Ho * p.Wo;
    const int et = tid & 127, eq = tid >> 7;
    int64_t eimg = 0, epix = 0;
    if (CONV) {
        const int64_t m = m0 + et;
        eimg = m / hw;
        epix = m - eimg * hw;
    }
    // (halves past the last channel / row are skipped: narrow layers fill few of the 128)
    const int nh = (CONV ? (p.N - n0) : (p.M - m0)) > 64 ? 2 : 1;
    for (int h = 0; h < nh; ++h) {
        __syncthreads();
        if ((CONV ? wc : wr) == h) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        if constexpr (CONV)  // D^T[n][m]: channel 16 j + 4 g + r of the half, pixel 64 wr + 16 i + r16
                            ct[(16 * j + 4 * g + r) * CP + 64 * wr + 16 * i + r16] = acc[i][j][r];
                        else  // D[m][n]: row 16 i + 4 g + r of the half, column 64 wc + 16 j + r16
                            ct[(16 * i + 4 * g + r) * CP + 64 * wc + 16 * j + r16] = acc[i][j][r];
                    }
        }
        __syncthreads();
        const int64_t left = (CONV ? p.N - n0 : p.M - m0) - 64 * h;
        const int nq = (int)min((int64_t)32, (left + 1) / 2);
#pragma unroll 4
        for (int q = 0; q < nq; ++q) {
            const int c = eq + 2 * q;  // the half's channel (conv) / row (matmul)
            if constexpr (CONV) {
                const int64_t m = m0 + et, n = n0 + 64 * h + c;
                if (m < p.M && n < p.N) p.y[(eimg * p.N + n) * hw + epix] = dn_out(p.fz, qv, n, ct[c * CP + et]);
            } else {
                const int64_t m = m0 + 64 * h + c, n = n0 + et;
                if (m < p.M && n < p.N) p.y[m * p.ldc + n] = dn_out(p.fz, qv, n, ct[c * CP + et]);
            }
        }
    }
}

// The marked units in fp32 (fmaf, k order) from the original operands.
// A persistent grid over the units: nothing to do (one word read) unless a unit is marked.
__global__ __launch_bounds__(256) void dn_fix(const DenseArgs p) {
    if (*p.anymark != p.gen) return;
    const int64_t num_um = p.mpad / DN_U, units = num_um * (p.npad / DN_U);
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&g_dense[0], 1ull);
    __shared__ float sa[16][DN_U + 1], sb[16][DN_U + 1];
    const int tid = threadIdx.x, ty = tid & 15, tx = tid >> 4;
    for (int64_t u = blockIdx.x; u < units; u += gridDim.x) {
    const int64_t um = u % num_um, un = u / num_um;
    if (p.urow[um] != p.gen && p.ucol[un] != p.gen) continue;
    if (tid == 0) atomicAdd(&g_dense[1], 1ull);
    const int64_t m0 = um * DN_U, n0 = un * DN_U;
    float acc[4][4] = {};
    for (int64_t k0 = 0; k0 < p.K; k0 += 16) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int idx = tid + 256 * e, kk = idx >> 6, rr = idx & 63;
            const int64_t k = k0 + kk, m = m0 + rr, n = n0 + rr;
            sa[kk][rr] = (k < p.K && m < p.M) ? dn_a(p, m, k) : 0.0f;
            sb[kk][rr] = (k < p.K && n < p.N) ? dn_w(p.fz, n, p.w[k * p.sbk + n * p.sbn]) : 0.0f;
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < 16; ++kk)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = __fmaf_rn(sa[kk][4 * ty + i], sb[kk][4 * tx + j], acc[i][j]);
        __syncthreads();
    }
    const int64_t hw = p.Ho * p.Wo;
    const DnQv qv = dn_qv(p.fz);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t m = m0 + 4 * ty + i, n = n0 + 4 * tx + j;
            if (m >= p.M || n >= p.N) continue;
            if (p.conv) {
                const int64_t img = m / hw, pix = m - img * hw;
                p.y[(img * p.N + n) * hw + pix] = dn_out(p.fz, qv, n, acc[i][j]);
            } else {
                p.y[m * p.ldc + n] = dn_out(p.fz, qv, n, acc[i][j]);
            }
        }
    }
}

// Small exact convolutions (K = Cin kh kw <= 32 and N = Cout <= 64: the stem conv of MobileNetV2 /
// ResNet, a 128 x 128 MFMA tile with 32 live columns and a 64-deep stage for 27 k): thread = output
// pixel, every channel, fp32 FMAs in k order from zero -- dn_fix's arithmetic, the fp32 contraction
// of the original operands, so no fallback units.  The weights (through the fused weight quantizer)
// sit in LDS as [N][32] rows read by 16-byte broadcasts, the pixel's K inputs (through the fused input
// quantizer) in registers; per channel the stores are coalesced over pixels.
constexpr int DD_K = 32, DD_N = 64;
__global__ __launch_bounds__(256) void dn_direct_kernel(const DenseArgs p) {
    __shared__ __attribute__((aligned(16))) float swt[DD_N * DD_K];
    const int tid = threadIdx.x, K = (int)p.K, N = (int)p.N;
    for (int d = tid; d < N * DD_K; d += 256) {
        const int n = d / DD_K, k = d - n * DD_K;
        swt[d] = k < K ? dn_w(p.fz, n, p.w[(int64_t)k * p.sbk + n * p.sbn]) : 0.0f;
    }
    if (blockIdx.x == 0)
        for (int n = tid; n < N; n += 256) dn_bias_out(p.fz, n);
    __syncthreads();
    const DnQv qv = dn_qv(p.fz);
    const int64_t hw = p.Ho * p.Wo;
    const int khw = p.kh * p.kw;
    for (int64_t m = (int64_t)blockIdx.x * 256 + tid; m < p.M; m += (int64_t)gridDim.x * 256) {
        const int64_t img = m / hw, pix = m - img * hw, ho = pix / p.Wo, wo = pix - ho * p.Wo;
        float a[DD_K];
        int c = 0, i = 0, j = 0;
#pragma unroll
        for (int k = 0; k < DD_K; ++k) {
            float v = 0.0f;
            if (k < K) {
                v = dn_in(p.fz, qv, dn_conv_elem(p, img, ho, wo, c, i, j));
                if (++j == p.kw) {
                    j = 0;
                    if (++i == p.kh) { i = 0; ++c; }
                }
            }
            a[k] = v;
        }
        (void)khw;
        float *yo = p.y + img * N * hw + pix;
        for (int n = 0; n < N; ++n) {
            const float4 *wr = reinterpret_cast<const float4 *>(swt + n * DD_K);
            float acc = 0.0f;
#pragma unroll
            for (int q = 0; q < DD_K / 4; ++q) {
                if (4 * q >= K) break;
                const float4 wv = wr[q];
                if (4 * q + 0 < K) acc = __fmaf_rn(a[4 * q + 0], wv.x, acc);
                if (4 * q + 1 < K) acc = __fmaf_rn(a[4 * q + 1], wv.y, acc);
                if (4 * q + 2 < K) acc = __fmaf_rn(a[4 * q + 2], wv.z, acc);
                if (4 * q + 3 < K) acc = __fmaf_rn(a[4 * q + 3], wv.w, acc);
            }
            yo[(int64_t)n * hw] = dn_out(p.fz, qv, n, acc);
        }
    }
}

// n / d for 0 <= n < 2^22 through the float reciprocal (inv = 1 / d rounded): the float quotient
// is off by at most one, the remainder's sign and range fix it.
__device__ __forceinline__ int dw_div(int n, int d, float inv) {
    int q = (int)((float)n * inv);
    const int r = n - q * d;
    q += r < 0 ? -1 : (r >= d ? 1 : 0);
    return q;
}

// Stage the input window of a depthwise workgroup (dn_dw3_kernel, conv_tbs_kernel) into LDS.  The
// rows the workgroup reads are one contiguous range of x -- whole planes, or a band of full rows
// of one plane -- so it is read with 16-byte loads (four in flight per thread) when the range is
// 16-byte aligned, and each value is scattered to its [plane][row][column] slot of the padded
// window (RS rows x WS columns per plane, WS a multiple of 4) as f(value); the slots no value
// lands on (padding, rows past the plane) are zero.  P0 / hi0: the first plane / window row.
// ox: the LDS column of input column 0 (the left padding is the ox columns before it).  With ox
// and W multiples of 4 each 16-byte load lands on one 16-byte LDS slot (one conflict-free write).
template <typename T, typename F>
__device__ __forceinline__ void dw_stage(const float *x, int64_t P0, int npl, int H, int W, int hi0, int ox, int RS,
                                         int WS, float inv_w, float inv_hw, bool plane_mode, T *sm, F f) {
    const int pst = RS * WS, nst = npl * pst, tid = threadIdx.x, hw = H * W;
    for (int d = 4 * tid; d < nst; d += 4 * 256) *reinterpret_cast<uint4 *>(sm + d) = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    // source range [g0, g0 + n): element i -> plane i / hw, row, column
    const int rlo = plane_mode ? 0 : max(hi0, 0), rhi = plane_mode ? H : min(hi0 + RS, H);
    const int n = plane_mode ? npl * hw : (rhi - rlo) * W;
    const float *src = x + P0 * hw + (int64_t)rlo * W;
    auto put = [&](int i, float v) {
        int pl = dw_div(i, hw, inv_hw);
        const int rem = i - pl * hw, row = dw_div(rem, W, inv_w) + rlo, col = rem - (row - rlo) * W;
        const int r = row - hi0, c = col + ox;
        if (r >= 0 && r < RS && c < WS) sm[pl * pst + r * WS + c] = f(v);
    };
    const bool slots = ((W | ox) & 3) == 0;
    if (((((uintptr_t)src) | (uintptr_t)n) & 3) == 0 && (((uintptr_t)src) & 15) == 0) {
        const int n4 = n >> 2;
        for (int q0 = tid; q0 < n4; q0 += 4 * 256) {
            float4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                v[u] = q0 + 256 * u < n4 ? reinterpret_cast<const float4 *>(src)[q0 + 256 * u] : make_float4(0, 0, 0, 0);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int q = q0 + 256 * u;
                if (q >= n4) break;
                if (slots) {  // the four values share a row: one 16-byte slot
                    const int i = 4 * q, pl = dw_div(i, hw, inv_hw), rem = i - pl * hw;
                    const int rr = dw_div(rem, W, inv_w), r = rr + rlo - hi0, col = rem - rr * W;
                    if (r >= 0 && r < RS) {
                        const T o[4] = {f(v[u].x), f(v[u].y), f(v[u].z), f(v[u].w)};
                        *reinterpret_cast<uint4 *>(sm + pl * pst + r * WS + col + ox) =
                            *reinterpret_cast<const uint4 *>(o);
                    }
                    continue;
                }
                put(4 * q, v[u].x);
                put(4 * q + 1, v[u].y);
                put(4 * q + 2, v[u].z);
                put(4 * q + 3, v[u].w);
            }
        }
    } else {
        for (int i0 = tid; i0 < n; i0 += 4 * 256) {
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = i0 + 256 * u < n ? src[i0 + 256 * u] : 0.0f;
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i0 + 256 * u < n) put(i0 + 256 * u, v[u]);
        }
    }
}

// The exact depthwise 3x3 (one input and one output channel per group, dilation 1, equal strides S
// = 1 / 2 -- MobileNetV2's depthwise layers in BASELINE config 1), staged through LDS: the
// workgroup owns PB consecutive planes (image x channel) x RB output rows, loads the input window
// those rows read -- RS = (RB - 1) S + 3 rows x WS >= (Wo - 1) S + 3 columns per plane, the padding
// and the rows past the plane as zeros (dw_stage: 16-byte loads) -- once, with the input quantizer
// (qin) applied once per value, and the PB x 9 weights; then thread = output (consecutive lanes = consecutive output
// columns, so the stores and the LDS reads are contiguous), nine fp32 FMAs in (ky, kx) order from
// zero, as dn_group_conv (the same bits; it stays the form for every other grouped geometry).
// HBM-bound: x read once (plus 2 halo rows per band), y written once.
constexpr int DW_OX = 4;  // dn_dw3_kernel's LDS column of input column 0 (padding pw <= 4 before it)
struct DwArgs {
    const float *x, *w;
    float *y;
    int64_t planes;                // Bn x C
    int C, H, W, Ho, Wo, ph, pw;
    int PB, RB, nb, RS, WS;        // planes per block, output rows per band, bands per plane, staged rows / columns
    float inv_c, inv_ws, inv_pst, inv_wo, inv_pout, inv_w, inv_hw;
    DnFuse fz;
    int64_t nx;                    // floats in x (dn_dw3g_kernel: the last 16-byte chunk's bound)
    int nimg;                      // dn_dw3g_kernel: LDS floats of the raw image (the weights follow)
    float inv_pq, inv_nqd;         // dn_dw3g_kernel: 1 / (quads per plane band), 1 / (quads per row)
};

template <int S>
__global__ __launch_bounds__(256) void dn_dw3_kernel(const DwArgs p) {
    extern __shared__ float dw_sm[];
    const int tid = threadIdx.x;
    const int band = (int)(blockIdx.x % (unsigned)p.nb);
    const int64_t P0 = (int64_t)(blockIdx.x / (unsigned)p.nb) * p.PB;
    const int npl = (int)min((int64_t)p.PB, p.planes - P0);
    const int oh0 = band * p.RB, nrow = min(p.RB, p.Ho - oh0), hi0 = oh0 * S - p.ph;
    const int pst = p.RS * p.WS, pout = p.RB * p.Wo;
    const int c0 = (int)(P0 % p.C);
    float *wsm = dw_sm + p.PB * pst;
    const DnQv qv = dn_qv(p.fz);
    for (int d = tid; d < npl * 9; d += 256) {
        int c = c0 + d / 9;
        c -= dw_div(c, p.C, p.inv_c) * p.C;
        wsm[d] = dn_w(p.fz, c, p.w[(int64_t)c * 9 + d % 9]);
    }
    if (blockIdx.x == 0)
        for (int c = tid; c < p.C; c += 256) dn_bias_out(p.fz, c);
    dw_stage(p.x, P0, npl, p.H, p.W, hi0, DW_OX, p.RS, p.WS, p.inv_w, p.inv_hw, p.RB == p.Ho, dw_sm,
             [&](float v) { return dn_in(p.fz, qv, v); });
    __syncthreads();
    for (int e = tid; e < npl * pout; e += 256) {
        const int pl = dw_div(e, pout, p.inv_pout), rem = e - pl * pout;
        const int orow = dw_div(rem, p.Wo, p.inv_wo), oc = rem - orow * p.Wo;
        if (orow >= nrow) continue;
        const float *xs = dw_sm + pl * pst + orow * S * p.WS + oc * S + DW_OX - p.pw, *ws = wsm + pl * 9;
        float acc = 0.0f;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) acc = __fmaf_rn(xs[ky * p.WS + kx], ws[3 * ky + kx], acc);
        int c = c0 + pl;
        c -= dw_div(c, p.C, p.inv_c) * p.C;
        p.y[((P0 + pl) * p.Ho + oh0 + orow) * p.Wo + oc] = dn_out(p.fz, qv, c, acc);
    }
}

// dn_dw3_kernel with the window staged by LDS-DMA (option "dw3" = 2): the workgroup's source
// range of x -- whole planes, or a band of full rows of one plane, one contiguous range -- is copied
// raw into LDS by global_load_lds_dwordx4 (16-byte chunks from the range's 16-byte-aligned start,
// `lead` floats before it), every chunk of the window in flight at once and no VGPR holding any of
// it; dn_dw3_kernel's register-staged form keeps four 16-byte loads per thread in flight and spent
// 41 % of its wave cycles waiting (§3l).  The padding is not stored: an output's taps read 0 for
// rows / columns outside the plane (the same fma(0, w, acc) as the zero-padded window, so the
// same bits, non-finite weights included).  A thread computes 4 consecutive outputs of a row.  The input quantizer, when fused, runs once per value
// over the landed image in place.  Chunks reaching past x's last float are copied per float.
template <int S>
__global__ __launch_bounds__(256) void dn_dw3g_kernel(const DwArgs p) {
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
    float *img = dw_sm, *wsm = dw_sm + p.nimg;
    const float *src = p.x + a0;
    for (int q0 = 0; q0 < nq; q0 += 256) {
        const int q = q0 + tid;
        if (q < nq) {
            if (a0 + 4 * (int64_t)q + 4 <= p.nx) {
                __builtin_amdgcn_global_load_lds(src + 4 * q, img + 4 * (q0 + 64 * wv), 16, 0, 0);
            } else {  // (the tensor's last floats: never read past x)
                for (int e = 0; e < 4; ++e)
                    if (a0 + 4 * (int64_t)q + e < p.nx) img[4 * q + e] = src[4 * q + e];
            }
        }
    }
    const int c0 = (int)(P0 % p.C);
    const DnQv qv = dn_qv(p.fz);
    for (int d = tid; d < npl * 9; d += 256) {
        int c = c0 + d / 9;
        c -= dw_div(c, p.C, p.inv_c) * p.C;
        wsm[d] = dn_w(p.fz, c, p.w[(int64_t)c * 9 + d % 9]);
    }
    if (blockIdx.x == 0)
        for (int c = tid; c < p.C; c += 256) dn_bias_out(p.fz, c);
    __syncthreads();  // (waits for the LDS-DMA: vmcnt(0) before the barrier)
    if (p.fz.qin.mx) {
        for (int i = 4 * tid; i < 4 * nq; i += 1024) {
            float4 v = *reinterpret_cast<const float4 *>(img + i);
            v.x = dn_in(p.fz, qv, v.x);
            v.y = dn_in(p.fz, qv, v.y);
            v.z = dn_in(p.fz, qv, v.z);
            v.w = dn_in(p.fz, qv, v.w);
            *reinterpret_cast<float4 *>(img + i) = v;
        }
        __syncthreads();
    }
    // thread = 4 consecutive outputs of one row (a quad): the 3 x (3 S + 3) input window they share
    // read once, the plane's 9 weights once, the index arithmetic once per quad
    constexpr int NC = 3 * S + 3;
    const int nqd = (p.Wo + 3) >> 2, pq = p.RB * nqd;
    for (int e = tid; e < npl * pq; e += 256) {
        const int pl = dw_div(e, pq, p.inv_pq), rem = e - pl * pq;
        const int orow = dw_div(rem, nqd, p.inv_nqd), qd = rem - orow * nqd;
        if (orow >= nrow) continue;
        const int r0 = (oh0 + orow) * S - p.ph, cl = 4 * S * qd - p.pw;
        const float *xs = img + lead + pl * hw + (r0 - rlo) * p.W + cl, *ws = wsm + pl * 9;
        float wv[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) wv[t] = ws[t];
        bool cok[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) cok[c] = (unsigned)(cl + c) < (unsigned)p.W;
        float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
            const bool rok = (unsigned)(r0 + ky) < (unsigned)p.H;
            float v[NC];
#pragma unroll
            for (int c = 0; c < NC; ++c) v[c] = (rok && cok[c]) ? xs[ky * p.W + c] : 0.0f;
#pragma unroll
            for (int kx = 0; kx < 3; ++kx)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[j] = __fmaf_rn(v[j * S + kx], wv[3 * ky + kx], acc[j]);
        }
        int c = c0 + pl;
        c -= dw_div(c, p.C, p.inv_c) * p.C;
        float *yo = p.y + ((P0 + pl) * p.Ho + oh0 + orow) * p.Wo + 4 * qd;
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = dn_out(p.fz, qv, c, acc[j]);
        if ((p.Wo & 3) == 0) {
            *reinterpret_cast<float4 *>(yo) = make_float4(o[0], o[1], o[2], o[3]);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (4 * qd + j < p.Wo) yo[j] = o[j];
        }
    }
}

// The exact grouped / depthwise convolution: QCustomConv2dTorch's per-group im2col + x @ w^T
// (approx_calculation.py:686-711) and the exact branch of QCustomBNConv2dTorch for groups > 1
// (x @ y[:, i], :797 -- MobileNetV2's depthwise layers, BASELINE config 1).  One output = fp32
// FMAs in the im2col k order (input channel, ky, kx) with the padding read as zeros (0 * w keeps a
// non-finite weight's NaN, as the im2col product does); any fp32 input.  Thread = (image, output
// channel, output row, GC_OW consecutive output columns), the input row segment the GC_OW outputs
// share loaded once per (channel, ky) when the window's width and stride are compile-time (KW > 0;
// KW = 0: the general loop).  HBM-bound: x is read about once (the row overlap of neighbouring
// threads hits L2), y written once -- (x + y + w) bytes per launch.
struct GcArgs {
    const float *x, *w;
    float *y;
    int64_t Cin, H, W, Cout, Ho, Wo, total;  // total = Bn Cout Ho ceil(Wo / GC_OW)
    int cig, cog, kh, kw, sh, sw, ph, pw, dh, dw;
    DnFuse fz;                               // the fused layer tail (DenseArgs)
};
constexpr int GC_OW = 4;

template <typename I, int KW, int SW>
__global__ __launch_bounds__(256) void dn_group_conv(const GcArgs p) {
    constexpr int SEG = KW > 0 ? (GC_OW - 1) * SW + KW : 1;
    const I wq = (I)((p.Wo + GC_OW - 1) / GC_OW), Ho = (I)p.Ho, Cout = (I)p.Cout;
    const int kh = p.kh, kw = KW > 0 ? KW : p.kw, sw = KW > 0 ? SW : p.sw;
    const DnQv qv = dn_qv(p.fz);
    if (blockIdx.x == 0)
        for (int64_t c = threadIdx.x; c < p.Cout; c += 256) dn_bias_out(p.fz, c);
    for (I t = (I)blockIdx.x * 256 + (I)threadIdx.x; t < (I)p.total; t += (I)gridDim.x * 256) {
        const I q = t % wq, r = t / wq, ho = r % Ho, plane = r / Ho;  // plane = image Cout + co
        const I co = plane % Cout, n = plane / Cout, c0 = (co / (I)p.cog) * (I)p.cig;
        const int64_t wo0 = (int64_t)q * GC_OW, wi0 = wo0 * sw - p.pw;
        float acc[GC_OW];
#pragma unroll
        for (int j = 0; j < GC_OW; ++j) acc[j] = 0.0f;
        const float *wp = p.w + (int64_t)co * p.cig * kh * kw;
        float wmx = 0.0f, wb = 0.0f;
        if (p.fz.wq.mx) {
            wmx = dn_wmx(p.fz, co);
            wb = fq_bias(wmx, p.fz.wq.E, p.fz.wq.M);
        }
        for (int ci = 0; ci < p.cig; ++ci) {
            const float *xp = p.x + ((int64_t)n * p.Cin + c0 + ci) * p.H * p.W;
            for (int ky = 0; ky < kh; ++ky) {
                const int64_t hi = (int64_t)ho * p.sh - p.ph + (int64_t)ky * p.dh;
                const bool hok = hi >= 0 && hi < p.H;
                const float *xr = xp + (hok ? hi : 0) * p.W;
                const float *wr = wp + (ci * kh + ky) * kw;
                if constexpr (KW > 0) {  // dilation 1 (dn_group_conv launch)
                    float seg[SEG];
#pragma unroll
                    for (int s = 0; s < SEG; ++s) {
                        const int64_t wi = wi0 + s;
                        seg[s] = (hok && wi >= 0 && wi < p.W) ? dn_in(p.fz, qv, xr[wi]) : 0.0f;
                    }
#pragma unroll
                    for (int kx = 0; kx < KW; ++kx) {
                        const float wv = dn_wq(p.fz, wmx, wb, wr[kx]);
#pragma unroll
                        for (int j = 0; j < GC_OW; ++j) acc[j] = __fmaf_rn(seg[j * SW + kx], wv, acc[j]);
                    }
                } else {
                    for (int kx = 0; kx < kw; ++kx) {
                        const float wv = dn_wq(p.fz, wmx, wb, wr[kx]);
#pragma unroll
                        for (int j = 0; j < GC_OW; ++j) {
                            const int64_t wi = wi0 + (int64_t)j * sw + (int64_t)kx * p.dw;
                            acc[j] = __fmaf_rn((hok && wi >= 0 && wi < p.W) ? dn_in(p.fz, qv, xr[wi]) : 0.0f, wv, acc[j]);
                        }
                    }
                }
            }
        }
        float *yp = p.y + ((int64_t)plane * p.Ho + ho) * p.Wo;
#pragma unroll
        for (int j = 0; j < GC_OW; ++j)
            if (wo0 + j < p.Wo) yp[wo0 + j] = dn_out(p.fz, qv, co, acc[j]);
    }
}

}  // namespace fp8a
