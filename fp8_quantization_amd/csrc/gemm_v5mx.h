// gemm_v5mx.h -- the v5 integer-adder model's GEMM / implicit-GEMM convolution on the matrix core.
// DESIGN.md §3h.
//
// The v5 term (exact_term_v5, fp8approx_device.h; the reference's approx_mult_new,
// approx_matmul_whole_v5.py:155-182) is integer arithmetic on the operands' codes:
//     r = c_a + c_b' + T[m_a][m_b]      c = (expo << M) + mant (exact decode, clip_OF),
//                                        c_b' = c_b - (bA + bB - bR) << M
//     r = v5_ofuf(r)                     the (E+M)-bit adder's wrap with the OF / UF switches
//     term = sign(a) sign(b) x the E5M2 value of code r at bias bR
// With the wrap on (sim_hw_add_OFUF, BASELINE config 3) r is a 7-bit E5M2 code, and bf16 bits
// r << 5 are EXACTLY that code's value at bias 127 -- the subnormal band (r < 4) lands on bf16
// denormals, which v_mfma_f32_16x16x32_bf16 keeps exactly (measured: tools/mfma_bf16_denorm.hip,
// profiles/mfma_bf16_denorm_r04.txt).  So per (A element, 16 columns) the kernel computes the 16
// terms' bf16 bits with packed 16-bit integer ops and the matrix core sums them against a
// one-hot selection operand worth 2^(127 - bR) (the bias moved back), in fp32.
//
// The packed form, per column pair (two 16-bit lanes; the constants apply to both halves):
//   B side (v5mx_decode_b, per (k, n, m_a)): e = sign(b) << 15 | (0x2000 + (T' << 5)), T' =
//     c_b' + T[m_a][m_b] folded into [-256, 255] modulo 128 beyond [-128, 128] (there r < 0, or
//     r > 127, whatever c_a, and the wrap / OF / UF read only r mod 128 and which side) -- so
//     every lane value 0x2000 + 32 r stays in [0, 0x4FC0] and the addition below never carries
//     into bit 15;
//   A side (the A pre-pass, wfmt 4): w = (sign(a) << 15 | c_a << 5) in both halves;
//   t = e + w: bit 15 = sign(a) xor sign(b), low bits 0x2000 + 32 r;
//   UF (r < 0 -> r & 3):   lo = (t & 0x8060) | 0x2000,  t = max_u16(t, lo)   (same sign bit)
//   OF (r > 127 -> 127):   hi = (t & 0x8000) | 0x2FE0,  t = min_u16(t, hi)
//   wrap (r & 127) and the offset off: bits = t & 0x8FE0.
// Each switch drops its two operations when off (template UF / OF); the wrap alone is one AND.
// Zero-padded K slots would add the nonzero term of a zero operand (the reference pads the
// K dimension only where its im2col does, which the word image's zero border reproduces), so the
// last staged tile masks the lanes of K-steps past the end.
//
// Tile 128 x 32: 4 waves = 2 column groups of 16 x 2 row groups of 64 rows (4 16-row blocks);
// per staged tile of 8 K-steps, lane (r16, g) holds the A words of K-steps 2 g, 2 g + 1 of its
// rows; per (block, K-step) 2 ds_read_b128 fetch the 16 columns' table words of its m_a, 8
// column pairs give 16 bf16 terms, 2 MFMAs (16x16x32, 8 terms per lane) sum them.
// E5M2 (M = 2) only; E4M3 / E3M4 v5 and the unwrapped adder keep gemm_fast_kernel<TM_V5>.
#pragma once
#include "fp8approx_common.h"
#include "gemm_f8mx.h"

namespace fp8a {

constexpr int V5_BMT = 128, V5_BNT = 32, V5_TTW = 4 * 16 + 8;  // table words per K-step: [m_a][16 pairs] + pad
constexpr uint32_t V5_OFF = 0x20002000u;

// (the A words, wfmt 4: v5_word_a in gemm_f8mx.h, written by xm_decode_a)

// B pre-pass: per (k, n) of [kpad][npad] the four table words (m_a = 0..3) of the column as
// u16 lanes (uint2: m_a 0 | 1 << 16, 2 | 3 << 16); padding entries are zero (masked / dropped).
#if FP8A_OWN_V5
__global__ __launch_bounds__(256) void v5mx_decode_b(const GemmArgs p, int64_t kpad) {
    const int a_b = *p.bA, r_b = *p.bR, M = p.Mw;
    uint2 *out = reinterpret_cast<uint2 *>(const_cast<uint2 *>(p.bqw));
    const int64_t total = kpad * p.npad;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = i / p.npad, n = i - k * p.npad;
        uint2 o = make_uint2(0u, 0u);
        if (k < p.K && n < p.N) {
            const float b = p.B[k * p.sbk + n * p.sbn];
            const int b_b = p.bB[n * p.bBs];
            int e, m;
            exact_dec(b, dfmt(p.E, M, b_b, false), true, e, m);
            const int32_t cb = (e - (a_b + b_b - r_b)) * (1 << M) + m;
            const uint32_t sg = b < 0.0f ? 0x8000u : 0u;
            uint32_t h[4];
#pragma unroll
            for (int ma = 0; ma < 4; ++ma) {
                int32_t t = cb + p.tab.raw[(ma << M) | m];
                // r = c_a + t, c_a in [0, 127]: beyond [-128, 128] the sign of r (or r > 127) no
                // longer depends on c_a, and the switches read only r mod 128 there
                if (t > 128) t = 128 + ((t - 128) & 127);
                if (t < -128) t = -256 + (t & 127);
                h[ma] = sg | (uint32_t)(0x2000 + t * 32);
            }
            o = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
        }
        out[i] = o;
    }
}
#else
__global__ void v5mx_decode_b(const GemmArgs p, int64_t kpad);
#endif  // FP8A_OWN_V5

typedef unsigned short v5_u2 __attribute__((ext_vector_type(2)));
typedef short v5_s8 __attribute__((ext_vector_type(8)));
typedef __bf16 v5_bf8 __attribute__((ext_vector_type(8)));
typedef float v5_f4 __attribute__((ext_vector_type(4)));

template <bool UF, bool OF>
__device__ __forceinline__ uint32_t v5_bits(uint32_t e, uint32_t w) {
    v5_u2 t = __builtin_bit_cast(v5_u2, e) + __builtin_bit_cast(v5_u2, w);
    if (UF) {
        const uint32_t lo = (__builtin_bit_cast(uint32_t, t) & 0x80608060u) | V5_OFF;
        t = __builtin_elementwise_max(t, __builtin_bit_cast(v5_u2, lo));
    }
    if (OF) {
        const uint32_t hi = (__builtin_bit_cast(uint32_t, t) & 0x80008000u) | 0x2FE02FE0u;
        t = __builtin_elementwise_min(t, __builtin_bit_cast(v5_u2, hi));
    }
    return __builtin_bit_cast(uint32_t, t) & 0x8FE08FE0u;
}

#if FP8A_OWN_V5
template <bool UF, bool OF>
__global__ __launch_bounds__(256) void gemm_v5mx_kernel(const GemmArgs p) {
    constexpr int NT = 256, BMT = V5_BMT, BNT = V5_BNT, APR = BMT / 64, SR = 4096 / BNT, CP = BNT + 1;
    struct Stage {
        uint32_t tt[XBK][V5_TTW];          // [kk][m_a][16 column pairs] (+ pad: 8 banks per K-step)
        uint32_t aw[XBK / 2][2 * BMT + 32];  // [kk / 2][row][kk % 2], as gemm_f8mx_kernel
    };
    union Smem {
        Stage st;
        float ct[SR * CP];
    };
    __shared__ __attribute__((aligned(16))) Smem smu;
    auto &sm = smu.st;

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wvu = __builtin_amdgcn_readfirstlane(wv);
    const int wc = wvu & 1, wr = wvu >> 1;  // the wave's column group and row group
    const int64_t num_mt = (p.M + BMT - 1) / BMT;
    const int64_t tiles = num_mt * ((p.N + BNT - 1) / BNT);
    const int64_t bid = (int64_t)blockIdx.x % tiles, split = (int64_t)blockIdx.x / tiles;
    const int64_t m0 = (bid % num_mt) * BMT;
    const int64_t n0 = (bid / num_mt) * BNT;
    const int kbeg = (int)(split * p.kchunk), kend = (int)min(p.K, (int64_t)kbeg + p.kchunk), K32 = (int)p.K;
    const int bR = *p.bR;
    const bool biasbad = !(bR >= -60 && bR <= 120);
    // the selection operand's value 2^s and the epilogue's remaining power of two
    const int s_sel = min(127 - bR, 126);
    const float escale = __uint_as_float((uint32_t)min(max(127 + (127 - bR - s_sel), 1), 254) << 23);

    // B staging: thread = (K-step kk, column n) of the tile: one uint2 (four table words)
    const int bkk = tid >> 5, bn = tid & 31;
    const uint2 *bsrc = p.bqw + (int64_t)(kbeg + bkk) * p.npad + n0 + bn;

    // A staging as gemm_f8mx_kernel (word image / matrix words)
    const int arow = p.conv ? lane : (tid >> 2), akp = p.conv ? wvu : (tid & 3);
    uint32_t aoff[APR];
    const uint32_t phw = (uint32_t)(p.awH * p.awW), uW = (uint32_t)p.awW;
#pragma unroll
    for (int i = 0; i < APR; ++i) {
        const int64_t m = min(m0 + arow + 64 * i, p.M - 1);
        if (p.conv) {
            const int64_t hw = p.Ho * p.Wo, img = m / hw, pix = m - img * hw, ho = pix / p.Wo, wo = pix - ho * p.Wo;
            aoff[i] = (uint32_t)(4 * (img * p.aw_c * (int64_t)phw + ho * p.sh * p.awW + wo * p.sw + (p.awpw - p.pw)));
        } else {
            aoff[i] = (uint32_t)(4 * (m * p.awld + 2 * akp));
        }
    }
    const __amdgpu_buffer_rsrc_t arsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(p.aw), (short)0, -1, 0x00020000);
    const int khw = p.kh * p.kw;
    uint32_t wa[APR][2];
    uint2 wb;
    auto load_tile = [&](int k0) {
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            uint32_t ko;
            if (p.conv) {
                const int k = min(k0 + 2 * akp + r, K32 - 1);
                const uint32_t c = fastdiv((uint32_t)k, p.kk_mul, p.kk_shift);
                const uint32_t t = (uint32_t)k - c * (uint32_t)khw;
                const uint32_t ky = fastdiv(t, p.kw_mul, p.kw_shift);
                const uint32_t kx = t - ky * (uint32_t)p.kw;
                ko = 4u * (c * phw + ky * (uint32_t)p.dh * uW + kx * (uint32_t)p.dw);
            } else {
                ko = 4u * (uint32_t)(k0 + r);
            }
            ko = __builtin_amdgcn_readfirstlane(ko);
#pragma unroll
            for (int i = 0; i < APR; ++i) wa[i][r] = __builtin_amdgcn_raw_buffer_load_b32(arsrc, (int)aoff[i], (int)ko, 0);
        }
        wb = bsrc[(int64_t)(k0 - kbeg) * p.npad];
    };
    load_tile(kbeg);

    // the one-hot selection operands: MFMA q sums columns 8 q .. 8 q + 7 of a K-step; lane (n, g')
    // holds B rows 8 g' .. 8 g' + 7 of column n: 2^s at row 8 g' + (n - 8 q) when n is in the half
    v5_s8 sel[2];
    {
        const int n = lane & 15;
        const short sv = (short)((127 + s_sel) << 7);
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int i = 0; i < 8; ++i) sel[q][i] = (n - 8 * q == i) ? sv : (short)0;
    }
    v5_f4 dq[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) dq[b] = (v5_f4){0.0f, 0.0f, 0.0f, 0.0f};

    for (int k0 = kbeg; k0 < kend; k0 += XBK) {
#pragma unroll
        for (int i = 0; i < APR; ++i)
            *reinterpret_cast<uint2 *>(&sm.aw[akp][2 * (arow + 64 * i)]) = make_uint2(wa[i][0], wa[i][1]);
        {  // table words [kk][m_a][pair]: this thread's column n = 2 pair + (n & 1) -> u16 lanes
            uint16_t *tt16 = reinterpret_cast<uint16_t *>(&sm.tt[bkk][0]);
            tt16[0 * 32 + bn] = (uint16_t)wb.x;
            tt16[1 * 32 + bn] = (uint16_t)(wb.x >> 16);
            tt16[2 * 32 + bn] = (uint16_t)wb.y;
            tt16[3 * 32 + bn] = (uint16_t)(wb.y >> 16);
        }
        __syncthreads();
        if (k0 + XBK < kend) load_tile(k0 + XBK);

        const int r16 = lane & 15, g = lane >> 4;
        const bool ragged = k0 + XBK > kend;  // (wave-uniform) the last tile: mask K-steps past the end
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint2 aw2 = *reinterpret_cast<const uint2 *>(&sm.aw[g][2 * (16 * (4 * wr + b) + r16)]);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint32_t w = h ? aw2.y : aw2.x;
                const uint32_t *row = &sm.tt[2 * g + h][((w >> 5) & 3u) * 16 + wc * 8];
                const uint4 e0 = *reinterpret_cast<const uint4 *>(row);
                const uint4 e1 = *reinterpret_cast<const uint4 *>(row + 4);
                uint32_t t[8] = {v5_bits<UF, OF>(e0.x, w), v5_bits<UF, OF>(e0.y, w), v5_bits<UF, OF>(e0.z, w),
                                 v5_bits<UF, OF>(e0.w, w), v5_bits<UF, OF>(e1.x, w), v5_bits<UF, OF>(e1.y, w),
                                 v5_bits<UF, OF>(e1.z, w), v5_bits<UF, OF>(e1.w, w)};
                if (ragged && k0 + 2 * g + h >= kend) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) t[j] = 0u;
                }
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    v5_s8 av;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        av[2 * j] = (short)(t[4 * q + j] & 0xFFFFu);
                        av[2 * j + 1] = (short)(t[4 * q + j] >> 16);
                    }
                    dq[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v5_bf8, av),
                                                                   __builtin_bit_cast(v5_bf8, sel[q]), dq[b], 0, 0, 0);
                }
            }
        }
        __syncthreads();
    }
    if (biasbad && blockIdx.x == 0 && tid == 0) atomicOr(p.flag, fb_bits(p, true));

    // D of row block b: lane l holds rows 4 (l >> 4) .. + 3, column l & 15 -> the [SR][BNT] slab
    float *ct = smu.ct;
    const int ety = tid & 15, etx = tid >> 4, cb = etx % (BNT / 4), sub = etx / (BNT / 4);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int rb = 16 * (4 * wr + b);
#pragma unroll
        for (int i = 0; i < 4; ++i) ct[(rb + 4 * (lane >> 4) + i) * CP + 16 * wc + (lane & 15)] = dq[b][i] * escale;
    }
    __syncthreads();
    float acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = ct[(64 * sub + ety * TM + i) * CP + cb * TN + j];
    store_tile<false>(p, split, m0 + 64 * sub, n0, ety, cb, acc);
}
#endif  // FP8A_OWN_V5

}  // namespace fp8a
