// gemm_tt16.h -- the E3M4 tile-table kernel in packed f16 with matrix-core summation.  DESIGN.md §3c.
//
// Same term as gemm_tt_kernel<4, F7> (gemm_tt.h; v9:51-113):
//     term = Q_R(V(m_a, m_b) c_a c_b),   V = min(sig_a sig_b - T[m_a][m_b] 2^-4, kb x its binade)
// For E3M4 every quantity the rounding sees is f16-exact in a shifted frame: V has at most 10
// significant bits (sig_a, sig_b have 5), c_a, c_b are powers of two, and the rounded term has 5.
// Per tile the kernel works in units of 2^-(bA - 1 + S),
//     c_a' = c_a 2^(bA-1) in [2^-4, 2^7],   c_b' = c_b 2^S,   S = min(min bB - 7, bR - bA + 9)
// over the tile's columns (operands reach one binade above the format's top: the quantizer's
// rint bias), which puts every product x = V c_a' c_b' below 2^10 and the result grid's smallest
// normal 2^Emn, Emn = bA - bR + S, inside [2^-10, 2^9]: x is exact (its last bit is at or above
// 2^-24 whenever x >= half the grid's spacing; smaller products round to 0 either way) and the
// magic constant C = max(2^floor(log2 x), 2^Emn) x 1.5 x 2^6 is a normal f16.  Q_R is then, on two
// columns at once: x = t c_a', pe = x & EXP, C = max(pe x 96, cmin), r = (x + C) - C (v_pk_*
// f16 ops; measured ~2x the issue cost of an f32 add each, for two products).  The pre-clamp bound is
// (2 - 2^-4 - 2^-10) x binade (f16-exact; rounds like the reference's saturating mantissa, F6,
// and its subnormal top tie).  F7 (signed tables): sign of fma(sig_a sig_b c_b', c_a', 2^(Emn-5)).
// A tile whose biases leave this window (Emn < -10, or max bB > S + 13: a nonzero c_b' below
// 2^-16, where V c_b' would lose bits) sets a bit of the launch's flag word (as do the pre-passes
// for an operand more than one binade above the format's top, or V >= 4), and gemm_tt_kernel<4, F7, true> (the f32
// form, reading these same pre-decoded operands) reruns the launch.
//
// Summation: the rounded terms are f16-exact, so the matrix core adds them -- one
// v_mfma_f32_16x16x32_f16 per 16-row block and 8 columns multiplies the lanes' terms by a
// constant 0/1 selection operand (the f32 sum differs from an in-order sum only by order).
// Lane = (row r16 of each 16-row block, K-step g of the 4-step tile); per A element the lane
// reads its 16 columns (four ds_read_b64, conflict-free: rows 136 B and K-steps 2176 B apart)
// and spends 6 packed ops per column pair.
#pragma once
#include "fp8approx_common.h"
#include "gemm_f8mx.h"
#include "gemm_tt.h"

namespace fp8a {

// Sub-stages per staged tile: NS x TT16_XK K-steps share one barrier pair, one prefetch and one
// table build phase (round 6: 2, was 1 -- the E2M5 tile-table kernel's lesson, §3r: the kernel's
// per-tile overhead, not its math, was the larger share)
#ifndef TT16_NSUB
#define TT16_NSUB 2
#endif
#ifndef TT16_NSUB_F7
#define TT16_NSUB_F7 TT16_NSUB  // (F7 doubles the LDS tables: 2 sub-stages = 40 KB, 4 blocks per CU)
#endif
template <bool F7> struct Tt16Cfg {
    static constexpr int RB = 8;             // 16-row blocks per wave
    static constexpr int BMR = 16 * RB;      // tile rows
    static constexpr int AWS = BMR + 16;     // A words per K-step in LDS (K-steps 16 banks apart)
    static constexpr int APT = TT16_XK * BMR / NT;  // A words staged per thread and sub-stage
    static constexpr int NS = F7 ? TT16_NSUB_F7 : TT16_NSUB;
    static constexpr int XKT = NS * TT16_XK;        // K-steps per staged tile
};

template <bool F7> struct Tt16Smem {
    using C = Tt16Cfg<F7>;
    union {
        struct {
            uint32_t tt[C::XKT * TT16_KS];                  // V c_b' pairs [kk][m_a][column pair]
            uint32_t tg[F7 ? C::XKT * TT16_KS : 1];         // sig_a sig_b c_b' pairs (F7)
            uint32_t img[F7 ? 256 : 128];                   // the static image, f16 [m_b][m_a]
            uint32_t aw[C::XKT * C::AWS];                   // A words [kk][row]
            int bmin, bmax;                                 // the tile's column biases
        } t;
        float ct[64 * XM_CP];  // epilogue transpose slice
    } u;
};

#if FP8A_OWN_TT
template <bool F7>
__global__ __launch_bounds__(NT, 6) void gemm_tt16_kernel(const GemmArgs p) {
    using Cf = Tt16Cfg<F7>;
    constexpr int RB = Cf::RB, BMR = Cf::BMR, AWS = Cf::AWS, APT = Cf::APT, NS = Cf::NS, XKT = Cf::XKT;
    __shared__ __attribute__((aligned(16))) Tt16Smem<F7> sm;
    auto &S = sm.u.t;

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wvu = __builtin_amdgcn_readfirstlane(wv);
    const int64_t num_mt = (p.M + BMR - 1) / BMR;
    const int64_t tiles = num_mt * ((p.N + BN - 1) / BN);
    const int64_t bid = (int64_t)blockIdx.x % tiles, split = (int64_t)blockIdx.x / tiles;
    const int64_t m0 = (bid % num_mt) * BMR;
    const int64_t n0 = (bid / num_mt) * BN;
    const int kbeg = (int)(split * p.kchunk), kend = (int)min(p.K, (int64_t)kbeg + p.kchunk), K32 = (int)p.K;
    const int bA = *p.bA, bR = *p.bR;

    // static image -> LDS; the tile's column-bias range -> the frame shift S
    for (int e = tid; e < (F7 ? 256 : 128); e += NT) S.img[e] = p.lutw[TT16_IMG + e];
    if (tid == 0) {
        S.bmin = 1 << 30;
        S.bmax = -(1 << 30);
    }
    __syncthreads();
    if (tid < BN) {
        const int bb = p.bB[min(n0 + tid, p.N - 1) * p.bBs];
        atomicMin(&S.bmin, bb);
        atomicMax(&S.bmax, bb);
    }
    __syncthreads();
    const int bmin = S.bmin, bmax = S.bmax;
    const int fs = min(bmin - 7, bR - bA + 9), emn = bA - bR + fs;
    if (tid == 0 && (emn < -10 || bmax > fs + 13)) atomicOr(p.flag, emn < -10 ? 2u : 16u);  // outside the f16 window
    const int ec = min(max(emn, -10), 9);
    const uint32_t cm1 = tt16_pow2(ec + 6, 0u) | 0x200u;                                    // 1.5 x 2^(Emn + 6)
    const uint32_t th1 = ec - 5 >= -14 ? tt16_pow2(ec - 5, 0u) : (1u << (ec - 5 + 24));  // 2^(Emn - 5)
    const tt16_h2 cmin2 = __builtin_bit_cast(tt16_h2, cm1 | (cm1 << 16));
    const tt16_h2 thr2 = __builtin_bit_cast(tt16_h2, th1 | (th1 << 16));
    const float osc = p2(-(bA - 1 + fs));  // D units -> output units
    const int sb16 = fs - 127 + 15;    // f32 exponent field of c_b -> f16 exponent field of c_b'

    // build units: thread = (column pair cp, K-step bkk, rows 8 rp .. 8 rp + 7)
    const int cp = tid & 31, bkk = (tid >> 5) & 3, rp = tid >> 7;
    const uint32_t npad4 = (uint32_t)p.npad * 4u;
    const uint32_t boff = (uint32_t)(kbeg + bkk) * npad4 + (uint32_t)(n0 + 2 * cp) * 4u;
    const __amdgpu_buffer_rsrc_t brsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint2 *>(p.bqw), (short)0, -1, 0x00020000);

    // A staging: words (rows arow + 64 i, K-step akk); conv: lane = row, K-step = wave (uniform);
    // matrix: four threads per row.  Rows past M re-read row M - 1.
    const int arow = p.conv ? lane : (tid >> 2), akk = p.conv ? wvu : (tid & 3);
    uint32_t aoff[APT];
    const uint32_t phw = (uint32_t)(p.awH * p.awW), uW = (uint32_t)p.awW;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
        const int64_t m = min(m0 + arow + 64 * i, p.M - 1);
        if (p.conv) {
            const int64_t hw = p.Ho * p.Wo, img_i = m / hw, pix = m - img_i * hw, ho = pix / p.Wo, wo = pix - ho * p.Wo;
            aoff[i] = (uint32_t)(4 * (img_i * p.aw_c * (int64_t)phw + ho * p.sh * p.awW + wo * p.sw + (p.awpw - p.pw)));
        } else {
            aoff[i] = (uint32_t)(4 * (m * p.awld + akk));
        }
    }
    const __amdgpu_buffer_rsrc_t arsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(p.aw), (short)0, -1, 0x00020000);
    const int khw = p.kh * p.kw;
    uint32_t wa[NS][APT];
    uint2 wb[NS];
    auto load_tile = [&](int k0) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int ks = k0 + TT16_XK * s;
            uint32_t ko;
            if (p.conv) {
                const int k = min(ks + akk, K32 - 1);  // wave-uniform; clamped: the word image ends at channel K - 1
                const uint32_t c = fastdiv((uint32_t)k, p.kk_mul, p.kk_shift);
                const uint32_t t = (uint32_t)k - c * (uint32_t)khw;
                const uint32_t ky = fastdiv(t, p.kw_mul, p.kw_shift);
                const uint32_t kx = t - ky * (uint32_t)p.kw;
                ko = 4u * (c * phw + ky * (uint32_t)p.dh * uW + kx * (uint32_t)p.dw);
            } else {
                ko = 4u * (uint32_t)ks;  // (the matrix words are zero-padded to Kpad)
            }
            ko = __builtin_amdgcn_readfirstlane(ko);
#pragma unroll
            for (int i = 0; i < APT; ++i) {
                wa[s][i] = __builtin_amdgcn_raw_buffer_load_b32(arsrc, (int)aoff[i], (int)ko, 0);  // (past K: zeroed at staging)
            }
            const uint32_t kb = __builtin_amdgcn_readfirstlane((uint32_t)(ks - kbeg) * npad4);
            wb[s] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(brsrc, (int)boff, (int)kb, 0));
        }
    };
    load_tile(kbeg);

    // selection operands of v_mfma_f32_16x16x32_f16: lane l holds B[k = 8 (l >> 4) + j][col l & 15];
    // sh[0] has 1.0 at j = col (col < 8), sh[1] at j = col - 8 (col >= 8)
    tt16_h8 sh[2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < 8; ++j) sh[h][j] = ((lane & 15) == 8 * h + j) ? (_Float16)1.0f : (_Float16)0.0f;
    tt16_f4 dq[RB];
#pragma unroll
    for (int b = 0; b < RB; ++b) dq[b] = (tt16_f4){0.0f, 0.0f, 0.0f, 0.0f};
    const tt16_h2 kc2 = __builtin_bit_cast(tt16_h2, 0x56005600u);  // 96 = 1.5 x 2^6
    const int r16 = lane & 15, g = lane >> 4;
    const uint32_t tbase = (uint32_t)g * (TT16_KS * 4) + (uint32_t)wvu * 32u;  // bytes: K-step g, the wave's columns
    typedef const volatile __attribute__((address_space(3))) uint64_t tt16_lds_u64;
    const char *tt0 = reinterpret_cast<const char *>(S.tt);
    const char *tg0 = reinterpret_cast<const char *>(S.tg);
    __syncthreads();  // the static image is in LDS

    for (int k0 = kbeg; k0 < kend; k0 += XKT) {
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int i = 0; i < APT; ++i)  // (K-steps past the group's last channel: zero words)
                S.aw[(TT16_XK * s + akk) * AWS + arow + 64 * i] = (p.conv && k0 + TT16_XK * s + akk >= K32) ? 0u : wa[s][i];
#pragma unroll
        for (int s = 0; s < NS; ++s) {  // build: tt[kk][m_a][cp] = (V(m_a, m_b1) c_b1' : V(m_a, m_b0) c_b0') for m_a = 8 rp .. 8 rp + 7
            const uint2 wbs = wb[s];
            const int kkb = TT16_XK * s + bkk;
            auto cbf16 = [&](uint32_t w) -> uint32_t {  // f32 c_b bits -> f16 c_b' bits (0 for a zero B)
                const int e = (int)((w >> 23) & 0xFFu) + sb16;  // f16 exponent field; <= 0: subnormal
                const uint32_t mag = e >= 1 ? ((uint32_t)min(e, 30) << 10) : (e >= -9 ? (0x200u >> (-e)) : 0u);
                return (w & 0x7F800000u) ? (((w >> 16) & 0x8000u) | mag) : 0u;
            };
            const tt16_h2 cbh = __builtin_bit_cast(tt16_h2, cbf16(wbs.x) | (cbf16(wbs.y) << 16));  // (c_b1' : c_b0')
            const uint4 v0 = *reinterpret_cast<const uint4 *>(&S.img[(wbs.x & 15u) * 8 + 4 * rp]);
            const uint4 v1 = *reinterpret_cast<const uint4 *>(&S.img[(wbs.y & 15u) * 8 + 4 * rp]);
            const uint32_t a0[4] = {v0.x, v0.y, v0.z, v0.w}, a1[4] = {v1.x, v1.y, v1.z, v1.w};
            uint32_t *d = &S.tt[kkb * TT16_KS + 8 * rp * TT16_RS + cp];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const tt16_h2 lo = __builtin_bit_cast(tt16_h2, __builtin_amdgcn_perm(a1[i], a0[i], 0x05040100u)) * cbh;
                const tt16_h2 hi = __builtin_bit_cast(tt16_h2, __builtin_amdgcn_perm(a1[i], a0[i], 0x07060302u)) * cbh;
                d[(2 * i) * TT16_RS] = __builtin_bit_cast(uint32_t, lo);
                d[(2 * i + 1) * TT16_RS] = __builtin_bit_cast(uint32_t, hi);
            }
            if (F7) {
                const uint4 g0 = *reinterpret_cast<const uint4 *>(&S.img[128 + (wbs.x & 15u) * 8 + 4 * rp]);
                const uint4 g1 = *reinterpret_cast<const uint4 *>(&S.img[128 + (wbs.y & 15u) * 8 + 4 * rp]);
                const uint32_t b0[4] = {g0.x, g0.y, g0.z, g0.w}, b1[4] = {g1.x, g1.y, g1.z, g1.w};
                uint32_t *e = &S.tg[kkb * TT16_KS + 8 * rp * TT16_RS + cp];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const tt16_h2 lo = __builtin_bit_cast(tt16_h2, __builtin_amdgcn_perm(b1[i], b0[i], 0x05040100u)) * cbh;
                    const tt16_h2 hi = __builtin_bit_cast(tt16_h2, __builtin_amdgcn_perm(b1[i], b0[i], 0x07060302u)) * cbh;
                    e[(2 * i) * TT16_RS] = __builtin_bit_cast(uint32_t, lo);
                    e[(2 * i + 1) * TT16_RS] = __builtin_bit_cast(uint32_t, hi);
                }
            }
        }
        __syncthreads();
        if (k0 + XKT < kend) load_tile(k0 + XKT);  // next tile's loads fly during this tile's math

#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int b = 0; b < RB; ++b) {
            const uint32_t w = S.aw[(TT16_XK * s + g) * AWS + 16 * b + r16];
            const tt16_h2 c2 = __builtin_bit_cast(tt16_h2, w & TT16_EXP2);
            const uint32_t a = ((w & 0x3FFu) << 1) + tbase + (uint32_t)(s * TT16_XK * TT16_KS * 4);
            uint32_t t[8], tg[F7 ? 8 : 1];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const uint64_t v = *(tt16_lds_u64 *)(tt0 + a + 8 * c);
                t[2 * c] = (uint32_t)v;
                t[2 * c + 1] = (uint32_t)(v >> 32);
                if (F7) {
                    const uint64_t u = *(tt16_lds_u64 *)(tg0 + a + 8 * c);
                    tg[2 * c] = (uint32_t)u;
                    tg[2 * c + 1] = (uint32_t)(u >> 32);
                }
            }
            uint32_t r[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const tt16_h2 x = __builtin_bit_cast(tt16_h2, t[q]) * c2;  // exact
                const tt16_h2 pe = __builtin_bit_cast(tt16_h2, __builtin_bit_cast(uint32_t, x) & 0x7C007C00u);
                const tt16_h2 cc = __builtin_elementwise_max(pe * kc2, cmin2);
                uint32_t rq = __builtin_bit_cast(uint32_t, (x + cc) - cc);
                if (F7) {  // sign of a b + 2^(Emn-5) (its rounding never crosses zero)
                    const tt16_h2 s = __builtin_elementwise_fma(__builtin_bit_cast(tt16_h2, tg[q]), c2,
                                                                thr2);
                    rq = (rq & 0x7FFF7FFFu) | (__builtin_bit_cast(uint32_t, s) & 0x80008000u);
                }
                r[q] = rq;
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint4 rv = make_uint4(r[4 * h], r[4 * h + 1], r[4 * h + 2], r[4 * h + 3]);
                dq[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(tt16_h8, rv), sh[h], dq[b], 0, 0, 0);
            }
        }
        __syncthreads();
    }

    // D of row block b: lane l holds rows 4 (l >> 4) + i, column l & 15 -> 64-row slices in LDS
    // (scaled to output units per column) -> each thread's 4x4 block
    float *ct = sm.u.ct;
    const int ety = tid & 15, etx = tid >> 4;
#pragma unroll
    for (int hs = 0; hs < BMR / 64; ++hs) {
        if (hs > 0) __syncthreads();
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                ct[(16 * b + 4 * (lane >> 4) + i) * XM_CP + 16 * wvu + (lane & 15)] = dq[4 * hs + b][i] * osc;
        __syncthreads();
        float acc[TM][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = ct[(ety * TM + i) * XM_CP + etx * TN + j];
        store_tile<false>(p, split, m0 + 64 * hs, n0, ety, etx, acc);
    }
}
#endif  // FP8A_OWN_TT

}  // namespace fp8a
