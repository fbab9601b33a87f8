// gemm_tt.h -- the tile-table kernel for the wider-mantissa formats (E3M4, E2M5).  DESIGN.md §3b.
//
// Same term as gemm_fast_kernel's table modes (v9:51-113) for on-grid operands
// with s2n and per-product quantization, no golden clip:
//     term = Q_R(V(m_a, m_b) c_a c_b),   V = min(sig_a sig_b - T[m_a][m_b] 2^-M, kb x its binade)
// with c = sign 2^floor(log2|x|) and kb = 2 - 2^-M - 2^-22, Q_R's pre-clamp (the mantissa
// saturates instead of carrying, F6, and the subnormal top tie rounds down).  The clamp scales
// with the value's binade, and c_a c_b is a power of two, so the clamp is applied once to the
// table value; Q_R is then its magic-constant rounding alone: pe = x & EXP, C = max(pe 1.5
// 2^(23-M), 2^(1-bR) 1.5 2^(23-M)), r = (x + C) - C.
//
// Tile table.  c_b depends only on the column, so every staged K-step builds, for the tile's 64
// columns, tt[kk][m_a][col] = V(m_a, m_b(col)) c_b(col) (2^M rows of 64 floats); the math loop
// (lane = tile row, wave = 16 columns, as gemm_f8mx_kernel) reads its row's 16 values with four
// ds_read_b128 and spends per product: one multiply by c_a, the 5-op rounding, one add.
//
// F7 (tables with negative entries): the reference takes the product's sign from Q_R(a b),
// which is -0 (sign +) for a b in [-2^(-bR-M), 0).  Since V > 0, the term's sign is then the
// sign of a b + 2^(-bR-M): one fma on a second table tg = sig_a sig_b c_b, and one v_bfi_b32.
//
// Operands are pre-decoded once per launch: an A element becomes c_a's sign and exponent bits
// (mantissa field zero) | m_a x the table row stride in its low bits; a B element c_b's bits | m_b.
// The pre-passes carry the fallback checks into the flag word (gemm_exact_kernel reruns).
#pragma once
#include "fp8approx_common.h"
#include "gemm_f8mx.h"

namespace fp8a {

constexpr int TT_IMG_FLOATS = 2048;       // static image: V [m_b][m_a] then sig_a sig_b [m_b][m_a]

// K-steps per staged tile of gemm_tt_kernel<MW, F7>: ~17 KB of table per tile
// E2M5 (unsigned table): 4 K-steps per staged tile (35 KB of table; 2 before round 6) -- half the
// per-tile staging, build barriers and prefetch waits per K-step: ResNet-50 E2M5 1,434 -> 1,520
// images/s with the band forms below (profiles/r06_ttxk/)
#ifndef TT_XK5
#define TT_XK5 4
#endif
__host__ __device__ constexpr int tt_xk(int MW, bool F7) { return (MW == 5 && !F7) ? TT_XK5 : (4 << (F7 ? 0 : 1)) >> (MW - 3); }

template <int MW, bool F7> struct TtCfg {
    static constexpr int NM = 1 << MW;                     // table rows (m_a codes)
    static constexpr int XK = tt_xk(MW, F7);
    static constexpr int PARTS = NM / 16;                  // build: 16 rows per thread
    static constexpr int UNITS = XK * 64 * PARTS;          // build units (<= 256 threads)
};

// B pre-pass for gemm_tt_kernel: words [Kpad][Npad] (c_b's bits | m_b, 0 for zeros and padding),
// and (block 0) the static image V / sig_a sig_b.
#if FP8A_OWN_TT
__global__ __launch_bounds__(256) void tt_decode_b(const GemmArgs p, int64_t kpad) {
    const int bA = *p.bA, bR = *p.bR, M = p.Mw, nm = 1 << M;
    const bool biasbad = !(xm_bias_ok(bA) && xm_bias_ok(bR));  // every output unit falls back
    bool bad = biasbad, win = true;  // win: gemm_tt16_kernel's f16 window
    if (blockIdx.x == 0) {
        float *img = const_cast<float *>(reinterpret_cast<const float *>(p.lutw));
        const float ulp = p2(-M), kb = 2.0f - p2(-M) - p2(-22);
        for (int e = threadIdx.x; e < nm * nm; e += blockDim.x) {
            const int mb = e >> M, ma = e & (nm - 1);
            const float s = (1.0f + ulp * ma) * (1.0f + ulp * mb);  // exact: 2M + 2 bits
            float v = __fmaf_rn(-(float)p.tab.raw[ma * nm + mb], ulp, s);  // exact
            v = fminf(v, __uint_as_float(__float_as_uint(v) & 0x7F800000u) * kb);
            img[e] = v;
            img[TT_IMG_FLOATS / 2 + e] = s;
            if (p.wfmt == 2) {  // gemm_tt16_kernel's f16 image (E3M4): V with the pre-clamp bound
                                // (2 - 2^-4 - 2^-10) x binade, then sig_a sig_b (gemm_tt16.h)
                uint16_t *h = reinterpret_cast<uint16_t *>(img + TT16_IMG);
                const float v16 = fminf(v, __uint_as_float(__float_as_uint(v) & 0x7F800000u) * (2.0f - p2(-M) - p2(-10)));
                h[e] = __builtin_bit_cast(uint16_t, (_Float16)v16);
                win = win && v16 < 4.0f;
                h[256 + e] = __builtin_bit_cast(uint16_t, (_Float16)s);
            }
        }
    }
    uint32_t *const bw = reinterpret_cast<uint32_t *>(const_cast<uint2 *>(p.bqw));
    const int64_t n = kpad * p.npad;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = i / p.npad, col = i - k * p.npad;
        uint32_t w = 0;
        if (k < p.K && col < p.N) {
            const int bb = p.bB[col * p.bBs];
            float c;
            uint32_t mc;
            const bool ok = stage_decode(p.B[k * p.sbk + col * p.sbn], M, (uint32_t)(128 - bb) << 23, true, c, mc) &&
                            xm_bias_ok(bb);
            if (!ok) fb_col(p, col);
            bad |= !ok;
            const uint32_t cb = __float_as_uint(c);
            win = win && ((cb >> 23) & 0xFFu) <= (uint32_t)(127 + 8 - bb);  // c_b at most one binade above the format's top
            if ((cb & 0x7FFFFFFFu) != 0u) w = (cb & TT_EXP) | mc;
        }
        bw[i] = w;
    }
    if (p.wfmt == 1 && p.Mw == 5 && p.ebr != nullptr) {  // gemm_tt_kernel's band test (E2M5): per (staged tile, 16 columns) the largest c_b exponent field
        const int xk = tt_xk(M, p.ttf7 != 0);
        const int64_t ng = p.npad / 16, nkg = kpad / xk;
        uint16_t *eb = const_cast<uint16_t *>(p.ebr);
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nkg * ng; i += (int64_t)gridDim.x * blockDim.x) {
            const int64_t kg = i / ng, g = i - kg * ng;
            uint32_t emax = 0;  // (0: every B element of the group is zero)
            for (int kk = 0; kk < xk; ++kk) {
                const int64_t k = kg * xk + kk;
                for (int j = 0; j < 16 && k < p.K; ++j) {
                    const int64_t col = 16 * g + j;
                    if (col >= p.N) break;
                    float c;
                    uint32_t mc;
                    stage_decode(p.B[k * p.sbk + col * p.sbn], M, (uint32_t)(128 - p.bB[col * p.bBs]) << 23, true, c, mc);
                    if ((__float_as_uint(c) & 0x7FFFFFFFu) != 0u) emax = max(emax, (__float_as_uint(c) >> 23) & 0xFFu);
                }
            }
            eb[i] = (uint16_t)emax;
        }
    }
    if (__syncthreads_or(bad ? 1 : 0) && threadIdx.x == 0) atomicOr(p.flag, fb_bits(p, biasbad));
    if (p.wfmt == 2 && __syncthreads_or(win ? 0 : 1) && threadIdx.x == 0) atomicOr(p.flag, 8u);  // (B, image)
}
#else
__global__ void tt_decode_b(const GemmArgs p, int64_t kpad);
#endif  // FP8A_OWN_TT

// Row halves per tile: E2M5 runs 128-row tiles on 8-wave workgroups that share one table build
// (its 32-row table makes the build ~20 % of the work at 64 rows; 99.5 -> 79.8 ms on the ResNet-18
// layer set), E3M4 64-row tiles (128 rows measured +-0 there).
template <int MW> constexpr int tt_rh() { return MW == 5 ? 2 : 1; }
template <int MW, bool F7> struct TtSmem {
    using C = TtCfg<MW, F7>;
    union {
        struct {
            float tt[C::XK][C::NM][TT_RS];  // V c_b
            float tg[F7 ? C::XK : 1][F7 ? C::NM : 1][TT_RS];  // sig_a sig_b c_b (F7)
        } t;
        float ct[64 * XM_CP];  // epilogue transpose slice
    } u;
    float img[F7 ? TT_IMG_FLOATS : TT_IMG_FLOATS / 2];
    uint32_t aw[C::XK][64 * tt_rh<MW>()];
};

// A16: the A words are gemm_tt16_kernel's (E3M4; c_a 2^bA as f16 in the high half, m_a x 68 in the
// low bits), and the kernel runs only when that kernel left its f16 window (flag bit 1).
#if FP8A_OWN_TT
// launches rerun in the f32 form (fp8a_fallback_stats [2], read by tt_rerun_stats in k_tt.hip)
__device__ unsigned long long g_tt_reruns;
#endif
#if FP8A_OWN_TT
template <int MW, bool F7, bool A16>
__global__ __launch_bounds__(NT * tt_rh<MW>()) void gemm_tt_kernel(const GemmArgs p) {
    constexpr int TT_RH = tt_rh<MW>();
    using C = TtCfg<MW, F7>;
    if (A16) {
        if ((__hip_atomic_load(p.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 30u) == 0u) return;
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&g_tt_reruns, 1ull);
    }
    constexpr int NM = C::NM, XK = C::XK;
    static_assert(C::UNITS <= NT * TT_RH && XK >= 1 && XK <= 8, "tile-table configuration");
    __shared__ __attribute__((aligned(16))) TtSmem<MW, F7> sm;
    auto &tt = sm.u.t.tt;
    auto &tg = sm.u.t.tg;
    auto &img = sm.img;
    auto &aw = sm.aw;

    constexpr int BMT = 64 * TT_RH;  // tile rows
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wvu = __builtin_amdgcn_readfirstlane(wv);
    const int wc = wvu & 3, wr = wvu >> 2;  // the wave's column group and row half
    const int64_t num_mt = (p.M + BMT - 1) / BMT;
    const int64_t tiles = num_mt * ((p.N + BN - 1) / BN);
    const int64_t bid = (int64_t)blockIdx.x % tiles, split = (int64_t)blockIdx.x / tiles;
    const int64_t m0 = (bid % num_mt) * BMT;
    const int64_t n0 = (bid / num_mt) * BN;
    const int kbeg = (int)(split * p.kchunk), kend = (int)min(p.K, (int64_t)kbeg + p.kchunk), K32 = (int)p.K;
    const int bR = *p.bR, bA16 = A16 ? *p.bA : 0;
    // Q_R constants: C = max(2^floor(log2|x|) kc15, cmin); thr = the largest |a b| Q_R flushes
    const float kc15 = 1.5f * p2(23 - MW), cmin = 1.5f * p2(1 - bR + 23 - MW), thr = p2(-bR - MW);

    // static image: V (and sig_a sig_b for F7), [m_b][m_a]
    for (int e = tid; e < NM * NM; e += NT * TT_RH) {
        img[e] = reinterpret_cast<const float *>(p.lutw)[e];
        if (F7) img[TT_IMG_FLOATS / 2 + e] = reinterpret_cast<const float *>(p.lutw)[TT_IMG_FLOATS / 2 + e];
    }

    // build unit (threads < UNITS): K-step bkk, column bcol, rows 16 bpart .. 16 bpart + 15
    const bool bunit = tid < C::UNITS;
    const int bcol = tid & 63, bkk = (tid >> 6) % XK, bpart = min((tid >> 6) / XK, C::PARTS - 1);
    const uint32_t npad4 = (uint32_t)p.npad * 4u;
    const uint32_t boff = (uint32_t)(kbeg + bkk) * npad4 + (uint32_t)(n0 + bcol) * 4u;
    const __amdgpu_buffer_rsrc_t brsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint2 *>(p.bqw), (short)0, -1, 0x00020000);

    // A staging: one word per thread (threads < XK x BMT; conv: lane = row, K-step and row half
    // from the wave; matrix: XK threads per row).  Rows past M re-read row M - 1.
    const bool astage = tid < XK * BMT;
    const int arow = p.conv ? lane + 64 * (wvu / XK) : (tid / XK), akk = p.conv ? wvu % XK : (tid % XK);
    uint32_t aoff;
    const uint32_t phw = (uint32_t)(p.awH * p.awW), uW = (uint32_t)p.awW;
    {
        const int64_t m = min(m0 + arow, p.M - 1);
        if (p.conv) {
            const int64_t hw = p.Ho * p.Wo, img_i = m / hw, pix = m - img_i * hw, ho = pix / p.Wo, wo = pix - ho * p.Wo;
            aoff = (uint32_t)(4 * (img_i * p.aw_c * (int64_t)phw + ho * p.sh * p.awW + wo * p.sw + (p.awpw - p.pw)));
        } else {
            aoff = (uint32_t)(4 * (m * p.awld + akk));
        }
    }
    const __amdgpu_buffer_rsrc_t arsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(p.aw), (short)0, -1, 0x00020000);
    const int khw = p.kh * p.kw;
    uint32_t wa = 0, wb = 0;
    auto load_tile = [&](int k0) {
        if (astage) {
            uint32_t ko;
            if (p.conv) {
                const int k = min(k0 + akk, K32 - 1);  // wave-uniform; clamped: the word image ends at channel K - 1
                const uint32_t c = fastdiv((uint32_t)k, p.kk_mul, p.kk_shift);
                const uint32_t t = (uint32_t)k - c * (uint32_t)khw;
                const uint32_t ky = fastdiv(t, p.kw_mul, p.kw_shift);
                const uint32_t kx = t - ky * (uint32_t)p.kw;
                ko = 4u * (c * phw + ky * (uint32_t)p.dh * uW + kx * (uint32_t)p.dw);
            } else {
                ko = 4u * (uint32_t)k0;
            }
            ko = __builtin_amdgcn_readfirstlane(ko);
            wa = __builtin_amdgcn_raw_buffer_load_b32(arsrc, (int)aoff, (int)ko, 0);  // (past K: zeroed at staging)
        }
        const uint32_t kb = __builtin_amdgcn_readfirstlane((uint32_t)(k0 - kbeg) * npad4);
        if (bunit) wb = __builtin_amdgcn_raw_buffer_load_b32(brsrc, (int)boff, (int)kb, 0);
    };
    load_tile(kbeg);

    float acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0.0f;
    const uint32_t wvo = (uint32_t)wc * 64u;  // the wave's 16 columns, bytes into a table row
    __syncthreads();  // the static image is in LDS

    for (int k0 = kbeg; k0 < kend; k0 += XK) {
        // (K-steps past the group's last channel: zero words, selected here where the loads have
        // landed -- a select at load time made the compiler wait for the prefetch at once)
        if (astage) aw[akk][arow] = (p.conv && k0 + akk >= K32) ? 0u : wa;
        if (bunit) {  // build: tt[bkk][m_a][bcol] = V(m_a, m_b) c_b for the unit's 16 rows
            const float cb = __uint_as_float(wb & TT_EXP);
            const int mb = (int)(wb & (uint32_t)(NM - 1));
            const float4 *vr = reinterpret_cast<const float4 *>(&img[mb * NM + 16 * bpart]);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 v = vr[q];
                tt[bkk][16 * bpart + 4 * q + 0][bcol] = v.x * cb;
                tt[bkk][16 * bpart + 4 * q + 1][bcol] = v.y * cb;
                tt[bkk][16 * bpart + 4 * q + 2][bcol] = v.z * cb;
                tt[bkk][16 * bpart + 4 * q + 3][bcol] = v.w * cb;
            }
            if (F7) {
                const float4 *gr = reinterpret_cast<const float4 *>(&img[TT_IMG_FLOATS / 2 + mb * NM + 16 * bpart]);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 v = gr[q];
                    tg[bkk][16 * bpart + 4 * q + 0][bcol] = v.x * cb;
                    tg[bkk][16 * bpart + 4 * q + 1][bcol] = v.y * cb;
                    tg[bkk][16 * bpart + 4 * q + 2][bcol] = v.z * cb;
                    tg[bkk][16 * bpart + 4 * q + 3][bcol] = v.w * cb;
                }
            }
        }
        __syncthreads();
        if (k0 + XK < kend) load_tile(k0 + XK);  // next tile's loads fly during this tile's math

        // The band test (round 6): per staged tile and wave, when every product
        // |t c_a| of its 64 rows x 16 columns x XK K-steps lies below the result grid's smallest
        // normal 2^(1 - bR) -- e_a + e_b + 1 <= -bR from the largest A exponent (a ballot over the
        // lanes) and the largest c_b exponent of the 16 columns (tt_decode_b) -- Q_R's rounding
        // constant is cmin for all of them and the term is fma(t, c_a, cmin) - cmin: 3 ops instead
        // of 7, the same value (x + cmin rounds x at cmin's ulp, the subnormal quantum, exactly as
        // the general form does in the band).  When every product is also below half the quantum,
        // every term is 0 and the tile adds nothing (+-0 never changes acc: it is never -0).
        // ResNet-50 E2M5: 72 % of the wave-tiles are in the band (tools/census.py; E3M4 0.1 %: the
        // test is compiled for E2M5 only).  Measured: the 3x3 layers 13-21 % faster, the model +6 %
        // (the math loop is about half the kernel: staging, table build and LDS reads are the rest).
        uint32_t wk[XK];
        uint32_t amax = 0;
#pragma unroll
        for (int kk = 0; kk < XK; ++kk) {
            wk[kk] = aw[kk][64 * wr + lane];
            amax = max(amax, (wk[kk] >> 23) & 0xFFu);
        }
        int tmode = 0;  // 0 general, 1 band, 2 zero
        if (!A16 && MW == 5 && p.ebr != nullptr) {  // (E2M5 only: E3M4's tiles are hardly ever in the band;
                                                    // nullptr: option "tt_band" off)
            const int64_t ng = p.npad / 16;
            const int ebm = (int)p.ebr[(int64_t)(k0 / XK) * ng + (n0 >> 4) + wc];  // (wave-uniform)
            const int thb = 253 - bR - ebm, thz = 252 - bR - MW - ebm;
            if (ebm == 0 || __builtin_amdgcn_ballot_w64((int)amax > thz) == 0) tmode = 2;
            else if (__builtin_amdgcn_ballot_w64((int)amax > thb) == 0) tmode = 1;
        }
        if (tmode == 1) {
#pragma unroll
            for (int kk = 0; kk < XK; ++kk) {
                const uint32_t w = wk[kk];
                const float ca = __uint_as_float(w & TT_EXP);
                const char *tb = reinterpret_cast<const char *>(&tt[kk][0][0]) + (w & ~TT_EXP) + wvo;
                float t[16];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 v = *reinterpret_cast<const float4 *>(tb + 16 * q);
                    t[4 * q] = v.x; t[4 * q + 1] = v.y; t[4 * q + 2] = v.z; t[4 * q + 3] = v.w;
                }
                float g[16];
                if (F7) {
                    const char *gb = reinterpret_cast<const char *>(&tg[kk][0][0]) + (w & ~TT_EXP) + wvo;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const float4 v = *reinterpret_cast<const float4 *>(gb + 16 * q);
                        g[4 * q] = v.x; g[4 * q + 1] = v.y; g[4 * q + 2] = v.z; g[4 * q + 3] = v.w;
                    }
                }
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    float r = __fmaf_rn(t[j], ca, cmin) - cmin;
                    if (F7)
                        r = __uint_as_float((__float_as_uint(r) & 0x7FFFFFFFu) |
                                            (__float_as_uint(__fmaf_rn(g[j], ca, thr)) & 0x80000000u));
                    acc[j] += r;
                }
            }
        }
        if (tmode == 0) {
#pragma unroll
        for (int kk = 0; kk < XK; ++kk) {
            const uint32_t w = wk[kk];
            float ca;
            uint32_t off;
            if (A16) {  // c_a = the f16 high half / 2^bA; row offset in 2-byte units of the f16 table
                const uint32_t h = w >> 16, e16 = (h >> 10) & 31u;
                ca = e16 ? __uint_as_float(((h & 0x8000u) << 16) | ((e16 + (uint32_t)(113 - bA16)) << 23)) : 0.0f;
                off = (w & 0x3FFu) * (uint32_t)(4 * TT_RS / TT16_RSH) + wvo;
            } else {
                ca = __uint_as_float(w & TT_EXP);
                off = (w & ~TT_EXP) + wvo;  // m_a row | the wave's columns
            }
            const char *tb = reinterpret_cast<const char *>(&tt[kk][0][0]) + off;
            float t[16];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 v = *reinterpret_cast<const float4 *>(tb + 16 * q);
                t[4 * q] = v.x; t[4 * q + 1] = v.y; t[4 * q + 2] = v.z; t[4 * q + 3] = v.w;
            }
            float g[16];
            if (F7) {
                const char *gb = reinterpret_cast<const char *>(&tg[kk][0][0]) + off;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 v = *reinterpret_cast<const float4 *>(gb + 16 * q);
                    g[4 * q] = v.x; g[4 * q + 1] = v.y; g[4 * q + 2] = v.z; g[4 * q + 3] = v.w;
                }
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const float x = t[j] * ca;  // exact: V c_b c_a, already pre-clamped
                const float pe = __uint_as_float(__float_as_uint(x) & 0x7F800000u);
                const float cc = fmaxf(pe * kc15, cmin);
                float r = (x + cc) - cc;
                if (F7)  // sign of a b + 2^(-bR-M) (its rounding never crosses zero)
                    r = __uint_as_float((__float_as_uint(r) & 0x7FFFFFFFu) |
                                        (__float_as_uint(__fmaf_rn(g[j], ca, thr)) & 0x80000000u));
                acc[j] += r;
            }
        }
        }
        __syncthreads();
    }

    // lane = row, 16 columns -> per row half a [64][BN] slice in LDS -> each thread's 4x4 block
    // (threads < 256, store_tile)
    float *ct = sm.u.ct;
    const int ety = tid & 15, etx = (tid >> 4) & 15;
#pragma unroll
    for (int hs = 0; hs < TT_RH; ++hs) {
        if (hs > 0) __syncthreads();
        if (wr == hs) {
#pragma unroll
            for (int j = 0; j < 16; ++j) ct[lane * XM_CP + 16 * wc + j] = acc[j];
        }
        __syncthreads();
        if (tid < NT) {
            float o[TM][TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) o[i][j] = ct[(ety * TM + i) * XM_CP + etx * TN + j];
            store_tile<false>(p, split, m0 + 64 * hs, n0, ety, etx, o);
        }
    }
}
#endif  // FP8A_OWN_TT

}  // namespace fp8a
