// gemm_fast.h -- the VALU tiled approx GEMM (gemm_fast_kernel), every table mode / flag set that
// has no matrix-core form; compiled only in k_fast.hip.
#pragma once
#include "fp8approx_common.h"

namespace fp8a {

#if FP8A_OWN_FAST
template <bool S2N, bool QBMA, bool GCLIP, int TMODE>
__global__ __launch_bounds__(NT) void gemm_fast_kernel(const GemmArgs p) {
    constexpr bool QAMAA = TMODE == TM_QAMAA;
    constexpr bool V5 = TMODE == TM_V5;
    constexpr bool F8 = TMODE == TM_F8;
    constexpr bool TBL = TMODE != TM_NONE && !QAMAA && !F8;
    constexpr int R = (TMODE == TM_W2S2 || TMODE == TM_W2U2) ? 2 : 1;
    constexpr bool SGN = (TMODE == TM_W2S1 || TMODE == TM_W2S2 || TMODE == TM_LUT);

    __shared__ __attribute__((aligned(16))) float sA[BK][AP];
    __shared__ __attribute__((aligned(16))) float sB[BK][BP];
    __shared__ __attribute__((aligned(16))) float sAc[TBL ? BK : 1][AP];
    __shared__ __attribute__((aligned(16))) uint32_t sAr[(TBL || F8) ? R * BK : 1][AP];
    __shared__ __attribute__((aligned(16))) float sBc[TBL ? BK : 1][BP];
    __shared__ __attribute__((aligned(16))) uint32_t sBm[(TBL || F8) ? BK : 1][BP];
    // F8: the normalised term V'(sign a, m_a, m_b) = min(sig_a sig_b - T[m_a][m_b] 2^-M, top of
    // its binade), 17 rows (2 signs x 8 codes + a zero row) x 2 copies x 8 (see F8_ROW)
    __shared__ __attribute__((aligned(16))) float sF8[F8 ? 17 * 16 : 1];
    __shared__ float sLut[TMODE == TM_LUT ? 1024 : 1];
    __shared__ int32_t sLutI[V5 ? 1024 : 1];
    __shared__ uint32_t sRows[TBL ? 64 * 2 : 1];

    const int tid = threadIdx.x;
    const int ty = tid >> 4, tx = tid & 15;
    const int64_t num_mt = (p.M + BM - 1) / BM;
    const int64_t tiles = num_mt * ((p.N + BN - 1) / BN);
    const int64_t bid = (int64_t)blockIdx.x % tiles, split = (int64_t)blockIdx.x / tiles;
    const int64_t m0 = (bid % num_mt) * BM;   // consecutive blocks: same column tile, so the
    const int64_t n0 = (bid / num_mt) * BN;   // B tile is shared by the 8 XCDs' L2s
    const int64_t kbeg = split * p.kchunk, kend = min(p.K, kbeg + p.kchunk);
    const int M = p.Mw;
    const int bA = QAMAA ? 0 : *p.bA, bR = QAMAA ? 0 : *p.bR;
    const QC qc = make_qc(p.E, M, bR, p.kexp, p.kdc);
    FQ fq;
    if (QAMAA) fq = make_fq(*p.qmax, p.qE, p.qM, p.qsign);
    const uint32_t emnA = (uint32_t)(128 - bA) << 23;
    const float ulpM = p2(-M);

    // F8 Q_R: the result grid of bias bR (floor step 2^(-2-bR), binades from 2^(1-bR)) is the
    // OCP e4m3 grid scaled by 2^(7-bR), so Q_R(y) = 2^(7-bR) * cvt_fp8(y / 2^(7-bR)) (RNE) for y
    // already clamped to Q_R's bound (the clamp scales with y's binade, so it is folded into the
    // LUT value V'), except beyond the e4m3 range (NaN: flagged in the epilogue, the exact kernel
    // reruns the launch)
    const float f8S = F8 ? __uint_as_float((uint32_t)min(max(134 - bR, 1), 254) << 23) : 0.0f;
    if (F8) {
        for (int e = tid; e < 17 * 16; e += NT) {
            const int r = e >> 4, mb = e & 7;  // both 8-entry copies of a row hold the same values
            float v = 0.0f;
            if (r < 16) {
                const int ma = r & 7;
                const float t = (float)p.tab.raw[ma * 8 + mb];
                v = __fmaf_rn(1.0f + 0.125f * ma, 1.0f + 0.125f * mb, -t * 0.125f);  // exact
                // Q_R's pre-clamp bound 2^e (2 - 2^-M - 2^-22) (QC::kb): the mantissa saturates
                // instead of carrying, and on the subnormal grid the top tie rounds down
                v = fminf(v, __uint_as_float(__float_as_uint(v) & 0x7F800000u) * (1.875f - p2(-22)));
                if (r >= 8) v = -v;
            }
            sF8[e] = v;
        }
        __syncthreads();
    }
    if (TBL) {
        const int n = 1 << M;
        for (int i = tid; i < n * 2; i += NT) sRows[i] = p.tab.rows[i >> 1][i & 1];
        if (TMODE == TM_LUT)
            for (int i = tid; i < n * n; i += NT) sLut[i] = (float)p.tab.raw[i];
        if (V5)
            for (int i = tid; i < n * n; i += NT) sLutI[i] = p.tab.raw[i];
        __syncthreads();
    }

    // B staging map: n-contiguous B reads along n, k-contiguous (W[N][K]) along k
    const bool b_ncontig = (p.sbn == 1);
    int bcol[4], bkk[4];
    uint32_t emnB[4];
    int bbv[4];
    // Q_R constants 2^(1-bR), 2^(-bR-M), 1.5 * 2^(1-bR+23-M) stay normal; decode fields fit
    bool bias_ok = bR >= -100 && bR <= 120 && bA >= -100 && bA <= 120;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int e = tid + NT * r;
        bcol[r] = b_ncontig ? (e & 63) : (e >> 4);
        bkk[r] = b_ncontig ? (e >> 6) : (e & 15);
        const int64_t n = n0 + bcol[r];
        const int bb = (!QAMAA && n < p.N) ? p.bB[n * p.bBs] : 0;
        bias_ok = bias_ok && bb >= -100 && bb <= 120;
        // v5: every decoded term 2^(e - bR) (1 + m/2^M) stays a normal float, so the ldexp form
        // below equals the reference's pow(2, e - bR) * (1 + m/2^M)
        if (V5) bias_ok = bias_ok && bA + bb <= 120;
        emnB[r] = (uint32_t)(128 - bb) << 23;
        bbv[r] = V5 ? bb : 0;
    }
    DFmt fA5 = {};
    int32_t v5max = 0;
    if (V5) {
        fA5 = dfmt(p.E, M, bA, false);
        v5max = ((1 << p.E) << M) - 1;
    }

    // implicit-conv row of this thread (fixed across k tiles)
    bool crow_ok = false;
    int64_t cxoff = 0, chi0 = 0, cwi0 = 0;
    if (p.conv) {
        const int64_t m = m0 + (tid & 63);
        crow_ok = m < p.M;
        const int64_t hw = p.Ho * p.Wo;
        const int64_t img = crow_ok ? m / hw : 0, pix = crow_ok ? m - img * hw : 0;
        const int64_t ho = pix / p.Wo, wo = pix - ho * p.Wo;
        cxoff = (img * p.Cin + p.cbase) * p.H * p.W;
        chi0 = ho * p.sh - p.ph;
        cwi0 = wo * p.sw - p.pw;
    }

    float acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = 0.0f;

    // per-thread staging slots (fixed across k tiles)
    int arow[(BM * BK) / NT], akk[(BM * BK) / NT];
#pragma unroll
    for (int r = 0; r < (BM * BK) / NT; ++r) {
        const int e = tid + NT * r;
        arow[r] = p.conv ? (tid & 63) : (e >> 4);       // conv: lanes along m (consecutive pixels)
        akk[r] = p.conv ? ((tid >> 6) + 4 * r) : (e & 15);  // matrix: lanes along k (row-major A)
    }
    float xa[(BM * BK) / NT], xb[(BN * BK) / NT];
    // global -> registers for the tile at k0 (issued one tile ahead of its use)
    auto load_tile = [&](int64_t k0) {
#pragma unroll
        for (int r = 0; r < (BM * BK) / NT; ++r) {
            float x = 0.0f;
            const int64_t k = k0 + akk[r];
            if (!p.conv) {
                const int64_t m = m0 + arow[r];
                if (m < p.M && k < kend) x = p.A[m * p.lda + k];
            } else if (crow_ok && k < kend) {  // implicit im2col
                const uint32_t c = fastdiv((uint32_t)k, p.kk_mul, p.kk_shift);
                const uint32_t t = (uint32_t)k - c * (uint32_t)(p.kh * p.kw);
                const uint32_t ky = fastdiv(t, p.kw_mul, p.kw_shift);
                const uint32_t kx = t - ky * (uint32_t)p.kw;
                const int64_t hi = chi0 + (int64_t)ky * p.dh, wi = cwi0 + (int64_t)kx * p.dw;
                if (hi >= 0 && hi < p.H && wi >= 0 && wi < p.W) x = p.X[cxoff + ((int64_t)c * p.H + hi) * p.W + wi];
            }
            xa[r] = x;
        }
#pragma unroll
        for (int r = 0; r < (BN * BK) / NT; ++r) {
            const int64_t n = n0 + bcol[r], k = k0 + bkk[r];
            xb[r] = (n < p.N && k < kend) ? p.B[k * p.sbk + n * p.sbn] : 0.0f;
        }
    };
    load_tile(kbeg);

    for (int64_t k0 = kbeg; k0 < kend; k0 += BK) {
        bool bad = !bias_ok;
        // ---- decode + stage A (64 x 16)
#pragma unroll
        for (int r = 0; r < (BM * BK) / NT; ++r) {
            const int row = arow[r], kk = akk[r];
            const float x = xa[r];
            float c;
            uint32_t mc;
            if (V5) {  // exact decode with clip_OF (v5:22, 27-38): any fp32 input
                int e, m;
                exact_dec(x, fA5, true, e, m);
                sA[kk][row] = __int_as_float((e << M) + m);
                sAc[kk][row] = __uint_as_float(x < 0.0f ? 0x80000000u : 0u);
                sAr[kk][row] = (uint32_t)m << M;
                continue;
            }
            if (F8) {
                // cvt scale 2^(7-bR) / |c| (applied to x' = V' * c_b inside the conversion) and the
                // byte offset of the LUT row; rows with ty even / odd read copies on disjoint banks
                bad |= !stage_decode(x, M, emnA, true, c, mc);
                const uint32_t cb = __float_as_uint(c);
                const int se = 261 - bR - (int)((cb >> 23) & 0xFFu);
                const bool zero = (cb & 0x7FFFFFFFu) == 0u;
                bad |= !zero && (se < 1 || se > 254);
                sA[kk][row] = zero ? f8S : __uint_as_float((uint32_t)min(max(se, 1), 254) << 23);
                const uint32_t rr = zero ? 16u : ((cb >> 31) * 8u + mc);
                sAr[kk][row] = (rr * 16u + (uint32_t)((row >> 2) & 1) * 8u) * 4u;
                continue;
            }
            if (!QAMAA) bad |= !stage_decode(x, M, emnA, S2N, c, mc);
            sA[kk][row] = x;
            if (TBL) {
                sAc[kk][row] = c * ulpM;  // the 2^-M of mult_result_mant's table term (v9:182)
                if (TMODE == TM_LUT) {
                    sAr[kk][row] = mc << M;
                } else {
                    sAr[kk][row] = sRows[mc * 2];
                    if (R == 2) sAr[BK + kk][row] = sRows[mc * 2 + 1];
                }
            }
        }
        // ---- decode + stage B (16 x 64)
#pragma unroll
        for (int r = 0; r < (BN * BK) / NT; ++r) {
            const int col = bcol[r], kk = bkk[r];
            const float x = xb[r];
            float c;
            uint32_t mc;
            if (V5) {  // B code with the product's exponent offset folded in: -(bA + bB - bR) << M
                int e, m;
                exact_dec(x, dfmt(p.E, M, bbv[r], false), true, e, m);
                sB[kk][col] = __int_as_float(((e - (bA + bbv[r] - bR)) << M) + m);
                sBc[kk][col] = __uint_as_float(x < 0.0f ? 0x80000000u : 0u);
                sBm[kk][col] = (uint32_t)m;
                continue;
            }
            if (F8) {
                bad |= !stage_decode(x, M, emnB[r], true, c, mc);
                sB[kk][col] = c;  // sign(b) 2^floor(log2|b|), 0 for b = 0
                sBm[kk][col] = mc * 4u;
                continue;
            }
            if (!QAMAA) bad |= !stage_decode(x, M, emnB[r], S2N, c, mc);
            sB[kk][col] = x;
            if (TBL) {
                sBc[kk][col] = c;
                sBm[kk][col] = (TMODE == TM_LUT || TMODE == TM_W1U) ? mc : mc * 2u;
            }
        }
        // Off-grid operands / biases outside the exact window: flag the launch; the gated
        // exact kernel that follows on the stream then recomputes the whole product.
        const int anybad = __syncthreads_or(bad ? 1 : 0);
        if (anybad && tid == 0) {
            fb_tile(p, m0, BM, n0);  // (every column tile staging the bad rows marks itself)
            atomicOr(p.flag, fb_bits(p));
        }
        if (k0 + BK < kend) load_tile(k0 + BK);  // next tile's loads fly during this tile's math

        // fp32 accumulation in k order: measured max |error| ~3e-7 x sum|terms| at K = 4608 on
        // realistic data, 30x inside the 1e-5 parity tolerance
        float (&tacc)[TM][TN] = acc;

        // v5 terms of zero operands are not zero (the code sum of a zero is still decoded), so
        // the zero padding of a ragged last K-tile must not be summed there
        const int kk_end = V5 ? (int)min<int64_t>(BK, kend - k0) : BK;
#pragma unroll 2
        for (int kk = 0; kk < kk_end; ++kk) {
            const float4 a4 = *reinterpret_cast<const float4 *>(&sA[kk][ty * TM]);
            const float4 b4 = *reinterpret_cast<const float4 *>(&sB[kk][tx * TN]);
            const float a[TM] = {a4.x, a4.y, a4.z, a4.w};
            const float b[TN] = {b4.x, b4.y, b4.z, b4.w};
            if (QAMAA) {
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) tacc[i][j] += fq_fast(a[i] * b[j], fq);
            } else if (F8) {
                // a = scales, b = c_b; term = Q_R(V' * c_a * c_b) via the scaled fp8 round trip
                const uint4 ia4 = *reinterpret_cast<const uint4 *>(&sAr[kk][ty * TM]);
                const uint4 ib4 = *reinterpret_cast<const uint4 *>(&sBm[kk][tx * TN]);
                const uint32_t ia[TM] = {ia4.x, ia4.y, ia4.z, ia4.w};
                const uint32_t ib[TN] = {ib4.x, ib4.y, ib4.z, ib4.w};
                const char *lut = reinterpret_cast<const char *>(sF8);
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    float xv[TN];
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        xv[j] = *reinterpret_cast<const float *>(lut + (ia[i] + ib[j])) * b[j];
                    typedef short s2 __attribute__((ext_vector_type(2)));
                    s2 code = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32((s2){0, 0}, xv[0], xv[1], a[i], false);
                    code = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(code, xv[2], xv[3], a[i], true);
                    const uint32_t cu = __builtin_bit_cast(uint32_t, code);
                    const auto lo = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(cu, f8S, false);
                    const auto hi = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(cu, f8S, true);
                    tacc[i][0] += lo[0];
                    tacc[i][1] += lo[1];
                    tacc[i][2] += hi[0];
                    tacc[i][3] += hi[1];
                }
            } else if (V5) {
                const float4 ac4 = *reinterpret_cast<const float4 *>(&sAc[kk][ty * TM]);
                const uint4 ar4 = *reinterpret_cast<const uint4 *>(&sAr[kk][ty * TM]);
                const float4 bc4 = *reinterpret_cast<const float4 *>(&sBc[kk][tx * TN]);
                const uint4 bm4 = *reinterpret_cast<const uint4 *>(&sBm[kk][tx * TN]);
                const uint32_t as[TM] = {__float_as_uint(ac4.x), __float_as_uint(ac4.y), __float_as_uint(ac4.z),
                                         __float_as_uint(ac4.w)};
                const uint32_t bs[TN] = {__float_as_uint(bc4.x), __float_as_uint(bc4.y), __float_as_uint(bc4.z),
                                         __float_as_uint(bc4.w)};
                const uint32_t ar[TM] = {ar4.x, ar4.y, ar4.z, ar4.w};
                const uint32_t bm[TN] = {bm4.x, bm4.y, bm4.z, bm4.w};
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) {
                        int32_t r = __float_as_int(a[i]) + __float_as_int(b[j]) + sLutI[ar[i] + bm[j]];
                        r = v5_ofuf(r, v5max, M, p.flags);
                        const int32_t e = r >> M, m = r & ((1 << M) - 1);
                        // expo 0: m * 2^(1-bR-M); else (2^M + m) * 2^(e-bR-M) (also for e < 0)
                        const float v = (e == 0) ? ldexpf((float)m, 1 - bR - M)
                                                 : ldexpf((float)(m + (1 << M)), e - bR - M);
                        tacc[i][j] += __uint_as_float(__float_as_uint(v) ^ as[i] ^ bs[j]);
                    }
            } else if (!TBL) {
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) {
                        const float g = a[i] * b[j];
                        tacc[i][j] += QBMA ? q_fast<GCLIP, true>(g, qc) : g;
                    }
            } else {
                const float4 ac4 = *reinterpret_cast<const float4 *>(&sAc[kk][ty * TM]);
                const uint4 ar4 = *reinterpret_cast<const uint4 *>(&sAr[kk][ty * TM]);
                const uint4 ar4h = (R == 2) ? *reinterpret_cast<const uint4 *>(&sAr[BK + kk][ty * TM]) : make_uint4(0, 0, 0, 0);
                const float4 bc4 = *reinterpret_cast<const float4 *>(&sBc[kk][tx * TN]);
                const uint4 bm4 = *reinterpret_cast<const uint4 *>(&sBm[kk][tx * TN]);
                const float ac[TM] = {ac4.x, ac4.y, ac4.z, ac4.w};
                const uint32_t ar0[TM] = {ar4.x, ar4.y, ar4.z, ar4.w};
                const uint32_t ar1[TM] = {ar4h.x, ar4h.y, ar4h.z, ar4h.w};
                const float bc[TN] = {bc4.x, bc4.y, bc4.z, bc4.w};
                const uint32_t bm[TN] = {bm4.x, bm4.y, bm4.z, bm4.w};
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) {
                        // v0 = a*b - t*cA*cB is exactly representable, so one
                        // fused op yields it; g = a*b is formed only where a mask needs it.
                        const float cab = ac[i] * bc[j];
                        constexpr bool NEED_G = !S2N || (QBMA && SGN);
                        // g = a*b is exact (two (M+1)-bit significands); formed only where a mask
                        // needs it, and then the table term is folded into one fma on it
                        const float g = NEED_G ? a[i] * b[j] : 0.0f;
                        float v0;
                        if (TMODE == TM_W1U) {
                            const int t = __builtin_amdgcn_sbfe((int)ar0[i], bm[j], 1);
                            const float tc = __uint_as_float(__float_as_uint(cab) & (uint32_t)t);
                            v0 = NEED_G ? g - tc : __fmaf_rn(a[i], b[j], -tc);
                        } else {
                            float tf;  // the table entry
                            if (TMODE == TM_LUT) {
                                tf = sLut[ar0[i] + bm[j]];
                            } else {
                                const uint32_t w = (R == 2 && (bm[j] & 32u)) ? ar1[i] : ar0[i];
                                const int t = SGN ? (int)__builtin_amdgcn_sbfe((int)w, bm[j], 2)
                                                  : (int)__builtin_amdgcn_ubfe(w, bm[j], 2);
                                tf = (float)t;
                            }
                            v0 = NEED_G ? __fmaf_rn(-tf, cab, g) : __fmaf_rn(a[i], b[j], -(tf * cab));
                        }
                        if (!S2N) v0 = (fabsf(g) >= qc.mnR) ? v0 : g;  // norm mask, v9:87
                        // F7: the sign comes from Q_R(g), which is -0 (sign +1) for g in [-thr, 0);
                        // v0 has g's sign, so for every g >= -thr the term is |v0|
                        if (S2N && QBMA && SGN) v0 = (g >= -qc.thr) ? fabsf(v0) : v0;
                        tacc[i][j] += QBMA ? q_fast<GCLIP>(v0, qc) : v0;
                    }
            }
        }
        __syncthreads();
    }

    if (F8) {  // a term beyond the e4m3 range came back NaN: the exact kernel reruns the launch
        bool nan = false;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) nan |= __builtin_isnan(acc[i][j]);
        if (__syncthreads_or(nan ? 1 : 0) && tid == 0) {
            fb_tile(p, m0, BM, n0);
            atomicOr(p.flag, fb_bits(p));
        }
    }
    // ---- epilogue
    store_tile(p, split, m0, n0, ty, tx, acc);
}
#endif  // FP8A_OWN_FAST

}  // namespace fp8a
