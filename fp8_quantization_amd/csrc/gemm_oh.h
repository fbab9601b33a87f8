// gemm_oh.h -- the E4M3 approx product as a dense e4m3 x bf8 matrix-core GEMM plus an exact
// correction of the few pairs whose product falls below the result grid's smallest normal
// (included by fp8approx.hip inside namespace fp8a, after gemm_f8mx.h).  DESIGN.md §3d.
//
// Identity.  For on-grid E4M3 operands with s2n and per-product quantization and an E4M3 {0,1}
// (or zero) error table, the reference's term (v9:51-113) is Q_R(V'(m_a, m_b) c_a c_b) with
// c = sign * 2^floor(log2|x|) and V' = sig_a sig_b - T[m_a][m_b] / 8 in [1, 3.75].  Q_R rounds to
// 3 mantissa bits with a saturating mantissa (F6) and, below the result grid's smallest normal
// 2^(1 - bR), to the subnormal step 2^(-2 - bR).  Above that threshold (and at any height: Q_R
// has no upper clip without golden_clip_OF) it is scale-invariant:
//     term = L(m_a, m_b) c_a c_b,   L = e4m3(V') (RNE, saturated in its binade: gemm_f8mx.h)
// -- a rank-8 contraction: A'[m][8k + j] = [m_a(m, k) = j] c_a(m, k) and
// B'[8k + j][n] = L(j, m_b(k, n)) c_b(k, n), i.e. a plain GEMM over K' = 8K whose operands are
// EXACT in fp8: A' is a power of two (bf8: 30 normal binades, shift sA = 6 - bA), B' has four
// significant bits (e4m3 with one MX block scale per column and 4 k -- 32 K' bytes -- chosen
// from the block's largest weight; a weight more than 12 binades below it is "excluded": B' = 0).
// v_mfma_scale_f32_16x16x128_f8f6f4 multiplies those exactly and accumulates in fp32.
//
// Correction.  The pairs with e_a + e_b <= -bR (a superset of the products below 2^(1 - bR):
// V' >= 1) and the pairs with an excluded weight are the only ones whose term is not the dense
// one.  Weights are static and per k the candidate columns of an A element are a PREFIX of the
// columns sorted by e_b: excluded weights first, then the others by e_b, zeros never.  The
// B pre-pass (oh_decode_b) writes per (k, 64-column tile) that order and a count table
// cnt[t - t_min] = #columns with key <= t; oh_correct_kernel looks up each A element's prefix
// length from e_a alone, spreads the (A element, prefix column) entries evenly over the lanes
// of a wave (wave scan), and adds delta = true term - dense term into an LDS tile:
//     true  = Q_R(V' c_a c_b) by the scaled fp8 conversion (subnormal band included, as
//             gemm_f8mx_kernel does), dense = L c_a c_b (0 for an excluded weight).
// delta is exact in fp32 (its bits span at most ~10 binades, or it is -dense); the tile is
// written as one more split-K partial slice, which gemm_oh_kernel's store (unsplit) or the
// split-K reduction adds before the fused epilogue.  With K = 1 each output is dense + delta
// = the reference's term exactly (tests/test_gpu_oh.py); sums differ from an in-order fp32 sum
// only by order (1e-5 sum|term| bar).  About 1-3 % of the nonzero products are candidates on
// the benchmark networks (profiles/unsafe_stats_r02*.json).

// diagnostics switch (fp8a_set_option("oh_stats", 1)): the kernels count into g_ohstat
#ifndef FP8A_OH_STATS
#define FP8A_OH_STATS 1
#endif
#define g_opt_stats_dev (FP8A_OH_STATS && p.ohstats)

constexpr int OH_KC = 32;               // k per staged chunk of gemm_oh_kernel (K' = 256: two MFMA K-steps)
constexpr int OH_BRS = OH_KC * 8 + 16;  // B' LDS row (column n) stride, bytes
constexpr int OH_ARS = OH_KC + 4;       // A code LDS row stride, u16 (72 B: 8-B aligned staging rows; the 4-B
                                        // fragment reads of 16 rows fall on distinct banks)
constexpr int OH_CT = 64;               // columns per candidate-list tile
constexpr int OH_CB = 72;               // count block bytes: cnt[64], t_min + 128, n_excluded, n_all
constexpr uint32_t OH_BZ = 0x78u;       // B code of a zero / excluded weight (exponent field 15)

// Index of output (m, n) in a split-K partial slice (store_tile's partial mapping: ldc = ctot = N,
// coff = 0): the correction slice's layout.
__device__ __forceinline__ int64_t oh_pidx(const GemmArgs &p, int64_t m, int64_t n) {
    if (!p.nchw) return m * p.N + n;
    const int64_t img = m / p.hw, pix = m - img * p.hw;
    return (img * p.N + n) * p.hw + pix;
}

// L(j, m_b) as e4m3 bytes (scale 1) for the 8 A mantissas j: the B' row of a weight with m_b
// before its exponent shift.  V' as gemm_f8mx's table (bf16-exact, pre-clamped), rounded by the
// same conversion.
__device__ __forceinline__ uint2 oh_lrow(const TablePack &tab, int mb) {
    uint32_t w[2] = {0u, 0u};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float t = (float)tab.raw[j * 8 + mb];
        float v = __fmaf_rn(1.0f + 0.125f * j, 1.0f + 0.125f * mb, -t * 0.125f);
        v = fminf(v, __uint_as_float(__float_as_uint(v) & 0x7F800000u) * 1.8671875f);
        xm_s2 cv = {0, 0};
        cv = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(cv, v, v, 1.0f, false);
        w[j >> 2] |= ((uint32_t)__builtin_bit_cast(uint32_t, cv) & 0xFFu) << (8 * (j & 3));
    }
    return make_uint2(w[0], w[1]);
}

// B pre-pass: one 64-thread block per (4-k block kb, 64-column tile); lane = column.  Writes the
// B codes (sign << 7 | (e_b - sB + 6) << 3 | m_b, OH_BZ for zero / excluded weights), the block
// scale (E8M0 of sB = the block's largest e_b - 6), and for each of the 4 k the candidate order
// and count block (see the file comment).  Off-grid weights / biases outside the window mark
// their column for the exact kernel.
__global__ __launch_bounds__(64) void oh_decode_b(const GemmArgs p, int64_t kpad) {
    const int lane = threadIdx.x;
    const int64_t kb = blockIdx.x, ct = blockIdx.y, nct = gridDim.y;
    const int64_t n = ct * OH_CT + lane;
    const int bA = *p.bA, bR = *p.bR;
    const bool biasbad = !(xm_bias_ok(bA) && xm_bias_ok(bR));
    bool bad = biasbad;
    int eb[4], mb[4], sb[4];
    bool nz[4];
    int emax = -100000;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int64_t k = 4 * kb + i;
        nz[i] = false;
        eb[i] = 0;
        mb[i] = 0;
        sb[i] = 0;
        if (k < p.K && n < p.N) {
            const int bb = p.bB[n * p.bBs];
            float c;
            uint32_t mc;
            const bool ok = stage_decode(p.B[k * p.sbk + n * p.sbn], 3, (uint32_t)(128 - bb) << 23, true, c, mc) &&
                            xm_bias_ok(bb);
            if (!ok) fb_col(p, n);
            bad |= !ok;
            const uint32_t cb = __float_as_uint(c);
            if ((cb & 0x7FFFFFFFu) != 0u) {
                nz[i] = true;
                eb[i] = (int)((cb >> 23) & 0xFFu) - 127;
                mb[i] = (int)mc;
                sb[i] = (int)(cb >> 31);
                emax = max(emax, eb[i]);
            }
        }
    }
    // codes and the block scale
    uint8_t *codes = const_cast<uint8_t *>(p.ohb);
    uint8_t *scales = const_cast<uint8_t *>(p.ohs);
    bool excl[4];
    uint32_t cw = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int f = eb[i] - emax + 12;
        excl[i] = nz[i] && f < 0;
        const uint32_t code = (nz[i] && !excl[i]) ? (((uint32_t)sb[i] << 7) | ((uint32_t)f << 3) | (uint32_t)mb[i]) : OH_BZ;
        cw |= code << (8 * i);
    }
    if (n < p.npad) {
        *reinterpret_cast<uint32_t *>(codes + n * kpad + 4 * kb) = cw;
        scales[n * (kpad / 4) + kb] = (uint8_t)(emax > -100000 ? min(max(emax - 6 + 127, 1), 254) : 127);
    }
    // per k: the candidate order of the tile's 64 columns and its count block
    uint32_t *lists = const_cast<uint32_t *>(p.ohl);
    uint8_t *cnts = const_cast<uint8_t *>(p.ohc);
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    bool wide = false;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int64_t k = 4 * kb + i;
        const bool ne = nz[i] && !excl[i];
        const uint64_t mx = __ballot(excl[i]), mn = __ballot(ne), mz = __ballot(!nz[i] && !excl[i]);
        const int nexcl = __popcll(mx), nne = __popcll(mn);
        int tmin = ne ? eb[i] : 100000, tmax = ne ? eb[i] : -100000;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            tmin = min(tmin, __shfl_xor(tmin, o));
            tmax = max(tmax, __shfl_xor(tmax, o));
        }
        if (nne == 0) tmin = tmax = 0;
        wide |= tmax - tmin > 62;
        // rank among the non-excluded: the number with a smaller e_b, then lane order on ties
        int pos, cnt_mine = nexcl, acc = 0;
        pos = excl[i] ? __popcll(mx & below) : (ne ? 0 : nexcl + nne + __popcll(mz & below));
        for (int t = tmin; t <= tmin + 63 && t <= tmax; ++t) {
            const uint64_t mt = __ballot(ne && eb[i] == t);
            if (ne && eb[i] == t) pos = nexcl + acc + __popcll(mt & below);
            acc += __popcll(mt);
            if (lane == t - tmin) cnt_mine = nexcl + acc;
        }
        if (lane > tmax - tmin) cnt_mine = nexcl + nne;  // (levels above the largest e_b)
        if (k < kpad) {
            uint32_t *L = lists + (k * nct + ct) * OH_CT;
            const uint32_t e = (uint32_t)lane | ((uint32_t)(eb[i] + 128) << 8) | ((uint32_t)mb[i] << 16) |
                               ((uint32_t)sb[i] << 19) | (excl[i] ? (1u << 20) : 0u);
            if (nz[i] || excl[i]) L[pos] = e;
            uint8_t *C = cnts + (k * nct + ct) * OH_CB;
            C[lane] = (uint8_t)cnt_mine;
            if (lane == 0) {
                C[64] = (uint8_t)(tmin + 128);
                C[65] = (uint8_t)nexcl;
                C[66] = (uint8_t)(nexcl + nne);
            }
        }
    }
    // a count table wider than 64 exponent levels (weights spanning > 62 binades in one k): the
    // launch falls back (never seen on the grid of one FP8 format)
    if (g_opt_stats_dev) {
        const int nx = __popcll(__ballot(excl[0])) + __popcll(__ballot(excl[1])) + __popcll(__ballot(excl[2])) +
                       __popcll(__ballot(excl[3]));
        if (lane == 0 && nx) atomicAdd(&g_ohstat[1], (unsigned long long)nx);
    }
    if (__any(bad ? 1 : 0) && lane == 0) atomicOr(p.flag, fb_bits(p, biasbad));
    if (__any(wide ? 1 : 0) && lane == 0) atomicOr(p.flag, FB_ANY | FB_ALL);
}

// The dense GEMM.  Workgroup = 4 waves of 64 x 64 outputs: TNW = 1 -> 256 x 64 tiles (waves
// stacked along M: every wave reads the same B'), TNW = 2 -> 128 x 128 (2 x 2).  Per chunk of
// OH_KC = 32 k: the A codes of the tile's rows (u16, gathered from the word image like
// gemm_f8mx_kernel's, next chunk prefetched into registers) and the B' bytes (expanded from the
// B codes: L row of m_b + exponent shift, sign) go to LDS; per MFMA K-step (16 k) a lane builds
// its A' fragment (4 k x 8 bytes: one 64-bit shift per k) for each of its 4 row blocks and
// issues 4 MFMAs (one per column block) with the B' fragments read once per K-step.
template <int TNW>
struct OhSmem {
    static constexpr int TM = 256 / TNW, TN = 64 * TNW;
    union {
        struct {
            uint8_t b[TN][OH_BRS];   // B' [column][k][8 bytes]
            uint16_t a[TM][OH_ARS];  // A codes [row][k]
            uint8_t sc[TN][8];       // B block scales of the chunk [column][k / 4]
            uint2 lut[8];            // L rows
        } s;
        float ct[64 * XM_CP];  // epilogue transpose slice [64][65]
    } u;
};

template <int TNW>
__global__ __launch_bounds__(256, 2) void gemm_oh_kernel(const GemmArgs p) {
    using S = OhSmem<TNW>;
    constexpr int TMR = S::TM, TNC = S::TN;  // tile rows / columns
    __shared__ __attribute__((aligned(16))) S sm;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wr = __builtin_amdgcn_readfirstlane(TNW == 1 ? wv : (wv >> 1));  // the wave's 64-row group
    const int wc = __builtin_amdgcn_readfirstlane(TNW == 1 ? 0 : (wv & 1));    // and 64-column group
    const int64_t num_mt = (p.M + TMR - 1) / TMR;
    const int64_t tiles = num_mt * ((p.N + TNC - 1) / TNC);
    const int64_t bid = (int64_t)blockIdx.x % tiles, split = (int64_t)blockIdx.x / tiles;
    const int64_t m0 = (bid % num_mt) * TMR, n0 = (bid / num_mt) * TNC;
    const int sA = 6 - *p.bA;
    const int kbeg = (int)(split * p.kchunk), kend = (int)min(p.K, (int64_t)kbeg + p.kchunk), K32 = (int)p.K;
    const int64_t kpad = p.awld;  // B codes row length (= Kpad, a multiple of OH_KC)

    if (tid < 8) sm.u.s.lut[tid] = oh_lrow(p.tab, tid);

    // A staging: TNW = 1: thread = row (all 32 k of the chunk); TNW = 2: (row, k half)
    constexpr int AK = OH_KC / TNW;  // codes per thread per chunk
    static_assert(AK * 256 == TMR * OH_KC, "A staging split");
    const int arow = TNW == 1 ? tid : (tid & 127), ak0 = TNW == 1 ? 0 : (tid >> 7) * AK;
    const int64_t am = min(m0 + arow, p.M - 1);
    uint32_t aoff;  // byte offset of the row's element (k = 0) in the u16 code image
    const uint32_t phw = (uint32_t)(p.awH * p.awW), uW = (uint32_t)p.awW;
    if (p.conv) {
        const int64_t hw = p.Ho * p.Wo, img = am / hw, pix = am - img * hw, ho = pix / p.Wo, wo = pix - ho * p.Wo;
        aoff = (uint32_t)(2 * (img * p.aw_c * (int64_t)phw + ho * p.sh * p.awW + wo * p.sw + (p.awpw - p.pw)));
    } else {
        aoff = (uint32_t)(2 * am * p.awld);
    }
    const __amdgpu_buffer_rsrc_t arsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(p.aw), (short)0, -1, 0x00020000);
    const int khw = p.kh * p.kw;
    uint32_t ra[AK / 2];  // the next chunk's codes, two per register
    auto load_a = [&](int k0) {
        if (p.conv) {
#pragma unroll
            for (int e = 0; e < AK; ++e) {
                const int k = min(k0 + ak0 + e, K32 - 1);  // wave-uniform (TNW = 2: per half, still uniform per wave)
                const uint32_t c = fastdiv((uint32_t)k, p.kk_mul, p.kk_shift);
                const uint32_t t = (uint32_t)k - c * (uint32_t)khw;
                const uint32_t ky = fastdiv(t, p.kw_mul, p.kw_shift);
                const uint32_t kx = t - ky * (uint32_t)p.kw;
                const uint32_t ko = __builtin_amdgcn_readfirstlane(2u * (c * phw + ky * (uint32_t)p.dh * uW + kx * (uint32_t)p.dw));
                uint32_t v = __builtin_amdgcn_raw_buffer_load_b16(arsrc, (int)aoff, (int)ko, 0);
                if (k0 + ak0 + e >= K32) v = 0u;  // past the group's last channel
                if (e & 1) ra[e >> 1] |= v << 16;
                else ra[e >> 1] = v;
            }
        } else {  // the matrix code rows are zero-padded to Kpad: 16-B loads
#pragma unroll
            for (int e = 0; e < AK; e += 8) {
                const uint4 v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                             arsrc, (int)aoff, (int)(2u * (uint32_t)(k0 + ak0 + e)), 0));
                ra[e / 2] = v.x; ra[e / 2 + 1] = v.y; ra[e / 2 + 2] = v.z; ra[e / 2 + 3] = v.w;
            }
        }
    };
    // B staging: thread = (column, 32 / (4 / TNW) consecutive k)
    constexpr int BQ = 4 / TNW;  // threads per column
    constexpr int BK = OH_KC / BQ;  // codes per thread: 8 (TNW 1) or 16 (TNW 2)
    const int bcol = tid / BQ, bk0 = (tid % BQ) * BK;
    const int64_t bn = n0 + bcol;  // < npad
    uint32_t rb[BK / 4];
    uint32_t rs0 = 0, rs1 = 0;  // the column's 8 block scales of the chunk (threads with bk0 == 0)
    auto load_b = [&](int k0) {
        const uint8_t *src = p.ohb + bn * kpad + k0 + bk0;
        if constexpr (BK == 8) {
            const uint2 v = *reinterpret_cast<const uint2 *>(src);
            rb[0] = v.x; rb[1] = v.y;
        } else {
            const uint4 v = *reinterpret_cast<const uint4 *>(src);
            rb[0] = v.x; rb[1] = v.y; rb[2] = v.z; rb[3] = v.w;
        }
        if (bk0 == 0) {
            const uint2 v = *reinterpret_cast<const uint2 *>(p.ohs + bn * (kpad / 4) + k0 / 4);
            rs0 = v.x;
            rs1 = v.y;
        }
    };
    load_a(kbeg);
    load_b(kbeg);

    xm_v4f acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (xm_v4f){0.0f, 0.0f, 0.0f, 0.0f};
    const int r16 = lane & 15, g = lane >> 4;
    __syncthreads();  // the L rows

    for (int k0 = kbeg; k0 < kend; k0 += OH_KC) {
        // stage: A codes as they are; B codes expanded to B' rows
        {
            uint32_t *ad = reinterpret_cast<uint32_t *>(&sm.u.s.a[arow][ak0]);
#pragma unroll
            for (int e = 0; e < AK / 2; e += 2) *reinterpret_cast<uint2 *>(ad + e) = make_uint2(ra[e], ra[e + 1]);
            uint8_t *bd = &sm.u.s.b[bcol][bk0 * 8];
#pragma unroll
            for (int q = 0; q < BK / 4; ++q) {
                uint32_t o[8];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint32_t c = (rb[q] >> (8 * e)) & 0xFFu;
                    const uint2 l = sm.u.s.lut[c & 7u];
                    const uint32_t f = (c >> 3) & 15u;
                    const uint32_t add = (f - 6u) * 0x08080808u;  // exponent shift f - 6 in every byte (no carries: fields stay in [1, 14])
                    const uint32_t sg = (c & 0x80u) ? 0x80808080u : 0u;
                    o[2 * e] = f == 15u ? 0u : ((l.x + add) ^ sg);
                    o[2 * e + 1] = f == 15u ? 0u : ((l.y + add) ^ sg);
                }
                *reinterpret_cast<uint4 *>(bd + 32 * q) = make_uint4(o[0], o[1], o[2], o[3]);
                *reinterpret_cast<uint4 *>(bd + 32 * q + 16) = make_uint4(o[4], o[5], o[6], o[7]);
            }
            if (bk0 == 0) *reinterpret_cast<uint2 *>(&sm.u.s.sc[bcol][0]) = make_uint2(rs0, rs1);
        }
        __syncthreads();
        if (k0 + OH_KC < kend) {  // next chunk's loads fly during this chunk's MFMAs
            load_a(k0 + OH_KC);
            load_b(k0 + OH_KC);
        }
#pragma unroll
        for (int ks = 0; ks < OH_KC / 16; ++ks) {
            xm_v8i bf[4];
            int bsc[4];
            // operand K layout of v_mfma_scale_f32_16x16x128_f8f6f4 (measured, tools/mfma_scale_layout.hip):
            // bytes 0-15 of lane group g are K 16 g .. 16 g + 15 and bytes 16-31 are K 64 + 16 g ..; the
            // MX block b (K 32 b .. 32 b + 31) takes its scale from lane group b.  So lane group g holds
            // k = 2 g, 2 g + 1 (low half) and 8 + 2 g, 8 + 2 g + 1 (high half) of the 16-k step: the
            // 4-k scale block b = {4 b .. 4 b + 3} is exactly MX block b, scaled by lane group b.
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int col = 64 * wc + 16 * j + r16;
                const uint8_t *pb = &sm.u.s.b[col][128 * ks + 16 * g];
                const uint4 b0 = *reinterpret_cast<const uint4 *>(pb), b1 = *reinterpret_cast<const uint4 *>(pb + 64);
                bf[j] = (xm_v8i){(int)b0.x, (int)b0.y, (int)b0.z, (int)b0.w, (int)b1.x, (int)b1.y, (int)b1.z, (int)b1.w};
                bsc[j] = sm.u.s.sc[col][4 * ks + g];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint16_t *ar = &sm.u.s.a[64 * wr + 16 * i + r16][16 * ks + 2 * g];
                const uint32_t w0 = *reinterpret_cast<const uint32_t *>(ar), w1 = *reinterpret_cast<const uint32_t *>(ar + 8);
                const uint32_t cs[4] = {w0 & 0xFFFFu, w0 >> 16, w1 & 0xFFFFu, w1 >> 16};
                xm_v8i af;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint64_t x = (uint64_t)(cs[e] & 0xFFu) << (cs[e] >> 8);
                    af[2 * e] = (int)(uint32_t)x;
                    af[2 * e + 1] = (int)(uint32_t)(x >> 32);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j)  // A bf8 (cbsz 1), B e4m3 (blgp 0), B scaled per (column, 4 k)
                    acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, bf[j], acc[i][j], 1, 0, 0, 127, 0,
                                                                                bsc[j]);
            }
        }
        __syncthreads();
    }

    // epilogue: D (units of 2^-sA) of wave (wr, wc) -> one 64 x 64 slice at a time through LDS ->
    // each thread's 4 x 4 block, + the correction slice (unsplit), store_tile's mapping
    const float sAf = __uint_as_float((uint32_t)(127 + sA) << 23);
    float *ct = sm.u.ct;
    const int ety = tid & 15, etx = (tid >> 4) & 15;
    const bool partial = p.splits > 1;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        if (h > 0) __syncthreads();
        if (wv == h) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        ct[(16 * i + 4 * g + r) * XM_CP + 16 * j + r16] = acc[i][j][r] * sAf;
        }
        __syncthreads();
        const int hr = TNW == 1 ? h : (h >> 1), hc = TNW == 1 ? 0 : (h & 1);
        const int64_t sm0 = m0 + 64 * hr, sn0 = n0 + 64 * hc;
        float a4[TM][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) a4[i][j] = ct[(ety * TM + i) * XM_CP + etx * TN + j];
        if (!partial && p.ohd) {  // the correction slice (same layout as a split-K partial)
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int64_t m = sm0 + ety * TM + i;
                if (m >= p.M) continue;
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int64_t nn = sn0 + etx * TN + j;
                    if (nn < p.N) a4[i][j] += p.ohd[oh_pidx(p, m, nn)];
                }
            }
        }
        store_tile(p, split, sm0, sn0, ety, etx, a4);
    }
}

// The correction.  Workgroup = 4 waves over a 128-row x 64-column output tile (wave = 32 rows), an
// LDS accumulator per tile; per chunk of OC_KC k: the tile's A codes, the k's candidate lists and
// count blocks in LDS; per wave the 32 x OC_KC (row, k) prefix lengths, a wave scan, then every
// lane walks an equal share of the entries, adding delta = true - dense into acc[row][column]
// (LDS float atomics; a wave owns its 32 rows, so no two waves touch one address).
constexpr int OC_KC = 32;
constexpr int OC_AP = 130;  // acc row stride (floats)
struct OcSmem {
    float acc[128][OC_AP / 2];      // [row][column] (65 floats per row)
    uint16_t a[128][OC_KC + 2];     // A codes [row][k]
    uint32_t lst[OC_KC][OH_CT];     // candidate lists of the chunk's k
    uint8_t cnt[OC_KC][OH_CB];      // count blocks
    uint32_t seg[4][32 * OC_KC];    // per wave: prefix length << 16 | A code of its (row, k) segments
    uint32_t lsum[4][64];           // per wave: exclusive scan of the lanes' entry counts
    float vt[2][8][8];              // V' (pre-clamped, bf16-exact) and L per (m_a, m_b)
};

__global__ __launch_bounds__(256, 2) void oh_correct_kernel(const GemmArgs p) {
    __shared__ __attribute__((aligned(16))) OcSmem sm;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int64_t nct = p.npad / OH_CT, nmt = (p.M + 127) / 128;  // (the lists' tile count: npad / 64)
    const int64_t mt = blockIdx.x % nmt, ct = blockIdx.x / nmt;
    const int64_t m0 = mt * 128, n0 = ct * OH_CT;
    const int bR = *p.bR, sA = 6 - *p.bA;
    const int64_t kpad = p.awld;
    const int K32 = (int)p.K;
    for (int e = tid; e < 128 * (OC_AP / 2); e += 256) (&sm.acc[0][0])[e] = 0.0f;
    if (tid < 64) {
        const int ma = tid >> 3, mbb = tid & 7;
        const float t = (float)p.tab.raw[ma * 8 + mbb];
        float v = __fmaf_rn(1.0f + 0.125f * ma, 1.0f + 0.125f * mbb, -t * 0.125f);
        v = fminf(v, __uint_as_float(__float_as_uint(v) & 0x7F800000u) * 1.8671875f);
        xm_s2 cv = {0, 0};
        cv = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(cv, v, v, 1.0f, false);
        sm.vt[0][ma][mbb] = v;
        sm.vt[1][ma][mbb] = __builtin_amdgcn_cvt_scalef32_f32_fp8(__builtin_bit_cast(int, cv), 1.0f, 0);  // L
    }
    // A staging (thread = (row, k half)), conv gather as gemm_oh_kernel
    const int arow = tid & 127, ak0 = (tid >> 7) * (OC_KC / 2);
    const int64_t am = min(m0 + arow, p.M - 1);
    uint32_t aoff;
    const uint32_t phw = (uint32_t)(p.awH * p.awW), uW = (uint32_t)p.awW;
    if (p.conv) {
        const int64_t hw = p.Ho * p.Wo, img = am / hw, pix = am - img * hw, ho = pix / p.Wo, wo = pix - ho * p.Wo;
        aoff = (uint32_t)(2 * (img * p.aw_c * (int64_t)phw + ho * p.sh * p.awW + wo * p.sw + (p.awpw - p.pw)));
    } else {
        aoff = (uint32_t)(2 * am * p.awld);
    }
    const __amdgpu_buffer_rsrc_t arsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(p.aw), (short)0, -1, 0x00020000);
    const int khw = p.kh * p.kw;
    const float f8S = __uint_as_float((uint32_t)min(max(134 - bR, 1), 254) << 23);  // 2^(7 - bR)

    for (int k0 = 0; k0 < K32; k0 += OC_KC) {
        __syncthreads();  // (previous chunk's LDS consumers done)
        for (int e = 0; e < OC_KC / 2; ++e) {
            const int k = k0 + ak0 + e;
            uint32_t v = 0u;
            if (k < K32) {
                uint32_t ko;
                if (p.conv) {
                    const uint32_t c = fastdiv((uint32_t)k, p.kk_mul, p.kk_shift);
                    const uint32_t t = (uint32_t)k - c * (uint32_t)khw;
                    const uint32_t ky = fastdiv(t, p.kw_mul, p.kw_shift);
                    const uint32_t kx = t - ky * (uint32_t)p.kw;
                    ko = 2u * (c * phw + ky * (uint32_t)p.dh * uW + kx * (uint32_t)p.dw);
                } else {
                    ko = 2u * (uint32_t)k;
                }
                v = __builtin_amdgcn_raw_buffer_load_b16(arsrc, (int)aoff, (int)__builtin_amdgcn_readfirstlane(ko), 0);
            }
            sm.a[arow][ak0 + e] = (uint16_t)v;
        }
        for (int e = tid; e < OC_KC * OH_CT; e += 256) {
            const int kk = e / OH_CT, i = e - kk * OH_CT;
            sm.lst[kk][i] = (k0 + kk < kpad) ? p.ohl[((int64_t)(k0 + kk) * nct + ct) * OH_CT + i] : 0u;
        }
        for (int e = tid; e < OC_KC * OH_CB / 4; e += 256) {
            const int kk = e / (OH_CB / 4), i = e - kk * (OH_CB / 4);
            reinterpret_cast<uint32_t *>(&sm.cnt[kk][0])[i] =
                (k0 + kk < kpad) ? reinterpret_cast<const uint32_t *>(p.ohc + ((int64_t)(k0 + kk) * nct + ct) * OH_CB)[i] : 0u;
        }
        __syncthreads();
        // segments of this wave: (row 32 wv + (lane & 31), k (lane >> 5) * 16 + s), s < 16
        const int srow = 32 * wv + (lane & 31), sk0 = (lane >> 5) * (OC_KC / 2);
        uint32_t tot = 0;
        uint32_t *seg = sm.seg[wv];
        for (int s = 0; s < OC_KC / 2; ++s) {
            const int kk = sk0 + s;
            const uint32_t code = sm.a[srow][kk];
            uint32_t P = 0;
            if (code != 0u && k0 + kk < K32 && m0 + srow < p.M) {
                const int ea = (int)((code >> 2) & 31u) - 15 + sA;
                const int t = -bR - ea;  // candidates: e_b <= t
                const uint8_t *C = sm.cnt[kk];
                const int tmin = (int)C[64] - 128;
                P = t < tmin ? C[65] : (t - tmin >= 64 ? C[66] : C[t - tmin]);
            }
            seg[(lane & 31) * OC_KC + kk] = (P << 16) | code;
            tot += P;
        }
        // exclusive scan of the lanes' totals, in segment order lane-major: (lane & 31, k half)
        // -> the order is row-major over the wave's 32 x 32 (row, k) grid
        // exclusive scan of the lanes' totals in position order: position pos = 2 r + h (row r, k
        // half h) is held by lane 32 h + r, so the positions run row-major over the (row, k) grid
        const uint32_t v = __shfl(tot, ((lane & 1) << 5) | (lane >> 1));  // the total of position `lane`
        uint32_t incl = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = __shfl_up(incl, o);
            if (lane >= o) incl += u;
        }
        sm.lsum[wv][lane] = incl - v;  // exclusive prefix of position `lane`
        const uint32_t T = __shfl(incl, 63);
        if (g_opt_stats_dev) {
            uint32_t nzs = 0;
            for (int s2 = 0; s2 < OC_KC / 2; ++s2) nzs += (seg[(lane & 31) * OC_KC + sk0 + s2] >> 16) != 0u;
            for (int o = 32; o >= 1; o >>= 1) nzs += __shfl_xor(nzs, o);
            if (lane == 0) {
                atomicAdd(&g_ohstat[0], (unsigned long long)T);
                atomicAdd(&g_ohstat[2], (unsigned long long)nzs);
                atomicAdd(&g_ohstat[3], (unsigned long long)(32 * OC_KC));
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (T == 0u) continue;
        // this lane's entries [e0, e1)
        const uint32_t q = (T + 63u) / 64u, e0 = min(T, q * (uint32_t)lane), e1 = min(T, e0 + q);
        if (e0 >= e1) continue;
        // position of e0: largest pos with lsum[pos] <= e0
        int pos = 0;
#pragma unroll
        for (int b = 32; b >= 1; b >>= 1)
            if (pos + b < 64 && sm.lsum[wv][pos + b] <= e0) pos += b;
        // position -> (row r = pos >> 1, k half h = pos & 1); walk its 16 segments
        int r = pos >> 1, kk = (pos & 1) * (OC_KC / 2);
        uint32_t off = e0 - sm.lsum[wv][pos];  // entries to skip from the segment block's start
        uint32_t sv = seg[r * OC_KC + kk];
        while ((sv >> 16) <= off) {
            off -= sv >> 16;
            ++kk;
            if (kk == OC_KC) { kk = 0; ++r; }
            sv = seg[r * OC_KC + kk];
        }
        for (uint32_t e = e0; e < e1; ++e) {
            while ((sv >> 16) <= off) {  // next nonempty segment
                off = 0;
                ++kk;
                if (kk == OC_KC) { kk = 0; ++r; }
                sv = seg[r * OC_KC + kk];
            }
            const uint32_t code = sv & 0xFFFFu;
            const uint32_t en = sm.lst[kk][off];
            ++off;
            const int col = (int)(en & 63u);
            const int ebb = (int)((en >> 8) & 0xFFu) - 128, mbb = (int)((en >> 16) & 7u);
            const bool excl = (en >> 20) & 1u;
            const uint32_t ma = code >> 11, sa = (code >> 7) & 1u, sgn = (sa ^ ((en >> 19) & 1u)) << 31;
            const int ea = (int)((code >> 2) & 31u) - 15 + sA;
            // true term: Q_R(V' c_a c_b) = 2^(7 - bR) e4m3(V' |c_b| / 2^(7 - bR - e_a)), signed
            const float vb = sm.vt[0][ma][mbb] * __uint_as_float((uint32_t)(ebb + 127) << 23);
            const float scl = __uint_as_float((uint32_t)min(max(134 - bR - ea, 1), 254) << 23);
            xm_s2 cv = {0, 0};
            cv = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(cv, vb, vb, scl, false);
            const float tru = __builtin_amdgcn_cvt_scalef32_f32_fp8(__builtin_bit_cast(int, cv), f8S, 0);
            const float den = excl ? 0.0f : sm.vt[1][ma][mbb] * __uint_as_float((uint32_t)(ea + ebb + 127) << 23);
            const float d = __uint_as_float(__float_as_uint(tru - den) ^ sgn);
            if (d != 0.0f) atomicAdd(&sm.acc[r + 32 * wv][col], d);
        }
    }
    __syncthreads();
    // the tile -> the correction slice (partial layout), NaN (a term beyond the e4m3 range) marks the tile
    bool nan = false;
    for (int e = tid; e < 128 * OH_CT; e += 256) {
        // NCHW partial layout: consecutive threads on consecutive pixels (rows); row-major: columns
        const int r = p.nchw ? (e & 127) : e / OH_CT, c = p.nchw ? (e >> 7) : e - (e / OH_CT) * OH_CT;
        const int64_t m = m0 + r, n = n0 + c;
        if (m >= p.M || n >= p.N) continue;
        const float v = sm.acc[r][c];
        nan |= __builtin_isnan(v);
        p.ohd[oh_pidx(p, m, n)] = v;
    }
    if (__syncthreads_or(nan ? 1 : 0) && tid == 0) {
        fb_tile(p, m0, 128, n0);
        atomicOr(p.flag, fb_bits(p));
    }
}
