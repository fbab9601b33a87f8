// gemm_f8mx.h -- the E4M3 fast path with matrix-core accumulation (included by fp8approx.hip,
// inside namespace fp8a, after GemmArgs / stage_decode / store_tile).  DESIGN.md §3a.
//
// Same arithmetic as gemm_fast_kernel<.., TM_F8>: for on-grid E4M3 operands with
// s2n and per-product quantization (v9:51-113), each term is
//     Q_R(V'(s_a, m_a, m_b) * c_b * |c_a|)  =  2^(7-bR) * e4m3(V' * c_b / scale_a),
// scale_a = 2^(7-bR) / |c_a|, where V' = min(sig_a sig_b - T[m_a][m_b] 2^-M, pre-clamp bound of
// its binade) is an LDS table value and e4m3() is gfx950's scaled fp8 conversion (RNE; the bR
// grid is the OCP e4m3 grid scaled by 2^(7-bR), subnormal band included).
//
// Summation on the matrix core: the fp8 codes are not decoded and added on the VALU; one
// v_mfma_scale_f32_32x32x64_f8f6f4 per two K-steps multiplies the wave's 2048 codes by a
// constant 0/1 selection operand S, so that
//     D[m][n] += the two K-steps' codes of output (n mod 16) of lane m + 32 (n / 16).
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
// form of the scaled conversion.  Per product pair the VALU issues one LDS address add, one
// packed add and one conversion; the table read is one ds_read_b32.  (A/B on the ResNet-18
// layer set: +15 % over the f32 form, which paid two multiplies per pair and a ds_read_b64.)
//
// Operands are decoded ONCE per launch by two pre-pass kernels (xm_decode_a / xm_decode_b):
// an A element becomes one 32-bit word (cvt scale exponent << 23 | table row offset; the
// conversion reads only the scale's exponent field), a B column pair one (addend pair, pair
// block offset) uint2.  The GEMM's staging is then a gather and stores (a 3x3 conv gathers
// each input element 9 times).  The pre-passes also carry the fallback checks (off-grid
// operand, exactness window, e4m3 scale range, bias window) into the launch's flag word.
//
// LDS table layout [pair (code0 + 9 code1)][copy][row (8 s_a + m_a)] u32: zero A operands take
// scale 2^127 (the conversion returns 0), so they need no row; copy = parity of the consuming
// thread's column group.  Threads are mapped so that each 32-lane half-wave holds 16 row groups
// x 2 column groups: a read touches at most 16 rows of one copy per column group, each on its
// own bank -- conflict-free (MI355X_MICROARCH.md §LDS: ds_read_b32 banks (a/4) mod 32).

typedef int xm_v8i __attribute__((ext_vector_type(8)));
typedef float xm_v16f __attribute__((ext_vector_type(16)));
typedef short xm_s2 __attribute__((ext_vector_type(2)));
typedef unsigned short xm_u2 __attribute__((ext_vector_type(2)));
typedef __bf16 xm_b2 __attribute__((ext_vector_type(2)));

constexpr int XM_NPAIR = 81;
constexpr int XM_LUT_WORDS = XM_NPAIR * 2 * 16;  // [pair][copy][row] u32, 10.1 KiB
constexpr uint32_t XM_ROW_SHIFT = 2, XM_ROW_MASK = 0x3Cu;
constexpr int XM_BQ = BN / 2 + 2;              // pair slots per staged K row (padded)
constexpr uint32_t XM_ZERO_WORD = 254u << 23;  // A = 0: cvt scale 2^127 (the code is 0), row 0
struct XmSmem {
    uint32_t lut[XM_LUT_WORDS];
    uint32_t aw[BK][AP];     // A(m, k)'s word: cvt scale exponent << 23 | table row offset

    uint2 bq[BK][XM_BQ];     // per column pair: (c_b addend pair, byte offset of the pair block)
};
constexpr int XM_CP = BN + 1;  // epilogue transpose tile [BM][BN + 1] floats, aliased on XmSmem
static_assert(sizeof(float) * BM * XM_CP <= sizeof(XmSmem), "epilogue tile must fit the staging LDS");

// Exactness / range window shared by the pre-passes (as bias_ok in gemm_fast_kernel)
__device__ __forceinline__ bool xm_bias_ok(int b) { return b >= -100 && b <= 120; }

// Table word e of layout [pair][copy][row]: the bf16 pair V'(row, code0), V'(row, code1).
__device__ __forceinline__ uint32_t xm_lut_word(const TablePack &tab, int e) {
    const int pr = e >> 5, row = e & 15;
    const int ma = row & 7;
    uint32_t w = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int cd = h ? (pr / 9) : (pr % 9);
        if (cd == 8) continue;  // zero B: +0
        const float t = (float)tab.raw[ma * 8 + cd];
        float v = __fmaf_rn(1.0f + 0.125f * ma, 1.0f + 0.125f * cd, -t * 0.125f);  // exact, <= 8 bits
        // Q_R's pre-clamp in bf16: any bound in (1.8125, 1.875) x binade rounds like the
        // reference's saturating mantissa (and the subnormal top tie rounding down)
        v = fminf(v, __uint_as_float(__float_as_uint(v) & 0x7F800000u) * 1.8671875f);
        if (row >= 8) v = -v;
        w |= (__float_as_uint(v) >> 16) << (16 * h);
    }
    return w;
}

// A element -> word: bits 23-30 the cvt scale exponent se (scale 2^(se-127) = 2^(7-bR-e_a)),
// bits 3-6 the table row (8 s_a + m_a); zeros XM_ZERO_WORD.  ok = on the (3, bA) grid, inside the
// exactness window and the scale range.
__device__ __forceinline__ uint32_t xm_word_a(float x, uint32_t emnA, int bR, bool &ok) {
    float c;
    uint32_t mc;
    ok = stage_decode(x, 3, emnA, true, c, mc);
    const uint32_t cb = __float_as_uint(c);
    const int se = 261 - bR - (int)((cb >> 23) & 0xFFu);
    if ((cb & 0x7FFFFFFFu) == 0u) return XM_ZERO_WORD;
    ok = ok && se >= 1 && se <= 254;
    return ((uint32_t)min(max(se, 1), 254) << 23) | (((cb >> 31) * 8u + mc) << XM_ROW_SHIFT);
}

// A pre-pass, one (image | row) per blockIdx.y step.  conv: the group's channel slice of x
// [Bn][Cin][H][W] (channels cbase..cbase+aw_c) -> words [Bn][aw_c][H][W]; matrix: A [M][lda] ->
// words [M][awld] (columns >= K zero words).
__global__ __launch_bounds__(256) void xm_decode_a(const GemmArgs p) {
    // fused input quantization: A = fq(X) with the quantizer's own bias, which becomes bA
    const float fmx = p.fqin.mx ? *p.fqin.mx : 0.0f;
    const float fbias = p.fqin.mx ? fq_bias(fmx, p.fqin.E, p.fqin.M) : 0.0f;
    const int bA = p.fqin.mx ? (int)fbias : *p.bA, bR = *p.bR;
    if (p.fqin.mx && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
        *p.fq_bias = fbias;
        *p.fq_ibias = bA;
    }
    const uint32_t emnA = (uint32_t)(128 - bA) << 23;
    bool bad = !(xm_bias_ok(bA) && xm_bias_ok(bR));
    uint32_t *const out = const_cast<uint32_t *>(p.aw);
    const int64_t hw = p.H * p.W;
    const int64_t rows = p.conv ? p.M / (p.Ho * p.Wo) : p.M, cols = p.conv ? p.aw_c * hw : p.awld;
    for (int64_t r = blockIdx.y; r < rows; r += gridDim.y) {
        const float *in = p.conv ? p.X + (r * p.Cin + p.cbase) * hw : p.A + r * p.lda;
        const int64_t lim = p.conv ? cols : p.K;
        uint32_t *o = out + r * cols;
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cols; i += (int64_t)gridDim.x * blockDim.x) {
            bool ok = true;
            float v = (i < lim) ? in[i] : 0.0f;
            if (p.fqin.mx) v = fq_apply(v, fmx, fbias, p.fqin.M, p.fqin.S);
            o[i] = (i < lim) ? xm_word_a(v, emnA, bR, ok) : XM_ZERO_WORD;
            bad |= !ok;
        }
    }
    if (__syncthreads_or(bad ? 1 : 0) && threadIdx.x == 0) atomicOr(p.flag, 1u);
}

// B pre-pass: per (k, pair Q) of the padded [Kpad][npad / 2] pair grid, the addend pair
// ((s_b << 15) + (e_b << 7) per bf16 half, 0 for a zero B) and the pair block's byte offset
// ((code0 + 9 code1) * 128 + copy * 64, copy = parity of the consuming thread's 4-column group
// = (Q >> 1) & 1); out-of-range elements are zeros.
__global__ __launch_bounds__(256) void xm_decode_b(const GemmArgs p, int64_t kpad) {
    const int bA = *p.bA, bR = *p.bR;
    bool bad = !(xm_bias_ok(bA) && xm_bias_ok(bR));
    const int64_t hq = p.npad / 2, n = kpad * hq;
    uint2 *const bq = const_cast<uint2 *>(p.bqw);
    if (blockIdx.x == 0)  // the table image every GEMM workgroup copies into LDS
        for (int e = threadIdx.x; e < XM_LUT_WORDS; e += blockDim.x) const_cast<uint32_t *>(p.lutw)[e] = xm_lut_word(p.tab, e);
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
                const bool ok = stage_decode(p.B[k * p.sbk + col * p.sbn], 3, (uint32_t)(128 - bb) << 23, true,
                                             c[h], mc[h]);
                bad |= !ok || !xm_bias_ok(bb);
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
        bq[i] = make_uint2(add, ((code[0] + 9u * code[1]) * 2u + (uint32_t)((q >> 1) & 1)) * 64u);
    }
    if (__syncthreads_or(bad ? 1 : 0) && threadIdx.x == 0) atomicOr(p.flag, 1u);
}

#ifndef XM_WAVES
#define XM_WAVES 1
#endif
__global__ __launch_bounds__(NT, XM_WAVES) void gemm_f8mx_kernel(const GemmArgs p) {
    __shared__ __attribute__((aligned(16))) XmSmem sm;

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wvu = __builtin_amdgcn_readfirstlane(wv);
    const int ty = lane & 15, tx = 4 * wv + (lane >> 4);  // half-wave = 16 row groups x 2 column groups
    const int64_t num_mt = (p.M + BM - 1) / BM;
    const int64_t tiles = num_mt * ((p.N + BN - 1) / BN);
    const int64_t bid = (int64_t)blockIdx.x % tiles, split = (int64_t)blockIdx.x / tiles;
    const int64_t m0 = (bid % num_mt) * BM;
    const int64_t n0 = (bid / num_mt) * BN;
    const int64_t kbeg = split * p.kchunk, kend = min(p.K, kbeg + p.kchunk);
    const int bR = *p.bR;

    // table: copied from the launch's pre-computed image (xm_decode_b), 16-B per thread and step
    for (int e = 4 * tid; e < XM_LUT_WORDS; e += 4 * NT)
        *reinterpret_cast<uint4 *>(&sm.lut[e]) = *reinterpret_cast<const uint4 *>(&p.lutw[e]);

    // B staging slots: pair q = e & 31 (lanes along n: coalesced), k row kk = e >> 5
    const int64_t hq = p.npad / 2;
    int bq[2], bkk[2];
    int64_t boff[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int e = tid + NT * r;
        bq[r] = e & 31;
        bkk[r] = e >> 5;
        boff[r] = (kbeg + bkk[r]) * hq + n0 / 2 + bq[r];  // pair index
    }

    // A staging.  conv: lanes along m (consecutive pixels), k row = wave + 4 r (wave-uniform: the
    // k -> (c, ky, kx) split runs on the scalar unit); matrix: lanes along k.
    bool crow_ok = false;
    int64_t cbase_w = 0;
    int chi0 = 0, cwi0 = 0;
    if (p.conv) {
        const int64_t m = m0 + lane;
        crow_ok = m < p.M;
        const int64_t hw = p.Ho * p.Wo;
        const int64_t img = crow_ok ? m / hw : 0, pix = crow_ok ? m - img * hw : 0;
        const int64_t ho = pix / p.Wo, wo = pix - ho * p.Wo;
        chi0 = (int)(ho * p.sh - p.ph);
        cwi0 = (int)(wo * p.sw - p.pw);
        cbase_w = img * p.aw_c * p.H * p.W + (int64_t)chi0 * p.W + cwi0;
    }
    int arow[(BM * BK) / NT], akk[(BM * BK) / NT];
#pragma unroll
    for (int r = 0; r < (BM * BK) / NT; ++r) {
        const int e = tid + NT * r;
        arow[r] = p.conv ? lane : (e >> 4);
        akk[r] = p.conv ? (wvu + 4 * r) : (e & 15);
    }
    uint32_t wa[(BM * BK) / NT];
    uint2 wbq[2];
    auto load_tile = [&](int64_t k0) {
#pragma unroll
        for (int r = 0; r < (BM * BK) / NT; ++r) {
            uint32_t w = XM_ZERO_WORD;
            if (!p.conv) {
                const int64_t m = m0 + arow[r];
                if (m < p.M) w = p.aw[m * p.awld + k0 + akk[r]];
            } else {
                const int64_t k = k0 + akk[r];  // wave-uniform
                if (k < kend) {
                    const uint32_t c = fastdiv((uint32_t)k, p.kk_mul, p.kk_shift);
                    const uint32_t t = (uint32_t)k - c * (uint32_t)(p.kh * p.kw);
                    const uint32_t ky = fastdiv(t, p.kw_mul, p.kw_shift);
                    const uint32_t kx = t - ky * (uint32_t)p.kw;
                    const int dy = (int)ky * p.dh, dx = (int)kx * p.dw;
                    const int64_t koff = (int64_t)c * p.H * p.W + (int64_t)dy * p.W + dx;
                    if (crow_ok && (uint32_t)(chi0 + dy) < (uint32_t)p.H && (uint32_t)(cwi0 + dx) < (uint32_t)p.W)
                        w = p.aw[cbase_w + koff];
                }
            }
            wa[r] = w;
        }
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int64_t o = boff[r] + (k0 - kbeg) * hq;
            wbq[r] = p.bqw[o];
        }
    };
    load_tile(kbeg);

    // the constant 0/1 selection operand: lane (n + 32 h) holds column n, k-half h; byte p of it
    // is 1.0 (e4m3 0x38) where the same byte of A lane (m + 32 h) holds a code of output n mod 16
    xm_v8i sel;
    {
        const int n = lane & 31, h = lane >> 5;
#pragma unroll
        for (int v = 0; v < 8; ++v) {
            uint32_t w = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int pb = 4 * v + b;
                if ((n >> 4) == h && (pb & 15) == (n & 15)) w |= 0x38u << (8 * b);
            }
            sel[v] = (int)w;
        }
    }
    xm_v16f dacc;
#pragma unroll
    for (int r = 0; r < 16; ++r) dacc[r] = 0.0f;
    xm_v8i av = {0, 0, 0, 0, 0, 0, 0, 0};
    const char *lut = reinterpret_cast<const char *>(sm.lut);

    for (int64_t k0 = kbeg; k0 < kend; k0 += BK) {
#pragma unroll
        for (int r = 0; r < (BM * BK) / NT; ++r) {
            sm.aw[akk[r]][arow[r]] = wa[r];
        }
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            sm.bq[bkk[r]][bq[r]] = wbq[r];
        }
        __syncthreads();
        if (k0 + BK < kend) load_tile(k0 + BK);  // next tile's loads fly during this tile's math

        // per K-step: one word per A element (the conversion reads only the scale's exponent
        // field; the table row offset is a bit field of it), the thread's two column pairs, all 8
        // table reads of the step, then the math; the next step's reads follow the math
#pragma unroll
        for (int kk = 0; kk < BK; ++kk) {
            const uint4 aw4 = *reinterpret_cast<const uint4 *>(&sm.aw[kk][ty * TM]);
            const uint32_t awv[TM] = {aw4.x, aw4.y, aw4.z, aw4.w};
            const uint4 bq4 = *reinterpret_cast<const uint4 *>(&sm.bq[kk][tx * 2]);  // add0, off0, add1, off1
            uint32_t v0[TM], v1[TM];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                // (one word per A element; two LDS arrays without the mask: -2.6 % in A/B)
                v0[i] = *reinterpret_cast<const uint32_t *>(lut + ((awv[i] & XM_ROW_MASK) + bq4.y));
                v1[i] = *reinterpret_cast<const uint32_t *>(lut + ((awv[i] & XM_ROW_MASK) + bq4.w));
            }
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const uint32_t x0 = __builtin_bit_cast(uint32_t, __builtin_bit_cast(xm_u2, v0[i]) +
                                                                     __builtin_bit_cast(xm_u2, bq4.x));
                const xm_u2 x1 = __builtin_bit_cast(xm_u2, v1[i]) + __builtin_bit_cast(xm_u2, bq4.z);
                const float sc = __uint_as_float(awv[i]);
                xm_s2 cv;  // low word: no input register needed (see the f32 form)
                asm("v_cvt_scalef32_pk_fp8_bf16 %0, %1, %2" : "=v"(cv) : "v"(x0), "v"(sc));
                cv = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(cv, __builtin_bit_cast(xm_b2, x1), sc, true);
                av[4 * (kk & 1) + i] = __builtin_bit_cast(int, cv);
            }
            if (kk & 1) dacc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, sel, dacc, 0, 0, 0, 127, 0, 127);
        }
        __syncthreads();
    }

    // a term beyond the e4m3 range came back NaN (and poisons its column): the exact kernel
    // reruns the launch
    bool nan = false;
#pragma unroll
    for (int r = 0; r < 16; ++r) nan |= __builtin_isnan(dacc[r]);
    if (__syncthreads_or(nan ? 1 : 0) && tid == 0) atomicOr(p.flag, 1u);

    // D (units of 2^(7-bR)) -> [BM][BN] tile in LDS -> each thread's 4x4 block, epilogue mapping
    // with consecutive lanes on consecutive pixels (coalesced NCHW stores)
    const float f8S = __uint_as_float((uint32_t)min(max(134 - bR, 1), 254) << 23);
    float *ct = reinterpret_cast<float *>(&sm);
    {
        const int n = lane & 31, src = 32 * (n >> 4), o = n & 15;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            const int L = m + src;
            const int row = (L & 15) * TM + (o >> 2), col = (4 * wv + (L >> 4)) * TN + (o & 3);
            ct[row * XM_CP + col] = dacc[r] * f8S;
        }
    }
    __syncthreads();
    const int ety = tid & 15, etx = tid >> 4;
    float acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = ct[(ety * TM + i) * XM_CP + etx * TN + j];
    store_tile(p, split, m0, n0, ety, etx, acc);
}
