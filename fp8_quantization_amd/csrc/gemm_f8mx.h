// gemm_f8mx.h -- the E4M3 fast path with matrix-core accumulation (included by fp8approx.hip).
//
// Same arithmetic as gemm_fast_kernel<.., TM_F8>: for on-grid E4M3 operands with
// s2n and per-product quantization (v9:51-113), each term is
//     Q_R(V'(s_a, m_a, m_b) * c_b * |c_a|)  =  2^(7-bR) * e4m3(V' * c_b / scale_a),
// scale_a = 2^(7-bR) / |c_a|, where V' = min(sig_a sig_b - T[m_a][m_b] 2^-M, top of its binade)
// is an LDS table value and e4m3() is gfx950's scaled fp8 conversion (RNE; the bR grid is the
// OCP e4m3 grid scaled by 2^(7-bR), subnormal band included).
//
// What is new: the fp8 codes the conversion produces are NOT decoded and added on the VALU.
// They are summed by the matrix core: one v_mfma_scale_f32_32x32x64_f8f6f4 per two K-steps
// multiplies the wave's 2048 codes by a constant 0/1 selection matrix S, so that
//     D[m][n] += sum over the two K-steps of the code of output (n mod 16) of lane m + 32 (n / 16).
// Products with 1.0 and 0 are exact, the accumulator is fp32 (D is in units of 2^(7-bR)), so the
// sum differs from an in-order fp32 sum only by accumulation order -- inside the reference's own
// order freedom (v9:113, torch's sum) and the 1e-5 * sum|term| bar.  Per product the VALU now
// issues: half an LDS address add, one multiply and half a scaled conversion (the f32 decode and
// the add are gone), and the table read is one ds_read_b64 per two products.
//
// Operands are decoded ONCE per launch by two pre-pass kernels (xm_decode_a / xm_decode_b):
// an A element becomes one 32-bit word (cvt scale bits | table row offset), a B element its c_b
// plus, per column pair, the pair block offset.  The GEMM's staging is then a gather and two
// bit-field ops, instead of a full decode for every element of every tile (a 3x3 conv gathers
// each input element 9 times).  The pre-passes also carry the fallback checks (off-grid operand,
// exactness window, e4m3 scale range, bias window) into the launch's flag word.
//
// LDS table layout [pair][copy][row][2 floats]: pair = (m_b of column 2q) + 8 (m_b of column
// 2q+1), row = 8 s_a + m_a (zero A operands take scale 2^127, so the conversion returns 0 for
// them and they need no row of their own), copy = parity of the consuming thread's column
// group.  Threads are mapped so that each 32-lane half-wave holds 16 row groups x 2 column
// groups: per read it touches at most 16 rows of one copy per column group, each on its own
// bank pair -- conflict-free (MI355X_MICROARCH.md §LDS: ds_read_b64 banks (a/4) mod 64).
// (included inside namespace fp8a, after GemmArgs / stage_decode / store_tile)

typedef int xm_v8i __attribute__((ext_vector_type(8)));
typedef float xm_v16f __attribute__((ext_vector_type(16)));
typedef short xm_s2 __attribute__((ext_vector_type(2)));
typedef float xm_f2 __attribute__((ext_vector_type(2)));  // (a plain pair: v_pk_mul_f32 lost in A/B)

constexpr int XM_LUT_FLOATS = 64 * 2 * 16 * 2;  // 16 KiB
constexpr int XM_BQ = BN / 2 + 2;                // pair slots per staged K row (padded)
constexpr uint32_t XM_ZERO_WORD = 254u << 23;    // A = 0: cvt scale 2^127 (the code is 0), row 0
struct XmSmem {
    float lut[XM_LUT_FLOATS];
    uint32_t aw[BK][AP];     // A(m, k)'s word: cvt scale exponent << 23 | table row << 3
    float bc[BK][BP];        // c_b = sign(b) 2^floor(log2|b|), 0 for b = 0
    uint32_t bp[BK][XM_BQ];  // byte offset of the (column 2q, 2q+1) pair block incl. the copy
};
constexpr int XM_CP = BN + 1;  // epilogue transpose tile [BM][BN + 1] floats, aliased on XmSmem
static_assert(sizeof(float) * BM * XM_CP <= sizeof(XmSmem), "epilogue tile must fit the staging LDS");

// Exactness / range window shared by the pre-passes (as bias_ok in gemm_fast_kernel)
__device__ __forceinline__ bool xm_bias_ok(int b) { return b >= -100 && b <= 120; }

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
    return ((uint32_t)min(max(se, 1), 254) << 23) | (((cb >> 31) * 8u + mc) << 3);
}

// A pre-pass, one (image | row) per blockIdx.y step.  conv: the group's channel slice of x
// [Bn][Cin][H][W] (channels cbase..cbase+aw_c) -> words [Bn][aw_c][H][W]; matrix: A [M][lda] ->
// words [M][awld] (columns >= K zero words).
__global__ __launch_bounds__(256) void xm_decode_a(const GemmArgs p) {
    const int bA = *p.bA, bR = *p.bR;
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
            o[i] = (i < lim) ? xm_word_a(in[i], emnA, bR, ok) : XM_ZERO_WORD;
            bad |= !ok;
        }
    }
    if (__syncthreads_or(bad ? 1 : 0) && threadIdx.x == 0) atomicOr(p.flag, 1u);
}

// B pre-pass: per (k, pair Q) of the padded [Kpad][npad] extent, c_b of both columns and the
// pair block offset ((m_b0 + 8 m_b1) * 256 + copy * 128 bytes, copy = parity of the consuming
// thread's 4-column group = (Q >> 1) & 1); out-of-range elements are zeros.
__global__ __launch_bounds__(256) void xm_decode_b(const GemmArgs p, int64_t kpad) {
    const int bA = *p.bA, bR = *p.bR;
    bool bad = !(xm_bias_ok(bA) && xm_bias_ok(bR));
    const int64_t hq = p.npad / 2, n = kpad * hq;
    float *const bc = const_cast<float *>(p.bcw);
    uint32_t *const bp = const_cast<uint32_t *>(p.bpw);
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
        *reinterpret_cast<float2 *>(&bc[k * p.npad + 2 * q]) = make_float2(c[0], c[1]);
        bp[i] = (mc[0] + 8u * mc[1]) * 256u + (uint32_t)((q >> 1) & 1) * 128u;
    }
    if (__syncthreads_or(bad ? 1 : 0) && threadIdx.x == 0) atomicOr(p.flag, 1u);
}

#ifndef XM_PIPE
#define XM_PIPE 0
#endif
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

    // table: V'(s_a, m_a, m_b) for both columns of a pair, both copies
    for (int e = tid; e < XM_LUT_FLOATS / 2; e += NT) {
        const int pr = e >> 5, row = e & 15;
        const int ma = row & 7;
        float v2[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int mb = h ? (pr >> 3) : (pr & 7);
            const float t = (float)p.tab.raw[ma * 8 + mb];
            float v = __fmaf_rn(1.0f + 0.125f * ma, 1.0f + 0.125f * mb, -t * 0.125f);  // exact
            // Q_R's pre-clamp (QC::kb): the mantissa saturates instead of carrying, and on the
            // subnormal grid the top tie rounds down
            v = fminf(v, __uint_as_float(__float_as_uint(v) & 0x7F800000u) * (1.875f - p2(-22)));
            v2[h] = (row >= 8) ? -v : v;
        }
        *reinterpret_cast<float2 *>(&sm.lut[2 * e]) = make_float2(v2[0], v2[1]);
    }

    // B staging slots: pair q = e & 31 (lanes along n: coalesced), k row kk = e >> 5
    const int64_t hq = p.npad / 2;
    const float *bcg[2];
    const uint32_t *bpg[2];
    int bq[2], bkk[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int e = tid + NT * r;
        bq[r] = e & 31;
        bkk[r] = e >> 5;
        bcg[r] = p.bcw + (kbeg + bkk[r]) * p.npad + n0 + 2 * bq[r];
        bpg[r] = p.bpw + (kbeg + bkk[r]) * hq + n0 / 2 + bq[r];
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
    float2 wbc[2];
    uint32_t wbp[2];
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
            const int64_t o = k0 - kbeg;
            wbc[r] = *reinterpret_cast<const float2 *>(bcg[r] + o * p.npad);
            wbp[r] = bpg[r][o * hq];
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
            *reinterpret_cast<float2 *>(&sm.bc[bkk[r]][2 * bq[r]]) = wbc[r];
            sm.bp[bkk[r]][bq[r]] = wbp[r];
        }
        __syncthreads();
        if (k0 + BK < kend) load_tile(k0 + BK);  // next tile's loads fly during this tile's math

        // per K-step: one word per A element (the conversion reads only the scale's exponent
        // field; the table row offset is bits 3-6), c_b and the pair offsets of the thread's
        // columns, then all 8 table reads of the step, then the math.  XM_PIPE issues the next
        // step's reads before this step's math.
        uint4 aw4 = *reinterpret_cast<const uint4 *>(&sm.aw[0][ty * TM]);
        float4 bc4 = *reinterpret_cast<const float4 *>(&sm.bc[0][tx * TN]);
        uint2 bp2 = *reinterpret_cast<const uint2 *>(&sm.bp[0][tx * 2]);
        float2 v01s[TM], v23s[TM];
        auto lut_reads = [&](const uint4 &w4, const uint2 &p2, float2 (&a01)[TM], float2 (&a23)[TM]) {
            const uint32_t ar[TM] = {w4.x & 0x78u, w4.y & 0x78u, w4.z & 0x78u, w4.w & 0x78u};
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                a01[i] = *reinterpret_cast<const float2 *>(lut + (ar[i] + p2.x));
                a23[i] = *reinterpret_cast<const float2 *>(lut + (ar[i] + p2.y));
            }
        };
        lut_reads(aw4, bp2, v01s, v23s);
#pragma unroll
        for (int kk = 0; kk < BK; ++kk) {
            const float as[TM] = {__uint_as_float(aw4.x), __uint_as_float(aw4.y), __uint_as_float(aw4.z),
                                  __uint_as_float(aw4.w)};
            const float4 bcc = bc4;
            float2 c01[TM], c23[TM];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                c01[i] = v01s[i];
                c23[i] = v23s[i];
            }
            if (XM_PIPE && kk + 1 < BK) {
                aw4 = *reinterpret_cast<const uint4 *>(&sm.aw[kk + 1][ty * TM]);
                bc4 = *reinterpret_cast<const float4 *>(&sm.bc[kk + 1][tx * TN]);
                bp2 = *reinterpret_cast<const uint2 *>(&sm.bp[kk + 1][tx * 2]);
                lut_reads(aw4, bp2, v01s, v23s);
            }
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const xm_f2 x01 = {c01[i].x * bcc.x, c01[i].y * bcc.y};
                const xm_f2 x23 = {c23[i].x * bcc.z, c23[i].y * bcc.w};
                // the low-word conversion's high half is overwritten by the high-word one, so it
                // needs no input register (the builtin ties one, and the compiler zeroes it)
                xm_s2 cv;
                asm("v_cvt_scalef32_pk_fp8_f32 %0, %1, %2, %3" : "=v"(cv) : "v"(x01.x), "v"(x01.y), "v"(as[i]));
                cv = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(cv, x23.x, x23.y, as[i], true);
                av[4 * (kk & 1) + i] = __builtin_bit_cast(int, cv);
            }
            if (!XM_PIPE && kk + 1 < BK) {
                aw4 = *reinterpret_cast<const uint4 *>(&sm.aw[kk + 1][ty * TM]);
                bc4 = *reinterpret_cast<const float4 *>(&sm.bc[kk + 1][tx * TN]);
                bp2 = *reinterpret_cast<const uint2 *>(&sm.bp[kk + 1][tx * 2]);
                lut_reads(aw4, bp2, v01s, v23s);
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
