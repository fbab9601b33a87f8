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

constexpr int XM_LUT_FLOATS = 64 * 2 * 16 * 2;  // 16 KiB
constexpr int XM_BQ = BN / 2 + 2;                // pair slots per staged K row (padded)
struct XmSmem {
    float lut[XM_LUT_FLOATS];
    float as[BK][AP];        // cvt scale of A(m, k): 2^(7-bR)/|c_a|, 2^127 for zeros (as bits)
    uint32_t ar[BK][AP];     // byte offset of A(m, k)'s table row
    float bc[BK][BP];        // c_b = sign(b) 2^floor(log2|b|), 0 for b = 0
    uint32_t bp[BK][XM_BQ];  // byte offset of the (column 2q, 2q+1) pair block incl. the copy
};
constexpr int XM_CP = BN + 1;  // epilogue transpose tile [BM][BN + 1] floats, aliased on XmSmem
static_assert(sizeof(float) * BM * XM_CP <= sizeof(XmSmem), "epilogue tile must fit the staging LDS");

__global__ __launch_bounds__(NT) void gemm_f8mx_kernel(const GemmArgs p) {
    __shared__ __attribute__((aligned(16))) XmSmem sm;

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int ty = lane & 15, tx = 4 * wv + (lane >> 4);  // half-wave = 16 row groups x 2 column groups
    const int64_t num_mt = (p.M + BM - 1) / BM;
    const int64_t tiles = num_mt * ((p.N + BN - 1) / BN);
    const int64_t bid = (int64_t)blockIdx.x % tiles, split = (int64_t)blockIdx.x / tiles;
    const int64_t m0 = (bid % num_mt) * BM;
    const int64_t n0 = (bid / num_mt) * BN;
    const int64_t kbeg = split * p.kchunk, kend = min(p.K, kbeg + p.kchunk);
    constexpr int M = 3;
    const int bA = *p.bA, bR = *p.bR;
    const uint32_t emnA = (uint32_t)(128 - bA) << 23;

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

    // B staging slots: (pair q, k row kk), two per thread; lanes along k for k-contiguous weights
    const bool b_ncontig = (p.sbn == 1);
    int bq[2], bkk[2];
    uint32_t emnB[2][2];
    bool bias_ok = bR >= -100 && bR <= 120 && bA >= -100 && bA <= 120;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int e = tid + NT * r;
        bq[r] = b_ncontig ? (e & 31) : (e >> 4);
        bkk[r] = b_ncontig ? (e >> 5) : (e & 15);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int64_t n = n0 + 2 * bq[r] + h;
            const int bb = (n < p.N) ? p.bB[n * p.bBs] : 0;
            bias_ok = bias_ok && bb >= -100 && bb <= 120;
            emnB[r][h] = (uint32_t)(128 - bb) << 23;
        }
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
    int arow[(BM * BK) / NT], akk[(BM * BK) / NT];
#pragma unroll
    for (int r = 0; r < (BM * BK) / NT; ++r) {
        const int e = tid + NT * r;
        arow[r] = p.conv ? (tid & 63) : (e >> 4);
        akk[r] = p.conv ? ((tid >> 6) + 4 * r) : (e & 15);
    }
    float xa[(BM * BK) / NT], xb[2][2];
    auto load_tile = [&](int64_t k0) {
#pragma unroll
        for (int r = 0; r < (BM * BK) / NT; ++r) {
            float x = 0.0f;
            const int64_t k = k0 + akk[r];
            if (!p.conv) {
                const int64_t m = m0 + arow[r];
                if (m < p.M && k < kend) x = p.A[m * p.lda + k];
            } else if (crow_ok && k < kend) {  // implicit im2col (approx_calculation.py:724-747)
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
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int64_t n = n0 + 2 * bq[r] + h, k = k0 + bkk[r];
                xb[r][h] = (n < p.N && k < kend) ? p.B[k * p.sbk + n * p.sbn] : 0.0f;
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
    const char *lut = reinterpret_cast<const char *>(sm.lut);

    for (int64_t k0 = kbeg; k0 < kend; k0 += BK) {
        bool bad = !bias_ok;
#pragma unroll
        for (int r = 0; r < (BM * BK) / NT; ++r) {
            float c;
            uint32_t mc;
            bad |= !stage_decode(xa[r], M, emnA, true, c, mc);
            const uint32_t cb = __float_as_uint(c);
            const int se = 261 - bR - (int)((cb >> 23) & 0xFFu);
            const bool zero = (cb & 0x7FFFFFFFu) == 0u;
            bad |= !zero && (se < 1 || se > 254);
            sm.as[akk[r]][arow[r]] = __uint_as_float((uint32_t)(zero ? 254 : min(max(se, 1), 254)) << 23);
            sm.ar[akk[r]][arow[r]] = zero ? 0u : ((cb >> 31) * 8u + mc) * 8u;
        }
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            float c0, c1;
            uint32_t m0c, m1c;
            bad |= !stage_decode(xb[r][0], M, emnB[r][0], true, c0, m0c);
            bad |= !stage_decode(xb[r][1], M, emnB[r][1], true, c1, m1c);
            *reinterpret_cast<float2 *>(&sm.bc[bkk[r]][2 * bq[r]]) = make_float2(c0, c1);
            sm.bp[bkk[r]][bq[r]] = (m0c + 8u * m1c) * 256u + (uint32_t)((bq[r] >> 1) & 1) * 128u;
        }
        const int anybad = __syncthreads_or(bad ? 1 : 0);
        if (anybad && tid == 0) atomicOr(p.flag, 1u);
        if (k0 + BK < kend) load_tile(k0 + BK);

#pragma unroll
        for (int kp = 0; kp < BK; kp += 2) {
            uint32_t code[8];
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int kk = kp + s;
                const float4 as4 = *reinterpret_cast<const float4 *>(&sm.as[kk][ty * TM]);
                const uint4 ar4 = *reinterpret_cast<const uint4 *>(&sm.ar[kk][ty * TM]);
                const float4 bc4 = *reinterpret_cast<const float4 *>(&sm.bc[kk][tx * TN]);
                const uint2 bp2 = *reinterpret_cast<const uint2 *>(&sm.bp[kk][tx * 2]);
                const float as[TM] = {as4.x, as4.y, as4.z, as4.w};
                const uint32_t ar[TM] = {ar4.x, ar4.y, ar4.z, ar4.w};
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const float2 v01 = *reinterpret_cast<const float2 *>(lut + (ar[i] + bp2.x));
                    const float2 v23 = *reinterpret_cast<const float2 *>(lut + (ar[i] + bp2.y));
                    xm_s2 cv = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32((xm_s2){0, 0}, v01.x * bc4.x, v01.y * bc4.y,
                                                                        as[i], false);
                    cv = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(cv, v23.x * bc4.z, v23.y * bc4.w, as[i], true);
                    code[4 * s + i] = __builtin_bit_cast(uint32_t, cv);
                }
            }
            const xm_v8i av = {(int)code[0], (int)code[1], (int)code[2], (int)code[3],
                               (int)code[4], (int)code[5], (int)code[6], (int)code[7]};
            dacc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, sel, dacc, 0, 0, 0, 127, 0, 127);
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

