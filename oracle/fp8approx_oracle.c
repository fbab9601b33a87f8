/*
 * fp8approx_oracle.c -- CPU restatement of the reference approx_v9 arithmetic.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path links, loads or calls this file:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it, and only
 * as the checker.  It is a scalar, literal restatement of the reference's op sequence in
 * IEEE float32 (compile with -ffp-contract=off: every torch op rounds once), so each
 * per-product term is bit-identical to the reference's (pinned against tests/golden/g*.npz,
 * which were produced by the reference itself -- see tests/golden/gen_golden.py).
 *
 * Reference: revollllt/FP8_quantization @ 2024-11-08, approx/approx_matmul_whole_v9.py.
 * Each function cites the lines it restates.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#define ORC_APPROX 1u  /* with_approx                */
#define ORC_S2N    2u  /* with_s2nn2s_opt            */
#define ORC_QBMA   4u  /* quant_btw_mult_accu        */
#define ORC_GCLIP  8u  /* golden_clip_OF             */
#define ORC_TB     16u /* biases passed as int tensors (single-column call) */
#define ORC_V5     32u /* superseded integer-adder model, approx_matmul_whole_v5.py         */
#define ORC_OFUF   64u /* v5 sim_hw_add_OFUF                                               */
#define ORC_OF    128u /* v5 with_OF_opt                                                   */
#define ORC_UF    256u /* v5 with_UF_opt                                                   */

/* torch float32 pow(2.0, k) for an int32 exponent: correctly rounded 2^k (0 below
 * 2^-150, inf above 2^127).  Used wherever the reference writes 2.0**(int tensor) or
 * torch.ldexp(x, k) (= x * pow(2.0, k)). */
static float pow2f(int k) { return ldexpf(1.0f, k); }

/* param_prepare, approx_matmul_whole_v9.py:189-229.  With an int bias the powers are
 * Python floats; with an int32 tensor bias (tb) 2**(negative) is an INTEGER power and
 * evaluates to 0 (quirk F5), so min_norm = 0 once b >= 2. */
typedef struct {
    int E, M, b, tb;
    float min_norm, max_norm;
    int max_expo, max_mant;
} orc_fmt;

static orc_fmt orc_param(int E, int M, int b, int tb) {
    orc_fmt p;
    p.E = E; p.M = M; p.b = b; p.tb = tb;
    p.max_expo = (1 << E) - 1;
    p.max_mant = (1 << M) - 1;
    double frac = 2.0 - ldexp(1.0, -M);
    if (!tb) {
        p.min_norm = (float)ldexp(1.0, 1 - b);
        p.max_norm = (float)(ldexp(1.0, p.max_expo - b) * frac);
    } else {
        p.min_norm = (1 - b >= 0) ? (float)ldexp(1.0, 1 - b) : 0.0f;
        p.max_norm = (p.max_expo - b >= 0) ? (float)ldexp(1.0, p.max_expo - b) * (float)frac : 0.0f;
    }
    return p;
}

/* float_to_fpany_absint_torch, v9:233-291. */
static void orc_dec1(float x, const orc_fmt *p, int clip, int32_t *expo_out, int32_t *mant_out) {
    int e;
    float f = frexpf(x, &e);
    int sub = fabsf(x) < p->min_norm;
    float t;
    if (sub) t = fabsf(f) * pow2f(e + (p->b - 1 + p->M));          /* v9:274 */
    else     t = (fabsf(f) * 2.0f - 1.0f) * pow2f(p->M);            /* v9:275 */
    float r = rintf(t);                                             /* torch.round: half-even */
    if (r > (float)p->max_mant) r = (float)p->max_mant;             /* clamp(max=) only      */
    int32_t mant = (int32_t)r;
    int32_t expo = sub ? 0 : e + (p->b - 1);                        /* v9:280 */
    if (clip && ((x < -p->max_norm) || (x > p->max_norm))) {        /* v9:283-286 */
        expo = p->max_expo;
        mant = p->max_mant;
    }
    *expo_out = expo;
    *mant_out = mant;
}

/* fpany_absint_to_float_torch, v9:295-329 (expo/mant form). */
static float orc_rec1(float sign, int32_t expo, int32_t mant, const orc_fmt *p) {
    float ms = (float)mant / (float)(1 << p->M);
    float v = (expo == 0) ? pow2f(1 - p->b) * ms : pow2f(expo - p->b) * (1.0f + ms);
    return v * sign;
}

/* quant_to_fp_any_vectorize_torch (Q_R), v9:333-362. */
static float orc_q1(float x, const orc_fmt *p, int clip) {
    int32_t e, m;
    orc_dec1(x, p, clip, &e, &m);
    float sign = (x < 0.0f) ? -1.0f : 1.0f;
    return orc_rec1(sign, e, m, p);
}

/* One product term of the v5 integer-adder model (approx_matmul_whole_v5.py:10-183),
 * generalised to per-operand biases: A and B decode with clip_OF=True (v5:22, 27-49), the
 * product is the integer sum of the two (expo << M | mant) codes minus (bA + bB - bR) << M
 * (v5:56-59 with B_neg, v5:162: with one bias b that is b << M) plus the compensation table
 * entry; optionally wrapped like a hardware adder of E+M bits (v5:165-178); decoded with bR
 * (v5:285-313: expo = floor(r / 2^M), mant = r mod 2^M, so a zero operand gives a NONZERO
 * term) and signed with sign(a) * sign(b) (v5:108-111).  The whole v5 call uses one
 * custom_bias for A, B and the result (bA = bB = bR). */
static float orc_term_v5(float a, float b, int M, const orc_fmt *pA, const orc_fmt *pB,
                         const orc_fmt *pR, const int32_t *table, unsigned flags) {
    const int E = pA->E, n = 1 << M;
    int32_t eA, mA, eB, mB;
    orc_dec1(a, pA, 1, &eA, &mA);
    orc_dec1(b, pB, 1, &eB, &mB);
    int32_t r = eA * n + mA + eB * n + mB - (pA->b + pB->b - pR->b) * n + table[mA * n + mB];
    if (flags & ORC_OFUF) {                                         /* v5:165-178 */
        const int32_t maxi = (1 << (E + M)) - 1, mod = 1 << (E + M);
        int of = r > maxi, uf = r < 0;
        r = ((r % mod) + mod) % mod;                                /* torch %: sign of divisor */
        if ((flags & ORC_OF) && of) r = maxi;
        if ((flags & ORC_UF) && uf) r = r % n;
    }
    int32_t expo = (r >= 0) ? r / n : -((-r + n - 1) / n);          /* floor division */
    int32_t mant = r - expo * n;
    float ms = (float)mant / (float)n;
    float v = (expo == 0) ? pow2f(1 - pR->b) * ms : pow2f(expo - pR->b) * (1.0f + ms);
    float sign = ((a < 0.0f) ? -1.0f : 1.0f) * ((b < 0.0f) ? -1.0f : 1.0f);
    return v * sign;
}

/* One product term of custom_matmul_vectorize, v9:29-108, for element (a, b). */
static float orc_term1(float a, float b, int M, const orc_fmt *pA, const orc_fmt *pB,
                       const orc_fmt *pR, const int32_t *table, unsigned flags) {
    if (flags & ORC_V5) return orc_term_v5(a, b, M, pA, pB, pR, table, flags);
    const int s2n = (flags & ORC_S2N) != 0, qbma = (flags & ORC_QBMA) != 0;
    const int gclip = (flags & ORC_GCLIP) != 0, approx = (flags & ORC_APPROX) != 0;
    float g = a * b;                                                /* v9:30 */
    int zero = (g == 0.0f);                                         /* v9:32 */
    if (qbma) g = orc_q1(g, pR, gclip);                             /* v9:35-36 */
    int a_sub = fabsf(a) < pA->min_norm;                            /* v9:47-48 */
    int b_sub = fabsf(b) < pB->min_norm;
    float scale = (float)(1 << M);
    float a2 = a, b2 = b;
    if (s2n) {                                                      /* v9:52-54 */
        if (a_sub) a2 = a * scale;
        if (b_sub) b2 = b * scale;
    }
    int32_t eA, mA, eB, mB;
    orc_dec1(a2, pA, 0, &eA, &mA);                                  /* v9:58-59 */
    orc_dec1(b2, pB, 0, &eB, &mB);
    int32_t approx_expo = eA + eB - (pA->b + pB->b - pR->b);        /* v9:66-67, 173-175 */
    float sgn = (g < 0.0f) ? -1.0f : 1.0f;                          /* v9:68 (quirk F7) */
    /* mult_result_mant, v9:178-184; negative mantissa codes wrap like torch indexing */
    float ulp = pow2f(-M);
    float mp = (1.0f + (float)mA * ulp) * (1.0f + (float)mB * ulp);
    if (approx) {
        int n = 1 << M;
        int ia = mA < 0 ? mA + n : mA, ib = mB < 0 ? mB + n : mB;
        mp = mp - ulp * (float)table[ia * n + ib];
    }
    float v;
    if (s2n) {                                                      /* v9:72-81 */
        v = pow2f(approx_expo - pR->b) * mp * sgn;
        if (a_sub) v = v / scale;
        if (b_sub) v = v / scale;
        if (zero) v = 0.0f;
    } else {                                                        /* v9:85-98 */
        int norm = (eA > 0) && (eB > 0) && (fabsf(g) >= pR->min_norm);
        v = norm ? pow2f(approx_expo - pR->b) * mp * sgn : g;
    }
    if (qbma) v = orc_q1(v, pR, gclip);                             /* v9:107-108 */
    return v;
}

/* ------------------------------------------------------------------ exported entry points */

void orc_decompose(const float *x, int64_t n, int E, int M, int b, int tb, int clip,
                   int32_t *expo, int32_t *mant) {
    orc_fmt p = orc_param(E, M, b, tb);
    for (int64_t i = 0; i < n; ++i) orc_dec1(x[i], &p, clip, &expo[i], &mant[i]);
}

void orc_quant(const float *x, int64_t n, int E, int M, int b, int tb, int clip, float *q) {
    orc_fmt p = orc_param(E, M, b, tb);
    for (int64_t i = 0; i < n; ++i) q[i] = orc_q1(x[i], &p, clip);
}

/* terms[m][k][n] for A[M][K] (lda), B[K][N] (ldb); bB is per column (length N). */
void orc_terms(const float *A, int64_t lda, const float *B, int64_t ldb, float *T,
               int Mr, int N, int K, int E, int Mw, int bA, const int32_t *bB, int bR,
               const int32_t *table, unsigned flags) {
    int tb = (flags & ORC_TB) != 0;
    orc_fmt pA = orc_param(E, Mw, bA, tb), pR = orc_param(E, Mw, bR, tb);
    for (int n = 0; n < N; ++n) {
        orc_fmt pB = orc_param(E, Mw, bB[n], tb);
        for (int m = 0; m < Mr; ++m)
            for (int k = 0; k < K; ++k)
                T[((int64_t)m * K + k) * N + n] =
                    orc_term1(A[m * lda + k], B[k * ldb + n], Mw, &pA, &pB, &pR, table, flags);
    }
}

/* C[m][n] = sum_k term, accumulated in double (a tighter reference than any fp32 order). */
void orc_matmul(const float *A, int64_t lda, const float *B, int64_t ldb, float *C, int64_t ldc,
                int Mr, int N, int K, int E, int Mw, int bA, const int32_t *bB, int bR,
                const int32_t *table, unsigned flags, float *abs_sum /* nullable [M][N] */) {
    int tb = (flags & ORC_TB) != 0;
    orc_fmt pA = orc_param(E, Mw, bA, tb), pR = orc_param(E, Mw, bR, tb);
    for (int n = 0; n < N; ++n) {
        orc_fmt pB = orc_param(E, Mw, bB[n], tb);
        for (int m = 0; m < Mr; ++m) {
            double s = 0.0, sa = 0.0;
            for (int k = 0; k < K; ++k) {
                float v = orc_term1(A[m * lda + k], B[k * ldb + n], Mw, &pA, &pB, &pR, table, flags);
                s += (double)v;
                sa += fabs((double)v);
            }
            C[m * ldc + n] = (float)s;
            if (abs_sum) abs_sum[m * ldc + n] = (float)sa;
        }
    }
}

/* One quantize_to_fp8_ste_MM value (fp8_quantizer.py:111-154), bias given. */
static float orc_fq1(float v, float mx, float bias, int M, int sign_bits) {
    float xc = fminf(fmaxf(v, sign_bits ? -mx : 0.0f), mx);
    int e;
    frexpf(xc, &e);
    float ls = (xc == 0.0f) ? 1.0f : fmaxf((float)(e - 1) + bias, 1.0f);
    float sc = ldexpf(1.0f, (int)(ls - (float)M - bias));
    return rintf(xc / sc) * sc;
}

static float orc_fq_bias(float mx, int E, int M) {
    return rintf((float)(1 << E) - log2f(mx) + log2f(2.0f - ldexpf(1.0f, -M)) - 1.0f);
}

/* quantize_after_mult_and_add (approx_calculation.py:787-795): C = fq(sum_k fq(a*b)).
 * The sum is accumulated in float32 in k order (the GPU kernel's order), so C is comparable
 * bit for bit; Cpre (nullable) receives the pre-quantisation sums. */
void orc_matmul_qamaa(const float *A, int64_t lda, const float *B, int64_t ldb, float *C, float *Cpre,
                      int Mr, int N, int K, float mx, int n_bits, int M, int sign_bits) {
    int E = n_bits - sign_bits - M;
    float bias = orc_fq_bias(mx, E, M);
    for (int m = 0; m < Mr; ++m)
        for (int n = 0; n < N; ++n) {
            float s = 0.0f;
            for (int k = 0; k < K; ++k) s += orc_fq1(A[m * lda + k] * B[k * ldb + n], mx, bias, M, sign_bits);
            if (Cpre) Cpre[m * N + n] = s;
            C[m * N + n] = orc_fq1(s, mx, bias, M, sign_bits);
        }
}

/* quantize_to_fp8_ste_MM forward value (fp8_quantizer.py:97-173) for a per-tensor or
 * per-row maxval: bias = round(2^E - log2(maxval) + log2(2 - 2^-M) - 1), then
 * round-half-even onto the grid 2^(max(floor(log2|x|)+bias, 1) - M - bias).
 * floor(log2|x|) is taken exactly from frexp (values where a float log2
 * would round up sit within a few ulps of a power of two and land on it either way). */
void orc_fp8_fake_quant(const float *x, int64_t rows, int64_t cols, const float *maxval,
                        int per_row, int E, int M, float *out, float *bias_out) {
    for (int64_t r = 0; r < rows; ++r) {
        float mx = maxval[per_row ? r : 0];
        float bias = rintf((float)(1 << E) - log2f(mx) + log2f(2.0f - ldexpf(1.0f, -M)) - 1.0f);
        if (bias_out && (per_row || r == 0)) bias_out[per_row ? r : 0] = bias;
        for (int64_t c = 0; c < cols; ++c) {
            float v = x[r * cols + c];
            float xc = fminf(fmaxf(v, -mx), mx);
            int e;
            frexpf(xc, &e);
            float ls = (xc == 0.0f) ? 1.0f : fmaxf((float)(e - 1) + bias, 1.0f);
            float sc = ldexpf(1.0f, (int)(ls - (float)M - bias));
            out[r * cols + c] = rintf(xc / sc) * sc;
        }
    }
}
