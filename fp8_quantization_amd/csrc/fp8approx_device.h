// fp8approx_device.h -- device-side arithmetic of the approx_v9 FP8 multiplier for gfx950.
//
// Two families of functions:
//   * exact_*  : a literal float32 restatement of the reference op sequence
//                (approx/approx_matmul_whole_v9.py).  Every reference torch op is one IEEE
//                float32 op here (the library is compiled with -ffp-contract=off), so each
//                product term is bit-identical to the reference.  Used for the tensor-bias
//                (single-column) path, for off-grid operand tiles and for fp8a_terms.
//   * q_fast   : a branch-free Q_R on the float32 bit pattern (6-7 VALU ops), valid for the
//                int-bias path; exactness argument in DESIGN.md §3.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fp8a {

enum : uint32_t { F_APPROX = 1u, F_S2N = 2u, F_QBMA = 4u, F_GCLIP = 8u, F_TB = 16u,
                  // superseded integer-adder model (approx_matmul_whole_v5.py) and its switches
                  F_V5 = 32u, F_OFUF = 64u, F_OF = 128u, F_UF = 256u };

__device__ __forceinline__ float p2(int k) { return ldexpf(1.0f, k); }

// param_prepare (v9:189-229).  Int bias: Python float powers.  Tensor bias (tb): 2**(negative)
// is an integer power and evaluates to 0 (quirk F5).
struct DFmt {
    float mn;   // min_norm
    float mx;   // max_norm
    int b, M, maxe, maxm;
};

__device__ __forceinline__ DFmt dfmt(int E, int M, int b, bool tb) {
    DFmt f;
    f.b = b;
    f.M = M;
    f.maxe = (1 << E) - 1;
    f.maxm = (1 << M) - 1;
    const float frac = 2.0f - p2(-M);
    if (!tb) {
        f.mn = p2(1 - b);
        f.mx = ldexpf(frac, f.maxe - b);
    } else {
        f.mn = (1 - b >= 0) ? p2(1 - b) : 0.0f;
        f.mx = (f.maxe - b >= 0) ? p2(f.maxe - b) * frac : 0.0f;
    }
    return f;
}

// float_to_fpany_absint_torch (v9:233-291).
__device__ __forceinline__ void exact_dec(float x, const DFmt &f, bool clip, int &expo, int &mant) {
    int e;
    const float fr = frexpf(x, &e);
    const bool sub = fabsf(x) < f.mn;
    const float t = sub ? fabsf(fr) * p2(e + (f.b - 1 + f.M)) : (fabsf(fr) * 2.0f - 1.0f) * p2(f.M);
    float r = rintf(t);
    r = (r > (float)f.maxm) ? (float)f.maxm : r;
    mant = (int)r;
    expo = sub ? 0 : e + (f.b - 1);
    if (clip && ((x < -f.mx) || (x > f.mx))) {
        expo = f.maxe;
        mant = f.maxm;
    }
}

// fpany_absint_to_float_torch (v9:295-329).
__device__ __forceinline__ float exact_rec(float sign, int expo, int mant, const DFmt &f) {
    const float ms = (float)mant * p2(-f.M);
    const float v = (expo == 0) ? p2(1 - f.b) * ms : p2(expo - f.b) * (1.0f + ms);
    return v * sign;
}

// quant_to_fp_any_vectorize_torch, Q_R (v9:333-362).
__device__ __forceinline__ float exact_q(float x, const DFmt &f, bool clip) {
    int e, m;
    exact_dec(x, f, clip, e, m);
    return exact_rec(x < 0.0f ? -1.0f : 1.0f, e, m, f);
}

// v5 adder wrap (approx_mult_new, v5:163-178): an (E+M)-bit hardware adder; overflow to
// max_norm_int with with_OF_opt, underflow to (r mod 2^M) with with_UF_opt.
__device__ __forceinline__ int32_t v5_ofuf(int32_t r, int32_t maxi, int M, uint32_t flags) {
    if (flags & F_OFUF) {
        const bool of = r > maxi, uf = r < 0;
        r &= maxi;  // mod 2^(E+M), two's complement: torch's % with a positive modulus
        if ((flags & F_OF) && of) r = maxi;
        if ((flags & F_UF) && uf) r &= (1 << M) - 1;
    }
    return r;
}

// One term of the v5 integer-adder model (approx_matmul_whole_v5.py:10-183), per-operand
// biases (v5 itself uses one custom_bias for A, B and the result): operands decode with
// clip_OF = True, the product is the sum of the (expo << M | mant) codes minus
// (bA + bB - bR) << M plus the compensation entry, decoded with floor division (a zero
// operand gives a nonzero term), signed with sign(a) * sign(b).
__device__ __forceinline__ float exact_term_v5(float a, float b, const DFmt &fA, const DFmt &fB, const DFmt &fR,
                                               const int8_t *tab, uint32_t flags) {
    const int M = fA.M, n = 1 << M;
    int eA, mA, eB, mB;
    exact_dec(a, fA, true, eA, mA);
    exact_dec(b, fB, true, eB, mB);
    int32_t r = (eA + eB - (fA.b + fB.b - fR.b)) * n + mA + mB + tab[mA * n + mB];
    r = v5_ofuf(r, ((fA.maxe + 1) << M) - 1, M, flags);
    const int32_t expo = r >> M, mant = r & (n - 1);  // floor division / modulo by 2^M
    const float ms = (float)mant * p2(-M);
    const float v = (expo == 0) ? p2(1 - fR.b) * ms : p2(expo - fR.b) * (1.0f + ms);
    return v * (((a < 0.0f) ? -1.0f : 1.0f) * ((b < 0.0f) ? -1.0f : 1.0f));
}

// One product term of custom_matmul_vectorize (v9:29-108).  tab: int8 [2^M][2^M].
__device__ __forceinline__ float exact_term(float a, float b, const DFmt &fA, const DFmt &fB,
                                            const DFmt &fR, const int8_t *tab, uint32_t flags) {
    if (flags & F_V5) return exact_term_v5(a, b, fA, fB, fR, tab, flags);
    const bool s2n = flags & F_S2N, qbma = flags & F_QBMA, gclip = flags & F_GCLIP;
    const int M = fA.M;
    float g = a * b;
    const bool zero = (g == 0.0f);
    if (qbma) g = exact_q(g, fR, gclip);
    const bool as = fabsf(a) < fA.mn, bs = fabsf(b) < fB.mn;
    const float scale = (float)(1 << M);
    float a2 = a, b2 = b;
    if (s2n) {
        if (as) a2 = a * scale;
        if (bs) b2 = b * scale;
    }
    int eA, mA, eB, mB;
    exact_dec(a2, fA, false, eA, mA);
    exact_dec(b2, fB, false, eB, mB);
    const int aexp = eA + eB - (fA.b + fB.b - fR.b);
    const float sgn = (g < 0.0f) ? -1.0f : 1.0f;
    const float ulp = p2(-M);
    float mp = (1.0f + (float)mA * ulp) * (1.0f + (float)mB * ulp);
    if (flags & F_APPROX) {
        const int n = 1 << M;
        const int ia = mA < 0 ? mA + n : mA, ib = mB < 0 ? mB + n : mB;
        mp = mp - ulp * (float)tab[ia * n + ib];
    }
    float v;
    if (s2n) {
        v = p2(aexp - fR.b) * mp * sgn;
        if (as) v = v / scale;
        if (bs) v = v / scale;
        if (zero) v = 0.0f;
    } else {
        const bool norm = (eA > 0) && (eB > 0) && (fabsf(g) >= fR.mn);
        v = norm ? p2(aexp - fR.b) * mp * sgn : g;
    }
    if (qbma) v = exact_q(v, fR, gclip);
    return v;
}

// ---------------------------------------------------------------------------- fast path
// Q_R for the int-bias path on the float32 bit pattern.  For |x| in binade e:
//   step  = 2^(max(e, e_min) - M)               (e_min = 1 - bR: subnormal grid below it)
//   bound = 2^e (2 - 2^-M) - ulp                (pre-clamp: rounding can no longer carry
//                                                past the largest M-bit mantissa, F6)
//   r     = ((min(|x|, bound) + C) - C),  C = 2^(max(e, e_min) + 23 - M)   (RNE at `step`)
struct QC {
    uint32_t emn;   // exponent field of 2^(1 - bR)
    uint32_t kexp;  // 0x7F800000
    uint32_t kbm;   // mantissa field of kb = 2 - 2^-M - 2^-22: bound = 2^e * kb = (x & EXP) | kbm
                    //   sits in (max - step/2, max] of binade e
    uint32_t dc;    // (23 - M) << 23: C = bound * 2^(23-M) has ulp(C) = step, C/step is even and
                    //   C +- 2^(e+1) stays in C's binade, so (x + C) - C rounds SIGNED x half-to-even
    uint32_t cmin;  // bits of 2^(e_min) * 1.5 * 2^(23 - M): the subnormal grid's C
    float kb;       // 2 - 2^-M - 2^-22 (float form)
    float kc;       // 1.5 * 2^(23 - M) (float form: C = 2^max(e, e_min) * kc)
    float cminf;    // 2^(e_min) * kc (float form)
    float maxnorm;  // max_norm(bR) (golden_clip_OF)
    float mnR;      // min_norm(bR)
    float thr;      // largest |g| that Q_R flushes to 0: 2^(-bR - M)
};

// kexp = 0x7F800000 and kdc = (23 - M) << 23 arrive as launch arguments: as literals the
// selector splits (x & EXP) | kbm into two ops (gfx9 VOP3 takes no literal) and re-associates
// the add of kdc into two adds.  Call once per kernel, outside loops.
__device__ __forceinline__ QC make_qc(int E, int M, int bR, uint32_t kexp, uint32_t kdc) {
    QC q;
    q.emn = (uint32_t)(127 + 1 - bR) << 23;
    // kbm lives in a VGPR: with kexp it would be the second scalar operand of v_and_or_b32,
    // which gfx9's one-constant-bus-read rule forbids, and the selector would emit and + or
    const uint32_t kbm = __float_as_uint(2.0f - p2(-M) - p2(-22)) & 0x007FFFFFu;
    asm("v_mov_b32 %0, %1" : "=v"(q.kbm) : "s"(kbm));
    q.kexp = kexp;
    q.dc = kdc;
    q.cmin = __float_as_uint(1.5f * p2(1 - bR + 23 - M));
    q.kb = 2.0f - p2(-M) - p2(-22);
    q.kc = 1.5f * p2(23 - M);
    q.cminf = 1.5f * p2(1 - bR + 23 - M);
    q.maxnorm = ldexpf(2.0f - p2(-M), (1 << E) - 1 - bR);
    q.mnR = p2(1 - bR);
    q.thr = p2(-bR - M);
    return q;
}

// Two equivalent instruction forms, picked per kernel by measurement (tools/q_variants.hip and
// tools/gemm_bench.py A/B on MI355X):
//   BITS = false, float form, 7 VALU ops (and, mul, med3, mul, max, add, sub): one int->float
//     hand-off per product; 1-2 % faster where an error-table term precedes it;
//   BITS = true, bit form, 6 VALU ops (and_or, med3, add_u32, max_u32, add, sub): one op fewer
//     but three half-rate ops and three int<->float hand-offs; 3 % faster with no table.
// No sign handling in either: the magic constant rounds negative and positive values alike.
// All min/max/med3 inputs are canonical (float arithmetic or positive bit patterns), so no
// canonicalisation is emitted.  Zero gives C = the subnormal grid's C, i.e. 0.  A negative value
// that rounds to zero comes back as +0 (the reference gives -0 or +0; both add nothing).
template <bool GCLIP, bool BITS = false>
__device__ __forceinline__ float q_fast(float x, const QC &q) {
    float xs = x;
    if (GCLIP) xs = __builtin_amdgcn_fmed3f(xs, -q.maxnorm, q.maxnorm);  // clip_OF first
    float c;
    if (BITS) {
        const uint32_t bdb = (__float_as_uint(xs) & q.kexp) | q.kbm;  // 2^floor(log2|x|) * kb
        const float bd = __uint_as_float(bdb);
        xs = __builtin_amdgcn_fmed3f(xs, -bd, bd);
        c = __uint_as_float(max(bdb + q.dc, q.cmin));
    } else {
        const float pe = __uint_as_float(__float_as_uint(xs) & 0x7F800000u);  // 2^floor(log2|x|)
        const float bd = pe * q.kb;
        xs = __builtin_amdgcn_fmed3f(xs, -bd, bd);
        c = fmaxf(pe * q.kc, q.cminf);
    }
    return (xs + c) - c;
}

// quantize_to_fp8_ste_MM (fp8_quantizer.py:97-173) as the qamaa per-product quantizer, for a
// per-tensor maxval: xc = clamp(x, [-]maxval, maxval); step = 2^(max(floor(log2|xc|), 1-bias) - M);
// round half-even; unlike Q_R the rounding MAY carry into the next binade.  6 VALU ops.
struct FQ {
    float lo, hi;   // clamp range
    float kc;       // 1.5 * 2^(23 - M)
    float cmin;     // 1.5 * 2^(1 - bias + 23 - M)
};

__device__ __forceinline__ FQ make_fq(float mx, int E, int M, int sign_bits) {
    FQ f;
    const float bias = rintf((float)(1 << E) - log2f(mx) + log2f(2.0f - p2(-M)) - 1.0f);
    f.hi = mx;
    f.lo = sign_bits ? -mx : 0.0f;
    f.kc = 1.5f * p2(23 - M);
    f.cmin = 1.5f * p2((int)(1.0f - bias) + 23 - M);
    return f;
}

__device__ __forceinline__ float fq_fast(float x, const FQ &f) {
    const float xc = __builtin_amdgcn_fmed3f(x, f.lo, f.hi);
    const float pe = __uint_as_float(__float_as_uint(xc) & 0x7F800000u);
    const float c = fmaxf(pe * f.kc, f.cmin);
    return (xc + c) - c;
}

}  // namespace fp8a
