// Accumulation precision of v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3): how far below the
// largest product (or the C input) a product still lands exactly in D.  One wave, row 0 of A set
// per case, B all ones (scale 1), D[0][0] printed against the exact sum.
// hipcc --offload-arch=gfx950 -O2 -o tools/bin_mfma_acc_precision tools/mfma_acc_precision.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

__global__ void k_mfma(const unsigned char *A, const int *asc, float cin, float *out, const int *bsc) {
    const int lane = threadIdx.x, r16 = lane & 15, g = lane >> 4;
    int a[8], b[8];
    for (int q = 0; q < 8; ++q) {
        unsigned w = 0;
        for (int e = 0; e < 4; ++e) {
            const int byte = 4 * q + e;
            const int k = (byte < 16) ? 16 * g + byte : 64 + 16 * g + (byte - 16);
            w |= (unsigned)A[r16 * 128 + k] << (8 * e);
        }
        a[q] = (int)w;
        b[q] = 0x38383838;  // 1.0 in e4m3
    }
    v8i av = {a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7]};
    v8i bv = {b[0], b[1], b[2], b[3], b[4], b[5], b[6], b[7]};
    v4f c = {cin, cin, cin, cin};
    v4f d = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 0, 0, 0, asc[r16 * 4 + g], 0, bsc[lane]);
    // lane (r16, g) holds D[4 g + r][r16]: D[0][0] is lane 0, r 0
    if (lane == 0) out[0] = d[0];
}

static unsigned char e4m3(double v) {  // exact small powers of two and 1.x only
    if (v == 0) return 0;
    int e;
    double f = frexp(v, &e);  // v = f 2^e, f in [0.5, 1)
    int E = e - 1 + 7;
    int m = (int)lround((f * 2 - 1) * 8);
    if (E <= 0) {  // subnormal: v = m/8 2^-6
        return (unsigned char)lround(v / ldexp(1.0, -9));
    }
    return (unsigned char)((E << 3) | m);
}

int main() {
    unsigned char *dA;
    int *dS;
    float *dO;
    hipMalloc(&dA, 16 * 128);
    hipMalloc(&dS, 16 * 4 * sizeof(int));
    hipMalloc(&dO, sizeof(float));
    int *dB;
    hipMalloc(&dB, 64 * sizeof(int));
    {
        int hb[64];
        for (int i = 0; i < 64; ++i) hb[i] = 127;
        hipMemcpy(dB, hb, sizeof(hb), hipMemcpyHostToDevice);
    }
    auto run = [&](const unsigned char *A, const int *S, float cin) {
        hipMemcpy(dA, A, 16 * 128, hipMemcpyHostToDevice);
        hipMemcpy(dS, S, 64 * sizeof(int), hipMemcpyHostToDevice);
        k_mfma<<<1, 64>>>(dA, dS, cin, dO, dB);
        float o;
        hipMemcpy(&o, dO, sizeof(float), hipMemcpyDeviceToHost);
        return o;
    };
    unsigned char A[16 * 128];
    int S[64];
    // case 1: product 1.0 at k = 0 and 2^-e at k = 1 (same block) / k = 40 (block 1, scaled)
    printf("case: 1 + 2^-e, the small product in the same 32-k block (e <= 9) or block 1 via its scale\n");
    for (int e = 1; e <= 30; ++e) {
        memset(A, 0, sizeof(A));
        for (int i = 0; i < 64; ++i) S[i] = 127;
        A[0] = 0x38;
        if (e <= 9) {
            A[1] = e4m3(ldexp(1.0, -e));
        } else {
            A[40] = 0x38;
            S[1] = 127 - e;  // row 0, block 1 scale 2^-e
        }
        const float o = run(A, S, 0.0f);
        printf("  e=%2d  D=%.10g  exact=%.10g  %s\n", e, o, 1.0 + ldexp(1.0, -e), o == (float)(1.0 + ldexp(1.0, -e)) ? "exact" : "LOST");
    }
    printf("case: C = 1, one product 2^-e (block 0 scale)\n");
    for (int e = 1; e <= 30; e += 1) {
        memset(A, 0, sizeof(A));
        for (int i = 0; i < 64; ++i) S[i] = 127;
        A[0] = 0x38;
        S[0] = 127 - e;
        const float o = run(A, S, 1.0f);
        printf("  e=%2d  D=%.10g  exact=%.10g  %s\n", e, o, 1.0 + ldexp(1.0, -e), o == (float)(1.0 + ldexp(1.0, -e)) ? "exact" : "LOST");
    }
    printf("case: 1.0 + 64 products of 2^-e (blocks 1-2)\n");
    for (int e = 6; e <= 30; e += 2) {
        memset(A, 0, sizeof(A));
        for (int i = 0; i < 64; ++i) S[i] = 127;
        A[0] = 0x38;
        for (int k = 32; k < 96; ++k) A[k] = 0x38;
        S[1] = S[2] = 127 - e;
        const float o = run(A, S, 0.0f);
        const double ex = 1.0 + 64 * ldexp(1.0, -e);
        printf("  e=%2d  D=%.10g  exact=%.10g  err/2^-23=%.3g\n", e, o, ex, (o - ex) / ldexp(1.0, -23));
    }
    printf("case: 1.0 + 1.125 * 2^-e (3 significant bits)\n");
    for (int e = 10; e <= 26; ++e) {
        memset(A, 0, sizeof(A));
        for (int i = 0; i < 64; ++i) S[i] = 127;
        A[0] = 0x38;
        A[40] = 0x39;  // 1.125
        S[1] = 127 - e;
        const float o = run(A, S, 0.0f);
        const double ex = 1.0 + 1.125 * ldexp(1.0, -e);
        printf("  e=%2d  D=%.10g  exact=%.10g  err/2^-23=%.3g\n", e, o, ex, (o - (float)ex) / ldexp(1.0, -23));
    }
    printf("case: probes (k, value) pairs with per-block scales\n");
    struct Probe { int k0; double v0; int k1; double v1; int s0, s1, s2, s3; };
    const Probe probes[] = {
        {40, 1.0, -1, 0, 127, 127, 127, 127}, {40, 1.0, -1, 0, 127, 121, 127, 127}, {40, 1.0, -1, 0, 127, 127, 121, 127},
        {0, 1.0, 40, 1.0, 127, 127, 127, 127}, {0, 1.0, 40, 1.0, 127, 126, 127, 127}, {0, 1.0, 40, 1.0, 127, 121, 127, 127},
        {0, 1.0, 40, 1.0, 127, 120, 127, 127}, {0, 1.0, 40, 1.0, 127, 119, 127, 127}, {0, 1.0, 40, 1.0, 127, 118, 127, 127},
        {0, 1.0, 40, 1.0, 127, 117, 127, 127}, {0, 1.0, 100, 1.0, 127, 127, 127, 121}, {0, 1.0, 20, 1.0, 127, 121, 127, 127},
        {0, 1.0, 40, 1.0, 133, 127, 127, 127}, {0, 1.0, 40, 1.0, 127, 133, 127, 127}, {0, 256.0, 40, 1.0, 127, 127, 127, 127},
        {0, 256.0, 1, 1.0, 127, 127, 127, 127}, {0, 256.0, 1, 0.125, 127, 127, 127, 127},
    };
    for (const Probe &pr : probes) {
        memset(A, 0, sizeof(A));
        for (int i = 0; i < 64; ++i) S[i] = 127;
        S[0] = pr.s0; S[1] = pr.s1; S[2] = pr.s2; S[3] = pr.s3;
        A[pr.k0] = e4m3(pr.v0);
        if (pr.k1 >= 0) A[pr.k1] = e4m3(pr.v1);
        const float o = run(A, S, 0.0f);
        printf("  k%d=%g k%d=%g scales %d %d %d %d -> D=%.10g\n", pr.k0, pr.v0, pr.k1, pr.v1, pr.s0 - 127, pr.s1 - 127,
               pr.s2 - 127, pr.s3 - 127, o);
    }
    return 0;
}
