// Denormal bf16 inputs of v_mfma_f32_16x16x32_bf16 (probe, not product): does the matrix core keep
// bf16 operands with exponent field 0 (value m / 128 x 2^-126), scaled up by a 2^s B operand, or
// flush them?  (The v5 matrix-core design puts an E5M2 code r as bf16 bits r << 5: the grid's
// subnormal band lands on bf16 denormals.)  Each case: row 0 of A as listed, B = 2^s everywhere,
// D[0][0] against the exact double sum.
// hipcc --offload-arch=gfx950 -O2 -o tools/bin_mfma_bf16_denorm tools/mfma_bf16_denorm.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>

typedef short v8s __attribute__((ext_vector_type(8)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

__global__ void k_bf16(const unsigned short *A, unsigned short bsel, float *out) {
    const int lane = threadIdx.x, r16 = lane & 15, g = lane >> 4;
    v8s a, b;
    for (int i = 0; i < 8; ++i) {
        a[i] = (short)A[r16 * 32 + 8 * g + i];
        b[i] = (short)bsel;
    }
    v4f d = {0, 0, 0, 0};
    d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, a), __builtin_bit_cast(v8bf, b), d, 0, 0, 0);
    if (lane == 0) out[0] = d[0];
}

static double bf16_val(unsigned short h) {
    const int s = h >> 15, e = (h >> 7) & 0xFF, m = h & 0x7F;
    double v = e == 0 ? ldexp(m / 128.0, -126) : ldexp(1.0 + m / 128.0, e - 127);
    return s ? -v : v;
}

int main() {
    unsigned short *dA;
    float *dO;
    hipMalloc(&dA, 16 * 32 * 2);
    hipMalloc(&dO, 4);
    unsigned short A[16 * 32];
    struct Case { const char *name; int n; unsigned short v[32]; int s; };
    Case cases[] = {
        {"one denormal 0x0020, B 2^120", 1, {0x0020}, 120},
        {"denormals 0x0020 0x0040 0x0060, B 2^127", 3, {0x0020, 0x0040, 0x0060}, 127},
        {"negative denormal 0x8060 + normal 0x0080, B 2^127", 2, {0x8060, 0x0080}, 127},
        {"denormal 0x0001 (2^-133), B 2^127", 1, {0x0001}, 127},
        {"E5M2 codes r << 5, r = 0..31, B 2^110", 32, {}, 110},
        {"E5M2 codes r << 5, r = 96..127, B 2^110", 32, {}, 110},
    };
    for (int i = 0; i < 32; ++i) {
        cases[4].v[i] = (unsigned short)(i << 5);
        cases[5].v[i] = (unsigned short)((96 + i) << 5);
    }
    int bad = 0;
    for (const Case &c : cases) {
        memset(A, 0, sizeof(A));
        double ex = 0.0;
        for (int j = 0; j < c.n; ++j) {
            A[j] = c.v[j];
            ex += bf16_val(c.v[j]) * ldexp(1.0, c.s);
        }
        hipMemcpy(dA, A, sizeof(A), hipMemcpyHostToDevice);
        k_bf16<<<1, 64>>>(dA, (unsigned short)((127 + c.s) << 7), dO);
        float o;
        hipMemcpy(&o, dO, 4, hipMemcpyDeviceToHost);
        const bool ok = (double)o == (double)(float)ex;
        bad += !ok;
        printf("%-52s got %.9g expected %.9g %s\n", c.name, o, ex, ok ? "exact" : "DIFFERENT");
    }
    printf("%s\n", bad ? "denormal bf16 inputs are NOT kept" : "denormal bf16 inputs kept exactly");
    return 0;
}
