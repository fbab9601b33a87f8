// Accumulation of v_mfma_f32_16x16x32_bf16 and v_mfma_f32_16x16x32_fp8_fp8 (probe, not product):
// row 0 of A = 1.0 at k = 0 and 2^-e at k = j, B = ones; D[0][0] against 1 + 2^-e.
// hipcc --offload-arch=gfx950 -O2 -o tools/bin_mfma_bf16_precision tools/mfma_bf16_precision.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>

typedef short v8s __attribute__((ext_vector_type(8)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

__global__ void k_bf16(const unsigned short *A, float *out) {
    const int lane = threadIdx.x, r16 = lane & 15, g = lane >> 4;
    v8s a, b;
    for (int i = 0; i < 8; ++i) {
        a[i] = (short)A[r16 * 32 + 8 * g + i];  // lane (r16, g): K 8 g .. 8 g + 7
        b[i] = (short)0x3F80;                   // 1.0
    }
    v4f d = {0, 0, 0, 0};
    d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, a), __builtin_bit_cast(v8bf, b), d, 0, 0, 0);
    if (lane == 0) out[0] = d[0];
}

__global__ void k_fp8(const unsigned char *A, float *out) {
    const int lane = threadIdx.x, r16 = lane & 15, g = lane >> 4;
    long a = 0;
    for (int i = 0; i < 8; ++i) a |= (long)A[r16 * 32 + 8 * g + i] << (8 * i);
    const long b = 0x3838383838383838l;
    v4f d = {0, 0, 0, 0};
    d = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a, b, d, 0, 0, 0);
    if (lane == 0) out[0] = d[0];
}

static unsigned short bf16(double v) {
    float f = (float)v;
    unsigned u;
    memcpy(&u, &f, 4);
    return (unsigned short)(u >> 16);
}

int main() {
    unsigned short *dA;
    unsigned char *dA8;
    float *dO;
    hipMalloc(&dA, 16 * 32 * 2);
    hipMalloc(&dA8, 16 * 32);
    hipMalloc(&dO, 4);
    unsigned short A[16 * 32];
    printf("bf16: 1 + 2^-e at k = j\n");
    for (int j : {1, 8, 16, 31}) {
        for (int e = 8; e <= 26; e += 2) {
            memset(A, 0, sizeof(A));
            A[0] = bf16(1.0);
            A[j] = bf16(ldexp(1.0, -e));
            hipMemcpy(dA, A, sizeof(A), hipMemcpyHostToDevice);
            k_bf16<<<1, 64>>>(dA, dO);
            float o;
            hipMemcpy(&o, dO, 4, hipMemcpyDeviceToHost);
            const double ex = 1.0 + ldexp(1.0, -e);
            printf("  j=%2d e=%2d D=%.10g exact=%.10g %s\n", j, e, o, ex, o == (float)ex ? "exact" : "LOST");
        }
    }
    printf("bf16: 2^40 + 1 + (-2^40) at k = 0, 1, 2\n");
    {
        memset(A, 0, sizeof(A));
        A[0] = bf16(ldexp(1.0, 40));
        A[1] = bf16(1.0);
        A[2] = bf16(-ldexp(1.0, 40));
        hipMemcpy(dA, A, sizeof(A), hipMemcpyHostToDevice);
        k_bf16<<<1, 64>>>(dA, dO);
        float o;
        hipMemcpy(&o, dO, 4, hipMemcpyDeviceToHost);
        printf("  D=%.10g (exact 1)\n", o);
    }
    unsigned char A8[16 * 32];
    printf("fp8 (non-scaled): 1 + 2^-e at k = j\n");
    for (int j : {1, 2, 3, 4, 5, 6, 7, 8, 12, 16, 31}) {
        for (int e = 6; e <= 9; e += 3) {
            memset(A8, 0, sizeof(A8));
            A8[0] = 0x38;
            A8[j] = e <= 6 ? (unsigned char)((7 - e) << 3) : (unsigned char)(1 << (9 - e));  // 2^-e
            hipMemcpy(dA8, A8, sizeof(A8), hipMemcpyHostToDevice);
            k_fp8<<<1, 64>>>(dA8, dO);
            float o;
            hipMemcpy(&o, dO, 4, hipMemcpyDeviceToHost);
            const double ex = 1.0 + ldexp(1.0, -e);
            printf("  j=%2d e=%2d D=%.10g exact=%.10g %s\n", j, e, o, ex, o == (float)ex ? "exact" : "LOST");
        }
        // 256 + 2^-9 (17 binades)
        memset(A8, 0, sizeof(A8));
        A8[0] = (unsigned char)(15 << 3);  // 256
        A8[j] = 1;                          // 2^-9
        hipMemcpy(dA8, A8, sizeof(A8), hipMemcpyHostToDevice);
        k_fp8<<<1, 64>>>(dA8, dO);
        float o;
        hipMemcpy(&o, dO, 4, hipMemcpyDeviceToHost);
        printf("  j=%2d 256 + 2^-9: D=%.10g exact=%.10g\n", j, o, 256.0 + ldexp(1.0, -9));
    }
    return 0;
}
