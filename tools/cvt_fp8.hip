// cvt_fp8.hip -- gfx950 fp8 (OCP e4m3) conversion instructions as a Q_R candidate: issue rate
// (relative to v_add_f32) and semantics (rounding, carry, subnormal floor, overflow, scale).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/cvt_fp8 tools/cvt_fp8.hip && tools/cvt_fp8
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>

typedef float f2 __attribute__((ext_vector_type(2)));

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

__global__ void k_add(float *out, int iters) {
    float r[8];
    for (int c = 0; c < 8; ++c) r[c] = threadIdx.x + c;
    float s = 1.0001f;
    for (int i = 0; i < iters; ++i) {
#define A(c) asm volatile("v_add_f32 %0, %0, %1" : "+v"(r[c]) : "v"(s));
        REP8(A) REP8(A)
    }
    float t = 0;
    for (int c = 0; c < 8; ++c) t += r[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

// f32 pair -> packed fp8 (dependent: the result feeds the next input via bit reinterpretation)
__global__ void k_to_fp8(float *out, int iters) {
    unsigned r[8];
    for (int c = 0; c < 8; ++c) r[c] = threadIdx.x + c;
    float s = 1.0001f;
    for (int i = 0; i < iters; ++i) {
#define B(c) asm volatile("v_cvt_pk_fp8_f32 %0, %0, %1" : "+v"(r[c]) : "v"(s));
        REP8(B) REP8(B)
    }
    unsigned t = 0;
    for (int c = 0; c < 8; ++c) t += r[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

__global__ void k_from_fp8(float *out, int iters) {
    f2 r[8];
    unsigned x[8];
    for (int c = 0; c < 8; ++c) x[c] = threadIdx.x * 77 + c;
    for (int i = 0; i < iters; ++i) {
#define C(c) asm volatile("v_cvt_pk_f32_fp8 %0, %1" : "=v"(r[c]) : "v"(x[c])); x[c] ^= __float_as_uint(r[c].x);
        REP8(C) REP8(C)
    }
    float t = 0;
    for (int c = 0; c < 8; ++c) t += r[c].x + r[c].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

__global__ void k_from_fp8_only(float *out, int iters) {
    f2 r[8];
    unsigned x = threadIdx.x * 77;
    for (int i = 0; i < iters; ++i) {
#define D(c) asm volatile("v_cvt_pk_f32_fp8 %0, %1" : "=v"(r[c]) : "v"(x));
        REP8(D) REP8(D)
        x += 1;
    }
    float t = 0;
    for (int c = 0; c < 8; ++c) t += r[c].x + r[c].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

__global__ void k_to_fp8_scaled(float *out, int iters, float sc) {
    unsigned r[8];
    for (int c = 0; c < 8; ++c) r[c] = threadIdx.x + c;
    float s = 1.0001f;
    for (int i = 0; i < iters; ++i) {
#define E(c) asm volatile("v_cvt_scalef32_pk_fp8_f32 %0, %0, %1, %2" : "+v"(r[c]) : "v"(s), "s"(sc));
        REP8(E) REP8(E)
    }
    unsigned t = 0;
    for (int c = 0; c < 8; ++c) t += r[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

__global__ void k_from_fp8_scaled(float *out, int iters, float sc) {
    f2 r[8];
    unsigned x = threadIdx.x * 77;
    for (int i = 0; i < iters; ++i) {
#define F(c) asm volatile("v_cvt_scalef32_pk_f32_fp8 %0, %1, %2" : "=v"(r[c]) : "v"(x), "s"(sc));
        REP8(F) REP8(F)
        x += 1;
    }
    float t = 0;
    for (int c = 0; c < 8; ++c) t += r[c].x + r[c].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

// semantics: round trip of each input through the plain and the scaled conversions
__global__ void k_sem(const float *x, float *y, int n, float sc) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int p = __builtin_amdgcn_cvt_pk_fp8_f32(x[i], 0.0f, 0, false);
    const f2 r = __builtin_amdgcn_cvt_pk_f32_fp8(p, false);
    y[4 * i] = r[0];
    y[4 * i + 1] = __uint_as_float((unsigned)p & 0xFF);
    auto q = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32((__attribute__((ext_vector_type(2))) short){0, 0}, x[i], 0.0f,
                                                       sc, false);
    const unsigned qb = (unsigned)__builtin_bit_cast(int, q);
    const auto s2 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(qb, sc, false);
    y[4 * i + 2] = s2[0];
    y[4 * i + 3] = __uint_as_float(qb & 0xFF);
}

typedef void (*kfn)(float *, int);

int main() {
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount, iters = 4096;
    float *out;
    hipMalloc(&out, sizeof(float) * 1024 * 1024 * 8);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    struct {
        const char *name;
        int kind;
    } ks[] = {{"add_f32", 0}, {"cvt_pk_fp8_f32", 1}, {"cvt_pk_f32_fp8 (+xor)", 2}, {"cvt_pk_f32_fp8", 3},
              {"cvt_scalef32_pk_fp8_f32", 4}, {"cvt_scalef32_pk_f32_fp8", 5}};
    for (int waves = 4; waves <= 8; waves *= 2) {
        const int blocks = cus * waves;
        double base = 0;
        for (auto &k : ks) {
            for (int rep = 0; rep < 2; ++rep) {
                const int it = rep ? iters : 16;
                if (rep) hipEventRecord(a);
                switch (k.kind) {
                    case 0: k_add<<<blocks, 256>>>(out, it); break;
                    case 1: k_to_fp8<<<blocks, 256>>>(out, it); break;
                    case 2: k_from_fp8<<<blocks, 256>>>(out, it); break;
                    case 3: k_from_fp8_only<<<blocks, 256>>>(out, it); break;
                    case 4: k_to_fp8_scaled<<<blocks, 256>>>(out, it, 0.25f); break;
                    case 5: k_from_fp8_scaled<<<blocks, 256>>>(out, it, 0.25f); break;
                }
                if (rep) hipEventRecord(b);
            }
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            const double winstr = (double)blocks * 4 * iters * 16;
            const double per = winstr / (cus * 4) / (ms * 1e6);
            if (base == 0) base = per;
            printf("waves/SIMD %d  %-26s %8.3f ms  %.3f winstr/SIMD/ns  rel %.2f\n", waves, k.name, ms, per,
                   per / base);
        }
    }
    // semantics
    const float xs[] = {1.0f, 1.0625f, 1.125f, 1.1875f, 1.9375f, 1.96875f, 1.90625f, 1.875f, 3.875f, 3.9375f,
                        448.0f, 456.0f, 464.0f, 480.0f, 500.0f, 1000.0f, 1e30f, INFINITY, -INFINITY, NAN,
                        0.015625f, 0.0078125f, 0.001953125f, 0.0009765625f, 0.00146484375f, 0.0029296875f,
                        0.00048828125f, 0.0f, -0.0f, -1.9375f, -0.0009765625f, 0.017578125f, 0.01708984375f};
    const int n = sizeof(xs) / sizeof(float);
    float *dx, *dy;
    hipMalloc(&dx, sizeof(xs));
    hipMalloc(&dy, 4 * sizeof(xs));
    hipMemcpy(dx, xs, sizeof(xs), hipMemcpyHostToDevice);
    const float scales[] = {1.0f, 0.25f, 4.0f, 1.5f};
    for (float sc : scales) {
        k_sem<<<1, 64>>>(dx, dy, n, sc);
        float y[4 * 64];
        hipMemcpy(y, dy, 4 * sizeof(xs), hipMemcpyDeviceToHost);
        printf("scale %g\n", sc);
        for (int i = 0; i < n; ++i) {
            unsigned c0, c1;
            memcpy(&c0, &y[4 * i + 1], 4);
            memcpy(&c1, &y[4 * i + 3], 4);
            printf("  x % .9g  plain % .9g (0x%02x)  scaled % .9g (0x%02x)\n", xs[i], y[4 * i], c0, y[4 * i + 2], c1);
        }
    }
    hipFree(out);
    return 0;
}
