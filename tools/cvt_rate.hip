// cvt_rate.hip -- issue cost (shader cycles per wave-instruction per SIMD) of the gfx950
// conversion / packed instructions the E4M3 kernel could round its terms with, measured
// in-kernel with s_memtime at 4 and 8 waves per SIMD (independent 8-register chains).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/cvt_rate tools/cvt_rate.hip && tools/cvt_rate
#include <hip/hip_runtime.h>

#include <cstdio>

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int KIND>
__global__ void k_rate(unsigned long long *cyc, unsigned *out, int iters, float sc) {
    unsigned r[8];
    for (int c = 0; c < 8; ++c) r[c] = threadIdx.x * 7 + c;
    const unsigned x = threadIdx.x * 3 + 0x3c003c00u;
    const float f = 1.0001f;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#define K0(c) asm volatile("v_add_f32 %0, %0, %1" : "+v"(r[c]) : "v"(f));
#define K1(c) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(r[c]) : "v"(f));
#define K2(c) asm volatile("v_cvt_scalef32_pk_fp8_f32 %0, %1, %2, %3" : "+v"(r[c]) : "v"(f), "v"(x), "v"(sc));
#define K3(c) asm volatile("v_cvt_scalef32_pk_fp8_f16 %0, %1, %2" : "+v"(r[c]) : "v"(x), "v"(sc));
#define K4(c) asm volatile("v_cvt_scalef32_pk_fp8_bf16 %0, %1, %2" : "+v"(r[c]) : "v"(x), "v"(sc));
#define K5(c) asm volatile("v_pk_mul_f16 %0, %0, %1" : "+v"(r[c]) : "v"(x));
#define K6(c) asm volatile("v_cvt_pk_fp8_f32 %0, %1, %2" : "+v"(r[c]) : "v"(f), "v"(x));
#define K7(c) asm volatile("v_cvt_scalef32_pk_fp4_f32 %0, %1, %2, %3" : "+v"(r[c]) : "v"(f), "v"(x), "v"(sc));
#define K8(c) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r[c]) : "v"(x));
#define K9(c) asm volatile("v_pk_add_f16 %0, %0, %1" : "+v"(r[c]) : "v"(x));
#define K10(c) asm volatile("v_cvt_f32_f16 %0, %1" : "=v"(r[c]) : "v"(r[c]));
#define K11(c) asm volatile("v_cvt_pk_f32_fp8 %0, %1" : "=v"(*(double *)&r[c & 6]) : "v"(r[c]));
        if (KIND == 0) { REP8(K0) REP8(K0) }
        if (KIND == 1) { REP8(K1) REP8(K1) }
        if (KIND == 2) { REP8(K2) REP8(K2) }
        if (KIND == 3) { REP8(K3) REP8(K3) }
        if (KIND == 4) { REP8(K4) REP8(K4) }
        if (KIND == 5) { REP8(K5) REP8(K5) }
        if (KIND == 6) { REP8(K6) REP8(K6) }
        if (KIND == 7) { REP8(K7) REP8(K7) }
        if (KIND == 8) { REP8(K8) REP8(K8) }
        if (KIND == 9) { REP8(K9) REP8(K9) }
        if (KIND == 10) { REP8(K10) REP8(K10) }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned t = 0;
    for (int c = 0; c < 8; ++c) t += r[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = t;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

typedef void (*kfn)(unsigned long long *, unsigned *, int, float);

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int iters = 2048;
    unsigned *out;
    unsigned long long *cyc;
    hipMalloc(&out, sizeof(unsigned) * 256 * 4096);
    hipMalloc(&cyc, sizeof(unsigned long long) * 4096);
    const char *names[] = {"v_add_f32", "v_mul_f32", "cvt_scalef32_pk_fp8_f32", "cvt_scalef32_pk_fp8_f16",
                           "cvt_scalef32_pk_fp8_bf16", "v_pk_mul_f16", "v_cvt_pk_fp8_f32", "cvt_scalef32_pk_fp4_f32",
                           "v_add_u32", "v_pk_add_f16", "v_cvt_f32_f16"};
    kfn fns[] = {k_rate<0>, k_rate<1>, k_rate<2>, k_rate<3>, k_rate<4>, k_rate<5>, k_rate<6>, k_rate<7>, k_rate<8>,
                 k_rate<9>, k_rate<10>};
    for (int waves = 4; waves <= 8; waves *= 2) {
        const int blocks = cus * waves;  // 256-thread blocks: one wave per SIMD each
        for (int f = 0; f < 11; ++f) {
            fns[f]<<<blocks, 256>>>(cyc, out, 16, 1.0f);
            hipEvent_t a, b;
            hipEventCreate(&a);
            hipEventCreate(&b);
            hipEventRecord(a);
            fns[f]<<<blocks, 256>>>(cyc, out, iters, 1.0f);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            unsigned long long h[4096];
            hipMemcpy(h, cyc, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
            double avg = 0;
            for (int i = 0; i < blocks; ++i) avg += (double)h[i];
            avg /= blocks;
            // s_memtime ticks at the shader clock on gfx950 (MI355X_MICROARCH.md); waves per SIMD
            // share the issue: cycles per wave-instruction per SIMD = ticks / (instr per wave * waves)
            const double per = avg / ((double)iters * 16 * waves);
            printf("waves/SIMD %d  %-26s %7.3f ms  %.2f cycles/winstr/SIMD  (%.2f GHz implied by wall)\n", waves,
                   names[f], ms, per, avg / (ms * 1e6));
        }
    }
    return 0;
}
