// valu_dep.hip -- VALU issue rate vs dependency-chain count per wave and waves per SIMD (gfx950).
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_dep tools/valu_dep.hip && tools/valu_dep
#include <hip/hip_runtime.h>

#include <cstdio>

template <int CH>
__global__ void k_chain(float *out, int iters) {
    float r[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) r[c] = threadIdx.x + c;
    const float s1 = 1.0001f;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 16 / CH; ++u)
#pragma unroll
            for (int c = 0; c < CH; ++c) asm volatile("v_add_f32 %0, %0, %1" : "+v"(r[c]) : "v"(s1));
    }
    float t = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) t += r[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

template <int CH>
__global__ void k_chain_mix(float *out, int iters) {  // F,F,H,F,F,H pattern (like Q_R)
    float r[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) r[c] = threadIdx.x + c;
    const float s1 = 1.0001f, s2 = 3.0f;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 16 / CH / 4; ++u)
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(r[c]) : "v"(s1));
                asm volatile("v_mul_f32 %0, %0, %1" : "+v"(r[c]) : "v"(s1));
                asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(r[c]) : "v"(s1), "v"(s2));
                asm volatile("v_sub_f32 %0, %0, %1" : "+v"(r[c]) : "v"(s1));
            }
    }
    float t = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) t += r[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

typedef void (*kfn)(float *, int);

int main() {
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount, iters = 4096;
    float *out;
    (void)hipMalloc(&out, sizeof(float) * 1024 * 1024 * 8);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    struct {
        const char *n;
        kfn f;
    } ks[] = {{"add x1 chain", k_chain<1>}, {"add x2", k_chain<2>},     {"add x4", k_chain<4>},
              {"add x8", k_chain<8>},       {"mix x1", k_chain_mix<1>}, {"mix x2", k_chain_mix<2>},
              {"mix x4", k_chain_mix<4>}};
    for (int waves = 2; waves <= 8; waves *= 2)
        for (auto &k : ks) {
            k.f<<<cus * waves, 256>>>(out, 16);
            (void)hipEventRecord(a);
            k.f<<<cus * waves, 256>>>(out, iters);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            const double w = (double)cus * waves * 4 * iters * 16 / (cus * 4) / (ms * 1e6);
            printf("waves/SIMD %d  %-14s %.3f winstr/SIMD/ns\n", waves, k.n, w);
        }
    return 0;
}
