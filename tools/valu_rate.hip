// valu_rate.hip -- issue-rate microbenchmark of the VALU instructions the approx GEMM's inner
// loop is made of (gfx950).  Each lane runs 8 independent chains of one instruction in a loop;
// the grid fills every SIMD with `waves` waves.  Prints ns and the chip-wide rate in
// wave-instructions per SIMD per ns, relative to v_add_f32.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_rate tools/valu_rate.hip && tools/valu_rate
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHAINS8(INS)                                                                                  \
    asm volatile(INS : "+v"(r0) : "v"(s1), "v"(s2));                                                  \
    asm volatile(INS : "+v"(r1) : "v"(s1), "v"(s2));                                                  \
    asm volatile(INS : "+v"(r2) : "v"(s1), "v"(s2));                                                  \
    asm volatile(INS : "+v"(r3) : "v"(s1), "v"(s2));                                                  \
    asm volatile(INS : "+v"(r4) : "v"(s1), "v"(s2));                                                  \
    asm volatile(INS : "+v"(r5) : "v"(s1), "v"(s2));                                                  \
    asm volatile(INS : "+v"(r6) : "v"(s1), "v"(s2));                                                  \
    asm volatile(INS : "+v"(r7) : "v"(s1), "v"(s2));

#define KERNEL(NAME, INS)                                                                             \
    __global__ void NAME(float *out, int iters) {                                                     \
        float r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4, r5 = r0 + 5,      \
              r6 = r0 + 6, r7 = r0 + 7;                                                               \
        float s1 = 1.0001f, s2 = 0.5f + threadIdx.x;                                                  \
        for (int i = 0; i < iters; ++i) {                                                             \
            CHAINS8(INS) CHAINS8(INS)                                                                 \
        }                                                                                             \
        out[blockIdx.x * blockDim.x + threadIdx.x] = r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7;          \
    }

KERNEL(k_add_f32, "v_add_f32 %0, %0, %1")
KERNEL(k_sub_f32, "v_sub_f32 %0, %0, %1")
KERNEL(k_mul_f32, "v_mul_f32 %0, %0, %1")
KERNEL(k_fma_f32, "v_fma_f32 %0, %0, %1, %2")
KERNEL(k_fmac_f32, "v_fmac_f32 %0, %1, %2")
KERNEL(k_med3_f32, "v_med3_f32 %0, %0, %1, %2")
KERNEL(k_max_f32, "v_max_f32 %0, %0, %1")
KERNEL(k_min_f32, "v_min_f32 %0, %0, %1")
KERNEL(k_max3_f32, "v_max3_f32 %0, %0, %1, %2")
KERNEL(k_and_or, "v_and_or_b32 %0, %0, %1, %2")
KERNEL(k_bfe_i32, "v_bfe_i32 %0, %0, %1, 1")
KERNEL(k_bfe_u32, "v_bfe_u32 %0, %0, %1, 1")
KERNEL(k_bfi_b32, "v_bfi_b32 %0, %0, %1, %2")
KERNEL(k_perm_b32, "v_perm_b32 %0, %0, %1, %2")
KERNEL(k_lshl_or, "v_lshl_or_b32 %0, %0, %1, %2")
KERNEL(k_lshl_add, "v_lshl_add_u32 %0, %0, %1, %2")
KERNEL(k_add3_u32, "v_add3_u32 %0, %0, %1, %2")
KERNEL(k_add_u32, "v_add_u32 %0, %0, %1")
KERNEL(k_sub_u32, "v_sub_u32 %0, %0, %1")
KERNEL(k_sub_u32_clamp, "v_sub_u32_e64 %0, %0, %1 clamp")
KERNEL(k_add_u32_clamp, "v_add_u32_e64 %0, %0, %1 clamp")
KERNEL(k_max_u32, "v_max_u32 %0, %0, %1")
KERNEL(k_max_i32, "v_max_i32 %0, %0, %1")
KERNEL(k_min_u32, "v_min_u32 %0, %0, %1")
KERNEL(k_and_b32, "v_and_b32 %0, %0, %1")
KERNEL(k_or_b32, "v_or_b32 %0, %0, %1")
KERNEL(k_xor_b32, "v_xor_b32 %0, %0, %1")
KERNEL(k_lshlrev, "v_lshlrev_b32 %0, %1, %0")
KERNEL(k_lshrrev, "v_lshrrev_b32 %0, %1, %0")
KERNEL(k_ashrrev, "v_ashrrev_i32 %0, %1, %0")
KERNEL(k_cvt_f32_i32, "v_cvt_f32_i32 %0, %0")
KERNEL(k_cvt_f32_ubyte0, "v_cvt_f32_ubyte0 %0, %0")
KERNEL(k_ldexp, "v_ldexp_f32 %0, %0, %1")
KERNEL(k_mul_u24, "v_mul_u32_u24 %0, %0, %1")
KERNEL(k_mad_u24, "v_mad_u32_u24 %0, %0, %1, %2")
KERNEL(k_mul_lo, "v_mul_lo_u32 %0, %0, %1")
KERNEL(k_add_f32_e64, "v_add_f32_e64 %0, %0, %1")
KERNEL(k_mul_f32_abs, "v_mul_f32_e64 %0, |%0|, %1")
KERNEL(k_cmp_cnd, "v_cmp_gt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc")
KERNEL(k_cndmask_s, "v_cndmask_b32_e64 %0, %0, %1, s[0:1]")
KERNEL(k_fract, "v_fract_f32 %0, %0")
KERNEL(k_rndne, "v_rndne_f32 %0, %0")
KERNEL(k_frexp_exp, "v_frexp_exp_i32_f32 %0, %0")
KERNEL(k_pk_add_f16, "v_pk_add_f16 %0, %0, %1")
KERNEL(k_pk_mul_f16, "v_pk_mul_f16 %0, %0, %1")
KERNEL(k_pk_fma_f16, "v_pk_fma_f16 %0, %0, %1, %2")
KERNEL(k_pk_max_f16, "v_pk_max_f16 %0, %0, %1")
KERNEL(k_pk_max_u16, "v_pk_max_u16 %0, %0, %1")
KERNEL(k_pk_add_u16, "v_pk_add_u16 %0, %0, %1")
KERNEL(k_pk_sub_f16, "v_pk_add_f16 %0, %0, %1 neg_lo:[0,1] neg_hi:[0,1]")

#define PCHAINS8(INS)                                                                                 \
    asm volatile(INS : "+v"(r0) : "v"(s1), "v"(s2));                                                  \
    asm volatile(INS : "+v"(r1) : "v"(s1), "v"(s2));                                                  \
    asm volatile(INS : "+v"(r2) : "v"(s1), "v"(s2));                                                  \
    asm volatile(INS : "+v"(r3) : "v"(s1), "v"(s2));                                                  \
    asm volatile(INS : "+v"(r4) : "v"(s1), "v"(s2));                                                  \
    asm volatile(INS : "+v"(r5) : "v"(s1), "v"(s2));                                                  \
    asm volatile(INS : "+v"(r6) : "v"(s1), "v"(s2));                                                  \
    asm volatile(INS : "+v"(r7) : "v"(s1), "v"(s2));
typedef float f2 __attribute__((ext_vector_type(2)));
#define PKERNEL(NAME, INS)                                                                            \
    __global__ void NAME(float *out, int iters) {                                                     \
        f2 r0 = {(float)threadIdx.x, 1.f}, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4,        \
           r5 = r0 + 5, r6 = r0 + 6, r7 = r0 + 7;                                                     \
        f2 s1 = {1.0001f, 1.0f}, s2 = {0.5f, 0.25f};                                                  \
        for (int i = 0; i < iters; ++i) {                                                             \
            PCHAINS8(INS) PCHAINS8(INS)                                                               \
        }                                                                                             \
        f2 t = r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7;                                                 \
        out[blockIdx.x * blockDim.x + threadIdx.x] = t.x + t.y;                                       \
    }
PKERNEL(k_pk_add_f32, "v_pk_add_f32 %0, %0, %1")
PKERNEL(k_pk_mul_f32, "v_pk_mul_f32 %0, %0, %1")
PKERNEL(k_pk_fma_f32, "v_pk_fma_f32 %0, %0, %1, %2")

typedef void (*kfn)(float *, int);

int main() {
    struct {
        const char *name;
        kfn f;
    } ks[] = {{"add_f32", k_add_f32}, {"sub_f32", k_sub_f32}, {"mul_f32", k_mul_f32}, {"fma_f32", k_fma_f32}, {"fmac_f32", k_fmac_f32}, {"med3_f32", k_med3_f32}, {"max_f32", k_max_f32}, {"min_f32", k_min_f32}, {"max3_f32", k_max3_f32}, {"and_or", k_and_or}, {"bfe_i32", k_bfe_i32}, {"bfe_u32", k_bfe_u32}, {"bfi_b32", k_bfi_b32}, {"perm_b32", k_perm_b32}, {"lshl_or", k_lshl_or}, {"lshl_add", k_lshl_add}, {"add3_u32", k_add3_u32}, {"add_u32", k_add_u32}, {"sub_u32", k_sub_u32}, {"sub_u32_clamp", k_sub_u32_clamp}, {"add_u32_clamp", k_add_u32_clamp}, {"max_u32", k_max_u32}, {"max_i32", k_max_i32}, {"min_u32", k_min_u32}, {"and_b32", k_and_b32}, {"or_b32", k_or_b32}, {"xor_b32", k_xor_b32}, {"lshlrev", k_lshlrev}, {"lshrrev", k_lshrrev}, {"ashrrev", k_ashrrev}, {"cvt_f32_i32", k_cvt_f32_i32}, {"cvt_f32_ubyte0", k_cvt_f32_ubyte0}, {"ldexp", k_ldexp}, {"mul_u24", k_mul_u24}, {"mad_u24", k_mad_u24}, {"mul_lo", k_mul_lo}, {"add_f32_e64", k_add_f32_e64}, {"mul_f32_abs", k_mul_f32_abs}, {"cmp_cnd", k_cmp_cnd}, {"cndmask_s", k_cndmask_s}, {"fract", k_fract}, {"rndne", k_rndne}, {"frexp_exp", k_frexp_exp}, {"pk_add_f16", k_pk_add_f16}, {"pk_mul_f16", k_pk_mul_f16}, {"pk_fma_f16", k_pk_fma_f16}, {"pk_max_f16", k_pk_max_f16}, {"pk_max_u16", k_pk_max_u16}, {"pk_add_u16", k_pk_add_u16}, {"pk_sub_f16", k_pk_sub_f16}, {"pk_add_f32", k_pk_add_f32}, {"pk_mul_f32", k_pk_mul_f32}, {"pk_fma_f32", k_pk_fma_f32}};
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    const int iters = 4096;
    float *out;
    hipMalloc(&out, sizeof(float) * 1024 * 1024 * 8);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    printf("CUs %d clock %d kHz\n", cus, prop.clockRate);
    for (int waves = 4; waves <= 8; waves *= 2) {
        const int blocks = cus * waves;  // 256-thread blocks: one wave per SIMD each
        double base = 0;
        for (auto &k : ks) {
            k.f<<<blocks, 256>>>(out, 16);
            hipEventRecord(a);
            k.f<<<blocks, 256>>>(out, iters);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            const double winstr = (double)blocks * 4 * iters * 16;        // wave-instructions
            const double per_simd_ns = winstr / (cus * 4) / (ms * 1e6);   // per SIMD per ns
            if (base == 0) base = per_simd_ns;
            printf("waves/SIMD %d  %-22s %8.3f ms  %.3f winstr/SIMD/ns  rel %.2f\n", waves, k.name, ms, per_simd_ns,
                   per_simd_ns / base);
        }
    }
    hipFree(out);
    return 0;
}
