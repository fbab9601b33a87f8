// q_variants.hip -- throughput of candidate per-product instruction sequences of the approx GEMM
// inner loop (gfx950), each as the compiler schedules it: one dependent chain per product,
// 16 products per iteration, `waves` waves per SIMD.  Prints ns per product per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o tools/q_variants tools/q_variants.hip && tools/q_variants
#include <hip/hip_runtime.h>

#include <cstdio>

// operands: a, b (products), acc; constants in registers
#define OLD_Q                                                                                         \
    "v_mul_f32 %[x], %[a], %[b]\n"                                                                    \
    "v_and_b32 %[t], 0x7f800000, %[x]\n"                                                              \
    "v_mul_f32 %[u], %[t], %[kb]\n"                                                                   \
    "v_med3_f32 %[x], %[x], -%[u], %[u]\n"                                                            \
    "v_mul_f32 %[u], %[t], %[kc]\n"                                                                   \
    "v_max_f32 %[u], %[u], %[cmin]\n"                                                                 \
    "v_add_f32 %[x], %[x], %[u]\n"                                                                    \
    "v_sub_f32 %[x], %[x], %[u]\n"                                                                    \
    "v_add_f32 %[acc], %[acc], %[x]\n"
#define NEW_Q                                                                                         \
    "v_mul_f32 %[x], %[a], %[b]\n"                                                                    \
    "v_and_or_b32 %[u], %[x], %[sexp], %[kbm]\n"                                                      \
    "v_med3_f32 %[x], %[x], -%[u], %[u]\n"                                                            \
    "v_add_u32 %[u], %[sdc], %[u]\n"                                                                  \
    "v_max_u32 %[u], %[u], %[cminb]\n"                                                                \
    "v_add_f32 %[x], %[x], %[u]\n"                                                                    \
    "v_sub_f32 %[x], %[x], %[u]\n"                                                                    \
    "v_add_f32 %[acc], %[acc], %[x]\n"
#define SAT_Q                                                                                         \
    "v_mul_f32 %[x], %[a], %[b]\n"                                                                    \
    "v_and_b32 %[t], 0x7f800000, %[x]\n"                                                              \
    "v_or_b32 %[u], %[t], %[kbm]\n"                                                                   \
    "v_med3_f32 %[x], %[x], -%[u], %[u]\n"                                                            \
    "v_sub_u32_e64 %[u], %[u], %[sbdmin] clamp\n"                                                     \
    "v_add_u32 %[u], %[sdc], %[u]\n"                                                                  \
    "v_add_f32 %[x], %[x], %[u]\n"                                                                    \
    "v_sub_f32 %[x], %[x], %[u]\n"                                                                    \
    "v_add_f32 %[acc], %[acc], %[x]\n"
#define SATM_Q                                                                                        \
    "v_mul_f32 %[x], %[a], %[b]\n"                                                                    \
    "v_and_b32 %[t], 0x7f800000, %[x]\n"                                                              \
    "v_mul_f32 %[u], %[t], %[kb]\n"                                                                   \
    "v_med3_f32 %[x], %[x], -%[u], %[u]\n"                                                            \
    "v_sub_u32_e64 %[u], %[u], %[sbdmin] clamp\n"                                                     \
    "v_add_u32 %[u], %[sdc], %[u]\n"                                                                  \
    "v_add_f32 %[x], %[x], %[u]\n"                                                                    \
    "v_sub_f32 %[x], %[x], %[u]\n"                                                                    \
    "v_add_f32 %[acc], %[acc], %[x]\n"
#define W1U_T                                                                                         \
    "v_mul_f32 %[t], %[a], %[b]\n"                                                                    \
    "v_bfe_i32 %[u], %[row], %[mb], 1\n"                                                              \
    "v_and_b32 %[u], %[t], %[u]\n"                                                                    \
    "v_fma_f32 %[x], %[a], %[b], -%[u]\n"
#define W1U_T2 /* shift-right + and + sub-from-zero mask */                                           \
    "v_mul_f32 %[t], %[a], %[b]\n"                                                                    \
    "v_lshrrev_b32 %[u], %[mb], %[row]\n"                                                             \
    "v_and_b32 %[u], 1, %[u]\n"                                                                       \
    "v_sub_u32 %[u], 0, %[u]\n"                                                                       \
    "v_and_b32 %[u], %[t], %[u]\n"                                                                    \
    "v_fma_f32 %[x], %[a], %[b], -%[u]\n"
#define QTAIL_SAT                                                                                     \
    "v_and_b32 %[t], 0x7f800000, %[x]\n"                                                              \
    "v_or_b32 %[u], %[t], %[kbm]\n"                                                                   \
    "v_med3_f32 %[x], %[x], -%[u], %[u]\n"                                                            \
    "v_sub_u32_e64 %[u], %[u], %[sbdmin] clamp\n"                                                     \
    "v_add_u32 %[u], %[sdc], %[u]\n"                                                                  \
    "v_add_f32 %[x], %[x], %[u]\n"                                                                    \
    "v_sub_f32 %[x], %[x], %[u]\n"                                                                    \
    "v_add_f32 %[acc], %[acc], %[x]\n"
#define QTAIL_NEW                                                                                     \
    "v_and_or_b32 %[u], %[x], %[sexp], %[kbm]\n"                                                      \
    "v_med3_f32 %[x], %[x], -%[u], %[u]\n"                                                            \
    "v_add_u32 %[u], %[sdc], %[u]\n"                                                                  \
    "v_max_u32 %[u], %[u], %[cminb]\n"                                                                \
    "v_add_f32 %[x], %[x], %[u]\n"                                                                    \
    "v_sub_f32 %[x], %[x], %[u]\n"                                                                    \
    "v_add_f32 %[acc], %[acc], %[x]\n"
#define QTAIL_OLD                                                                                     \
    "v_and_b32 %[t], 0x7f800000, %[x]\n"                                                              \
    "v_mul_f32 %[u], %[t], %[kb]\n"                                                                   \
    "v_med3_f32 %[x], %[x], -%[u], %[u]\n"                                                            \
    "v_mul_f32 %[u], %[t], %[kc]\n"                                                                   \
    "v_max_f32 %[u], %[u], %[cmin]\n"                                                                 \
    "v_add_f32 %[x], %[x], %[u]\n"                                                                    \
    "v_sub_f32 %[x], %[x], %[u]\n"                                                                    \
    "v_add_f32 %[acc], %[acc], %[x]\n"

#define BODY(SEQ, J)                                                                                  \
    asm volatile(SEQ                                                                                  \
                 : [x] "=&v"(x), [t] "=&v"(t), [u] "=&v"(u), [acc] "+v"(acc[J])                      \
                 : [a] "v"(av[J & 3]), [b] "v"(bv[J >> 2]), [kb] "v"(kb), [kc] "v"(kc), [cmin] "v"(cmin), \
                   [kbm] "v"(kbm), [sexp] "s"(sexp), [sdc] "s"(sdc), [cminb] "v"(cminb),                  \
                   [sbdmin] "s"(sbdmin), [row] "v"(row[J & 3]), [mb] "v"(mb[J >> 2]));

#define KER(NAME, SEQ)                                                                                \
    __global__ void NAME(float *out, int iters, float k0) {                                           \
        float acc[16];                                                                                \
        for (int j = 0; j < 16; ++j) acc[j] = 0;                                                      \
        float av[4], bv[4];                                                                           \
        unsigned row[4], mb[4];                                                                       \
        for (int j = 0; j < 4; ++j) {                                                                 \
            av[j] = k0 * (1 + j + threadIdx.x % 7);                                                   \
            bv[j] = k0 * (3 - j);                                                                     \
            row[j] = 0x5a5a5a5a >> j;                                                                 \
            mb[j] = (threadIdx.x + j) & 7;                                                            \
        }                                                                                             \
        const float kb = 1.87f * k0, kc = 1048576.0f * k0, cmin = 3e-5f * k0;                         \
        const unsigned kbm = 0x700000u, sexp = 0x7f800000u, sdc = 0x0a000000u, cminb = 0x30000000u,    \
                       sbdmin = 0x30700000u;                                                          \
        float x, t, u;                                                                                \
        for (int i = 0; i < iters; ++i) {                                                             \
            BODY(SEQ, 0) BODY(SEQ, 1) BODY(SEQ, 2) BODY(SEQ, 3) BODY(SEQ, 4) BODY(SEQ, 5)            \
            BODY(SEQ, 6) BODY(SEQ, 7) BODY(SEQ, 8) BODY(SEQ, 9) BODY(SEQ, 10) BODY(SEQ, 11)          \
            BODY(SEQ, 12) BODY(SEQ, 13) BODY(SEQ, 14) BODY(SEQ, 15)                                  \
        }                                                                                             \
        float s = 0;                                                                                  \
        for (int j = 0; j < 16; ++j) s += acc[j];                                                     \
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                               \
    }

KER(k_none_old, OLD_Q)
KER(k_none_new, NEW_Q)
KER(k_none_sat, SAT_Q)
KER(k_none_satm, SATM_Q)
KER(k_w1u_old, W1U_T QTAIL_OLD)
KER(k_w1u_new, W1U_T QTAIL_NEW)
KER(k_w1u_sat, W1U_T QTAIL_SAT)
KER(k_w1u_t2sat, W1U_T2 QTAIL_SAT)

typedef void (*kfn)(float *, int, float);

int main() {
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount, iters = 2048;
    float *out;
    (void)hipMalloc(&out, sizeof(float) * 1024 * 1024 * 8);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    struct {
        const char *n;
        int ops;
        kfn f;
    } ks[] = {{"none old (9)", 9, k_none_old},   {"none new (8)", 8, k_none_new},  {"none sat (9)", 9, k_none_sat},
              {"none satm (9)", 9, k_none_satm}, {"w1u old (12)", 12, k_w1u_old},  {"w1u new (11)", 11, k_w1u_new},
              {"w1u sat (12)", 12, k_w1u_sat},   {"w1u t2sat (14)", 14, k_w1u_t2sat}};
    for (int rep = 0; rep < 2; ++rep)
        for (int waves = 4; waves <= 8; waves *= 2)
            for (auto &k : ks) {
                k.f<<<cus * waves, 256>>>(out, 16, 1.0f);
                (void)hipEventRecord(a);
                k.f<<<cus * waves, 256>>>(out, iters, 1.0f);
                (void)hipEventRecord(b);
                (void)hipEventSynchronize(b);
                float ms;
                (void)hipEventElapsedTime(&ms, a, b);
                const double prods = (double)cus * waves * 4 * iters * 16 * 64;  // lane-products
                printf("waves/SIMD %d  %-16s %.3f ms  %.3f Tprod/s  %.3f winstr/SIMD/ns\n", waves, k.n, ms,
                       prods / (ms * 1e9), prods / 64 * k.ops / (cus * 4) / (ms * 1e6));
            }
    return 0;
}
