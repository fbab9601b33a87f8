// seg_bench.hip -- products per SIMD-cycle of gemm_f8mx_kernel's instruction stream, by parts
// (VERDICT r4 item 1).  One workgroup = 4 waves x the kernel's 128 x 64 tile mapping (lane = row of
// each of 8 16-row blocks x K-step pair); every wave loops over staged tiles of 8 K-steps doing
// exactly the kernel's math segment per (16-row block, A element): one v_and_or_b32, four
// ds_read_b64 of the c_b-applied table, eight v_cvt_scalef32_pk_fp8_bf16, and per block one
// v_mfma_scale_f32_16x16x128_f8f6f4 -- optionally with the per-tile table build (static-table
// reads, packed adds, ds_write_b128) and the two workgroup barriers, and the A-word staging write.
// Parts are switched off by template bits to attribute the time.  Clock: s_memtime around the loop
// (shader cycles), so results are cycles, independent of DVFS.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/bin/seg_bench tools/seg_bench.hip
//   tools/bin/seg_bench [tiles]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef short s2 __attribute__((ext_vector_type(2)));
typedef unsigned short u2 __attribute__((ext_vector_type(2)));
typedef __bf16 b2 __attribute__((ext_vector_type(2)));

constexpr int XBK = 8, TXN = 16, TTK = TXN * 32 + 16, BMT = 128, AWQ = 2 * BMT + 32, LUTW = 81 * 8, RB = 8;

struct Stage {
    uint32_t tt[XBK][TTK];
    uint32_t lut[LUTW];
    uint32_t aw[XBK / 2][AWQ];
};

enum { P_LDS = 1, P_CVT = 2, P_MFMA = 4, P_BUILD = 8, P_BAR = 16, P_STAGE = 32, P_GLOAD = 64 };

template <int P, int WAVES>
__global__ __launch_bounds__(256, WAVES) void seg(const uint32_t *seed, float *out, unsigned long long *cyc, int tiles,
                                                  const uint32_t *gbuf) {
    __shared__ __attribute__((aligned(16))) Stage sm;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    // fill LDS with plausible data: table words = random bf16 pairs near 1.0, A words = se << 23 | row << 3
    for (int e = tid; e < XBK * TTK; e += 256) (&sm.tt[0][0])[e] = 0x3F803F80u + ((seed[e & 1023] & 0x007F007Fu));
    for (int e = tid; e < LUTW; e += 256) sm.lut[e] = 0x3F803F80u + (seed[(e + 7) & 1023] & 0x007F007Fu);
    for (int e = tid; e < XBK / 2 * AWQ; e += 256)
        (&sm.aw[0][0])[e] = ((110u + (seed[(e + 3) & 1023] & 15u)) << 23) | ((seed[(e + 5) & 1023] & 15u) << 3);
    const uint4 wb = make_uint4(seed[tid & 1023] & 0x00FF00FFu, (seed[(tid + 1) & 1023] % 81) * 32u,
                                seed[(tid + 2) & 1023] & 0x00FF00FFu, (seed[(tid + 3) & 1023] % 81) * 32u);
    const int q4 = tid & 3, btx = (tid >> 3) % TXN;
    int bkk[2];
    for (int u = 0; u < 2; ++u) {
        const int e = tid + 256 * u;
        bkk[u] = 2 * (e / (8 * TXN)) + ((e >> 2) & 1);
    }
    v8i sel;
    {
        const int n = lane & 15;
        for (int v = 0; v < 8; ++v) {
            uint32_t w = 0;
            for (int b = 0; b < 4; ++b)
                if (((4 * v + b) & 15) == n) w |= 0x38u << (8 * b);
            sel[v] = (int)w;
        }
    }
    v4f dq[RB];
    for (int b = 0; b < RB; ++b) dq[b] = (v4f){0.0f, 0.0f, 0.0f, 0.0f};
    v8i av = {0, 0, 0, 0, 0, 0, 0, 0};
    const char *lut = reinterpret_cast<const char *>(sm.lut);
    const uint32_t wvo = (uint32_t)wv * 512u;
    typedef const volatile __attribute__((address_space(3))) uint64_t lds_u64;
    uint32_t stw = seed[tid & 1023];
    // P_GLOAD: the kernel's per-tile global traffic -- per thread 4 A words (b32, lane-consecutive
    // rows, a K-step's plane offset in the uniform soffset) and 2 B pair units (b128), one tile ahead
    const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(gbuf), (short)0, -1, 0x00020000);
    const uint32_t gA = (uint32_t)(blockIdx.x * 128 + lane) * 4u, gB = (uint32_t)(blockIdx.x * 256 + tid) * 16u;
    uint32_t ga[4] = {0, 0, 0, 0};
    uint4 gb[2] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
    auto gload = [&](int it) {
        const uint32_t ko = (uint32_t)((it * 8 + 2 * wv) & 1023) * 262144u;  // 1 MiB per K-step plane
        for (int i = 0; i < 4; ++i)
            ga[i] = __builtin_amdgcn_raw_buffer_load_b32(grs, (int)(gA + 256u * (i >> 1)), (int)(ko + 1048576u * (i & 1)), 0);
        for (int u = 0; u < 2; ++u)
            gb[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(grs, (int)(gB + 4096u * u), (int)(ko & 0x3FFFFFu), 0));
    };
    if (P & P_GLOAD) gload(0);
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < tiles; ++it) {
        if (P & P_STAGE) {
            stw = stw * 1664525u + 1013904223u;
            if (P & P_GLOAD) stw ^= ga[0] ^ ga[1] ^ ga[2] ^ ga[3] ^ gb[0].x ^ gb[1].y;
            *reinterpret_cast<uint2 *>(&sm.aw[wv][2 * lane]) = make_uint2((110u << 23) | (stw & 0x78u), (111u << 23) | ((stw >> 8) & 0x78u));
            *reinterpret_cast<uint2 *>(&sm.aw[wv][2 * (lane + 64)]) = make_uint2((112u << 23) | ((stw >> 4) & 0x78u), (110u << 23) | ((stw >> 12) & 0x78u));
        }
        if (P & P_BUILD) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const uint4 b = wb;
                const uint2 s0 = *reinterpret_cast<const uint2 *>(lut + b.y + 8 * q4);
                const uint2 s1 = *reinterpret_cast<const uint2 *>(lut + b.w + 8 * q4);
                const u2 a0 = __builtin_bit_cast(u2, b.x), a1 = __builtin_bit_cast(u2, b.z);
                const u2 n0 = __builtin_bit_cast(u2, b.x ^ 0x80008000u), n1 = __builtin_bit_cast(u2, b.z ^ 0x80008000u);
                auto pk = [](uint32_t v, u2 ad) { return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u2, v) + ad); };
                uint32_t *d = &sm.tt[bkk[u]][btx * 32 + q4 * 4];
                *reinterpret_cast<uint4 *>(d) = make_uint4(pk(s0.x, a0), pk(s1.x, a1), pk(s0.y, a0), pk(s1.y, a1));
                *reinterpret_cast<uint4 *>(d + 16) = make_uint4(pk(s0.x, n0), pk(s1.x, n1), pk(s0.y, n0), pk(s1.y, n1));
            }
        }
        if (P & P_BAR) __syncthreads();
        if ((P & P_GLOAD) && it + 1 < tiles) gload(it + 1);
        {
            const int r16 = lane & 15, g = lane >> 4;
            const uint32_t base = wvo + (uint32_t)(2 * g) * (uint32_t)(TTK * 4);
            const char *tt0 = reinterpret_cast<const char *>(&sm.tt[0][0]);
#pragma unroll
            for (int b = 0; b < RB; ++b) {
                const uint2 aw2 = *reinterpret_cast<const uint2 *>(&sm.aw[g][2 * (16 * b + r16)]);
                uint32_t awh[2] = {aw2.x, aw2.y};
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    uint32_t a;
                    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(a) : "v"(awh[h]), "s"(0x78u), "v"(base));
                    __builtin_assume((a & 7u) == 0u);
                    lds_u64 *ttk = (lds_u64 *)(tt0 + h * TTK * 4);
                    uint2 v[4];
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        if (P & P_LDS) {
                            const uint64_t w = ttk[(a >> 3) + 16 * c];
                            v[c] = make_uint2((uint32_t)w, (uint32_t)(w >> 32));
                        } else {
                            v[c] = make_uint2(a + c, a ^ (c << 9));
                        }
                    }
                    const float sc = __uint_as_float(awh[h]);
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        s2 cv;
                        if (P & P_CVT) {
                            asm("v_cvt_scalef32_pk_fp8_bf16 %0, %1, %2" : "=v"(cv) : "v"(v[c].x), "v"(sc));
                            cv = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(cv, __builtin_bit_cast(b2, v[c].y), sc, true);
                        } else {
                            cv = __builtin_bit_cast(s2, v[c].x ^ v[c].y);
                        }
                        av[4 * h + c] = __builtin_bit_cast(int, cv);
                    }
                }
                if (P & P_MFMA)
                    dq[b] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, sel, dq[b], 0, 0, 0, 127, 0, 127);
                else
                    dq[b][0] += __int_as_float(av[0] ^ av[1] ^ av[2] ^ av[3] ^ av[4] ^ av[5] ^ av[6] ^ av[7]);
            }
        }
        if (P & P_BAR) __syncthreads();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.0f;
    for (int b = 0; b < RB; ++b) s += dq[b][0] + dq[b][1] + dq[b][2] + dq[b][3];
    out[blockIdx.x * 256 + tid] = s;
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

typedef void (*kfn)(const uint32_t *, float *, unsigned long long *, int, const uint32_t *);

template <int P, int W>
static void run(const char *name, int cus, const uint32_t *seed, float *out, unsigned long long *cyc, int tiles,
                const uint32_t *gbuf) {
    const int blocks = cus * W;  // one workgroup = one wave per SIMD; W workgroups per CU
    kfn f = seg<P, W>;
    f<<<blocks, 256>>>(seed, out, cyc, 4, gbuf);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    f<<<blocks, 256>>>(seed, out, cyc, tiles, gbuf);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    static unsigned long long h[8192];
    hipMemcpy(h, cyc, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
    double avg = 0, mx = 0;
    for (int i = 0; i < blocks; ++i) {
        avg += (double)h[i];
        mx = mx > (double)h[i] ? mx : (double)h[i];
    }
    avg /= blocks;
    // products per wave per tile: 8 blocks x 2048 / 64 lanes x 64 = 8 x 2048
    const double prod_wave = (double)tiles * RB * 2048.0;
    // W waves share each SIMD for the whole loop (all resident at once)
    printf("%-34s waves/SIMD %d  %8.1f cyc/tile/wave  %6.2f products/SIMD-cycle  (%.3f ms, %.2f GHz by wall)\n", name,
           W, avg / tiles, prod_wave * W / avg, ms, mx / (ms * 1e6));
}

int main(int argc, char **argv) {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int tiles = argc > 1 ? atoi(argv[1]) : 400;
    uint32_t *seed;
    float *out;
    unsigned long long *cyc;
    hipMalloc(&seed, 4096);
    hipMalloc(&out, sizeof(float) * 256 * 8192);
    hipMalloc(&cyc, sizeof(unsigned long long) * 8192);
    uint32_t hs[1024];
    uint32_t x = 12345;
    for (int i = 0; i < 1024; ++i) hs[i] = (x = x * 1664525u + 1013904223u);
    hipMemcpy(seed, hs, 4096, hipMemcpyHostToDevice);
    uint32_t *gbuf;  // 1 GiB + margin of words for the global-load variants (L2 / MALL / HBM mix)
    hipMalloc(&gbuf, (1ull << 30) + (64ull << 20));
    hipMemset(gbuf, 0, (1ull << 30) + (64ull << 20));
    constexpr int ALL = P_LDS | P_CVT | P_MFMA | P_BUILD | P_BAR | P_STAGE;
    constexpr int ALLG = ALL | P_GLOAD;
    run<ALLG, 5>("full + global loads", cus, seed, out, cyc, tiles, gbuf);
    run<ALLG, 6>("full + global loads", cus, seed, out, cyc, tiles, gbuf);
    run<ALL, 5>("full (stage+build+bar+lds+cvt+mfma)", cus, seed, out, cyc, tiles, gbuf);
    run<ALL, 6>("full (stage+build+bar+lds+cvt+mfma)", cus, seed, out, cyc, tiles, gbuf);
    run<ALL, 4>("full", cus, seed, out, cyc, tiles, gbuf);
    run<ALL, 2>("full", cus, seed, out, cyc, tiles, gbuf);
    run<ALL & ~P_BAR, 6>("no barriers", cus, seed, out, cyc, tiles, gbuf);
    run<ALL & ~(P_BUILD | P_STAGE), 6>("no build/stage (bar kept)", cus, seed, out, cyc, tiles, gbuf);
    run<P_LDS | P_CVT | P_MFMA, 6>("segment only (lds+cvt+mfma)", cus, seed, out, cyc, tiles, gbuf);
    run<P_LDS | P_CVT | P_MFMA, 4>("segment only", cus, seed, out, cyc, tiles, gbuf);
    run<P_LDS | P_CVT | P_MFMA, 2>("segment only", cus, seed, out, cyc, tiles, gbuf);
    run<P_CVT | P_MFMA, 6>("cvt+mfma (no table reads)", cus, seed, out, cyc, tiles, gbuf);
    run<P_LDS | P_MFMA, 6>("lds+mfma (no cvt)", cus, seed, out, cyc, tiles, gbuf);
    run<P_LDS | P_CVT, 6>("lds+cvt (no mfma)", cus, seed, out, cyc, tiles, gbuf);
    run<P_CVT, 6>("cvt only", cus, seed, out, cyc, tiles, gbuf);
    run<P_LDS, 6>("lds only", cus, seed, out, cyc, tiles, gbuf);
    run<ALL & ~P_CVT, 6>("full minus cvt", cus, seed, out, cyc, tiles, gbuf);
    run<ALL & ~P_LDS, 6>("full minus table reads", cus, seed, out, cyc, tiles, gbuf);
    run<ALL & ~P_MFMA, 6>("full minus mfma", cus, seed, out, cyc, tiles, gbuf);
    return 0;
}
