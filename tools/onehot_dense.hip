// Design prototype ("Where that leaves the next kernel step"): the SAFE part of
// the E4M3 approx_v9 product as a plain e4m3 matrix-core GEMM over K' = 8K.
//
// For a pair whose exact product sits at or above the result grid's smallest normal, the
// reference's term Q_R(V'(m_a, m_b) c_a c_b) equals L(m_a, m_b) c_a c_b with L = Q_R's saturating
// 4-significant-bit rounding of V' (scale invariance).  So with
//   A'[m][8k + j] = (j == m_a(m, k)) ? sign_a 2^(e_a - 7) : 0           (e4m3 exponent field = e_a)
//   B'[8k + j][n] = sign_b L(j, m_b(k, n)) 2^(e_b - 9)                   (e4m3-normal for e_b >= 3 - pmin)
// the safe part of C is (A' @ B')[m][n] 2^(16 - bA - bB(n)).  Elements below the split (e_a < tA,
// e_b < tB(n)) are zero here -- they belong to the compacted per-pair path (not in this file).
//
// This program generates E4M3-grid operands, splits them, runs the dense kernel
// (v_mfma_scale_f32_16x16x128_f8f6f4, 128x128 workgroup tiles, 64x64 per wave, K chunks of 16),
// checks sampled rows against a scalar restatement of the reference's term (full Q_R, subnormal
// band included, restricted to the hi x hi pairs) and reports the dense rate in products/s.
// Build: hipcc --offload-arch=gfx950 -O3 -o onehot_dense tools/onehot_dense.hip
// Run:   ./onehot_dense [M N K]   (M, N multiples of 128, K of 16)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

constexpr int TM = 128, TN = 128, KC = 16;  // workgroup tile, original k per chunk (K' = 128)
constexpr int RS = 8 * KC + 16;             // LDS row stride in bytes (padded)

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

// A1: [M][K] uint2 one-hot images, B1: [N][K] uint2; C [M][N] = scale(n) * sum
__global__ __launch_bounds__(256) void onehot_gemm(const uint2 *__restrict__ A1, const uint2 *__restrict__ B1,
                                                   const float *__restrict__ cscale, float *__restrict__ C, int M,
                                                   int N, int K) {
    __shared__ __attribute__((aligned(16))) char As[TM * RS];
    __shared__ __attribute__((aligned(16))) char Bs[TN * RS];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wr = wv >> 1, wc = wv & 1;
    // XCD-aware order: consecutive block ids land on different XCDs; keep column tiles together
    const int nbn = N / TN, nbm = M / TM;
    const int bid = blockIdx.x;
    const int bm = bid % nbm, bn = bid / nbm;
    const int m0 = bm * TM, n0 = bn * TN;
    // global -> register staging: each thread moves 4 x 16 B of A and of B per chunk
    uint4 ra[4], rb[4];
    auto gload = [&](int k0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int e = tid + 256 * i;  // 1024 16-B pieces: row e / 8, piece e % 8
            const int r = e >> 3, pc = e & 7;
            ra[i] = *reinterpret_cast<const uint4 *>(A1 + (size_t)(m0 + r) * K + k0 + 2 * pc);
            rb[i] = *reinterpret_cast<const uint4 *>(B1 + (size_t)(n0 + r) * K + k0 + 2 * pc);
        }
    };
    v4f acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
    gload(0);
    for (int k0 = 0; k0 < K; k0 += KC) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int e = tid + 256 * i, r = e >> 3, pc = e & 7;
            *reinterpret_cast<uint4 *>(As + r * RS + 16 * pc) = ra[i];
            *reinterpret_cast<uint4 *>(Bs + r * RS + 16 * pc) = rb[i];
        }
        __syncthreads();
        if (k0 + KC < K) gload(k0 + KC);
        const int r16 = lane & 15, g = lane >> 4;
        v8i af[4], bf[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const char *pa = As + (64 * wr + 16 * i + r16) * RS + 32 * g;
            const char *pb = Bs + (64 * wc + 16 * i + r16) * RS + 32 * g;
            const uint4 a0 = *reinterpret_cast<const uint4 *>(pa), a1 = *reinterpret_cast<const uint4 *>(pa + 16);
            const uint4 b0 = *reinterpret_cast<const uint4 *>(pb), b1 = *reinterpret_cast<const uint4 *>(pb + 16);
            af[i] = (v8i){(int)a0.x, (int)a0.y, (int)a0.z, (int)a0.w, (int)a1.x, (int)a1.y, (int)a1.z, (int)a1.w};
            bf[i] = (v8i){(int)b0.x, (int)b0.y, (int)b0.z, (int)b0.w, (int)b1.x, (int)b1.y, (int)b1.z, (int)b1.w};
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bf[j], acc[i][j], 0, 0, 0, 127, 0,
                                                                            127);
        __syncthreads();
    }
    // D layout: col = lane & 15, row = 4 (lane >> 4) + reg
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int col = n0 + 64 * wc + 16 * j + (lane & 15);
            const float s = cscale[col];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m0 + 64 * wr + 16 * i + 4 * (lane >> 4) + r;
                C[(size_t)row * N + col] = acc[i][j][r] * s;
            }
        }
    (void)nbn;
}

// Compact form: A and B as one byte per element (the operand's own e4m3-like code: sign, the
// exponent field, the mantissa m in the low 3 bits), expanded to the one-hot / L-row operands in
// registers.  A byte a -> 8 bytes (a & 0xF8) << 8 (a & 7); B byte b -> the L row of m_b with
// (e_b - 9) added to every byte's exponent field and the sign bit set by s_b.  Workgroup 256 x 128
// (4 waves of 128 x 64), K chunks of 16.
constexpr int TM2 = 256, TN2 = 128;
template <int RB>  // 16-row blocks per wave: 8 -> 256 x 128 workgroup tiles, 4 -> 128 x 128
__global__ __launch_bounds__(256) void onehot_gemm2(const uint8_t *__restrict__ Ac, const uint8_t *__restrict__ Bc,
                                                    const uint2 *__restrict__ lut, const float *__restrict__ cscale,
                                                    float *__restrict__ C, int M, int N, int K) {
    constexpr int TMR = 32 * RB;
    __shared__ uint32_t As[TMR * 4];  // [row][4 dwords = 16 k]
    __shared__ uint32_t Bs[TN2 * 4];
    __shared__ uint2 Ls[8];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wr = wv >> 1, wc = wv & 1;
    const int nbm = M / TMR;
    const int bm = blockIdx.x % nbm, bn = blockIdx.x / nbm;
    const int m0 = bm * TMR, n0 = bn * TN2;
    if (tid < 8) Ls[tid] = lut[tid];
    uint4 ra, rb = make_uint4(0, 0, 0, 0);
    auto gload = [&](int k0) {
        if (tid < TMR) ra = *reinterpret_cast<const uint4 *>(Ac + (size_t)(m0 + tid) * K + k0);
        if (tid < TN2) rb = *reinterpret_cast<const uint4 *>(Bc + (size_t)(n0 + tid) * K + k0);
    };
    v4f acc[RB][4];
#pragma unroll
    for (int i = 0; i < RB; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
    gload(0);
    const int r16 = lane & 15, g = lane >> 4;
    for (int k0 = 0; k0 < K; k0 += KC) {
        if (tid < TMR) *reinterpret_cast<uint4 *>(&As[4 * tid]) = ra;
        if (tid < TN2) *reinterpret_cast<uint4 *>(&Bs[4 * tid]) = rb;
        __syncthreads();
        if (k0 + KC < K) gload(k0 + KC);
        v8i bf[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t w = Bs[4 * (64 * wc + 16 * j + r16) + g];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t b = (w >> (8 * e)) & 0xFFu;
                const uint2 l = Ls[b & 7u];
                const uint32_t add = (((b >> 3) & 15u) - 9u) * 0x08080808u;
                const uint32_t sg = (b & 0x80u) ? 0x80808080u : 0u;
                // a zero (or small) weight: all-zero operand bytes
                bf[j][2 * e] = b ? (int)((l.x + add) ^ sg) : 0;
                bf[j][2 * e + 1] = b ? (int)((l.y + add) ^ sg) : 0;
            }
        }
#pragma unroll
        for (int i = 0; i < RB; ++i) {
            const uint32_t w = As[4 * (16 * RB * wr + 16 * i + r16) + g];
            v8i af;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t a = (w >> (8 * e)) & 0xFFu;
                const uint64_t x = (uint64_t)(a & 0xF8u) << (8 * (a & 7u));
                af[2 * e] = (int)(uint32_t)x;
                af[2 * e + 1] = (int)(uint32_t)(x >> 32);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, bf[j], acc[i][j], 0, 0, 0, 127, 0,
                                                                            127);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < RB; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int col = n0 + 64 * wc + 16 * j + (lane & 15);
            const float sc = cscale[col];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m0 + 16 * RB * wr + 16 * i + 4 * (lane >> 4) + r;
                C[(size_t)row * N + col] = acc[i][j][r] * sc;
            }
        }
}

// Mixed form: A as one byte per element expanded in registers (as onehot_gemm2), B' as the 8-B
// L-row image of onehot_gemm (weights are static: a per-layer pre-pass).  Workgroup 128 x 128,
// 64 x 64 per wave (64 accumulator registers: 2 waves / SIMD).
__global__ __launch_bounds__(256) void onehot_gemm3(const uint8_t *__restrict__ Ac, const uint2 *__restrict__ B1,
                                                    const float *__restrict__ cscale, float *__restrict__ C, int M,
                                                    int N, int K) {
    __shared__ uint32_t As[TM * 4];
    __shared__ __attribute__((aligned(16))) char Bs[TN * RS];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wr = wv >> 1, wc = wv & 1;
    const int nbm = M / TM;
    const int bm = blockIdx.x % nbm, bn = blockIdx.x / nbm;
    const int m0 = bm * TM, n0 = bn * TN;
    uint4 ra = make_uint4(0, 0, 0, 0), rb[4];
    auto gload = [&](int k0) {
        if (tid < TM) ra = *reinterpret_cast<const uint4 *>(Ac + (size_t)(m0 + tid) * K + k0);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int e = tid + 256 * i, r = e >> 3, pc = e & 7;
            rb[i] = *reinterpret_cast<const uint4 *>(B1 + (size_t)(n0 + r) * K + k0 + 2 * pc);
        }
    };
    v4f acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
    gload(0);
    const int r16 = lane & 15, g = lane >> 4;
    for (int k0 = 0; k0 < K; k0 += KC) {
        if (tid < TM) *reinterpret_cast<uint4 *>(&As[4 * tid]) = ra;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int e = tid + 256 * i, r = e >> 3, pc = e & 7;
            *reinterpret_cast<uint4 *>(Bs + r * RS + 16 * pc) = rb[i];
        }
        __syncthreads();
        if (k0 + KC < K) gload(k0 + KC);
        v8i bf[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const char *pb = Bs + (64 * wc + 16 * j + r16) * RS + 32 * g;
            const uint4 b0 = *reinterpret_cast<const uint4 *>(pb), b1 = *reinterpret_cast<const uint4 *>(pb + 16);
            bf[j] = (v8i){(int)b0.x, (int)b0.y, (int)b0.z, (int)b0.w, (int)b1.x, (int)b1.y, (int)b1.z, (int)b1.w};
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t w = As[4 * (64 * wr + 16 * i + r16) + g];
            v8i af;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t a = (w >> (8 * e)) & 0xFFu;
                const uint64_t x = (uint64_t)(a & 0xF8u) << (8 * (a & 7u));
                af[2 * e] = (int)(uint32_t)x;
                af[2 * e + 1] = (int)(uint32_t)(x >> 32);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, bf[j], acc[i][j], 0, 0, 0, 127, 0,
                                                                            127);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int col = n0 + 64 * wc + 16 * j + (lane & 15);
            const float sc = cscale[col];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m0 + 64 * wr + 16 * i + 4 * (lane >> 4) + r;
                C[(size_t)row * N + col] = acc[i][j][r] * sc;
            }
        }
}

// onehot_gemm3 with KCH original k per staged chunk (KCH / 16 MFMA k-steps between barriers).
template <int KCH>
__global__ __launch_bounds__(256) void onehot_gemm4(const uint8_t *__restrict__ Ac, const uint2 *__restrict__ B1,
                                                    const float *__restrict__ cscale, float *__restrict__ C, int M,
                                                    int N, int K) {
    constexpr int AW = KCH / 4;           // A dwords per row
    constexpr int BRS = 8 * KCH + 16;     // B' row stride (bytes)
    constexpr int APT = TM * KCH / 16;    // 16-B A pieces per chunk
    constexpr int BPT = TN * KCH / 2 / 256;  // 16-B B' pieces per thread
    static_assert(APT <= 256, "one 16-B A piece per thread at most");
    __shared__ uint32_t As[TM * AW];
    __shared__ __attribute__((aligned(16))) char Bs[TN * BRS];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wr = wv >> 1, wc = wv & 1;
    const int nbm = M / TM;
    const int bm = blockIdx.x % nbm, bn = blockIdx.x / nbm;
    const int m0 = bm * TM, n0 = bn * TN;
    uint4 ra = make_uint4(0, 0, 0, 0), rb[BPT];
    auto gload = [&](int k0) {
        if (tid < APT) {
            const int r = tid / (KCH / 16), pc = tid % (KCH / 16);
            ra = *reinterpret_cast<const uint4 *>(Ac + (size_t)(m0 + r) * K + k0 + 16 * pc);
        }
#pragma unroll
        for (int i = 0; i < BPT; ++i) {
            const int e = tid + 256 * i, r = e / (KCH / 2), pc = e % (KCH / 2);
            rb[i] = *reinterpret_cast<const uint4 *>(B1 + (size_t)(n0 + r) * K + k0 + 2 * pc);
        }
    };
    v4f acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
    gload(0);
    const int r16 = lane & 15, g = lane >> 4;
    for (int k0 = 0; k0 < K; k0 += KCH) {
        if (tid < APT) {
            const int r = tid / (KCH / 16), pc = tid % (KCH / 16);
            *reinterpret_cast<uint4 *>(&As[r * AW + 4 * pc]) = ra;
        }
#pragma unroll
        for (int i = 0; i < BPT; ++i) {
            const int e = tid + 256 * i, r = e / (KCH / 2), pc = e % (KCH / 2);
            *reinterpret_cast<uint4 *>(Bs + r * BRS + 16 * pc) = rb[i];
        }
        __syncthreads();
        if (k0 + KCH < K) gload(k0 + KCH);
#pragma unroll
        for (int ks = 0; ks < KCH / 16; ++ks) {
            v8i bf[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const char *pb = Bs + (64 * wc + 16 * j + r16) * BRS + 128 * ks + 32 * g;
                const uint4 b0 = *reinterpret_cast<const uint4 *>(pb), b1 = *reinterpret_cast<const uint4 *>(pb + 16);
                bf[j] = (v8i){(int)b0.x, (int)b0.y, (int)b0.z, (int)b0.w, (int)b1.x, (int)b1.y, (int)b1.z, (int)b1.w};
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t w = As[(64 * wr + 16 * i + r16) * AW + 4 * ks + g];
                v8i af;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint32_t a = (w >> (8 * e)) & 0xFFu;
                    const uint64_t x = (uint64_t)(a & 0xF8u) << (8 * (a & 7u));
                    af[2 * e] = (int)(uint32_t)x;
                    af[2 * e + 1] = (int)(uint32_t)(x >> 32);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, bf[j], acc[i][j], 0, 0, 0, 127, 0,
                                                                                127);
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int col = n0 + 64 * wc + 16 * j + (lane & 15);
            const float sc = cscale[col];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m0 + 64 * wr + 16 * i + 4 * (lane >> 4) + r;
                C[(size_t)row * N + col] = acc[i][j][r] * sc;
            }
        }
}

// Both operands as 1-B codes in HBM; per 32-k chunk the workgroup expands B into the 8-B L-row
// operand ONCE in LDS (shared by the two row-waves of each column half), A is expanded in
// registers.  128 x 128 tiles, 64 x 64 per wave.
__global__ __launch_bounds__(256) void onehot_gemm5(const uint8_t *__restrict__ Ac, const uint8_t *__restrict__ Bc,
                                                    const uint2 *__restrict__ lut, const float *__restrict__ cscale,
                                                    float *__restrict__ C, int M, int N, int K) {
    constexpr int KCH = 32, BRS5 = 8 * KCH + 16, AW5 = KCH / 4 + 1;  // B' row stride (bytes), A row (dwords)
    __shared__ uint32_t As[TM * AW5];
    __shared__ __attribute__((aligned(16))) char Bs[TN * BRS5];
    __shared__ uint2 Ls[8];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wr = wv >> 1, wc = wv & 1;
    const int nbm = M / TM;
    const int bm = blockIdx.x % nbm, bn = blockIdx.x / nbm;
    const int m0 = bm * TM, n0 = bn * TN;
    if (tid < 8) Ls[tid] = lut[tid];
    // thread t stages A row t / 2 (16 B half t & 1) and B column t / 2 (16 k half t & 1)
    const int sr = tid >> 1, sh = tid & 1;
    uint4 ra, rb;
    auto gload = [&](int k0) {
        ra = *reinterpret_cast<const uint4 *>(Ac + (size_t)(m0 + sr) * K + k0 + 16 * sh);
        rb = *reinterpret_cast<const uint4 *>(Bc + (size_t)(n0 + sr) * K + k0 + 16 * sh);
    };
    v4f acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
    gload(0);
    __syncthreads();  // Ls
    const int r16 = lane & 15, g = lane >> 4;
    for (int k0 = 0; k0 < K; k0 += KCH) {
        // A codes as they are; B codes expanded to the L-row operand
        As[sr * AW5 + 4 * sh + 0] = ra.x;
        As[sr * AW5 + 4 * sh + 1] = ra.y;
        As[sr * AW5 + 4 * sh + 2] = ra.z;
        As[sr * AW5 + 4 * sh + 3] = ra.w;
        {
            const uint32_t wb[4] = {rb.x, rb.y, rb.z, rb.w};
            char *dst = Bs + sr * BRS5 + 128 * sh;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                uint32_t o[8];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint32_t b = (wb[q] >> (8 * e)) & 0xFFu;
                    const uint2 l = Ls[b & 7u];
                    const uint32_t add = (((b >> 3) & 15u) - 9u) * 0x08080808u;
                    const uint32_t sg = (b & 0x80u) ? 0x80808080u : 0u;
                    o[2 * e] = b ? ((l.x + add) ^ sg) : 0u;
                    o[2 * e + 1] = b ? ((l.y + add) ^ sg) : 0u;
                }
                *reinterpret_cast<uint4 *>(dst + 32 * q) = make_uint4(o[0], o[1], o[2], o[3]);
                *reinterpret_cast<uint4 *>(dst + 32 * q + 16) = make_uint4(o[4], o[5], o[6], o[7]);
            }
        }
        __syncthreads();
        if (k0 + KCH < K) gload(k0 + KCH);
#pragma unroll
        for (int ks = 0; ks < KCH / 16; ++ks) {
            v8i bf[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const char *pb = Bs + (64 * wc + 16 * j + r16) * BRS5 + 128 * ks + 32 * g;
                const uint4 b0 = *reinterpret_cast<const uint4 *>(pb), b1 = *reinterpret_cast<const uint4 *>(pb + 16);
                bf[j] = (v8i){(int)b0.x, (int)b0.y, (int)b0.z, (int)b0.w, (int)b1.x, (int)b1.y, (int)b1.z, (int)b1.w};
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t w = As[(64 * wr + 16 * i + r16) * AW5 + 4 * ks + g];
                v8i af;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint32_t a = (w >> (8 * e)) & 0xFFu;
                    const uint64_t x = (uint64_t)(a & 0xF8u) << (8 * (a & 7u));
                    af[2 * e] = (int)(uint32_t)x;
                    af[2 * e + 1] = (int)(uint32_t)(x >> 32);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, bf[j], acc[i][j], 0, 0, 0, 127, 0,
                                                                                127);
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int col = n0 + 64 * wc + 16 * j + (lane & 15);
            const float sc = cscale[col];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m0 + 64 * wr + 16 * i + 4 * (lane >> 4) + r;
                C[(size_t)row * N + col] = acc[i][j][r] * sc;
            }
        }
}

// ---- host: the reference's E4M3 term, scalar, in double
static double rne(double x) { return std::nearbyint(x); }  // default rounding mode: nearest-even

static double q_r(double x, int b) {  // Q(x, b, clip = false) for E4M3
    if (x == 0) return 0;
    const double ax = std::fabs(x), s = x < 0 ? -1 : 1;
    const double mn = std::ldexp(1.0, 1 - b);
    if (ax < mn) {
        double m = std::min(rne(ax / std::ldexp(1.0, 1 - b - 3)), 7.0);
        return s * std::ldexp(m, 1 - b - 3);
    }
    int p;
    double f = std::frexp(ax, &p);  // ax = f 2^p, f in [0.5, 1)
    double mant = std::min(rne((2 * f - 1) * 8), 7.0);
    return s * std::ldexp(1 + mant / 8, p - 1);
}

struct Code {
    int s, e, m;  // sign, biased exponent 1..15 (0 = zero), mantissa 0..7
};

int main(int argc, char **argv) {
    const int M = argc > 1 ? atoi(argv[1]) : 8192, N = argc > 2 ? atoi(argv[2]) : 512,
              K = argc > 3 ? atoi(argv[3]) : 2304;
    if (M % TM2 || N % TN || K % 32) {
        fprintf(stderr, "M must be a multiple of 256, N of 128 and K of 32\n");
        return 2;
    }
    const int bA = 12, bR = 14;
    std::vector<int> bB(N);
    std::mt19937 rng(5);
    std::normal_distribution<double> nd(0.0, 1.0);
    // E4M3 {0,1} table pattern (a stand-in for get_error_table_NN(4, 3)): V' >= 7/8 always
    int T[8][8];
    for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 8; ++j) T[i][j] = ((i * 3 + j * 5) % 4 == 0) ? 1 : 0;
    double L[8][8];
    int pmin = 0;
    for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 8; ++j) {
            const double v = (1 + i / 8.0) * (1 + j / 8.0) - T[i][j] / 8.0;
            L[i][j] = q_r(v, 100);  // far above the subnormal band: pure 4-bit saturating rounding
            if (v < 1) pmin = -1;
        }
    // operands on the normal E4M3 grid: A = relu(N(0,1)) at bias bA, B = N(0, 0.05) per column bias
    std::vector<Code> a((size_t)M * K), b((size_t)N * K);
    auto enc = [](double v, int bias) {
        Code c{v < 0, 0, 0};
        const double av = std::fabs(v);
        if (av == 0) return c;
        int p;
        std::frexp(av, &p);
        int e = p - 1 + bias;
        if (e < 1) return Code{0, 0, 0};  // (subnormals of the operand grid: zero in this prototype)
        if (e > 15) e = 15;
        double m = std::min(rne((av / std::ldexp(1.0, e - bias) - 1) * 8), 7.0);
        c.e = e;
        c.m = (int)m;
        return c;
    };
    for (size_t i = 0; i < a.size(); ++i) a[i] = enc(std::max(nd(rng), 0.0) * std::ldexp(1.0, 15 - bA - 3), bA);
    for (int n = 0; n < N; ++n) {
        bB[n] = 18 + (n % 3);
        for (int k = 0; k < K; ++k) b[(size_t)n * K + k] = enc(nd(rng) * 0.05 * std::ldexp(1.0, bB[n] - 5), bB[n]);
    }
    // split: A hi iff e_a >= tA; B hi iff e_b >= tB(n); hi x hi pairs are safe
    const int tA = argc > 4 ? atoi(argv[4]) : 6;
    std::vector<int> tB(N);
    size_t nzA = 0, loA = 0, nzB = 0, loB = 0;
    for (int n = 0; n < N; ++n) tB[n] = std::max(3 - pmin, bA + bB[n] + 1 - bR - pmin - tA);
    std::vector<uint2> A1((size_t)M * K), B1((size_t)N * K);
    for (size_t i = 0; i < a.size(); ++i) {
        uint64_t w = 0;
        if (a[i].e) {
            ++nzA;
            if (a[i].e >= tA) w = (uint64_t)((a[i].s << 7) | (a[i].e << 3)) << (8 * a[i].m);
            else ++loA;
        }
        A1[i] = make_uint2((uint32_t)w, (uint32_t)(w >> 32));
    }
    for (int n = 0; n < N; ++n)
        for (int k = 0; k < K; ++k) {
            const Code c = b[(size_t)n * K + k];
            uint64_t w = 0;
            if (c.e) {
                ++nzB;
                if (c.e >= tB[n]) {
                    for (int j = 0; j < 8; ++j) {
                        int p;
                        const double f = std::frexp(L[j][c.m], &p);  // L = 2f 2^(p-1)
                        const int fe = c.e - 9 + (p - 1) + 7, fm = (int)rne((2 * f - 1) * 8);
                        if (fe < 1 || fe > 15 || (fe == 15 && fm == 7)) {
                            fprintf(stderr, "B' out of e4m3 range\n");
                            return 3;
                        }
                        w |= (uint64_t)((c.s << 7) | (fe << 3) | fm) << (8 * j);
                    }
                } else {
                    ++loB;
                }
            }
            B1[(size_t)n * K + k] = make_uint2((uint32_t)w, (uint32_t)(w >> 32));
        }
    std::vector<float> cs(N);
    for (int n = 0; n < N; ++n) cs[n] = (float)std::ldexp(1.0, 16 - bA - bB[n]);
    printf("M %d N %d K %d  tA %d  small A %.4f of nonzero, small B %.4f of nonzero\n", M, N, K, tA,
           (double)loA / std::max<size_t>(nzA, 1), (double)loB / std::max<size_t>(nzB, 1));

    // compact operands: A byte = sign | e_a << 3 | m_a (0 for zero / small), B byte likewise;
    // lut[m_b] = the 8 bytes e4m3(L(j, m_b)) (exponent field p + 7), the kernel adds e_b - 9
    std::vector<uint8_t> Ac((size_t)M * K), Bc((size_t)N * K);
    for (size_t i = 0; i < a.size(); ++i)
        Ac[i] = (a[i].e && a[i].e >= tA) ? (uint8_t)((a[i].s << 7) | (a[i].e << 3) | a[i].m) : 0;
    for (int n = 0; n < N; ++n)
        for (int k = 0; k < K; ++k) {
            const Code c = b[(size_t)n * K + k];
            Bc[(size_t)n * K + k] = (c.e && c.e >= tB[n]) ? (uint8_t)((c.s << 7) | (c.e << 3) | c.m) : 0;
        }
    std::vector<uint2> lut(8);
    for (int mb = 0; mb < 8; ++mb) {
        uint64_t w = 0;
        for (int j = 0; j < 8; ++j) {
            int p;
            const double f = std::frexp(L[j][mb], &p);
            w |= (uint64_t)((((p - 1) + 7) << 3) | (int)rne((2 * f - 1) * 8)) << (8 * j);
        }
        lut[mb] = make_uint2((uint32_t)w, (uint32_t)(w >> 32));
    }

    uint2 *dA, *dB, *dL;
    uint8_t *dAc, *dBc;
    float *dC, *dS;
    CK(hipMalloc(&dA, A1.size() * 8));
    CK(hipMalloc(&dB, B1.size() * 8));
    CK(hipMalloc(&dAc, Ac.size()));
    CK(hipMalloc(&dBc, Bc.size()));
    CK(hipMalloc(&dL, 64));
    CK(hipMalloc(&dC, (size_t)M * N * 4));
    CK(hipMalloc(&dS, N * 4));
    CK(hipMemcpy(dA, A1.data(), A1.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B1.data(), B1.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dAc, Ac.data(), Ac.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dBc, Bc.data(), Bc.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dL, lut.data(), 64, hipMemcpyHostToDevice));
    CK(hipMemcpy(dS, cs.data(), N * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double prods = (double)M * N * K;
    std::vector<float> C((size_t)M * N);
    int bad_total = 0;
    for (int form = 1; form <= 6; ++form) {
        auto launch = [&]() {
            if (form == 1)
                hipLaunchKernelGGL(onehot_gemm, dim3((M / TM) * (N / TN)), dim3(256), 0, 0, dA, dB, dS, dC, M, N, K);
            else if (form == 2)
                hipLaunchKernelGGL(onehot_gemm2<8>, dim3((M / TM2) * (N / TN2)), dim3(256), 0, 0, dAc, dBc, dL, dS, dC,
                                   M, N, K);
            else if (form == 5)
                hipLaunchKernelGGL(onehot_gemm2<4>, dim3((M / 128) * (N / TN2)), dim3(256), 0, 0, dAc, dBc, dL, dS, dC,
                                   M, N, K);
            else if (form == 6)
                hipLaunchKernelGGL(onehot_gemm5, dim3((M / TM) * (N / TN)), dim3(256), 0, 0, dAc, dBc, dL, dS, dC, M, N,
                                   K);
            else if (form == 3)
                hipLaunchKernelGGL(onehot_gemm3, dim3((M / TM) * (N / TN)), dim3(256), 0, 0, dAc, dB, dS, dC, M, N, K);
            else if (form == 4)
                hipLaunchKernelGGL(onehot_gemm4<32>, dim3((M / TM) * (N / TN)), dim3(256), 0, 0, dAc, dB, dS, dC, M, N,
                                   K);
        };
        CK(hipMemset(dC, 0xFF, (size_t)M * N * 4));
        launch();
        CK(hipDeviceSynchronize());
        const int reps = 20;
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%s: %.3f ms, %.2f T products/s (%.1f products / cycle / SIMD at 2.4 GHz)\n",
               form == 1 ? "dense one-hot, 8-B operand images"
               : form == 2 ? "dense one-hot, 1-B operands expanded in registers"
               : form == 3 ? "dense one-hot, 1-B A expanded in registers, 8-B B' image"
               : form == 4 ? "  same, 32 k per staged chunk"
               : form == 5 ? "1-B operands expanded in registers, 128 x 128 tiles (64 x 64 per wave)"
                           : "1-B operands, B expanded once per 32-k chunk into LDS, A in registers, 128 x 128",
               ms, prods / ms / 1e9, prods / (ms * 1e-3) / (1024 * 2.4e9));
        CK(hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost));
        // check sampled rows against the reference term over hi x hi pairs
        int bad = 0, checked = 0;
        double worst = 0;
        for (int t = 0; t < 32; ++t) {
            const int m = (int)((t * 2654435761u) % (unsigned)M);
            for (int n = 0; n < N; ++n) {
                double s = 0, sa = 0;
                for (int k = 0; k < K; ++k) {
                    const Code ca = a[(size_t)m * K + k], cb = b[(size_t)n * K + k];
                    if (!ca.e || !cb.e || ca.e < tA || cb.e < tB[n]) continue;
                    const double v = ((1 + ca.m / 8.0) * (1 + cb.m / 8.0) - T[ca.m][cb.m] / 8.0) *
                                     std::ldexp(1.0, ca.e - bA + cb.e - bB[n]) * ((ca.s ^ cb.s) ? -1 : 1);
                    const double term = q_r(v, bR);
                    s += term;
                    sa += std::fabs(term);
                }
                const double d = std::fabs(C[(size_t)m * N + n] - s);
                worst = std::max(worst, d / (sa + 1e-30));
                bad += !(d <= 1e-5 * sa + 1e-30);
                ++checked;
            }
        }
        printf("  check: %d of %d sampled outputs outside 1e-5 sum|term| (worst rel %.3g)\n", bad, checked, worst);
        bad_total += bad;
    }
    const int bad = bad_total;
    return bad ? 1 : 0;
}
