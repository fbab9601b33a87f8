// Design prototype, the other half of DESIGN.md §3a's plan: the per-pair path over compacted
// lists of "small" A elements (the pairs the dense one-hot GEMM of tools/onehot_dense.hip must not
// take).  Per 16-row block, every row's small entries (k, A word) are padded to the block's
// longest list; a wave's lanes are (row r16, list slot group g) exactly as in gemm_f8mx_kernel, so
// per MFMA each lane converts its row's 2 entries against the wave's 16 columns and one
// v_mfma_scale_f32_16x16x128_f8f6f4 with the constant column-selection operand sums them into
// D[row][column].  Unlike the tile-table kernel the entries of a wave have different k, so the
// c_b-applied table values are formed per product pair: B pair word (c_b addend pair, pair code
// offset) from global memory, one LDS read of the static [pair][m_a] table, one packed add.
//
// The program builds random E4M3-grid operands and lists (a fraction of each row's nonzero
// elements), runs the kernel, checks sampled rows against a scalar restatement of the
// reference's term (full Q_R incl. its subnormal band) summed over the listed pairs, and
// reports products / s (listed entries x N).
// Build: hipcc --offload-arch=gfx950 -O3 -o small_rows tools/small_rows.hip
// Run:   ./small_rows [M N K frac]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef short s2 __attribute__((ext_vector_type(2)));
typedef unsigned short u2 __attribute__((ext_vector_type(2)));
typedef __bf16 b2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

constexpr uint32_t ZERO_WORD = 254u << 23;  // scale 2^127: the code is 0

// lists: [block][round][g][r16] uint4 = (k0, word0, k1, word1) -- the lane's two entries of a
// round; rounds[block] = padded list length / 8.  bpw: [K][N / 2] uint2 (addend pair, pair byte
// offset into the static table); lut: [81 pairs][8 m_a] u32 bf16 pairs.
__global__ __launch_bounds__(256) void small_rows(const uint4 *__restrict__ lists, const int *__restrict__ roff,
                                                  const int *__restrict__ rounds, const uint2 *__restrict__ bpw,
                                                  const uint32_t *__restrict__ lut, float *__restrict__ C, int N,
                                                  float outscale) {
    __shared__ uint32_t L[81 * 8];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (int i = tid; i < 81 * 8; i += 256) L[i] = lut[i];
    __syncthreads();
    const int blk = blockIdx.x, n0 = blockIdx.y * 64 + 16 * wv;  // the wave's 16 columns
    const int r16 = lane & 15, g = lane >> 4;
    // selection operand: byte p of every lane is 1.0 where (p & 15) == its column
    v8i sel;
    for (int v = 0; v < 8; ++v) {
        uint32_t w = 0;
        for (int b = 0; b < 4; ++b)
            if (((4 * v + b) & 15) == r16) w |= 0x38u << (8 * b);
        sel[v] = (int)w;
    }
    v4f d = {0.f, 0.f, 0.f, 0.f};
    const uint4 *lp = lists + (size_t)roff[blk] * 64;
    const int nr = rounds[blk];
    const char *Lc = reinterpret_cast<const char *>(L);
    for (int r = 0; r < nr; ++r) {
        const uint4 e = lp[(size_t)r * 64 + g * 16 + r16];
        v8i av;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t k = h ? e.z : e.x, w = h ? e.w : e.y;
            const uint2 *bp = bpw + (size_t)k * (N / 2) + n0 / 2;
            const uint4 q0 = *reinterpret_cast<const uint4 *>(bp), q1 = *reinterpret_cast<const uint4 *>(bp + 2);
            const uint4 q2 = *reinterpret_cast<const uint4 *>(bp + 4), q3 = *reinterpret_cast<const uint4 *>(bp + 6);
            const uint2 pw[8] = {make_uint2(q0.x, q0.y), make_uint2(q0.z, q0.w), make_uint2(q1.x, q1.y),
                                 make_uint2(q1.z, q1.w), make_uint2(q2.x, q2.y), make_uint2(q2.z, q2.w),
                                 make_uint2(q3.x, q3.y), make_uint2(q3.z, q3.w)};
            const uint32_t row = w & 0x1Fu;  // m_a * 4: byte offset of column m_a in a pair row; 0x20: sign
            const uint32_t sgn = (w & 0x20u) ? 0x80008000u : 0u;
            const float sc = __uint_as_float(w & 0x7F800000u);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const uint32_t v0 = *reinterpret_cast<const uint32_t *>(Lc + pw[2 * c].y + row);
                const uint32_t v1 = *reinterpret_cast<const uint32_t *>(Lc + pw[2 * c + 1].y + row);
                const uint32_t a0 = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u2, v0) +
                                                                     __builtin_bit_cast(u2, pw[2 * c].x ^ sgn));
                const uint32_t a1 = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u2, v1) +
                                                                     __builtin_bit_cast(u2, pw[2 * c + 1].x ^ sgn));
                s2 cv = {0, 0};
                cv = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(cv, __builtin_bit_cast(b2, a0), sc, false);
                cv = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(cv, __builtin_bit_cast(b2, a1), sc, true);
                av[4 * h + c] = __builtin_bit_cast(int, cv);
            }
        }
        d = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, sel, d, 0, 0, 0, 127, 0, 127);
    }
    // D[row][col]: col = lane & 15, row = 4 g + i
#pragma unroll
    for (int i = 0; i < 4; ++i) C[(size_t)(16 * blk + 4 * g + i) * N + n0 + r16] = d[i] * outscale;
}

// Windowed form: per K window of KW steps the workgroup stages the window's B pair words for its
// 64 columns in LDS (KW x 32 x 8 B), so every entry of the window reads them from LDS instead of
// L2; the lists are per (16-row block, window), each row padded to the block's longest list in
// that window.  lists2: [(block, window)][round][g][r16] uint4 (k0 - window base, word0, k1 -
// window base, word1).
template <int KW>
__global__ __launch_bounds__(256) void small_win(const uint4 *__restrict__ lists, const int *__restrict__ roff,
                                                 const int *__restrict__ rounds, const uint2 *__restrict__ bpw,
                                                 const uint32_t *__restrict__ lut, float *__restrict__ C, int N, int K,
                                                 float outscale) {
    __shared__ uint32_t L[81 * 8];
    __shared__ __attribute__((aligned(16))) uint2 Bw[KW * 32];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (int i = tid; i < 81 * 8; i += 256) L[i] = lut[i];
    const int blk = blockIdx.x, nw = K / KW;
    const int nwg = blockIdx.y * 64, n0 = nwg + 16 * wv;
    const int r16 = lane & 15, g = lane >> 4;
    v8i sel;
    for (int v = 0; v < 8; ++v) {
        uint32_t w = 0;
        for (int b = 0; b < 4; ++b)
            if (((4 * v + b) & 15) == r16) w |= 0x38u << (8 * b);
        sel[v] = (int)w;
    }
    v4f d = {0.f, 0.f, 0.f, 0.f};
    const char *Lc = reinterpret_cast<const char *>(L);
    for (int w = 0; w < nw; ++w) {
        const int nr = rounds[blk * nw + w];
        if (nr == 0) continue;  // (uniform per workgroup)
        __syncthreads();
        // stage: KW rows of 32 pairs (256 B) = 16 uint4 each
        for (int q = tid; q < KW * 16; q += 256) {
            const int kr = q >> 4, pc = q & 15;
            *reinterpret_cast<uint4 *>(&Bw[kr * 32 + 2 * pc]) =
                *reinterpret_cast<const uint4 *>(bpw + (size_t)(w * KW + kr) * (N / 2) + nwg / 2 + 2 * pc);
        }
        __syncthreads();
        const uint4 *lp = lists + (size_t)roff[blk * nw + w] * 64;
        for (int r = 0; r < nr; ++r) {
            const uint4 e = lp[(size_t)r * 64 + g * 16 + r16];
            v8i av;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint32_t kl = h ? e.z : e.x, wd = h ? e.w : e.y;
                const uint2 *bp = &Bw[kl * 32 + 8 * wv];
                const uint4 q0 = *reinterpret_cast<const uint4 *>(bp), q1 = *reinterpret_cast<const uint4 *>(bp + 2);
                const uint4 q2 = *reinterpret_cast<const uint4 *>(bp + 4), q3 = *reinterpret_cast<const uint4 *>(bp + 6);
                const uint2 pw[8] = {make_uint2(q0.x, q0.y), make_uint2(q0.z, q0.w), make_uint2(q1.x, q1.y),
                                     make_uint2(q1.z, q1.w), make_uint2(q2.x, q2.y), make_uint2(q2.z, q2.w),
                                     make_uint2(q3.x, q3.y), make_uint2(q3.z, q3.w)};
                const uint32_t row = wd & 0x1Fu;
                const uint32_t sgn = (wd & 0x20u) ? 0x80008000u : 0u;
                const float sc = __uint_as_float(wd & 0x7F800000u);
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const uint32_t v0 = *reinterpret_cast<const uint32_t *>(Lc + pw[2 * c].y + row);
                    const uint32_t v1 = *reinterpret_cast<const uint32_t *>(Lc + pw[2 * c + 1].y + row);
                    const uint32_t a0 = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u2, v0) +
                                                                         __builtin_bit_cast(u2, pw[2 * c].x ^ sgn));
                    const uint32_t a1 = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u2, v1) +
                                                                         __builtin_bit_cast(u2, pw[2 * c + 1].x ^ sgn));
                    s2 cv = {0, 0};
                    cv = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(cv, __builtin_bit_cast(b2, a0), sc, false);
                    cv = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(cv, __builtin_bit_cast(b2, a1), sc, true);
                    av[4 * h + c] = __builtin_bit_cast(int, cv);
                }
            }
            d = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, sel, d, 0, 0, 0, 127, 0, 127);
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) C[(size_t)(16 * blk + 4 * g + i) * N + n0 + r16] = d[i] * outscale;
}

static double rne(double x) { return std::nearbyint(x); }
static double q_r(double x, int b) {  // the reference's Q(x, b, clip = false), E4M3
    if (x == 0) return 0;
    const double ax = std::fabs(x), s = x < 0 ? -1 : 1;
    if (ax < std::ldexp(1.0, 1 - b)) return s * std::ldexp(std::min(rne(ax / std::ldexp(1.0, -2 - b)), 7.0), -2 - b);
    int p;
    const double f = std::frexp(ax, &p);
    return s * std::ldexp(1 + std::min(rne((2 * f - 1) * 8), 7.0) / 8, p - 1);
}
static uint16_t bf16_bits(float v) {  // v is bf16-exact here
    uint32_t u;
    memcpy(&u, &v, 4);
    return (uint16_t)(u >> 16);
}

int main(int argc, char **argv) {
    const int M = argc > 1 ? atoi(argv[1]) : 65536, N = argc > 2 ? atoi(argv[2]) : 512,
              K = argc > 3 ? atoi(argv[3]) : 2304;
    const double frac = argc > 4 ? atof(argv[4]) : 0.06;
    if (M % 16 || N % 64) return 2;
    const int bA = 12, bR = 10;
    std::vector<int> bB(N);
    std::mt19937 rng(7);
    std::normal_distribution<double> nd(0.0, 1.0);
    std::uniform_real_distribution<double> ud(0.0, 1.0);
    int T[8][8];
    for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 8; ++j) T[i][j] = ((i * 3 + j * 5) % 4 == 0) ? 1 : 0;
    // static table [pair = code0 + 9 code1][m_a]: bf16 pair V'(m_a, code), code 8 = zero weight
    std::vector<uint32_t> lut(81 * 8);
    for (int pr = 0; pr < 81; ++pr)
        for (int ma = 0; ma < 8; ++ma) {
            uint32_t w = 0;
            for (int h = 0; h < 2; ++h) {
                const int cd = h ? pr / 9 : pr % 9;
                if (cd == 8) continue;
                float v = std::fma(1.0f + 0.125f * ma, 1.0f + 0.125f * cd, -T[ma][cd] * 0.125f);
                int p;
                std::frexp(v, &p);
                v = std::min(v, std::ldexp(1.0f, p - 1) * 1.8671875f);
                w |= (uint32_t)bf16_bits(v) << (16 * h);
            }
            lut[pr * 8 + ma] = w;
        }
    // operands: A codes (e_a, m_a, s_a) relu(N(0,1)) at bias bA; B per column at bias bB(n)
    struct Code {
        int s, e, m;
    };
    auto enc = [](double v, int bias) {
        Code c{v < 0, 0, 0};
        const double av = std::fabs(v);
        if (av == 0) return c;
        int p;
        std::frexp(av, &p);
        const int e = p - 1 + bias;
        if (e < 1 || e > 15) return Code{0, 0, 0};
        c.e = e;
        c.m = (int)std::min(rne((av / std::ldexp(1.0, e - bias) - 1) * 8), 7.0);
        return c;
    };
    std::vector<Code> b((size_t)K * N);
    for (int n = 0; n < N; ++n) bB[n] = 18 + n % 3;
    for (int k = 0; k < K; ++k)
        for (int n = 0; n < N; ++n) b[(size_t)k * N + n] = enc(nd(rng) * std::ldexp(1.0, 12 - bB[n]), bB[n]);
    // B pair words: addend pair (s_b << 15 | (e_b - bB) << 7 per half) and the pair's byte offset
    std::vector<uint2> bpw((size_t)K * N / 2);
    for (int k = 0; k < K; ++k)
        for (int p = 0; p < N / 2; ++p) {
            uint32_t add = 0;
            int code[2];
            for (int h = 0; h < 2; ++h) {
                const Code c = b[(size_t)k * N + 2 * p + h];
                code[h] = c.e ? c.m : 8;
                const uint32_t ad = c.e ? ((uint32_t)(c.s << 15) + (uint32_t)((c.e - bB[2 * p + h]) * 128)) : 0u;
                add |= (ad & 0xFFFFu) << (16 * h);
            }
            bpw[(size_t)k * (N / 2) + p] = make_uint2(add, (uint32_t)((code[0] + 9 * code[1]) * 32));
        }
    // lists: each row's nonzero A elements picked with probability frac, padded per 16-row block
    const int nblk = M / 16;
    std::vector<std::vector<std::pair<int, Code>>> rowl(M);
    std::vector<Code> arow(K);
    size_t entries = 0;
    for (int m = 0; m < M; ++m) {
        for (int k = 0; k < K; ++k) {
            const Code c = enc(std::max(nd(rng), 0.0) * std::ldexp(1.0, 15 - bA - 3), bA);
            if (c.e && ud(rng) < frac) rowl[m].push_back({k, c});
        }
        entries += rowl[m].size();
    }
    std::vector<int> roff(nblk), rounds(nblk);
    size_t tot = 0, slots = 0;
    for (int bk = 0; bk < nblk; ++bk) {
        size_t mx = 0;
        for (int r = 0; r < 16; ++r) mx = std::max(mx, rowl[16 * bk + r].size());
        rounds[bk] = (int)((mx + 7) / 8);
        roff[bk] = (int)tot;
        tot += rounds[bk];
        slots += (size_t)rounds[bk] * 8 * 16;
    }
    auto word = [&](Code c) -> uint32_t {  // cvt scale 2^(7 - bR - (e_a - bA)), m_a * 4, sign
        const int se = 127 + 7 - bR - (c.e - bA);
        return ((uint32_t)se << 23) | (uint32_t)(c.m * 4) | (c.s ? 0x20u : 0u);
    };
    std::vector<uint4> lists(tot * 64);
    for (int bk = 0; bk < nblk; ++bk)
        for (int rd = 0; rd < rounds[bk]; ++rd)
            for (int g = 0; g < 4; ++g)
                for (int r = 0; r < 16; ++r) {
                    const auto &L = rowl[16 * bk + r];
                    const int s0 = 8 * rd + 2 * g, s1 = s0 + 1;
                    uint4 e = make_uint4(0, ZERO_WORD, 0, ZERO_WORD);
                    if (s0 < (int)L.size()) e.x = L[s0].first, e.y = word(L[s0].second);
                    if (s1 < (int)L.size()) e.z = L[s1].first, e.w = word(L[s1].second);
                    lists[((size_t)roff[bk] + rd) * 64 + g * 16 + r] = e;
                }
    printf("M %d N %d K %d  listed %.4f of the A elements, slot efficiency %.3f\n", M, N, K,
           (double)entries / ((double)M * K), (double)entries / (double)slots);
    // windowed lists (per block and K window of KWIN)
    constexpr int KWIN = 256;
    const int nw = K / KWIN;
    std::vector<int> roff2(nblk * nw), rounds2(nblk * nw);
    size_t tot2 = 0, slots2 = 0;
    std::vector<std::vector<std::pair<int, Code>>> perw(16);
    std::vector<uint4> lists2;
    for (int bk = 0; bk < nblk; ++bk)
        for (int w = 0; w < nw; ++w) {
            size_t mx = 0;
            for (int r = 0; r < 16; ++r) {
                perw[r].clear();
                for (const auto &en : rowl[16 * bk + r])
                    if (en.first / KWIN == w) perw[r].push_back(en);
                mx = std::max(mx, perw[r].size());
            }
            const int nr = (int)((mx + 7) / 8);
            roff2[bk * nw + w] = (int)tot2;
            rounds2[bk * nw + w] = nr;
            tot2 += nr;
            slots2 += (size_t)nr * 128;
            for (int rd = 0; rd < nr; ++rd)
                for (int g = 0; g < 4; ++g)
                    for (int r = 0; r < 16; ++r) {
                        const auto &Lr = perw[r];
                        const int s0 = 8 * rd + 2 * g, s1 = s0 + 1;
                        uint4 e = make_uint4(0, ZERO_WORD, 0, ZERO_WORD);
                        if (s0 < (int)Lr.size()) e.x = Lr[s0].first - w * KWIN, e.y = word(Lr[s0].second);
                        if (s1 < (int)Lr.size()) e.z = Lr[s1].first - w * KWIN, e.w = word(Lr[s1].second);
                        lists2.push_back(e);
                    }
        }
    // (lists2 is filled in (block, window, round, g, r16) order, matching roff2)
    printf("windowed (KW %d): slot efficiency %.3f\n", KWIN, (double)entries / (double)slots2);
    uint4 *dl;
    int *dro, *drn;
    uint2 *db;
    uint32_t *dlut;
    float *dC;
    CK(hipMalloc(&dl, lists.size() * 16));
    CK(hipMalloc(&dro, nblk * 4));
    CK(hipMalloc(&drn, nblk * 4));
    CK(hipMalloc(&db, bpw.size() * 8));
    CK(hipMalloc(&dlut, lut.size() * 4));
    CK(hipMalloc(&dC, (size_t)M * N * 4));
    CK(hipMemcpy(dl, lists.data(), lists.size() * 16, hipMemcpyHostToDevice));
    CK(hipMemcpy(dro, roff.data(), nblk * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(drn, rounds.data(), nblk * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, bpw.data(), bpw.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dlut, lut.data(), lut.size() * 4, hipMemcpyHostToDevice));
    uint4 *dl2;
    int *dro2, *drn2;
    CK(hipMalloc(&dl2, lists2.size() * 16 + 16));
    CK(hipMalloc(&dro2, roff2.size() * 4));
    CK(hipMalloc(&drn2, rounds2.size() * 4));
    CK(hipMemcpy(dl2, lists2.data(), lists2.size() * 16, hipMemcpyHostToDevice));
    CK(hipMemcpy(dro2, roff2.data(), roff2.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(drn2, rounds2.data(), rounds2.size() * 4, hipMemcpyHostToDevice));
    const float outscale = (float)std::ldexp(1.0, 7 - bR);
    const dim3 grid(nblk, N / 64);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double prods = (double)entries * N;
    std::vector<float> C((size_t)M * N);
    int bad = 0;
    for (int form = 1; form <= 2; ++form) {
        if (form == 2 && K % KWIN) continue;
        auto launch = [&]() {
            if (form == 1)
                hipLaunchKernelGGL(small_rows, grid, dim3(256), 0, 0, dl, dro, drn, db, dlut, dC, N, outscale);
            else
                hipLaunchKernelGGL(small_win<KWIN>, grid, dim3(256), 0, 0, dl2, dro2, drn2, db, dlut, dC, N, K,
                                   outscale);
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
        printf("%s: %.3f ms, %.2f T listed products/s\n",
               form == 1 ? "small-row kernel (B pair words from L2)" : "windowed small-row kernel (B window in LDS)", ms,
               prods / ms / 1e9);
        CK(hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost));
        int bd = 0, checked = 0, nonfinite = 0;
        double worst = 0;
        for (int t = 0; t < 64; ++t) {
            const int m = (int)((t * 2654435761u) % (unsigned)M);
            for (int n = 0; n < N; ++n) {
                double sum = 0, sa = 0;
                for (const auto &en : rowl[m]) {
                    const Code ca = en.second, cb = b[(size_t)en.first * N + n];
                    if (!cb.e) continue;
                    const double v = ((1 + ca.m / 8.0) * (1 + cb.m / 8.0) - T[ca.m][cb.m] / 8.0) *
                                     std::ldexp(1.0, ca.e - bA + cb.e - bB[n]) * ((ca.s ^ cb.s) ? -1 : 1);
                    const double q = q_r(v, bR);
                    sum += q;
                    sa += std::fabs(q);
                }
                const double got = C[(size_t)m * N + n];
                if (!std::isfinite(got)) ++nonfinite;
                const double dd = std::fabs(got - sum);
                worst = std::max(worst, dd / (sa + 1e-30));
                bd += !(dd <= 1e-5 * sa + 1e-30);
                ++checked;
            }
        }
        printf("  check: %d of %d sampled outputs outside 1e-5 sum|term| (%d non-finite, worst rel %.3g)\n", bd,
               checked, nonfinite, worst);
        bad += bd;
    }
    return bad ? 1 : 0;
}
