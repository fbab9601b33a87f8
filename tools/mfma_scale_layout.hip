// Probe (tools/, not product): which MX scale block and which scale lane
// v_mfma_scale_f32_16x16x128_f8f6f4 applies to byte i of lane l of its B operand.
// Each wave runs one experiment: B = 1.0 (e4m3) only at (lane lb, byte ib), A = 1.0 everywhere,
// scale_b of lane l = 2^(l >> 4) (E8M0 127 + (l >> 4)), scale_a = 1.  D[r][c] (lane c + 16 q,
// reg r: row 4q + r) = 2^(the scale group of the lane whose scale the hardware used) for the
// column holding the byte, 0 elsewhere.  Prints, per experiment, the nonzero D entries.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

__global__ void probe(float *out, const int *lbs, const int *ibs) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int lb = lbs[w], ib = ibs[w];
    v8i a, b;
    for (int v = 0; v < 8; ++v) {
        a[v] = 0x38383838;
        b[v] = 0;
    }
    if (lane == lb) b[ib >> 2] = 0x38 << (8 * (ib & 3));
    v4f d = {0, 0, 0, 0};
    d = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, d, 0, 0, 0, 127, 0, 127 + (lane >> 4));
    for (int r = 0; r < 4; ++r) out[(w * 64 + lane) * 4 + r] = d[r];
}

int main() {
    const int lbs_h[16] = {0, 0, 0, 0, 0, 16, 16, 16, 32, 32, 48, 48, 5, 5, 37, 37};
    const int ibs_h[16] = {0, 8, 15, 16, 31, 0, 16, 31, 0, 16, 0, 16, 0, 16, 0, 16};
    int *lbs, *ibs;
    float *out;
    hipMalloc(&lbs, 64);
    hipMalloc(&ibs, 64);
    hipMalloc(&out, 16 * 64 * 4 * 4);
    hipMemcpy(lbs, lbs_h, 64, hipMemcpyHostToDevice);
    hipMemcpy(ibs, ibs_h, 64, hipMemcpyHostToDevice);
    probe<<<1, 1024>>>(out, lbs, ibs);
    static float h[16 * 64 * 4];
    hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
    for (int w = 0; w < 16; ++w) {
        printf("B byte (lane %2d, byte %2d):", lbs_h[w], ibs_h[w]);
        float v = 0;
        int cnt = 0, col = -1;
        for (int l = 0; l < 64; ++l)
            for (int r = 0; r < 4; ++r)
                if (h[(w * 64 + l) * 4 + r] != 0) {
                    v = h[(w * 64 + l) * 4 + r];
                    col = l & 15;
                    ++cnt;
                }
        printf(" %d nonzero outputs, column %d, value %g (scale lane group %d)\n", cnt, col, v,
               v > 0 ? (int)__builtin_log2(v) : -1);
    }
    return 0;
}
