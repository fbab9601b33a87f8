// Probe (tools/, not product): which MX scale lane v_mfma_scale_f32_16x16x128_f8f6f4 applies to
// byte i of lane l of its A operand (the B-side probe is mfma_scale_layout.hip).
// Each wave runs one experiment: A = 1.0 (e4m3) only at (lane la, byte ia), B = 1.0 everywhere,
// scale_a of lane l = 2^(l >> 4) (E8M0 127 + (l >> 4)), scale_b = 1.  The nonzero D entries sit
// in row (la & 15) and have the value 2^(the lane group whose scale the hardware used).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

__global__ void probe(float *out, const int *las, const int *ias) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int la = las[w], ia = ias[w];
    v8i a, b;
    for (int v = 0; v < 8; ++v) {
        b[v] = 0x38383838;
        a[v] = 0;
    }
    if (lane == la) a[ia >> 2] = 0x38 << (8 * (ia & 3));
    v4f d = {0, 0, 0, 0};
    d = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, d, 0, 0, 0, 127 + (lane >> 4), 0, 127);
    for (int r = 0; r < 4; ++r) out[(w * 64 + lane) * 4 + r] = d[r];
}

int main() {
    const int n = 16;
    const int las_h[n] = {0, 0, 0, 0, 16, 16, 32, 32, 48, 48, 5, 21, 37, 53, 5, 53};
    const int ias_h[n] = {0, 15, 16, 31, 0, 16, 0, 16, 0, 16, 0, 0, 0, 0, 31, 31};
    int *las, *ias;
    float *out;
    hipMalloc(&las, 64);
    hipMalloc(&ias, 64);
    hipMalloc(&out, n * 64 * 4 * 4);
    hipMemcpy(las, las_h, 64, hipMemcpyHostToDevice);
    hipMemcpy(ias, ias_h, 64, hipMemcpyHostToDevice);
    probe<<<1, 64 * n>>>(out, las, ias);
    static float h[n * 64 * 4];
    hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
    for (int w = 0; w < n; ++w) {
        printf("A byte (lane %2d, byte %2d):", las_h[w], ias_h[w]);
        float v = 0;
        int cnt = 0, row = -1;
        for (int l = 0; l < 64; ++l)
            for (int r = 0; r < 4; ++r)
                if (h[(w * 64 + l) * 4 + r] != 0) {
                    v = h[(w * 64 + l) * 4 + r];
                    row = 4 * (l >> 4) + r;
                    ++cnt;
                }
        printf(" %d nonzero outputs, row %d, value %g (scale lane group %d)\n", cnt, row, v,
               v > 0 ? (int)__builtin_log2(v) : -1);
    }
    return 0;
}
