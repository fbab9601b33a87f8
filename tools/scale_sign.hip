// scale_sign.hip -- does v_cvt_scalef32_pk_fp8_bf16 use the scale operand's sign bit (and its
// mantissa bits)?  Prints the fp8 bytes for a few bf16 pairs under scales +-2^e, with and without
// low mantissa bits set.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/scale_sign tools/scale_sign.hip && tools/scale_sign
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

typedef short s2 __attribute__((ext_vector_type(2)));

__global__ void k(const uint32_t *pairs, const uint32_t *scales, uint32_t *out, int np, int ns) {
    const int i = threadIdx.x;
    if (i >= np * ns) return;
    const uint32_t v = pairs[i / ns];
    const float sc = __uint_as_float(scales[i % ns]);
    s2 cv = {0, 0};
    asm volatile("v_cvt_scalef32_pk_fp8_bf16 %0, %1, %2" : "+v"(cv) : "v"(v), "v"(sc));
    out[i] = (uint32_t)(uint16_t)cv.x;
}

int main() {
    // bf16 pairs (lo, hi): 1.5 / -1.5, 0.3125 / 3.0, tiny / 100
    const uint32_t pairs[] = {0xBFC03FC0u, 0x40403EA0u, 0x42C83A80u};
    const uint32_t scales[] = {0x3F800000u, 0xBF800000u, 0x40000000u, 0xC0000000u, 0x3F800078u, 0x3F800000u | 0x80000000u | 0x78u};
    const int np = 3, ns = 6;
    uint32_t *dp, *ds, *dout;
    hipMalloc(&dp, sizeof(pairs));
    hipMalloc(&ds, sizeof(scales));
    hipMalloc(&dout, 4 * np * ns);
    hipMemcpy(dp, pairs, sizeof(pairs), hipMemcpyHostToDevice);
    hipMemcpy(ds, scales, sizeof(scales), hipMemcpyHostToDevice);
    k<<<1, 64>>>(dp, ds, dout, np, ns);
    uint32_t out[np * ns];
    hipMemcpy(out, dout, sizeof(out), hipMemcpyDeviceToHost);
    for (int p = 0; p < np; ++p)
        for (int s = 0; s < ns; ++s)
            printf("pair %08x scale %08x -> fp8 lo %02x hi %02x\n", pairs[p], scales[s], out[p * ns + s] & 0xFF,
                   (out[p * ns + s] >> 8) & 0xFF);
    return 0;
}
