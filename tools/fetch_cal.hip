// fetch_cal.hip -- calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the access widths the
// approx GEMM uses (MI355X_MICROARCH.md, HBM section: "other access widths are uncalibrated").
// Streams a 1 GiB buffer (past the 256 MiB Infinity Cache) through buffer loads of 4 B / lane
// (the A-word gather's width) and 16 B / lane (the B words'), and writes 256 MiB with 16 B / lane
// and 4 B / lane stores.  Each kernel is its own dispatch: compare FETCH_SIZE x 1024 (and
// WRITE_SIZE x 1024) with the byte counts printed here.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/fetch_cal tools/fetch_cal.hip
//   rocprofv3 --kernel-trace --pmc FETCH_SIZE -d out -o run -- tools/fetch_cal   (then WRITE_SIZE)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__global__ void read_b32(const uint32_t *p, int64_t n, uint32_t *out) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(p), (short)0, -1, 0x00020000);
    uint32_t acc = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int64_t base = (i - threadIdx.x) * 4;  // the wave-uniform part goes into soffset
        acc ^= __builtin_amdgcn_raw_buffer_load_b32(r, (int)(threadIdx.x * 4), (int)base, 0);
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void read_b128(const uint32_t *p, int64_t n16, uint32_t *out) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(p), (short)0, -1, 0x00020000);
    uint32_t acc = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
        const int64_t base = (i - threadIdx.x) * 16;
        const uint4 v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(threadIdx.x * 16), (int)base, 0));
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void write_b128(uint4 *p, int64_t n16) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
        p[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

__global__ void write_b32(uint32_t *p, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = (uint32_t)i;
}

int main() {
    const int64_t rbytes = 1ll << 30, wbytes = 1ll << 28;
    uint32_t *buf, *out;
    if (hipMalloc(&buf, rbytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    hipMemset(buf, 1, rbytes);
    hipDeviceSynchronize();
    const int blocks = 256 * 8;
    read_b32<<<blocks, 256>>>(buf, rbytes / 4, out);
    read_b128<<<blocks, 256>>>(buf, rbytes / 16, out);
    write_b128<<<blocks, 256>>>(reinterpret_cast<uint4 *>(buf), wbytes / 16);
    write_b32<<<blocks, 256>>>(buf + wbytes / 4, wbytes / 4);
    hipDeviceSynchronize();
    printf("read_b32 %lld B, read_b128 %lld B, write_b128 %lld B, write_b32 %lld B\n", (long long)rbytes,
           (long long)rbytes, (long long)wbytes, (long long)wbytes);
    return 0;
}
