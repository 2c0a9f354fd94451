// fetch_calib.hip -- calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// widths the call kernels use (MI355X_MICROARCH.md: "Other access widths are uncalibrated:
// calibrate on a known byte count in your own access pattern").  Each kernel reads (or writes)
// a known number of bytes of a 4 GiB buffer (far beyond the 256 MiB Infinity Cache, touched
// once) in one pattern:
//   stream16     16 B per lane, consecutive lanes consecutive (the scan's key chunks)
//   stream8_nt   8 B per lane, nontemporal (the scan's sum mapQ^2 pairs)
//   stream2_nt   2 B per lane, nontemporal (the scan's u8 k pairs)
//   gather16     16 B per lane at scattered chunks, 3 consecutive chunks per lane (the scan's
//                list pass: a listed task's 1-3 key chunks), each chunk read once
//   store16      16 B per lane stores (rows, queue records)
// Run under `rocprofv3 --pmc FETCH_SIZE` (then WRITE_SIZE) and divide the known bytes printed
// here by the counter's bytes (tools/pmc_calib.py).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHK(x)                                                                   \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
            return 1;                                                            \
        }                                                                        \
    } while (0)

__global__ void stream16(const uint4 *__restrict__ p, size_t n16, uint32_t *__restrict__ out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;   // keeps the loads
}
__global__ void stream8_nt(const uint64_t *__restrict__ p, size_t n8, uint32_t *__restrict__ out) {
    uint64_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n8; i += (size_t)gridDim.x * blockDim.x)
        acc ^= __builtin_nontemporal_load(p + i);
    if ((uint32_t)acc == 0x12345678u) out[0] = (uint32_t)acc;
}
__global__ void stream2_nt(const uint16_t *__restrict__ p, size_t n2, uint32_t *__restrict__ out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x)
        acc ^= __builtin_nontemporal_load(p + i);
    if (acc == 0x12345678u) out[0] = acc;
}
// lane t reads chunks 3j, 3j+1, 3j+2 of group j = perm(t): every chunk once, groups scattered
__global__ void gather16(const uint4 *__restrict__ p, size_t ngroups, uint32_t *__restrict__ out) {
    uint32_t acc = 0;
    for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < ngroups; t += (size_t)gridDim.x * blockDim.x) {
        const size_t j = (t * 2654435761ull) % ngroups;   // a bijection when ngroups is not a multiple of 2654435761's factors
        const uint4 a = p[3 * j], b = p[3 * j + 1], c = p[3 * j + 2];
        acc ^= a.x ^ b.y ^ c.z ^ a.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}
__global__ void store16(uint4 *__restrict__ p, size_t n16) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

int main() {
    const size_t bytes = (size_t)4 << 30;
    void *buf = nullptr;
    uint32_t *out = nullptr;
    CHK(hipMalloc(&buf, bytes));
    CHK(hipMalloc(&out, 64));
    CHK(hipMemset(buf, 1, bytes));
    CHK(hipDeviceSynchronize());
    const dim3 g(256 * 64), b(256);
    // each kernel reads the whole buffer once (gather16: 3 * ngroups chunks); the buffer is
    // rewritten between kernels so no line survives in the Infinity Cache
    const size_t ng = bytes / 48 - 7;   // odd-ish group count (bijective multiplicative hash)
    printf("{\"stream16\": %zu, \"stream8_nt\": %zu, \"stream2_nt\": %zu, \"gather16\": %zu, \"store16\": %zu}\n", bytes,
           bytes, bytes / 8, ng * 48, bytes);
    hipLaunchKernelGGL(stream16, g, b, 0, 0, (const uint4 *)buf, bytes / 16, out);
    CHK(hipMemset(buf, 2, bytes));
    hipLaunchKernelGGL(stream8_nt, g, b, 0, 0, (const uint64_t *)buf, bytes / 8, out);
    CHK(hipMemset(buf, 3, bytes));
    hipLaunchKernelGGL(stream2_nt, g, b, 0, 0, (const uint16_t *)buf, bytes / 8 / 2, out);   // 512 MiB of it
    CHK(hipMemset(buf, 4, bytes));
    hipLaunchKernelGGL(gather16, g, b, 0, 0, (const uint4 *)buf, ng, out);
    CHK(hipMemset(buf, 5, bytes));
    hipLaunchKernelGGL(store16, g, b, 0, 0, (uint4 *)buf, bytes / 16);
    CHK(hipDeviceSynchronize());
    CHK(hipFree(buf));
    CHK(hipFree(out));
    return 0;
}
