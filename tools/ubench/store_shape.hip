// Store-shape microbenchmark for the generator's key writes (r05): how fast can HBM take 16 GB
// written (a) by a plain coalesced grid-stride kernel, (b) in the generator's shape -- a wave per
// 64-position block writing rounds of ~1280 contiguous bytes, one full 16-byte-per-lane store and
// one with 16 active lanes per round (buffer stores, idle lanes out of range), (c) the same plus
// a 2-byte store with every lane out of range, (d) rounds of two full stores (2 KiB).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench/store_shape tools/ubench/store_shape.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef __attribute__((ext_vector_type(4))) unsigned int v4u;

__global__ __launch_bounds__(256) void plain_kernel(uint4 *out, size_t nwords) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords; i += stride)
        out[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

// wave w owns [w * rounds * words_per_round, ...) 16-byte words; each round writes
// words_per_round words as ceil(words / 64) stores per lane
template <int kMode>
__global__ __launch_bounds__(256) void shape_kernel(uint16_t *keys, uint32_t rounds, uint32_t wpr, uint32_t nwaves) {
    const uint32_t wave = blockIdx.x * 4u + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    if (wave >= nwaves) return;
    const size_t base_words = (size_t)wave * rounds * wpr;
    const uint32_t bytes = rounds * wpr * 16u;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)(keys + base_words * 8), 0, (int)bytes, 0x00020000);
    for (uint32_t r = 0; r < rounds; ++r) {
        const uint32_t w0 = r * wpr, w1 = w0 + wpr;
        if (kMode == 2) __builtin_amdgcn_raw_buffer_store_b16((uint16_t)r, rs, 0x80000000u, 0, 0);
#pragma unroll
        for (int q = 0; q < (kMode == 3 ? 2 : 2); ++q) {
            const uint32_t W = w0 + lane + 64u * q;
            const bool act = W < w1;
            const v4u v = {W, r, lane, 7u};
            __builtin_amdgcn_raw_buffer_store_b128(v, rs, act ? W * 16u : 0x80000000u, 0, 0);
        }
    }
}

int main() {
    const size_t bytes = 16ull << 30;
    uint16_t *d = nullptr;
    if (hipMalloc(&d, bytes + 4096) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto timeit = [&](const char *name, auto launch, double useful) {
        launch();
        hipDeviceSynchronize();
        float best = 1e30f;
        for (int it = 0; it < 5; ++it) {
            hipEventRecord(a);
            launch();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            if (ms < best) best = ms;
        }
        printf("{\"case\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, best, useful / best / 1e6);
    };
    const size_t nwords = bytes / 16;
    timeit("plain grid-stride b128", [&] { hipLaunchKernelGGL(plain_kernel, dim3(256 * 64), dim3(256), 0, 0, (uint4 *)d, nwords); },
           (double)bytes);
    // generator shape: 24 rounds of 80 words (1280 B) per wave
    const uint32_t rounds = 24, wpr = 80;
    const uint32_t nwaves = (uint32_t)(nwords / ((size_t)rounds * wpr));
    const double useful = (double)nwaves * rounds * wpr * 16.0;
    timeit("rounds of 80 words (64 + 16 lanes)", [&] {
        hipLaunchKernelGGL(shape_kernel<1>, dim3((nwaves + 3) / 4), dim3(256), 0, 0, d, rounds, wpr, nwaves); }, useful);
    timeit("rounds of 80 words + masked b16", [&] {
        hipLaunchKernelGGL(shape_kernel<2>, dim3((nwaves + 3) / 4), dim3(256), 0, 0, d, rounds, wpr, nwaves); }, useful);
    const uint32_t wpr2 = 128, nw2 = (uint32_t)(nwords / ((size_t)rounds * wpr2));
    timeit("rounds of 128 words (64 + 64 lanes)", [&] {
        hipLaunchKernelGGL(shape_kernel<3>, dim3((nw2 + 3) / 4), dim3(256), 0, 0, d, rounds, wpr2, nw2); },
           (double)nw2 * rounds * wpr2 * 16.0);
    const uint32_t wpr3 = 64, nw3 = (uint32_t)(nwords / ((size_t)rounds * wpr3));
    timeit("rounds of 64 words (one full store)", [&] {
        hipLaunchKernelGGL(shape_kernel<1>, dim3((nw3 + 3) / 4), dim3(256), 0, 0, d, rounds, wpr3, nw3); },
           (double)nw3 * rounds * wpr3 * 16.0);
    hipFree(d);
    return 0;
}
