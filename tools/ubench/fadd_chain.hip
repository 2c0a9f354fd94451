// Microbenchmark: cycles per dependent f64 add (ZnS chain model).  One launch per mode; each
// wave runs `n` dependent adds on one accumulator; clock64() brackets the loop.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void chain_reg(double *out, const double *in, int n, long long *cyc) {
    double acc = 0.0, x = in[threadIdx.x & 63];
    const long long t0 = clock64();
#pragma unroll 16
    for (int i = 0; i < n; ++i) acc += x;
    const long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}
__global__ void chain_lds(double *out, const double *in, int n, long long *cyc) {
    __shared__ double s[16][34];
    const int g = threadIdx.x & 15, q = threadIdx.x >> 4;
    for (int i = g; i < 34; i += 16) s[q][i] = in[i];
    __syncthreads();
    double acc = 0.0;
    const long long t0 = clock64();
    for (int i = 0; i < n; i += 32) {
        if (g == 0) {
            const double2 *v2 = reinterpret_cast<const double2 *>(s[q]);
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const double2 v = v2[x];
                acc += v.x;
                acc += v.y;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    const long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

// the same with the 16 reads forced ahead of the 32 adds (sched_barrier between the phases)
__global__ void chain_lds_ahead(double *out, const double *in, int n, long long *cyc) {
    __shared__ double s[16][34];
    const int g = threadIdx.x & 15, q = threadIdx.x >> 4;
    for (int i = g; i < 34; i += 16) s[q][i] = in[i];
    __syncthreads();
    double acc = 0.0;
    const long long t0 = clock64();
    for (int i = 0; i < n; i += 32) {
        if (g == 0) {
            const double2 *v2 = reinterpret_cast<const double2 *>(s[q]);
            double2 v[16];
#pragma unroll
            for (int x = 0; x < 16; ++x) v[x] = v2[x];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                acc += v[x].x;
                acc += v[x].y;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    const long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

int main() {
    const int n = 1 << 18;
    double *in, *out;
    long long *cyc;
    hipMalloc(&in, 64 * 8);
    hipMalloc(&out, 1 << 24);
    hipMalloc(&cyc, 1 << 20);
    std::vector<double> h(64, 1e-3);
    hipMemcpy(in, h.data(), 64 * 8, hipMemcpyHostToDevice);
    for (int mode = 0; mode < 3; ++mode)
        for (int threads : {64, 256, 1024}) {
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(e0);
                if (mode == 0) hipLaunchKernelGGL(chain_reg, dim3(1), dim3(threads), 0, 0, out, in, n, cyc);
                else if (mode == 1) hipLaunchKernelGGL(chain_lds, dim3(1), dim3(threads), 0, 0, out, in, n, cyc);
                else hipLaunchKernelGGL(chain_lds_ahead, dim3(1), dim3(threads), 0, 0, out, in, n, cyc);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
            }
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            long long c = 0;
            hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            printf("%s threads=%4d  %.3f ms  %.2f ns/add  %.2f clock64/add\n", mode == 2 ? "lds_ahead" : mode ? "lds" : "reg", threads, ms,
                   ms * 1e6 / n, (double)c / n);
        }
    return 0;
}
