// Process-exit cost of a HIP process (what a fresh `popbam` pays after its output): init, then
// allocate DEV_MB of device memory and PIN_MB of pinned host memory in CHUNKS pieces, touch them,
// print the time since start, _exit.  The parent measures exit -> reaped.
// HOST_MB of ordinary heap memory in 20 MB pieces (the feeder's pieces), freed before the exit
// when FREE is 1, else left to the exit.
// usage: exit_teardown DEV_MB PIN_MB CHUNKS [HOST_MB FREE]
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char **argv) {
    const size_t dev_mb = argc > 1 ? std::atol(argv[1]) : 0, pin_mb = argc > 2 ? std::atol(argv[2]) : 0;
    const int chunks = argc > 3 ? std::atoi(argv[3]) : 1;
    const size_t host_mb = argc > 4 ? std::atol(argv[4]) : 0;
    const int do_free = argc > 5 ? std::atoi(argv[5]) : 0;
    const auto t0 = std::chrono::steady_clock::now();
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n < 1) return 2;
    const auto t1 = std::chrono::steady_clock::now();
    std::vector<void *> d, h;
    for (int i = 0; i < chunks; ++i) {
        void *p = nullptr;
        if (dev_mb && hipMalloc(&p, (dev_mb << 20) / chunks) == hipSuccess) {
            (void)hipMemset(p, 1, (dev_mb << 20) / chunks);
            d.push_back(p);
        }
        if (pin_mb && hipHostMalloc(&p, (pin_mb << 20) / chunks, hipHostMallocDefault) == hipSuccess) {
            ((char *)p)[0] = 1;
            h.push_back(p);
        }
    }
    (void)hipDeviceSynchronize();
    std::vector<char *> hp;
    for (size_t m = 0; m < host_mb; m += 20) {
        char *q = (char *)std::malloc(20u << 20);
        for (size_t i = 0; i < (20u << 20); i += 4096) q[i] = 1;
        hp.push_back(q);
    }
    const auto tf = std::chrono::steady_clock::now();
    if (do_free)
        for (char *q : hp) std::free(q);
    const auto t2 = std::chrono::steady_clock::now();
    std::printf("{\"init_s\": %.4f, \"alloc_s\": %.4f, \"free_s\": %.4f, \"exit_epoch\": %.6f}\n",
                std::chrono::duration<double>(t1 - t0).count(), std::chrono::duration<double>(tf - t1).count(),
                std::chrono::duration<double>(t2 - tf).count(),
                std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count());
    std::fflush(stdout);
    _exit(0);
}
