// Microbenchmark: random dependent 16 B gathers (the walk's access shape).
// Each lane chases a chain: idx = f(load(table[idx])), STEPS loads per lane,
// persistent grid.  Reports loads/s and "line GB/s" for table sizes that fit
// L2 (4 MiB/XCD), the Infinity Cache (256 MiB) and only HBM.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <chrono>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int W>   // W = 16-byte words read per access (1 or 2)
__global__ void __launch_bounds__(256) chase(const uint4* __restrict__ t, uint64_t mask, int steps, uint32_t* out) {
    uint64_t i = ((uint64_t)(blockIdx.x * 256 + threadIdx.x) * 0x9E3779B97F4A7C15ull) & mask;
    uint32_t acc = 0;
    for (int s = 0; s < steps; ++s) {
        uint4 v = t[i * W];
        if (W == 2) { uint4 u = t[i * W + 1]; v.x ^= u.y; }
        acc += v.y;
        i = (uint64_t)(v.x ^ (s * 0x632BE5ABu) ^ (acc << 7)) & mask;
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

__global__ void fill(uint4* t, uint64_t n) {
    uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    for (; i < n; i += (uint64_t)gridDim.x * 256) {
        uint64_t h = i * 0xD6E8FEB86659FD93ull; h ^= h >> 32; h *= 0x9E3779B97F4A7C15ull; h ^= h >> 29;
        t[i] = make_uint4((uint32_t)h, (uint32_t)(h >> 32), (uint32_t)i, 0);
    }
}

// no arguments: the sweep below; "W WAVES MIB": one configuration (for PMC
// passes, so each chase dispatch of the run is the same shape)
int main(int argc, char** argv) {
    int cus = 0; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint64_t maxb = 4ull << 30;
    uint4* t; CK(hipMalloc(&t, maxb));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, t, maxb / 16);
    uint32_t* out; CK(hipMalloc(&out, 64ull << 20));
    CK(hipDeviceSynchronize());
    std::vector<uint64_t> sizes = {2ull << 20, 16ull << 20, 128ull << 20, 512ull << 20, 1ull << 30, 4ull << 30};
    std::vector<int> Ws = {1, 2}, waves = {8, 16, 32};
    if (argc == 4) {
        Ws = {atoi(argv[1])};
        waves = {atoi(argv[2])};
        sizes = {(uint64_t)atoll(argv[3]) << 20};
    }
    for (int W : Ws)
    for (int waves_per_cu : waves)
    for (uint64_t sz : sizes) {
        uint64_t nslots = sz / (16 * W);
        uint64_t mask = 1; while (mask * 2 <= nslots) mask *= 2; mask -= 1;
        int blocks = cus * waves_per_cu / 4, steps = 256;
        auto run = [&]() {
            if (W == 1) hipLaunchKernelGGL(chase<1>, dim3(blocks), dim3(256), 0, 0, t, mask, steps, out);
            else hipLaunchKernelGGL(chase<2>, dim3(blocks), dim3(256), 0, 0, t, mask, steps, out);
        };
        run(); CK(hipDeviceSynchronize());
        hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
        CK(hipEventRecord(a)); for (int r = 0; r < 5; ++r) run(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); ms /= 5;
        double loads = (double)blocks * 256 * steps;
        printf("W=%d x16B waves/CU=%2d table=%6.0f MiB: %7.2f ms  %6.2f G lane-accesses/s  (%.1f ns/access/lane)"
               "  %.0f accesses per dispatch\n",
               W, waves_per_cu, sz / 1048576.0, ms, loads / ms / 1e6, ms * 1e6 / steps, loads);
        fflush(stdout);
    }
    return 0;
}
