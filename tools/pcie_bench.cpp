// Device -> pinned host copy rates for a frame's outputs (50 MB linear RGB): one hipMemcpyAsync, the
// same split over 2 / 4 streams, and a copy kernel storing into the pinned buffer.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/pcie_bench.cpp -o tools/_build/pcie_bench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e = (x);                                                \
        if (e != hipSuccess) {                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));         \
            exit(1);                                                       \
        }                                                                  \
    } while (0)

__global__ void k_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

int main() {
    const size_t bytes = 50u << 20;
    void *dev, *host;
    CK(hipMalloc(&dev, bytes));
    CK(hipHostMalloc(&host, bytes, hipHostMallocDefault));
    CK(hipMemset(dev, 1, bytes));
    hipStream_t st[4];
    for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto run = [&](const char* name, int ns, bool kernel) {
        std::vector<float> v;
        for (int it = 0; it < 12; ++it) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a, st[0]));
            for (int k = 1; k < ns; ++k) CK(hipStreamWaitEvent(st[k], a, 0));
            const size_t part = bytes / ns;
            for (int k = 0; k < ns; ++k) {
                char* d = (char*)dev + k * part;
                char* h = (char*)host + k * part;
                if (kernel)
                    hipLaunchKernelGGL(k_copy, dim3(1024), dim3(256), 0, st[k], (const uint4*)d, (uint4*)h, part / 16);
                else
                    CK(hipMemcpyAsync(h, d, part, hipMemcpyDeviceToHost, st[k]));
            }
            for (int k = 1; k < ns; ++k) {
                hipEvent_t ev;
                CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
                CK(hipEventRecord(ev, st[k]));
                CK(hipStreamWaitEvent(st[0], ev, 0));
                CK(hipEventDestroy(ev));
            }
            CK(hipEventRecord(b, st[0]));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (it >= 2) v.push_back(ms);
        }
        std::sort(v.begin(), v.end());
        printf("%-28s %6.2f GB/s (median of %zu, %.3f ms)\n", name, bytes / (v[v.size() / 2] * 1e6), v.size(),
               v[v.size() / 2]);
    };
    run("1 x hipMemcpyAsync", 1, false);
    run("2 streams x hipMemcpyAsync", 2, false);
    run("4 streams x hipMemcpyAsync", 4, false);
    run("copy kernel, 1 stream", 1, true);
    run("copy kernel, 2 streams", 2, true);
    return 0;
}
