// Timing harness for the numpy-stream jump kernels (python-raytracer_amd/csrc/rt_mt_kernel.h):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -x hip tools/mt_jump_bench.cpp -I python-raytracer_amd/csrc \
//         -o tools/_build/mt_jump_bench && tools/_build/mt_jump_bench [bands] [parts]
// Times (HIP events, median of 20): k_mt_y; k_mt_jump over `bands` band segments without and with the
// end block; the end block alone; k_mt_gen over the bands.  Checks one jumped window against the
// serial scheme (rt_mt.h jump_serial).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rt_mt_kernel.h"

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                   \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

using namespace rtmt_dev;

template <class F>
float time_ms(F launch) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> v;
    for (int i = 0; i < 21; ++i) {
        CK(hipEventRecord(a, 0));
        launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (i) v.push_back(ms);
    }
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char** argv) {
    const int nb = argc > 1 ? atoi(argv[1]) : 204;
    const int64_t band = 8 * 1920;  // doubles of one 8-row band at 1080p
    std::vector<uint32_t> key(rtmt::N);
    uint32_t s = 5489u;
    for (int i = 0; i < rtmt::N; ++i) key[i] = s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)i;
    std::vector<int64_t> bands(4 * nb);
    std::vector<uint32_t> polys((size_t)nb * rtmt::N);
    for (int b = 0; b < nb; ++b) {
        bands[4 * b] = (int64_t)(b + 1) * 8 * band;  // every 8th band
        bands[4 * b + 1] = band;
        bands[4 * b + 2] = 0;
        bands[4 * b + 3] = bands[4 * b];  // (stored in the frame's layout: compact = 0)
        std::vector<uint32_t> p = rtmt::xpow_mod((uint64_t)(2 * bands[4 * b] - 1));
        std::copy(p.begin(), p.end(), polys.begin() + (size_t)b * rtmt::N);
    }
    const int64_t n_words = 2 * (bands[4 * nb - 4] + band) + 4000;
    std::vector<uint32_t> endp = rtmt::xpow_mod(rtmt::end_jump(n_words));
    uint32_t *dkey, *dy, *dyn, *dwin, *dpoly, *dend, *ddump, *dacc;
    int64_t* dbands;
    double* dout;
    CK(hipMalloc(&dkey, rtmt::N * 4));
    CK(hipMalloc(&dy, MT_YBLOCKS * rtmt::N * 4));
    CK(hipMalloc(&dyn, MT_YBLOCKS * rtmt::N * 4));
    CK(hipMalloc(&dwin, (size_t)(nb + 1) * rtmt::N * 4));
    CK(hipMalloc(&dpoly, polys.size() * 4));
    CK(hipMalloc(&dend, rtmt::N * 4));
    CK(hipMalloc(&ddump, rtmt::N * 4));
    CK(hipMalloc(&dacc, (rtmt::N + 1) * 4));  // end accumulator + counter (zero between uses)
    CK(hipMemset(dacc, 0, (rtmt::N + 1) * 4));
    CK(hipMalloc(&dbands, bands.size() * 8));
    CK(hipMalloc(&dout, (size_t)(n_words / 2 + 1) * 8));
    CK(hipMemcpy(dkey, key.data(), rtmt::N * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dpoly, polys.data(), polys.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dend, endp.data(), rtmt::N * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dbands, bands.data(), bands.size() * 8, hipMemcpyHostToDevice));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_mt_jump), hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)MT_LDS_BYTES));
    MtArgs A{};
    A.key = dkey;
    A.tab = dpoly;
    A.bands = dbands;
    A.out = dout;
    A.words = n_words;
    A.n_out = INT64_MAX;
    A.pos = 624;
    A.y = dy;
    A.key_in_win = 1;
    const int64_t abs_end = A.pos + n_words;
    A.dump_at = ((abs_end + rtmt::N - 1) / rtmt::N - 1) * rtmt::N;
    A.end_at = (int64_t)rtmt::end_jump(n_words);
    A.dump_dst = ddump;
    A.end_acc = dacc;
    A.end_cnt = dacc + rtmt::N;
    const int P = argc > 2 ? atoi(argv[2]) : MT_MAX_PARTS;
    A.parts = P;
    const size_t LDS = mt_jump_lds_bytes(P);
    float t_y = time_ms([&] { hipLaunchKernelGGL(k_mt_y, dim3(1), dim3(MT_THREADS), 0, 0, (const uint32_t*)dkey, dy); });
    float t_j = time_ms([&] { hipLaunchKernelGGL(k_mt_jump, dim3(nb * P), dim3(MT_THREADS), LDS, 0, A, dwin); });
    MtArgs E = A;
    E.end_poly = dend;
    E.y_next = dyn;
    float t_je = time_ms([&] { hipLaunchKernelGGL(k_mt_jump, dim3((nb + 1) * P), dim3(MT_THREADS), LDS, 0, E, dwin); });
    MtArgs E1 = E;
    E1.bands = nullptr;  // one unit: only the end window (no band segments)
    float t_e = time_ms([&] { hipLaunchKernelGGL(k_mt_jump, dim3(P), dim3(MT_THREADS), LDS, 0, E1, dwin); });
    MtArgs E2 = E1;
    E2.y_next = nullptr;
    float t_e2 = time_ms([&] { hipLaunchKernelGGL(k_mt_jump, dim3(P), dim3(MT_THREADS), LDS, 0, E2, dwin); });
    MtArgs G = A;
    G.dump_dst = nullptr;
    float t_g = time_ms(
        [&] { hipLaunchKernelGGL(k_mt_gen<MT_GEN_THREADS>, dim3(nb), dim3(MT_GEN_THREADS), 0, 0, G, dwin); });
    // check band 0's window against the serial jump (windows are XOR-accumulated: zero them first)
    CK(hipMemset(dwin + rtmt::N, 0, (size_t)nb * rtmt::N * 4));
    hipLaunchKernelGGL(k_mt_jump, dim3(nb * P), dim3(MT_THREADS), LDS, 0, A, dwin);
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> w(rtmt::N), ref(rtmt::N);
    CK(hipMemcpy(w.data(), dwin + rtmt::N, rtmt::N * 4, hipMemcpyDeviceToHost));
    rtmt::jump_serial(key.data(), polys.data(), ref.data());
    int bad = 0;
    for (int m = 1; m < rtmt::N; ++m) bad += w[m] != ref[m];
    printf("bands %d: k_mt_y %.1f us, jump %.1f us, jump+end %.1f us, end block alone %.1f us (without y_next %.1f), "
           "gen %.1f us; window check %s\n",
           nb, 1e3 * t_y, 1e3 * t_j, 1e3 * t_je, 1e3 * t_e, 1e3 * t_e2, 1e3 * t_g, bad ? "FAIL" : "ok");
    return bad ? 1 : 0;
}
