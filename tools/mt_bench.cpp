// Stand-alone timing + correctness harness for k_mt_round (python-raytracer_amd/csrc/rt_mt_kernel.h):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -x hip tools/mt_bench.cpp -I python-raytracer_amd/csrc \
//         -o tools/_build/mt_bench && tools/_build/mt_bench [segments] [plane] [plane_mask]
// Runs of up to 3 segments are checked double by double against the serial scheme (rt_mt.h); every
// run times one launch of `segments` segments (HIP events, median of 20).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rt_mt_kernel.h"

#ifndef MT_GEN_THREADS
#define MT_GEN_THREADS rtmt_dev::MT_GEN_THREADS
#endif

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                   \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

int main(int argc, char** argv) {
    const int segs = argc > 1 ? atoi(argv[1]) : 222;
    const int64_t plane = argc > 2 ? atoll(argv[2]) : 0;
    const int mask = argc > 3 ? atoi(argv[3]) : 15;
    // an arbitrary full key window (numpy's init_genrand(5489) recurrence), position 624
    std::vector<uint32_t> key(rtmt::N);
    key[0] = 5489u;
    for (int i = 1; i < rtmt::N; ++i) key[i] = 1812433253u * (key[i - 1] ^ (key[i - 1] >> 30)) + (uint32_t)i;
    const int pos = rtmt::N;
    const int64_t n_out = (int64_t)segs * rtmt::L / 2 - 7;
    const rtmt::Plan P = rtmt::make_plan(pos, 2 * n_out);
    if (P.rounds.size() != 1) {
        fprintf(stderr, "one round only\n");
        return 1;
    }
    const rtmt::Round& R = P.rounds[0];
    uint32_t *d_key, *d_tab, *d_dump, *d_win;
    double* d_out;
    CK(hipMalloc(&d_key, rtmt::N * 4));
    CK(hipMalloc(&d_tab, rtmt::TABLE_WORDS * 4));
    CK(hipMalloc(&d_dump, rtmt::N * 4));
    CK(hipMalloc(&d_win, (size_t)rtmt::SEGS * rtmt::N * 4));
    CK(hipMalloc(&d_out, n_out * 8));
    CK(hipMemcpy(d_key, key.data(), rtmt::N * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_tab, rtmt::tables_flat(), rtmt::TABLE_WORDS * 4, hipMemcpyHostToDevice));
    CK(hipMemset(d_out, 0, n_out * 8));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&rtmt_dev::k_mt_jump),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)rtmt_dev::MT_LDS_BYTES));
    rtmt_dev::MtArgs A{};
    A.key = d_key;
    A.tab = d_tab;
    A.out = d_out;
    A.dump_dst = d_dump;
    A.words = R.words;
    A.double_base = R.double_base;
    A.n_out = n_out;
    A.dump_at = R.dump_at;
    A.pos = R.pos;
    A.plane = plane;
    A.plane_mask = mask;
    auto launch = [&] {
        if (R.nseg > 1)
            hipLaunchKernelGGL(rtmt_dev::k_mt_jump, dim3(R.nseg - 1), dim3(rtmt_dev::MT_THREADS), rtmt_dev::MT_LDS_BYTES, 0,
                               A, d_win);
        hipLaunchKernelGGL(rtmt_dev::k_mt_gen<MT_GEN_THREADS>, dim3(R.nseg), dim3(MT_GEN_THREADS), 0, 0, A,
                           (const uint32_t*)d_win);
    };
    launch();
    CK(hipDeviceSynchronize());
    // correctness (runs of up to 3 segments): every stored double vs the serial scheme (rt_mt.h)
    int bad = 0;
    if (segs <= 3) {
        std::vector<double> got(n_out), want(n_out);
        CK(hipMemcpy(got.data(), d_out, n_out * 8, hipMemcpyDeviceToHost));
        std::vector<uint32_t> ko(rtmt::N), kd(rtmt::N);
        int po = 0;
        rtmt::uniforms_serial(key.data(), pos, n_out, 0, want.data(), ko.data(), &po);
        for (int64_t d = 0; d < n_out; ++d) {
            const bool kept = plane == 0 || ((mask >> ((d / plane) & 3)) & 1);
            if (kept && got[d] != want[d] && bad++ < 5) fprintf(stderr, "mismatch at %lld\n", (long long)d);
        }
        CK(hipMemcpy(kd.data(), d_dump, rtmt::N * 4, hipMemcpyDeviceToHost));
        for (int m = 1; m < rtmt::N; ++m)
            if (kd[m] != ko[m] && bad++ < 5) fprintf(stderr, "final window word %d differs\n", m);
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ms;
    for (int r = 0; r < 20; ++r) {
        CK(hipEventRecord(e0, 0));
        launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float t;
        CK(hipEventElapsedTime(&t, e0, e1));
        ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    printf("segments %d (launched %d) plane %lld mask %d: %.3f ms median, %.3f min; mismatches %d\n", segs, R.nseg,
           (long long)plane, mask, ms[ms.size() / 2], ms[0], bad);
    return bad ? 2 : 0;
}
