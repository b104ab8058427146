// Phase profile of the sequential-rounding sum (pfdr_monosum.hpp) on 10M
// synthetic f32 terms: each kernel timed alone with events, and the walk's
// phases from its compiled-in probes.  Build + run (GPU box):
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off
//         -I cp_pfdr_graph_d1_amd/csrc -o gpurun_out/monoprof tools/monoprof.hip
//   gpurun_out/monoprof [n] [kind]     kind 0: X^2 uniform, 1: log-uniform 1e-20..1e-6
#define PFDR_MONO_PROFILE 1
#include <cmath>
#include <random>
#include <vector>

#include "pfdr_monosum.hpp"

using namespace pfdr;

#define CK(x)                                                             \
    do {                                                                  \
        hipError_t e_ = (x);                                              \
        if (e_ != hipSuccess) {                                           \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
            return 1;                                                     \
        }                                                                 \
    } while (0)

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : 10000000L;
    const int kind = argc > 2 ? atoi(argv[2]) : 0;
    std::mt19937_64 g(3);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    std::vector<float> h(n);
    for (long i = 0; i < n; i++) {
        const double u = U(g);
        h[i] = kind == 0 ? (float)(u * u) : (float)std::exp(std::log(1e-20) + u * std::log(1e14));
    }
    float ref = 0.f;
    for (long i = 0; i < n; i++) ref += h[i];
    float *a, *out;
    void *ws;
    const long nt = (n + MonoTile<float>::TILE - 1) / MonoTile<float>::TILE;
    CK(hipMalloc(&a, n * sizeof(float)));
    CK(hipMalloc(&out, sizeof(float)));
    CK(hipMalloc(&ws, mono_ws_bytes<float>(n, 1)));
    CK(hipMemcpy(a, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
    const MonoWs<float> w(ws, nt, 1);
    hipEvent_t ev[5];
    for (auto &e : ev) CK(hipEventCreate(&e));
    float best[4] = {1e9f, 1e9f, 1e9f, 1e9f};
    for (int rep = 0; rep < 7; rep++) {
        CK(hipEventRecord(ev[0], 0));
        k_mono_tile_sums<float><<<dim3(nt, 1), 256>>>(n, a, 0, w.tsum, nullptr);
        CK(hipEventRecord(ev[1], 0));
        k_mono_predict<float><<<dim3(1, 1), kPredThreads>>>((int)nt, w.tsum, nullptr, 0, w.ebase,
                                                            nullptr);
        CK(hipEventRecord(ev[2], 0));
        k_mono_summaries<float><<<dim3(nt, 1), kMonoThreads>>>(n, a, 0, w.ebase, w.summ, w.subs,
                                                               nullptr);
        CK(hipEventRecord(ev[3], 0));
        k_mono_walk<float><<<dim3(1, 1), kMonoThreads>>>(n, a, 0, (int)nt, w.ebase, w.summ, w.subs,
                                                         nullptr, 0, 0, nullptr, out, nullptr,
                                                         nullptr);
        CK(hipEventRecord(ev[4], 0));
        CK(hipDeviceSynchronize());
        for (int k = 0; k < 4; k++) {
            float ms;
            CK(hipEventElapsedTime(&ms, ev[k], ev[k + 1]));
            best[k] = std::min(best[k], ms);
        }
    }
    float got;
    CK(hipMemcpy(&got, out, sizeof(float), hipMemcpyDeviceToHost));
    int rate_khz = 100000;
    CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
    const double tick_us = 1e3 / rate_khz;
    unsigned long long pr[32];
    CK(hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_mono_prof), sizeof(pr)));
    printf("n %ld kind %d tiles %ld: sum %s (%.9g vs %.9g)\n", n, kind, nt,
           got == ref ? "equal" : "DIFFERS", got, ref);
    const char *nm[4] = {"tile_sums", "predict", "summaries", "walk"};
    for (int k = 0; k < 4; k++) printf("  %-10s %8.1f us (best of 7)\n", nm[k], 1e3 * best[k]);
    const char *ph[11] = {"chain step",   "stage tile",  "sub-chain",   "fine return", "tail",
                          "fine scan",    "barrier A",   "fine total",  "fine exit",   "barrier B",
                          "fine serial"};
    for (int k = 0; k < 11; k++)
        printf("  walk %-11s %6llu x  %8.2f us total  %6.2f us each\n", ph[k], pr[16 + k],
               pr[k] * tick_us, pr[16 + k] ? pr[k] * tick_us / pr[16 + k] : 0.0);
    return 0;
}
