// Experiment: the GPU-side cost of a kernel boundary on one stream (MI355X).
// Back-to-back launches of (a) an empty 1-block kernel, (b) a 2048-block
// kernel touching 8 MB, each with and without a hipEvent pair around every
// launch (what the sessions' per-kernel profiling adds), and (c) the same
// empty launches captured once into a hipGraph and replayed.
//   hipcc --offload-arch=gfx950 -O2 -o tools/exp_launch_gap tools/exp_launch_gap.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_empty(int *p) { if (threadIdx.x == 1023) p[0] = 1; }
__global__ void k_touch(float *p, long n) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = p[i] * 0.5f + 1.0f;
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int *d;
    float *buf;
    const long n = 2 << 20;  // 8 MB
    CK(hipMalloc(&d, 4));
    CK(hipMalloc(&buf, n * 4));
    CK(hipMemset(buf, 0, n * 4));
    const int reps = 2000;
    std::vector<hipEvent_t> ev(2 * reps), evf(2 * reps), evd(2 * reps);
    for (auto &e : ev) CK(hipEventCreate(&e));
    for (auto &e : evf) CK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    for (auto &e : evd) CK(hipEventCreateWithFlags(&e, hipEventReleaseToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<hipEvent_t> *use = &ev;
    auto run = [&](const char *name, int mode, bool events) -> int {
        for (int w = 0; w < 2; w++) {
            CK(hipEventRecord(a, s));
            for (int i = 0; i < reps; i++) {
                if (events) CK(hipEventRecord((*use)[2 * i], s));
                if (mode == 0) k_empty<<<1, 256, 0, s>>>(d);
                else k_touch<<<(int)((n + 255) / 256), 256, 0, s>>>(buf, n);
                if (events) CK(hipEventRecord((*use)[2 * i + 1], s));
            }
            CK(hipEventRecord(b, s));
            CK(hipStreamSynchronize(s));
        }
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("%-40s %8.3f us per launch\n", name, ms * 1e3 / reps);
        return 0;
    };
    if (run("empty, back to back", 0, false)) return 1;
    if (run("empty, event pair per launch", 0, true)) return 1;
    if (run("8 MB touch (8192 blocks)", 1, false)) return 1;
    if (run("8 MB touch, event pair per launch", 1, true)) return 1;
    use = &evf;
    if (run("empty, DisableSystemFence event pair", 0, true)) return 1;
    if (run("8 MB touch, DisableSystemFence pair", 1, true)) return 1;
    use = &evd;
    if (run("empty, ReleaseToDevice event pair", 0, true)) return 1;
    if (run("8 MB touch, ReleaseToDevice pair", 1, true)) return 1;
    {   // are the fence-free timestamps still the kernel's duration?
        float tot = 0;
        for (int i = 0; i < reps; i++) {
            float m = 0;
            CK(hipEventElapsedTime(&m, evd[2 * i], evd[2 * i + 1]));
            tot += m;
        }
        printf("%-40s %8.3f us mean between the pair\n", "ReleaseToDevice: touch duration", tot * 1e3 / reps);
    }
    // graph replay of 100 empty launches
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < 100; i++) k_empty<<<1, 256, 0, s>>>(d);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int w = 0; w < 2; w++) {
        CK(hipEventRecord(a, s));
        for (int i = 0; i < reps / 100; i++) CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(b, s));
        CK(hipStreamSynchronize(s));
    }
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("%-40s %8.3f us per launch\n", "empty, hipGraph of 100", ms * 1e3 / reps);
    // host-side enqueue rate
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < reps; i++) k_empty<<<1, 256, 0, s>>>(d);
    auto t1 = std::chrono::steady_clock::now();
    CK(hipStreamSynchronize(s));
    printf("%-40s %8.3f us per launch\n", "host enqueue (empty)",
           std::chrono::duration<double, std::micro>(t1 - t0).count() / reps);
    return 0;
}
