// Shared device/host helpers of the MI355X PFDR library (gfx950 only).
//
// Everything here is written for CDNA4: 64-lane wavefronts, 256-thread
// workgroups (4 waves, one per SIMD), 16-byte per-lane vector memory
// accesses on every streamed array.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "../../include/pfdr_mi355x.h"

namespace pfdr {

constexpr int kBlock = 256;   // threads per workgroup (4 wave64)
constexpr int kWave = 64;

// --------------------------------------------------------------- errors --
struct HipError {
    hipError_t err;
    const char *what;
    int line;
};

#define PFDR_HIP(call)                                                     \
    do {                                                                   \
        hipError_t _e = (call);                                            \
        if (_e != hipSuccess) throw ::pfdr::HipError{_e, #call, __LINE__}; \
    } while (0)

// convert an exception escaping a solver into a C status code
int report_error(const char *fn, const HipError &h);
int report_error(const char *fn, const char *msg);

// ----------------------------------------------------------- real types --
template <typename real> struct Vec;
template <> struct Vec<float> {
    using v2 = float2;
    using v4 = float4;
    static constexpr int kPer16B = 4;
};
template <> struct Vec<double> {
    using v2 = double2;
    using v4 = double4;
    static constexpr int kPer16B = 2;
};

// machine epsilon / huge of the reference (src/PFDR_graph_quadratic_d1_l1.cpp:286-292,
// src/PFDR_graph_quadratic_d1_bounds.cpp:260-278)
template <typename real> struct Lim;
template <> struct Lim<float> {
    static constexpr float eps = 1.19209290e-07f;
    static constexpr float huge = __builtin_huge_valf();
};
template <> struct Lim<double> {
    static constexpr double eps = 2.2204460492503131e-16;
    static constexpr double huge = __builtin_huge_val();
};

// ---------------------------------------------------- loop control block --
// Device-resident iteration state.  The per-iteration kernels return at once
// when `halt` is set, so the host can enqueue iterations in chunks and read
// the state back only between chunks (no per-iteration host round trip).
template <typename real>
struct Ctrl {
    int it;        // completed iterations (reference it_)
    int halt;      // 1: stop issuing updates (stop or reconditioning)
    int stop;      // 1: converged or itMax reached
    int recond;    // 1: reconditioning requested (dif < difRcd)
    int obj_it;    // last iteration index whose objective has been written
    int itMax;
    real dif;      // last iterate evolution (reference dif)
    real difTol;   // compared with dif (squared for the quadratic solvers)
    real difRcd;   // idem, updated by the host after each reconditioning
    real eps;      // denominator floor of the relative evolution
    real c;        // scratch scalar: amplitude of the preconditioner
    int cnt;       // scratch count
};

// ------------------------------------------------------------ reductions --
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Deterministic block sum (fixed tree), result valid in thread 0.
template <typename T>
__device__ __forceinline__ T block_sum(T v, T *lds /* >= kBlock/64 */) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) lds[w] = v;
    __syncthreads();
    T s = T(0);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 0; i < kBlock / kWave; i++) s += lds[i];
    }
    __syncthreads();
    return s;
}

// packed vector of N T (16-byte accesses)
template <typename T, int N>
struct alignas(sizeof(T) * N) Pk { T v[N]; };

// s + q[0] + q[1] + ... + q[m-1], left to right, from LDS.  Two register
// sets A / B of U x 16 bytes: the reads of one set are in flight while the
// other set's values are added, so the dependent add chain (one v_add per
// element) never waits for LDS (LDS ops complete in order: waiting for A
// leaves B's U reads outstanding).
template <typename real>
__device__ __forceinline__ real ordered_add(real s, const real *q, int m) {
    constexpr int W = Vec<real>::kPer16B, U = 8, S = W * U;
    using P = Pk<real, W>;
    const int ns = m / S;  // whole sets
    P A[U], B[U];
    auto ld = [&](P *r, int set) {
#pragma unroll
        for (int u = 0; u < U; u++) r[u] = *reinterpret_cast<const P *>(q + set * S + u * W);
    };
    auto add = [&](const P *r) {
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int k = 0; k < W; k++) s += r[u].v[k];
    };
    if (ns > 0) ld(A, 0);
    int i = 0;
    for (; i + 1 < ns; i += 2) {
        ld(B, i + 1);
        add(A);
        if (i + 2 < ns) ld(A, i + 2);
        add(B);
    }
    if (i < ns) add(A);
    for (int j = ns * S; j < m; j++) s += q[j];
    return s;
}

// XCD-aware block order: the dispatcher deals blocks round-robin over the 8
// XCDs (blocks b, b+8, ... share one L2).  mode 0: identity; 1: each XCD
// gets a CONTIGUOUS eighth of the logical blocks (neighbouring blocks, which
// gather the same neighbour bands of the graph, share an L2); C >= 2: runs
// of C consecutive logical blocks per XCD, the 8 XCDs side by side on a
// window of 8C blocks.  Placement is a speed hint only.  Launch
// xcd_grid(nb, mode) blocks; a block whose logical id is >= nb returns.
__device__ __forceinline__ int xcd_block(int b, int nb, int mode) {
    if (mode == 0) return b;
    if (mode == 1) {
        const int per = (nb + 7) >> 3;
        return (b & 7) * per + (b >> 3);
    }
    const int r = b >> 3;
    return ((r / mode) * 8 + (b & 7)) * mode + r % mode;
}
// chunked mode C of a launch of nb blocks: halved until every XCD gets at
// least 4 runs (small launches must still spread over all 8 XCDs)
inline int xcd_fit(int nb, int mode) {
    if (mode < 2) return mode;
    while (mode >= 2 && nb < 32 * mode) mode >>= 1;
    return mode >= 2 ? mode : 0;
}
inline int xcd_grid(int nb, int mode) {
    const int q = mode <= 1 ? 8 : 8 * mode;
    return mode ? (nb + q - 1) / q * q : nb;
}

inline int grid_for(long n, int per_thread = 1) {
    long t = (n + per_thread - 1) / per_thread;
    long g = (t + kBlock - 1) / kBlock;
    return (int)(g > 0 ? g : 1);
}

// ------------------------------------------------------- device buffers --
// Device memory through a per-process cache (pfdr_runtime.cpp): a freed
// block is kept under its size class and handed out again once the stream
// that freed it is idle, so repeated calls of similar size (cut pursuit's
// reduced problems, a caller's solve loop) skip hipMalloc / hipFree, which
// synchronise the device and cost milliseconds per call.  Bounded by
// PFDR_DEVICE_CACHE_MB (default 2048; 0 disables); on an out-of-memory
// hipMalloc the cache is emptied and the allocation retried.
void *dev_malloc(size_t bytes);
void dev_free(void *p, size_t bytes) noexcept;

// Small pinned host blocks (kPinnedSmall bytes: loop-control mirrors, flags)
// pooled for the process: hipHostMalloc / hipHostFree cost ~30 / ~250 us
// (the free synchronises the device), a large share of a small drop-in call.
// Return a block only once no copy into or out of it is in flight.
constexpr size_t kPinnedSmall = 256;
void *pinned_small_get();
void pinned_small_put(void *p) noexcept;

// RAII device allocation (dev_malloc'd, freed on scope exit).
template <typename T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    explicit DevBuf(size_t count) { alloc(count); }
    void alloc(size_t count) {
        release();
        if (count) p = static_cast<T *>(dev_malloc(count * sizeof(T)));
        n = count;
    }
    void release() {
        if (p) dev_free(p, n * sizeof(T));
        p = nullptr;
        n = 0;
    }
    ~DevBuf() { release(); }
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    T *get() const { return p; }
};

// Library-owned stream of the calling thread's current device, or, inside
// a StreamScope, the stream of the session being driven: every allocation,
// free and copy of a session call is then ordered on the session's stream
// whichever thread makes the call (the device cache's idle test included).
hipStream_t lib_stream();

// Binds the calling thread to a session's device and stream for the
// duration of one C-ABI call (run, result, destroy from any thread).
class StreamScope {
  public:
    StreamScope(hipStream_t s, int device);
    ~StreamScope();
    StreamScope(const StreamScope &) = delete;
    StreamScope &operator=(const StreamScope &) = delete;

  private:
    hipStream_t prev_s_;
    int prev_dev_ = -1, dev_ = -1;
};

// Returns a pinned_small_get() block on scope exit, after synchronising the
// stream that may still copy into it (error paths included).
struct PinnedSmall {
    void *p;
    hipStream_t s;
    explicit PinnedSmall(hipStream_t st) : p(pinned_small_get()), s(st) {}
    ~PinnedSmall() {
        (void)hipStreamSynchronize(s);
        pinned_small_put(p);
    }
    PinnedSmall(const PinnedSmall &) = delete;
    PinnedSmall &operator=(const PinnedSmall &) = delete;
};

// Copies between the caller's host arrays and the device.  A host range of
// at least 1 MiB is pinned (hipHostRegister) for its DMA and unpinned once
// the stream has drained (release(), or the destructor): the runtime's
// pageable path stages through its own buffers at 3-10 GB/s, a pinned DMA
// runs at ~55 GB/s (profiles/r1/r2b_h2d.log).  A range that cannot be
// pinned (already registered, read-only mapping) is copied as before.
class HostPins {
  public:
    explicit HostPins(hipStream_t s = nullptr) : s_(s) {}
    ~HostPins();
    HostPins(const HostPins &) = delete;
    HostPins &operator=(const HostPins &) = delete;
    void set_stream(hipStream_t s) { s_ = s; }
    // asynchronous on the stream; kind: hipMemcpyHostToDevice or DeviceToHost
    void copy(void *dst, const void *src, size_t bytes, hipMemcpyKind kind);
    void release();  // synchronise the stream, unpin everything pinned here

  private:
    hipStream_t s_;
    void *pinned_[64];
    int n_ = 0;
};

// Upload a host array into a fresh device buffer (nullptr stays nullptr).
template <typename T>
void upload(DevBuf<T> &d, const T *h, size_t n, hipStream_t s) {
    if (!h || !n) { d.release(); return; }
    d.alloc(n);
    PFDR_HIP(hipMemcpyAsync(d.p, h, n * sizeof(T), hipMemcpyHostToDevice, s));
}

}  // namespace pfdr
