// Stable LSD radix sort of (key, value) pairs (pfdr_sort.hpp): the count
// scan and the host driver of the passes.
#include <stdexcept>

#include "pfdr_sort.hpp"

namespace pfdr {

constexpr int kRsIpt = 16;                        // keys per lane per tile
constexpr int kRsTile = kBlock * kRsIpt;          // 4096 keys per tile
constexpr int kRsScanChunk = kBlock * 16;         // counts per scan block

template <typename K>
__global__ __launch_bounds__(kBlock) void k_rs_hist(const K *__restrict__ key, long n, int shift,
                                                    int ntiles, int *__restrict__ hist) {
    __shared__ int cnt[256];
    const int t = threadIdx.x;
    cnt[t] = 0;
    __syncthreads();
    const long base = (long)blockIdx.x * kRsTile;
#pragma unroll
    for (int j = 0; j < kRsIpt; j++) {
        const long i = base + (long)j * kBlock + t;
        if (i < n) atomicAdd(&cnt[(int)((key[i] >> shift) & 255u)], 1);
    }
    __syncthreads();
    hist[(long)t * ntiles + blockIdx.x] = cnt[t];
}

template <typename K>
__global__ __launch_bounds__(kBlock) void k_rs_scatter(const K *__restrict__ kin,
                                                       const unsigned *__restrict__ vin, long n,
                                                       int shift, int ntiles,
                                                       const int *__restrict__ off,
                                                       K *__restrict__ kout,
                                                       unsigned *__restrict__ vout) {
    __shared__ int base[256];
    __shared__ int cnt[kBlock / kWave][256];
    const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
    const long tb = (long)blockIdx.x * kRsTile;
    base[t] = off[(long)t * ntiles + blockIdx.x];
    for (int q = 0; q < kBlock / kWave; q++) cnt[q][t] = 0;
    // the tile's keys and values, loaded up front (kRsIpt loads in flight)
    K k[kRsIpt];
    unsigned v[kRsIpt];
#pragma unroll
    for (int j = 0; j < kRsIpt; j++) {
        const long i = tb + (long)j * kBlock + t;
        if (i < n) { k[j] = kin[i]; v[j] = vin[i]; }
    }
    __syncthreads();
    const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int j = 0; j < kRsIpt; j++) {
        const long i = tb + (long)j * kBlock + t;
        const bool ok = i < n;
        const int d = ok ? (int)((k[j] >> shift) & 255u) : 0;
        // lanes of this wave holding the same digit (valid ones only)
        unsigned long long m = __ballot(ok);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const unsigned long long bb = __ballot((d >> b) & 1);
            m &= ((d >> b) & 1) ? bb : ~bb;
        }
        const int below = __popcll(m & lt);
        if (ok && below == 0) cnt[w][d] = __popcll(m);  // one leader per digit and wave
        __syncthreads();
        if (ok) {
            long pos = (long)base[d] + below;
            for (int q = 0; q < w; q++) pos += cnt[q][d];
            kout[pos] = k[j];
            vout[pos] = v[j];
        }
        __syncthreads();
        int add = 0;
#pragma unroll
        for (int q = 0; q < kBlock / kWave; q++) { add += cnt[q][t]; cnt[q][t] = 0; }
        base[t] += add;
        __syncthreads();
    }
}

// exclusive scan of the counts in place, three launches: chunk sums, their
// scan (one block, any number of chunks), chunk scans + offsets

// exclusive prefix of x over the block's lanes (lane order); all lanes call
__device__ __forceinline__ long long rs_block_excl(long long x, long long *lds /* kBlock/kWave */,
                                                   long long *total) {
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    long long inc = x;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const long long y = __shfl_up(inc, o, kWave);
        if (lane >= o) inc += y;
    }
    if (lane == kWave - 1) lds[w] = inc;
    __syncthreads();
    long long b = 0, tot = 0;
    for (int i = 0; i < kBlock / kWave; i++) {
        if (i < w) b += lds[i];
        tot += lds[i];
    }
    if (total) *total = tot;
    __syncthreads();
    return b + inc - x;
}

__global__ __launch_bounds__(kBlock) void k_rs_chunk_sums(const int *__restrict__ a, long m,
                                                          long long *__restrict__ sums) {
    __shared__ long long lds[kBlock / kWave];
    const long c0 = (long)blockIdx.x * kRsScanChunk;
    long long x = 0;
    for (int j = 0; j < kRsScanChunk / kBlock; j++) {
        const long i = c0 + (long)j * kBlock + threadIdx.x;
        if (i < m) x += a[i];
    }
    long long tot;
    rs_block_excl(x, lds, &tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kBlock) void k_rs_scan_sums(long long *__restrict__ sums, int nc) {
    __shared__ long long lds[kBlock / kWave];
    const int per = (nc + kBlock - 1) / kBlock;
    const int a = threadIdx.x * per, b = min(nc, a + per);
    long long x = 0;
    for (int i = a; i < b; i++) x += sums[i];
    long long run = rs_block_excl(x, lds, nullptr);
    for (int i = a; i < b; i++) {
        const long long y = sums[i];
        sums[i] = run;
        run += y;
    }
}

__global__ __launch_bounds__(kBlock) void k_rs_chunk_scan(int *__restrict__ a, long m,
                                                          const long long *__restrict__ sums) {
    __shared__ long long lds[kBlock / kWave];
    constexpr int P = kRsScanChunk / kBlock;  // consecutive counts per lane
    const long i0 = (long)blockIdx.x * kRsScanChunk + (long)threadIdx.x * P;
    int v[P];
    long long x = 0;
#pragma unroll
    for (int j = 0; j < P; j++) {
        v[j] = (i0 + j < m) ? a[i0 + j] : 0;
        x += v[j];
    }
    long long run = rs_block_excl(x, lds, nullptr) + sums[blockIdx.x];
#pragma unroll
    for (int j = 0; j < P; j++) {
        if (i0 + j < m) a[i0 + j] = (int)run;
        run += v[j];
    }
}

template <typename K>
void radix_sort_pairs_stable(const K *kin, K *kout, const unsigned *vin, unsigned *vout, long n,
                             int bits, hipStream_t s) {
    if (n <= 0) return;
    if (n >= (1L << 31)) throw std::runtime_error("radix_sort_pairs_stable: n must be < 2^31");
    const int maxbits = (int)(8 * sizeof(K));
    if (bits < 1) bits = 1;
    if (bits > maxbits) bits = maxbits;
    const int passes = (bits + 7) / 8;
    const long ntiles = (n + kRsTile - 1) / kRsTile;
    const long m = 256 * ntiles;
    const long nc = (m + kRsScanChunk - 1) / kRsScanChunk;
    DevBuf<int> hist(m);
    DevBuf<long long> sums(nc);
    // ping-pong: the last pass writes kout / vout
    DevBuf<K> kt(passes > 1 ? n : 1);
    DevBuf<unsigned> vt(passes > 1 ? n : 1);
    const K *ksrc = kin;
    const unsigned *vsrc = vin;
    for (int p = 0; p < passes; p++) {
        // pass p writes kout when passes - 1 - p is even
        K *kdst = ((passes - 1 - p) & 1) ? kt.p : kout;
        unsigned *vdst = ((passes - 1 - p) & 1) ? vt.p : vout;
        const int shift = 8 * p;
        k_rs_hist<K><<<(unsigned)ntiles, kBlock, 0, s>>>(ksrc, n, shift, (int)ntiles, hist.p);
        k_rs_chunk_sums<<<(unsigned)nc, kBlock, 0, s>>>(hist.p, m, sums.p);
        k_rs_scan_sums<<<1, kBlock, 0, s>>>(sums.p, (int)nc);
        k_rs_chunk_scan<<<(unsigned)nc, kBlock, 0, s>>>(hist.p, m, sums.p);
        k_rs_scatter<K><<<(unsigned)ntiles, kBlock, 0, s>>>(ksrc, vsrc, n, shift, (int)ntiles,
                                                            hist.p, kdst, vdst);
        PFDR_HIP(hipGetLastError());
        ksrc = kdst;
        vsrc = vdst;
    }
    // temporaries: freed at scope exit, reused only once the stream is idle
}

template void radix_sort_pairs_stable<unsigned>(const unsigned *, unsigned *, const unsigned *,
                                                unsigned *, long, int, hipStream_t);
template void radix_sort_pairs_stable<unsigned long long>(const unsigned long long *,
                                                          unsigned long long *, const unsigned *,
                                                          unsigned *, long, int, hipStream_t);

}  // namespace pfdr

// ---------------------------------------------------------------- C entry --
// the sort behind the incidence CSR, exposed for its own tests (host arrays)
template <typename K>
static int sort_host(const char *fn, int64_t n, K *keys, unsigned *vals, int bits, double *ms) {
    using namespace pfdr;
    try {
        if (n < 0 || n >= (1LL << 31) || (n && (!keys || !vals)))
            return report_error(fn, "invalid argument");
        if (n == 0) return PFDR_OK;
        hipStream_t s = lib_stream();
        DevBuf<K> ki(n), ko(n);
        DevBuf<unsigned> vi(n), vo(n);
        PFDR_HIP(hipMemcpyAsync(ki.p, keys, sizeof(K) * n, hipMemcpyHostToDevice, s));
        PFDR_HIP(hipMemcpyAsync(vi.p, vals, sizeof(unsigned) * n, hipMemcpyHostToDevice, s));
        hipEvent_t e0, e1;
        PFDR_HIP(hipEventCreate(&e0));
        PFDR_HIP(hipEventCreate(&e1));
        PFDR_HIP(hipEventRecord(e0, s));
        radix_sort_pairs_stable<K>(ki.p, ko.p, vi.p, vo.p, (long)n, bits, s);
        PFDR_HIP(hipEventRecord(e1, s));
        PFDR_HIP(hipMemcpyAsync(keys, ko.p, sizeof(K) * n, hipMemcpyDeviceToHost, s));
        PFDR_HIP(hipMemcpyAsync(vals, vo.p, sizeof(unsigned) * n, hipMemcpyDeviceToHost, s));
        PFDR_HIP(hipStreamSynchronize(s));
        float t = 0.f;
        PFDR_HIP(hipEventElapsedTime(&t, e0, e1));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        if (ms) *ms = t;
    } catch (const HipError &h) {
        return report_error(fn, h);
    } catch (const std::exception &ex) {
        return report_error(fn, ex.what());
    }
    return PFDR_OK;
}

extern "C" int pfdr_radix_sort_pairs_u32(int64_t n, uint32_t *keys, uint32_t *vals, int bits,
                                         double *ms) {
    return sort_host<unsigned>("pfdr_radix_sort_pairs_u32", n, keys, vals, bits, ms);
}
extern "C" int pfdr_radix_sort_pairs_u64(int64_t n, uint64_t *keys, uint32_t *vals, int bits,
                                         double *ms) {
    return sort_host<unsigned long long>("pfdr_radix_sort_pairs_u64", n,
                                         reinterpret_cast<unsigned long long *>(keys), vals, bits,
                                         ms);
}
