// C entry for the sequential sum of nonnegative terms (pfdr_monosum.hpp):
// the preconditioner's amplitude sum, exposed so that its rounding can be
// checked term by term against a one-thread loop on adversarial inputs.
#include <stdexcept>

#include "pfdr_monosum.hpp"

namespace pfdr {

template <typename real>
static int seqsum_host(const char *fn, int64_t n, const real *a, int mem, real seed, int method,
                       real *out, double *ms) {
    try {
        if (n < 0 || (n && !a) || !out || (mem != PFDR_MEM_HOST && mem != PFDR_MEM_DEVICE) ||
            (method != 0 && method != 1))
            return report_error(fn, "invalid argument");
        if (n > 0x7fffffffL && method == 1) return report_error(fn, "n too large for method 1");
        hipStream_t s = lib_stream();
        DevBuf<real> bA, bio(2);
        DevBuf<long long> cnt(1);
        DevBuf<char> ws(mono_ws_bytes<real>(n));
        const real *dA = a;
        if (mem != PFDR_MEM_DEVICE && n) {
            bA.alloc(n);
            HostPins pins(s);
            pins.copy(bA.p, a, n * sizeof(real), hipMemcpyHostToDevice);
            pins.release();
            dA = bA.p;
        }
        PFDR_HIP(hipMemcpyAsync(bio.p, &seed, sizeof(real), hipMemcpyHostToDevice, s));
        hipEvent_t e0, e1;
        PFDR_HIP(hipEventCreate(&e0));
        PFDR_HIP(hipEventCreate(&e1));
        PFDR_HIP(hipEventRecord(e0, s));
        if (method == 0)
            mono_sum<real>(n, dA, bio.p, 0, nullptr, bio.p + 1, nullptr, ws.p, s);
        else
            k_seq_sum<real><<<1, kBlock, 0, s>>>(n, dA, bio.p, 0, nullptr, bio.p + 1, cnt.p);
        PFDR_HIP(hipGetLastError());
        PFDR_HIP(hipEventRecord(e1, s));
        PFDR_HIP(hipMemcpyAsync(out, bio.p + 1, sizeof(real), hipMemcpyDeviceToHost, s));
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

}  // namespace pfdr

extern "C" int pfdr_sequential_sum_f32(int64_t n, const float *a, int mem, float seed, int method,
                                       float *out, double *ms) {
    return pfdr::seqsum_host<float>("pfdr_sequential_sum_f32", n, a, mem, seed, method, out, ms);
}
extern "C" int pfdr_sequential_sum_f64(int64_t n, const double *a, int mem, double seed,
                                       int method, double *out, double *ms) {
    return pfdr::seqsum_host<double>("pfdr_sequential_sum_f64", n, a, mem, seed, method, out, ms);
}
