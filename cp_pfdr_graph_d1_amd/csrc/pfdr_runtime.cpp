// Runtime pieces of libpfdr_mi355x.so that are not kernels: error state,
// library stream, profiler, session C ABI dispatch.
#include <chrono>
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstring>
#include <map>
#include <mutex>
#include <string>

#include "pfdr_session.hpp"

namespace pfdr {

static thread_local std::string g_last_error;

static void set_error(const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
}

static double now_ms() {
    return std::chrono::duration<double, std::milli>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

static bool trace_enabled() {
    static const bool on = [] {
        const char *v = getenv("PFDR_TRACE");
        return v && v[0] && v[0] != '0';
    }();
    return on;
}

CallTrace::CallTrace(const char *name) : fn(name), on(trace_enabled()), t0(on ? now_ms() : 0) {}
void CallTrace::setup_done() { if (on) t_setup = now_ms(); }
void CallTrace::run_done() { if (on) t_run = now_ms(); }
void CallTrace::finish(long V, long E, long N, int K, int it) {
    if (!on) return;
    const double t1 = now_ms();
    fprintf(stderr, "[pfdr] %s V=%ld E=%ld N=%ld K=%d it=%d setup_ms=%.3f run_ms=%.3f "
            "copy_ms=%.3f total_ms=%.3f\n", fn, V, E, N, K, it, t_setup - t0,
            t_run - t_setup, t1 - t_run, t1 - t0);
}

int report_error(const char *fn, const HipError &h) {
    set_error("%s: HIP error %d (%s) in `%s` (line %d)", fn, (int)h.err,
              hipGetErrorString(h.err), h.what, h.line);
    return PFDR_ERR_HIP;
}

int report_error(const char *fn, const char *msg) {
    set_error("%s: %s", fn, msg);
    return PFDR_ERR_ARG;
}

static thread_local hipStream_t g_scope_stream = nullptr;

StreamScope::StreamScope(hipStream_t s, int device) : prev_s_(g_scope_stream) {
    int cur = 0;
    if (hipGetDevice(&cur) == hipSuccess && cur != device) {
        PFDR_HIP(hipSetDevice(device));
        prev_dev_ = cur;
    }
    dev_ = device;
    g_scope_stream = s;
}

StreamScope::~StreamScope() {
    g_scope_stream = prev_s_;
    if (prev_dev_ >= 0) (void)hipSetDevice(prev_dev_);
}

hipStream_t lib_stream() {
    if (g_scope_stream) return g_scope_stream;
    // one non-blocking stream per (thread, device)
    static thread_local hipStream_t streams[64] = {};
    int dev = 0;
    PFDR_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) throw HipError{hipErrorInvalidDevice, "device id", __LINE__};
    if (!streams[dev]) {
        PFDR_HIP(hipStreamCreateWithFlags(&streams[dev], hipStreamNonBlocking));
    }
    return streams[dev];
}

// -------------------------------------------------- device memory cache --
namespace {
struct CachedBlock {
    void *p;
    int dev;
    hipStream_t freed_on;  // reusable once this stream is idle
};
struct DevCache {
    std::mutex m;
    std::multimap<size_t, CachedBlock> free_;  // size class -> blocks
    size_t cached = 0;
    size_t cap = 0;
    DevCache() {
        const char *e = getenv("PFDR_DEVICE_CACHE_MB");
        cap = (size_t)(e ? atol(e) : 2048) << 20;
    }
};
DevCache &dev_cache() {
    static DevCache *c = new DevCache();  // never destroyed: no HIP calls at exit
    return *c;
}
// size classes: powers of two up to 1 MiB, multiples of 2 MiB above
size_t size_class(size_t b) {
    if (b <= (size_t(1) << 20)) {
        size_t r = 256;
        while (r < b) r <<= 1;
        return r;
    }
    const size_t g = size_t(2) << 20;
    return (b + g - 1) / g * g;
}
void trim_cache(DevCache &c) {  // caller holds c.m
    for (auto &kv : c.free_) (void)hipFree(kv.second.p);
    c.free_.clear();
    c.cached = 0;
}
}  // namespace

void *dev_malloc(size_t bytes) {
    DevCache &c = dev_cache();
    const size_t sc = size_class(bytes);
    int dev = 0;
    PFDR_HIP(hipGetDevice(&dev));
    if (c.cap) {
        std::lock_guard<std::mutex> lk(c.m);
        auto range = c.free_.equal_range(sc);
        for (auto it = range.first; it != range.second; ++it) {
            const CachedBlock &b = it->second;
            if (b.dev != dev) continue;
            if (b.freed_on && hipStreamQuery(b.freed_on) != hipSuccess) {
                (void)hipGetLastError();
                continue;  // kernels queued before the free may still use it
            }
            void *p = b.p;
            c.free_.erase(it);
            c.cached -= sc;
            return p;
        }
    }
    void *p = nullptr;
    hipError_t e = hipMalloc(&p, sc);
    if (e == hipErrorOutOfMemory) {
        (void)hipGetLastError();
        {
            std::lock_guard<std::mutex> lk(c.m);
            (void)hipDeviceSynchronize();
            trim_cache(c);
        }
        e = hipMalloc(&p, sc);
    }
    if (e != hipSuccess) throw HipError{e, "hipMalloc", __LINE__};
    return p;
}

void dev_free(void *p, size_t bytes) noexcept {
    if (!p) return;
    DevCache &c = dev_cache();
    const size_t sc = size_class(bytes);
    try {
        int dev = 0;
        hipPointerAttribute_t at{};
        // cached only when freed under the device that owns it (the idle
        // test needs that device's library stream); otherwise hipFree
        if (c.cap && hipGetDevice(&dev) == hipSuccess &&
            hipPointerGetAttributes(&at, p) == hipSuccess && at.device == dev) {
            const hipStream_t s = lib_stream();
            std::lock_guard<std::mutex> lk(c.m);
            if (c.cached + sc <= c.cap) {
                c.free_.insert({sc, CachedBlock{p, dev, s}});
                c.cached += sc;
                return;
            }
        }
    } catch (...) {
    }
    // not cached: no kernel may still use it (callers free scratch right
    // after enqueuing its last use on the library / session stream, relying
    // on the cache's idle rule): drain that stream -- on the pointer's own
    // device -- before hipFree, not the whole device
    int cur = -1, owner = -1;
    hipPointerAttribute_t at{};
    if (hipGetDevice(&cur) == hipSuccess && hipPointerGetAttributes(&at, p) == hipSuccess)
        owner = at.device;
    (void)hipGetLastError();
    if (owner >= 0 && owner != cur) {
        (void)hipSetDevice(owner);
        (void)hipDeviceSynchronize();  // another device's block: its streams are not ours
        (void)hipFree(p);
        (void)hipSetDevice(cur);
        return;
    }
    try {
        (void)hipStreamSynchronize(lib_stream());
    } catch (...) {
        (void)hipDeviceSynchronize();
    }
    (void)hipFree(p);
}

// ------------------------------------------------------ pinned blocks --
namespace {
struct PinnedPool {
    std::mutex m;
    std::vector<void *> free_;
};
PinnedPool &pinned_pool() {
    static PinnedPool *p = new PinnedPool;  // outlives the HIP runtime's teardown
    return *p;
}
}  // namespace

void *pinned_small_get() {
    PinnedPool &pp = pinned_pool();
    {
        std::lock_guard<std::mutex> lk(pp.m);
        if (!pp.free_.empty()) {
            void *p = pp.free_.back();
            pp.free_.pop_back();
            return p;
        }
    }
    void *p = nullptr;
    PFDR_HIP(hipHostMalloc(&p, kPinnedSmall, hipHostMallocDefault));
    return p;
}

void pinned_small_put(void *p) noexcept {
    if (!p) return;
    PinnedPool &pp = pinned_pool();
    try {
        std::lock_guard<std::mutex> lk(pp.m);
        pp.free_.push_back(p);
    } catch (...) {
    }
}

// ------------------------------------------------------------ HostPins --
void HostPins::copy(void *dst, const void *src, size_t bytes, hipMemcpyKind kind) {
    if (!bytes) return;
    void *host = kind == hipMemcpyHostToDevice ? const_cast<void *>(src)
               : kind == hipMemcpyDeviceToHost ? dst : nullptr;
    if (host && bytes >= (size_t(1) << 20) && n_ < 64) {
        if (hipHostRegister(host, bytes, hipHostRegisterDefault) == hipSuccess)
            pinned_[n_++] = host;
        else
            (void)hipGetLastError();  // not pinnable: the pageable path copies it
    }
    PFDR_HIP(hipMemcpyAsync(dst, src, bytes, kind, s_));
}

void HostPins::release() {
    if (!n_) return;
    const hipError_t e = hipStreamSynchronize(s_);
    for (int i = 0; i < n_; i++) (void)hipHostUnregister(pinned_[i]);
    n_ = 0;
    if (e != hipSuccess) throw HipError{e, "hipStreamSynchronize (HostPins)", __LINE__};
}

HostPins::~HostPins() {
    if (!n_) return;
    (void)hipStreamSynchronize(s_);  // never unpin under a DMA in flight
    for (int i = 0; i < n_; i++) (void)hipHostUnregister(pinned_[i]);
}

// ------------------------------------------------------------ Profiler --
// Timing events without the system-scope fence: a default event pair costs
// ~9 us of GPU time per bracketed launch on MI355X, ~6 us without the fence
// (tools/exp_launch_gap.hip, profiles/r2/r2d_launch_gap.log).  The events
// are only read after the stream is synchronised.
static constexpr unsigned kProfEventFlags = hipEventDisableSystemFence;

Profiler::~Profiler() {
    for (auto &p : pend_) { (void)hipEventDestroy(p.a); (void)hipEventDestroy(p.b); }
    for (auto e : pool_) (void)hipEventDestroy(e);
    if (open_ev_) (void)hipEventDestroy(open_ev_);
}

hipEvent_t Profiler::take() {
    if (!pool_.empty()) {
        hipEvent_t e = pool_.back();
        pool_.pop_back();
        return e;
    }
    hipEvent_t e;
    PFDR_HIP(hipEventCreateWithFlags(&e, kProfEventFlags));
    return e;
}

void Profiler::reserve(int n) {
    for (int i = (int)pool_.size(); i < n; i++) {
        hipEvent_t e;
        PFDR_HIP(hipEventCreateWithFlags(&e, kProfEventFlags));
        pool_.push_back(e);
    }
}

bool Profiler::begin(const char *name, hipStream_t s) {
    if (!only.empty()) {
        bool hit = false;
        for (const auto &o : only) hit |= (o == name);
        if (!hit) return false;
    }
    auto it = ids_.find(name);
    int id;
    if (it == ids_.end()) {
        id = (int)total_ms_.size();
        ids_[name] = id;
        total_ms_.push_back(0.0);
        count_.push_back(0);
        seen_.push_back(0);
    } else {
        id = it->second;
    }
    if (seen_[id]++ % (period > 0 ? period : 1)) return false;
    open_id_ = id;
    open_ev_ = take();
    PFDR_HIP(hipEventRecord(open_ev_, s));
    return true;
}

void Profiler::end(hipStream_t s) {
    hipEvent_t b = take();
    PFDR_HIP(hipEventRecord(b, s));
    pend_.push_back({open_id_, open_ev_, b});
    open_ev_ = nullptr;
    open_id_ = -1;
}

void Profiler::resolve() {
    for (auto &p : pend_) {
        float ms = 0.f;
        PFDR_HIP(hipEventSynchronize(p.b));
        PFDR_HIP(hipEventElapsedTime(&ms, p.a, p.b));
        total_ms_[p.id] += ms;
        count_[p.id] += 1;
        pool_.push_back(p.a);
        pool_.push_back(p.b);
    }
    pend_.clear();
}

bool Profiler::stats(const char *name, int *launches, double *mean_ms) const {
    auto it = ids_.find(name);
    if (it == ids_.end()) { *launches = 0; *mean_ms = 0.0; return false; }
    int c = count_[it->second];
    *launches = c;
    *mean_ms = c ? total_ms_[it->second] / c : 0.0;
    return true;
}

// defined in the solver translation units
SessionBase *create_quadratic_session(const pfdr_problem *p);
SessionBase *create_simplex_session(const pfdr_problem *p);

}  // namespace pfdr

using namespace pfdr;

#define PFDR_GUARD(fn, body)                                         \
    try {                                                            \
        body;                                                        \
    } catch (const HipError &h) {                                    \
        return report_error(fn, h);                                  \
    } catch (const std::exception &ex) {                             \
        return report_error(fn, ex.what());                          \
    }

extern "C" const char *pfdr_last_error(void) { return g_last_error.c_str(); }
extern "C" int pfdr_abi_version(void) { return 4; }
extern "C" int pfdr_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return -1;
    return n;
}

extern "C" int pfdr_session_create(pfdr_session **out, const pfdr_problem *p) {
    if (!out || !p) return report_error("pfdr_session_create", "null argument");
    *out = nullptr;
    PFDR_GUARD("pfdr_session_create", {
        SessionBase *impl = nullptr;
        if (p->kind == PFDR_KIND_L1 || p->kind == PFDR_KIND_BOUNDS)
            impl = create_quadratic_session(p);
        else if (p->kind == PFDR_KIND_SIMPLEX)
            impl = create_simplex_session(p);
        else
            return report_error("pfdr_session_create", "unknown problem kind");
        *out = new pfdr_session{impl};
    });
    return PFDR_OK;
}

extern "C" int pfdr_session_run(pfdr_session *s, int iters, int *it_total) {
    if (!s) return report_error("pfdr_session_run", "null session");
    PFDR_GUARD("pfdr_session_run", {
        StreamScope sc(s->impl->stream, s->impl->device);
        int it = s->impl->run(iters);
        if (it_total) *it_total = it;
    });
    return PFDR_OK;
}

extern "C" int pfdr_session_prepare(pfdr_session *s, int iters) {
    if (!s) return report_error("pfdr_session_prepare", "null session");
    PFDR_GUARD("pfdr_session_prepare", {
        StreamScope sc(s->impl->stream, s->impl->device);
        s->impl->prepare(iters);
    });
    return PFDR_OK;
}

extern "C" int pfdr_session_result(pfdr_session *s, void *X, int *it,
                                   void *Obj, void *Dif) {
    if (!s) return report_error("pfdr_session_result", "null session");
    PFDR_GUARD("pfdr_session_result", {
        StreamScope sc(s->impl->stream, s->impl->device);
        s->impl->result(X, it, Obj, Dif);
    });
    return PFDR_OK;
}

extern "C" void *pfdr_session_device_x(pfdr_session *s) {
    if (!s) return nullptr;
    try {
        StreamScope sc(s->impl->stream, s->impl->device);
        return s->impl->device_x();
    } catch (const HipError &h) {
        report_error("pfdr_session_device_x", h);
    } catch (const std::exception &ex) {
        report_error("pfdr_session_device_x", ex.what());
    }
    return nullptr;
}

extern "C" int pfdr_session_profile_filter(pfdr_session *s, const char *names) {
    if (!s) return report_error("pfdr_session_profile_filter", "null session");
    auto &o = s->impl->prof.only;
    o.clear();
    if (names) {
        std::string n(names);
        size_t a = 0;
        while (a <= n.size()) {
            size_t b = n.find(',', a);
            if (b == std::string::npos) b = n.size();
            if (b > a) o.push_back(n.substr(a, b - a));
            a = b + 1;
        }
    }
    return PFDR_OK;
}

extern "C" int pfdr_session_set_profiling(pfdr_session *s, int on) {
    if (!s) return report_error("pfdr_session_set_profiling", "null session");
    PFDR_GUARD("pfdr_session_set_profiling", {
        s->impl->prof.on = (on != 0);
        s->impl->prof.period = on > 1 ? on : 1;
        if (on) s->impl->prof.reserve(1024);  // no event creation between timed launches
    });
    return PFDR_OK;
}

extern "C" int pfdr_session_kernel_stats(pfdr_session *s, const char *kernel,
                                         int *launches, double *mean_ms) {
    if (!s || !kernel || !launches || !mean_ms)
        return report_error("pfdr_session_kernel_stats", "null argument");
    PFDR_GUARD("pfdr_session_kernel_stats", {
        StreamScope sc(s->impl->stream, s->impl->device);
        PFDR_HIP(hipStreamSynchronize(s->impl->stream));
        s->impl->prof.resolve();
        s->impl->prof.stats(kernel, launches, mean_ms);
    });
    return PFDR_OK;
}

extern "C" int pfdr_session_sync(pfdr_session *s) {
    if (!s) return report_error("pfdr_session_sync", "null session");
    PFDR_GUARD("pfdr_session_sync", {
        PFDR_HIP(hipStreamSynchronize(s->impl->stream));
    });
    return PFDR_OK;
}

extern "C" int64_t pfdr_session_device_bytes(pfdr_session *s) {
    return s ? s->impl->device_bytes : -1;
}

extern "C" int pfdr_session_query(pfdr_session *s, const char *what, int64_t *value) {
    if (!s || !what || !value) return report_error("pfdr_session_query", "null argument");
    if (!strcmp(what, "reordered")) *value = s->impl->reordered;
    else if (!strcmp(what, "split_blocks")) *value = s->impl->split_blocks;
    else if (!strcmp(what, "tiled_blocks")) *value = s->impl->tiled_blocks;
    else if (!strcmp(what, "record_blocks")) *value = s->impl->record_blocks;
    else if (!strcmp(what, "slot_patterns")) *value = s->impl->slot_patterns;
    else if (!strcmp(what, "edge_ratio")) *value = s->impl->edge_ratio;
    else if (!strcmp(what, "vertex_pair")) *value = s->impl->vertex_pair;
    else if (!strcmp(what, "ustaged")) *value = s->impl->ustaged;
    else if (!strcmp(what, "symv")) *value = s->impl->symv;
    else if (!strcmp(what, "tiny")) *value = s->impl->tiny;
    else if (!strcmp(what, "fused")) *value = s->impl->fused;
    else if (!strcmp(what, "padded")) *value = s->impl->padded;
    else if (!strcmp(what, "seqdif")) *value = s->impl->seqdif;
    else if (!strcmp(what, "la_uniform")) *value = s->impl->la_uniform;
    else if (!strcmp(what, "ghosts")) *value = s->impl->ghosts;
    else if (!strcmp(what, "graphs")) *value = s->impl->graphs;
    else if (!strcmp(what, "speculative")) *value = s->impl->speculative;
    else if (!strcmp(what, "dense_exact")) *value = s->impl->dense_exact;
    else if (!strcmp(what, "interior_edges")) *value = s->impl->interior_edges;
    else if (!strcmp(what, "device_bytes")) *value = s->impl->device_bytes;
    else return report_error("pfdr_session_query", (std::string("unknown key ") + what).c_str());
    return PFDR_OK;
}

extern "C" void pfdr_session_destroy(pfdr_session *s) {
    if (!s) return;
    try {
        StreamScope sc(s->impl->stream, s->impl->device);
        (void)hipStreamSynchronize(s->impl->stream);
        delete s->impl;
    } catch (...) {
    }
    delete s;
}
