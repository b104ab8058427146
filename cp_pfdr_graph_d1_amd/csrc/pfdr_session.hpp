// Session base class shared by the quadratic and simplex solvers: stream,
// kernel-launch profiling with HIP events, chunked device-controlled
// iteration loop bookkeeping.
#pragma once
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "pfdr_dev.hpp"

namespace pfdr {

// HIP-event timing of named kernels on the session stream.  When enabled,
// every `period`-th launch of a profiled kernel (all kernels, or those named
// in `only`) is bracketed by two events; durations are resolved after the
// stream has been synchronised.  An event pair costs ~9 us of GPU time on
// MI355X (profiles/r2/r2d_launch_gap.log): sampling keeps that out of the
// timed iterations of small or partitioned graphs.
class Profiler {
  public:
    bool on = false;
    int period = 1;
    std::vector<std::string> only;
    ~Profiler();
    bool begin(const char *name, hipStream_t s);  // false: this launch not timed
    void end(hipStream_t s);
    void resolve();  // call after the stream has been synchronised
    void reserve(int n);  // pre-create n events (no hipEventCreate between launches)
    bool stats(const char *name, int *launches, double *mean_ms) const;

  private:
    struct Pending { int id; hipEvent_t a, b; };
    std::vector<Pending> pend_;
    std::vector<hipEvent_t> pool_;
    std::map<std::string, int> ids_;
    std::vector<double> total_ms_;
    std::vector<int> count_, seen_;
    int open_id_ = -1;
    hipEvent_t open_ev_ = nullptr;
    hipEvent_t take();
};

struct ProfScope {
    Profiler &p;
    hipStream_t s;
    bool on;
    ProfScope(Profiler &pr, const char *name, hipStream_t st)
        : p(pr), s(st), on(pr.on && pr.begin(name, st)) {}
    ~ProfScope() { if (on) p.end(s); }
};

class SessionBase {
  public:
    virtual ~SessionBase() = default;
    // run up to `iters` more iterations; returns total iterations so far
    virtual int run(int iters) = 0;
    virtual void result(void *X_host, int *it, void *Obj_host,
                        void *Dif_host) = 0;
    virtual void *device_x() = 0;
    // capture (once) the graphs a later run(iters) replays; no iteration runs
    virtual void prepare(int iters) { (void)iters; }
    int64_t device_bytes = 0;
    int64_t reordered = 0;  // internal locality relabelling applied
    int64_t split_blocks = 0;  // vertex blocks on the split-incidence path
    int64_t tiled_blocks = 0;  // vertex blocks staging tile-ordered contributions
    int64_t record_blocks = 0;  // of those, blocks read through a one-load record (tile_sum_rec)
    int64_t slot_patterns = 0;  // distinct slot patterns of their runs (0: per-entry slots)
    int64_t edge_ratio = 0;     // 1: the tiled edge sweep reads formed per-vertex ratios
    int64_t vertex_pair = 0;    // >0: pair vertex sweep, entries of the largest record block
    int64_t ustaged = 0;       // edge sweep stages the u ends (k_edge_sweep_us)
    int64_t symv = 0;          // A^tA products from the block upper triangle
    int64_t tiny = 0;          // small graph: iterations in one workgroup launch
    int64_t fused = 0;         // small graph: loop decision inside the next edge sweep
    int64_t padded = 0;        // fused graph: contributions stored in per-block lists
    int64_t seqdif = 0;        // evolution statistic with the reference's sequential rounding
    int64_t la_uniform = 0;    // one La_d1 value for every edge: the array is not streamed
    int64_t dense_exact = 0;   // dense A: dot products in the reference's order
    int64_t ghosts = 0;        // partitioned: ghost (halo) vertices of this rank
    int64_t graphs = 0;        // chunks of iterations replayed as hipGraphs
    int64_t speculative = 0;   // 1: evolution decision overlapped with the next iteration
                               // (its own stream / split communicator), 2: serial (PFDR_SPEC_SERIAL)
    int64_t interior_edges = -1;  // edges of the "edge_sweep" launch (E unless halo overlap)
    hipStream_t stream = nullptr;
    Profiler prof;
    int device = 0;
};

// the speculation mode of a problem: p->spec, or the env PFDR_SPEC (auto |
// serial | off) when set
inline int spec_mode(const pfdr_problem *p) {
    const char *e = getenv("PFDR_SPEC");
    int m = p->spec;
    if (e && *e) {
        const std::string v(e);
        if (v == "auto") m = PFDR_SPEC_AUTO;
        else if (v == "serial") m = PFDR_SPEC_SERIAL;
        else if (v == "off") m = PFDR_SPEC_OFF;
        else throw std::runtime_error("PFDR_SPEC must be auto, serial or off");
    }
    if (m < PFDR_SPEC_AUTO || m > PFDR_SPEC_OFF)
        throw std::runtime_error("spec must be PFDR_SPEC_AUTO, _SERIAL or _OFF");
    return m;
}

// PFDR_TRACE=1: one stderr line per drop-in call (sizes, iterations, setup /
// iteration / copy-back wall times) -- the view of a CP caller's inner loop.
struct CallTrace {
    const char *fn;
    bool on;
    double t0, t_setup = 0, t_run = 0;
    explicit CallTrace(const char *name);
    void setup_done();
    void run_done();
    void finish(long V, long E, long N, int K, int it);
};

// Several GPUs behind one drop-in call (pfdr_multidev.hip): the devices a
// host-pointer problem is partitioned across (empty: the one-GPU session),
// and the synchronous partitioned solve over them.
std::vector<int> multidev_devices(const pfdr_problem *p);
void multidev_solve(const pfdr_problem *p, const std::vector<int> &devs, int *it, void *Obj,
                    void *Dif);

}  // namespace pfdr

struct pfdr_session {
    pfdr::SessionBase *impl;
};
