// Several GPUs behind ONE synchronous drop-in call (SURVEY.md §3 CS-5, §5
// "single process, ncclCommInitAll, one stream per GPU", §8(b) Threading).
//
// The reference's PFDR entry points are one blocking host call each
// (include/PFDR_graph_quadratic_d1_bounds.hpp:34-40; cut pursuit calls them
// synchronously, e.g. src/CP_PFDR_graph_quadratic_d1_bounds.cpp:824-835), so
// a CP caller -- or a MEX wrapper -- cannot be asked to launch one process
// per GPU.  When several devices are configured (pfdr_set_devices, or the
// PFDR_DEVICES environment variable) and the graph is large enough, the call
// is served by the vertex-range partition of pfdr_halo.hpp driven from this
// process: the caller's graph is split on the host (rank r owns global
// vertices [off[r], off[r+1]) and the edges whose Eu it owns, with their
// global edge ids, which key every per-vertex sum -- so the result equals
// the one-GPU solve bit for bit), one host thread per device runs that
// rank's session (its own stream on its own device) over an RCCL
// communicator of the process's device group (ncclCommInitAll, created once
// and cached across calls), and every rank copies its slice of X straight
// into the caller's array.  A device list that repeats one device runs the
// ranks as threads on it with the loopback transport (how the path is
// tested on a one-GPU box).
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "pfdr_halo.hpp"
#include "pfdr_session.hpp"

namespace pfdr {

SessionBase *create_quadratic_session(const pfdr_problem *p);
SessionBase *create_simplex_session(const pfdr_problem *p);

namespace {

// below this many vertices a call stays on one GPU: CP's reduced problems
// are latency-bound, and a split only adds exchanges to them
constexpr long kMultiMinVertices = 1L << 20;

// Persistent host threads, one per rank slot: a thread keeps its library
// stream (lib_stream is per thread and device) and its device's cached
// blocks across calls, instead of a fresh thread -- and a fresh stream --
// for every drop-in call.  Never destroyed (like the device cache).
class RankPool {
  public:
    // run f(r) for r in [0, n) on n pool threads; returns when all are done
    void run(int n, const std::function<void(int)> &f) {
        std::unique_lock<std::mutex> lk(m_);
        while ((int)slots_.size() < n) {
            slots_.emplace_back(new Slot());
            Slot *sl = slots_.back().get();
            const int r = (int)slots_.size() - 1;
            std::thread([this, sl, r] { loop(sl, r); }).detach();
        }
        fn_ = &f;
        pending_ = n;
        for (int r = 0; r < n; r++) { slots_[r]->go = true; slots_[r]->cv.notify_one(); }
        done_.wait(lk, [&] { return pending_ == 0; });
        fn_ = nullptr;
    }

  private:
    struct Slot {
        std::condition_variable cv;
        bool go = false;
    };
    void loop(Slot *sl, int r) {
        std::unique_lock<std::mutex> lk(m_);
        for (;;) {
            sl->cv.wait(lk, [&] { return sl->go; });
            sl->go = false;
            const std::function<void(int)> *f = fn_;
            lk.unlock();
            (*f)(r);  // never throws (rank_main catches)
            lk.lock();
            if (--pending_ == 0) done_.notify_all();
        }
    }
    std::mutex m_;
    std::condition_variable done_;
    std::vector<std::unique_ptr<Slot>> slots_;
    const std::function<void(int)> *fn_ = nullptr;
    int pending_ = 0;
};

RankPool &rank_pool() {
    static RankPool *p = new RankPool();
    return *p;
}

// one drop-in multi-device call at a time (the pool and the communicators
// serve one partitioned solve)
std::mutex &multidev_call_mutex() {
    static std::mutex *m = new std::mutex();
    return *m;
}

struct DeviceConfig {
    std::mutex m;
    bool set = false;            // pfdr_set_devices called (overrides PFDR_DEVICES)
    std::vector<int> devs;       // empty: one GPU (the current device)
    long min_vertices = kMultiMinVertices;
    // the RCCL communicators of `devs` (distinct devices), cached across calls
    std::vector<ncclComm_t> comms;
    std::vector<int> comm_devs;
};

DeviceConfig &config() {
    static DeviceConfig *c = new DeviceConfig();  // never destroyed: no RCCL calls at exit
    return *c;
}

// PFDR_DEVICES = N (devices 0 .. N-1) or "all"; read once
void load_env(DeviceConfig &c) {
    static bool done = false;
    if (done || c.set) return;
    done = true;
    const char *e = getenv("PFDR_DEVICES");
    if (!e || !*e) return;
    int n = 0;
    if (!strcmp(e, "all")) {
        if (hipGetDeviceCount(&n) != hipSuccess) { (void)hipGetLastError(); n = 0; }
    } else {
        n = atoi(e);
    }
    if (n > 1)
        for (int d = 0; d < n; d++) c.devs.push_back(d);
}

bool distinct(const std::vector<int> &d) {
    std::vector<int> s(d);
    std::sort(s.begin(), s.end());
    return std::adjacent_find(s.begin(), s.end()) == s.end();
}

// the communicators of the device group `devs` (created on first use,
// re-created after a watchdog abort or for another group); caller holds c.m.
// comms[r] belongs to devs[r].
std::vector<ncclComm_t> group_comms(DeviceConfig &c, const std::vector<int> &devs) {
    bool ok = c.comm_devs == devs && c.comms.size() == devs.size();
    for (ncclComm_t cm : c.comms) ok = ok && !comm_aborted(cm);
    if (!ok) {
        for (ncclComm_t cm : c.comms) {  // aborted ones were released by ncclCommAbort
            comm_release_split(cm);  // (its kept split communicator first)
            if (comm_aborted(cm)) comm_created(cm);  // forget the released handle
            else (void)ncclCommDestroy(cm);
        }
        c.comms.clear();
        c.comm_devs.clear();
        std::vector<ncclComm_t> cm(devs.size());
        const ncclResult_t r = ncclCommInitAll(cm.data(), (int)devs.size(), devs.data());
        if (r != ncclSuccess)
            throw std::runtime_error(std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
        for (ncclComm_t x : cm) comm_created(x);  // a new handle at an aborted one's address
        c.comms = cm;
        c.comm_devs = devs;
    }
    return c.comms;
}

// rank r's part of the caller's graph: edges whose Eu it owns, in the
// caller's order, with their global ids
struct RankEdges {
    std::vector<int> Eu, Ev;
    std::vector<int64_t> eg;
    std::vector<char> La;  // La_d1 of these edges (raw reals)
};

void split_edges(long E, long V, const int *Eu, const int *Ev, const char *La, size_t rsz,
                 const std::vector<int64_t> &off, std::vector<RankEdges> &out) {
    const int n = (int)off.size() - 1;
    out.assign(n, RankEdges());
    const int T = (int)std::max(1L, std::min<long>(16, E / (1L << 20)));
    std::vector<std::vector<long>> cnt(T, std::vector<long>(n, 0));
    auto owner = [&](int u) {
        return (int)(std::upper_bound(off.begin(), off.end(), (int64_t)u) - off.begin()) - 1;
    };
    std::atomic<long> bad{0};
    auto chunk = [&](int t, long &b, long &e) { b = E * t / T; e = E * (t + 1) / T; };
    {
        std::vector<std::thread> th;
        for (int t = 0; t < T; t++)
            th.emplace_back([&, t] {
                long b, e;
                chunk(t, b, e);
                for (long i = b; i < e; i++) {
                    const int u = Eu[i], v = Ev[i];
                    if (u < 0 || u >= V || v < 0 || v >= V) { bad++; continue; }
                    cnt[t][owner(u)]++;
                }
            });
        for (auto &x : th) x.join();
    }
    if (bad) throw std::runtime_error("edge endpoint outside [0, V)");
    std::vector<std::vector<long>> base(T, std::vector<long>(n, 0));
    for (int r = 0; r < n; r++) {
        long s = 0;
        for (int t = 0; t < T; t++) { base[t][r] = s; s += cnt[t][r]; }
        if (s > 0x7fffffffL) throw std::runtime_error("a rank's edges exceed 2^31");
        out[r].Eu.resize(s);
        out[r].Ev.resize(s);
        out[r].eg.resize(s);
        out[r].La.resize(s * rsz);
    }
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
        th.emplace_back([&, t] {
            long b, e;
            chunk(t, b, e);
            std::vector<long> pos(base[t]);
            for (long i = b; i < e; i++) {
                const int r = owner(Eu[i]);
                const long k = pos[r]++;
                RankEdges &q = out[r];
                q.Eu[k] = Eu[i];
                q.Ev[k] = Ev[i];
                q.eg[k] = i;
                memcpy(q.La.data() + k * rsz, La + i * rsz, rsz);
            }
        });
    for (auto &x : th) x.join();
}

}  // namespace

// Devices a drop-in call with this problem runs on (empty: the plain
// one-GPU session; one device: a one-rank partition over RCCL).  Dense A
// partitions by columns like the sessions.
std::vector<int> multidev_devices(const pfdr_problem *p) {
    DeviceConfig &c = config();
    std::lock_guard<std::mutex> lk(c.m);
    load_env(c);
    if (c.devs.empty() || (long)p->V < c.min_vertices) return {};
    return c.devs;
}

// The partitioned solve of a host-pointer drop-in problem (pfdr_problem with
// nranks == 0) over `devs`; X (or P), it, Obj, Dif as the one-GPU entry.
void multidev_solve(const pfdr_problem *p, const std::vector<int> &devs, int *it_out,
                    void *Obj, void *Dif) {
    const int n = (int)devs.size();
    const long V = p->V, E = p->E;
    const int Kw = p->kind == PFDR_KIND_SIMPLEX ? p->K : 1;
    const size_t rsz = p->dtype == PFDR_F32 ? 4 : 8;
    // the sessions' own preconditions, checked before the host split reads
    // the caller's arrays
    if (V <= 0 || E < 0 || (p->kind == PFDR_KIND_SIMPLEX && p->K <= 0))
        throw std::runtime_error("V (and K) must be > 0 and E >= 0");
    if (!p->X || !p->Y || (E > 0 && (!p->Eu || !p->Ev || !p->La_d1)))
        throw std::runtime_error("X, Y, Eu, Ev and La_d1 are required");
    if (n > (int)V) throw std::runtime_error("more devices than vertices");
    std::vector<int64_t> off(n + 1);
    for (int r = 0; r <= n; r++) off[r] = V * r / n;
    std::vector<RankEdges> parts;
    split_edges(E, V, p->Eu, p->Ev, static_cast<const char *>(p->La_d1), rsz, off, parts);
    const bool loop = !distinct(devs);
    std::vector<ncclComm_t> comms;
    void *hub = nullptr;
    // one partitioned call at a time, from fetching the group's communicators
    // to the end of the solve: another thread's call for another device group
    // (pfdr_set_devices in between) re-creates the cached communicators, which
    // must not happen while these are in use
    std::lock_guard<std::mutex> call(multidev_call_mutex());
    if (loop) {
        if (pfdr_loopback_create(&hub, n) != PFDR_OK) throw std::runtime_error(pfdr_last_error());
    } else {
        DeviceConfig &c = config();
        std::lock_guard<std::mutex> lk(c.m);
        comms = group_comms(c, devs);
    }
    const bool ata = p->N < 0, direct = p->N > 0;
    std::vector<std::string> err(n);
    std::vector<int> its(n, -1);
    auto rank_main = [&](int r) {
        try {
            PFDR_HIP(hipSetDevice(devs[r]));
            const long v0 = off[r], Vr = off[r + 1] - off[r];
            const char *X0 = static_cast<const char *>(p->X);
            auto at = [&](const void *a, long i) -> const void * {
                return a ? static_cast<const char *>(a) + i * rsz : nullptr;
            };
            pfdr_problem q = *p;
            q.V = (int)Vr;
            q.E = (int)parts[r].Eu.size();
            q.X = const_cast<char *>(X0) + v0 * Kw * rsz;
            q.Y = direct ? p->Y : at(p->Y, v0 * Kw);
            q.A = !p->A ? nullptr : direct ? at(p->A, (long)p->N * v0)
                                  : ata ? at(p->A, V * v0) : at(p->A, v0);
            q.La_l1 = at(p->La_l1, v0);
            q.L = (p->L && p->Ltype == PFDR_LIPSCHITZ_DIAG) ? at(p->L, v0) : p->L;
            q.Eu = parts[r].Eu.data();
            q.Ev = parts[r].Ev.data();
            q.La_d1 = parts[r].La.data();
            q.e_global = parts[r].eg.data();
            q.e_offset = 0;
            q.nranks = n;
            q.rank = r;
            q.comm = loop ? hub : (void *)comms[r];
            q.comm_kind = loop ? PFDR_COMM_LOOPBACK : PFDR_COMM_RCCL;
            q.vtx_begin = v0;
            q.V_global = V;
            q.vtx_label = nullptr;
            q.reorder = PFDR_REORDER_OFF;
            if (r != 0) q.verbose = 0;
            std::unique_ptr<SessionBase> s(p->kind == PFDR_KIND_SIMPLEX
                                               ? create_simplex_session(&q)
                                               : create_quadratic_session(&q));
            s->run(p->itMax);
            s->result(q.X, &its[r], r == 0 ? Obj : nullptr, r == 0 ? Dif : nullptr);
        } catch (const HipError &h) {
            char m[512];
            snprintf(m, sizeof m, "rank %d (device %d): HIP error %d (%s) in `%s`", r, devs[r],
                     (int)h.err, hipGetErrorString(h.err), h.what);
            err[r] = m;
        } catch (const std::exception &ex) {
            err[r] = "rank " + std::to_string(r) + " (device " + std::to_string(devs[r]) + "): " +
                     ex.what();
        } catch (...) {
            err[r] = "rank " + std::to_string(r) + ": unknown exception";
        }
        if (!err[r].empty()) {  // wake the other ranks: their collectives fail too
            if (loop) pfdr_loopback_abort(hub, err[r].c_str());
            else for (ncclComm_t cm : comms) comm_abort(cm);
        }
    };
    rank_pool().run(n, rank_main);
    if (hub) pfdr_loopback_destroy(hub);
    // the first failure is the cause, the others its consequence
    std::string first;
    for (const std::string &e : err)
        if (!e.empty() && e.find("abort") == std::string::npos) { first = e; break; }
    if (first.empty())
        for (const std::string &e : err) if (!e.empty()) { first = e; break; }
    if (!first.empty()) throw std::runtime_error(first);
    for (int r = 1; r < n; r++)
        if (its[r] != its[0]) throw std::runtime_error("ranks disagree on the iteration count");
    if (it_out) *it_out = its[0];
}

}  // namespace pfdr

// Device group of the drop-in entry points (pfdr_mi355x.h).
extern "C" int pfdr_set_devices(int n, const int *devices, int64_t min_vertices) {
    using namespace pfdr;
    if (n < 0 || n > 64 || (n > 0 && !devices && n != 1))
        return report_error("pfdr_set_devices", "invalid arguments");
    DeviceConfig &c = config();
    std::lock_guard<std::mutex> lk(c.m);
    int count = 0;
    if (n > 0 && hipGetDeviceCount(&count) != hipSuccess) {
        (void)hipGetLastError();
        return report_error("pfdr_set_devices", "no HIP device");
    }
    std::vector<int> devs;
    for (int i = 0; i < n; i++) {
        const int d = devices ? devices[i] : 0;
        if (d < 0 || d >= count) return report_error("pfdr_set_devices", "device id out of range");
        devs.push_back(d);
    }
    // distinct devices (RCCL) or one device repeated (loopback ranks on it)
    if (!distinct(devs) && std::count(devs.begin(), devs.end(), devs[0]) != n)
        return report_error("pfdr_set_devices",
                            "devices must be all distinct or all the same one");
    c.set = true;
    c.devs = devs;
    c.min_vertices = min_vertices >= 0 ? (long)min_vertices : kMultiMinVertices;
    return PFDR_OK;
}
