// Partition plan, halo exchanges and the two transports (see pfdr_halo.hpp).
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <thread>

#include "pfdr_halo.hpp"

namespace pfdr {

// ------------------------------------------------------------- kernels --
template <int B>
__global__ void k_pack_u(int n, const unsigned *__restrict__ idx, const char *__restrict__ src,
                         char *__restrict__ dst) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    struct alignas(B) Blk { char b[B]; };
    reinterpret_cast<Blk *>(dst)[i] = reinterpret_cast<const Blk *>(src)[idx[i]];
}

// any element size that is a multiple of 4 bytes: one lane per word
template <typename I>
__global__ void k_pack_words(long n, int words, const I *__restrict__ idx,
                             const unsigned *__restrict__ src, unsigned *__restrict__ dst) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * words) return;
    const long i = t / words;
    const int w = (int)(t - i * words);
    dst[t] = src[(long)idx[i] * words + w];
}

template <typename I>
static void pack_any(int n, const I *idx, const void *src, void *dst, int eb, hipStream_t s) {
    if (n <= 0) return;
    const int g = grid_for(n);
    switch (eb) {
        case 4: k_pack_u<4><<<g, kBlock, 0, s>>>(n, (const unsigned *)idx, (const char *)src,
                                                 (char *)dst); break;
        case 8: k_pack_u<8><<<g, kBlock, 0, s>>>(n, (const unsigned *)idx, (const char *)src,
                                                 (char *)dst); break;
        case 16: k_pack_u<16><<<g, kBlock, 0, s>>>(n, (const unsigned *)idx, (const char *)src,
                                                   (char *)dst); break;
        default:
            if (eb % 4) throw std::runtime_error("pack: element size");
            k_pack_words<I><<<grid_for((long)n * (eb / 4)), kBlock, 0, s>>>(
                n, eb / 4, idx, (const unsigned *)src, (unsigned *)dst);
    }
    PFDR_HIP(hipGetLastError());
}

static void pack(int n, const int *idx, const void *src, void *dst, int eb, hipStream_t s) {
    // owned local ids are non-negative: the unsigned gather reads them alike
    pack_any<int>(n, idx, src, dst, eb, s);
}

static void pack_u(int n, const unsigned *idx, const void *src, void *dst, int eb, hipStream_t s) {
    pack_any<unsigned>(n, idx, src, dst, eb, s);
}

// ------------------------------------------------------------ Transport --
double Transport::comm_timeout_s() {
    const char *t = getenv("PFDR_COMM_TIMEOUT");
    const double v = t ? atof(t) : 120.0;
    return v > 0 ? v : 120.0;
}

std::string Transport::describe() const {
    char m[160];
    snprintf(m, sizeof m, "rank %d of %d, %s, iteration %ld, last collective: ", rank, nranks,
             phase, iteration);
    return std::string(m) + last_op;
}

// poll the stream; past the timeout, report what this rank was waiting for
void Transport::wait(hipStream_t s) {
    const auto t0 = std::chrono::steady_clock::now();
    int spins = 0;
    while (true) {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipSuccess) return;
        if (e != hipErrorNotReady) PFDR_HIP(e);
        const double el =
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (el > timeout_s) {
            char m[96];
            snprintf(m, sizeof m, "halo exchange stalled for %.0f s (PFDR_COMM_TIMEOUT): ", el);
            const std::string msg = m + describe();
            fprintf(stderr, "[pfdr watchdog] %s\n", msg.c_str());
            fflush(stderr);
            on_timeout();
            throw std::runtime_error(msg);
        }
        if (++spins > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

static std::string peers_bytes(const std::vector<size_t> &b, int self) {
    std::string out = "{";
    char m[48];
    for (size_t q = 0; q < b.size(); q++) {
        if ((int)q == self || !b[q]) continue;
        snprintf(m, sizeof m, "%s%zu: %zu B", out.size() > 1 ? ", " : "", q, b[q]);
        out += m;
    }
    return out + "}";
}

void Transport::allgather_i64(int64_t mine, std::vector<int64_t> &all, hipStream_t s) {
    all.assign(nranks, 0);
    all[rank] = mine;
    if (nranks == 1) return;
    DevBuf<int64_t> d(nranks);
    PFDR_HIP(hipMemsetAsync(d.p, 0, sizeof(int64_t) * nranks, s));
    PFDR_HIP(hipMemcpyAsync(d.p + rank, &mine, sizeof(int64_t), hipMemcpyHostToDevice, s));
    allreduce_sum(d.p, nranks, 2, s);
    PFDR_HIP(hipMemcpyAsync(all.data(), d.p, sizeof(int64_t) * nranks, hipMemcpyDeviceToHost, s));
    wait(s);
}

void Transport::alltoallv_host(const std::vector<std::vector<int64_t>> &send,
                               std::vector<std::vector<int64_t>> &recv, hipStream_t s) {
    const int n = nranks;
    recv.assign(n, {});
    // counts: everyone learns how much each peer sends it (allreduce of an n x n matrix)
    DevBuf<int64_t> cnt((size_t)n * n);
    std::vector<int64_t> hc((size_t)n * n, 0);
    for (int q = 0; q < n; q++) hc[(size_t)rank * n + q] = (int64_t)send[q].size();
    PFDR_HIP(hipMemcpyAsync(cnt.p, hc.data(), sizeof(int64_t) * n * n, hipMemcpyHostToDevice, s));
    allreduce_sum(cnt.p, n * n, 2, s);
    PFDR_HIP(hipMemcpyAsync(hc.data(), cnt.p, sizeof(int64_t) * n * n, hipMemcpyDeviceToHost, s));
    wait(s);
    std::vector<DevBuf<int64_t>> ds(n), dr(n);
    std::vector<const void *> sp(n, nullptr);
    std::vector<void *> rp(n, nullptr);
    std::vector<size_t> sb(n, 0), rb(n, 0);
    for (int q = 0; q < n; q++) {
        if (q == rank) continue;
        if (!send[q].empty()) {
            ds[q].alloc(send[q].size());
            PFDR_HIP(hipMemcpyAsync(ds[q].p, send[q].data(), sizeof(int64_t) * send[q].size(),
                                    hipMemcpyHostToDevice, s));
            sp[q] = ds[q].p;
            sb[q] = sizeof(int64_t) * send[q].size();
        }
        const int64_t m = hc[(size_t)q * n + rank];
        if (m > 0) {
            dr[q].alloc(m);
            rp[q] = dr[q].p;
            rb[q] = sizeof(int64_t) * m;
        }
    }
    exchange(sp, sb, rp, rb, s);
    for (int q = 0; q < n; q++) {
        if (q == rank) { recv[q] = send[q]; continue; }
        recv[q].resize(rb[q] / sizeof(int64_t));
        if (rb[q])
            PFDR_HIP(hipMemcpyAsync(recv[q].data(), dr[q].p, rb[q], hipMemcpyDeviceToHost, s));
    }
    wait(s);
}

// ----------------------------------------------------------------- RCCL --
class RcclTransport final : public Transport {
    ncclComm_t comm_;
    bool owned_ = false;             // a split communicator: destroyed with the transport
    bool kept_ = false;              // the parent's kept split communicator: given back
    ncclComm_t parent_ = nullptr;    // the communicator it was split from (comm_add_child)
    // PFDR_RCCL_SELF=1 (test flag): the collectives of a 1-rank
    // communicator (all-reduces, broadcasts) are issued as real RCCL calls
    // instead of returning early, so that a one-GPU run executes -- and
    // hipGraph-captures -- the RCCL operations a real partition's chain,
    // decision and objective use.  (A grouped send / receive to the rank
    // itself, which would cover the point-to-point exchanges, crashed inside
    // RCCL on this image: gpurun_out/r6p)
    bool self_ = false;
    void init_self() {
        const char *e = getenv("PFDR_RCCL_SELF");
        self_ = e && e[0] == '1';
    }
    static void ck(ncclResult_t r, const char *what) {
        if (r != ncclSuccess) {
            char m[256];
            snprintf(m, sizeof m, "RCCL %s: %s", what, ncclGetErrorString(r));
            throw std::runtime_error(m);
        }
    }

  public:
    RcclTransport(void *comm, int n, int r) : comm_((ncclComm_t)comm) {
        nranks = n;
        rank = r;
        init_self();
    }
    ~RcclTransport() override {
        if (kept_) comm_split_return(parent_, comm_);
        if (!owned_) return;
        comm_forget_child(parent_, comm_);  // (no abort through the parent after this)
        if (comm_aborted(comm_)) comm_created(comm_);  // released by the abort
        else (void)ncclCommDestroy(comm_);
    }
    // a stalled communicator cannot be used again: abort it so the peers'
    // operations fail too instead of waiting on this rank (recorded, so the
    // owner's pfdr_comm_destroy skips the freed handle)
    void on_timeout() override { comm_abort(comm_); }  // (its split ones first)
    std::unique_ptr<Transport> split(hipStream_t) override {
        last_op = "communicator split";
        // the parent's kept split communicator when free (every rank runs
        // the same sessions on its communicator, so all take it or all
        // split, collectively); PFDR_SPLIT_CACHE=0: a new one per session
        const char *e = getenv("PFDR_SPLIT_CACHE");
        const bool cache = !(e && e[0] == '0');
        ncclComm_t nc = cache ? (ncclComm_t)comm_split_take(comm_) : nullptr;
        bool kept = nc != nullptr;
        if (!nc) {
            // its own resources (streams, buffers): operations on the two
            // communicators must not be ordered behind each other
            ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
            cfg.splitShare = 0;
            ck(ncclCommSplit(comm_, 0, rank, &nc, &cfg), "comm split");
            comm_created(nc);
            kept = cache && comm_split_keep(comm_, nc);
            if (!kept) comm_add_child(comm_, nc);
        }
        std::unique_ptr<RcclTransport> t(new RcclTransport(nc, nranks, rank));
        t->owned_ = !kept;
        t->kept_ = kept;
        t->parent_ = comm_;
        return std::unique_ptr<Transport>(t.release());
    }
    bool capturable() const override { return true; }
    void exchange(const std::vector<const void *> &send, const std::vector<size_t> &sbytes,
                  const std::vector<void *> &recv, const std::vector<size_t> &rbytes,
                  hipStream_t s) override {
        last_op = "grouped send/recv, send " + peers_bytes(sbytes, rank) + " recv " +
                  peers_bytes(rbytes, rank);
        bool any = false;  // (an exchange with nothing to move issues no RCCL call)
        for (int q = 0; q < nranks; q++) any = any || (q != rank && (sbytes[q] || rbytes[q]));
        if (!any) return;
        ck(ncclGroupStart(), "group start");
        for (int q = 0; q < nranks; q++) {
            if (q == rank) continue;
            if (sbytes[q]) ck(ncclSend(send[q], sbytes[q], ncclChar, q, comm_, s), "send");
            if (rbytes[q]) ck(ncclRecv(recv[q], rbytes[q], ncclChar, q, comm_, s), "recv");
        }
        ck(ncclGroupEnd(), "group end");
    }
    void allreduce_sum(void *dev, int n, int dtype, hipStream_t s) override {
        ncclDataType_t t = dtype == PFDR_F32 ? ncclFloat32 : dtype == PFDR_F64 ? ncclFloat64 : ncclInt64;
        last_op = "all-reduce of " + std::to_string(n) + " values, all peers";
        if (nranks == 1 && !self_) return;  // (in place: the sum over one rank is the data)
        ck(ncclAllReduce(dev, dev, n, t, ncclSum, comm_, s), "allreduce");
    }
    void chain_recv(void *dev, size_t bytes, hipStream_t s) override {
        if (rank > 0) {
            last_op = "chain recv of " + std::to_string(bytes) + " B from " + std::to_string(rank - 1);
            ck(ncclRecv(dev, bytes, ncclChar, rank - 1, comm_, s), "chain recv");
        }
    }
    void chain_send(const void *dev, size_t bytes, hipStream_t s) override {
        if (rank + 1 < nranks) {
            last_op = "chain send of " + std::to_string(bytes) + " B to " + std::to_string(rank + 1);
            ck(ncclSend(dev, bytes, ncclChar, rank + 1, comm_, s), "chain send");
        }
    }
    void broadcast(void *dev, size_t bytes, int root, hipStream_t s) override {
        last_op = "broadcast of " + std::to_string(bytes) + " B from " + std::to_string(root);
        if (nranks == 1 && !self_) return;
        ck(ncclBroadcast(dev, dev, bytes, ncclChar, root, comm_, s), "broadcast");
    }
};

std::unique_ptr<Transport> make_rccl_transport(void *comm, int n, int r) {
    if (comm_aborted(comm))
        throw std::runtime_error("RCCL communicator aborted by the watchdog (PFDR_COMM_TIMEOUT); "
                                 "destroy it and create a new one");
    return std::unique_ptr<Transport>(new RcclTransport(comm, n, r));
}

// ------------------------------------------------------------- Loopback --
struct LoopHub {
    int k;
    std::mutex m;
    std::condition_variable cv;
    int count = 0;
    long gen = 0;
    bool aborted = false;        // a rank failed or stalled: every waiter throws
    std::string why;
    struct Post {
        std::vector<const void *> send;
        std::vector<size_t> sbytes;
        const void *ptr = nullptr;
        hipEvent_t ready = nullptr, done = nullptr, chain = nullptr;
        long chain_seq = 0;
    };
    std::vector<Post> post;
    explicit LoopHub(int n) : k(n), post(n) {}
    ~LoopHub() {
        for (auto &p : post) {
            if (p.ready) (void)hipEventDestroy(p.ready);
            if (p.done) (void)hipEventDestroy(p.done);
            if (p.chain) (void)hipEventDestroy(p.chain);
        }
    }
    void abort(const std::string &reason) {
        std::unique_lock<std::mutex> l(m);
        if (!aborted) { aborted = true; why = reason; }
        cv.notify_all();
    }
    [[noreturn]] void fail_locked(const Transport &t, const char *what) {
        throw std::runtime_error(std::string("loopback ") + what + " (" + t.describe() + "): " + why);
    }
    // wait until `ready()` (hub mutex held) under the watchdog
    template <typename F>
    void wait_until(std::unique_lock<std::mutex> &l, const Transport &t, F ready) {
        const auto dl = std::chrono::steady_clock::now() +
                        std::chrono::duration<double>(t.timeout_s);
        if (!cv.wait_until(l, dl, [&] { return aborted || ready(); })) {
            aborted = true;
            char b[96];
            snprintf(b, sizeof b, "rank %d stalled for %.0f s (PFDR_COMM_TIMEOUT)", t.rank,
                     t.timeout_s);
            why = b;
            fprintf(stderr, "[pfdr watchdog] loopback %s: %s\n", t.describe().c_str(), b);
            cv.notify_all();
        }
        if (aborted) fail_locked(t, "aborted");
    }
    void barrier(const Transport &t) {
        std::unique_lock<std::mutex> l(m);
        if (aborted) fail_locked(t, "aborted");
        const long g = gen;
        if (++count == k) {
            count = 0;
            gen++;
            cv.notify_all();
        } else {
            wait_until(l, t, [&] { return gen != g; });
        }
    }
};

template <typename T>
__global__ void k_sum_ranks(int n, int k, const T *const *src, T *dst) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    T s = src[0][i];
    for (int r = 1; r < k; r++) s += src[r][i];  // rank order: same result on every rank
    dst[i] = s;
}

class LoopbackTransport final : public Transport {
    LoopHub *hub_;
    void ensure_events() {
        auto &p = hub_->post[rank];
        if (!p.ready) {
            PFDR_HIP(hipEventCreateWithFlags(&p.ready, hipEventDisableTiming));
            PFDR_HIP(hipEventCreateWithFlags(&p.done, hipEventDisableTiming));
            PFDR_HIP(hipEventCreateWithFlags(&p.chain, hipEventDisableTiming));
        }
    }

  public:
    LoopbackTransport(void *hub, int n, int r) : hub_((LoopHub *)hub) {
        nranks = n;
        rank = r;
        if (hub_->k != n) throw std::runtime_error("loopback hub size differs from nranks");
    }
    std::unique_ptr<Transport> split(hipStream_t) override {
        return std::unique_ptr<Transport>(new LoopbackTransport(hub_, nranks, rank));
    }
    void exchange(const std::vector<const void *> &send, const std::vector<size_t> &sbytes,
                  const std::vector<void *> &recv, const std::vector<size_t> &rbytes,
                  hipStream_t s) override {
        ensure_events();
        last_op = "exchange, send " + peers_bytes(sbytes, rank) + " recv " + peers_bytes(rbytes, rank);
        auto &me = hub_->post[rank];
        me.send = send;
        me.sbytes = sbytes;
        PFDR_HIP(hipEventRecord(me.ready, s));
        hub_->barrier(*this);
        for (int q = 0; q < nranks; q++) {
            if (q == rank || !rbytes[q]) continue;
            auto &pq = hub_->post[q];
            if (pq.sbytes[rank] != rbytes[q]) throw std::runtime_error("loopback exchange size mismatch");
            PFDR_HIP(hipStreamWaitEvent(s, pq.ready, 0));
            PFDR_HIP(hipMemcpyAsync(recv[q], pq.send[rank], rbytes[q], hipMemcpyDeviceToDevice, s));
        }
        PFDR_HIP(hipEventRecord(me.done, s));
        hub_->barrier(*this);
        for (int q = 0; q < nranks; q++)
            if (q != rank) PFDR_HIP(hipStreamWaitEvent(s, hub_->post[q].done, 0));
        hub_->barrier(*this);  // nobody re-records `done` before every wait is enqueued
    }
    void allreduce_sum(void *dev, int n, int dtype, hipStream_t s) override {
        ensure_events();
        last_op = "all-reduce of " + std::to_string(n) + " values";
        auto &me = hub_->post[rank];
        me.ptr = dev;
        PFDR_HIP(hipEventRecord(me.ready, s));
        hub_->barrier(*this);
        for (int q = 0; q < nranks; q++)
            if (q != rank) PFDR_HIP(hipStreamWaitEvent(s, hub_->post[q].ready, 0));
        const size_t eb = dtype == PFDR_F32 ? 4 : 8;
        DevBuf<char> tmp((size_t)n * eb);
        DevBuf<const void *> ptrs(nranks);
        std::vector<const void *> hp(nranks);
        for (int q = 0; q < nranks; q++) hp[q] = hub_->post[q].ptr;
        PFDR_HIP(hipMemcpyAsync(ptrs.p, hp.data(), sizeof(void *) * nranks, hipMemcpyHostToDevice, s));
        const int g = grid_for(n);
        if (dtype == PFDR_F32)
            k_sum_ranks<float><<<g, kBlock, 0, s>>>(n, nranks, (const float *const *)ptrs.p, (float *)tmp.p);
        else if (dtype == PFDR_F64)
            k_sum_ranks<double><<<g, kBlock, 0, s>>>(n, nranks, (const double *const *)ptrs.p, (double *)tmp.p);
        else
            k_sum_ranks<long long><<<g, kBlock, 0, s>>>(n, nranks, (const long long *const *)ptrs.p,
                                                         (long long *)tmp.p);
        PFDR_HIP(hipGetLastError());
        PFDR_HIP(hipEventRecord(me.done, s));
        hub_->barrier(*this);
        for (int q = 0; q < nranks; q++)
            if (q != rank) PFDR_HIP(hipStreamWaitEvent(s, hub_->post[q].done, 0));
        PFDR_HIP(hipMemcpyAsync(dev, tmp.p, (size_t)n * eb, hipMemcpyDeviceToDevice, s));
        PFDR_HIP(hipStreamSynchronize(s));  // tmp / ptrs die here
        hub_->barrier(*this);
    }
    void chain_recv(void *dev, size_t bytes, hipStream_t s) override {
        ensure_events();
        if (rank == 0) return;
        auto &prev = hub_->post[rank - 1];
        auto &me = hub_->post[rank];
        {
            std::unique_lock<std::mutex> l(hub_->m);
            hub_->wait_until(l, *this, [&] { return prev.chain_seq > me.chain_seq; });
        }
        PFDR_HIP(hipStreamWaitEvent(s, prev.chain, 0));
        PFDR_HIP(hipMemcpyAsync(dev, prev.ptr, bytes, hipMemcpyDeviceToDevice, s));
        PFDR_HIP(hipStreamSynchronize(s));
    }
    void chain_send(const void *dev, size_t bytes, hipStream_t s) override {
        ensure_events();
        auto &me = hub_->post[rank];
        (void)bytes;
        if (rank + 1 < nranks) {
            PFDR_HIP(hipEventRecord(me.chain, s));
            PFDR_HIP(hipStreamSynchronize(s));
            std::unique_lock<std::mutex> l(hub_->m);
            me.ptr = dev;
            me.chain_seq++;
            hub_->cv.notify_all();
        } else {
            std::unique_lock<std::mutex> l(hub_->m);
            me.chain_seq++;
        }
        hub_->barrier(*this);  // keep dev alive until the successor copied it
    }
    void broadcast(void *dev, size_t bytes, int root, hipStream_t s) override {
        ensure_events();
        auto &me = hub_->post[rank];
        if (rank == root) {
            me.ptr = dev;
            PFDR_HIP(hipEventRecord(me.ready, s));
        }
        hub_->barrier(*this);
        if (rank != root) {
            PFDR_HIP(hipStreamWaitEvent(s, hub_->post[root].ready, 0));
            PFDR_HIP(hipMemcpyAsync(dev, hub_->post[root].ptr, bytes, hipMemcpyDeviceToDevice, s));
        }
        PFDR_HIP(hipStreamSynchronize(s));
        hub_->barrier(*this);
    }
};

void loopback_abort(void *hub, const char *reason) {
    static_cast<LoopHub *>(hub)->abort(reason ? reason : "a peer rank failed");
}

std::unique_ptr<Transport> make_loopback_transport(void *hub, int n, int r) {
    return std::unique_ptr<Transport>(new LoopbackTransport(hub, n, r));
}

// ------------------------------------------------------------------ Halo --
void Halo::pull(void *base, int eb, hipStream_t s) {
    const int n = tr->nranks;
    const int tot = pull_send_off[n];
    if ((size_t)tot * eb > sendbuf.n) sendbuf.alloc((size_t)tot * eb);
    pack(tot, pull_idx.p, base, sendbuf.p, eb, s);
    std::vector<const void *> sp(n);
    std::vector<void *> rp(n);
    std::vector<size_t> sb(n), rb(n);
    for (int q = 0; q < n; q++) {
        sp[q] = sendbuf.p + (size_t)pull_send_off[q] * eb;
        sb[q] = (size_t)pull_send_cnt[q] * eb;
        rp[q] = (char *)base + ((size_t)V + ghost_off[q]) * eb;
        rb[q] = (size_t)ghost_cnt[q] * eb;
    }
    tr->exchange(sp, sb, rp, rb, s);
}

void Halo::push(const void *wz, void *tail, int eb, hipStream_t s) {
    pack_u(push_send_off[tr->nranks], push_addr.p, wz, push_buffer(eb), eb, s);
    push_packed(sendbuf.p, tail, eb, s);
}

void *Halo::push_buffer(int eb) {
    const size_t need = (size_t)push_send_off[tr->nranks] * eb;
    if (need > sendbuf.n) sendbuf.alloc(need);
    return sendbuf.p;
}

void Halo::push_packed(const void *packed, void *tail, int eb, hipStream_t s) {
    const int n = tr->nranks;
    std::vector<const void *> sp(n);
    std::vector<void *> rp(n);
    std::vector<size_t> sb(n), rb(n);
    for (int q = 0; q < n; q++) {
        sp[q] = (const char *)packed + (size_t)push_send_off[q] * eb;
        sb[q] = (size_t)push_send_cnt[q] * eb;
        rp[q] = (char *)tail + (size_t)push_recv_off[q] * eb;
        rb[q] = (size_t)push_recv_cnt[q] * eb;
    }
    tr->exchange(sp, sb, rp, rb, s);
}

void plan_local(PlanHost &p, int nranks, int rank, const int64_t *off, long E, const int *Eu_g,
                const int *Ev_g, const int64_t *e_global, int64_t e_offset) {
    const int n = nranks;
    p.nranks = n;
    p.rank = rank;
    p.E = E;
    p.off.assign(off, off + n + 1);
    for (int q = 0; q < n; q++)
        if (p.off[q + 1] < p.off[q]) throw std::runtime_error("partition: offsets must increase");
    p.lo = p.off[rank];
    p.hi = p.off[rank + 1];
    p.V = (int)(p.hi - p.lo);
    const int64_t lo = p.lo, hi = p.hi, Vglob = p.off[n];
    auto owner = [&](int64_t g) {
        return (int)(std::upper_bound(p.off.begin(), p.off.end(), g) - p.off.begin()) - 1;
    };
    // ghosts: endpoints outside the owned range, sorted (hence grouped by owner)
    std::vector<int64_t> &ghosts = p.ghosts;
    ghosts.clear();
    for (long e = 0; e < E; e++) {
        const int64_t u = Eu_g[e], v = Ev_g[e];
        if (u < 0 || u >= Vglob || v < 0 || v >= Vglob)
            throw std::runtime_error("partition: edge endpoint outside [0, V_global)");
        if (u < lo || u >= hi) ghosts.push_back(u);
        if (v < lo || v >= hi) ghosts.push_back(v);
    }
    std::sort(ghosts.begin(), ghosts.end());
    ghosts.erase(std::unique(ghosts.begin(), ghosts.end()), ghosts.end());
    p.ghost_cnt.assign(n, 0);
    for (int64_t g : ghosts) p.ghost_cnt[owner(g)]++;
    p.ghost_off.assign(n + 1, 0);
    for (int q = 0; q < n; q++) p.ghost_off[q + 1] = p.ghost_off[q] + p.ghost_cnt[q];
    const int V = p.V;
    auto local = [&](int64_t g) -> int {
        if (g >= lo && g < hi) return (int)(g - lo);
        return V + (int)(std::lower_bound(ghosts.begin(), ghosts.end(), g) - ghosts.begin());
    };
    p.Eu_l.resize(E);
    p.Ev_l.resize(E);
    p.req.assign(n, {});
    p.items.assign(n, {});
    p.addr.assign(n, {});
    for (int q = 0; q < n; q++)
        p.req[q].assign(ghosts.begin() + p.ghost_off[q], ghosts.begin() + p.ghost_off[q + 1]);
    for (long e = 0; e < E; e++) {
        const int64_t eg = e_global ? e_global[e] : e_offset + e;
        if (eg < 0 || 2 * eg + 1 > 0xffffffffLL)
            throw std::runtime_error("partition: global edge ids must lie in [0, 2^31)");
        for (int side = 0; side < 2; side++) {
            const int64_t g = side ? Ev_g[e] : Eu_g[e];
            const int l = local(g);
            (side ? p.Ev_l : p.Eu_l)[e] = l;
            if (l >= V) {
                const int q = owner(g);
                p.items[q].push_back(g);
                p.items[q].push_back(2 * eg + side);
                p.addr[q].push_back((unsigned)(side * E + e));
            }
        }
    }
}

void plan_finish(PlanHost &p, const std::vector<std::vector<int64_t>> &inreq,
                 const std::vector<std::vector<int64_t>> &initems) {
    const int n = p.nranks, me = p.rank;
    const int64_t lo = p.lo, hi = p.hi;
    p.pull_send_cnt.assign(n, 0);
    p.pull_send_off.assign(n + 1, 0);
    p.pull_idx.clear();
    for (int q = 0; q < n; q++) {
        if (q != me) {
            for (int64_t g : inreq[q]) {
                if (g < lo || g >= hi) throw std::runtime_error("partition: bad pull request");
                p.pull_idx.push_back((int)(g - lo));
            }
            p.pull_send_cnt[q] = (int)inreq[q].size();
        }
        p.pull_send_off[q + 1] = p.pull_send_off[q] + p.pull_send_cnt[q];
    }
    p.push_send_cnt.assign(n, 0);
    p.push_send_off.assign(n + 1, 0);
    p.push_addr.clear();
    for (int q = 0; q < n; q++) {
        p.push_send_cnt[q] = (int)p.addr[q].size();
        p.push_send_off[q + 1] = p.push_send_off[q] + p.push_send_cnt[q];
        p.push_addr.insert(p.push_addr.end(), p.addr[q].begin(), p.addr[q].end());
    }
    p.push_recv_cnt.assign(n, 0);
    p.push_recv_off.assign(n + 1, 0);
    p.recv_keys.clear();
    for (int q = 0; q < n; q++) {
        if (q != me) {
            const auto &it = initems[q];
            for (size_t j = 0; j + 1 < it.size(); j += 2) {
                const int64_t g = it[j];
                if (g < lo || g >= hi) throw std::runtime_error("partition: bad push item");
                p.recv_keys.push_back(((unsigned long long)(g - lo) << 32) |
                                      (unsigned long long)it[j + 1]);
            }
            p.push_recv_cnt[q] = (int)(it.size() / 2);
        }
        p.push_recv_off[q + 1] = p.push_recv_off[q] + p.push_recv_cnt[q];
    }
}

void build_halo(Halo &h, int V, int64_t vtx_begin, long E, const int *Eu_g, const int *Ev_g,
                const int64_t *e_global, int64_t e_offset, std::vector<int> &Eu_l,
                std::vector<int> &Ev_l, hipStream_t s) {
    Transport &tr = *h.tr;
    const int n = tr.nranks, me = tr.rank;
    // global offsets (rank order must be vertex order)
    std::vector<int64_t> cnt;
    tr.allgather_i64(V, cnt, s);
    std::vector<int64_t> off(n + 1, 0);
    for (int q = 0; q < n; q++) off[q + 1] = off[q] + cnt[q];
    if (off[me] != vtx_begin)
        throw std::runtime_error("partition: vtx_begin must equal the sum of V over lower ranks");
    PlanHost p;
    plan_local(p, n, me, off.data(), E, Eu_g, Ev_g, e_global, e_offset);
    std::vector<std::vector<int64_t>> inreq, initems;
    tr.alltoallv_host(p.req, inreq, s);
    tr.alltoallv_host(p.items, initems, s);
    plan_finish(p, inreq, initems);
    h.V = V;
    h.E = E;
    h.vtx_begin = vtx_begin;
    h.off = off;
    h.G = (int)p.ghosts.size();
    h.ghost_cnt = p.ghost_cnt;
    h.ghost_off = p.ghost_off;
    h.pull_send_cnt = p.pull_send_cnt;
    h.pull_send_off = p.pull_send_off;
    h.push_send_cnt = p.push_send_cnt;
    h.push_send_off = p.push_send_off;
    h.push_recv_cnt = p.push_recv_cnt;
    h.push_recv_off = p.push_recv_off;
    h.R = (long)p.recv_keys.size();
    h.pull_idx.alloc(p.pull_idx.size() ? p.pull_idx.size() : 1);
    if (!p.pull_idx.empty())
        PFDR_HIP(hipMemcpyAsync(h.pull_idx.p, p.pull_idx.data(), sizeof(int) * p.pull_idx.size(),
                                hipMemcpyHostToDevice, s));
    h.push_addr.alloc(p.push_addr.size() ? p.push_addr.size() : 1);
    if (!p.push_addr.empty())
        PFDR_HIP(hipMemcpyAsync(h.push_addr.p, p.push_addr.data(),
                                sizeof(unsigned) * p.push_addr.size(), hipMemcpyHostToDevice, s));
    h.recv_keys.alloc(p.recv_keys.size() ? p.recv_keys.size() : 1);
    if (!p.recv_keys.empty())
        PFDR_HIP(hipMemcpyAsync(h.recv_keys.p, p.recv_keys.data(),
                                sizeof(unsigned long long) * p.recv_keys.size(),
                                hipMemcpyHostToDevice, s));
    Eu_l.swap(p.Eu_l);
    Ev_l.swap(p.Ev_l);
    PFDR_HIP(hipStreamSynchronize(s));
}

void partition_setup(const pfdr_problem *p, int V, long E, std::unique_ptr<Halo> &halo,
                     DevBuf<int> &Eu, DevBuf<int> &Ev, DevBuf<unsigned> &eg, long *e_offset,
                     hipStream_t s) {
    if (p->nranks < 1 || p->rank < 0 || p->rank >= p->nranks || !p->comm)
        throw std::runtime_error("distributed session needs nranks, rank and comm");
    halo.reset(new Halo());
    halo->tr = p->comm_kind == PFDR_COMM_LOOPBACK
                   ? make_loopback_transport(p->comm, p->nranks, p->rank)
                   : make_rccl_transport(p->comm, p->nranks, p->rank);
    // the plan is built on the host from the global endpoint ids
    std::vector<int> hu, hv, lu, lv;
    std::vector<int64_t> heg;
    const int *pu = p->Eu, *pv = p->Ev;
    const int64_t *peg = p->e_global;
    if (p->mem == PFDR_MEM_DEVICE) {
        hu.resize(E); hv.resize(E);
        PFDR_HIP(hipMemcpy(hu.data(), p->Eu, E * 4, hipMemcpyDeviceToHost));
        PFDR_HIP(hipMemcpy(hv.data(), p->Ev, E * 4, hipMemcpyDeviceToHost));
        pu = hu.data(); pv = hv.data();
        if (peg) {
            heg.resize(E);
            PFDR_HIP(hipMemcpy(heg.data(), p->e_global, E * 8, hipMemcpyDeviceToHost));
            peg = heg.data();
        }
    }
    build_halo(*halo, V, p->vtx_begin, E, pu, pv, peg, p->e_offset, lu, lv, s);
    Eu.alloc(E ? E : 1);
    Ev.alloc(E ? E : 1);
    if (E) {
        PFDR_HIP(hipMemcpyAsync(Eu.p, lu.data(), E * 4, hipMemcpyHostToDevice, s));
        PFDR_HIP(hipMemcpyAsync(Ev.p, lv.data(), E * 4, hipMemcpyHostToDevice, s));
    }
    *e_offset = 0;
    if (peg) {
        std::vector<unsigned> e32(E);
        for (long e = 0; e < E; e++) e32[e] = (unsigned)peg[e];
        eg.alloc(E ? E : 1);
        PFDR_HIP(hipMemcpyAsync(eg.p, e32.data(), E * 4, hipMemcpyHostToDevice, s));
    } else {
        *e_offset = (long)p->e_offset;
    }
    PFDR_HIP(hipStreamSynchronize(s));
}

// keys of the 2E local slots (rows >= V dropped: ghost ends are pushed)
__global__ void k_slot_keys(long E, const int *__restrict__ Eu, const int *__restrict__ Ev,
                            int V, const unsigned *__restrict__ eg, long e_offset,
                            unsigned long long *__restrict__ keys, unsigned *__restrict__ vals) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const unsigned long long g = eg ? (unsigned long long)eg[e] : (unsigned long long)(e_offset + e);
    const int u = Eu[e], v = Ev[e];
    keys[e] = (u < V) ? (((unsigned long long)u << 32) | (2 * g)) : ~0ull;
    keys[E + e] = (v < V) ? (((unsigned long long)v << 32) | (2 * g + 1)) : ~0ull;
    vals[e] = (unsigned)e;
    vals[E + e] = (unsigned)(E + e);
}

// rows of the 2E local slots in slot order 2e + side (rows >= V -> V)
__global__ void k_slot_rows(long E, const int *__restrict__ Eu, const int *__restrict__ Ev, int V,
                            unsigned *__restrict__ rows, unsigned *__restrict__ vals) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const int u = Eu[e], v = Ev[e];
    reinterpret_cast<uint2 *>(rows)[e] = make_uint2(u < V ? u : V, v < V ? v : V);
    reinterpret_cast<uint2 *>(vals)[e] = make_uint2((unsigned)e, (unsigned)(E + e));
}

void contribution_incidence(const int *Eu, const int *Ev, long E, int V, const unsigned *eg,
                            long e_offset, const Halo *halo, Incidence &inc, hipStream_t s) {
    const long R = halo ? halo->R : 0;
    const long n = 2 * E + R;
    if (!R && !eg && E) {
        // edge ids ascend with e and nothing is received: listed in slot
        // order, the slots only need a STABLE sort by row (radix passes over
        // the row bits alone, 32-bit keys)
        DevBuf<unsigned> rows(n), vals(n), srows(n);
        k_slot_rows<<<grid_for(E), kBlock, 0, s>>>(E, Eu, Ev, V, rows.p, vals.p);
        PFDR_HIP(hipGetLastError());
        build_incidence_rows(rows.p, srows.p, vals.p, n, V, inc, s);
        return;
    }
    DevBuf<unsigned long long> keys(n ? n : 1);
    DevBuf<unsigned> vals(n ? n : 1);
    if (E) {
        k_slot_keys<<<grid_for(E), kBlock, 0, s>>>(E, Eu, Ev, V, eg, e_offset, keys.p, vals.p);
        PFDR_HIP(hipGetLastError());
    }
    if (R) {
        PFDR_HIP(hipMemcpyAsync(keys.p + 2 * E, halo->recv_keys.p, R * sizeof(unsigned long long),
                                hipMemcpyDeviceToDevice, s));
        std::vector<unsigned> tail(R);
        for (long j = 0; j < R; j++) tail[j] = (unsigned)(2 * E + j);
        PFDR_HIP(hipMemcpyAsync(vals.p + 2 * E, tail.data(), R * 4, hipMemcpyHostToDevice, s));
        PFDR_HIP(hipStreamSynchronize(s));
    }
    build_incidence_keyed(keys.p, vals.p, n, V, inc, s);
}

static __global__ void k_label_count(int n, const int *__restrict__ lab,
                                     unsigned long long *__restrict__ cnt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) atomicAdd(&cnt[lab[i]], 1ull);
}
static __global__ void k_count_not_one(long n, const unsigned long long *__restrict__ cnt,
                                       unsigned long long *__restrict__ bad) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && cnt[i] != 1ull) atomicAdd(bad, 1ull);
}

// the labels of all ranks (vtx_label) must be a permutation of [0, V_global):
// the relabelled amplitude and evolution sums all-reduce arrays with one
// writer per position (collective, once at setup)
void check_permutation(const int *lab, int V, long Vglob, Transport &tr, hipStream_t s) {
    DevBuf<unsigned long long> cnt(Vglob), bad(1);
    PFDR_HIP(hipMemsetAsync(cnt.p, 0, sizeof(unsigned long long) * Vglob, s));
    PFDR_HIP(hipMemsetAsync(bad.p, 0, sizeof(unsigned long long), s));
    if (V) k_label_count<<<grid_for(V), kBlock, 0, s>>>(V, lab, cnt.p);
    PFDR_HIP(hipGetLastError());
    if (Vglob > 0x7fffffffL) throw std::runtime_error("V_global too large");
    tr.allreduce_sum(cnt.p, (int)Vglob, 2, s);
    k_count_not_one<<<grid_for(Vglob), kBlock, 0, s>>>(Vglob, cnt.p, bad.p);
    PFDR_HIP(hipGetLastError());
    unsigned long long nb = 0;
    PFDR_HIP(hipMemcpyAsync(&nb, bad.p, sizeof(nb), hipMemcpyDeviceToHost, s));
    tr.wait(s);
    if (nb) throw std::runtime_error("vtx_label of the ranks is not a permutation of [0, V_global)");
}

}  // namespace pfdr

extern "C" int pfdr_loopback_create(void **hub_out, int nranks) {
    if (!hub_out || nranks < 1 || nranks > 64)
        return pfdr::report_error("pfdr_loopback_create", "invalid arguments");
    *hub_out = new pfdr::LoopHub(nranks);
    return PFDR_OK;
}

extern "C" int pfdr_loopback_abort(void *hub, const char *reason) {
    if (!hub) return pfdr::report_error("pfdr_loopback_abort", "null hub");
    pfdr::loopback_abort(hub, reason);
    return PFDR_OK;
}

extern "C" int pfdr_loopback_destroy(void *hub) {
    delete (pfdr::LoopHub *)hub;
    return PFDR_OK;
}

// ---------------------------------------------- host planner (C ABI) --
struct pfdr_plan {
    pfdr::PlanHost p;
    std::vector<std::vector<int64_t>> inreq, initems;
};

extern "C" int pfdr_plan_create(pfdr_plan **out, int nranks, int rank, const int64_t *offsets,
                                int E, const int *Eu, const int *Ev, const int64_t *e_global,
                                int64_t e_offset) {
    if (!out || nranks < 1 || rank < 0 || rank >= nranks || !offsets || E < 0 ||
        (E > 0 && (!Eu || !Ev)))
        return pfdr::report_error("pfdr_plan_create", "invalid arguments");
    try {
        pfdr_plan *pl = new pfdr_plan();
        pfdr::plan_local(pl->p, nranks, rank, offsets, E, Eu, Ev, e_global, e_offset);
        pl->inreq.assign(nranks, {});
        pl->initems.assign(nranks, {});
        *out = pl;
    } catch (const std::exception &ex) {
        return pfdr::report_error("pfdr_plan_create", ex.what());
    }
    return PFDR_OK;
}

template <typename T>
static int64_t copy_out(const std::vector<T> &v, void *out) {
    if (out && !v.empty()) memcpy(out, v.data(), v.size() * sizeof(T));
    return (int64_t)v.size();
}

extern "C" int64_t pfdr_plan_get(pfdr_plan *pl, int what, int peer, void *out) {
    if (!pl) return -1;
    const auto &p = pl->p;
    if (peer < 0 || peer >= p.nranks) peer = 0;
    switch (what) {
        case PFDR_PLAN_GHOSTS: return copy_out(p.ghosts, out);
        case PFDR_PLAN_EU_LOCAL: return copy_out(p.Eu_l, out);
        case PFDR_PLAN_EV_LOCAL: return copy_out(p.Ev_l, out);
        case PFDR_PLAN_PULL_REQUEST: return copy_out(p.req[peer], out);
        case PFDR_PLAN_PUSH_ITEMS: return copy_out(p.items[peer], out);
        case PFDR_PLAN_PUSH_ADDR: return copy_out(p.push_addr, out);
        case PFDR_PLAN_PULL_INDEX: return copy_out(p.pull_idx, out);
        case PFDR_PLAN_RECV_KEYS: return copy_out(p.recv_keys, out);
        case PFDR_PLAN_GHOST_OFFSETS: return copy_out(p.ghost_off, out);
        case PFDR_PLAN_PULL_OFFSETS: return copy_out(p.pull_send_off, out);
        case PFDR_PLAN_PUSH_OFFSETS: return copy_out(p.push_send_off, out);
        case PFDR_PLAN_RECV_OFFSETS: return copy_out(p.push_recv_off, out);
        default: return -1;
    }
}

extern "C" int pfdr_plan_set_incoming(pfdr_plan *pl, int peer, int what, int64_t n,
                                      const int64_t *data) {
    if (!pl || peer < 0 || peer >= pl->p.nranks || n < 0 || (n > 0 && !data))
        return pfdr::report_error("pfdr_plan_set_incoming", "invalid arguments");
    if (what == PFDR_PLAN_PULL_REQUEST) pl->inreq[peer].assign(data, data + n);
    else if (what == PFDR_PLAN_PUSH_ITEMS) pl->initems[peer].assign(data, data + n);
    else return pfdr::report_error("pfdr_plan_set_incoming", "what must be PULL_REQUEST or PUSH_ITEMS");
    return PFDR_OK;
}

extern "C" int pfdr_plan_finish(pfdr_plan *pl) {
    if (!pl) return pfdr::report_error("pfdr_plan_finish", "null plan");
    try {
        pfdr::plan_finish(pl->p, pl->inreq, pl->initems);
    } catch (const std::exception &ex) {
        return pfdr::report_error("pfdr_plan_finish", ex.what());
    }
    return PFDR_OK;
}

extern "C" void pfdr_plan_destroy(pfdr_plan *pl) { delete pl; }
