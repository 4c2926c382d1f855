// msx_transport.cpp — bootstrap hub, IPC peer mapping, schedules and engine.
//
// Reference anchors (src/mpi/msmpi/mpid/reduce.cpp):
//   MPIR_Allreduce_intra_flat            :3768-4104  (fold, RD / Rabenseifner, unfold)
//   MPIR_Reduce_scatter_intra_impl       :1636-1770  (algorithm gate, 32-bit nbytes)
//   MPIR_Reduce_scatter_commutative_short:917-1219   (recursive halving)
//   MPIR_Reduce_scatter_commutative_long :1225-1334  (pairwise exchange)
// The reference moves partial results between ranks step by step
// (MPIC_Sendrecv) and combines after each step (MPID_Uop_call).  Here each
// rank reads every contribution it needs straight from its peers' HBM and
// evaluates the SAME expression tree (same association, same inout/in roles)
// in one kernel, so results are bit-identical to the reference schedule.
#include "msx_transport.h"

#include <arpa/inet.h>
#include <condition_variable>
#include <deque>
#include <errno.h>
#include <functional>
#include <future>
#include <map>
#include <mutex>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>
#include <sys/socket.h>
#include <thread>
#include <unistd.h>

#include "msx_kernels.h"
#include "msx_runtime.h"

namespace msx {

// ===========================================================================
// bootstrap hub: rank 0 listens, every other rank keeps one TCP connection
// ===========================================================================
namespace {

double now_s()
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int io_all(int fd, void* buf, size_t n, bool wr, double timeout_s)
{
    char* p = static_cast<char*>(buf);
    const double t_end = now_s() + timeout_s;
    while (n) {
        struct pollfd pf = {fd, (short)(wr ? POLLOUT : POLLIN), 0};
        int ms = (int)((t_end - now_s()) * 1000);
        if (ms <= 0) { set_error("bootstrap: timed out"); return MPI_ERR_OTHER; }
        int pr = poll(&pf, 1, ms < 1000 ? ms : 1000);
        if (pr < 0 && errno == EINTR) continue;
        if (pr < 0) { set_error("bootstrap poll: %s", strerror(errno)); return MPI_ERR_OTHER; }
        if (pr == 0) continue;
        ssize_t k = wr ? send(fd, p, n, MSG_NOSIGNAL) : recv(fd, p, n, 0);
        if (k < 0 && (errno == EINTR || errno == EAGAIN)) continue;
        if (k <= 0) { set_error("bootstrap: peer connection lost (%s)", k ? strerror(errno) : "eof"); return MPI_ERR_OTHER; }
        p += k;
        n -= (size_t)k;
    }
    return MPI_SUCCESS;
}

class Hub {
public:
    ~Hub()
    {
        for (int fd : fd_) if (fd >= 0) close(fd);
        if (lfd_ >= 0) close(lfd_);
    }

    int init(int rank, int size)
    {
        rank_ = rank;
        size_ = size;
        timeout_ = 600.0;
        if (const char* t = getenv("MSX_BOOTSTRAP_TIMEOUT")) timeout_ = atof(t);
        const char* addr = getenv("MSX_BOOTSTRAP_ADDR");
        if (!addr) addr = getenv("MASTER_ADDR");
        if (!addr) addr = "127.0.0.1";
        int port = 29571;
        if (const char* v = getenv("MSX_BOOTSTRAP_PORT")) port = atoi(v);
        else if (const char* v = getenv("MASTER_PORT")) port = (atoi(v) + 97) % 65536;
        if (port < 1024) port += 1024;

        struct addrinfo hints = {}, *res = nullptr;
        hints.ai_family = AF_INET;
        hints.ai_socktype = SOCK_STREAM;
        char ps[16];
        snprintf(ps, sizeof(ps), "%d", port);
        if (getaddrinfo(addr, ps, &hints, &res) != 0 || !res) {
            set_error("bootstrap: cannot resolve %s", addr);
            return MPI_ERR_OTHER;
        }
        struct sockaddr_in sa;
        memcpy(&sa, res->ai_addr, sizeof(sa));
        freeaddrinfo(res);
        fd_.assign((size_t)size, -1);

        if (rank == 0) {
            lfd_ = socket(AF_INET, SOCK_STREAM, 0);
            int one = 1;
            setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
            struct sockaddr_in any = sa;
            if (bind(lfd_, (struct sockaddr*)&any, sizeof(any)) != 0) {
                set_error("bootstrap: bind %s:%d: %s", addr, port, strerror(errno));
                return MPI_ERR_OTHER;
            }
            listen(lfd_, size + 8);
            const double t_end = now_s() + timeout_;
            for (int got = 1; got < size;) {
                struct pollfd pf = {lfd_, POLLIN, 0};
                int ms = (int)((t_end - now_s()) * 1000);
                if (ms <= 0) { set_error("bootstrap: only %d of %d ranks connected", got, size); return MPI_ERR_OTHER; }
                if (poll(&pf, 1, ms) <= 0) continue;
                int fd = accept(lfd_, nullptr, nullptr);
                if (fd < 0) continue;
                setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
                int32_t r = -1;
                if (io_all(fd, &r, 4, false, timeout_) != MPI_SUCCESS || r <= 0 || r >= size || fd_[r] >= 0) {
                    close(fd);
                    continue;
                }
                fd_[r] = fd;
                ++got;
            }
        } else {
            const double t_end = now_s() + timeout_;
            int fd = -1;
            while (true) {
                fd = socket(AF_INET, SOCK_STREAM, 0);
                if (connect(fd, (struct sockaddr*)&sa, sizeof(sa)) == 0) break;
                close(fd);
                fd = -1;
                if (now_s() > t_end) { set_error("bootstrap: cannot reach rank 0 at %s:%d", addr, port); return MPI_ERR_OTHER; }
                usleep(20000);
            }
            int one = 1;
            setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
            int32_t r = rank;
            if (io_all(fd, &r, 4, true, timeout_) != MPI_SUCCESS) { close(fd); return MPI_ERR_OTHER; }
            fd_[0] = fd;
        }
        return MPI_SUCCESS;
    }

    // Every rank contributes n bytes; all receive size*n bytes in rank order.
    int allgather(const void* mine, size_t n, void* all)
    {
        std::lock_guard<std::mutex> g(mu_);
        char* out = static_cast<char*>(all);
        if (rank_ == 0) {
            memcpy(out, mine, n);
            for (int r = 1; r < size_; ++r)
                if (io_all(fd_[r], out + (size_t)r * n, n, false, timeout_) != MPI_SUCCESS) return MPI_ERR_OTHER;
            for (int r = 1; r < size_; ++r)
                if (io_all(fd_[r], out, (size_t)size_ * n, true, timeout_) != MPI_SUCCESS) return MPI_ERR_OTHER;
            return MPI_SUCCESS;
        }
        if (io_all(fd_[0], const_cast<void*>(mine), n, true, timeout_) != MPI_SUCCESS) return MPI_ERR_OTHER;
        return io_all(fd_[0], out, (size_t)size_ * n, false, timeout_);
    }

private:
    int rank_ = 0, size_ = 1, lfd_ = -1;
    double timeout_ = 600.0;
    std::vector<int> fd_;
    std::mutex mu_;
};

// ===========================================================================
// IPC transport
// ===========================================================================
struct IpcRec {
    hipIpcMemHandle_t h;
    uint64_t offset;
    int32_t ok;
    int32_t pad;
};

class IpcTransport : public Transport {
public:
    ~IpcTransport() override
    {
        for (auto& kv : opened_) (void)hipIpcCloseMemHandle(kv.second);
        if (win_) (void)hipFree(win_);
        if (stream_) (void)hipStreamDestroy(stream_);
    }

    int init(int r, int s)
    {
        rank = r;
        size = s;
        return hub_.init(r, s);
    }

    int allgather(const void* mine, size_t n, void* all) override { return hub_.allgather(mine, n, all); }

    int barrier() override
    {
        char b = 0;
        std::vector<char> all((size_t)size);
        return hub_.allgather(&b, 1, all.data());
    }

    hipStream_t stream() override
    {
        if (!stream_) (void)hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking);
        return stream_;
    }

    int map_peers(const void* ptr, std::vector<char*>& out) override
    {
        IpcRec mine;
        memset(&mine, 0, sizeof(mine));
        void* base = nullptr;
        size_t asz = 0;
        hipError_t e = hipMemGetAddressRange(&base, &asz, const_cast<void*>(ptr));
        trace("map_peers: ptr=%p base=%p size=%zu rc=%d", ptr, base, asz, (int)e);
        if (e == hipSuccess) e = hipIpcGetMemHandle(&mine.h, base);
        trace("map_peers: handle rc=%d", (int)e);
        if (e == hipSuccess) {
            mine.ok = 1;
            mine.offset = (uint64_t)((const char*)ptr - (const char*)base);
        } else {
            (void)hipGetLastError();
            set_error("rank %d: buffer %p cannot be shared over IPC (%s)", rank, ptr, hipGetErrorString(e));
        }
        std::vector<IpcRec> all((size_t)size);
        int rc = hub_.allgather(&mine, sizeof(mine), all.data());
        trace("map_peers: exchanged rc=%d", rc);
        if (rc != MPI_SUCCESS) return rc;
        out.assign((size_t)size, nullptr);
        for (int r = 0; r < size; ++r) {
            if (!all[r].ok) {
                if (r != rank) set_error("rank %d's buffer cannot be shared over IPC", r);
                return MPI_ERR_OTHER;
            }
            if (r == rank) { out[r] = const_cast<char*>(static_cast<const char*>(ptr)); continue; }
            std::string key(reinterpret_cast<const char*>(&all[r].h), sizeof(hipIpcMemHandle_t));
            auto it = opened_.find(key);
            void* pbase = nullptr;
            if (it != opened_.end()) {
                pbase = it->second;
            } else {
                e = hipIpcOpenMemHandle(&pbase, all[r].h, hipIpcMemLazyEnablePeerAccess);
                trace("map_peers: opened rank %d handle -> %p rc=%d", r, pbase, (int)e);
                if (e != hipSuccess) return hip_fail(e, "hipIpcOpenMemHandle");
                opened_[key] = pbase;
            }
            out[r] = static_cast<char*>(pbase) + all[r].offset;
        }
        return MPI_SUCCESS;
    }

    int window(size_t bytes, std::vector<char*>& out) override
    {
        // Collective: every rank asks for the same size.
        if (bytes > win_bytes_) {
            if (win_) {
                (void)hipFree(win_);
                win_ = nullptr;
            }
            size_t want = bytes < ((size_t)1 << 20) ? ((size_t)1 << 20) : bytes;
            hipError_t e = hipMalloc(&win_, want);
            if (e != hipSuccess) return hip_fail(e, "window hipMalloc");
            win_bytes_ = want;
            win_peers_.clear();
        }
        if (win_peers_.empty()) {
            int rc = map_peers(win_, win_peers_);
            if (rc != MPI_SUCCESS) return rc;
        }
        out = win_peers_;
        return MPI_SUCCESS;
    }

private:
    Hub hub_;
    hipStream_t stream_ = nullptr;
    std::map<std::string, void*> opened_;
    void* win_ = nullptr;
    size_t win_bytes_ = 0;
    std::vector<char*> win_peers_;
};

}  // namespace

int transport_create(int rank, int size, Transport** out)
{
    auto* t = new IpcTransport();
    int rc = t->init(rank, size);
    if (rc != MPI_SUCCESS) {
        delete t;
        return rc;
    }
    *out = t;
    return MPI_SUCCESS;
}

void transport_destroy(Transport* t) { delete t; }

// ===========================================================================
// schedules
// ===========================================================================
int pof2_floor(int p)
{
    int v = 1;
    while (v * 2 <= p) v *= 2;
    return v;
}

int newrank_of(int rank, int p)
{
    const int rem = p - pof2_floor(p);
    if (rank < 2 * rem) return (rank & 1) ? rank / 2 : -1;
    return rank - rem;
}

int real_of_newrank(int n, int p)
{
    const int rem = p - pof2_floor(p);
    return n < rem ? 2 * n + 1 : n + rem;
}

Leaf leaf_of(int n, int p)
{
    // fold: odd rank 2n+1 computes MPID_Uop_call(tmp=x_{2n}, recvbuf=x_{2n+1})
    // (reduce.cpp:3858-3865): inout = x_{2n+1}, in = x_{2n}.
    const int rem = p - pof2_floor(p);
    Leaf l;
    if (n < rem) { l.a = 2 * n + 1; l.b = 2 * n; }
    else { l.a = n + rem; }
    return l;
}

int allreduce_algo(int p, size_t count, int type_size, bool builtin)
{
    // reduce.cpp:3884-3888; count*type_size is evaluated in 32 bits.
    const uint32_t nbytes = (uint32_t)((uint64_t)count * (uint64_t)type_size);
    if (nbytes <= 262144u || !builtin || count < (size_t)pof2_floor(p)) return A_RECURSIVE_DOUBLING;
    return A_RABENSEIFNER;
}

int reduce_scatter_algo(int p, size_t total_count, int type_size, bool commutative)
{
    (void)p;
    if (!commutative) return -1;
    // reduce.cpp:1705: nbytes = (unsigned)(total_count * type_size) wraps at 4 GiB.
    const uint32_t nbytes = (uint32_t)((uint64_t)total_count * (uint64_t)type_size);
    return nbytes < 524288u ? A_RS_HALVING : A_RS_PAIRWISE;
}

static int log2i(int v)
{
    int l = 0;
    while ((1 << l) < v) ++l;
    return l;
}

static int bitrev(int x, int bits)
{
    int r = 0;
    for (int i = 0; i < bits; ++i) r |= ((x >> i) & 1) << (bits - 1 - i);
    return r;
}

void allreduce_block(int p, size_t count, int j, size_t* start, size_t* len)
{
    const int pof2 = pof2_floor(p);
    const size_t rs = count / (size_t)pof2, es = count % (size_t)pof2;
    *start = (size_t)j * rs;
    *len = rs + (j == pof2 - 1 ? es : 0);   // endSize on the last block (:3935-3936)
}

// Recursive halving with mask = 1, 2, 4, ... keeps the lower half when the
// newrank bit is 0: the final block of newrank n is bitrev(n).
int allreduce_block_of_newrank(int p, int n) { return bitrev(n, log2i(pof2_floor(p))); }
int allreduce_block_owner(int p, int j) { return bitrev(j, log2i(pof2_floor(p))); }

static RankTree tree_from_leaves(int p, const int* leaf_newranks, int P)
{
    RankTree t;
    t.P = P;
    t.chain = false;
    t.pairmask = 0;
    for (int i = 0; i < 32; ++i) t.src[i] = -1;
    for (int k = 0; k < P; ++k) {
        Leaf l = leaf_of(leaf_newranks[k], p);
        t.src[2 * k] = l.a;
        if (l.b >= 0) {
            t.src[2 * k + 1] = l.b;
            t.pairmask |= 1u << k;
        }
    }
    return t;
}

RankTree tree_allreduce(int p, int n)
{
    const int P = pof2_floor(p);
    int lv[16];
    for (int k = 0; k < P; ++k) lv[k] = n ^ k;   // step mask pairs with n^mask
    return tree_from_leaves(p, lv, P);
}

RankTree tree_reduce_scatter(int p, int n)
{
    const int P = pof2_floor(p);
    const int bits = log2i(P);
    int lv[16];
    for (int k = 0; k < P; ++k) lv[k] = n ^ bitrev(k, bits);   // masks P/2, ..., 1
    return tree_from_leaves(p, lv, P);
}

RankTree tree_pairwise(int p, int r)
{
    RankTree t;
    t.P = p;
    t.chain = true;
    for (int i = 0; i < 32; ++i) t.src[i] = -1;
    for (int k = 0; k < p; ++k) t.src[k] = ((r - k) % p + p) % p;   // src = r-1, r-2, ...
    return t;
}

// ===========================================================================
// engine
// ===========================================================================
namespace {

// Collectives on one communicator run in issue order on one worker thread,
// so blocking and non-blocking calls share the hub in the order every rank
// issued them (MPI requires the same order on all ranks).
class Worker {
public:
    ~Worker()
    {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        if (th_.joinable()) th_.join();
    }
    std::shared_future<int> submit(std::function<int()> fn)
    {
        if (std::this_thread::get_id() == tid_) {
            // re-entrant call from a collective already on the worker: run inline
            std::promise<int> pr;
            pr.set_value(fn());
            return pr.get_future().share();
        }
        auto task = std::make_shared<std::packaged_task<int()>>(std::move(fn));
        std::shared_future<int> f = task->get_future().share();
        {
            std::lock_guard<std::mutex> g(mu_);
            if (!th_.joinable()) {
                th_ = std::thread([this] { loop(); });
                tid_ = th_.get_id();
            }
            q_.push_back(task);
        }
        cv_.notify_all();
        return f;
    }

private:
    void loop()
    {
        for (;;) {
            std::shared_ptr<std::packaged_task<int()>> t;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [this] { return stop_ || !q_.empty(); });
                if (q_.empty()) return;
                t = q_.front();
                q_.pop_front();
            }
            (*t)();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::shared_ptr<std::packaged_task<int()>>> q_;
    std::thread th_;
    std::thread::id tid_;
    bool stop_ = false;
};

Worker& worker()
{
    static Worker w;
    return w;
}

int sync_stream(hipStream_t s, const char* what)
{
    hipError_t e = hipStreamSynchronize(s);
    return e == hipSuccess ? MPI_SUCCESS : hip_fail(e, what);
}

// A device-resident view of a user buffer: the buffer itself if it is in
// HBM, else a staging slice of the window.
struct DevView {
    char* dev = nullptr;
    bool staged = false;
};

// Evaluate RankTree `t` over [start, start+len) elements of the per-rank
// source pointers `srcs` into `out`.
int run_rank_tree(int opidx, Kind k, const RankTree& t, const std::vector<char*>& srcs, size_t esz,
                  size_t start, size_t len, char* out, hipStream_t s)
{
    if (len == 0) return MPI_SUCCESS;
    TreeSpec spec;
    spec.P = t.P;
    spec.pairmask = t.pairmask;
    spec.chain = t.chain;
    spec.sys = true;
    const int nslots = t.chain ? t.P : 2 * t.P;
    for (int i = 0; i < nslots; ++i)
        spec.src[i] = t.src[i] >= 0 ? srcs[(size_t)t.src[i]] + start * esz : nullptr;
    hipError_t e = launch_tree_spec(opidx, k, spec, out, len, s);
    return e == hipSuccess ? MPI_SUCCESS : hip_fail(e, "tree combine");
}

// ---- host path for user-defined ops --------------------------------------
// User functions are host code; gather every contribution to host memory and
// evaluate the reference's recursive-doubling order (reduce.cpp:3890-3925,
// non-commutative branch included) with the user's function.
int host_user_allreduce(Comm* c, const void* sendbuf, void* recvbuf, size_t count,
                        MPI_Datatype dt, const OpRef& op)
{
    const int p = c->size, esz = type_size(dt);
    const size_t bytes = count * (size_t)esz;
    std::vector<char> mine(bytes), all((size_t)p * bytes);
    int rc = copy_any(mine.data(), sendbuf == MPI_IN_PLACE ? recvbuf : sendbuf, bytes);
    if (rc == MPI_SUCCESS) rc = c->tp->allgather(mine.data(), bytes, all.data());
    if (rc != MPI_SUCCESS) return rc;
    auto call = [&](const char* in, char* io) {
        size_t off = 0;
        while (off < count) {
            size_t n = count - off;
            if (n > 0x7fffffff) n = 0x7fffffff;
            int len = (int)n;
            MPI_Datatype d = dt;
            op.user_fn(const_cast<char*>(in) + off * esz, io + off * esz, &len, &d);
            off += n;
        }
    };
    // Simulate every rank's recursive doubling; keep our own rank's result.
    const int pof2 = pof2_floor(p), rem = p - pof2;
    std::vector<std::vector<char>> v((size_t)p);
    for (int r = 0; r < p; ++r) v[r].assign(all.begin() + (size_t)r * bytes, all.begin() + (size_t)(r + 1) * bytes);
    for (int r = 0; r < 2 * rem; r += 2) call(v[r].data(), v[r + 1].data());   // fold into odd
    for (int mask = 1; mask < pof2; mask <<= 1) {
        std::vector<std::vector<char>> nv = v;
        for (int n = 0; n < pof2; ++n) {
            const int r = real_of_newrank(n, p), dst = real_of_newrank(n ^ mask, p);
            if (op.commutative || dst < r) {
                call(v[dst].data(), nv[r].data());
            } else {
                std::vector<char> tmp = v[dst];
                call(v[r].data(), tmp.data());
                nv[r] = tmp;
            }
        }
        v.swap(nv);
    }
    const int me = c->rank;
    const int src = (me < 2 * rem && (me & 1) == 0) ? me + 1 : me;
    return copy_any(recvbuf, v[src].data(), bytes);
}

int do_allreduce(Comm* c, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
                 const OpRef& op)
{
    // user functions are host code: no GPU needed on this path
    if (op.opidx == O_NULL) return host_user_allreduce(c, sendbuf, recvbuf, count, dt, op);
    int rc = ensure_device();
    if (rc != MPI_SUCCESS) return rc;

    Transport* tp = c->tp;
    const int p = c->size, me = c->rank;
    const TypeInfo* ti = type_info(dt);
    const Kind k = ti->kind;
    const size_t esz = (size_t)ti->size, bytes = count * esz;
    hipStream_t s = tp->stream();
    const void* src = (sendbuf == MPI_IN_PLACE) ? recvbuf : sendbuf;
    const bool in_place = (sendbuf == MPI_IN_PLACE);
    const BufInfo bsrc = classify(src), bdst = classify(recvbuf);
    const int algo = allreduce_algo(p, count, (int)esz, true);

    // Window layout: [0, bytes) staged input, [bytes, 2*bytes) result/temp.
    // Every rank decides identically whether it needs the window? No: staging
    // is per-rank, so the window is sized collectively for the worst case.
    const bool need_stage_in = bsrc.place != Place::Device;
    const bool need_stage_out = bdst.place != Place::Device;
    // Recursive doubling reads every peer's whole input, so an in-place result
    // goes to a temporary until the closing barrier.
    const bool need_temp = (algo == A_RECURSIVE_DOUBLING) && in_place;
    uint8_t need = (uint8_t)(need_stage_in || need_stage_out || need_temp);
    std::vector<uint8_t> needs((size_t)p);
    rc = tp->allgather(&need, 1, needs.data());
    if (rc != MPI_SUCCESS) return rc;
    bool any_window = false;
    for (uint8_t v : needs) any_window = any_window || v;
    std::vector<char*> win;
    if (any_window) {
        rc = tp->window(2 * bytes, win);   // [0,bytes) input, [bytes,2*bytes) result
        if (rc != MPI_SUCCESS) return rc;
    }
    char* dev_in = need_stage_in ? win[me] : static_cast<char*>(bsrc.dev);
    char* dev_out = need_stage_out ? win[me] + bytes : static_cast<char*>(bdst.dev);
    if (in_place) dev_out = dev_in;
    if (need_stage_in) {
        hipError_t e = hipMemcpyAsync(dev_in, src, bytes, hipMemcpyDefault, s);
        if (e != hipSuccess) return hip_fail(e, "stage in");
        if ((rc = sync_stream(s, "stage in")) != MPI_SUCCESS) return rc;
    }

    // Exchange: every rank's input (this allgather is also the entry barrier).
    std::vector<char*> pin, pout;
    trace("allreduce: count=%zu esz=%zu algo=%d map inputs", count, esz, algo);
    if ((rc = tp->map_peers(dev_in, pin)) != MPI_SUCCESS) return rc;
    trace("allreduce: inputs mapped");

    const int n = newrank_of(me, p);
    if (algo == A_RECURSIVE_DOUBLING) {
        // Every rank evaluates its own lineage's tree over the whole vector
        // (folded even ranks receive their odd partner's result, :4071-4092).
        const int nn = n >= 0 ? n : newrank_of(me + 1, p);
        RankTree t = tree_allreduce(p, nn);
        char* out = (dev_out == dev_in) ? win[me] + bytes : dev_out;
        rc = run_rank_tree(op.opidx, k, t, pin, esz, 0, count, out, s);
        if (rc == MPI_SUCCESS) rc = sync_stream(s, "allreduce combine");
        if (rc == MPI_SUCCESS) rc = tp->barrier();   // everyone has read the inputs
        if (rc == MPI_SUCCESS && out != dev_out) {
            hipError_t e = hipMemcpyAsync(dev_out, out, bytes, hipMemcpyDeviceToDevice, s);
            if (e != hipSuccess) return hip_fail(e, "allreduce result copy");
        }
    } else {
        // Rabenseifner: newrank n owns block bitrev(n); evaluate it in place,
        // then pull every other block from its owner.
        if ((rc = tp->map_peers(dev_out, pout)) != MPI_SUCCESS) return rc;
        trace("allreduce: outputs mapped");
        const int pof2 = pof2_floor(p);
        if (n >= 0) {
            const int j = allreduce_block_of_newrank(p, n);
            size_t st, ln;
            allreduce_block(p, count, j, &st, &ln);
            RankTree t = tree_allreduce(p, n);
            rc = run_rank_tree(op.opidx, k, t, pin, esz, st, ln, dev_out + st * esz, s);
            trace("allreduce: block %d launched (%zu elems)", j, ln);
            if (rc == MPI_SUCCESS) rc = sync_stream(s, "allreduce reduce-scatter");
            trace("allreduce: block done rc=%d", rc);
        }
        if (rc == MPI_SUCCESS) rc = tp->barrier();   // every block reduced
        trace("allreduce: barrier 2 rc=%d", rc);
        if (rc != MPI_SUCCESS) return rc;
        std::vector<const void*> srcs;
        std::vector<void*> dsts;
        std::vector<size_t> nbs;
        for (int j = 0; j < pof2; ++j) {
            const int owner = real_of_newrank(allreduce_block_owner(p, j), p);
            if (owner == me) continue;
            size_t st, ln;
            allreduce_block(p, count, j, &st, &ln);
            srcs.push_back(pout[owner] + st * esz);
            dsts.push_back(dev_out + st * esz);
            nbs.push_back(ln * esz);
        }
        hipError_t e = launch_copy_segs(srcs.data(), dsts.data(), nbs.data(), (int)srcs.size(), true, s);
        if (e != hipSuccess) return hip_fail(e, "allreduce allgather");
    }
    trace("allreduce: gather launched");
    if (rc == MPI_SUCCESS) rc = sync_stream(s, "allreduce");
    trace("allreduce: gather done rc=%d", rc);
    if (rc == MPI_SUCCESS) rc = tp->barrier();   // nobody reads our buffers any more
    if (rc == MPI_SUCCESS && need_stage_out) {
        hipError_t e = hipMemcpyAsync(recvbuf, dev_out, bytes, hipMemcpyDefault, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return hip_fail(e, "stage out");
    }
    return rc;
}

int do_reduce_scatter(Comm* c, const void* sendbuf, void* recvbuf, const int* recvcounts,
                      MPI_Datatype dt, const OpRef& op)
{
    int rc = ensure_device();
    if (rc != MPI_SUCCESS) return rc;
    Transport* tp = c->tp;
    const int p = c->size, me = c->rank;
    const int esz_i = type_size(dt);
    const size_t esz = (size_t)esz_i;
    std::vector<size_t> disp((size_t)p + 1, 0);
    for (int r = 0; r < p; ++r) disp[r + 1] = disp[r] + (size_t)recvcounts[r];
    const size_t total = disp[p];
    if (total == 0) return MPI_SUCCESS;
    const size_t bytes = total * esz;
    const bool in_place = (sendbuf == MPI_IN_PLACE);
    const void* src = in_place ? recvbuf : sendbuf;

    if (op.opidx == O_NULL) {
        // user op: full allreduce on host, keep our block.
        std::vector<char> full(bytes);
        rc = copy_any(full.data(), src, bytes);
        if (rc == MPI_SUCCESS) rc = host_user_allreduce(c, full.data(), full.data() + 0, total, dt, op);
        if (rc == MPI_SUCCESS && recvcounts[me])
            rc = copy_any(recvbuf, full.data() + disp[me] * esz, (size_t)recvcounts[me] * esz);
        return rc;
    }

    const Kind k = type_info(dt)->kind;
    hipStream_t s = tp->stream();
    const BufInfo bsrc = classify(src), bdst = classify(recvbuf);
    const bool mine_stage_in = bsrc.place != Place::Device;
    const bool mine_stage_out = recvcounts[me] > 0 && bdst.place != Place::Device;
    // In place, our own block's result overwrites input that others read, so
    // it is produced into the window and copied after the closing barrier.
    const bool mine_temp = in_place && recvcounts[me] > 0;
    uint8_t need = (uint8_t)(mine_stage_in || mine_stage_out || mine_temp);
    std::vector<uint8_t> needs((size_t)p);
    if ((rc = tp->allgather(&need, 1, needs.data())) != MPI_SUCCESS) return rc;
    bool any = false;
    for (uint8_t v : needs) any = any || v;
    std::vector<char*> win;
    if (any && (rc = tp->window(2 * bytes, win)) != MPI_SUCCESS) return rc;

    char* dev_in = mine_stage_in ? win[me] : static_cast<char*>(bsrc.dev);
    if (mine_stage_in) {
        hipError_t e = hipMemcpyAsync(dev_in, src, bytes, hipMemcpyDefault, s);
        if (e != hipSuccess) return hip_fail(e, "stage in");
        if ((rc = sync_stream(s, "stage in")) != MPI_SUCCESS) return rc;
    }
    std::vector<char*> pin;
    if ((rc = tp->map_peers(dev_in, pin)) != MPI_SUCCESS) return rc;

    const int algo = reduce_scatter_algo(p, total, esz_i, op.commutative);
    const size_t mycnt = (size_t)recvcounts[me];
    char* out = nullptr;
    if (mycnt) {
        out = (mine_stage_out || mine_temp) ? win[me] + bytes : static_cast<char*>(bdst.dev);
        RankTree t = (algo == A_RS_PAIRWISE) ? tree_pairwise(p, me)
                                             : tree_reduce_scatter(p, newrank_of(me, p) >= 0
                                                                          ? newrank_of(me, p)
                                                                          : newrank_of(me + 1, p));
        rc = run_rank_tree(op.opidx, k, t, pin, esz, disp[me], mycnt, out, s);
        if (rc == MPI_SUCCESS) rc = sync_stream(s, "reduce_scatter combine");
    }
    if (rc == MPI_SUCCESS) rc = tp->barrier();
    if (rc == MPI_SUCCESS && mycnt && out != static_cast<char*>(bdst.dev)) {
        hipError_t e = hipMemcpyAsync(recvbuf, out, mycnt * esz, hipMemcpyDefault, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return hip_fail(e, "reduce_scatter result copy");
    }
    return rc;
}

}  // namespace

// ---- public engine entry points --------------------------------------------
int engine_allreduce(Comm* c, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
                     const OpRef& op)
{
    return worker().submit([=] { return do_allreduce(c, sendbuf, recvbuf, count, dt, op); }).get();
}

int engine_reduce_scatter(Comm* c, const void* sendbuf, void* recvbuf, const int* recvcounts,
                          MPI_Datatype dt, const OpRef& op)
{
    std::vector<int> counts(recvcounts, recvcounts + c->size);
    return worker()
        .submit([=] { return do_reduce_scatter(c, sendbuf, recvbuf, counts.data(), dt, op); })
        .get();
}

int engine_reduce(Comm* c, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
                  const OpRef& op, int root)
{
    // Root receives the allreduce result (root-0 trees coincide with the
    // allreduce trees, reduce.cpp:226-299, 489-537); other ranks discard it.
    return worker()
        .submit([=]() -> int {
            const size_t bytes = count * (size_t)type_size(dt);
            if (c->rank == root) return do_allreduce(c, sendbuf, recvbuf, count, dt, op);
            std::vector<char> scratch(bytes);
            const void* sb = sendbuf;
            return do_allreduce(c, sb, scratch.data(), count, dt, op);
        })
        .get();
}

int engine_scan(Comm* c, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
                const OpRef& op, bool exclusive)
{
    (void)c; (void)sendbuf; (void)recvbuf; (void)count; (void)dt; (void)op; (void)exclusive;
    set_error("MPI_Scan/MPI_Exscan on more than one rank is not implemented yet");
    return MPI_ERR_INTERN;
}

std::shared_future<int> engine_async(std::function<int()> fn) { return worker().submit(std::move(fn)); }

}  // namespace msx
