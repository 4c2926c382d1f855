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
#include <algorithm>
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

int reduce_algo(int p, size_t count, int type_size, bool builtin)
{
    // reduce.cpp:151: (unsigned)(count*type_size) > reduce_short_msg (64 KiB)
    const uint32_t nbytes = (uint32_t)((uint64_t)count * (uint64_t)type_size);
    return (nbytes > 65536u && builtin && count >= (size_t)pof2_floor(p)) ? A_RABENSEIFNER : A_BINOMIAL;
}

RankTree tree_reduce_rsag(int p, int n)
{
    // MPI_Reduce folds the ODD rank into the even one below it (reduce.cpp:
    // 136-165: Uop(tmp = x_{2n+1}, recvbuf = x_{2n})), newrank n -> real 2n.
    const int P = pof2_floor(p), rem = p - P;
    RankTree t;
    t.P = P;
    for (int i = 0; i < 32; ++i) t.src[i] = -1;
    for (int k = 0; k < P; ++k) {
        const int m = n ^ k;
        if (m < rem) {
            t.src[2 * k] = 2 * m;
            t.src[2 * k + 1] = 2 * m + 1;
            t.pairmask |= 1u << k;
        } else {
            t.src[2 * k] = m + rem;
        }
    }
    return t;
}

RankTree tree_reduce_binomial(int p, int root)
{
    // relrank k receives from k|mask (reduce.cpp:489-537): a balanced tree over
    // relative ranks with the leaves >= p absent
    RankTree t;
    int P = 1;
    while (P < p) P *= 2;
    t.P = P;
    t.nleaves = p;
    for (int i = 0; i < 32; ++i) t.src[i] = -1;
    for (int k = 0; k < p; ++k) t.src[2 * k] = (k + root) % p;
    return t;
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

// Evaluate RankTree `t` over [start, start+len) elements of the per-rank
// source pointers `srcs` into `out`.
int run_rank_tree(int opidx, Kind k, const RankTree& t, const std::vector<char*>& srcs, size_t esz,
                  size_t start, size_t len, char* out, hipStream_t s)
{
    if (len == 0) return MPI_SUCCESS;
    TreeSpec spec;
    spec.P = t.P;
    spec.nleaves = t.nleaves;
    spec.pairmask = t.pairmask;
    spec.chain = t.chain;
    spec.sys = true;
    const int nslots = t.chain ? t.P : 2 * (t.nleaves ? t.nleaves : t.P);
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

// Engine-private device scratch (grows, never shrinks; engine worker only).
char* dev_scratch(size_t bytes)
{
    static char* p = nullptr;
    static size_t cap = 0;
    if (bytes > cap) {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        if (hipMalloc(reinterpret_cast<void**>(&p), bytes) != hipSuccess) return nullptr;
        cap = bytes;
    }
    return p;
}

// ---- window-staged collectives ---------------------------------------------
// Every rank owns one IPC-mapped device window of 4*C bytes: two slots, each an
// IN half (this rank's staged input chunk) and an OUT half (this rank's
// reduced part).  User buffers are never IPC-mapped (ROCm 7.2 hangs opening
// handles of allocations > 2 GiB, and user memory may be host memory), so a
// collective streams chunks of C bytes through the windows:
//   stage  : my chunk of input -> IN(me, s)            (HBM copy / H2D)
//   barrier A (every input chunk staged)
//   reduce : my part of the chunk, reading IN(r, s) of every rank over xGMI,
//            the reference's expression tree per element -> OUT(me, s)
//   barrier B (every part reduced)            [allreduce only]
//   gather : every rank's part OUT(r, s) -> my recvbuf  [allreduce only]
// Slot s alternates; a rank syncs its stream before the next barrier, so a
// slot is never rewritten while a peer still reads it.
size_t chunk_bytes()
{
    static size_t c = [] {
        size_t v = (size_t)256 << 20;
        if (const char* e = getenv("MSX_CHUNK_BYTES")) v = (size_t)atoll(e);
        if (v < ((size_t)1 << 16)) v = (size_t)1 << 16;
        if (v > ((size_t)480 << 20)) v = (size_t)480 << 20;   // window 4*C < 2 GiB
        return v & ~(size_t)4095;
    }();
    return c;
}

struct Windows {
    std::vector<char*> base;
    size_t C = 0;
    char* in(int r, int s) const { return base[(size_t)r] + (size_t)s * 2 * C; }
    char* out(int r, int s) const { return base[(size_t)r] + (size_t)s * 2 * C + C; }
};

int get_windows(Transport* tp, Windows* w)
{
    w->C = chunk_bytes();
    return tp->window(4 * w->C, w->base);
}

int copy_async(void* dst, const void* src, size_t bytes, hipStream_t s)
{
    if (!bytes) return MPI_SUCCESS;
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, s);
    return e == hipSuccess ? MPI_SUCCESS : hip_fail(e, "stage copy");
}

// root < 0: allreduce; root >= 0: only `root` gathers the result (MPI_Reduce).
int do_allreduce(Comm* c, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
                 const OpRef& op, int root = -1)
{
    // user functions are host code: no GPU needed on this path
    if (op.opidx == O_NULL) return host_user_allreduce(c, sendbuf, recvbuf, count, dt, op);
    int rc = ensure_device();
    if (rc != MPI_SUCCESS) return rc;

    Transport* tp = c->tp;
    const int p = c->size, me = c->rank;
    const TypeInfo* ti = type_info(dt);
    const Kind k = ti->kind;
    const size_t esz = (size_t)ti->size;
    hipStream_t s = tp->stream();
    const char* src = static_cast<const char*>(sendbuf == MPI_IN_PLACE ? recvbuf : sendbuf);
    char* dst = static_cast<char*>(recvbuf);
    const bool want = (root < 0 || root == me);          // this rank receives the result
    const bool is_reduce = root >= 0;
    const int algo = is_reduce ? reduce_algo(p, count, (int)esz, true)
                               : allreduce_algo(p, count, (int)esz, true);
    Windows w;
    if ((rc = get_windows(tp, &w)) != MPI_SUCCESS) return rc;
    // chunk = whole 16-byte vectors of whole elements
    size_t ce = w.C / esz;
    ce -= ce % (16 / (esz < 16 ? esz : 16) ? 16 / (esz < 16 ? esz : 16) : 1);
    const int pof2 = pof2_floor(p);
    const int n = newrank_of(me, p);
    const int lineage = n >= 0 ? n : newrank_of(me + 1, p);
    trace("allreduce: count=%zu esz=%zu algo=%d chunk=%zu elems", count, esz, algo, ce);

    std::vector<char*> ins((size_t)p), outs((size_t)p);
    int slot = 0;
    for (size_t o = 0; o < count && rc == MPI_SUCCESS; o += ce, slot ^= 1) {
        const size_t len = (count - o < ce) ? count - o : ce;
        for (int r = 0; r < p; ++r) { ins[r] = w.in(r, slot); outs[r] = w.out(r, slot); }
        if ((rc = copy_async(ins[me], src + o * esz, len * esz, s)) != MPI_SUCCESS) break;
        if ((rc = sync_stream(s, "allreduce stage")) != MPI_SUCCESS) break;
        if ((rc = tp->barrier()) != MPI_SUCCESS) break;                  // A
        if (algo == A_RECURSIVE_DOUBLING || algo == A_BINOMIAL) {
            // recursive doubling: every rank evaluates its own lineage's tree on
            // the whole chunk; binomial reduce: the root evaluates its tree
            RankTree t = (algo == A_BINOMIAL) ? tree_reduce_binomial(p, root) : tree_allreduce(p, lineage);
            if (want) rc = run_rank_tree(op.opidx, k, t, ins, esz, 0, len, outs[me], s);
            if (rc == MPI_SUCCESS && want) rc = copy_async(dst + o * esz, outs[me], len * esz, s);
            if (rc == MPI_SUCCESS) rc = sync_stream(s, "allreduce chunk");
            continue;
        }
        // Rabenseifner order: element e of the vector belongs to block j(e),
        // whose value the reference computes at newrank bitrev(j).  The chunk
        // is split evenly over all p ranks (work balance only); each piece is
        // evaluated with the tree of its block's owner.
        const size_t q = (len + p - 1) / p;
        const size_t qv = (q + 15) & ~(size_t)15;                        // 16-element granules
        const size_t plo = std::min(len, (size_t)me * qv), phi = std::min(len, plo + qv);
        for (size_t e0 = plo; e0 < phi && rc == MPI_SUCCESS;) {
            const size_t ge = o + e0;                                    // global element
            const size_t rs = count / (size_t)pof2;
            int j = rs ? (int)std::min((size_t)pof2 - 1, ge / rs) : pof2 - 1;
            size_t bs, bl;
            allreduce_block(p, count, j, &bs, &bl);
            const size_t e1 = std::min(phi, bs + bl - o);
            const int owner = allreduce_block_owner(p, j);
            RankTree t = is_reduce ? tree_reduce_rsag(p, owner) : tree_allreduce(p, owner);
            rc = run_rank_tree(op.opidx, k, t, ins, esz, e0, e1 - e0, outs[me] + e0 * esz, s);
            e0 = e1;
        }
        if (rc == MPI_SUCCESS) rc = sync_stream(s, "allreduce reduce");
        if (rc == MPI_SUCCESS) rc = tp->barrier();                       // B
        if (rc != MPI_SUCCESS) break;
        if (!want) continue;
        // gather every part (peer OUT windows over xGMI) into recvbuf
        const BufInfo bd = classify(dst);
        char* gdst = (bd.place == Place::Device) ? static_cast<char*>(bd.dev) + o * esz : ins[me];
        std::vector<const void*> gs;
        std::vector<void*> gd;
        std::vector<size_t> gn;
        for (int r = 0; r < p; ++r) {
            const size_t lo = std::min(len, (size_t)r * qv), hi = std::min(len, lo + qv);
            if (hi <= lo) continue;
            gs.push_back(outs[r] + lo * esz);
            gd.push_back(gdst + lo * esz);
            gn.push_back((hi - lo) * esz);
        }
        hipError_t e = launch_copy_segs(gs.data(), gd.data(), gn.data(), (int)gs.size(), true, s);
        if (e != hipSuccess) { rc = hip_fail(e, "allreduce gather"); break; }
        if (bd.place != Place::Device) rc = copy_async(dst + o * esz, gdst, len * esz, s);
        if (rc == MPI_SUCCESS) rc = sync_stream(s, "allreduce gather");
    }
    if (rc == MPI_SUCCESS) rc = tp->barrier();   // windows free for the next collective
    trace("allreduce: done rc=%d", rc);
    return rc;
}

int do_reduce_scatter(Comm* c, const void* sendbuf, void* recvbuf, const int* recvcounts,
                      MPI_Datatype dt, const OpRef& op)
{
    Transport* tp = c->tp;
    const int p = c->size, me = c->rank;
    const size_t esz = (size_t)type_size(dt);
    std::vector<size_t> disp((size_t)p + 1, 0);
    size_t maxcnt = 0;
    for (int r = 0; r < p; ++r) {
        disp[r + 1] = disp[r] + (size_t)recvcounts[r];
        maxcnt = std::max(maxcnt, (size_t)recvcounts[r]);
    }
    const size_t total = disp[p];
    if (total == 0) return MPI_SUCCESS;
    const bool in_place = (sendbuf == MPI_IN_PLACE);
    const char* src = static_cast<const char*>(in_place ? recvbuf : sendbuf);

    if (op.opidx == O_NULL) {
        // user op: full allreduce on host, keep our block
        std::vector<char> full(total * esz), res(total * esz);
        int rc = copy_any(full.data(), src, total * esz);
        if (rc == MPI_SUCCESS) rc = host_user_allreduce(c, full.data(), res.data(), total, dt, op);
        if (rc == MPI_SUCCESS && recvcounts[me])
            rc = copy_any(recvbuf, res.data() + disp[me] * esz, (size_t)recvcounts[me] * esz);
        return rc;
    }
    int rc = ensure_device();
    if (rc != MPI_SUCCESS) return rc;
    const Kind k = type_info(dt)->kind;
    hipStream_t s = tp->stream();
    Windows w;
    if ((rc = get_windows(tp, &w)) != MPI_SUCCESS) return rc;
    // IN slot holds p sub-chunks of `ce` elements, one per destination rank
    size_t ce = w.C / esz / (size_t)p;
    ce -= ce % 16;
    if (ce == 0) ce = 1;
    const int algo = reduce_scatter_algo(p, total, (int)esz, op.commutative);
    const int n = newrank_of(me, p);
    RankTree t = (algo == A_RS_PAIRWISE) ? tree_pairwise(p, me)
                                         : tree_reduce_scatter(p, n >= 0 ? n : newrank_of(me + 1, p));
    trace("reduce_scatter: total=%zu esz=%zu algo=%d chunk=%zu", total, esz, algo, ce);
    const size_t mycnt = (size_t)recvcounts[me];
    const BufInfo bd = classify(recvbuf);
    char* dst = static_cast<char*>(recvbuf);
    std::vector<char*> ins((size_t)p);
    char* hold = nullptr;
    if (in_place && mycnt) {
        hold = dev_scratch(mycnt * esz);
        if (!hold) { set_error("reduce_scatter: scratch allocation failed"); return MPI_ERR_NO_MEM; }
    }
    int slot = 0;
    for (size_t o = 0; o < maxcnt && rc == MPI_SUCCESS; o += ce, slot ^= 1) {
        // stage, for every destination r, our contribution to r's block range [o, o+ce)
        char* mine = w.in(me, slot);
        for (int r = 0; r < p && rc == MPI_SUCCESS; ++r) {
            const size_t cnt = (size_t)recvcounts[r];
            if (o >= cnt) continue;
            const size_t len = std::min(ce, cnt - o);
            rc = copy_async(mine + (size_t)r * ce * esz, src + (disp[r] + o) * esz, len * esz, s);
        }
        if (rc == MPI_SUCCESS) rc = sync_stream(s, "reduce_scatter stage");
        if (rc == MPI_SUCCESS) rc = tp->barrier();
        if (rc != MPI_SUCCESS) break;
        if (o < mycnt) {
            const size_t len = std::min(ce, mycnt - o);
            for (int r = 0; r < p; ++r) ins[r] = w.in(r, slot) + (size_t)me * ce * esz;
            // In place, recvbuf is still our input for later chunks: results go
            // to a private device scratch and are copied out at the end.
            char* out = in_place ? hold + o * esz
                                 : (bd.place == Place::Device ? static_cast<char*>(bd.dev) + o * esz
                                                              : w.out(me, slot));
            rc = run_rank_tree(op.opidx, k, t, ins, esz, 0, len, out, s);
            if (rc == MPI_SUCCESS && out == w.out(me, slot))
                rc = copy_async(dst + o * esz, out, len * esz, s);
        }
        if (rc == MPI_SUCCESS) rc = sync_stream(s, "reduce_scatter reduce");
    }
    if (rc == MPI_SUCCESS) rc = tp->barrier();   // every rank finished reading the windows
    if (rc == MPI_SUCCESS && in_place && mycnt) {
        rc = copy_async(recvbuf, hold, mycnt * esz, s);
        if (rc == MPI_SUCCESS) rc = sync_stream(s, "reduce_scatter result");
    }
    trace("reduce_scatter: done rc=%d", rc);
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
    // The root receives the allreduce expression tree (identical to the
    // reference's Rabenseifner / binomial reduce for root 0, reduce.cpp:226-299,
    // 489-537); other ranks only contribute.  User ops: host allreduce.
    return worker()
        .submit([=]() -> int {
            if (op.opidx == O_NULL) {
                const size_t bytes = count * (size_t)type_size(dt);
                std::vector<char> tmp(bytes);
                int rc = host_user_allreduce(c, sendbuf, c->rank == root ? recvbuf : tmp.data(), count, dt, op);
                return rc;
            }
            return do_allreduce(c, sendbuf, recvbuf, count, dt, op, root);
        })
        .get();
}

namespace {

// MPI_Scan / MPI_Exscan: the reference builds a recursive-doubling task list
// (IscanBuildTaskList reduce.cpp:5285-5576, IexscanBuildTaskList :5671-5960,
// NbcTask::ExecuteScan tasks.cpp:694-766).  At step mask, rank r exchanges its
// partial result with dst = r ^ mask; if r > dst it folds the received value
// into both its partial and its result (Uop(tmp, partial), Uop(tmp, recvbuf);
// the first such step of Exscan copies tmp into recvbuf), else only into its
// partial.  The schedule is run step by step here, the exchange going through
// the IPC windows, so every combine has the reference's operands and roles.
int host_user_scan(Comm* c, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
                   const OpRef& op, bool exclusive)
{
    const int p = c->size, me = c->rank, esz = type_size(dt);
    const size_t bytes = count * (size_t)esz;
    std::vector<char> mine(bytes), all((size_t)p * bytes);
    int rc = copy_any(mine.data(), sendbuf == MPI_IN_PLACE ? recvbuf : sendbuf, bytes);
    if (rc == MPI_SUCCESS) rc = c->tp->allgather(mine.data(), bytes, all.data());
    if (rc != MPI_SUCCESS) return rc;
    auto call = [&](const char* in, char* io) {
        for (size_t off = 0; off < count;) {
            size_t n = std::min(count - off, (size_t)0x7fffffff);
            int len = (int)n;
            MPI_Datatype d = dt;
            op.user_fn(const_cast<char*>(in) + off * esz, io + off * esz, &len, &d);
            off += n;
        }
    };
    std::vector<std::vector<char>> part((size_t)p), res((size_t)p);
    std::vector<bool> have((size_t)p, !exclusive);
    for (int r = 0; r < p; ++r) {
        part[r].assign(all.begin() + (size_t)r * bytes, all.begin() + (size_t)(r + 1) * bytes);
        res[r] = part[r];
    }
    for (int mask = 1; mask < p; mask <<= 1) {
        std::vector<std::vector<char>> snap = part;
        const bool last = (mask << 1) >= p;
        for (int r = 0; r < p; ++r) {
            const int dst = r ^ mask;
            if (dst >= p || (last && r < dst)) continue;
            std::vector<char> tmp = snap[dst];
            if (r > dst) {
                call(tmp.data(), part[r].data());
                if (exclusive && !have[r]) { res[r] = tmp; have[r] = true; }
                else call(tmp.data(), res[r].data());
            } else if (op.commutative) {
                call(tmp.data(), part[r].data());
            } else {
                call(part[r].data(), tmp.data());
                part[r] = tmp;
            }
        }
    }
    if (exclusive && !have[me]) return MPI_SUCCESS;     // rank 0: recvbuf undefined
    return copy_any(recvbuf, res[me].data(), bytes);
}

int combine2(int opidx, Kind k, const char* inout_src, const char* in, char* out, size_t n, hipStream_t s)
{
    TreeSpec t;
    t.P = 2;
    t.src[0] = inout_src;
    t.src[2] = in;
    t.sys = true;
    hipError_t e = launch_tree_spec(opidx, k, t, out, n, s);
    return e == hipSuccess ? MPI_SUCCESS : hip_fail(e, "scan combine");
}

int do_scan(Comm* c, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
            const OpRef& op, bool exclusive)
{
    if (op.opidx == O_NULL) return host_user_scan(c, sendbuf, recvbuf, count, dt, op, exclusive);
    int rc = ensure_device();
    if (rc != MPI_SUCCESS) return rc;
    Transport* tp = c->tp;
    const int p = c->size, me = c->rank;
    const Kind k = type_info(dt)->kind;
    const size_t esz = (size_t)type_info(dt)->size, bytes = count * esz;
    hipStream_t s = tp->stream();
    const char* src = static_cast<const char*>(sendbuf == MPI_IN_PLACE ? recvbuf : sendbuf);
    Windows w;
    if ((rc = get_windows(tp, &w)) != MPI_SUCCESS) return rc;
    size_t ce = w.C / esz;
    ce -= ce % 16;
    char* partial = dev_scratch(2 * bytes + 256);
    if (!partial) { set_error("scan: scratch allocation failed"); return MPI_ERR_NO_MEM; }
    char* res = partial + ((bytes + 255) & ~(size_t)255);
    rc = copy_async(partial, src, bytes, s);
    if (rc == MPI_SUCCESS && !exclusive) rc = copy_async(res, src, bytes, s);
    if (rc == MPI_SUCCESS) rc = sync_stream(s, "scan init");
    bool have = !exclusive;
    int slot = 0;
    for (int mask = 1; mask < p && rc == MPI_SUCCESS; mask <<= 1) {
        const int dst = me ^ mask;
        const bool last = (mask << 1) >= p;
        const bool use = dst < p && !(last && me < dst);     // this rank consumes dst's partial
        for (size_t o = 0; o < count && rc == MPI_SUCCESS; o += ce, slot ^= 1) {
            const size_t len = std::min(ce, count - o);
            char* stage = w.in(me, slot);
            rc = copy_async(stage, partial + o * esz, len * esz, s);       // partial at step start
            if (rc == MPI_SUCCESS) rc = sync_stream(s, "scan stage");
            if (rc == MPI_SUCCESS) rc = tp->barrier();
            if (rc != MPI_SUCCESS || !use) continue;
            const char* tmp = w.in(dst, slot);
            char* pp = partial + o * esz;
            char* rr = res + o * esz;
            if (me > dst) {
                rc = combine2(op.opidx, k, pp, tmp, pp, len, s);
                if (rc == MPI_SUCCESS)
                    rc = have ? combine2(op.opidx, k, rr, tmp, rr, len, s) : copy_async(rr, tmp, len * esz, s);
            } else {
                rc = combine2(op.opidx, k, pp, tmp, pp, len, s);             // builtins commute
            }
            if (rc == MPI_SUCCESS) rc = sync_stream(s, "scan step");
        }
        if (use && me > dst) have = true;
    }
    if (rc == MPI_SUCCESS) rc = tp->barrier();
    if (rc == MPI_SUCCESS && have) {
        rc = copy_async(recvbuf, res, bytes, s);
        if (rc == MPI_SUCCESS) rc = sync_stream(s, "scan result");
    }
    return rc;
}

}  // namespace

int engine_scan(Comm* c, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
                const OpRef& op, bool exclusive)
{
    return worker().submit([=] { return do_scan(c, sendbuf, recvbuf, count, dt, op, exclusive); }).get();
}

std::shared_future<int> engine_async(std::function<int()> fn) { return worker().submit(std::move(fn)); }

}  // namespace msx
