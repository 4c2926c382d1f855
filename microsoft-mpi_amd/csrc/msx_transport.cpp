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
#include <dlfcn.h>
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
#include <atomic>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sched.h>
#include <linux/futex.h>
#include <sys/syscall.h>
#include <thread>
#include <unistd.h>

#include <rccl/rccl.h>

#include "msx_dtype.h"
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

    // MPI_COMM_WORLD: the hub address from the launcher's environment
    int init(int rank, int size)
    {
        const char* addr = getenv("MSX_BOOTSTRAP_ADDR");
        if (!addr) addr = getenv("MASTER_ADDR");
        if (!addr) addr = "127.0.0.1";
        int port = 29571;
        if (const char* v = getenv("MSX_BOOTSTRAP_PORT")) port = atoi(v);
        else if (const char* v = getenv("MASTER_PORT")) port = (atoi(v) + 97) % 65536;
        if (port < 1024) port += 1024;
        return init_at(rank, size, addr, port, -1);
    }

    // A derived communicator: its rank 0 already listens on `lfd` (bound to
    // an ephemeral port published through the parent); the others connect.
    int init_at(int rank, int size, const char* addr, int port, int lfd)
    {
        rank_ = rank;
        size_ = size;
        timeout_ = 600.0;
        if (const char* t = getenv("MSX_BOOTSTRAP_TIMEOUT")) timeout_ = atof(t);

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
            int one = 1;
            if (lfd >= 0) {
                lfd_ = lfd;
            } else {
                lfd_ = socket(AF_INET, SOCK_STREAM, 0);
                setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
                struct sockaddr_in any = sa;
                if (bind(lfd_, (struct sockaddr*)&any, sizeof(any)) != 0) {
                    set_error("bootstrap: bind %s:%d: %s", addr, port, strerror(errno));
                    return MPI_ERR_OTHER;
                }
                listen(lfd_, size + 8);
            }
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
        auto fail = [&](int peer, const char* phase) {
            const std::string why = last_error();
            set_error("wait timeout: op=hub_allgather rank=%d phase=%s peer=%d limit_s=%.1f (%s)", rank_, phase, peer,
                      timeout_, why.c_str());
            return MPI_ERR_OTHER;
        };
        if (rank_ == 0) {
            memcpy(out, mine, n);
            for (int r = 1; r < size_; ++r)
                if (io_all(fd_[r], out + (size_t)r * n, n, false, timeout_) != MPI_SUCCESS) return fail(r, "gather");
            for (int r = 1; r < size_; ++r)
                if (io_all(fd_[r], out, (size_t)size_ * n, true, timeout_) != MPI_SUCCESS) return fail(r, "scatter");
            return MPI_SUCCESS;
        }
        if (io_all(fd_[0], const_cast<void*>(mine), n, true, timeout_) != MPI_SUCCESS) return fail(0, "send");
        if (io_all(fd_[0], out, (size_t)size_ * n, false, timeout_) != MPI_SUCCESS) return fail(0, "receive");
        return MPI_SUCCESS;
    }

private:
    int rank_ = 0, size_ = 1, lfd_ = -1;
    double timeout_ = 600.0;
    std::vector<int> fd_;
    std::mutex mu_;
};

// ===========================================================================
// node-local barrier in POSIX shared memory (all ranks of a communicator are
// on one node: the IPC engine requires it).  Sense-reversing counter: a few
// microseconds instead of a TCP round trip through the hub.
// ===========================================================================
constexpr int kDoneSlots = 480;
struct ShmBar {
    std::atomic<uint32_t> count;
    std::atomic<uint32_t> gen;
    // per rank: sequence number of the last barrier-free call it has finished
    // (its tree has read its IN half), see do_allreduce
    std::atomic<uint64_t> done[kDoneSlots];
    // per rank: 1 + the generation of the barrier it last entered (timeouts
    // name the ranks that never arrived)
    std::atomic<uint32_t> at[kDoneSlots];
};
constexpr size_t kShmBarBytes = 8192;
static_assert(sizeof(ShmBar) <= kShmBarBytes, "two pages");

class ShmBarrier {
public:
    ~ShmBarrier()
    {
        if (bar_) munmap(bar_, kShmBarBytes);
    }

    // Collective over the hub.  Returns false (and stays unused) when shared
    // memory is unavailable; the caller then keeps the hub barrier.
    bool init(Hub& hub, int rank, int size, double timeout_s)
    {
        size_ = size;
        rank_ = rank;
        timeout_ = timeout_s;
        char name[64] = {0};
        int fd = -1;
        if (rank == 0) {
            // created and sized before anyone learns the name
            snprintf(name, sizeof(name), "/msx_bar_%d_%ld", (int)getpid(), (long)(now_s() * 1e6));
            fd = shm_open(name, O_CREAT | O_RDWR, 0600);
            if (fd < 0 || ftruncate(fd, kShmBarBytes) != 0) name[0] = 0;
        }
        std::vector<char> all((size_t)size * sizeof(name));
        if (hub.allgather(name, sizeof(name), all.data()) != MPI_SUCCESS) {
            if (fd >= 0) close(fd);
            return false;
        }
        memcpy(name, all.data(), sizeof(name));
        int ok = name[0] != 0;
        if (ok && rank != 0) fd = shm_open(name, O_RDWR, 0600);
        std::vector<int> oks((size_t)size);
        void* m = MAP_FAILED;
        if (ok && fd >= 0) m = mmap(nullptr, kShmBarBytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        if (fd >= 0) close(fd);
        int mine = (m != MAP_FAILED) ? 1 : 0;
        if (hub.allgather(&mine, sizeof(int), oks.data()) != MPI_SUCCESS) mine = 0;
        bool all_ok = mine != 0;
        for (int v : oks) all_ok = all_ok && v;
        if (rank == 0) shm_unlink(name);
        if (!all_ok) {
            if (m != MAP_FAILED) munmap(m, kShmBarBytes);
            trace("shm barrier unavailable; hub barrier in use");
            return false;
        }
        bar_ = static_cast<ShmBar*>(m);    // zero-filled by ftruncate
        return true;
    }

    bool ready() const { return bar_ != nullptr; }
    bool has_done() const { return bar_ && size_ <= kDoneSlots; }
    void post_done(int rank, uint64_t v) { bar_->done[rank].store(v, std::memory_order_release); }
    int wait_done(int rank, uint64_t v)
    {
        const double t_end = now_s() + timeout_;
        for (int spin = 0; bar_->done[rank].load(std::memory_order_acquire) < v; ++spin) {
            if (now_s() > t_end) {
                set_error("wait timeout: op=flag_call rank=%d phase=previous_call_done peer=%d seq=%llu limit_s=%.1f",
                          rank_, rank, (unsigned long long)v, timeout_);
                return MPI_ERR_OTHER;
            }
            if (spin > 2000) sched_yield();
        }
        return MPI_SUCCESS;
    }

    int wait()
    {
        const uint32_t g = bar_->gen.load(std::memory_order_acquire);
        if (size_ <= kDoneSlots) bar_->at[rank_].store(g + 1, std::memory_order_relaxed);
        if (bar_->count.fetch_add(1, std::memory_order_acq_rel) + 1 == (uint32_t)size_) {
            bar_->count.store(0, std::memory_order_relaxed);
            bar_->gen.store(g + 1, std::memory_order_release);
            syscall(SYS_futex, reinterpret_cast<uint32_t*>(&bar_->gen), FUTEX_WAKE, INT32_MAX, nullptr, nullptr, 0);
            return MPI_SUCCESS;
        }
        // short spin (the common case when ranks arrive together), then sleep
        // in the kernel on the generation word
        for (int it = 0; it < 4000; ++it)
            if (bar_->gen.load(std::memory_order_acquire) != g) return MPI_SUCCESS;
        const double t_end = now_s() + timeout_;
        while (bar_->gen.load(std::memory_order_acquire) == g) {
            if (now_s() > t_end) {
                // the first rank that has not entered this barrier
                int missing = -1;
                for (int r = 0; r < size_ && r < kDoneSlots && missing < 0; ++r)
                    if (bar_->at[r].load(std::memory_order_relaxed) != g + 1) missing = r;
                set_error("wait timeout: op=barrier rank=%d phase=host_barrier peer=%d seq=%u limit_s=%.1f", rank_,
                          missing, g, timeout_);
                return MPI_ERR_OTHER;
            }
            struct timespec ts = {0, 100 * 1000 * 1000};
            syscall(SYS_futex, reinterpret_cast<uint32_t*>(&bar_->gen), FUTEX_WAIT, g, &ts, nullptr, 0);
        }
        return MPI_SUCCESS;
    }

private:
    ShmBar* bar_ = nullptr;
    int size_ = 1;
    int rank_ = 0;
    double timeout_ = 600.0;
};

// ===========================================================================
// Uncached device memory: taken from the driver, never given back
// ===========================================================================
// Engine windows and RMA staging areas are uncached device memory
// (hipDeviceMallocUncached) that the peers map over IPC.  hipFree of such
// memory leaves this ROCm stack returning wrong data to later allocations'
// kernels and copies in the same process: after uncached buffers were used and
// freed, torch.equal(a, a.clone()) on fresh tensors failed in 4-30 of 96 cases
// per variant and a kernel write + copy check of a fresh plain buffer in 3 of
// 32; with the uncached buffers kept, 0 of 192 and 0 of 32; plain buffers or
// page-locked host memory freed the same way, 0 (scripts/va_reuse_probe.py,
// profiles/r06/va_reuse/).  So a freed communicator's window returns to this
// pool and serves the next window of the process (best fit), and imported peer
// windows stay mapped (ipc_imports); creating and freeing communicators then
// also costs no further 2 GiB allocations.
struct UcPool {
    struct Block {
        void* p;
        size_t cap;
        bool used;
    };
    std::mutex mu;
    std::vector<Block> blocks;
};

UcPool& uc_pool()
{
    static UcPool* pool = new UcPool();   // outlives static destruction: nothing is freed at exit either
    return *pool;
}

// `bytes` of zeroed uncached device memory on the current device.
hipError_t uc_alloc(size_t bytes, void** out)
{
    UcPool& pool = uc_pool();
    std::lock_guard<std::mutex> g(pool.mu);
    int dev = 0;
    (void)hipGetDevice(&dev);
    UcPool::Block* best = nullptr;
    for (auto& b : pool.blocks) {
        hipPointerAttribute_t a;
        if (b.used || b.cap < bytes || (best && b.cap >= best->cap)) continue;
        if (hipPointerGetAttributes(&a, b.p) != hipSuccess || a.device != dev) {
            (void)hipGetLastError();
            continue;
        }
        best = &b;
    }
    void* p = nullptr;
    if (best) {
        p = best->p;
    } else {
        hipError_t e = hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached);
        if (e != hipSuccess) return e;
        pool.blocks.push_back({p, bytes, false});
        best = &pool.blocks.back();
    }
    hipError_t e = hipMemset(p, 0, bytes);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) return e;
    best->used = true;
    *out = p;
    return hipSuccess;
}

void uc_release(void* p)
{
    if (!p) return;
    UcPool& pool = uc_pool();
    std::lock_guard<std::mutex> g(pool.mu);
    for (auto& b : pool.blocks)
        if (b.p == p) b.used = false;
}

// Peer windows imported over IPC, by handle, for the life of the process (an
// imported window is uncached memory too; closing the mapping is the same
// release as a free).  The exporter never frees a window (uc_pool), so a
// handle keeps naming the same memory.
struct IpcImports {
    std::mutex mu;
    std::map<std::string, void*> opened;
};

IpcImports& ipc_imports()
{
    static IpcImports* m = new IpcImports();
    return *m;
}

// ===========================================================================
// IPC transport
// ===========================================================================
struct IpcRec {
    hipIpcMemHandle_t h;
    uint64_t offset;
    int32_t ok;
    int32_t pad;
};

size_t rma_bytes_for(int share);   // passive-target staging size for `share` ranks per GPU (below)

class IpcTransport : public Transport {
public:
    ~IpcTransport() override
    {
        uc_release(win_);    // windows go back to the pool, imports stay mapped (uc_pool)
        uc_release(rwin_);
        if (counter_) (void)hipFree(counter_);
        if (stream_) (void)hipStreamDestroy(stream_);
    }

    int init(int r, int s, int port = 0, int lfd = -1)
    {
        rank = r;
        size = s;
        int rc = port ? hub_.init_at(r, s, "127.0.0.1", port, lfd) : hub_.init(r, s);
        if (rc != MPI_SUCCESS) return rc;
        double t = 600.0;
        if (const char* v = getenv("MSX_BOOTSTRAP_TIMEOUT")) t = atof(v);
        (void)shm_.init(hub_, r, s, t);   // without it: the hub's barriers, no GPU-flag schedules
        // ranks that share a GPU (an unknown bus id shares nothing)
        char bus[32] = {0};
        int dev = -1;
        if (device_count_noinit() <= 0 || hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetPCIBusId(bus, sizeof(bus), dev) != hipSuccess) {
            (void)hipGetLastError();
            bus[0] = 0;
        }
        std::vector<char> buses((size_t)s * sizeof(bus));
        if ((rc = hub_.allgather(bus, sizeof(bus), buses.data())) != MPI_SUCCESS) return rc;
        for (int a = 0; a < s && !gpu_shared; ++a)
            for (int b = 0; b < a && !gpu_shared; ++b)
                gpu_shared = buses[(size_t)a * sizeof(bus)] != 0 &&
                             strncmp(buses.data() + (size_t)a * sizeof(bus), buses.data() + (size_t)b * sizeof(bus),
                                     sizeof(bus)) == 0;
        trace("transport: %d ranks, %s", s, gpu_shared ? "some share a GPU" : "one GPU each");
        return MPI_SUCCESS;
    }

    int allgather(const void* mine, size_t n, void* all) override { return hub_.allgather(mine, n, all); }

    bool has_done() const override { return shm_.has_done(); }
    void post_done(uint64_t v) override { shm_.post_done(rank, v); }
    int wait_done(int r, uint64_t v) override { return shm_.wait_done(r, v); }

    int barrier() override
    {
        if (shm_.ready()) return shm_.wait();
        char b = 0;
        std::vector<char> all((size_t)size);
        return hub_.allgather(&b, 1, all.data());
    }

    hipStream_t stream() override
    {
        if (!stream_) (void)hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking);
        return stream_;
    }

    unsigned* push_counter() override
    {
        if (!counter_) {
            // kCountBlocks blocks of kCountWords (msx_kernels.h)
            void* c = nullptr;
            const size_t bytes = (size_t)kCountBlocks * kCountWords * sizeof(unsigned);
            if (hipMalloc(&c, bytes) != hipSuccess) return nullptr;
            if (hipMemset(c, 0, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
                (void)hipFree(c);
                return nullptr;
            }
            counter_ = static_cast<unsigned*>(c);
        }
        return counter_;
    }

    int map_peers(const void* ptr, std::vector<char*>& out) override
    {
        IpcRec mine;
        memset(&mine, 0, sizeof(mine));
        void* base = nullptr;
        size_t asz = 0;
        hipError_t e = hipMemGetAddressRange(&base, &asz, const_cast<void*>(ptr));
        trace("map_peers: ptr=%p base=%p size=%zu rc=%d", ptr, base, asz, (int)e);
        if (e == hipSuccess) {
            PhaseScope ph("ipc_get_handle");
            e = hipIpcGetMemHandle(&mine.h, base);
        }
        trace("map_peers: handle rc=%d", (int)e);
        if (e == hipSuccess) {
            mine.ok = 1;
            mine.offset = (uint64_t)((const char*)ptr - (const char*)base);
        } else {
            (void)hipGetLastError();
            set_error("rank %d: buffer %p cannot be shared over IPC (%s)", rank, ptr, hipGetErrorString(e));
        }
        std::vector<IpcRec> all((size_t)size);
        int rc;
        {
            PhaseScope ph("ipc_handle_exchange");
            rc = hub_.allgather(&mine, sizeof(mine), all.data());
        }
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
            IpcImports& imp = ipc_imports();
            std::lock_guard<std::mutex> g(imp.mu);
            auto it = imp.opened.find(key);
            void* pbase = nullptr;
            if (it != imp.opened.end()) {
                pbase = it->second;
            } else {
                {
                    PhaseScope ph("ipc_open", r);
                    e = hipIpcOpenMemHandle(&pbase, all[r].h, hipIpcMemLazyEnablePeerAccess);
                }
                trace("map_peers: opened rank %d handle -> %p rc=%d", r, pbase, (int)e);
                if (e != hipSuccess) {
                    hip_fail(e, "hipIpcOpenMemHandle");
                    set_error("ipc error: op=map_peers rank=%d phase=ipc_open peer=%d (%s)", rank, r, hipGetErrorString(e));
                    return MPI_ERR_OTHER;
                }
                imp.opened[key] = pbase;
            }
            out[r] = static_cast<char*>(pbase) + all[r].offset;
        }
        return MPI_SUCCESS;
    }

    int window(size_t bytes, std::vector<char*>& out) override
    {
        // Collective: every rank asks for the same size.
        if (bytes > win_bytes_) {
            uc_release(win_);
            win_ = nullptr;
            size_t want = bytes < ((size_t)1 << 20) ? ((size_t)1 << 20) : bytes;
            // Uncached device memory: peers write it over xGMI, which does not
            // snoop this GPU's L2, so no reader (kernel, blit or DMA) may hold a
            // stale line of it.  The kernel driver maps such a buffer MTYPE_UC
            // on the owner and on every peer that imports it, so neither the
            // writer's nor the reader's L2 ever holds a line of it, and the
            // engine's kernels need no per-workgroup system fences (each one
            // writes back or invalidates a whole XCD L2; rounds 1-2 had them and
            // they halved the collectives' throughput: p = 2 reduce_scatter
            // 4.17 -> 2.17 ms, allreduce 64 MiB 511 -> 178 us without).
            // zeroed (uc_alloc) before any peer can map it (map_peers below is
            // collective): the arrival flags behind the data areas start at 0
            hipError_t e = uc_alloc(want, &win_);
            trace("window: %zu bytes uncached rc=%d", want, (int)e);
            if (e != hipSuccess) {
                win_ = nullptr;
                return hip_fail(e, "window allocation");
            }
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

    int rma_window(std::vector<char*>& out, size_t* bytes_out) override
    {
        // Collective, first passive-target window of the communicator only:
        // uncached like the engine window (peers write payloads into it)
        if (!rwin_) {
            // ranks sharing this GPU, counted from every rank's PCI bus id
            // (not guessed from WORLD_SIZE / device count: a launcher may show
            // each rank only its own GPU), then the minimum size over ranks
            char bus[64] = {0};
            int dev = 0;
            if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetPCIBusId(bus, (int)sizeof(bus) - 1, dev) != hipSuccess) {
                (void)hipGetLastError();
                snprintf(bus, sizeof(bus), "unknown-%d", rank);
            }
            std::vector<char> buses((size_t)size * sizeof(bus));
            int rc = hub_.allgather(bus, sizeof(bus), buses.data());
            if (rc != MPI_SUCCESS) return rc;
            int share = 0;
            for (int r = 0; r < size; ++r)
                share += strncmp(buses.data() + (size_t)r * sizeof(bus), bus, sizeof(bus)) == 0;
            uint64_t mine = rma_bytes_for(share), lo = mine;
            std::vector<uint64_t> all((size_t)size);
            if ((rc = hub_.allgather(&mine, sizeof(mine), all.data())) != MPI_SUCCESS) return rc;
            for (uint64_t v : all) lo = std::min(lo, v);
            const size_t bytes = (size_t)lo;
            trace("rma window: %d rank(s) on this GPU, %zu bytes here, %zu agreed", share, (size_t)mine, bytes);
            hipError_t e = uc_alloc(bytes, &rwin_);
            trace("rma window: %zu bytes rc=%d", bytes, (int)e);
            if (e != hipSuccess) {
                rwin_ = nullptr;
                return hip_fail(e, "rma staging allocation");
            }
            rc = map_peers(rwin_, rwin_peers_);
            if (rc != MPI_SUCCESS) return rc;
            rbytes_ = bytes;
        }
        out = rwin_peers_;
        *bytes_out = rbytes_;
        return MPI_SUCCESS;
    }

private:
    Hub hub_;
    ShmBarrier shm_;
    hipStream_t stream_ = nullptr;
    unsigned* counter_ = nullptr;
    void* win_ = nullptr;
    size_t win_bytes_ = 0;
    std::vector<char*> win_peers_;
    void* rwin_ = nullptr;                // passive-target staging (rma_window)
    size_t rbytes_ = 0;                   // its agreed size
    std::vector<char*> rwin_peers_;
};

}  // namespace

// Listening socket on an ephemeral loopback port (a derived communicator's hub).
static int listen_ephemeral(int* port)
{
    int fd = socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) return -1;
    struct sockaddr_in sa = {};
    sa.sin_family = AF_INET;
    sa.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    sa.sin_port = 0;
    socklen_t len = sizeof(sa);
    if (bind(fd, (struct sockaddr*)&sa, sizeof(sa)) != 0 || listen(fd, 64) != 0 ||
        getsockname(fd, (struct sockaddr*)&sa, &len) != 0) {
        close(fd);
        return -1;
    }
    *port = ntohs(sa.sin_port);
    return fd;
}

int transport_split(Transport* parent, int color, int key, int* new_rank, int* new_size, Transport** out,
                    std::vector<int>* members_out)
{
    *out = nullptr;
    *new_rank = -1;
    *new_size = 0;
    const int p = parent->size;
    // MPIR_Comm_split: (color, key) of every rank; members of a color ordered
    // by (key, parent rank)
    int32_t mine[2] = {color, key};
    std::vector<int32_t> all((size_t)p * 2);
    int rc = parent->allgather(mine, sizeof(mine), all.data());
    if (rc != MPI_SUCCESS) return rc;
    std::vector<std::pair<std::pair<int, int>, int>> members;   // ((key, parent rank), parent rank)
    if (color != MPI_UNDEFINED)
        for (int r = 0; r < p; ++r)
            if (all[(size_t)r * 2] == color) members.push_back({{all[(size_t)r * 2 + 1], r}, r});
    std::sort(members.begin(), members.end());
    for (size_t i = 0; i < members.size(); ++i)
        if (members[i].second == parent->rank) *new_rank = (int)i;
    *new_size = (int)members.size();
    if (members_out) {
        members_out->clear();
        for (auto& m : members) members_out->push_back(m.second);
    }
    // the new rank 0 of every group of >= 2 opens the group's hub
    int32_t port = 0;
    int lfd = -1;
    if (*new_rank == 0 && *new_size > 1) {
        int pt = 0;
        lfd = listen_ephemeral(&pt);
        port = lfd >= 0 ? pt : -1;
    }
    std::vector<int32_t> ports((size_t)p);
    rc = parent->allgather(&port, sizeof(port), ports.data());
    if (rc != MPI_SUCCESS || *new_size <= 1) {
        if (lfd >= 0) close(lfd);
        return rc;
    }
    const int leader_port = ports[(size_t)members[0].second];
    if (leader_port <= 0) {
        if (lfd >= 0) close(lfd);
        set_error("communicator split: the group's bootstrap socket could not be opened");
        return MPI_ERR_OTHER;
    }
    auto* t = new IpcTransport();
    rc = t->init(*new_rank, *new_size, leader_port, lfd);
    if (rc != MPI_SUCCESS) {
        delete t;
        return rc;
    }
    *out = t;
    return MPI_SUCCESS;
}

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

namespace {
void rccl_forget(Transport* tp);   // the RCCL plane's per-transport state (below)
}  // namespace

void transport_destroy(Transport* t)
{
    if (!t) return;
    rccl_forget(t);
    if (t->aux) (void)hipStreamDestroy(t->aux);
    delete t;
}

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

// The flat communicators' algorithm switch points (Mpi.SwitchoverSettings
// [COLL_SWITCHOVER_FLAT], mpid/env.cpp:514-608): MPICH_DEFAULT_*_MSG override
// the coll.h defaults as env_to_int does (common/mpiutil.cpp:65-91): unset or
// longer than the 11-character buffer -> default, else _wtoi's value,
// clamped below at 0.  Read once; every rank must see the same environment,
// as with the reference.
namespace {
uint32_t env_switch(const char* name, int defval)
{
    const char* v = getenv(name);
    if (!v || strlen(v) > 11) return (uint32_t)defval;
    long long x = strtoll(v, nullptr, 10);           // _wtoi: leading blanks, sign, digits
    if (x > INT32_MAX) x = INT32_MAX;
    if (x < 0) x = 0;                                // minval 0
    return (uint32_t)x;
}
struct SwitchPoints {
    uint32_t allreduce_short = env_switch("MPICH_DEFAULT_ALLREDUCE_SHORT_MSG", 262144);
    uint32_t reduce_short = env_switch("MPICH_DEFAULT_REDUCE_SHORT_MSG", 65536);
    uint32_t redscat_long = env_switch("MPICH_DEFAULT_REDSCAT_COMMUTATIVE_LONG_MSG", 524288);
};
const SwitchPoints& switch_points()
{
    static const SwitchPoints sp;
    return sp;
}
}  // namespace

int allreduce_algo(int p, size_t count, int type_size, bool builtin)
{
    // reduce.cpp:3884-3888; count*type_size is evaluated in 32 bits.
    const uint32_t nbytes = (uint32_t)((uint64_t)count * (uint64_t)type_size);
    if (nbytes <= switch_points().allreduce_short || !builtin || count < (size_t)pof2_floor(p))
        return A_RECURSIVE_DOUBLING;
    return A_RABENSEIFNER;
}

int reduce_scatter_algo(int p, size_t total_count, int type_size, bool commutative)
{
    (void)p;
    if (!commutative) return -1;
    // reduce.cpp:1705-1709: nbytes = (unsigned)(total_count * type_size) wraps at 4 GiB.
    const uint32_t nbytes = (uint32_t)((uint64_t)total_count * (uint64_t)type_size);
    return nbytes < switch_points().redscat_long ? A_RS_HALVING : A_RS_PAIRWISE;
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
    // reduce.cpp:151: (unsigned)(count*type_size) > reduce_short_msg (64 KiB by default)
    const uint32_t nbytes = (uint32_t)((uint64_t)count * (uint64_t)type_size);
    return (nbytes > switch_points().reduce_short && builtin && count >= (size_t)pof2_floor(p)) ? A_RABENSEIFNER
                                                                                                : A_BINOMIAL;
}

int gate_type_size(MPI_Datatype dt, bool nbc)
{
    if (dtype_is_derived(dt)) {            // user ops only; the builtin gates never see one
        const Dtype* t = dtype_lookup(dt);
        return t ? (int)(nbc ? t->extent : t->size) : 0;
    }
    return nbc ? type_size(dt) : (int)dtype_size(dt);
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

RankTree tree_ireduce_rsag(int p, int n, int root)
{
    // IreduceBuildScatterGatherTaskList (reduce.cpp:6267-6670) runs the same
    // fold and recursive halving over ranks RELATIVE TO THE ROOT: peer =
    // RankAdd(TrimmedToOriginalRankEven(rem, s ^ offset), root) (:6471), the
    // even relative rank combining Uop(tmp = x_{rel+1}, recvbuf) (:6403-6411).
    RankTree t = tree_reduce_rsag(p, n);
    for (int i = 0; i < 32; ++i)
        if (t.src[i] >= 0) t.src[i] = (t.src[i] + root) % p;
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

    // A blocking call: run it on the calling thread when the worker is idle
    // (no queued or running task -- the collective order is then the issue
    // order anyway), which saves two thread hand-offs (~10-20 us) per call;
    // otherwise queue it behind the pending non-blocking operations.
    int run(std::function<int()> fn)
    {
        if (std::this_thread::get_id() == tid_) return fn();
        {
            std::unique_lock<std::mutex> g(mu_);
            if (!q_.empty() || busy_ || inline_) {
                g.unlock();
                // the error text is thread-local: carry it back to the caller
                auto text = std::make_shared<std::string>();
                const int rc = submit([fn = std::move(fn), text]() -> int {
                                   const int r = fn();
                                   if (r != MPI_SUCCESS) *text = last_error();
                                   return r;
                               }).get();
                if (rc != MPI_SUCCESS) set_error("%s", text->c_str());
                return rc;
            }
            inline_ = true;
        }
        const int rc = fn();
        {
            std::lock_guard<std::mutex> g(mu_);
            inline_ = false;
        }
        cv_.notify_all();
        return rc;
    }

private:
    void loop()
    {
        // a new thread starts on HIP device 0: bind it to this rank's GPU
        // before any task allocates (one rank per GPU on a multi-GPU node)
        (void)ensure_device();
        for (;;) {
            std::shared_ptr<std::packaged_task<int()>> t;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [this] { return stop_ || (!q_.empty() && !inline_); });
                if (q_.empty()) return;
                t = q_.front();
                q_.pop_front();
                busy_ = true;
            }
            (*t)();
            std::lock_guard<std::mutex> g(mu_);
            busy_ = false;
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::shared_ptr<std::packaged_task<int()>>> q_;
    std::thread th_;
    std::thread::id tid_;
    bool stop_ = false;
    bool busy_ = false;     // the worker is running a task
    bool inline_ = false;   // a blocking call runs on its caller's thread
};

Worker& worker()
{
    static Worker w;
    return w;
}

// A GPU flag wait ran out of time: the kernel stored tag * 65536 + 1 + r
// into the pinned word (r = the first flag index still missing; for the
// collectives' per-rank flags, the peer's rank).  One structured line, the
// text of msx_last_error(), which bench_collectives.py parses into its JSON.
int flag_timeout(const char* op, int me, int word, unsigned long long seq, bool index_is_rank = true)
{
    const int tag = word >> 16, idx = (word & 0xffff) - 1;
    const char* phase = tag == 2 ? "result" : (tag == 3 ? "half_free" : "arrival");
    set_error("flag timeout: op=%s rank=%d phase=%s peer=%d seq=%llu limit_s=%.1f", op, me, phase,
              index_is_rank ? idx : -1, seq, flag_wait_seconds());
    trace("%s", last_error());
    return MPI_ERR_OTHER;
}

// Fault injection for the timeout diagnostics (test hook):
// MSX_TEST_DROP_FLAGS=<rank>:<seq> -- that rank does not post its arrival
// flags of flag-synchronised call <seq>, so its peers' waits run out.
bool fault_drop_flags(int me, unsigned long long seq)
{
    static const std::pair<int, unsigned long long> f = [] {
        const char* e = getenv("MSX_TEST_DROP_FLAGS");
        int r = -1;
        unsigned long long q = 0;
        if (e && sscanf(e, "%d:%llu", &r, &q) != 2) r = -1;
        return std::make_pair(r, q);
    }();
    if (f.first != me || f.second != seq) return false;
    trace("fault injection: rank %d drops the arrival flags of call %llu", me, seq);
    return true;
}

int sync_stream(hipStream_t s, const char* what)
{
    PhaseScope ph(what, -1, true);
    hipError_t e = hipStreamSynchronize(s);
    return e == hipSuccess ? MPI_SUCCESS : hip_fail(e, what);
}

// Evaluate RankTree `t` over [start, start+len) elements of the per-rank
// source pointers `srcs` into `out`.
struct TreeWait {
    // result-ready flags after the last of `done_launches` launches
    // (TreeSpec::done_*); done_counter: block 2 of push_counter()
    unsigned* done_counter = nullptr;
    unsigned done_launches = 1;
    const std::vector<unsigned long long*>* done_flags = nullptr;
    unsigned long long done_seq = 0;
};

int run_rank_tree(int opidx, Kind k, const RankTree& t, const std::vector<char*>& srcs, size_t esz,
                  size_t start, size_t len, char* out, hipStream_t s,
                  const std::vector<char*>& extra_outs = {}, const TreeWait* wait = nullptr)
{
    if (len == 0) return MPI_SUCCESS;
    TreeSpec spec;
    if (wait) {
        if (wait->done_counter) {
            const size_t nf = wait->done_flags ? wait->done_flags->size() : 0;
            if (nf > 64) { set_error("result flags: too many peers"); return MPI_ERR_INTERN; }
            spec.done_counter = wait->done_counter;
            spec.done_launches = wait->done_launches;
            spec.done_nflags = (int)nf;
            for (size_t i = 0; i < nf; ++i) spec.done_flags[i] = (*wait->done_flags)[i];
            spec.done_seq = wait->done_seq;
        }
    }
    if (extra_outs.size() > 31) { set_error("tree combine: too many destinations"); return MPI_ERR_INTERN; }
    spec.nextra = (int)extra_outs.size();
    for (size_t e = 0; e < extra_outs.size(); ++e) spec.extra[e] = extra_outs[e];
    spec.P = t.P;
    spec.nleaves = t.nleaves;
    spec.pairmask = t.pairmask;
    spec.chain = t.chain;
    const int nslots = t.chain ? t.P : 2 * (t.nleaves ? t.nleaves : t.P);
    for (int i = 0; i < nslots; ++i)
        spec.src[i] = t.src[i] >= 0 ? srcs[(size_t)t.src[i]] + start * esz : nullptr;
    hipError_t e = launch_tree_spec(opidx, k, spec, out, len, s);
    return e == hipSuccess ? MPI_SUCCESS : hip_fail(e, "tree combine");
}

// ---- host path for user-defined ops --------------------------------------
// User functions are host code; every contribution is gathered to host memory
// as an IMAGE: the bytes `count` elements of `dt` span.  For a predefined type
// that is the packed array; for a derived datatype (which only user ops
// accept, the builtin check tables reject it) it is the typed byte span, so
// the user function sees the layout it was written for.  Pointers handed
// around below are TYPED BASES (image start - lo), like the user's buffers.
struct Img {
    int64_t lo = 0;            // image byte 0 = typed byte lo
    size_t bytes = 0;
    const Dtype* t = nullptr;  // derived type, or null (predefined)
    size_t esz = 0;            // predefined element size
};

Img img_of(MPI_Datatype dt, size_t count)
{
    Img m;
    if (dtype_is_derived(dt)) {
        m.t = dtype_lookup(dt);
        int64_t lo, hi;
        dt_span(m.t, (int64_t)count, &lo, &hi);
        m.lo = lo;
        m.bytes = (size_t)(hi - lo);
    } else {
        m.esz = (size_t)type_size(dt);
        m.bytes = count * m.esz;
    }
    return m;
}

// image <- buf (any memory)
int img_load(const Img& m, const void* buf, char* img)
{
    return copy_any(img, static_cast<const char*>(buf) + m.lo, m.bytes);
}

// buf <- image: a derived type writes only the bytes its type map covers
// (MPIR_Localcopy through the type, gaps of `buf` untouched): the mapped bytes
// are gathered on the host and the GPU unpack kernel scatters them.
int img_store(const Img& m, size_t count, const char* typed_base, void* buf)
{
    if (!m.t) return copy_any(buf, typed_base, m.bytes);
    if (count == 0 || m.t->size == 0) return MPI_SUCCESS;
    std::vector<char> packed((size_t)m.t->size * count);
    Dtype* t = const_cast<Dtype*>(m.t);
    size_t p = 0;
    auto run = [&](int64_t i, int64_t disp, int64_t len) {
        memcpy(packed.data() + p, typed_base + i * t->extent + disp, (size_t)len);
        p += (size_t)len;
    };
    for (size_t i = 0; i < count; ++i)
        dtype_for_each_run(t, [&](int64_t disp, int64_t len) { run((int64_t)i, disp, len); });
    return dt_unpack_any(t, (int64_t)count, packed.data(), buf);
}

// inout = in (op) inout over `count` elements, typed bases
void img_call(const OpRef& op, MPI_Datatype dt, const Img& m, size_t count, const char* in, char* io)
{
    MPI_Datatype d = dt;
    if (m.t) {
        int len = (int)count;      // API counts are int
        op.user_fn(const_cast<char*>(in), io, &len, &d);
        return;
    }
    for (size_t off = 0; off < count;) {
        size_t n = std::min(count - off, (size_t)0x7fffffff);
        int len = (int)n;
        op.user_fn(const_cast<char*>(in) + off * m.esz, io + off * m.esz, &len, &d);
        off += n;
    }
}

// Evaluate the reference's recursive-doubling order (reduce.cpp:3890-3925,
// non-commutative branch included) with the user's function.
int host_user_allreduce(Comm* c, const void* sendbuf, void* recvbuf, size_t count,
                        MPI_Datatype dt, const OpRef& op)
{
    const int p = c->size;
    const Img m = img_of(dt, count);
    const size_t bytes = m.bytes;
    std::vector<char> mine(bytes), all((size_t)p * bytes);
    int rc = img_load(m, sendbuf == MPI_IN_PLACE ? recvbuf : sendbuf, mine.data());
    if (rc == MPI_SUCCESS) rc = c->tp->allgather(mine.data(), bytes, all.data());
    if (rc != MPI_SUCCESS) return rc;
    auto call = [&](const char* in, char* io) { img_call(op, dt, m, count, in - m.lo, io - m.lo); };
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
    return img_store(m, count, v[src].data() - m.lo, recvbuf);
}

// Evaluate RankTree `t` on host with a user function (same association and
// inout/in roles as k_tree: the left operand is `inout`).  x[r] = typed base of
// rank r's contribution (count elements, image `m`); the result image is
// written at typed base `out`.
void eval_tree_host(const RankTree& t, const std::vector<const char*>& x, char* out, size_t count,
                    MPI_Datatype dt, const OpRef& op, const Img& m)
{
    const size_t bytes = m.bytes;
    auto call = [&](const char* in, char* io) { img_call(op, dt, m, count, in, io); };
    auto img = [&](const char* base) { return base + m.lo; };
    if (t.chain) {
        memcpy(out + m.lo, img(x[(size_t)t.src[0]]), bytes);
        for (int k = 1; k < t.P; ++k) call(x[(size_t)t.src[k]], out);
        return;
    }
    const int nl = t.nleaves ? t.nleaves : t.P;
    std::vector<std::vector<char>> v((size_t)nl);
    for (int k = 0; k < nl; ++k) {
        v[(size_t)k].assign(img(x[(size_t)t.src[2 * k]]), img(x[(size_t)t.src[2 * k]]) + bytes);
        if ((t.pairmask >> k) & 1u) call(x[(size_t)t.src[2 * k + 1]], v[(size_t)k].data() - m.lo);
    }
    for (int w = 1; w < t.P; w *= 2)
        for (int k = 0; k + w < t.P; k += 2 * w)
            if (k + w < nl) call(v[(size_t)(k + w)].data() - m.lo, v[(size_t)k].data() - m.lo);
    memcpy(out + m.lo, v[0].data(), bytes);
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

// ---- window collectives (push model) ----------------------------------------
// Every rank owns one IPC-mapped device window of 2*C bytes: an IN area of p
// sub-slots of Q = C/p bytes (sub-slot k receives rank k's contribution) and an
// OUT area of C bytes (the reduced chunk, assembled from every owner's piece).
// User buffers are never IPC-mapped (ROCm 7.2 hangs opening handles of
// allocations > 2 GiB, and user memory may be host memory).  Data crosses
// xGMI only as REMOTE WRITES (posted stores, all peer links at once);
// reductions read local HBM only:
//   scatter : piece r of my chunk -> IN(r)[sub-slot me]             (xGMI writes)
//   barrier A (every contribution landed: writers synced before it)
//   reduce  : my piece from IN(me)[0..p-1], the reference's expression tree
//             per element -> OUT(me)[my piece]                        (local)
//   push    : OUT(me)[my piece] -> OUT(r)[my piece], every r          (xGMI writes)
//   barrier B (every piece landed)
//   collect : OUT(me) -> recvbuf                                      (local / D2H)
// One slot suffices: a peer scatters chunk i+1 into IN(me) only after barrier B
// of chunk i (I finished reading IN(me) before it) and pushes into OUT(me)
// only after barrier A of chunk i+1 (I collected chunk i before it).  After a
// collective's last barrier B no peer touches my window, so the next
// collective needs no extra barrier.
// Default C = 960 MiB, the largest whose window (2 C + flags) stays below the
// 2 GiB IPC mapping limit: 1.9 GB of each rank's 288 GB.  Rounds 1-4 used
// 512 MiB; with the larger window c3 takes 3 pipelined chunks instead of 5 at
// p = 8, and 2 ranks on one MI355X measured c3 1.87 -> 1.77 ms and c4 3.80 ->
// 3.60 ms (bench.py's engine-variant sweep, profiles/r04/bench_n2_variants.json).
size_t chunk_bytes()
{
    static size_t c = [] {
        size_t v = (size_t)960 << 20;
        if (const char* e = getenv("MSX_CHUNK_BYTES")) v = (size_t)atoll(e);
        if (v < ((size_t)1 << 16)) v = (size_t)1 << 16;
        if (v > ((size_t)960 << 20)) v = (size_t)960 << 20;   // whole window < 2 GiB (IPC limit)
        return v & ~(size_t)4095;
    }();
    return c;
}

// Arrival flags of the barrier-free allreduce live behind the two areas:
// flag k of window r (8 bytes) = the last call sequence rank k posted to r.
constexpr size_t kFlagBytes = 64 << 10;
// Passive-target RMA staging (its own IPC allocation, created by the first
// passive-target window of a communicator): p payload slots (written by each
// origin) then p fetch slots (written by each target), the agreed size / (2p) each.
// Every slot-sized piece of a lock / PSCW operation costs one host handshake
// with the target's service thread (~50 us), so the area is sized for large
// pieces (MSX_RMA_BYTES, default 512 MiB), below the 2 GiB IPC limit.  256 MiB lock / PSCW accumulates, 2 ranks on one MI355X
// (profiles/r02/rma_area_*.json): 1.27 ms with 64 MiB, 0.66 ms with 256 MiB,
// 0.53 ms with 512 MiB (= the fence epoch's 0.54 ms).
// The area belongs to the communicator's transport: every communicator with a
// window holds one per rank.  Without MSX_RMA_BYTES the default is capped per
// GPU: 512 MiB divided by the ranks that share this GPU (8 ranks on one GPU:
// 64 MiB each), at least 64 MiB.  `share` is counted by the transport from
// every rank's PCI bus id, and the ranks then take the minimum of their sizes
// (IpcTransport::rma_window), so all of them address the same slots.
size_t rma_bytes_for(int share)
{
    size_t b = (size_t)512 << 20;
    if (share > 1) b = std::max(b / (size_t)share, (size_t)64 << 20);
    if (const char* e = getenv("MSX_RMA_BYTES")) b = (size_t)atoll(e);
    const size_t cap = ((size_t)2 << 30) - ((size_t)1 << 20);      // IPC mapping limit
    b = std::min(b, cap);
    return std::max(b, (size_t)4 << 20) & ~(size_t)4095;
}

// Sub-slots are Q bytes long but S = Q + skew apart: the p-source tree reads
// every sub-slot at the same offset, and sources a power of two apart lose
// HBM bandwidth to channel aliasing (scripts/tree_skew_probe.py on MI355X,
// profiles/r01/tree_skew_probe.log: 8 x 32 MiB, 6.27 TB/s at a 32 MiB stride,
// 6.51-6.56 TB/s with 4-68 KiB added).
size_t sub_skew(size_t per_rank)
{
    if (per_rank >= ((size_t)16 << 20)) return (size_t)68 << 10;
    return (per_rank / 16) & ~(size_t)255;
}

// usable bytes of one sub-slot of a window with chunk C over p ranks: C/p
// minus the skew, so the IN area is exactly C.  (Late round 3 tried the whole
// C/p with the skew on top and reverted it; round 4 re-ran that layout to
// rule it out for the wrong results DESIGN.md §2 explains.)
size_t sub_len(size_t C, int p)
{
    const size_t per = C / (size_t)p;
    return (per - sub_skew(per)) & ~(size_t)255;
}

// IN area of a window: p sub-slots sub_skew apart, C bytes in all
size_t in_bytes(size_t C, int /*p*/) { return C; }

struct Windows {
    std::vector<char*> base;
    size_t C = 0, Q = 0, S = 0, I = 0;   // chunk, sub-slot length, sub-slot stride, IN area bytes
    char* in(int r) const { return base[(size_t)r]; }
    char* sub(int r, int k) const { return base[(size_t)r] + (size_t)k * S; }
    char* out(int r) const { return base[(size_t)r] + I; }
    unsigned long long* flags(int r) const { return reinterpret_cast<unsigned long long*>(base[(size_t)r] + I + C); }
    // passive-target staging (rma_window), when the communicator has one
    std::vector<char*> rbase;
    size_t rbytes = 0;                    // the agreed staging size (rma_window)
    size_t rma_slot() const { return (rbytes / (2 * rbase.size())) & ~(size_t)255; }
    // rank r's staging: payload slot written by origin o / fetch slot written by target t
    char* rma_in(int r, int o) const { return rbase[(size_t)r] + (size_t)o * rma_slot(); }
    char* rma_fetch(int r, int t) const { return rbase[(size_t)r] + (rbase.size() + (size_t)t) * rma_slot(); }
};

// Result-ready flags of the two-step allreduce live in the upper half of the
// flag area: slot kResultFlags + k of window r = the last call whose result
// rank k stored into r's OUT area.
constexpr size_t kResultFlags = 4096;
// Scan partials' arrival flags: slot kScanFlags + k of window r = (call << 6)
// | step of the last partial rank k pushed to r (only scan writes them).
constexpr size_t kScanFlags = 2048;
// GPU "done" flags of the pipelined two-step allreduce: slot kDoneFlags + k of
// window r = the last chunk (flag sequence number) whose IN / OUT halves rank
// k finished reading; a chunk two later may then overwrite them.
constexpr size_t kDoneFlags = 6144;

// Largest message (bytes) of the barrier-free two-step allreduce / reduce
// (MSX_TWO_STEP_MAX; 0 = always the host-barrier schedule).  By default every
// Rabenseifner-sized message takes it, longer ones as a GPU-synchronised
// pipeline of window-half chunks (round 4; rounds 1-3 stopped at 256 MiB and
// ran the rest through host barriers, five host syncs per chunk).  2 ranks on
// one MI355X (scripts/allreduce_probe.sh, profiles/r02/two_step_*) measured
// 1 MiB 62.6 -> 28.5 us, 4 MiB 64.3 -> 32.5, 16 MiB 75.6 -> 45.8,
// 64 MiB 154.8 -> 133.0, 128 MiB 265 -> 249; 4 ranks 64 MiB 310 -> 254.
// Defaults (round 5; same value on every rank, gpu_shared is agreed):
//  * ranks sharing a GPU: 0, the host-barrier schedules (round 4's default
//    there; the flag schedules run when MSX_TWO_STEP_MAX asks, as the tests
//    do).  The wrong results recorded on this path in rounds 3-4 were the test
//    harness's own pageable transfers, not the schedule.
//  * one rank per GPU: 256 MiB, the rounds 1-3 cap -- a single chunk of the
//    two-step schedule; longer messages run the host-barrier pipeline.  The
//    cross-GPU data plane has not run on hardware yet (no multi-GPU box has
//    been available to the tests), so the multi-chunk GPU-flag pipeline is
//    opt-in (MSX_TWO_STEP_MAX) until the one-rank-per-GPU suites pass.
size_t two_step_max(const Transport* tp)
{
    static const char* e = getenv("MSX_TWO_STEP_MAX");
    if (e) return (size_t)atoll(e);
    return tp->gpu_shared ? 0 : (size_t)256 << 20;
}

// Pinned bounce buffers of the engine (engine worker, or the one inline
// blocking call): 0 = this rank's contribution, 1 = the result.
Bounce& engine_bounce(int i)
{
    static Bounce b[2];
    return b[i];
}

// Pinned host word the arrival wait reports a timeout through (engine worker
// only); returns its device view.
int* wait_err_word(int** host)
{
    static int* h = nullptr;
    static int* d = nullptr;
    if (!h) {
        if (hipHostMalloc(reinterpret_cast<void**>(&h), sizeof(int), hipHostMallocCoherent | hipHostMallocMapped) !=
            hipSuccess) {
            h = nullptr;
            return nullptr;
        }
        if (hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0) != hipSuccess) d = h;
    }
    *host = h;
    return d;
}

int get_windows(Transport* tp, Windows* w, bool rd_single = false)
{
    w->C = chunk_bytes();
    w->Q = sub_len(w->C, tp->size);
    w->S = w->Q + sub_skew(w->C / (size_t)tp->size);
    w->I = in_bytes(w->C, tp->size);
    // [IN: p sub-slots, C bytes][OUT: C][flags]: 2 C + 64 KiB, below the
    // 2 GiB IPC mapping limit for C <= 960 MiB (checked: a larger allocation
    // would hang hipIpcOpenMemHandle, see map_peers)
    if (w->I + w->C + kFlagBytes > ((size_t)2046 << 20)) {
        set_error("window of %zu bytes exceeds the IPC mapping limit (MSX_CHUNK_BYTES too large)",
                  w->I + w->C + kFlagBytes);
        return MPI_ERR_INTERN;
    }
    int rc = tp->window(w->I + w->C + kFlagBytes, w->base);
    if (rc == MPI_SUCCESS && tp->window_open && !rd_single) {
        // the last recursive-doubling call left without its closing barrier:
        // peers may still be reading their IN areas
        rc = tp->barrier();
        tp->window_open = false;
    }
    if (!rd_single) tp->out_quiet = false;      // a host-barrier user of the OUT areas
    return rc;
}

// Copies of at least kKernelCopyMin bytes within this GPU's memory (HBM
// buffers, its own window) run on the engine's copy kernel: 256 MiB local
// copies take 68 us there and 99 us as hipMemcpyAsync's blit
// (profiles/r02/copy/copy_cmp.log).  Host memory keeps hipMemcpyAsync (DMA).
constexpr size_t kKernelCopyMin = (size_t)1 << 20;

int copy_async(void* dst, const void* src, size_t bytes, hipStream_t s)
{
    if (!bytes) return MPI_SUCCESS;
    if (bytes >= kKernelCopyMin) {
        const BufInfo bs = classify(src), bd = classify(dst);
        int cur = -1;
        (void)hipGetDevice(&cur);
        // both on this GPU (a peer's window or another GPU's buffer: the blit),
        // 16-byte aligned (otherwise the kernel falls back to one byte per
        // lane, far below the blit)
        if (bs.place == Place::Device && bd.place == Place::Device && bs.device == cur && bd.device == cur &&
            (((uintptr_t)bs.dev | (uintptr_t)bd.dev) & 15) == 0) {
            const void* ps = bs.dev;
            void* pd = bd.dev;
            hipError_t e = launch_copy_segs(&ps, &pd, &bytes, 1, s);
            return e == hipSuccess ? MPI_SUCCESS : hip_fail(e, "copy kernel");
        }
    }
    // a pageable host side never goes to HIP's copy path (xfer_sync)
    if (host_pageable(dst) || host_pageable(src)) return xfer_sync(dst, src, bytes, s);
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, s);   // xfer: device/pinned
    return e == hipSuccess ? MPI_SUCCESS : hip_fail(e, "stage copy");
}

// Phase timers of the window allreduce (host clock, engine worker only):
// t[0] stage + scatter, t[1] collect wait + barrier A, t[2] reduce + push,
// t[3] barrier B, t[4] last collect.  Read by msx_engine_stats().
struct EngineStats {
    double t[5] = {0, 0, 0, 0, 0};
    long chunks = 0, calls = 0;
    long flag_calls = 0;   // GPU-flag Rabenseifner calls (two-step allreduce / reduce, flag reduce_scatter)
};
EngineStats g_stats;

// The communicator's second engine stream: local copies that overlap xGMI
// work.  Created on first use; nullptr (callers then stay on their stream)
// if HIP refuses.
hipStream_t aux_stream(Transport* tp)
{
    if (!tp->aux && hipStreamCreateWithFlags(&tp->aux, hipStreamNonBlocking) != hipSuccess) {
        (void)hipGetLastError();
        tp->aux = nullptr;
    }
    return tp->aux;
}

// A batch of byte ranges moved by one k_copy_segs launch (one grid row each).
struct Segs {
    std::vector<const void*> src;
    std::vector<void*> dst;
    std::vector<size_t> n;
    void add(const void* s, void* d, size_t bytes)
    {
        if (!bytes) return;
        src.push_back(s);
        dst.push_back(d);
        n.push_back(bytes);
    }
    int run(hipStream_t s, const char* what)
    {
        if (src.empty()) return MPI_SUCCESS;
        hipError_t e = launch_copy_segs(src.data(), dst.data(), n.data(), (int)src.size(), s);
        return e == hipSuccess ? MPI_SUCCESS : hip_fail(e, what);
    }
};

// Device view of `len` bytes of a user buffer at byte offset `off`: the buffer
// itself when it is device memory, else staged into `stage` (H2D).
int device_view(const BufInfo& b, const char* user, size_t off, size_t len, char* stage,
                hipStream_t s, const char** out)
{
    if (b.place == Place::Device) {
        *out = static_cast<const char*>(b.dev) + off;
        return MPI_SUCCESS;
    }
    *out = stage;
    return copy_async(stage, user + off, len, s);
}

// ---- RCCL plane (MSX_TRANSPORT=rccl) -------------------------------------------
// The same reference-order trees, with the bytes moved by RCCL point-to-point
// (ncclSend/ncclRecv groups over xGMI) instead of IPC windows: no host
// barriers, no peer mappings, user device buffers sent and received in place,
// everything ordered on the engine stream.  RCCL needs one GPU per rank; a
// communicator whose ranks share a GPU keeps the IPC window engine.
// librccl is opened lazily so the library has no link-time RCCL dependency.
struct RcclApi {
    decltype(&ncclGetUniqueId) get_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) err = nullptr;
    // RCCL's own collectives (MSX_TRANSPORT=rccl_native)
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclReduce) reduce = nullptr;
    decltype(&ncclReduceScatter) reduce_scatter = nullptr;
    bool ok = false;
};

const RcclApi* rccl_api()
{
    static RcclApi a = [] {
        RcclApi r;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
        if (!h) return r;
        r.get_id = reinterpret_cast<decltype(r.get_id)>(dlsym(h, "ncclGetUniqueId"));
        r.init_rank = reinterpret_cast<decltype(r.init_rank)>(dlsym(h, "ncclCommInitRank"));
        r.destroy = reinterpret_cast<decltype(r.destroy)>(dlsym(h, "ncclCommDestroy"));
        r.send = reinterpret_cast<decltype(r.send)>(dlsym(h, "ncclSend"));
        r.recv = reinterpret_cast<decltype(r.recv)>(dlsym(h, "ncclRecv"));
        r.group_start = reinterpret_cast<decltype(r.group_start)>(dlsym(h, "ncclGroupStart"));
        r.group_end = reinterpret_cast<decltype(r.group_end)>(dlsym(h, "ncclGroupEnd"));
        r.err = reinterpret_cast<decltype(r.err)>(dlsym(h, "ncclGetErrorString"));
        r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(h, "ncclAllReduce"));
        r.reduce = reinterpret_cast<decltype(r.reduce)>(dlsym(h, "ncclReduce"));
        r.reduce_scatter = reinterpret_cast<decltype(r.reduce_scatter)>(dlsym(h, "ncclReduceScatter"));
        r.ok = r.get_id && r.init_rank && r.destroy && r.send && r.recv && r.group_start && r.group_end && r.err;
        return r;
    }();
    return a.ok ? &a : nullptr;
}

bool rccl_requested()
{
    static const bool v = [] {
        const char* e = getenv("MSX_TRANSPORT");
        return e && (strcmp(e, "rccl") == 0 || strcmp(e, "rccl_native") == 0);
    }();
    return v;
}

// MSX_TRANSPORT=rccl_native: (op, type) pairs that map onto RCCL's reductions
// run as ncclAllReduce / ncclReduce / ncclReduceScatter on the user's device
// buffers -- RCCL's ring/tree association, NOT the reference's: integer
// results are identical (two's-complement wrap), fp32/fp64 SUM and PROD agree
// within |y - y_ref| <= 2(p-1) 2^-p_mant sum_r |x_r|, MAX and
// MIN agree except where NaN / signed-zero ties decide.  Every other pair,
// host operands and ragged reduce_scatter counts keep the reference-order
// trees on the RCCL send/recv plane.
bool rccl_native_requested()
{
    static const bool v = [] {
        const char* e = getenv("MSX_TRANSPORT");
        return e && strcmp(e, "rccl_native") == 0;
    }();
    return v;
}

bool rccl_map(int opidx, Kind k, ncclRedOp_t* op, ncclDataType_t* t)
{
    switch (opidx) {
    case O_SUM: *op = ncclSum; break;
    case O_PROD: *op = ncclProd; break;
    case O_MAX: *op = ncclMax; break;
    case O_MIN: *op = ncclMin; break;
    default: return false;
    }
    switch (k) {
    case K_I8: *t = ncclInt8; return true;
    case K_U8: *t = ncclUint8; return true;
    case K_I32: *t = ncclInt32; return true;
    case K_U32: *t = ncclUint32; return true;
    case K_I64: *t = ncclInt64; return true;
    case K_U64: *t = ncclUint64; return true;
    case K_F32: *t = ncclFloat32; return true;
    case K_F64: *t = ncclFloat64; return true;
    default: return false;
    }
}

std::map<Transport*, ncclComm_t> g_rccl_comms;
std::map<Transport*, bool> g_rccl_refused;
// RCCL communicators of freed transports: retired, not destroyed.
// ncclCommDestroy would release RCCL's device buffers, and freeing uncached
// device memory corrupted later allocations on this stack.
std::vector<ncclComm_t> g_rccl_retired;

// Called when `tp` is destroyed (engine worker, or finalize): a later
// transport may get the same address and must not find this one's state.
void rccl_forget(Transport* tp)
{
    auto it = g_rccl_comms.find(tp);
    if (it != g_rccl_comms.end()) {
        g_rccl_retired.push_back(it->second);
        g_rccl_comms.erase(it);
    }
    g_rccl_refused.erase(tp);
}

// Communicator for `tp` (collective on first use; nullptr = use IPC windows).
ncclComm_t rccl_comm(Transport* tp)
{
    auto& comms = g_rccl_comms;
    auto& refused = g_rccl_refused;
    auto it = comms.find(tp);
    if (it != comms.end()) return it->second;
    if (refused.count(tp)) return nullptr;
    const RcclApi* api = rccl_api();
    // every rank must take the same decision: agree on (api ok, device identity)
    struct Id { int32_t ok; int32_t dev; char bus[32]; };
    Id mine;
    memset(&mine, 0, sizeof(mine));
    mine.ok = api ? 1 : 0;
    (void)hipGetDevice(&mine.dev);
    (void)hipDeviceGetPCIBusId(mine.bus, sizeof(mine.bus), mine.dev);
    std::vector<Id> all((size_t)tp->size);
    if (tp->allgather(&mine, sizeof(mine), all.data()) != MPI_SUCCESS) { refused[tp] = true; return nullptr; }
    bool usable = true;
    for (int r = 0; r < tp->size; ++r) {
        usable = usable && all[r].ok;
        for (int q = 0; q < r; ++q) usable = usable && strncmp(all[r].bus, all[q].bus, sizeof(all[r].bus)) != 0;
    }
    if (!usable) {
        trace("rccl: not usable (library missing or ranks share a GPU); IPC windows in use");
        refused[tp] = true;
        return nullptr;
    }
    ncclUniqueId id;
    memset(&id, 0, sizeof(id));
    if (tp->rank == 0) api->get_id(&id);
    std::vector<ncclUniqueId> ids((size_t)tp->size);
    if (tp->allgather(&id, sizeof(id), ids.data()) != MPI_SUCCESS) { refused[tp] = true; return nullptr; }
    ncclComm_t comm = nullptr;
    ncclResult_t r = api->init_rank(&comm, tp->size, ids[0], tp->rank);
    trace("rccl: ncclCommInitRank rc=%d", (int)r);
    // Every rank must take the same plane: a rank whose init failed while its
    // peers' succeeded would run the IPC schedules against their RCCL calls and
    // hang both.  Agree on the outcome; any failure sends all to IPC windows.
    int32_t ok = r == ncclSuccess ? 1 : 0;
    std::vector<int32_t> oks((size_t)tp->size);
    if (tp->allgather(&ok, sizeof(ok), oks.data()) != MPI_SUCCESS) ok = 0;
    for (int32_t o : oks) ok = ok && o;
    if (!ok) {
        if (r == ncclSuccess) (void)api->destroy(comm);
        else set_error("ncclCommInitRank: %s", api->err(r));
        trace("rccl: a rank's ncclCommInitRank failed; IPC windows in use");
        refused[tp] = true;
        return nullptr;
    }
    comms[tp] = comm;
    return comm;
}

// One ncclGroupStart/End batch of sends and receives (bytes), stream-ordered.
struct P2p {
    struct Op { bool send; void* buf; size_t n; int peer; };
    std::vector<Op> ops;
    void send(const void* b, size_t n, int peer) { if (n) ops.push_back({true, const_cast<void*>(b), n, peer}); }
    void recv(void* b, size_t n, int peer) { if (n) ops.push_back({false, b, n, peer}); }
    int run(ncclComm_t comm, hipStream_t s, const char* what)
    {
        if (ops.empty()) return MPI_SUCCESS;
        const RcclApi* api = rccl_api();
        ncclResult_t r = api->group_start();
        for (const Op& o : ops) {
            if (r != ncclSuccess) break;
            r = o.send ? api->send(o.buf, o.n, ncclUint8, o.peer, comm, s)
                       : api->recv(o.buf, o.n, ncclUint8, o.peer, comm, s);
        }
        ncclResult_t r2 = api->group_end();
        if (r == ncclSuccess) r = r2;
        if (r != ncclSuccess) { set_error("%s: %s", what, api->err(r)); return MPI_ERR_OTHER; }
        return MPI_SUCCESS;
    }
};

int rccl_allreduce(ncclComm_t comm, Comm* c, const void* sendbuf, void* recvbuf, size_t count,
                   MPI_Datatype dt, const OpRef& op, int root, bool nbc)
{
    Transport* tp = c->tp;
    const int p = c->size, me = c->rank;
    const TypeInfo* ti = type_info(dt);
    const Kind k = ti->kind;
    const size_t esz = (size_t)ti->size;
    hipStream_t s = tp->stream();
    const char* src = static_cast<const char*>(sendbuf == MPI_IN_PLACE ? recvbuf : sendbuf);
    char* dst = static_cast<char*>(recvbuf);
    const bool want = (root < 0 || root == me);
    ncclRedOp_t nop;
    ncclDataType_t nty;
    const RcclApi* api = rccl_api();
    if (rccl_native_requested() && rccl_map(op.opidx, k, &nop, &nty) &&
        (root < 0 ? api->all_reduce != nullptr : api->reduce != nullptr)) {
        // Every rank takes this branch for a mappable pair (the pair is the
        // same on every rank), so no per-call agreement is needed: a rank
        // whose operands are host memory stages them through device scratch
        // (H2D, RCCL in place on the scratch, D2H) instead of leaving the
        // others in an RCCL collective alone.
        const bool sdev = classify(src).place == Place::Device;
        const bool ddev = !want || classify(dst).place == Place::Device;
        const char* in = src;
        char* out = want ? dst : const_cast<char*>(src);
        char* tmp = nullptr;
        int rc = MPI_SUCCESS;
        if (!sdev || !ddev) {
            tmp = dev_scratch(count * esz);
            if (!tmp) { set_error("allreduce: scratch allocation failed"); return MPI_ERR_NO_MEM; }
            rc = copy_async(tmp, src, count * esz, s);
            in = out = tmp;
        }
        if (rc != MPI_SUCCESS) return rc;
        ncclResult_t r = root < 0 ? api->all_reduce(in, out, count, nty, nop, comm, s)
                                  : api->reduce(in, out, count, nty, nop, root, comm, s);
        trace("rccl native %s: count=%zu staged=%d rc=%d", root < 0 ? "allreduce" : "reduce", count, tmp != nullptr,
              (int)r);
        if (r != ncclSuccess) {
            set_error("%s: %s", root < 0 ? "ncclAllReduce" : "ncclReduce", api->err(r));
            return MPI_ERR_OTHER;
        }
        if (tmp && want) rc = copy_async(dst, tmp, count * esz, s);
        return rc == MPI_SUCCESS ? sync_stream(s, root < 0 ? "allreduce" : "reduce") : rc;
    }
    const bool is_reduce = root >= 0;
    const int gate = gate_type_size(dt, nbc);
    const int algo = is_reduce ? reduce_algo(p, count, gate, true) : allreduce_algo(p, count, gate, true);
    const BufInfo bs = classify(src), bd = classify(dst);
    size_t qmax = (chunk_bytes() / (size_t)p) / esz;
    qmax -= qmax % 16;
    // scratch: [IN: p sub-slots of qmax, skewed apart (sub_skew)][OUT: p*qmax][stage: p*qmax]
    const size_t sub_b = qmax * esz, area = (size_t)p * sub_b;
    const size_t sub_s = sub_b + sub_skew(chunk_bytes() / (size_t)p);
    char* scratch = dev_scratch((size_t)p * sub_s + 2 * area);
    if (!scratch) { set_error("allreduce: scratch allocation failed"); return MPI_ERR_NO_MEM; }
    char* inb = scratch;
    char* outb = scratch + (size_t)p * sub_s;
    char* stage = outb + area;
    std::vector<char*> srcs((size_t)p);
    const int pof2 = pof2_floor(p);
    const int n = newrank_of(me, p);
    const int lineage = n >= 0 ? n : newrank_of(me + 1, p);
    int rc = MPI_SUCCESS;
    trace("rccl allreduce: count=%zu algo=%d qmax=%zu", count, algo, qmax);
    if (algo == A_RECURSIVE_DOUBLING || algo == A_BINOMIAL) {
        const RankTree t = (algo == A_BINOMIAL) ? tree_reduce_binomial(p, root) : tree_allreduce(p, lineage);
        for (size_t o = 0; o < count && rc == MPI_SUCCESS; o += qmax) {
            const size_t len = std::min(qmax, count - o);
            const char* mine = nullptr;
            rc = device_view(bs, src, o * esz, len * esz, stage, s, &mine);
            P2p x;
            for (int r = 0; r < p; ++r) {
                if (r == me) continue;
                if (root < 0 || r == root) x.send(mine, len * esz, r);
                if (want) x.recv(inb + (size_t)r * sub_s, len * esz, r);
            }
            if (rc == MPI_SUCCESS) rc = x.run(comm, s, "allreduce exchange");
            if (rc == MPI_SUCCESS && want) {
                for (int r = 0; r < p; ++r) srcs[r] = (r == me) ? const_cast<char*>(mine) : inb + (size_t)r * sub_s;
                char* out = bd.place == Place::Device ? static_cast<char*>(bd.dev) + o * esz : outb;
                rc = run_rank_tree(op.opidx, k, t, srcs, esz, 0, len, out, s);
                if (rc == MPI_SUCCESS && out == outb) rc = copy_async(dst + o * esz, out, len * esz, s);
            }
        }
        return rc == MPI_SUCCESS ? sync_stream(s, "allreduce") : rc;
    }
    const size_t ce = (size_t)p * qmax;
    for (size_t o = 0; o < count && rc == MPI_SUCCESS; o += ce) {
        const size_t len = std::min(ce, count - o);
        const size_t q = (len + p - 1) / p;
        const size_t qv = (q + 15) & ~(size_t)15;
        auto lo_of = [&](int r) { return std::min(len, (size_t)r * qv); };
        auto hi_of = [&](int r) { return std::min(len, (size_t)(r + 1) * qv); };
        const size_t plo = lo_of(me), phi = hi_of(me);
        const char* mine = nullptr;
        rc = device_view(bs, src, o * esz, len * esz, stage, s, &mine);
        P2p x;                                        // reduce-scatter as all-to-all
        for (int r = 0; r < p; ++r) {
            if (r == me) continue;
            x.send(mine + lo_of(r) * esz, (hi_of(r) - lo_of(r)) * esz, r);
            x.recv(inb + (size_t)r * sub_s, (phi - plo) * esz, r);
        }
        if (rc == MPI_SUCCESS) rc = x.run(comm, s, "allreduce scatter");
        for (int r = 0; r < p; ++r) srcs[r] = (r == me) ? const_cast<char*>(mine) + plo * esz : inb + (size_t)r * sub_s;
        char* outp = (want && bd.place == Place::Device) ? static_cast<char*>(bd.dev) + o * esz : outb;
        for (size_t e0 = plo; e0 < phi && rc == MPI_SUCCESS;) {
            const size_t ge = o + e0;
            const size_t rs = count / (size_t)pof2;
            const int j = rs ? (int)std::min((size_t)pof2 - 1, ge / rs) : pof2 - 1;
            size_t bst, bl;
            allreduce_block(p, count, j, &bst, &bl);
            const size_t e1 = std::min(phi, bst + bl - o);
            const int owner = allreduce_block_owner(p, j);
            const RankTree t = !is_reduce ? tree_allreduce(p, owner)
                                          : (nbc ? tree_ireduce_rsag(p, owner, root) : tree_reduce_rsag(p, owner));
            rc = run_rank_tree(op.opidx, k, t, srcs, esz, e0 - plo, e1 - e0, outp + e0 * esz, s);
            e0 = e1;
        }
        P2p g;                                        // allgather (or gather at root)
        for (int r = 0; r < p; ++r) {
            if (r == me) continue;
            if (root < 0 || r == root) g.send(outp + plo * esz, (phi - plo) * esz, r);
            if (want) g.recv(outp + lo_of(r) * esz, (hi_of(r) - lo_of(r)) * esz, r);
        }
        if (rc == MPI_SUCCESS) rc = g.run(comm, s, "allreduce gather");
        if (rc == MPI_SUCCESS && want && outp == outb) rc = copy_async(dst + o * esz, outb, len * esz, s);
    }
    return rc == MPI_SUCCESS ? sync_stream(s, "allreduce") : rc;
}

int rccl_reduce_scatter(ncclComm_t comm, Comm* c, const void* sendbuf, void* recvbuf, const int* recvcounts,
                        MPI_Datatype dt, const OpRef& op)
{
    Transport* tp = c->tp;
    const int p = c->size, me = c->rank;
    const size_t esz = dtype_is_derived(dt) ? 0 : (size_t)type_size(dt);   // derived: user ops only
    std::vector<size_t> disp((size_t)p + 1, 0);
    size_t maxcnt = 0;
    for (int r = 0; r < p; ++r) {
        disp[r + 1] = disp[r] + (size_t)recvcounts[r];
        maxcnt = std::max(maxcnt, (size_t)recvcounts[r]);
    }
    const size_t total = disp[p];
    const bool in_place = (sendbuf == MPI_IN_PLACE);
    const char* src = static_cast<const char*>(in_place ? recvbuf : sendbuf);
    const Kind k = type_info(dt)->kind;
    hipStream_t s = tp->stream();
    ncclRedOp_t nop;
    ncclDataType_t nty;
    const RcclApi* api = rccl_api();
    if (rccl_native_requested() && api->reduce_scatter && rccl_map(op.opidx, k, &nop, &nty) &&
        maxcnt * (size_t)p == total) {
        // equal blocks (recvcounts are the same on every rank by MPI rule):
        // ncclReduceScatter.  Taken by every rank alike (no per-call
        // agreement): host operands are staged through device scratch, and in
        // place my block moves to recvbuf[0]
        const bool sdev = classify(src).place == Place::Device, ddev = classify(recvbuf).place == Place::Device;
        const char* in = src;
        void* out = recvbuf;
        char* tmp = nullptr;
        int rc = MPI_SUCCESS;
        if (!sdev || !ddev) {
            tmp = dev_scratch((total + maxcnt) * esz);          // [input][my block]
            if (!tmp) { set_error("reduce_scatter: scratch allocation failed"); return MPI_ERR_NO_MEM; }
            rc = copy_async(tmp, src, total * esz, s);
            in = tmp;
            out = tmp + total * esz;
        } else if (in_place && me != 0 && maxcnt) {
            tmp = dev_scratch(maxcnt * esz);      // RCCL's in-place form wants recvbuf + rank*count
            if (!tmp) { set_error("reduce_scatter: scratch allocation failed"); return MPI_ERR_NO_MEM; }
            out = tmp;
        }
        if (rc != MPI_SUCCESS) return rc;
        ncclResult_t r = api->reduce_scatter(in, out, maxcnt, nty, nop, comm, s);
        trace("rccl native reduce_scatter: count=%zu staged=%d rc=%d", maxcnt, (!sdev || !ddev), (int)r);
        if (r != ncclSuccess) { set_error("ncclReduceScatter: %s", api->err(r)); return MPI_ERR_OTHER; }
        if (out != recvbuf) rc = copy_async(recvbuf, out, maxcnt * esz, s);
        return rc == MPI_SUCCESS ? sync_stream(s, "reduce_scatter") : rc;
    }
    size_t qe = (chunk_bytes() / (size_t)p) / esz;
    qe -= qe % 16;
    const int algo = reduce_scatter_algo(p, total, gate_type_size(dt, false), op.commutative);
    const int n = newrank_of(me, p);
    const RankTree t = (algo == A_RS_PAIRWISE) ? tree_pairwise(p, me)
                                               : tree_reduce_scatter(p, n >= 0 ? n : newrank_of(me + 1, p));
    const size_t mycnt = (size_t)recvcounts[me];
    const BufInfo bs = classify(src), bd = classify(recvbuf);
    char* dst = static_cast<char*>(recvbuf);
    // scratch: [IN: p sub-slots of qe, skewed apart][OUT: qe][stage: p*qe][hold: mycnt if in place]
    const size_t sub_b = qe * esz, area = (size_t)p * sub_b;
    const size_t sub_s = sub_b + sub_skew(chunk_bytes() / (size_t)p);
    const size_t hold_b = in_place ? mycnt * esz : 0;
    char* scratch = dev_scratch((size_t)p * sub_s + area + sub_b + hold_b);
    if (!scratch) { set_error("reduce_scatter: scratch allocation failed"); return MPI_ERR_NO_MEM; }
    char* inb = scratch;
    char* outb = scratch + (size_t)p * sub_s;
    char* stage = outb + sub_b;
    char* hold = stage + area;
    std::vector<char*> srcs((size_t)p);
    int rc = MPI_SUCCESS;
    trace("rccl reduce_scatter: total=%zu algo=%d round=%zu", total, algo, qe);
    for (size_t o = 0; o < maxcnt && rc == MPI_SUCCESS; o += qe) {
        P2p x;
        const char* myseg = nullptr;
        for (int r = 0; r < p && rc == MPI_SUCCESS; ++r) {
            const size_t cnt = (size_t)recvcounts[r];
            if (o >= cnt) continue;
            const size_t len = std::min(qe, cnt - o);
            const char* v = nullptr;
            rc = device_view(bs, src, (disp[r] + o) * esz, len * esz, stage + (size_t)r * sub_b, s, &v);
            if (r == me) myseg = v;
            else x.send(v, len * esz, r);
        }
        const size_t len = o < mycnt ? std::min(qe, mycnt - o) : 0;
        for (int r = 0; r < p; ++r)
            if (r != me) x.recv(inb + (size_t)r * sub_s, len * esz, r);
        if (rc == MPI_SUCCESS) rc = x.run(comm, s, "reduce_scatter exchange");
        if (rc == MPI_SUCCESS && len) {
            for (int r = 0; r < p; ++r) srcs[r] = (r == me) ? const_cast<char*>(myseg) : inb + (size_t)r * sub_s;
            char* out = in_place ? hold + o * esz
                                 : (bd.place == Place::Device ? static_cast<char*>(bd.dev) + o * esz : outb);
            rc = run_rank_tree(op.opidx, k, t, srcs, esz, 0, len, out, s);
            if (rc == MPI_SUCCESS && out == outb) rc = copy_async(dst + o * esz, out, len * esz, s);
        }
    }
    if (rc == MPI_SUCCESS && in_place && mycnt) rc = copy_async(recvbuf, hold, mycnt * esz, s);
    return rc == MPI_SUCCESS ? sync_stream(s, "reduce_scatter") : rc;
}

}  // namespace

// Elements per chunk of the pipelined two-step allreduce / reduce for p ranks
// and elements of esz bytes: p pieces of at most half an IN sub-slot each, the
// whole chunk within half the OUT area above the recursive-doubling results,
// whole 16-element pieces (0: the window is too small).
size_t two_step_chunk_el(int p, size_t esz)
{
    const size_t Qh = (sub_len(chunk_bytes(), p) / 2) & ~(size_t)255;
    const size_t qh_el = (Qh / esz) & ~(size_t)15;
    const size_t out_half = ((chunk_bytes() - Qh) / 2) & ~(size_t)255;
    size_t pc_el = std::min((size_t)p * qh_el, out_half / esz);
    return pc_el - pc_el % ((size_t)p * 16);
}

// Rank me's part of chunk ci: its piece [plo, phi) of the chunk (16-element
// granules) cut where the owner tree changes -- the owner of an element is
// that of its block in the WHOLE vector (allreduce_block, reduce.cpp:3927-
// 4066), so the chunking never changes a result.  Offsets are relative to
// the chunk start o = ci * pc_el.
void two_step_plan(int p, size_t count, size_t pc_el, size_t ci, int me, std::vector<TwoStepRange>* ranges,
                   size_t* plo, size_t* phi, size_t* len_out)
{
    const int pof2 = pof2_floor(p);
    const size_t o = ci * pc_el, len = std::min(pc_el, count - o);
    const size_t pel = (((len + (size_t)p - 1) / (size_t)p) + 15) & ~(size_t)15;
    *plo = std::min(len, (size_t)me * pel);
    *phi = std::min(len, (size_t)(me + 1) * pel);
    *len_out = len;
    ranges->clear();
    const size_t rs = count / (size_t)pof2;
    for (size_t e0 = *plo; e0 < *phi;) {
        const size_t ge = o + e0;
        const int j = rs ? (int)std::min((size_t)pof2 - 1, ge / rs) : pof2 - 1;
        size_t bst, bl;
        allreduce_block(p, count, j, &bst, &bl);
        const size_t e1 = std::min(*phi, bst + bl - o);
        ranges->push_back({e0, e1, allreduce_block_owner(p, j)});
        e0 = e1;
    }
}

namespace {

// root < 0: allreduce; root >= 0: only `root` receives the result (MPI_Reduce).
int do_allreduce(Comm* c, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
                 const OpRef& op, int root = -1, bool nbc = false)
{
    // user functions are host code: no GPU needed on this path
    if (op.opidx == O_NULL) return host_user_allreduce(c, sendbuf, recvbuf, count, dt, op);
    int rc = ensure_device();
    if (rc != MPI_SUCCESS) return rc;

    Transport* tp = c->tp;
    if (rccl_requested())
        if (ncclComm_t rcomm = rccl_comm(tp)) return rccl_allreduce(rcomm, c, sendbuf, recvbuf, count, dt, op, root, nbc);
    const int p = c->size, me = c->rank;
    const TypeInfo* ti = type_info(dt);
    const Kind k = ti->kind;
    const size_t esz = (size_t)ti->size;
    hipStream_t s = tp->stream();
    const char* src = static_cast<const char*>(sendbuf == MPI_IN_PLACE ? recvbuf : sendbuf);
    char* dst = static_cast<char*>(recvbuf);
    const bool want = (root < 0 || root == me);          // this rank receives the result
    const bool is_reduce = root >= 0;
    const int gate = gate_type_size(dt, nbc);
    const int algo = is_reduce ? reduce_algo(p, count, gate, true) : allreduce_algo(p, count, gate, true);
    // A recursive-doubling (or binomial) call that fits half a sub-slot runs
    // barrier-free at its end: it uses the IN half `rd_parity`, alternating per
    // call.  Pushing into a peer's half P again (two calls later) happens only
    // after this rank passed the previous call's barrier A, which that peer
    // reached only after finishing its tree on half P.
    const size_t Qh = (sub_len(chunk_bytes(), p) / 2) & ~(size_t)255;
    const bool rd_single = (algo == A_RECURSIVE_DOUBLING || algo == A_BINOMIAL) &&
                           count * esz <= (Qh & ~(size_t)(16 * esz - 1)) && p <= 32 && tp->has_done();
    // Rabenseifner in two GPU-synchronised steps per chunk (see below): a
    // chunk is p pieces of at most half an IN sub-slot each and fits half the
    // OUT area above the recursive-doubling results; a longer message runs as
    // a pipeline of such chunks.  Only count, type, p and the environment
    // decide, so every rank takes the same branch and the same chunks.
    const size_t out_half = ((chunk_bytes() - Qh) / 2) & ~(size_t)255;
    const size_t pc_el = two_step_chunk_el(p, esz);
    const bool two_step = algo == A_RABENSEIFNER && p >= 2 && p <= 32 && tp->has_done() &&
                          count * esz <= two_step_max(tp) && pc_el > 0;
    Windows w;
    if ((rc = get_windows(tp, &w, rd_single || two_step)) != MPI_SUCCESS) return rc;
    // host buffers: device aliases for the call (pinned in place of staging)
    BufInfo bs = classify(src), bd = classify(dst);
    PinHold pins;
    pins.sync_before_release(s);
    if (hipStream_t a = aux_stream(tp)) pins.sync_before_release(a);
    alias_host_operands(pins, true, src, count * esz, &bs, want ? dst : nullptr, want ? count * esz : 0, &bd);
    // elements per sub-slot, whole 16-element granules
    size_t qmax = w.Q / esz;
    qmax -= qmax % 16;
    if (qmax == 0) { set_error("allreduce: window too small"); return MPI_ERR_INTERN; }
    char* stage = nullptr;
    if (bs.place != Place::Device) {
        stage = dev_scratch(std::min(count, (size_t)p * qmax) * esz);
        if (!stage) { set_error("allreduce: scratch allocation failed"); return MPI_ERR_NO_MEM; }
    }
    const int pof2 = pof2_floor(p);
    const int n = newrank_of(me, p);
    const int lineage = n >= 0 ? n : newrank_of(me + 1, p);
    std::vector<char*> subs((size_t)p);
    for (int r = 0; r < p; ++r) subs[r] = w.sub(me, r);
    trace("allreduce: count=%zu esz=%zu algo=%d qmax=%zu", count, esz, algo, qmax);

    if (algo == A_RECURSIVE_DOUBLING || algo == A_BINOMIAL) {
        // every rank that evaluates a tree needs every contribution whole:
        // recursive doubling -> all ranks evaluate their own lineage's tree;
        // binomial reduce -> only the root evaluates
        const RankTree t = (algo == A_BINOMIAL) ? tree_reduce_binomial(p, root) : tree_allreduce(p, lineage);
        if (rd_single) {
            // No host barrier at all.  Each rank pushes its vector into the IN
            // half of every rank that evaluates a tree (all peers for
            // allreduce, the root for reduce) and posts the call's sequence
            // number into their flag slots; ONE workgroup of the same launch
            // (k_push_wait) waits on the GPU until all peers' flags reached the
            // sequence, and the tree follows in stream order.  (Rounds 1-2 let
            // every tree workgroup spin on the flags instead, one launch less;
            // with a multi-MiB tree spinning, five ranks sharing one GPU starved
            // each other's pushes until the 20 s bound.)
            // A half is reused two calls later: before pushing call s into
            // rank r's half, this rank waits (host, shared memory) until r has
            // posted that it finished call s-2 -- normally long since true.
            const size_t half = (size_t)tp->rd_parity * Qh;
            for (int r = 0; r < p; ++r) subs[r] = w.sub(me, r) + half;
            // small host buffers go through the engine's pinned bounce buffers
            // (CPU copies in and out, the kernels read / write them over PCIe)
            // instead of synchronous pageable copies through HBM staging
            const size_t nbytes = count * esz;
            const bool bounce_src = bs.place != Place::Device && nbytes <= bounce_max_bytes() &&
                                    engine_bounce(0).get(nbytes);
            const bool bounce_dst = want && bd.place != Place::Device && nbytes <= bounce_max_bytes() &&
                                    engine_bounce(1).get(nbytes);
            const char* mine = nullptr;
            if (bounce_src) {
                memcpy(engine_bounce(0).host, src, nbytes);
                mine = engine_bounce(0).dev;
            } else {
                rc = device_view(bs, src, 0, nbytes, stage, s, &mine);
            }
            const unsigned long long seq = ++tp->rd_seq;
            Segs sg;
            std::vector<unsigned long long*> fl;
            for (int r = 0; r < p && rc == MPI_SUCCESS; ++r)
                if (r != me && (root < 0 || r == root)) {
                    if (seq > 2) rc = tp->wait_done(r, seq - 2);
                    sg.add(mine, w.sub(r, me) + half, count * esz);
                    if (!fault_drop_flags(me, seq)) fl.push_back(w.flags(r) + me);
                }
            subs[(size_t)me] = const_cast<char*>(mine);
            int* err_host = nullptr;
            int* err_dev = wait_err_word(&err_host);
            if (!err_dev) { set_error("allreduce: arrival word allocation failed"); return MPI_ERR_NO_MEM; }
            *err_host = 0;
            char* out = bd.place == Place::Device ? static_cast<char*>(bd.dev)
                                                  : (bounce_dst ? engine_bounce(1).dev : w.out(me));
            unsigned* counter = nullptr;
            if (rc == MPI_SUCCESS && !sg.src.empty()) {
                counter = tp->push_counter();
                if (!counter) { set_error("allreduce: push counter allocation failed"); return MPI_ERR_NO_MEM; }
            }
            if (rc == MPI_SUCCESS) {
                hipError_t e = launch_push_wait(sg.src.data(), sg.dst.data(), sg.n.data(), (int)sg.src.size(),
                                                fl.data(), (int)fl.size(), seq,
                                                counter ? counter + kCountWords : nullptr, w.flags(me),
                                                want ? p : 0, me, err_dev, s);
                if (e != hipSuccess) rc = hip_fail(e, "allreduce push");
            }
            if (rc == MPI_SUCCESS && want) {
                rc = run_rank_tree(op.opidx, k, t, subs, esz, 0, count, out, s);   // after the wait, in stream order
                if (rc == MPI_SUCCESS && out == w.out(me)) rc = copy_async(dst, out, count * esz, s);
            }
            const int rs = sync_stream(s, "allreduce tree");
            if (rc == MPI_SUCCESS) rc = rs;
            if (rc == MPI_SUCCESS && bounce_dst) memcpy(dst, engine_bounce(1).host, nbytes);
            if (rc == MPI_SUCCESS && __atomic_load_n(err_host, __ATOMIC_ACQUIRE))
                rc = flag_timeout(root < 0 ? "allreduce" : "reduce", me, __atomic_load_n(err_host, __ATOMIC_ACQUIRE),
                                  seq);
            tp->post_done(seq);                   // this rank's tree no longer reads the half
            tp->rd_parity ^= 1;
            tp->window_open = true;
            trace("allreduce: done (GPU arrival flags, seq %llu) rc=%d", seq, rc);
            return rc;
        }
        for (size_t o = 0; o < count && rc == MPI_SUCCESS; o += qmax) {
            const size_t len = std::min(qmax, count - o);
            const char* mine = nullptr;
            rc = device_view(bs, src, o * esz, len * esz, stage, s, &mine);
            Segs sg;                      // my own contribution is read in place
            for (int r = 0; r < p; ++r)
                if (r != me && (root < 0 || r == root)) sg.add(mine, w.sub(r, me), len * esz);
            subs[(size_t)me] = const_cast<char*>(mine);
            if (rc == MPI_SUCCESS) rc = sg.run(s, "allreduce push");
            if (rc == MPI_SUCCESS) rc = sync_stream(s, "allreduce push");
            if (rc == MPI_SUCCESS) rc = tp->barrier();                              // A
            if (rc == MPI_SUCCESS && want) {
                char* out = bd.place == Place::Device ? static_cast<char*>(bd.dev) + o * esz : w.out(me);
                rc = run_rank_tree(op.opidx, k, t, subs, esz, 0, len, out, s);
                if (rc == MPI_SUCCESS && out == w.out(me)) rc = copy_async(dst + o * esz, out, len * esz, s);
                if (rc == MPI_SUCCESS) rc = sync_stream(s, "allreduce tree");
            }
            if (rc == MPI_SUCCESS) rc = tp->barrier();                              // B
        }
        trace("allreduce: done rc=%d", rc);
        return rc;
    }

    if (two_step) {
        // Barrier-free Rabenseifner: the same pieces, trees and result
        // placement as the host-barrier schedule below, synchronised on the
        // GPU, chunk by chunk with no host synchronisation between chunks.
        // Per chunk (elements [o, o + len), pieces cut in 16-element granules):
        //  0. (chunks >= 2) one workgroup waits until every peer posted that it
        //     finished chunk seq - 2 (its GPU "done" flag): the IN / OUT halves
        //     this chunk writes are free.  The first two chunks of a call are
        //     guarded on the host by the previous flag calls' post_done.
        //  1. k_push_wait: piece r of my chunk -> rank r's IN half, then its
        //     arrival flag; one workgroup waits for every peer's piece of mine.
        //  2. my piece evaluated (one launch per owner tree, owners by GLOBAL
        //     element, reduce.cpp:3941-4065) into the OUT half of every
        //     receiver; the last workgroup posts result-ready flags (tree_done).
        //  3. receivers: one workgroup waits for every peer's result flag,
        //     then the OUT half is copied into recvbuf + o.
        //  4. (when a later chunk of this call reuses the halves) my "done"
        //     flag into every peer's window, after the copy in stream order.
        // Halves alternate with rd_parity per chunk.  One host sync per call
        // (rounds 1-3 paid five per 512 MiB chunk on the host-barrier path).
        // Only single workgroups spin, so ranks sharing a GPU cannot starve
        // each other's pushes.
        if (!tp->out_quiet && (rc = tp->barrier()) != MPI_SUCCESS) return rc;
        int* err_host = nullptr;
        int* err_dev = wait_err_word(&err_host);
        unsigned* counter = tp->push_counter();
        if (!err_dev || !counter) { set_error("allreduce: flag word allocation failed"); return MPI_ERR_NO_MEM; }
        *err_host = 0;
        std::vector<int> dests;
        if (want) dests.push_back(me);
        for (int r = 0; r < p; ++r)
            if (r != me && (root < 0 || r == root)) dests.push_back(r);
        std::vector<unsigned long long*> done_to;            // my GPU done flag in every peer's window
        for (int r = 0; r < p; ++r)
            if (r != me) done_to.push_back(w.flags(r) + kDoneFlags + me);
        const size_t nchunks = (count + pc_el - 1) / pc_el;
        unsigned long long seq = 0;
        size_t nranges = 0;
        std::vector<TwoStepRange> ranges;
        for (size_t ci = 0; ci < nchunks && rc == MPI_SUCCESS; ++ci) {
            const size_t o = ci * pc_el;
            size_t plo, phi, len;
            two_step_plan(p, count, pc_el, ci, me, &ranges, &plo, &phi, &len);
            const size_t pel = (((len + (size_t)p - 1) / (size_t)p) + 15) & ~(size_t)15;
            auto lo_of = [&](int r) { return std::min(len, (size_t)r * pel); };
            auto hi_of = [&](int r) { return std::min(len, (size_t)(r + 1) * pel); };
            const size_t half = (size_t)tp->rd_parity * Qh;
            const size_t obase = Qh + (size_t)tp->rd_parity * out_half;
            const char* mine = nullptr;
            rc = device_view(bs, src, o * esz, len * esz, stage, s, &mine);
            seq = ++tp->rd_seq;
            if (ci < 2) {
                for (int r = 0; r < p && rc == MPI_SUCCESS; ++r)
                    if (r != me && seq > 2) rc = tp->wait_done(r, seq - 2);
            } else if (rc == MPI_SUCCESS) {
                hipError_t e = launch_push_wait(nullptr, nullptr, nullptr, 0, nullptr, 0, seq - 2, nullptr,
                                                w.flags(me) + kDoneFlags, p, me, err_dev, s, 3);
                if (e != hipSuccess) rc = hip_fail(e, "allreduce half-free wait");
            }
            if (rc != MPI_SUCCESS) break;
            Segs sg;
            std::vector<unsigned long long*> fl, done;
            for (int r = 0; r < p; ++r) {
                if (r == me || hi_of(r) <= lo_of(r)) continue;
                sg.add(mine + lo_of(r) * esz, w.sub(r, me) + half, (hi_of(r) - lo_of(r)) * esz);
                if (!fault_drop_flags(me, seq)) fl.push_back(w.flags(r) + me);
            }
            for (int d : dests)
                if (d != me) done.push_back(w.flags(d) + kResultFlags + me);
            nranges += ranges.size();
            for (int r = 0; r < p; ++r) subs[r] = w.sub(me, r) + half;
            subs[(size_t)me] = const_cast<char*>(mine) + plo * esz;
            // step 1: push my pieces and their arrival flags; one workgroup
            // waits for the peers' pieces of mine (none when my piece is empty)
            hipError_t e = launch_push_wait(sg.src.data(), sg.dst.data(), sg.n.data(), (int)sg.src.size(), fl.data(),
                                            (int)fl.size(), seq, counter + kCountWords, w.flags(me),
                                            ranges.empty() ? 0 : p, me, err_dev, s);
            if (e != hipSuccess) rc = hip_fail(e, "allreduce push");
            // step 2: my piece into every receiver's OUT half; the last
            // workgroup of the last launch posts the result flags
            if (rc == MPI_SUCCESS && ranges.empty() && !done.empty()) {
                e = launch_post_flags(done.data(), (int)done.size(), seq, s);
                if (e != hipSuccess) rc = hip_fail(e, "allreduce result flags");
            }
            for (size_t i = 0; i < ranges.size() && rc == MPI_SUCCESS; ++i) {
                const TwoStepRange& g = ranges[i];
                const RankTree t = !is_reduce ? tree_allreduce(p, g.owner)
                                              : (nbc ? tree_ireduce_rsag(p, g.owner, root) : tree_reduce_rsag(p, g.owner));
                std::vector<char*> extra;
                for (size_t d = 1; d < dests.size(); ++d) extra.push_back(w.out(dests[d]) + obase + g.e0 * esz);
                TreeWait tw;
                tw.done_counter = counter + 2 * kCountWords;
                tw.done_launches = (unsigned)ranges.size();
                tw.done_flags = &done;
                tw.done_seq = seq;
                rc = run_rank_tree(op.opidx, k, t, subs, esz, g.e0 - plo, g.e1 - g.e0,
                                   w.out(dests[0]) + obase + g.e0 * esz, s, extra, &tw);
            }
            if (rc == MPI_SUCCESS && want) {
                // step 3: every peer's result in my OUT half, then into recvbuf
                e = launch_push_wait(nullptr, nullptr, nullptr, 0, nullptr, 0, seq, nullptr,
                                     w.flags(me) + kResultFlags, p, me, err_dev, s, 2);
                if (e != hipSuccess) rc = hip_fail(e, "allreduce result wait");
                char* out = bd.place == Place::Device ? static_cast<char*>(bd.dev) : dst;
                if (rc == MPI_SUCCESS) rc = copy_async(out + o * esz, w.out(me) + obase, len * esz, s);
            }
            // step 4: this chunk's halves are free again (read by my trees and
            // my copy, both earlier on the stream) -- only a later chunk of
            // this call waits on it
            if (rc == MPI_SUCCESS && ci + 2 < nchunks) {
                e = launch_post_flags(done_to.data(), (int)done_to.size(), seq, s);
                if (e != hipSuccess) rc = hip_fail(e, "allreduce done flags");
            }
            tp->rd_parity ^= 1;
        }
        ++g_stats.flag_calls;
        const int rsy = sync_stream(s, "allreduce two-step");
        if (rc == MPI_SUCCESS) rc = rsy;
        if (rc == MPI_SUCCESS && __atomic_load_n(err_host, __ATOMIC_ACQUIRE))
            rc = flag_timeout(root < 0 ? "allreduce" : "reduce", me, __atomic_load_n(err_host, __ATOMIC_ACQUIRE), seq);
        tp->post_done(seq);
        tp->window_open = true;
        tp->out_quiet = true;
        trace("allreduce: done (two-step, GPU flags, %zu chunk(s), last seq %llu, %zu ranges) rc=%d", nchunks, seq,
              nranges, rc);
        return rc;
    }

    // Rabenseifner order: element e belongs to block j(e), whose value the
    // reference computes at newrank bitrev(j).  Each chunk is cut into p
    // pieces (work balance only, 16-element granules); each element of a piece
    // is evaluated with the tree of its block's owner.
    const size_t ce = (size_t)p * qmax;
    hipStream_t s2 = aux_stream(tp) ? aux_stream(tp) : s;
    for (size_t o = 0; o < count && rc == MPI_SUCCESS; o += ce) {
        const double t0 = now_s();
        const size_t len = std::min(ce, count - o);
        const size_t q = (len + p - 1) / p;
        const size_t qv = (q + 15) & ~(size_t)15;
        auto lo_of = [&](int r) { return std::min(len, (size_t)r * qv); };
        auto hi_of = [&](int r) { return std::min(len, (size_t)(r + 1) * qv); };
        const char* mine = nullptr;
        rc = device_view(bs, src, o * esz, len * esz, stage, s, &mine);
        Segs scatter;
        for (int r = 0; r < p; ++r)                  // my own piece is read in place
            if (r != me) scatter.add(mine + lo_of(r) * esz, w.sub(r, me), (hi_of(r) - lo_of(r)) * esz);
        subs[(size_t)me] = const_cast<char*>(mine) + lo_of(me) * esz;
        if (rc == MPI_SUCCESS) rc = scatter.run(s, "allreduce scatter");
        if (rc == MPI_SUCCESS) rc = sync_stream(s, "allreduce scatter");
        const double t1 = now_s();
        if (rc == MPI_SUCCESS) rc = sync_stream(s2, "allreduce collect");           // OUT(me) free
        if (rc == MPI_SUCCESS) rc = tp->barrier();                                  // A
        const double t2 = now_s();
        if (rc != MPI_SUCCESS) break;
        const size_t plo = lo_of(me), phi = hi_of(me);
        // reduce my piece from my IN area (local) and store the result straight
        // into every receiver's OUT area: the push is fused into the tree
        // kernel (remote stores over xGMI)
        std::vector<int> dests;
        if (want) dests.push_back(me);
        for (int r = 0; r < p; ++r)
            if (r != me && (root < 0 || r == root)) dests.push_back(r);
        for (size_t e0 = plo; e0 < phi && rc == MPI_SUCCESS;) {
            const size_t ge = o + e0;                                             // global element
            const size_t rs = count / (size_t)pof2;
            const int j = rs ? (int)std::min((size_t)pof2 - 1, ge / rs) : pof2 - 1;
            size_t bst, bl;
            allreduce_block(p, count, j, &bst, &bl);
            const size_t e1 = std::min(phi, bst + bl - o);
            const int owner = allreduce_block_owner(p, j);
            const RankTree t = !is_reduce ? tree_allreduce(p, owner)
                                          : (nbc ? tree_ireduce_rsag(p, owner, root) : tree_reduce_rsag(p, owner));
            std::vector<char*> extra;
            for (size_t d = 1; d < dests.size(); ++d) extra.push_back(w.out(dests[d]) + e0 * esz);
            rc = run_rank_tree(op.opidx, k, t, subs, esz, e0 - plo, e1 - e0, w.out(dests[0]) + e0 * esz, s, extra);
            e0 = e1;
        }
        if (rc == MPI_SUCCESS) rc = sync_stream(s, "allreduce push");
        const double t3 = now_s();
        if (rc == MPI_SUCCESS) rc = tp->barrier();                                  // B
        const double t4 = now_s();
        g_stats.chunks += 1;
        g_stats.t[0] += t1 - t0;
        g_stats.t[1] += t2 - t1;
        g_stats.t[2] += t3 - t2;
        g_stats.t[3] += t4 - t3;
        // collect on a second stream: it overlaps the next chunk's scatter
        // (local HBM copy vs xGMI writes); synced before the next barrier A
        if (rc == MPI_SUCCESS && want) rc = copy_async(dst + o * esz, w.out(me), len * esz, s2);
    }
    const double tc = now_s();
    if (rc == MPI_SUCCESS) rc = sync_stream(s2, "allreduce collect");
    g_stats.t[4] += now_s() - tc;
    g_stats.calls += 1;
    trace("allreduce: done rc=%d", rc);
    return rc;
}

int do_reduce_scatter(Comm* c, const void* sendbuf, void* recvbuf, const int* recvcounts,
                      MPI_Datatype dt, const OpRef& op)
{
    Transport* tp = c->tp;
    const int p = c->size, me = c->rank;
    const size_t esz = dtype_is_derived(dt) ? 0 : (size_t)type_size(dt);   // derived: user ops only
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
        // images of the whole input (total elements) and of my block (mycnt);
        // block r starts disp[r] elements (x extent for a derived type) into it
        const Img mf = img_of(dt, total), mb = img_of(dt, (size_t)recvcounts[me]);
        const int64_t unit = mf.t ? mf.t->extent : (int64_t)esz;
        std::vector<char> full(mf.bytes);
        int rc = img_load(mf, src, full.data());
        if (rc != MPI_SUCCESS) return rc;
        const size_t mycnt = (size_t)recvcounts[me];
        if (op.commutative) {
            // commutative user op: the builtin schedules (recursive halving or
            // pairwise, same 32-bit gate) evaluated on host with the user's
            // function, reduce.cpp:917-1334
            std::vector<char> all((size_t)p * mf.bytes);
            if ((rc = c->tp->allgather(full.data(), mf.bytes, all.data())) != MPI_SUCCESS) return rc;
            const int algo = reduce_scatter_algo(p, total, gate_type_size(dt, false), true);
            const int n = newrank_of(me, p);
            const RankTree t = (algo == A_RS_PAIRWISE) ? tree_pairwise(p, me)
                                                       : tree_reduce_scatter(p, n >= 0 ? n : newrank_of(me + 1, p));
            std::vector<const char*> x((size_t)p);
            for (int r = 0; r < p; ++r)
                x[(size_t)r] = all.data() + (size_t)r * mf.bytes - mf.lo + (int64_t)disp[me] * unit;
            std::vector<char> res(mb.bytes);
            eval_tree_host(t, x, res.data() - mb.lo, mycnt, dt, op, mb);
            return mycnt ? img_store(mb, mycnt, res.data() - mb.lo, recvbuf) : MPI_SUCCESS;
        }
        // non-commutative: recursive doubling (MPIR_Reduce_scatter_non_commutative,
        // reduce.cpp:1340-1630) -- for a power-of-two p each block is exactly the
        // recursive-doubling allreduce value; other p share its lower-first order
        std::vector<char> res(mf.bytes);
        rc = host_user_allreduce(c, full.data() - mf.lo, res.data() - mf.lo, total, dt, op);
        if (rc == MPI_SUCCESS && mycnt)
            rc = img_store(mb, mycnt, res.data() - mf.lo + (int64_t)disp[me] * unit, recvbuf);
        return rc;
    }
    int rc = ensure_device();
    if (rc != MPI_SUCCESS) return rc;
    if (rccl_requested())
        if (ncclComm_t rcomm = rccl_comm(tp)) return rccl_reduce_scatter(rcomm, c, sendbuf, recvbuf, recvcounts, dt, op);
    const Kind k = type_info(dt)->kind;
    hipStream_t s = tp->stream();
    // GPU-synchronised rounds (decided by recvcounts, type, p and the
    // environment: the same on every rank): in round k, slice k of block r of
    // my input (at most half an IN sub-slot) goes into rank r's IN half with
    // its arrival flag while one workgroup waits for the peers' slices of my
    // block (k_push_wait), then my slice is evaluated.  One round when every
    // block fits half a sub-slot; longer blocks (c4: 512 MiB per rank at
    // p = 8) pipeline their rounds with GPU "half free" flags as the two-step
    // allreduce does, one host sync per call instead of four per round.
    const size_t Qh = (sub_len(chunk_bytes(), p) / 2) & ~(size_t)255;
    const size_t qh_el = esz ? (Qh / esz) & ~(size_t)15 : 0;
    const bool one_step = p >= 2 && p <= 32 && tp->has_done() && total * esz <= two_step_max(tp) && qh_el > 0;
    Windows w;
    if ((rc = get_windows(tp, &w, one_step)) != MPI_SUCCESS) return rc;
    // sub-slot k of IN(r) receives rank k's contribution to r's block, qe
    // elements per round
    size_t qe = w.Q / esz;
    qe -= qe % 16;
    if (qe == 0) { set_error("reduce_scatter: window too small"); return MPI_ERR_INTERN; }
    const int algo = reduce_scatter_algo(p, total, gate_type_size(dt, false), op.commutative);
    const int n = newrank_of(me, p);
    const RankTree t = (algo == A_RS_PAIRWISE) ? tree_pairwise(p, me)
                                               : tree_reduce_scatter(p, n >= 0 ? n : newrank_of(me + 1, p));
    trace("reduce_scatter: total=%zu esz=%zu algo=%d round=%zu", total, esz, algo, qe);
    const size_t mycnt = (size_t)recvcounts[me];
    BufInfo bs = classify(src), bd = classify(recvbuf);
    PinHold pins;                        // host buffers: device aliases for the call
    pins.sync_before_release(s);
    alias_host_operands(pins, true, src, total * esz, &bs, in_place ? nullptr : recvbuf, in_place ? 0 : mycnt * esz,
                        &bd);
    char* dst = static_cast<char*>(recvbuf);
    if (one_step) {
        const size_t hold_b = in_place ? ((mycnt * esz + 255) & ~(size_t)255) : 0;
        const size_t stage_b = bs.place == Place::Device ? 0 : total * esz;
        char* scratch = nullptr;
        if (hold_b + stage_b) {
            scratch = dev_scratch(hold_b + stage_b);
            if (!scratch) { set_error("reduce_scatter: scratch allocation failed"); return MPI_ERR_NO_MEM; }
        }
        int* err_host = nullptr;
        int* err_dev = wait_err_word(&err_host);
        unsigned* counter = tp->push_counter();
        if (!err_dev || !counter) { set_error("reduce_scatter: flag word allocation failed"); return MPI_ERR_NO_MEM; }
        *err_host = 0;
        std::vector<unsigned long long*> done_to;          // my GPU done flag in every peer's window
        for (int r = 0; r < p; ++r)
            if (r != me) done_to.push_back(w.flags(r) + kDoneFlags + me);
        // in place, recvbuf still holds the input later rounds push: results via hold
        char* out = in_place ? scratch : (bd.place == Place::Device ? static_cast<char*>(bd.dev) : w.out(me));
        const bool out_window = !in_place && out == w.out(me);   // host recvbuf: round by round via OUT
        const size_t nrounds = maxcnt ? (maxcnt + qh_el - 1) / qh_el : 1;
        unsigned long long seq = 0;
        std::vector<char*> subs((size_t)p);
        for (size_t ri = 0; ri < nrounds && rc == MPI_SUCCESS; ++ri) {
            const size_t o = ri * qh_el;
            const size_t half = (size_t)tp->rd_parity * Qh;
            seq = ++tp->rd_seq;
            if (ri < 2) {
                for (int r = 0; r < p && rc == MPI_SUCCESS; ++r)
                    if (r != me && seq > 2) rc = tp->wait_done(r, seq - 2);
            } else if (rc == MPI_SUCCESS) {
                hipError_t e = launch_push_wait(nullptr, nullptr, nullptr, 0, nullptr, 0, seq - 2, nullptr,
                                                w.flags(me) + kDoneFlags, p, me, err_dev, s, 3);
                if (e != hipSuccess) rc = hip_fail(e, "reduce_scatter half-free wait");
            }
            Segs sg;
            std::vector<unsigned long long*> fl;
            for (int r = 0; r < p && rc == MPI_SUCCESS; ++r) {
                const size_t cnt = (size_t)recvcounts[r];
                const size_t len = o < cnt ? std::min(qh_el, cnt - o) : 0;
                const char* v = nullptr;
                if (len)
                    rc = device_view(bs, src, (disp[r] + o) * esz, len * esz,
                                     scratch ? scratch + hold_b + (disp[r] + o) * esz : nullptr, s, &v);
                if (r == me) { subs[(size_t)me] = const_cast<char*>(v); continue; }
                subs[(size_t)r] = w.sub(me, r) + half;
                if (len && rc == MPI_SUCCESS) {
                    sg.add(v, w.sub(r, me) + half, len * esz);
                    if (!fault_drop_flags(me, seq)) fl.push_back(w.flags(r) + me);
                }
            }
            const size_t mylen = o < mycnt ? std::min(qh_el, mycnt - o) : 0;
            if (rc == MPI_SUCCESS) {
                hipError_t e = launch_push_wait(sg.src.data(), sg.dst.data(), sg.n.data(), (int)sg.src.size(),
                                                fl.data(), (int)fl.size(), seq, counter + kCountWords,
                                                w.flags(me), mylen ? p : 0, me, err_dev, s);
                if (e != hipSuccess) rc = hip_fail(e, "reduce_scatter push");
            }
            if (rc == MPI_SUCCESS && mylen) {
                char* ro = out_window ? out : out + o * esz;
                rc = run_rank_tree(op.opidx, k, t, subs, esz, 0, mylen, ro, s);
                if (rc == MPI_SUCCESS && out_window) rc = copy_async(dst + o * esz, ro, mylen * esz, s);
            }
            if (rc == MPI_SUCCESS && ri + 2 < nrounds) {     // this round's half is read: free two rounds on
                hipError_t e = launch_post_flags(done_to.data(), (int)done_to.size(), seq, s);
                if (e != hipSuccess) rc = hip_fail(e, "reduce_scatter done flags");
            }
            tp->rd_parity ^= 1;
        }
        if (rc == MPI_SUCCESS && mycnt && in_place) rc = copy_async(dst, out, mycnt * esz, s);
        ++g_stats.flag_calls;
        const int rs = sync_stream(s, "reduce_scatter one-step");
        if (rc == MPI_SUCCESS) rc = rs;
        if (rc == MPI_SUCCESS && __atomic_load_n(err_host, __ATOMIC_ACQUIRE))
            rc = flag_timeout("reduce_scatter", me, __atomic_load_n(err_host, __ATOMIC_ACQUIRE), seq);
        tp->post_done(seq);
        tp->window_open = true;
        trace("reduce_scatter: done (GPU flags, %zu round(s), last seq %llu) rc=%d", nrounds, seq, rc);
        return rc;
    }
    // scratch: [hold: in-place results][stage: host-resident input pieces]
    const size_t hold_b = in_place ? ((mycnt * esz + 255) & ~(size_t)255) : 0;
    const size_t stage_b = bs.place == Place::Device ? 0 : (size_t)p * qe * esz;
    char* scratch = nullptr;
    if (hold_b + stage_b) {
        scratch = dev_scratch(hold_b + stage_b);
        if (!scratch) { set_error("reduce_scatter: scratch allocation failed"); return MPI_ERR_NO_MEM; }
    }
    char* hold = scratch;
    char* stage = scratch ? scratch + hold_b : nullptr;
    std::vector<char*> subs((size_t)p);
    for (int r = 0; r < p; ++r) subs[r] = w.sub(me, r);
    for (size_t o = 0; o < maxcnt && rc == MPI_SUCCESS; o += qe) {
        // my contribution to every destination's block range [o, o+qe)
        Segs scatter;
        for (int r = 0; r < p && rc == MPI_SUCCESS; ++r) {
            const size_t cnt = (size_t)recvcounts[r];
            if (o >= cnt) continue;
            const size_t len = std::min(qe, cnt - o);
            const char* v = nullptr;
            rc = device_view(bs, src, (disp[r] + o) * esz, len * esz, stage ? stage + (size_t)r * qe * esz : nullptr,
                             s, &v);
            if (r == me) subs[(size_t)me] = const_cast<char*>(v);   // read in place
            else scatter.add(v, w.sub(r, me), len * esz);
        }
        if (rc == MPI_SUCCESS) rc = scatter.run(s, "reduce_scatter scatter");
        if (rc == MPI_SUCCESS) rc = sync_stream(s, "reduce_scatter scatter");
        if (rc == MPI_SUCCESS) rc = tp->barrier();                                  // A
        if (rc != MPI_SUCCESS) break;
        if (o < mycnt) {
            const size_t len = std::min(qe, mycnt - o);
            // In place, recvbuf is still our input for later rounds: results go
            // to a private device scratch and are copied out at the end.
            char* out = in_place ? hold + o * esz
                                 : (bd.place == Place::Device ? static_cast<char*>(bd.dev) + o * esz : w.out(me));
            rc = run_rank_tree(op.opidx, k, t, subs, esz, 0, len, out, s);
            if (rc == MPI_SUCCESS && out == w.out(me)) rc = copy_async(dst + o * esz, out, len * esz, s);
            if (rc == MPI_SUCCESS) rc = sync_stream(s, "reduce_scatter reduce");
        }
        if (rc == MPI_SUCCESS) rc = tp->barrier();                                  // B
    }
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
                     const OpRef& op, bool nbc)
{
    return worker().run([=] { return do_allreduce(c, sendbuf, recvbuf, count, dt, op, -1, nbc); });
}

int engine_reduce_scatter(Comm* c, const void* sendbuf, void* recvbuf, const int* recvcounts,
                          MPI_Datatype dt, const OpRef& op)
{
    std::vector<int> counts(recvcounts, recvcounts + c->size);
    return worker().run([=] { return do_reduce_scatter(c, sendbuf, recvbuf, counts.data(), dt, op); });
}

namespace {

// MPI_Reduce with a user function (host code): every contribution is gathered
// to host memory and the reference's binomial tree is evaluated with the
// user's function (reduce.cpp:440-540): relative ranks from lroot = root for
// commutative ops, else from 0 with the result sent to root; the parent
// combines a child's buffer as `in` (commutative) or as `inout` with its own
// as `in` (non-commutative, "the sender is above us").
int host_user_reduce(Comm* c, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
                     const OpRef& op, int root)
{
    const int p = c->size, me = c->rank;
    const Img m = img_of(dt, count);
    const size_t bytes = m.bytes;
    std::vector<char> mine(bytes), all((size_t)p * bytes);
    int rc = img_load(m, sendbuf == MPI_IN_PLACE ? recvbuf : sendbuf, mine.data());
    if (rc == MPI_SUCCESS) rc = c->tp->allgather(mine.data(), bytes, all.data());
    if (rc != MPI_SUCCESS || me != root) return rc;
    auto call = [&](const char* in, char* io) { img_call(op, dt, m, count, in - m.lo, io - m.lo); };
    const int lroot = op.commutative ? root : 0;
    auto buf = [&](int rel) { return all.data() + (size_t)((rel + lroot) % p) * bytes; };
    std::vector<char> tmp(bytes);
    for (int mask = 1; mask < p; mask <<= 1) {
        for (int rel = 0; rel < p; rel += 2 * mask) {     // receivers at this level
            const int src = rel | mask;
            if (src >= p) continue;
            if (op.commutative) {
                call(buf(src), buf(rel));
            } else {
                memcpy(tmp.data(), buf(src), bytes);
                call(buf(rel), tmp.data());
                memcpy(buf(rel), tmp.data(), bytes);
            }
        }
    }
    return img_store(m, count, buf(0) - m.lo, recvbuf);
}

}  // namespace

int engine_reduce(Comm* c, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
                  const OpRef& op, int root, bool nbc)
{
    // Builtin ops: the reference's binomial / Rabenseifner trees (do_allreduce
    // in reduce mode); user ops: host_user_reduce.
    return worker().run([=]() -> int {
        if (op.opidx == O_NULL) return host_user_reduce(c, sendbuf, recvbuf, count, dt, op, root);
        return do_allreduce(c, sendbuf, recvbuf, count, dt, op, root, nbc);
    });
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
    const int p = c->size, me = c->rank;
    const Img m = img_of(dt, count);
    const size_t bytes = m.bytes;
    std::vector<char> mine(bytes), all((size_t)p * bytes);
    int rc = img_load(m, sendbuf == MPI_IN_PLACE ? recvbuf : sendbuf, mine.data());
    if (rc == MPI_SUCCESS) rc = c->tp->allgather(mine.data(), bytes, all.data());
    if (rc != MPI_SUCCESS) return rc;
    auto call = [&](const char* in, char* io) { img_call(op, dt, m, count, in - m.lo, io - m.lo); };
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
    return img_store(m, count, res[me].data() - m.lo, recvbuf);
}

int combine2(int opidx, Kind k, const char* inout_src, const char* in, char* out, size_t n, hipStream_t s,
             char* out2 = nullptr)
{
    TreeSpec t;
    t.P = 2;
    t.src[0] = inout_src;
    t.src[2] = in;
    if (out2) {                          // the same result stored twice
        t.extra[0] = out2;
        t.nextra = 1;
    }
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
    // GPU-synchronised when the vector fits half an IN sub-slot (count, type,
    // p and the environment decide: the same on every rank)
    const size_t Qh = (sub_len(chunk_bytes(), p) / 2) & ~(size_t)255;
    const bool flags = p >= 2 && p <= 32 && tp->has_done() && bytes <= Qh && bytes <= two_step_max(tp);
    Windows w;
    if ((rc = get_windows(tp, &w, flags)) != MPI_SUCCESS) return rc;
    // Each step's partial is PUSHED into the consumer's IN window (an xGMI
    // remote write) and combined there from local HBM; two alternating halves
    // of IN: a peer writes step i+2's half only after the barrier of step i+1,
    // which this rank reaches after finishing its reads of step i.
    size_t ce = w.C / 2 / esz;
    ce -= ce % 16;
    if (ce == 0) { set_error("scan: window too small"); return MPI_ERR_INTERN; }
    const size_t bstride = (bytes + 255) & ~(size_t)255;
    char* partial = dev_scratch(4 * bstride + 256);
    if (!partial) { set_error("scan: scratch allocation failed"); return MPI_ERR_NO_MEM; }
    char* res = partial + bstride;
    char* src_stage = res + bstride;     // host operands the kernels cannot address
    char* dst_stage = src_stage + bstride;
    BufInfo bs = classify(src), bd = classify(recvbuf);
    PinHold pins;                        // host buffers: device aliases for the call
    pins.sync_before_release(s);
    alias_host_operands(pins, true, src, bytes, &bs, recvbuf, bytes, &bd);
    const char* srcv = bs.place == Place::Device ? static_cast<const char*>(bs.dev) : src;
    void* dstv = bd.place == Place::Device ? bd.dev : recvbuf;
    bool have = !exclusive;
    if (flags) {
        // Every step on the stream, one host sync: step i = one k_push_wait
        // (my partial -> IN(me ^ mask) half, sub-slot me, flag (seq << 6) | i;
        // one workgroup waits for the partial I consume), then the combines.
        // Halves alternate and are reused as in the two-step allreduce.
        // Launches are kept to the minimum (each costs a few us on its own GPU
        // and tens of us when ranks share one): step 0 reads the send buffer
        // in place; while partial and result hold the same value (inclusive
        // scan until this rank first folds a higher rank's partial) one
        // combine stores both; the last step stores the result straight into
        // recvbuf and drops the partial nobody reads again.
        const size_t half = (size_t)tp->rd_parity * Qh;
        const unsigned long long seq = ++tp->rd_seq;
        int* err_host = nullptr;
        int* err_dev = wait_err_word(&err_host);
        unsigned* counter = tp->push_counter();
        if (!err_dev || !counter) { set_error("scan: flag word allocation failed"); return MPI_ERR_NO_MEM; }
        *err_host = 0;
        // the kernels read the send buffer and write recvbuf in place when
        // they are device memory (or pinned aliases); host memory is staged
        const bool src_dev = bs.place == Place::Device, dst_dev = bd.place == Place::Device;
        if (!src_dev) {
            rc = copy_async(src_stage, src, bytes, s);
            srcv = src_stage;
        }
        const char* cur_p = srcv;                       // current partial
        const char* cur_r = exclusive ? nullptr : srcv; // current result (have)
        bool same = !exclusive;                         // partial and result hold one value
        char* outv = dst_dev ? static_cast<char*>(dstv) : dst_stage;
        int step = 0;
        for (int mask = 1; mask < p && rc == MPI_SUCCESS; mask <<= 1, ++step) {
            const int dst = me ^ mask;
            const bool last = (mask << 1) >= p;
            const bool use = dst < p && !(last && me < dst);
            const bool feeds = dst < p && !(last && dst < me);
            const unsigned long long v = (seq << 6) | (unsigned long long)step;
            if (feeds && seq > 2) rc = tp->wait_done(dst, seq - 2);
            if (rc != MPI_SUCCESS) break;
            const void* ps = cur_p;
            void* pd = feeds ? static_cast<void*>(w.sub(dst, me) + half) : nullptr;
            size_t pn = bytes;
            unsigned long long* pf = feeds ? w.flags(dst) + kScanFlags + me : nullptr;
            hipError_t e = launch_push_wait(&ps, &pd, &pn, feeds ? 1 : 0, &pf, feeds ? 1 : 0, v,
                                            counter + kCountWords,
                                            use ? w.flags(me) + kScanFlags + dst : w.flags(me), use ? 1 : 0, -1,
                                            err_dev, s);
            if (e != hipSuccess) { rc = hip_fail(e, "scan push"); break; }
            if (!use) continue;
            const char* tmp = w.sub(me, dst) + half;
            // the partial is read again only by a later step's push or combine
            char* np = last ? nullptr : partial;
            if (me > dst) {
                char* nr = last ? outv : res;
                if (have && same) {                      // one combine, stored twice
                    rc = np ? combine2(op.opidx, k, cur_p, tmp, np, count, s, nr)
                            : combine2(op.opidx, k, cur_r, tmp, nr, count, s);
                } else {
                    if (np) rc = combine2(op.opidx, k, cur_p, tmp, np, count, s);
                    if (rc == MPI_SUCCESS)
                        rc = have ? combine2(op.opidx, k, cur_r, tmp, nr, count, s) : copy_async(nr, tmp, bytes, s);
                    same = false;
                }
                cur_p = np;
                cur_r = nr;
                have = true;
            } else {                                     // never the last step (use)
                rc = combine2(op.opidx, k, cur_p, tmp, partial, count, s);
                cur_p = partial;
                same = false;
            }
        }
        // a result that never left the send buffer or the scratch (rank 0 of an
        // inclusive scan, or a last step that did not fold) goes to recvbuf
        if (rc == MPI_SUCCESS && have && (cur_r != outv || !dst_dev))
            rc = copy_async(dst_dev ? static_cast<void*>(outv) : recvbuf, cur_r, bytes, s);
        const int rs = sync_stream(s, "scan");
        if (rc == MPI_SUCCESS) rc = rs;
        if (rc == MPI_SUCCESS && __atomic_load_n(err_host, __ATOMIC_ACQUIRE))
            rc = flag_timeout("scan", me, __atomic_load_n(err_host, __ATOMIC_ACQUIRE), seq, false);
        tp->post_done(seq);
        tp->rd_parity ^= 1;
        tp->window_open = true;
        return rc;
    }
    rc = copy_async(partial, srcv, bytes, s);
    if (rc == MPI_SUCCESS && !exclusive) rc = copy_async(res, srcv, bytes, s);
    if (rc == MPI_SUCCESS) rc = sync_stream(s, "scan init");
    int slot = 0;
    for (int mask = 1; mask < p && rc == MPI_SUCCESS; mask <<= 1) {
        const int dst = me ^ mask;
        const bool last = (mask << 1) >= p;
        const bool use = dst < p && !(last && me < dst);     // this rank consumes dst's partial
        const bool feeds = dst < p && !(last && dst < me);   // dst consumes this rank's partial
        for (size_t o = 0; o < count && rc == MPI_SUCCESS; o += ce, slot ^= 1) {
            const size_t len = std::min(ce, count - o);
            if (feeds) {
                char* stage = w.in(dst) + (size_t)slot * (w.C / 2);
                rc = copy_async(stage, partial + o * esz, len * esz, s);   // partial at step start
                if (rc == MPI_SUCCESS) rc = sync_stream(s, "scan push");
            }
            if (rc == MPI_SUCCESS) rc = tp->barrier();
            if (rc != MPI_SUCCESS || !use) continue;
            const char* tmp = w.in(me) + (size_t)slot * (w.C / 2);
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
        rc = copy_async(dstv, res, bytes, s);
        if (rc == MPI_SUCCESS) rc = sync_stream(s, "scan result");
    }
    return rc;
}

}  // namespace

int engine_scan(Comm* c, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
                const OpRef& op, bool exclusive)
{
    return worker().run([=] { return do_scan(c, sendbuf, recvbuf, count, dt, op, exclusive); });
}

// ===========================================================================
// one-sided accumulate: target-side application at the fence
// ===========================================================================
namespace {

// target = target (op) origin for `d.count` elements at taddr; the reference's
// do_accumulate_op / MPIDI_Win_local_accumulate (packethandling.cpp:2917-2960,
// win.cpp:1405-1450).  An (op, type) pair outside the op's table reaches
// MPIR_Op_<op>, which only sets op_errno (op.cpp:1791) and leaves the target
// unchanged; nothing reports it, so neither do we.
int rma_combine(const RmaDesc& d, const char* payload, char* taddr, hipStream_t s)
{
    if (d.opidx == O_NOOP || d.count == 0) return MPI_SUCCESS;
    const size_t bytes = (size_t)d.count * (size_t)d.usize;
    if (d.opidx == O_REPLACE) return copy_async(taddr, payload, bytes, s);
    if (op_check_dtype(d.opidx, d.dt) != MPI_SUCCESS) return MPI_SUCCESS;
    const Kind k = type_info(d.dt)->kind;
    if (classify(taddr).place == Place::Device && classify(payload).place == Place::Device) {
        // the streaming combine in place on the target (payloads written by
        // peers sit in uncached window memory, so plain loads see them)
        const hipError_t e = launch_combine(d.opidx, k, payload, taddr, (size_t)d.count, s, LaunchCfg());
        return e == hipSuccess ? MPI_SUCCESS : hip_fail(e, "rma combine");
    }
    int rc = sync_stream(s, "rma");
    return rc == MPI_SUCCESS ? reduce_local_any(d.opidx, k, payload, taddr, (size_t)d.count) : rc;
}

// compare-and-swap of one element (bitwise compare, win.cpp:1909-1990)
int rma_cas(const RmaDesc& d, const char* origin, const char* cmp, char* taddr, char* fetch, hipStream_t s)
{
    const size_t esz = (size_t)d.usize;
    int rc = sync_stream(s, "rma cas");
    char old[16], c[16];
    if (rc == MPI_SUCCESS) rc = copy_any(old, taddr, esz);
    if (rc == MPI_SUCCESS) rc = copy_any(c, cmp, esz);
    if (rc == MPI_SUCCESS && fetch) rc = copy_any(fetch, old, esz);
    if (rc == MPI_SUCCESS && memcmp(old, c, esz) == 0) rc = copy_any(taddr, origin, esz);
    return rc;
}

// A derived target datatype: the gfx950 pack / unpack / accumulate kernels
// walk its layout at taddr (the reference's segment walk of
// packethandling.cpp:2969-3004).  Window memory the GPU cannot address
// (pageable host memory) is staged through HBM around the kernel.
int rma_apply_typed(const RmaDesc& d, const Dtype* T, const char* payload, char* taddr, char* fetch,
                    hipStream_t s)
{
    int64_t lo, hi;
    dt_span(T, d.count, &lo, &hi);
    const BufInfo bi = classify(taddr + lo);
    char* tdev = taddr;
    void* stage = nullptr;
    int rc = MPI_SUCCESS;
    if (bi.place == Place::Device) {
        tdev = static_cast<char*>(bi.dev) - lo;
    } else {
        const size_t span = (size_t)(hi - lo);
        const uintptr_t mis = (uintptr_t)(taddr + lo) & 15;
        if (hipMalloc(&stage, span + 16) != hipSuccess) { set_error("rma staging allocation"); return MPI_ERR_NO_MEM; }
        tdev = static_cast<char*>(stage) + mis - lo;
        rc = copy_async(tdev + lo, taddr + lo, span, s);
    }
    // payload / fetch live in engine windows or device temporaries (device memory)
    if (rc == MPI_SUCCESS && (d.kind == RMA_GET || d.kind == RMA_GACC))
        rc = dt_pack_dev(T, d.count, tdev, fetch, s);
    if (rc == MPI_SUCCESS && (d.kind == RMA_PUT || ((d.kind == RMA_ACC || d.kind == RMA_GACC))))
        rc = d.kind == RMA_PUT ? dt_unpack_dev(T, d.count, payload, tdev, s)
                               : dt_acc_dev(d.opidx, T, d.count, payload, tdev, s);
    if (stage) {
        if (rc == MPI_SUCCESS && d.kind != RMA_GET) rc = copy_async(taddr + lo, tdev + lo, (size_t)(hi - lo), s);
        const int rs = sync_stream(s, "rma typed stage");
        (void)hipFree(stage);
        if (rc == MPI_SUCCESS) rc = rs;
    }
    return rc;
}

// One operation on window memory `taddr` of this rank.  `fetch` receives the
// target's previous contents (GET / GACC / CAS).  T: derived target type or null.
int rma_apply(const RmaDesc& d, const Dtype* T, const char* payload, const char* cmp, char* taddr, char* fetch,
              hipStream_t s)
{
    if (T) return rma_apply_typed(d, T, payload, taddr, fetch, s);
    const size_t bytes = (size_t)d.count * (size_t)d.usize;
    switch (d.kind) {
    case RMA_PUT: return copy_async(taddr, payload, bytes, s);
    case RMA_GET: return copy_async(fetch, taddr, bytes, s);
    case RMA_ACC: return rma_combine(d, payload, taddr, s);
    case RMA_GACC: {
        int rc = copy_async(fetch, taddr, bytes, s);
        return rc == MPI_SUCCESS ? rma_combine(d, payload, taddr, s) : rc;
    }
    case RMA_CAS: return rma_cas(d, payload, cmp, taddr, fetch, s);
    default: set_error("rma: bad operation kind %d", d.kind); return MPI_ERR_INTERN;
    }
}

bool rma_in_bounds(const RmaDesc& d, int64_t winsize)
{
    if (d.tdisp < 0 || d.count < 0 || d.usize <= 0) return false;
    if (d.layout >= 0) return d.tdisp + d.span_lo >= 0 && d.span_hi <= winsize - d.tdisp;
    const int64_t n = (d.kind == RMA_CAS) ? 1 : d.count;
    if (n > (INT64_MAX - d.tdisp) / d.usize) return false;
    return d.tdisp + n * d.usize <= winsize;
}

hipStream_t rma_self_stream()
{
    static hipStream_t s = [] {
        hipStream_t t = nullptr;
        (void)hipStreamCreateWithFlags(&t, hipStreamNonBlocking);
        return t;
    }();
    return s;
}

// A slice [lo, hi) of one queued operation, staged through the engine
// windows: payload in the target's IN area, fetched bytes in the origin's OUT.
struct RmaPiece {
    int origin;
    int64_t idx;           // index in the origin's queue
    int64_t lo, hi;        // unit range
    size_t in_off, out_off;
    size_t in_b, out_b;
};

struct TypeCache {         // standalone target layouts rebuilt at this rank
    std::map<std::pair<int, int64_t>, Dtype*> m;
    ~TypeCache()
    {
        for (auto& kv : m) dtype_delete(kv.second);
    }
};

int do_rma_fence(RmaWin* win)
{
    Comm* c = win->comm;
    Transport* tp = c->tp;
    const int p = c->size, me = c->rank;
    int rc = ensure_device();
    if (rc != MPI_SUCCESS) return rc;
    // 1. every origin's queue and derived-layout blob, on every rank
    int64_t mine[2] = {(int64_t)win->q.size(), (int64_t)win->blob.size()};
    std::vector<int64_t> ns((size_t)p * 2);
    if ((rc = tp->allgather(mine, sizeof(mine), ns.data())) != MPI_SUCCESS) return rc;
    int64_t maxn = 0, maxb = 0;
    for (int r = 0; r < p; ++r) {
        maxn = std::max(maxn, ns[(size_t)r * 2]);
        maxb = std::max(maxb, ns[(size_t)r * 2 + 1]);
    }
    trace("rma fence: %lld local ops, max %lld", (long long)mine[0], (long long)maxn);
    if (maxn == 0) return tp->barrier();
    std::vector<RmaDesc> padded((size_t)maxn), all((size_t)p * (size_t)maxn);
    std::copy(win->q.begin(), win->q.end(), padded.begin());
    if ((rc = tp->allgather(padded.data(), (size_t)maxn * sizeof(RmaDesc), all.data())) != MPI_SUCCESS) return rc;
    std::vector<int64_t> blobs;
    if (maxb > 0) {
        std::vector<int64_t> pb((size_t)maxb, 0);
        std::copy(win->blob.begin(), win->blob.end(), pb.begin());
        blobs.resize((size_t)p * (size_t)maxb);
        if ((rc = tp->allgather(pb.data(), (size_t)maxb * sizeof(int64_t), blobs.data())) != MPI_SUCCESS) return rc;
    }
    TypeCache types;
    auto target_type = [&](int o, int64_t i, const RmaDesc& d) -> const Dtype* {
        if (d.layout < 0) return nullptr;
        auto key = std::make_pair(o, i);
        auto it = types.m.find(key);
        if (it != types.m.end()) return it->second;
        Dtype* t = dtype_from_blob(blobs.data() + (size_t)o * maxb + d.layout, ns[(size_t)o * 2 + 1] - d.layout);
        types.m[key] = t;
        return t;
    };
    Windows w;
    if ((rc = get_windows(tp, &w)) != MPI_SUCCESS) return rc;
    const size_t C = w.C;
    // 2. cut operations into pieces and pack them into rounds; a target
    //    applies its pieces in (origin, issue) order, round after round
    std::vector<std::vector<RmaPiece>> rounds(1);
    std::vector<size_t> in_used((size_t)p, 0), out_used((size_t)p, 0);
    int my_err = MPI_SUCCESS;
    for (int o = 0; o < p; ++o) {
        for (int64_t i = 0; i < ns[(size_t)o * 2]; ++i) {
            const RmaDesc& d = all[(size_t)o * maxn + i];
            const size_t esz = (size_t)d.usize;
            if (!rma_in_bounds(d, win->sizes[(size_t)d.target])) {
                // packethandling.cpp:1339-1383: **requestrmaoutofbounds
                if (o == me) {
                    my_err = MPI_ERR_REQUEST;
                    set_error("RMA operation outside the target window (target %d, disp %lld)", d.target,
                              (long long)d.tdisp);
                }
                continue;
            }
            if (esz > C / 2) {
                if (o == me) {
                    my_err = MPI_ERR_TYPE;
                    set_error("RMA target datatype of %zu bytes exceeds the staging window", esz);
                }
                continue;
            }
            const int64_t n = (d.kind == RMA_CAS) ? 1 : d.count;
            const bool sends = d.kind == RMA_PUT || d.kind == RMA_CAS || ((d.kind == RMA_ACC || d.kind == RMA_GACC) && d.opidx != O_NOOP);
            const bool fetches = d.kind == RMA_GET || d.kind == RMA_GACC || d.kind == RMA_CAS;
            int64_t per = (int64_t)(C / esz / 2) & ~(int64_t)15;
            if (per <= 0) per = 1;
            for (int64_t lo = 0; lo < n; lo += per) {
                const int64_t hi = std::min(n, lo + per);
                RmaPiece pc;
                pc.origin = o;
                pc.idx = i;
                pc.lo = lo;
                pc.hi = hi;
                pc.in_b = sends ? (size_t)(hi - lo) * esz * (d.kind == RMA_CAS ? 2 : 1) : 0;
                pc.out_b = fetches ? (size_t)(hi - lo) * esz : 0;
                const size_t ia = (pc.in_b + 255) & ~(size_t)255, oa = (pc.out_b + 255) & ~(size_t)255;
                if (in_used[(size_t)d.target] + ia > C || out_used[(size_t)o] + oa > C) {
                    rounds.emplace_back();
                    std::fill(in_used.begin(), in_used.end(), 0);
                    std::fill(out_used.begin(), out_used.end(), 0);
                }
                pc.in_off = in_used[(size_t)d.target];
                pc.out_off = out_used[(size_t)o];
                in_used[(size_t)d.target] += ia;
                out_used[(size_t)o] += oa;
                rounds.back().push_back(pc);
            }
        }
    }
    hipStream_t s = tp->stream();
    for (const auto& round : rounds) {
        // a. origins write payloads into the targets' IN areas (xGMI writes)
        for (const RmaPiece& pc : round) {
            if (pc.origin != me || !pc.in_b) continue;
            const RmaDesc& d = all[(size_t)me * maxn + pc.idx];
            const RmaLocal& l = win->ql[(size_t)pc.idx];
            const size_t esz = (size_t)d.usize;
            char* dst = w.in(d.target) + pc.in_off;
            if (d.kind == RMA_CAS) {
                rc = copy_async(dst, l.origin, esz, s);
                if (rc == MPI_SUCCESS) rc = copy_async(dst + esz, l.compare, esz, s);
            } else {
                rc = copy_async(dst, static_cast<const char*>(l.origin) + pc.lo * esz, pc.in_b, s);
            }
            if (rc != MPI_SUCCESS) return rc;
        }
        if ((rc = sync_stream(s, "rma payload")) != MPI_SUCCESS) return rc;
        if ((rc = tp->barrier()) != MPI_SUCCESS) return rc;
        // b. targets apply in (origin, issue) order; fetched bytes go to the
        //    origin's OUT area
        for (const RmaPiece& pc : round) {
            const RmaDesc& d0 = all[(size_t)pc.origin * maxn + pc.idx];
            if (d0.target != me) continue;
            const Dtype* T = target_type(pc.origin, pc.idx, d0);
            if (d0.layout >= 0 && !T) { set_error("rma: malformed datatype layout"); return MPI_ERR_INTERN; }
            RmaDesc d = d0;
            d.count = (d0.kind == RMA_CAS) ? 1 : pc.hi - pc.lo;
            char* taddr = win->base + d0.tdisp + pc.lo * d0.uext;
            const char* payload = w.in(me) + pc.in_off;
            char* fetch = pc.out_b ? w.out(pc.origin) + pc.out_off : nullptr;
            rc = rma_apply(d, T, payload, payload + d0.usize, taddr, fetch, s);
            if (rc != MPI_SUCCESS) return rc;
        }
        if ((rc = sync_stream(s, "rma apply")) != MPI_SUCCESS) return rc;
        if ((rc = tp->barrier()) != MPI_SUCCESS) return rc;
        // c. origins deliver fetched values to their result buffers
        for (const RmaPiece& pc : round) {
            if (pc.origin != me || !pc.out_b) continue;
            const RmaDesc& d = all[(size_t)me * maxn + pc.idx];
            rc = copy_async(static_cast<char*>(win->ql[(size_t)pc.idx].result) + pc.lo * d.usize,
                            w.out(me) + pc.out_off, pc.out_b, s);
            if (rc != MPI_SUCCESS) return rc;
        }
        if ((rc = sync_stream(s, "rma deliver")) != MPI_SUCCESS) return rc;
    }
    for (RmaLocal& l : win->ql) {
        const int r2 = rma_local_complete(l);
        if (rc == MPI_SUCCESS) rc = r2;
    }
    win->q.clear();
    win->ql.clear();
    win->blob.clear();
    trace("rma fence: %zu rounds done", rounds.size());
    return rc != MPI_SUCCESS ? rc : my_err;
}

}  // namespace

int rma_local_complete(RmaLocal& l)
{
    int rc = MPI_SUCCESS;
    if (l.tmp_result) {
        // a derived result type: the fetched bytes arrived packed
        Dtype* t = dtype_lookup(l.result_dt);
        rc = t ? dt_unpack_any(t, l.result_count, l.tmp_result, l.result_user) : MPI_ERR_TYPE;
        (void)hipFree(l.tmp_result);
        l.tmp_result = nullptr;
        MPI_Datatype h = l.result_dt;
        if (dtype_is_derived(h)) dtype_free(&h);     // the reference taken at issue
    }
    if (l.tmp_origin) {
        (void)hipFree(l.tmp_origin);
        l.tmp_origin = nullptr;
    }
    return rc;
}

int rma_apply_self(RmaWin* w, const RmaDesc& d, const RmaLocal& l, const Dtype* T)
{
    int rc = ensure_device();
    if (rc != MPI_SUCCESS) return rc;
    if (!rma_in_bounds(d, w->size)) {
        set_error("RMA operation outside the window (disp %lld)", (long long)d.tdisp);
        return MPI_ERR_REQUEST;
    }
    hipStream_t s = rma_self_stream();
    rc = rma_apply(d, T, static_cast<const char*>(l.origin), static_cast<const char*>(l.compare),
                   w->base + d.tdisp, static_cast<char*>(l.result), s);
    return rc == MPI_SUCCESS ? sync_stream(s, "rma self") : rc;
}

namespace {
int passive_init(RmaWin* w);   // below, with the passive-target machinery
}

int engine_rma_create(RmaWin* w)
{
    Comm* c = w->comm;
    const int p = c->size;
    w->sizes.assign((size_t)p, 0);
    w->disp_units.assign((size_t)p, 1);
    if (p == 1 || !c->tp) {
        w->sizes[0] = w->size;
        w->disp_units[0] = w->disp_unit;
        return MPI_SUCCESS;
    }
    return worker().run([w, c, p] {
        int64_t mine[2] = {w->size, (int64_t)w->disp_unit};
        std::vector<int64_t> all((size_t)p * 2);
        int rc = c->tp->allgather(mine, sizeof(mine), all.data());
        for (int r = 0; rc == MPI_SUCCESS && r < p; ++r) {
            w->sizes[(size_t)r] = all[(size_t)r * 2];
            w->disp_units[(size_t)r] = (int)all[(size_t)r * 2 + 1];
        }
        // passive target: mailbox + this rank's service thread (collective)
        if (rc == MPI_SUCCESS) rc = passive_init(w);
        return rc;
    });
}

// ---- passive target (MPI_Win_lock / unlock / flush) -----------------------------
struct PassiveReq {               // one request of a mailbox slot (plain data)
    RmaDesc d;                    // this piece: count, tdisp of its first unit
    int64_t blob_n = 0;           // int64 words of target layout at the payload slot's start
    int64_t payload_off = 0;      // payload bytes in the slot (after the layout)
    int32_t has_fetch = 0;
    int32_t pad_ = 0;
};
struct PassiveSlot {              // mailbox slot (target t, origin o)
    std::atomic<uint32_t> req;    // origin: +1 after writing r
    std::atomic<uint32_t> done;   // target: = req once applied
    std::atomic<int32_t> rc;
    int32_t pad_;
    PassiveReq r;
};

struct PassiveState {
    RmaWin* w = nullptr;
    int p = 1, me = 0;
    Windows win;                          // the communicator's engine windows
    void* shm = nullptr;
    size_t shm_bytes = 0;
    std::atomic<uint32_t>* door = nullptr;    // per target: doorbell of its service thread
    std::atomic<int32_t>* lock = nullptr;     // per target: 0 free, > 0 readers, -1 writer
    PassiveSlot* slots = nullptr;             // [target * p + origin]
    std::atomic<uint32_t>* post = nullptr;    // [target * p + origin]: exposure epochs posted
    std::atomic<uint32_t>* cmpl = nullptr;    // [target * p + origin]: access epochs completed
    std::thread th;
    std::atomic<bool> stop{false};
    std::mutex apply_mu;                      // service thread vs. self-target applies
    hipStream_t os = nullptr;                 // origin-side copies
};

namespace {

void futex_wake_all(void* addr)
{
    syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), FUTEX_WAKE, INT32_MAX, nullptr, nullptr, 0);
}

void futex_wait_ms(void* addr, uint32_t val, long ms)
{
    struct timespec ts = {ms / 1000, (ms % 1000) * 1000000};
    syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), FUTEX_WAIT, val, &ts, nullptr, 0);
}

// A shared-memory segment of `bytes` mapped by every rank (collective).
int shm_collective(Transport* tp, size_t bytes, void** out)
{
    *out = nullptr;
    static std::atomic<int> serial{0};
    char name[64] = {0};
    if (tp->rank == 0)
        snprintf(name, sizeof(name), "/msx_win_%d_%d_%ld", (int)getpid(), serial.fetch_add(1),
                 (long)(now_s() * 1e6) % 1000000000L);
    // rank 0 creates and sizes the segment BEFORE anyone learns its name
    int fd = -1;
    if (tp->rank == 0) {
        fd = shm_open(name, O_CREAT | O_RDWR, 0600);
        if (fd < 0 || ftruncate(fd, (off_t)bytes) != 0) name[0] = 0;
    }
    std::vector<char> all((size_t)tp->size * sizeof(name));
    int rc = tp->allgather(name, sizeof(name), all.data());
    if (rc != MPI_SUCCESS) {
        if (fd >= 0) close(fd);
        return rc;
    }
    memcpy(name, all.data(), sizeof(name));
    int ok = name[0] != 0;
    if (ok && tp->rank != 0) fd = shm_open(name, O_RDWR, 0600);
    std::vector<int> oks((size_t)tp->size);
    void* m = MAP_FAILED;
    if (ok && fd >= 0) m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (fd >= 0) close(fd);
    int mine = m != MAP_FAILED ? 1 : 0;
    rc = tp->allgather(&mine, sizeof(int), oks.data());
    if (tp->rank == 0) shm_unlink(name);
    bool all_ok = rc == MPI_SUCCESS && mine;
    for (int v : oks) all_ok = all_ok && v;
    if (!all_ok) {
        if (m != MAP_FAILED) munmap(m, bytes);
        set_error("passive target: shared-memory mailbox unavailable");
        return rc != MPI_SUCCESS ? rc : MPI_ERR_NO_MEM;
    }
    *out = m;                     // zero-filled by ftruncate
    return MPI_SUCCESS;
}

// Target side: apply one request of origin o to this rank's window memory.
int passive_apply(PassiveState* ps, int o, const PassiveReq& r, hipStream_t s)
{
    std::lock_guard<std::mutex> g(ps->apply_mu);
    const RmaDesc& d = r.d;
    const char* slot = ps->win.rma_in(ps->me, o);
    Dtype* T = nullptr;
    if (r.blob_n > 0) {
        std::vector<int64_t> blob((size_t)r.blob_n);
        int rc = copy_any(blob.data(), slot, (size_t)r.blob_n * sizeof(int64_t));
        if (rc != MPI_SUCCESS) return rc;
        T = dtype_from_blob(blob.data(), r.blob_n);
        if (!T) { set_error("passive target: malformed datatype layout"); return MPI_ERR_INTERN; }
    }
    const char* payload = slot + r.payload_off;
    char* fetch = r.has_fetch ? ps->win.rma_fetch(o, ps->me) : nullptr;
    int rc = rma_apply(d, T, payload, payload + d.usize, ps->w->base + d.tdisp, fetch, s);
    const int rs = sync_stream(s, "passive apply");
    if (T) dtype_delete(T);
    return rc != MPI_SUCCESS ? rc : rs;
}

// The service thread of one window: applies every origin's requests in
// arrival order, whatever this rank's own thread is doing.
void passive_serve(PassiveState* ps)
{
    (void)ensure_device();
    hipStream_t s = nullptr;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    std::atomic<uint32_t>& door = ps->door[ps->me];
    for (;;) {
        const uint32_t d0 = door.load(std::memory_order_acquire);
        bool any = false;
        for (int o = 0; o < ps->p; ++o) {
            PassiveSlot& sl = ps->slots[(size_t)ps->me * ps->p + o];
            const uint32_t q = sl.req.load(std::memory_order_acquire);
            if (q == sl.done.load(std::memory_order_relaxed)) continue;
            any = true;
            const int rc = s ? passive_apply(ps, o, sl.r, s) : MPI_ERR_OTHER;
            sl.rc.store(rc, std::memory_order_relaxed);
            sl.done.store(q, std::memory_order_release);
            futex_wake_all(&sl.done);
        }
        if (any) continue;
        if (ps->stop.load(std::memory_order_acquire)) break;
        futex_wait_ms(&door, d0, 100);
    }
    if (s) (void)hipStreamDestroy(s);
}

int passive_lock(PassiveState* ps, int t, int mode)
{
    std::atomic<int32_t>& lk = ps->lock[t];
    const double t_end = now_s() + 600.0;
    for (int spin = 0;; ++spin) {
        int32_t v = lk.load(std::memory_order_acquire);
        if (mode == MPI_LOCK_EXCLUSIVE ? v == 0 : v >= 0) {
            const int32_t nv = mode == MPI_LOCK_EXCLUSIVE ? -1 : v + 1;
            if (lk.compare_exchange_weak(v, nv, std::memory_order_acq_rel)) return MPI_SUCCESS;
            continue;
        }
        if (now_s() > t_end) {
            set_error("MPI_Win_lock: lock of rank %d not granted within 600 s", t);
            return MPI_ERR_OTHER;
        }
        if (spin < 1000) sched_yield();
        else futex_wait_ms(&lk, (uint32_t)v, 10);
    }
}

void passive_unlock(PassiveState* ps, int t, int mode)
{
    std::atomic<int32_t>& lk = ps->lock[t];
    if (mode == MPI_LOCK_EXCLUSIVE) lk.store(0, std::memory_order_release);
    else lk.fetch_sub(1, std::memory_order_acq_rel);
    futex_wake_all(&lk);
}

// Origin side: ship one queued operation to target t piece by piece (payload
// slot capacity) and wait for each piece to be applied.
int passive_ship(PassiveState* ps, int t, const RmaDesc& d0, const RmaLocal& l, const int64_t* blob, int64_t blob_n)
{
    const size_t S = ps->win.rma_slot();
    const size_t blob_b = ((size_t)blob_n * sizeof(int64_t) + 255) & ~(size_t)255;
    const bool sends = d0.kind == RMA_PUT || d0.kind == RMA_CAS ||
                       ((d0.kind == RMA_ACC || d0.kind == RMA_GACC) && d0.opidx != O_NOOP);
    const bool fetches = d0.kind == RMA_GET || d0.kind == RMA_GACC || d0.kind == RMA_CAS;
    const size_t esz = (size_t)d0.usize;
    const size_t unit_in = sends ? esz * (d0.kind == RMA_CAS ? 2 : 1) : 0;
    if (blob_b + unit_in > S || esz > S) {
        set_error("passive target: a %zu-byte unit does not fit the %zu-byte staging slot", esz, S);
        return MPI_ERR_TYPE;
    }
    const int64_t n = d0.kind == RMA_CAS ? 1 : d0.count;
    int64_t per = unit_in ? (int64_t)((S - blob_b) / unit_in) : n;
    if (fetches) per = std::min<int64_t>(per, (int64_t)(S / esz));
    per = std::max<int64_t>(per, 1);
    char* dst = ps->win.rma_in(t, ps->me);
    PassiveSlot& sl = ps->slots[(size_t)t * ps->p + ps->me];
    int rc = MPI_SUCCESS;
    for (int64_t lo = 0; lo < n && rc == MPI_SUCCESS; lo += per) {
        const int64_t hi = std::min(n, lo + per);
        if (blob_n) rc = copy_async(dst, blob, (size_t)blob_n * sizeof(int64_t), ps->os);
        if (rc == MPI_SUCCESS && sends) {
            if (d0.kind == RMA_CAS) {
                rc = copy_async(dst + blob_b, l.origin, esz, ps->os);
                if (rc == MPI_SUCCESS) rc = copy_async(dst + blob_b + esz, l.compare, esz, ps->os);
            } else {
                rc = copy_async(dst + blob_b, static_cast<const char*>(l.origin) + lo * esz, (size_t)(hi - lo) * esz,
                                ps->os);
            }
        }
        if (rc == MPI_SUCCESS) rc = sync_stream(ps->os, "passive payload");
        if (rc != MPI_SUCCESS) break;
        PassiveReq& r = sl.r;
        r.d = d0;
        r.d.count = d0.kind == RMA_CAS ? 1 : hi - lo;
        r.d.tdisp = d0.tdisp + lo * d0.uext;
        r.d.layout = blob_n ? 0 : -1;
        r.blob_n = blob_n;
        r.payload_off = (int64_t)blob_b;
        r.has_fetch = fetches ? 1 : 0;
        const uint32_t q = sl.req.load(std::memory_order_relaxed) + 1;
        sl.req.store(q, std::memory_order_release);
        ps->door[t].fetch_add(1, std::memory_order_acq_rel);
        futex_wake_all(&ps->door[t]);
        const double t_end = now_s() + 600.0;
        for (int spin = 0;; ++spin) {
            const uint32_t dn = sl.done.load(std::memory_order_acquire);
            if (dn == q) break;
            if (now_s() > t_end) {
                set_error("passive target: rank %d did not apply within 600 s", t);
                return MPI_ERR_OTHER;
            }
            if (spin < 2000) sched_yield();
            else futex_wait_ms(&sl.done, dn, 10);
        }
        rc = sl.rc.load(std::memory_order_relaxed);
        if (rc == MPI_SUCCESS && fetches)
            rc = copy_async(static_cast<char*>(l.result) + lo * esz, ps->win.rma_fetch(ps->me, t),
                            (size_t)(hi - lo) * esz, ps->os);
        if (rc == MPI_SUCCESS && fetches) rc = sync_stream(ps->os, "passive fetch");
    }
    return rc;
}

int passive_init(RmaWin* w)
{
    Comm* c = w->comm;
    auto* ps = new PassiveState();
    ps->w = w;
    ps->p = c->size;
    ps->me = c->rank;
    int rc = get_windows(c->tp, &ps->win);
    if (rc == MPI_SUCCESS) rc = c->tp->rma_window(ps->win.rbase, &ps->win.rbytes);
    const size_t p = (size_t)ps->p;
    const size_t hdr = ((p * sizeof(std::atomic<uint32_t>) + p * sizeof(std::atomic<int32_t>)) + 63) & ~(size_t)63;
    const size_t pscw = (2 * p * p * sizeof(std::atomic<uint32_t>) + 63) & ~(size_t)63;
    ps->shm_bytes = hdr + p * p * sizeof(PassiveSlot) + pscw;
    if (rc == MPI_SUCCESS) rc = shm_collective(c->tp, ps->shm_bytes, &ps->shm);
    if (rc == MPI_SUCCESS && hipStreamCreateWithFlags(&ps->os, hipStreamNonBlocking) != hipSuccess) {
        set_error("passive target: stream creation failed");
        rc = MPI_ERR_OTHER;
    }
    if (rc != MPI_SUCCESS) {
        if (ps->shm) munmap(ps->shm, ps->shm_bytes);
        delete ps;
        return rc;
    }
    char* base = static_cast<char*>(ps->shm);
    ps->door = reinterpret_cast<std::atomic<uint32_t>*>(base);
    ps->lock = reinterpret_cast<std::atomic<int32_t>*>(base + p * sizeof(std::atomic<uint32_t>));
    ps->slots = reinterpret_cast<PassiveSlot*>(base + hdr);
    ps->post = reinterpret_cast<std::atomic<uint32_t>*>(base + hdr + p * p * sizeof(PassiveSlot));
    ps->cmpl = ps->post + p * p;
    ps->th = std::thread(passive_serve, ps);
    w->passive = ps;
    return MPI_SUCCESS;
}

}  // namespace

int engine_rma_free(RmaWin* w)
{
    PassiveState* ps = w->passive;
    if (!ps) return MPI_SUCCESS;
    ps->stop.store(true, std::memory_order_release);
    ps->door[ps->me].fetch_add(1, std::memory_order_acq_rel);
    futex_wake_all(&ps->door[ps->me]);
    if (ps->th.joinable()) ps->th.join();
    if (ps->os) (void)hipStreamDestroy(ps->os);
    munmap(ps->shm, ps->shm_bytes);
    delete ps;
    w->passive = nullptr;
    return MPI_SUCCESS;
}

int engine_rma_lock(RmaWin* w, int target, int mode)
{
    return w->passive ? passive_lock(w->passive, target, mode) : MPI_SUCCESS;
}

int engine_rma_unlock_target(RmaWin* w, int target)
{
    if (w->passive && w->lock_held[(size_t)target]) passive_unlock(w->passive, target, w->lock_mode[(size_t)target]);
    return MPI_SUCCESS;
}

int engine_rma_flush(RmaWin* w, int target)
{
    PassiveState* ps = w->passive;
    if (!ps) return MPI_SUCCESS;                    // one rank: every operation was applied at its call
    int rc = MPI_SUCCESS;
    bool pending = false;
    for (const RmaDesc& d : w->q) pending = pending || d.target == target;
    if (!pending) return MPI_SUCCESS;
    if (w->lock_mode[(size_t)target] && !w->lock_held[(size_t)target]) {
        // the lazily requested lock is granted now
        if ((rc = passive_lock(ps, target, w->lock_mode[(size_t)target])) != MPI_SUCCESS) return rc;
        w->lock_held[(size_t)target] = 1;
    }
    std::vector<RmaDesc> keep_q;
    std::vector<RmaLocal> keep_l;
    for (size_t i = 0; i < w->q.size(); ++i) {
        const RmaDesc& d = w->q[i];
        if (d.target != target) {
            keep_q.push_back(d);
            keep_l.push_back(w->ql[i]);
            continue;
        }
        int r2 = MPI_SUCCESS;
        if (!rma_in_bounds(d, w->sizes[(size_t)target])) {
            set_error("RMA operation outside the target window (target %d, disp %lld)", target, (long long)d.tdisp);
            r2 = MPI_ERR_REQUEST;                   // packethandling.cpp:1339-1383
        } else if (rc == MPI_SUCCESS) {
            const int64_t* blob = d.layout >= 0 ? w->blob.data() + d.layout : nullptr;
            const int64_t blob_n = d.layout >= 0 ? (int64_t)w->blob.size() - d.layout : 0;
            r2 = passive_ship(ps, target, d, w->ql[i], blob, blob_n);
        }
        const int r3 = rma_local_complete(w->ql[i]);
        if (rc == MPI_SUCCESS) rc = r2 != MPI_SUCCESS ? r2 : r3;
    }
    w->q.swap(keep_q);
    w->ql.swap(keep_l);
    if (w->q.empty()) w->blob.clear();
    return rc;
}

namespace {
// Block until *word >= want (shared memory, another process bumps it).
int wait_counter(std::atomic<uint32_t>* word, uint32_t want, const char* what, int peer)
{
    const double t_end = now_s() + 600.0;
    for (int spin = 0;; ++spin) {
        const uint32_t v = word->load(std::memory_order_acquire);
        if ((int32_t)(v - want) >= 0) return MPI_SUCCESS;
        if (now_s() > t_end) {
            set_error("%s: rank %d did not synchronise within 600 s", what, peer);
            return MPI_ERR_OTHER;
        }
        if (spin < 2000) sched_yield();
        else futex_wait_ms(word, v, 10);
    }
}
}  // namespace

int engine_rma_post(RmaWin* w)
{
    PassiveState* ps = w->passive;
    for (int o : w->exposure_origins) {
        w->posts[(size_t)o] += 1;
        if (!ps) continue;                         // one rank: nothing to tell
        std::atomic<uint32_t>& word = ps->post[(size_t)ps->me * ps->p + o];
        word.fetch_add(1, std::memory_order_acq_rel);
        futex_wake_all(&word);
    }
    return MPI_SUCCESS;
}

int engine_rma_complete(RmaWin* w)
{
    PassiveState* ps = w->passive;
    int rc = MPI_SUCCESS;
    for (int t : w->access_targets) {
        w->starts[(size_t)t] += 1;
        if (!ps) continue;                         // one rank: every operation was applied at its call
        // MPID_Win_complete (win.cpp:3859-3874): the target's post first
        if (t != ps->me && !(w->access_assert & MPI_MODE_NOCHECK)) {
            const int r2 = wait_counter(&ps->post[(size_t)t * ps->p + ps->me], w->starts[(size_t)t],
                                        "MPI_Win_complete", t);
            if (rc == MPI_SUCCESS) rc = r2;
            if (r2 != MPI_SUCCESS) continue;
        }
        const int r3 = engine_rma_flush(w, t);     // applied at the target before it is counted
        if (rc == MPI_SUCCESS) rc = r3;
        std::atomic<uint32_t>& word = ps->cmpl[(size_t)t * ps->p + ps->me];
        word.fetch_add(1, std::memory_order_acq_rel);
        futex_wake_all(&word);
    }
    return rc;
}

int engine_rma_wait(RmaWin* w, bool block, int* flag)
{
    PassiveState* ps = w->passive;
    *flag = 1;
    if (!ps) return MPI_SUCCESS;
    for (int o : w->exposure_origins) {
        std::atomic<uint32_t>* word = &ps->cmpl[(size_t)ps->me * ps->p + o];
        const uint32_t want = w->posts[(size_t)o];
        if (!block) {
            if ((int32_t)(word->load(std::memory_order_acquire) - want) < 0) { *flag = 0; return MPI_SUCCESS; }
            continue;
        }
        const int rc = wait_counter(word, want, "MPI_Win_wait", o);
        if (rc != MPI_SUCCESS) return rc;
    }
    return MPI_SUCCESS;
}

void engine_rma_self_guard(RmaWin* w, bool enter)
{
    if (!w->passive) return;
    if (enter) w->passive->apply_mu.lock();
    else w->passive->apply_mu.unlock();
}

int engine_rma_fence(RmaWin* w)
{
    if (w->comm->size == 1 || !w->comm->tp) return MPI_SUCCESS;   // all operations were local
    return worker().run([w] { return do_rma_fence(w); });
}

int engine_stats(double* out, int n, int reset)
{
    return worker().submit([out, n, reset]() -> int {
        const double v[8] = {g_stats.t[0], g_stats.t[1], g_stats.t[2], g_stats.t[3], g_stats.t[4],
                             (double)g_stats.chunks, (double)g_stats.calls, (double)g_stats.flag_calls};
        for (int i = 0; i < n && i < 8; ++i) out[i] = v[i];
        if (reset) g_stats = EngineStats();
        return 8;
    }).get();
}

// Link roofline probe: every rank writes `bytes` from its own window into
// its sub-slot of EVERY peer's IN area at once (the scatter step's traffic
// pattern: p-1 concurrent remote-write streams per GPU, all xGMI links busy),
// `reps` times.  *seconds = median time of one all-peer write of *used
// bytes per peer (the request capped at one window sub-slot).  The result is
// the measured per-GPU outbound bandwidth that the collectives' busBW is
// judged against (confirm the link figures by measurement).
int engine_peer_write_probe(Comm* c, size_t bytes, int reps, double* seconds, int64_t* used)
{
    *used = 0;
    if (!c->tp || c->size == 1) {
        *seconds = 0;
        return MPI_SUCCESS;
    }
    int rc = ensure_device();
    if (rc != MPI_SUCCESS) return rc;
    return worker().submit([c, bytes, reps, seconds, used]() -> int {
        Transport* tp = c->tp;
        const int p = c->size, me = c->rank;
        Windows w;
        int rc = get_windows(tp, &w);
        if (rc != MPI_SUCCESS) return rc;
        const size_t n = std::min(bytes, w.Q) & ~(size_t)255;
        *used = (int64_t)n;
        hipStream_t s = tp->stream();
        std::vector<double> ts;
        for (int it = 0; it <= reps && rc == MPI_SUCCESS; ++it) {
            Segs sg;
            for (int r = 0; r < p; ++r)
                if (r != me) sg.add(w.out(me), w.sub(r, me), n);
            rc = tp->barrier();
            const double t0 = now_s();
            if (rc == MPI_SUCCESS) rc = sg.run(s, "peer write probe");
            if (rc == MPI_SUCCESS) rc = sync_stream(s, "peer write probe");
            const double t1 = now_s();
            if (rc == MPI_SUCCESS) rc = tp->barrier();
            if (it > 0) ts.push_back(t1 - t0);       // the first is a warm-up
        }
        if (rc == MPI_SUCCESS && !ts.empty()) {
            std::sort(ts.begin(), ts.end());
            *seconds = ts[ts.size() / 2];
        }
        return rc;
    }).get();
}

const char* engine_transport_name(Transport* tp)
{
    if (!tp) return "self";
    if (!worker().submit([tp]() -> int { return g_rccl_comms.count(tp) ? 1 : 0; }).get()) return "ipc";
    return rccl_native_requested() ? "rccl_native" : "rccl";
}

std::shared_future<int> engine_async(std::function<int()> fn) { return worker().submit(std::move(fn)); }

// ===========================================================================
// intercommunicators (api/mpi_comm.cpp:1482-1610 MPI_Intercomm_create,
// :1653-1830 MPI_Intercomm_merge; reduce.cpp:778-863 MPIR_Reduce_inter,
// 1821-1990 MPIR_Reduce_scatter[_block]_inter, 4109-4175 MPIR_Allreduce_inter)
// ===========================================================================
namespace {

// ---- world mailbox: one inbox per process in node shared memory ----------
constexpr size_t kMailBytes = 16384;
struct MailSlot {
    std::atomic<uint32_t> state;      // 0 empty, 1 being written, 2 full
    int32_t src, tag, len, pad_;
    char data[kMailBytes];
};
struct Mailbox {
    MailSlot* slots = nullptr;
    int me = 0, p = 0;
    std::deque<std::tuple<int, int, std::vector<char>>> pending;   // received, not yet matched
};
Mailbox g_mail;

// move a message waiting in my inbox (if any) to the pending list
void mail_drain()
{
    MailSlot& s = g_mail.slots[g_mail.me];
    if (s.state.load(std::memory_order_acquire) != 2) return;
    g_mail.pending.emplace_back(s.src, s.tag, std::vector<char>(s.data, s.data + s.len));
    s.state.store(0, std::memory_order_release);
    futex_wake_all(&s.state);
}

int mail_send(int dst, int tag, const void* data, size_t n)
{
    if (!g_mail.slots || dst < 0 || dst >= g_mail.p) { set_error("mailbox: no process %d", dst); return MPI_ERR_INTERN; }
    if (n > kMailBytes) { set_error("mailbox: %zu-byte message exceeds %zu", n, kMailBytes); return MPI_ERR_INTERN; }
    MailSlot& s = g_mail.slots[dst];
    const double t_end = now_s() + 600.0;
    for (int spin = 0;; ++spin) {
        uint32_t z = 0;
        if (s.state.compare_exchange_strong(z, 1, std::memory_order_acq_rel)) {
            s.src = g_mail.me;
            s.tag = tag;
            s.len = (int32_t)n;
            memcpy(s.data, data, n);
            s.state.store(2, std::memory_order_release);
            futex_wake_all(&s.state);
            return MPI_SUCCESS;
        }
        mail_drain();                 // a peer sending to me must never wait for my send
        if (now_s() > t_end) { set_error("mailbox: process %d's inbox stayed full for 600 s", dst); return MPI_ERR_OTHER; }
        if (spin < 1000) sched_yield();
        else futex_wait_ms(&s.state, z, 10);
    }
}

int mail_recv(int src, int tag, std::vector<char>* out)
{
    const double t_end = now_s() + 600.0;
    for (int spin = 0;; ++spin) {
        mail_drain();
        for (auto it = g_mail.pending.begin(); it != g_mail.pending.end(); ++it)
            if (std::get<0>(*it) == src && std::get<1>(*it) == tag) {
                *out = std::move(std::get<2>(*it));
                g_mail.pending.erase(it);
                return MPI_SUCCESS;
            }
        if (now_s() > t_end) { set_error("mailbox: no message from process %d (tag %d) in 600 s", src, tag); return MPI_ERR_OTHER; }
        if (spin < 1000) sched_yield();
        else futex_wait_ms(&g_mail.slots[g_mail.me].state, 0, 10);
    }
}

// every member of c gets root's v (same length everywhere)
int group_bcast(Comm* c, std::vector<int32_t>& v, int root)
{
    if (c->size == 1 || v.empty()) return MPI_SUCCESS;
    std::vector<int32_t> all(v.size() * (size_t)c->size);
    const int rc = c->tp->allgather(v.data(), v.size() * sizeof(int32_t), all.data());
    if (rc == MPI_SUCCESS) std::copy(all.begin() + (long)root * (long)v.size(), all.begin() + (long)(root + 1) * (long)v.size(), v.begin());
    return rc;
}

// A private duplicate of intracommunicator c (same group, own transport).
int dup_intra(Comm* c, Comm** out)
{
    auto* n = new Comm();
    n->rank = c->rank;
    n->size = c->size;
    n->lpid = c->lpid;
    n->errhandler = c->errhandler;
    if (c->tp) {
        int nr = 0, ns = 0;
        std::vector<int> members;
        const int rc = transport_split(c->tp, 0, c->rank, &nr, &ns, &n->tp, &members);
        if (rc != MPI_SUCCESS) { delete n; return rc; }
    }
    *out = n;
    return MPI_SUCCESS;
}

void free_intra(Comm* c)
{
    if (!c) return;
    if (c->tp) {
        (void)c->tp->barrier();                         // no peer still uses its windows
        transport_destroy(c->tp);
    }
    delete c;
}

// Separate scratch of the intercommunicator paths (the intra schedules they
// call use dev_scratch themselves).
char* inter_scratch(size_t bytes)
{
    static char* p = nullptr;
    static size_t cap = 0;
    if (bytes > cap) {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        if (hipMalloc(&p, bytes) != hipSuccess) { p = nullptr; return nullptr; }
        cap = bytes;
    }
    return p;
}

// ---- point-to-point between the groups over the union's windows ----------
// Rank `from` moves `bytes` to rank `to` of the union communicator u through
// sub-slot `from` of the receiver's IN area, in chunks of half a sub-slot
// alternating between the halves.  Chunk c of the pair (both sides count the
// pair's chunks in the same order: MPI orders collectives) carries data flag
// c (slot kP2PData + from at the receiver); the receiver acknowledges with
// flag c (slot kP2PAck + to at the sender) after copying it out, and the
// sender waits for ack c - 2 before reusing a half.  All waits are single
// GPU workgroups on the union's stream; the caller syncs the stream.
constexpr size_t kP2PData = 1024, kP2PAck = 1536;

int p2p_chunks(Comm* u, size_t bytes, size_t* chunk)
{
    const size_t Qh = (sub_len(chunk_bytes(), u->size) / 2) & ~(size_t)255;
    *chunk = Qh;
    return (int)((bytes + Qh - 1) / Qh);
}

int p2p_send(Comm* u, int to, const char* src, size_t bytes, int* err_dev)
{
    Windows w;
    int rc = get_windows(u->tp, &w, true);
    if (rc != MPI_SUCCESS) return rc;
    hipStream_t s = u->tp->stream();
    unsigned* counter = u->tp->push_counter();
    if (!counter) { set_error("p2p: counter allocation failed"); return MPI_ERR_NO_MEM; }
    size_t Qh;
    const int n = p2p_chunks(u, bytes, &Qh);
    uint64_t& sent = u->tp->p2p_sent(to);
    for (int i = 0; i < n && rc == MPI_SUCCESS; ++i) {
        const uint64_t c = ++sent;
        const size_t off = (size_t)i * Qh, len = std::min(Qh, bytes - off);
        if (c > 2) {                                  // the half's previous chunk was copied out
            hipError_t e = launch_push_wait(nullptr, nullptr, nullptr, 0, nullptr, 0, c - 2, nullptr,
                                            w.flags(u->rank) + kP2PAck + to, 1, -1, err_dev, s);
            if (e != hipSuccess) { rc = hip_fail(e, "p2p ack wait"); break; }
        }
        const void* ps = src + off;
        void* pd = w.sub(to, u->rank) + (size_t)(c & 1) * Qh;
        unsigned long long* pf = w.flags(to) + kP2PData + u->rank;
        hipError_t e = launch_push_wait(&ps, &pd, &len, 1, &pf, 1, c, counter + kCountWords,
                                        w.flags(u->rank), 0, -1, err_dev, s);
        if (e != hipSuccess) rc = hip_fail(e, "p2p push");
    }
    return rc;
}

int p2p_recv(Comm* u, int from, char* dst, size_t bytes, int* err_dev)
{
    Windows w;
    int rc = get_windows(u->tp, &w, true);
    if (rc != MPI_SUCCESS) return rc;
    hipStream_t s = u->tp->stream();
    size_t Qh;
    const int n = p2p_chunks(u, bytes, &Qh);
    uint64_t& got = u->tp->p2p_recv(from);
    for (int i = 0; i < n && rc == MPI_SUCCESS; ++i) {
        const uint64_t c = ++got;
        const size_t off = (size_t)i * Qh, len = std::min(Qh, bytes - off);
        hipError_t e = launch_push_wait(nullptr, nullptr, nullptr, 0, nullptr, 0, c, nullptr,
                                        w.flags(u->rank) + kP2PData + from, 1, -1, err_dev, s);
        if (e != hipSuccess) { rc = hip_fail(e, "p2p data wait"); break; }
        rc = copy_async(dst + off, w.sub(u->rank, from) + (size_t)(c & 1) * Qh, len, s);
        unsigned long long* ack = w.flags(from) + kP2PAck + u->rank;
        if (rc == MPI_SUCCESS) {
            e = launch_post_flags(&ack, 1, c, s);
            if (e != hipSuccess) rc = hip_fail(e, "p2p ack");
        }
    }
    return rc;
}

int p2p_finish(Comm* u, int rc, int* err_host)
{
    const int rs = sync_stream(u->tp->stream(), "intercommunicator transfer");
    if (rc == MPI_SUCCESS) rc = rs;
    if (rc == MPI_SUCCESS && __atomic_load_n(err_host, __ATOMIC_ACQUIRE))
        rc = flag_timeout("intercomm_p2p", u->rank, __atomic_load_n(err_host, __ATOMIC_ACQUIRE), 0, false);
    return rc;
}

// The union's windows are mapped collectively (every member allocates and
// imports), but a transfer between the groups involves only its two ends.  So
// every member maps them while the whole union is present: when the
// intercommunicator is created or duplicated.  Without a GPU there is nothing
// to map (and no reduction can run).
int map_union(Comm* u)
{
    if (device_count_noinit() <= 0) return MPI_SUCCESS;
    int rc = ensure_device();
    if (rc != MPI_SUCCESS) return rc;
    Windows w;
    return get_windows(u->tp, &w, true);
}

// union rank of rank r of the local (mine = true) or remote group
int urank_of(const Comm* ic, bool mine, int r)
{
    const bool low = mine ? ic->is_low : !ic->is_low;
    const int nlow = ic->is_low ? ic->size : (int)ic->remote_lpid.size();
    return low ? r : nlow + r;
}

// ---- intracommunicator broadcast / scatterv through the windows -----------
// (the local steps of the reference's inter algorithms: MPIR_Bcast_intra,
// scatterv from rank 0).  Root writes block r into rank r's IN sub-slot
// `root` (peer pointers), barrier, receivers copy out, barrier; chunked by
// the sub-slot.  Buffers may be host or device memory.
int do_scatterv(Comm* c, int root, const char* src, const std::vector<size_t>& off, const std::vector<size_t>& len,
                char* dst)
{
    if (c->size == 1) return len[0] ? copy_any(dst, src + off[0], len[0]) : MPI_SUCCESS;
    Windows w;
    int rc = get_windows(c->tp, &w);
    if (rc != MPI_SUCCESS) return rc;
    hipStream_t s = c->tp->stream();
    size_t maxlen = 0;
    for (size_t l : len) maxlen = std::max(maxlen, l);
    for (size_t o = 0; o < maxlen && rc == MPI_SUCCESS; o += w.Q) {
        if (c->rank == root)
            for (int r = 0; r < c->size && rc == MPI_SUCCESS; ++r) {
                if (o >= len[(size_t)r]) continue;
                const size_t n = std::min(w.Q, len[(size_t)r] - o);
                rc = r == root ? copy_async(dst + o, src + off[(size_t)r] + o, n, s)
                               : copy_async(w.sub(r, root), src + off[(size_t)r] + o, n, s);
            }
        if (rc == MPI_SUCCESS) rc = sync_stream(s, "scatter push");
        if (rc == MPI_SUCCESS) rc = c->tp->barrier();
        const size_t mine = len[(size_t)c->rank];
        if (rc == MPI_SUCCESS && c->rank != root && o < mine) {
            rc = copy_async(dst + o, w.sub(c->rank, root), std::min(w.Q, mine - o), s);
            if (rc == MPI_SUCCESS) rc = sync_stream(s, "scatter collect");
        }
        if (rc == MPI_SUCCESS) rc = c->tp->barrier();
    }
    return rc;
}

int do_bcast(Comm* c, int root, char* buf, size_t bytes)
{
    std::vector<size_t> off((size_t)c->size, 0), len((size_t)c->size, bytes);
    return do_scatterv(c, root, buf, off, len, buf);
}

// the intracommunicator reduce of one group to its rank 0 (reference order:
// MPIR_Reduce_intra on inter.local_comm)
int local_reduce0(Comm* lc, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt, const OpRef& op)
{
    if (lc->size == 1) return local_copy(sendbuf, recvbuf, count, dt);
    if (op.opidx == O_NULL) return host_user_reduce(lc, sendbuf, recvbuf, count, dt, op, 0);
    return do_allreduce(lc, sendbuf, recvbuf, count, dt, op, 0);
}

// bytes a transfer of count elements of dt moves (packed for a derived type)
size_t wire_bytes(MPI_Datatype dt, size_t count)
{
    return dtype_is_derived(dt) ? (size_t)dtype_lookup(dt)->size * count : (size_t)type_size(dt) * count;
}

// MPIR_Reduce_inter: the remote group reduces to its rank 0, which sends to root
int do_inter_reduce(Comm* ic, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt, const OpRef& op,
                    int root)
{
    if (root == MPI_PROC_NULL || count == 0) return MPI_SUCCESS;
    int rc = ensure_device();
    if (rc != MPI_SUCCESS) return rc;
    Comm* u = ic->uni;
    const bool derived = dtype_is_derived(dt);
    const size_t wb = wire_bytes(dt, count);
    int* err_host = nullptr;
    int* err_dev = wait_err_word(&err_host);
    if (!err_dev) { set_error("intercommunicator: flag word allocation failed"); return MPI_ERR_NO_MEM; }
    *err_host = 0;
    if (root == MPI_ROOT) {
        // receive the remote group's result from its rank 0
        char* land = static_cast<char*>(recvbuf);
        if (derived) {
            land = inter_scratch(wb);
            if (!land) { set_error("intercommunicator: scratch allocation failed"); return MPI_ERR_NO_MEM; }
        }
        rc = p2p_finish(u, p2p_recv(u, urank_of(ic, false, 0), land, wb, err_dev), err_host);
        if (rc == MPI_SUCCESS && derived) rc = dt_copy_any(land, (int64_t)wb, MPI_BYTE, recvbuf, (int64_t)count, dt);
        return rc;
    }
    // my group sends: local reduce to rank 0 into a private buffer, then rank 0 -> root
    int64_t lo = 0, hi = (int64_t)wb;
    if (derived) dt_span(dtype_lookup(dt), (int64_t)count, &lo, &hi);
    const size_t span = (size_t)(hi - lo);
    char* tmp = nullptr;
    if (ic->rank == 0) {
        tmp = inter_scratch(span + (derived ? wb : 0) + 256);
        if (!tmp) { set_error("intercommunicator: scratch allocation failed"); return MPI_ERR_NO_MEM; }
    }
    rc = local_reduce0(ic->local, sendbuf, tmp ? tmp - lo : nullptr, count, dt, op);
    if (rc != MPI_SUCCESS || ic->rank != 0) return rc;
    const char* wire = tmp;
    if (derived) {                                    // pack the typed result
        char* packed = tmp + ((span + 255) & ~(size_t)255);
        rc = dt_copy_any(tmp - lo, (int64_t)count, dt, packed, (int64_t)wb, MPI_BYTE);
        wire = packed;
    }
    if (rc == MPI_SUCCESS) rc = p2p_finish(u, p2p_send(u, urank_of(ic, false, root), wire, wb, err_dev), err_host);
    return rc;
}

}  // namespace

int engine_mailbox_init(Transport* world, int rank, int size)
{
    if (size < 2 || !world) return MPI_SUCCESS;
    void* m = nullptr;
    int rc = shm_collective(world, (size_t)size * sizeof(MailSlot), &m);
    if (rc != MPI_SUCCESS) return rc;
    g_mail.slots = static_cast<MailSlot*>(m);
    g_mail.me = rank;
    g_mail.p = size;
    return MPI_SUCCESS;
}

int engine_intercomm_create(Comm* local, int leader, Comm* peer, int remote_leader, int tag, Comm** out)
{
    *out = nullptr;
    return worker().run([=]() -> int {
        // 1. rank 0 of each group opens a bootstrap socket; its group learns the port
        int lfd = -1;
        std::vector<int32_t> pv{0};
        if (local->rank == 0) {
            int pt = 0;
            lfd = listen_ephemeral(&pt);
            pv[0] = lfd >= 0 ? pt : -1;
        }
        int rc = group_bcast(local, pv, 0);
        const int32_t gport = pv[0];
        // 2. the leaders swap {leader process id, group port, group size, members}
        std::vector<int32_t> hdr{MPI_SUCCESS, 0, 0, 0}, rem;
        if (rc == MPI_SUCCESS && local->rank == leader) {
            std::vector<int32_t> msg{local->lpid[(size_t)leader], gport, local->size};
            msg.insert(msg.end(), local->lpid.begin(), local->lpid.end());
            const int rl = peer->lpid[(size_t)remote_leader];
            int r2 = mail_send(rl, tag, msg.data(), msg.size() * sizeof(int32_t));
            std::vector<char> got;
            if (r2 == MPI_SUCCESS) r2 = mail_recv(rl, tag, &got);
            if (r2 == MPI_SUCCESS && got.size() >= 3 * sizeof(int32_t)) {
                std::vector<int32_t> g(got.size() / sizeof(int32_t));
                memcpy(g.data(), got.data(), g.size() * sizeof(int32_t));
                hdr = {MPI_SUCCESS, g[0], g[1], g[2]};
                rem.assign(g.begin() + 3, g.end());
            } else {
                hdr[0] = r2 != MPI_SUCCESS ? r2 : MPI_ERR_INTERN;
            }
        }
        if (rc == MPI_SUCCESS) rc = group_bcast(local, hdr, leader);
        if (rc == MPI_SUCCESS && hdr[0] != MPI_SUCCESS) rc = hdr[0];
        if (rc == MPI_SUCCESS && (hdr[2] <= 0 || hdr[3] <= 0)) {
            set_error("MPI_Intercomm_create: the remote group did not publish its bootstrap socket");
            rc = MPI_ERR_OTHER;
        }
        if (rc == MPI_SUCCESS) {
            rem.resize((size_t)hdr[3]);
            rc = group_bcast(local, rem, leader);
        }
        if (rc != MPI_SUCCESS) {
            if (lfd >= 0) close(lfd);
            return rc;
        }
        // 3. both groups in one communicator, the group with the lower leader id first
        const bool low = local->lpid[(size_t)leader] < hdr[1];
        const int nr = hdr[3], nlow = low ? local->size : nr;
        const int usize = local->size + nr, urank = low ? local->rank : nlow + local->rank;
        if (!(low && local->rank == 0) && lfd >= 0) {
            close(lfd);
            lfd = -1;
        }
        auto* t = new IpcTransport();
        rc = t->init(urank, usize, low ? gport : hdr[2], lfd);
        if (rc != MPI_SUCCESS) {
            delete t;
            return rc;
        }
        auto* u = new Comm();
        u->rank = urank;
        u->size = usize;
        u->tp = t;
        u->lpid = low ? local->lpid : rem;
        const std::vector<int>& second = low ? rem : local->lpid;
        u->lpid.insert(u->lpid.end(), second.begin(), second.end());
        rc = map_union(u);
        if (rc != MPI_SUCCESS) {
            free_intra(u);
            return rc;
        }
        // 4. the intercommunicator's own local group
        Comm* lc = nullptr;
        rc = dup_intra(local, &lc);
        if (rc != MPI_SUCCESS) {
            free_intra(u);
            return rc;
        }
        auto* ic = new Comm();
        ic->inter = true;
        ic->rank = local->rank;
        ic->size = local->size;
        ic->lpid = local->lpid;
        ic->remote_lpid.assign(rem.begin(), rem.end());
        ic->is_low = low;
        ic->local = lc;
        ic->uni = u;
        ic->errhandler = local->errhandler;
        *out = ic;
        return MPI_SUCCESS;
    });
}

int engine_intercomm_merge(Comm* ic, int high, Comm** out)
{
    *out = nullptr;
    return worker().run([=]() -> int {
        // every union member's (high, process id of its group's rank 0)
        const int32_t mine[3] = {high ? 1 : 0, ic->lpid[0], ic->is_low ? 1 : 0};
        std::vector<int32_t> all((size_t)ic->uni->size * 3);
        int rc = ic->uni->tp->allgather(mine, sizeof(mine), all.data());
        if (rc != MPI_SUCCESS) return rc;
        int lsum = 0, rhigh = -1, r0 = -1;
        for (int r = 0; r < ic->uni->size; ++r) {
            const int32_t* e = &all[(size_t)r * 3];
            if ((e[2] != 0) == ic->is_low) lsum += e[0];
            else { rhigh = e[0]; r0 = e[1]; }
        }
        if (lsum != 0 && lsum != ic->size) {          // **notsame high
            set_error("MPI_Intercomm_merge: high differs within the local group");
            return MPI_ERR_ARG;
        }
        // equal high values: the group whose rank 0 has the lower process id first
        const int eff = (high ? 1 : 0) != rhigh ? (high ? 1 : 0) : (ic->lpid[0] > r0 ? 1 : 0);
        int nr = 0, ns = 0;
        Transport* t = nullptr;
        std::vector<int> members;
        rc = transport_split(ic->uni->tp, 0, (eff << 20) | ic->rank, &nr, &ns, &t, &members);
        if (rc != MPI_SUCCESS) return rc;
        auto* c = new Comm();
        c->rank = nr;
        c->size = ns;
        c->tp = t;
        for (int m : members) c->lpid.push_back(ic->uni->lpid[(size_t)m]);
        c->errhandler = ic->errhandler;
        *out = c;
        return MPI_SUCCESS;
    });
}

int engine_intercomm_dup(Comm* ic, Comm** out)
{
    *out = nullptr;
    return worker().run([=]() -> int {
        Comm *lc = nullptr, *u = nullptr;
        int rc = dup_intra(ic->local, &lc);
        if (rc == MPI_SUCCESS) rc = dup_intra(ic->uni, &u);
        if (rc == MPI_SUCCESS) rc = map_union(u);
        if (rc != MPI_SUCCESS) {
            free_intra(lc);
            free_intra(u);
            return rc;
        }
        auto* n = new Comm();
        n->inter = true;
        n->rank = ic->rank;
        n->size = ic->size;
        n->lpid = ic->lpid;
        n->remote_lpid = ic->remote_lpid;
        n->is_low = ic->is_low;
        n->local = lc;
        n->uni = u;
        n->errhandler = ic->errhandler;
        *out = n;
        return MPI_SUCCESS;
    });
}

int engine_inter_reduce(Comm* ic, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
                        const OpRef& op, int root)
{
    return worker().run([=] { return do_inter_reduce(ic, sendbuf, recvbuf, count, dt, op, root); });
}

// MPIR_Allreduce_inter (reduce.cpp:4109-4175): reduce from the high group to
// the low group's rank 0, then from the low group to the high group's rank 0,
// then a broadcast within each group
int engine_inter_allreduce(Comm* ic, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
                           const OpRef& op)
{
    return worker().run([=]() -> int {
        const int into_me = ic->rank == 0 ? MPI_ROOT : MPI_PROC_NULL;
        int rc = ic->is_low ? do_inter_reduce(ic, sendbuf, recvbuf, count, dt, op, into_me)
                            : do_inter_reduce(ic, sendbuf, recvbuf, count, dt, op, 0);
        if (rc == MPI_SUCCESS)
            rc = ic->is_low ? do_inter_reduce(ic, sendbuf, recvbuf, count, dt, op, 0)
                            : do_inter_reduce(ic, sendbuf, recvbuf, count, dt, op, into_me);
        if (rc != MPI_SUCCESS || ic->size == 1) return rc;
        if (!dtype_is_derived(dt)) return do_bcast(ic->local, 0, static_cast<char*>(recvbuf), wire_bytes(dt, count));
        // derived type: broadcast the packed result, unpack everywhere
        const size_t wb = wire_bytes(dt, count);
        char* packed = inter_scratch(wb + 256);
        if (!packed) { set_error("intercommunicator: scratch allocation failed"); return MPI_ERR_NO_MEM; }
        if (ic->rank == 0) rc = dt_copy_any(recvbuf, (int64_t)count, dt, packed, (int64_t)wb, MPI_BYTE);
        if (rc == MPI_SUCCESS) rc = do_bcast(ic->local, 0, packed, wb);
        if (rc == MPI_SUCCESS && ic->rank != 0) rc = dt_copy_any(packed, (int64_t)wb, MPI_BYTE, recvbuf, (int64_t)count, dt);
        return rc;
    });
}

// MPIR_Reduce_scatter_inter (reduce.cpp:1852-1990): the whole vector of
// total = sum(recvcounts) elements is reduced to rank 0 of each group (low
// group first), then scattered within the group
int engine_inter_reduce_scatter(Comm* ic, const void* sendbuf, void* recvbuf, const int* recvcounts,
                                MPI_Datatype dt, const OpRef& op)
{
    std::vector<int> counts(recvcounts, recvcounts + ic->size);
    return worker().run([=]() -> int {
        size_t total = 0;
        for (int c : counts) total += (size_t)c;
        if (total == 0) return MPI_SUCCESS;
        if (dtype_is_derived(dt)) {
            set_error("MPI_Reduce_scatter on an intercommunicator: derived datatypes are not supported");
            return MPI_ERR_TYPE;
        }
        const size_t esz = (size_t)type_size(dt);
        // rank 0's landing buffer for the remote group's reduction (device)
        char* tmp = nullptr;
        std::vector<char> keep;
        if (ic->rank == 0) {
            if (hipMalloc(&tmp, total * esz) != hipSuccess) { set_error("reduce_scatter: allocation failed"); return MPI_ERR_NO_MEM; }
        }
        const int into_me = ic->rank == 0 ? MPI_ROOT : MPI_PROC_NULL;
        int rc = ic->is_low ? do_inter_reduce(ic, sendbuf, tmp, total, dt, op, into_me)
                            : do_inter_reduce(ic, sendbuf, tmp, total, dt, op, 0);
        if (rc == MPI_SUCCESS)
            rc = ic->is_low ? do_inter_reduce(ic, sendbuf, tmp, total, dt, op, 0)
                            : do_inter_reduce(ic, sendbuf, tmp, total, dt, op, into_me);
        std::vector<size_t> off((size_t)ic->size), len((size_t)ic->size);
        size_t o = 0;
        for (int r = 0; r < ic->size; ++r) {
            off[(size_t)r] = o * esz;
            len[(size_t)r] = (size_t)counts[(size_t)r] * esz;
            o += (size_t)counts[(size_t)r];
        }
        if (rc == MPI_SUCCESS) rc = do_scatterv(ic->local, 0, tmp, off, len, static_cast<char*>(recvbuf));
        if (tmp) (void)hipFree(tmp);
        return rc;
    });
}

int engine_comm_split(Comm* parent, int color, int key, Comm** out)
{
    *out = nullptr;
    return worker().run([parent, color, key, out]() -> int {
        int nr = 0, ns = 1;
        Transport* t = nullptr;
        std::vector<int> members(1, 0);
        if (parent->tp) {
            const int rc = transport_split(parent->tp, color, key, &nr, &ns, &t, &members);
            if (rc != MPI_SUCCESS) return rc;
        } else if (color == MPI_UNDEFINED) {
            ns = 0;
        }
        if (ns == 0 || nr < 0) return MPI_SUCCESS;         // MPI_COMM_NULL
        Comm* c = new Comm();
        c->rank = nr;
        c->size = ns;
        for (int m : members)                               // process ids of the members
            c->lpid.push_back(m >= 0 && (size_t)m < parent->lpid.size() ? parent->lpid[(size_t)m] : -1);
        c->errhandler = parent->errhandler;                 // inherited from the parent
        c->tp = t;
        *out = c;
        return MPI_SUCCESS;
    });
}

int engine_comm_free(Comm* c)
{
    return worker().run([c]() -> int {
        int rc = MPI_SUCCESS;
        if (c->inter) {
            free_intra(c->local);
            free_intra(c->uni);
            c->local = c->uni = nullptr;
            return MPI_SUCCESS;
        }
        if (c->tp) {
            rc = c->tp->barrier();                          // no peer still uses its windows
            transport_destroy(c->tp);
            c->tp = nullptr;
        }
        return rc;
    });
}

}  // namespace msx
