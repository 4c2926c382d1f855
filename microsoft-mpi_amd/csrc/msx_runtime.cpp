// msx_runtime.cpp — device bring-up, buffer placement and the host-staged path.
//
// The reference combines in place on host memory (op.cpp:42-52).  On MI355X
// the combine always runs on the GPU; host-resident MPI buffers are streamed
// through HBM in chunks: H2D(in), H2D(inout) -> combine -> D2H(inout), with two
// HIP streams so chunk i+1's copies overlap chunk i's combine and copy-back;
// pinned host operands are read and written in place by the kernel (zero-copy),
// and pageable ones are pinned for the duration of the call and treated the
// same way (host mode 0, the default); msx_set_host_mode(2) stages pageable
// operands, msx_set_host_mode(1) stages every host operand.
// There is no CPU fallback: without a GPU the call fails with MPI_ERR_OTHER.
#include "msx_runtime.h"

#include <algorithm>
#include <atomic>
#include <dlfcn.h>
#include <mutex>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <thread>
#include <time.h>
#include <unistd.h>
#include <utility>
#include <vector>

namespace msx {

namespace {

thread_local char g_err[512];

struct DevState {
    std::once_flag once;
    int rc = MPI_ERR_OTHER;
    int device = -1;
    hipStream_t stream = nullptr;
    // host staging
    std::mutex stage_mu;
    size_t chunk = 64u << 20;       // bytes per staged chunk and operand
    void* stage_in[2] = {nullptr, nullptr};
    void* stage_io[2] = {nullptr, nullptr};
    hipStream_t stage_s[2] = {nullptr, nullptr};
    size_t stage_cap = 0;
    // small host operands (reduce_local_any)
    std::mutex bounce_mu;
    Bounce bounce_in, bounce_io;
};

DevState& ds()
{
    static DevState s;
    return s;
}

LaunchCfg g_cfg;

}  // namespace

void set_error(const char* fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

const char* last_error() { return g_err; }

// ---- stuck-phase reporter ----------------------------------------------------
// Host steps that can block on another process or GPU (IPC handle opens, the
// bootstrap exchange, stream synchronisations) run inside a PhaseScope.  A
// watchdog thread prints one line per step that exceeds MSX_STUCK_REPORT_S
// (default 30 s; the bench children are killed at 120-150 s):
//   MSX_STUCK {"rank":R,"phase":"...","peer":Q,"seconds":T}
// so a hang on a multi-GPU node names the rank, the step and the peer in the
// parent's JSON instead of surfacing as a bare timeout.
namespace {
constexpr int kPhaseSlots = 64;
// A slot is claimed (used 0 -> 1), filled, published (used = 2, gen bumped),
// and released (used = 0).  Every field is atomic and the watchdog re-reads
// `gen` after reading the fields, so a slot reclaimed meanwhile is skipped
// instead of reported with a mix of two steps' fields.
struct PhaseSlot {
    std::atomic<int> used{0};
    std::atomic<uint64_t> gen{0};
    std::atomic<const char*> phase{nullptr};
    std::atomic<int> peer{-1};
    std::atomic<double> t0{0.0};
    std::atomic<bool> sync{false};
    std::atomic<uint64_t> reported{0};    // gen of the step last reported
};
PhaseSlot g_phase[kPhaseSlots];
std::atomic<int> g_diag_rank{0};
std::once_flag g_watch_once;

double mono_s()
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

void watchdog()
{
    const char* e = getenv("MSX_STUCK_REPORT_S");
    const double limit = e ? atof(e) : 30.0;
    const char* es = getenv("MSX_STUCK_SYNC_S");
    const double limit_sync = es ? atof(es) : 300.0;
    for (;;) {
        usleep(250 * 1000);
        const double now = mono_s();
        for (PhaseSlot& sl : g_phase) {
            const uint64_t g = sl.gen.load(std::memory_order_acquire);
            if (sl.used.load(std::memory_order_acquire) != 2 || sl.reported.load(std::memory_order_relaxed) == g)
                continue;
            const char* ph = sl.phase.load(std::memory_order_relaxed);
            const int peer = sl.peer.load(std::memory_order_relaxed);
            const double t0 = sl.t0.load(std::memory_order_relaxed);
            const bool sync = sl.sync.load(std::memory_order_relaxed);
            if (sl.gen.load(std::memory_order_acquire) != g || sl.used.load(std::memory_order_acquire) != 2) continue;
            const double lim = sync ? limit_sync : limit;
            if (lim <= 0 || now - t0 < lim) continue;
            sl.reported.store(g, std::memory_order_relaxed);
            fprintf(stderr, "MSX_STUCK {\"rank\":%d,\"phase\":\"%s\",\"peer\":%d,\"seconds\":%.1f}\n",
                    g_diag_rank.load(), ph ? ph : "?", peer, now - t0);
            fflush(stderr);
        }
    }
}
}  // namespace

void set_diag_rank(int r) { g_diag_rank.store(r); }

PhaseScope::PhaseScope(const char* phase, int peer, bool sync)
{
    std::call_once(g_watch_once, [] { std::thread(watchdog).detach(); });
    for (int i = 0; i < kPhaseSlots; ++i) {
        int z = 0;
        if (g_phase[i].used.compare_exchange_strong(z, 1, std::memory_order_acq_rel)) {
            PhaseSlot& sl = g_phase[i];
            sl.phase.store(phase, std::memory_order_relaxed);
            sl.peer.store(peer, std::memory_order_relaxed);
            sl.t0.store(mono_s(), std::memory_order_relaxed);
            sl.sync.store(sync, std::memory_order_relaxed);
            sl.gen.fetch_add(1, std::memory_order_release);
            sl.used.store(2, std::memory_order_release);
            slot_ = i;
            return;
        }
    }
}

PhaseScope::~PhaseScope()
{
    if (slot_ >= 0) {
        g_phase[slot_].gen.fetch_add(1, std::memory_order_release);
        g_phase[slot_].used.store(0, std::memory_order_release);
    }
}

void trace(const char* fmt, ...)
{
    static const bool on = getenv("MSX_TRACE") && atoi(getenv("MSX_TRACE")) > 0;
    if (!on) return;
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    fprintf(stderr, "[msx %ld.%06ld pid %d] %s\n", (long)ts.tv_sec, ts.tv_nsec / 1000, (int)getpid(), buf);
    fflush(stderr);
}

int hip_fail(hipError_t e, const char* what)
{
    set_error("%s: %s", what, hipGetErrorString(e));
    return MPI_ERR_OTHER;
}

int device_count_noinit()
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int ensure_device()
{
    DevState& s = ds();
    std::call_once(s.once, [&s] {
        int n = 0;
        hipError_t e = hipGetDeviceCount(&n);
        if (e != hipSuccess || n == 0) {
            s.rc = MPI_ERR_OTHER;
            return;
        }
        // One rank per GPU: LOCAL_RANK (torchrun) or MSX_DEVICE picks the card.
        int dev = 0;
        if (const char* v = getenv("MSX_DEVICE")) dev = atoi(v);
        else if (const char* v = getenv("LOCAL_RANK")) dev = atoi(v);
        dev = ((dev % n) + n) % n;
        if (hipSetDevice(dev) != hipSuccess) return;
        if (hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess) return;
        s.device = dev;
        s.rc = MPI_SUCCESS;
    });
    if (s.rc != MPI_SUCCESS) {
        set_error("no usable MI355X (gfx950) device: the HIP reduction path cannot run "
                  "(hipGetDeviceCount reports %d)", device_count_noinit());
        return s.rc;
    }
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur != s.device) (void)hipSetDevice(s.device);
    return MPI_SUCCESS;
}

hipStream_t internal_stream() { return ds().stream; }

void set_staging_chunk(size_t bytes)
{
    DevState& s = ds();
    std::lock_guard<std::mutex> g(s.stage_mu);
    if (bytes < (1u << 16)) bytes = 1u << 16;
    s.chunk = bytes & ~(size_t)255;
}

// ---- call-scoped pinning of pageable operands ---------------------------------
// MPI_Reduce_local on pageable host buffers pins them for the duration of the
// call (hipHostRegister, page-rounded) and lets the kernel read and write them
// in place over PCIe, both directions at once.  Measured on MI355X
// (scripts/host_path_probe.cpp, 2 x 256 MiB fp32): 10.5 ms per call with the
// register/unregister included, vs 14.5 ms staging through HBM with the
// runtime's synchronous pageable copies.  Ranges pinned this way are listed
// here and classify() reports them as pageable, so no other thread of the
// library ever launches a kernel on an address this call is about to unpin
// (memory copies retain the runtime's pin object until they complete).
namespace {
struct TempPins {
    std::mutex mu;
    std::atomic<int> n{0};
    std::vector<std::pair<uintptr_t, uintptr_t>> ranges;   // [lo, hi)
    bool covers(uintptr_t p)
    {
        std::lock_guard<std::mutex> g(mu);
        for (auto& r : ranges)
            if (p >= r.first && p < r.second) return true;
        return false;
    }
};
TempPins& temp_pins()
{
    static TempPins t;
    return t;
}

uintptr_t page_down(uintptr_t a)
{
    static const uintptr_t ps = (uintptr_t)sysconf(_SC_PAGESIZE);
    return a & ~(ps - 1);
}
uintptr_t page_up(uintptr_t a)
{
    static const uintptr_t ps = (uintptr_t)sysconf(_SC_PAGESIZE);
    return (a + ps - 1) & ~(ps - 1);
}

// One call-scoped pin of the pages covering [a, b).  pin() returns false, with
// nothing pinned, when another call holds an overlapping pin or the driver
// refuses the range (a read-only mapping, pages the user registered already).
class CallPin {
public:
    CallPin() = default;
    CallPin(const CallPin&) = delete;
    CallPin& operator=(const CallPin&) = delete;
    ~CallPin() { release(); }

    bool pin(uintptr_t a, uintptr_t b, unsigned flags = hipHostRegisterMapped)
    {
        lo_ = page_down(a);
        hi_ = page_up(b);
        TempPins& t = temp_pins();
        {
            std::lock_guard<std::mutex> g(t.mu);
            for (auto& r : t.ranges)
                if (lo_ < r.second && r.first < hi_) {
                    lo_ = hi_ = 0;
                    return false;
                }
            t.ranges.push_back({lo_, hi_});
            t.n.fetch_add(1, std::memory_order_release);
        }
        listed_ = true;
        hipError_t e = hipHostRegister(reinterpret_cast<void*>(lo_), hi_ - lo_, flags);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            trace("call pin of %zu bytes refused: %s", (size_t)(hi_ - lo_), hipGetErrorString(e));
            unlist();
            return false;
        }
        void* d = nullptr;
        if (hipHostGetDevicePointer(&d, reinterpret_cast<void*>(lo_), 0) != hipSuccess || !d) {
            (void)hipGetLastError();
            (void)hipHostUnregister(reinterpret_cast<void*>(lo_));
            unlist();
            return false;
        }
        dev_ = static_cast<char*>(d);
        return true;
    }
    // device alias of host address p (inside the pinned range)
    void* dev(const void* p) const { return dev_ + ((uintptr_t)p - lo_); }
    // the same for the CURRENT device of a portable pin: the registered base's
    // alias there plus p's offset (interior pointers are never queried)
    void* dev_here(const void* p) const
    {
        void* d = nullptr;
        if (hipHostGetDevicePointer(&d, reinterpret_cast<void*>(lo_), 0) != hipSuccess || !d) {
            (void)hipGetLastError();
            return nullptr;
        }
        return static_cast<char*>(d) + ((uintptr_t)p - lo_);
    }
    bool covers(const void* p) const { return dev_ && (uintptr_t)p >= lo_ && (uintptr_t)p < hi_; }
    bool active() const { return dev_ != nullptr; }
    void release()
    {
        if (dev_) (void)hipHostUnregister(reinterpret_cast<void*>(lo_));
        dev_ = nullptr;
        unlist();
    }

private:
    void unlist()
    {
        if (!listed_) return;
        TempPins& t = temp_pins();
        std::lock_guard<std::mutex> g(t.mu);
        for (size_t i = 0; i < t.ranges.size(); ++i)
            if (t.ranges[i].first == lo_ && t.ranges[i].second == hi_) {
                t.ranges.erase(t.ranges.begin() + (long)i);
                break;
            }
        t.n.fetch_sub(1, std::memory_order_release);
        listed_ = false;
    }
    uintptr_t lo_ = 0, hi_ = 0;
    char* dev_ = nullptr;
    bool listed_ = false;
};

// Smallest call (bytes per operand) worth pinning; below it the staged copies
// are cheaper than two register/unregister round trips.  MSX_TEST_HOST_PIN_MIN.
size_t pin_min_bytes()
{
    static const size_t v = [] {
        size_t m = (size_t)1 << 20;
        if (const char* e = getenv("MSX_TEST_HOST_PIN_MIN")) m = (size_t)atoll(e);
        return m;
    }();
    return v;
}
}  // namespace

struct PinHold::Impl {
    CallPin pins[2];
    std::vector<hipStream_t> streams;
};

PinHold::PinHold() : impl_(new Impl) {}

PinHold::~PinHold()
{
    // work still queued on these streams may read or write the pinned pages
    if (impl_->pins[0].active() || impl_->pins[1].active())
        for (hipStream_t st : impl_->streams) (void)hipStreamSynchronize(st);
}

void PinHold::sync_before_release(hipStream_t s) { impl_->streams.push_back(s); }

bool alias_host_operands(PinHold& hold, bool pin_pageable, const void* a, size_t na, BufInfo* ia, const void* b,
                         size_t nb, BufInfo* ib)
{
    auto promote = [](BufInfo* x) {
        if (x && x->place == Place::Host && x->dev) {
            x->place = Place::Device;
            x->pinned_host = true;
        }
    };
    promote(ia);
    promote(ib);
    auto wants = [&](const void* p, size_t n, BufInfo* x) {
        return pin_pageable && p && x && n && n >= pin_min_bytes() && x->place == Place::Host && !x->dev;
    };
    const bool wa = wants(a, na, ia), wb = wants(b, nb, ib);
    CallPin* pins = hold.impl_->pins;
    auto set = [](BufInfo* x, void* d) {
        x->place = Place::Device;
        x->dev = d;
        x->pinned_host = true;
    };
    const uintptr_t a0 = (uintptr_t)a, a1 = a0 + na, b0 = (uintptr_t)b, b1 = b0 + nb;
    if (wa && wb && page_down(a0) < page_up(b1) && page_down(b0) < page_up(a1)) {
        if (pins[0].pin(std::min(a0, b0), std::max(a1, b1))) {   // operands share pages: one pin
            set(ia, pins[0].dev(a));
            set(ib, pins[0].dev(b));
        }
    } else {
        if (wa && pins[0].pin(a0, a1)) set(ia, pins[0].dev(a));
        if (wb && pins[1].pin(b0, b1)) set(ib, pins[1].dev(b));
    }
    return (!ia || ia->place == Place::Device) && (!ib || ib->place == Place::Device);
}

bool Bounce::get(size_t bytes)
{
    if (bytes <= cap && host) return true;
    if (host) (void)hipHostFree(host);
    host = dev = nullptr;
    cap = 0;
    size_t want = std::max(bytes, (size_t)64 << 10);
    void* h = nullptr;
    if (hipHostMalloc(&h, want, hipHostMallocMapped) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || !d) {
        (void)hipGetLastError();
        (void)hipHostFree(h);
        return false;
    }
    host = static_cast<char*>(h);
    dev = static_cast<char*>(d);
    cap = want;
    return true;
}

size_t bounce_max_bytes()
{
    static const size_t v = [] {
        size_t m = (size_t)256 << 10;
        if (const char* e = getenv("MSX_TEST_HOST_BOUNCE_MAX")) m = (size_t)atoll(e);
        return m;
    }();
    return v;
}

BufInfo classify(const void* p)
{
    BufInfo b;
    if (temp_pins().n.load(std::memory_order_acquire) > 0 && temp_pins().covers((uintptr_t)p)) return b;
    hipPointerAttribute_t a;
    hipError_t e = hipPointerGetAttributes(&a, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();   // pageable host memory is not an error
        return b;
    }
    switch (a.type) {
    case hipMemoryTypeDevice:
    case hipMemoryTypeManaged:
    case hipMemoryTypeArray:
        b.place = Place::Device;
        b.dev = a.devicePointer ? a.devicePointer : const_cast<void*>(p);
        b.device = a.device;
        break;
    case hipMemoryTypeHost:
        // pinned host memory: device-visible (PCIe); combined in place by the
        // kernel in host mode 0, staged through HBM in mode 1.
        b.place = Place::Host;
        b.dev = a.devicePointer;
        b.device = a.device;
        break;
    default:
        b.place = Place::Host;
        break;
    }
    return b;
}

// ---- page-locked staging ring for pageable transfers (xfer_sync) -------------
namespace {
constexpr size_t kXferChunk = (size_t)8 << 20;
struct XferRing {
    std::mutex mu;
    char* buf[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    bool ok = false;
    bool init()
    {
        if (ok) return true;
        for (int i = 0; i < 2; ++i) {
            if (!buf[i] && hipHostMalloc(reinterpret_cast<void**>(&buf[i]), kXferChunk, hipHostMallocPortable) != hipSuccess) {
                (void)hipGetLastError();
                buf[i] = nullptr;
                return false;
            }
            if (!ev[i] && hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess) {
                (void)hipGetLastError();
                ev[i] = nullptr;
                return false;
            }
        }
        ok = true;
        return true;
    }
};
XferRing& xring()
{
    static XferRing r;
    return r;
}
}  // namespace

bool host_pageable(const void* p)
{
    const BufInfo b = classify(p);
    return b.place == Place::Host && !b.dev;
}

int xfer_sync(void* dst, const void* src, size_t bytes, hipStream_t s)
{
    if (!bytes) return MPI_SUCCESS;
    const bool pd = host_pageable(dst), ps = host_pageable(src);
    hipError_t e = hipSuccess;
    if (pd && ps) {
        memcpy(dst, src, bytes);
        return MPI_SUCCESS;
    }
    if (!pd && !ps) {
        e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, s);   // xfer: device/pinned
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        return e == hipSuccess ? MPI_SUCCESS : hip_fail(e, "copy");
    }
    // Earlier work on s (which may wait on other ranks' GPU flags) drains
    // BEFORE the process-wide ring lock is taken, so a thread holding the lock
    // only ever waits for its own DMA: two threads running collectives on
    // different communicators cannot deadlock through the ring.
    e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_fail(e, "copy: stream before the staging ring");
    XferRing& r = xring();
    std::lock_guard<std::mutex> g(r.mu);
    if (!r.init()) return hip_fail(hipErrorOutOfMemory, "page-locked staging ring");
    const size_t nch = (bytes + kXferChunk - 1) / kXferChunk;
    auto len = [&](size_t k) { return std::min(kXferChunk, bytes - k * kXferChunk); };
    if (ps) {
        // host -> device: fill a ring slot on the CPU, DMA it; a slot is
        // refilled only after its previous DMA completed
        for (size_t k = 0; k < nch && e == hipSuccess; ++k) {
            const int sl = (int)(k & 1);
            if (k >= 2) e = hipEventSynchronize(r.ev[sl]);
            if (e != hipSuccess) break;
            memcpy(r.buf[sl], static_cast<const char*>(src) + k * kXferChunk, len(k));
            e = hipMemcpyAsync(static_cast<char*>(dst) + k * kXferChunk, r.buf[sl], len(k), hipMemcpyDefault,
                               s);   // xfer: device/pinned (dst may be device or page-locked host memory)
            if (e == hipSuccess) e = hipEventRecord(r.ev[sl], s);
        }
        if (e == hipSuccess) e = hipStreamSynchronize(s);
    } else {
        // device -> host: DMA chunk k + 1 while the CPU drains chunk k
        auto issue = [&](size_t k) {
            const int sl = (int)(k & 1);
            hipError_t x = hipMemcpyAsync(r.buf[sl], static_cast<const char*>(src) + k * kXferChunk, len(k),
                                          hipMemcpyDefault, s);   // xfer: device/pinned (src device or page-locked)
            return x == hipSuccess ? hipEventRecord(r.ev[sl], s) : x;
        };
        e = issue(0);
        for (size_t k = 0; k < nch && e == hipSuccess; ++k) {
            if (k + 1 < nch) e = issue(k + 1);
            if (e == hipSuccess) e = hipEventSynchronize(r.ev[k & 1]);
            if (e == hipSuccess) memcpy(static_cast<char*>(dst) + k * kXferChunk, r.buf[k & 1], len(k));
        }
    }
    if (e != hipSuccess) {
        (void)hipStreamSynchronize(s);   // no DMA may still read or fill a ring slot the next call reuses
        return hip_fail(e, "page-locked staged copy");
    }
    return MPI_SUCCESS;
}

int reduce_local_device(int opidx, Kind k, const void* in, void* inout, size_t count,
                        hipStream_t s)
{
    hipError_t e = launch_combine(opidx, k, in, inout, count, s, g_cfg);
    if (e != hipSuccess) return hip_fail(e, "combine kernel launch");
    return MPI_SUCCESS;
}

namespace {

int ensure_staging(DevState& s)
{
    if (s.stage_cap >= s.chunk && s.stage_in[0]) return MPI_SUCCESS;
    for (int i = 0; i < 2; ++i) {
        if (s.stage_in[i]) (void)hipFree(s.stage_in[i]);
        if (s.stage_io[i]) (void)hipFree(s.stage_io[i]);
        s.stage_in[i] = s.stage_io[i] = nullptr;
    }
    s.stage_cap = 0;
    for (int i = 0; i < 2; ++i) {
        hipError_t e = hipMalloc(&s.stage_in[i], s.chunk);
        if (e == hipSuccess) e = hipMalloc(&s.stage_io[i], s.chunk);
        if (e != hipSuccess) return hip_fail(e, "staging hipMalloc");
        if (!s.stage_s[i]) {
            e = hipStreamCreateWithFlags(&s.stage_s[i], hipStreamNonBlocking);
            if (e != hipSuccess) return hip_fail(e, "staging stream");
        }
    }
    s.stage_cap = s.chunk;
    return MPI_SUCCESS;
}

}  // namespace

namespace {
std::atomic<int> g_host_mode{0};
}

void set_host_mode(int mode) { g_host_mode.store(mode); }

int reduce_local_any(int opidx, Kind k, const void* in, void* inout, size_t count)
{
    int rc = ensure_device();
    if (rc != MPI_SUCCESS) return rc;
    BufInfo bi = classify(in), bo = classify(inout);
    DevState& s = ds();

    // Device memory, or (host modes 0 and 2) pinned host memory the kernel
    // reads and writes in place over PCIe: reads and the write-back then use
    // both PCIe directions at once, with no staging copies.  Host mode 0 also
    // pins pageable operands for the call (PinHold); if the driver refuses,
    // they are staged.
    const int mode = g_host_mode.load();
    const size_t bytes_all = count * (size_t)kind_size(k);
    PinHold hold;
    hold.sync_before_release(s.stream);
    if (mode != 1) alias_host_operands(hold, mode == 0, in, bytes_all, &bi, inout, bytes_all, &bo);
    if (bi.place == Place::Device && bo.place == Place::Device) {
        LaunchCfg cfg = g_cfg;
        cfg.host = bi.pinned_host || bo.pinned_host;
        hipError_t le = launch_combine(opidx, k, bi.dev, bo.dev, count, s.stream, cfg);   // device aliases
        if (le != hipSuccess) return hip_fail(le, "combine kernel launch");
        hipError_t e = hipStreamSynchronize(s.stream);
        return e == hipSuccess ? MPI_SUCCESS : hip_fail(e, "combine kernel");
    }
    if (mode == 0 && bytes_all >= pin_min_bytes()) trace("reduce_local: call pin refused, staging %zu bytes", bytes_all);

    // Host mode 0, small host operands: the CPU copies them into pinned bounce
    // buffers that the kernel reads and writes over PCIe -- one launch and one
    // sync instead of three synchronous pageable copies.  Another thread
    // holding the bounce buffers sends this call down the staged path.
    if (mode == 0 && bytes_all <= bounce_max_bytes()) {
        std::unique_lock<std::mutex> bg(s.bounce_mu, std::try_to_lock);
        const bool need_in = bi.place != Place::Device, need_io = bo.place != Place::Device;
        if (bg.owns_lock() && (!need_in || s.bounce_in.get(bytes_all)) && (!need_io || s.bounce_io.get(bytes_all))) {
            const void* din = bi.dev;
            void* dio = bo.dev;
            if (need_in) { memcpy(s.bounce_in.host, in, bytes_all); din = s.bounce_in.dev; }
            if (need_io) { memcpy(s.bounce_io.host, inout, bytes_all); dio = s.bounce_io.dev; }
            LaunchCfg cfg = g_cfg;
            cfg.host = true;
            hipError_t e = launch_combine(opidx, k, din, dio, count, s.stream, cfg);
            if (e != hipSuccess) return hip_fail(e, "combine kernel launch");
            e = hipStreamSynchronize(s.stream);
            if (e != hipSuccess) return hip_fail(e, "combine kernel");
            if (need_io) memcpy(inout, s.bounce_io.host, bytes_all);
            return MPI_SUCCESS;
        }
    }

    // At least one operand in host memory: chunked, double-buffered staging.
    std::lock_guard<std::mutex> g(s.stage_mu);
    LaunchCfg host_cfg = g_cfg;
    host_cfg.host = true;
    rc = ensure_staging(s);
    if (rc != MPI_SUCCESS) return rc;
    const size_t esz = (size_t)kind_size(k);
    const size_t per = (s.chunk / esz) > 0 ? (s.chunk / esz) : 1;   // elements per chunk
    size_t off = 0;
    int slot = 0;
    hipError_t e = hipSuccess;
    while (off < count && e == hipSuccess) {
        const size_t n = (count - off < per) ? count - off : per;
        const size_t bytes = n * esz;
        hipStream_t st = s.stage_s[slot];
        const char* src_in = static_cast<const char*>(in) + off * esz;
        char* src_io = static_cast<char*>(inout) + off * esz;
        const void* din;
        void* dio;
        // page-locked operands (host modes 1 / 2) are copied by DMA on the
        // slot's stream; pageable ones through the page-locked ring (xfer_sync)
        auto h2d = [&](void* d, const void* h, const BufInfo& b) {
            if (!b.dev) return xfer_sync(d, h, bytes, st) == MPI_SUCCESS ? hipSuccess : hipErrorUnknown;
            return hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, st);   // xfer: device/pinned
        };
        if (bi.place == Place::Device) {
            din = static_cast<const char*>(bi.dev) + off * esz;
        } else {
            e = h2d(s.stage_in[slot], src_in, bi);
            din = s.stage_in[slot];
        }
        if (bo.place == Place::Device) {
            dio = static_cast<char*>(bo.dev) + off * esz;
        } else {
            if (e == hipSuccess) e = h2d(s.stage_io[slot], src_io, bo);
            dio = s.stage_io[slot];
        }
        if (e == hipSuccess) e = launch_combine(opidx, k, din, dio, n, st, host_cfg);
        if (e == hipSuccess && bo.place == Place::Host) {
            if (bo.dev) e = hipMemcpyAsync(src_io, dio, bytes, hipMemcpyDeviceToHost, st);   // xfer: device/pinned
            else e = xfer_sync(src_io, dio, bytes, st) == MPI_SUCCESS ? hipSuccess : hipErrorUnknown;
        }
        off += n;
        slot ^= 1;
        // Before re-using the other slot's staging buffers, its previous chunk
        // must have drained.
        if (e == hipSuccess && off < count) e = hipStreamSynchronize(s.stage_s[slot]);
    }
    for (int i = 0; i < 2; ++i) {
        hipError_t e2 = hipStreamSynchronize(s.stage_s[i]);
        if (e == hipSuccess) e = e2;
    }
    return e == hipSuccess ? MPI_SUCCESS : hip_fail(e, "host-staged combine");
}

// SURVEY §8(e), the local reduce strong-scaled: one MPI_Reduce_local-sized
// vector split into k contiguous ranges (256-byte aligned), one per GPU of the
// node, no exchange.  Host operands (the MPI path's send / receive buffers) are
// pinned once for the call, portable to every device, and each GPU reads and
// writes its range in place over its OWN PCIe link, so the host-memory rate
// scales with the links (one GPU: ~23 GiB/s payload, PCIe-bound).  Operands in
// HBM stay on their GPU: splitting them would move HBM bytes over xGMI, ~100x
// below the local roofline.  Falls back to the one-GPU path when the pin is
// refused or k = 1.
int reduce_local_multi(int opidx, Kind k, const void* in, void* inout, size_t count, int ngpus)
{
    int rc = ensure_device();
    if (rc != MPI_SUCCESS) return rc;
    const int nvis = device_count_noinit();
    int g = ngpus <= 0 || ngpus > nvis ? nvis : ngpus;
    // MSX_TEST_MULTI_SPLIT=1 (tests only): keep ngpus ranges (up to 16) even
    // with fewer GPUs, range d on device d % nvis, so a one-GPU box runs the
    // pinning, aliasing and range logic of the k-GPU split
    if (nvis >= 1 && ngpus > nvis && getenv("MSX_TEST_MULTI_SPLIT") && atoi(getenv("MSX_TEST_MULTI_SPLIT")) == 1)
        g = std::min(ngpus, 16);
    auto dev_of = [nvis](int d) { return d % nvis; };
    BufInfo bi = classify(in), bo = classify(inout);
    const size_t esz = (size_t)kind_size(k), bytes = count * esz;
    if (g <= 1 || bi.place == Place::Device || bo.place == Place::Device || bytes < ((size_t)1 << 20))
        return reduce_local_any(opidx, k, in, inout, count);
    // an operand the caller pinned already is mapped on other GPUs only if it
    // was pinned portable; otherwise the one-GPU path (no kernel on a device
    // that cannot address it)
    for (const void* p : {in, static_cast<const void*>(inout)}) {
        const BufInfo& b = p == in ? bi : bo;
        unsigned flags = 0;
        if (b.dev && (hipHostGetFlags(&flags, const_cast<void*>(p)) != hipSuccess || !(flags & hipHostMallocPortable))) {
            (void)hipGetLastError();
            trace("reduce_local_multi: caller-pinned operand not portable, one GPU");
            return reduce_local_any(opidx, k, in, inout, count);
        }
    }
    // Call-scoped pins (CallPin: listed in temp_pins, so classify() on other
    // threads sees these pages as pageable and never launches on them), portable
    // to every device, of the operands not pinned already (one range when they
    // share pages); caller-pinned ones (hipHostMalloc) are used as they are.
    // UNVERIFIED above one GPU: the one-GPU box clamps g to 1 and returns above.
    CallPin pins[2];
    const unsigned pflags = hipHostRegisterPortable | hipHostRegisterMapped;
    const uintptr_t a0 = (uintptr_t)in, a1 = a0 + bytes, b0 = (uintptr_t)inout, b1 = b0 + bytes;
    bool ok = true;
    if (!bi.dev && !bo.dev && page_down(a0) < page_up(b1) && page_down(b0) < page_up(a1)) {
        ok = pins[0].pin(std::min(a0, b0), std::max(a1, b1), pflags);
    } else {
        if (!bi.dev) ok = pins[0].pin(a0, a1, pflags);
        if (ok && !bo.dev) ok = pins[1].pin(b0, b1, pflags);
    }
    if (!ok) {
        pins[0].release();
        pins[1].release();
        trace("reduce_local_multi: pin refused or range in use, one GPU");
        return reduce_local_any(opidx, k, in, inout, count);
    }
    auto alias = [&](const void* p) -> void* {
        for (const CallPin& c : pins)
            if (c.covers(p)) return c.dev_here(p);
        void* d = nullptr;
        if (hipHostGetDevicePointer(&d, const_cast<void*>(p), 0) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        return d;
    };
    static std::mutex mu;
    static std::vector<hipStream_t> streams;
    std::lock_guard<std::mutex> lk(mu);
    if ((int)streams.size() < g) streams.resize((size_t)g, nullptr);
    int cur = 0;
    (void)hipGetDevice(&cur);
    LaunchCfg cfg = g_cfg;
    cfg.host = true;
    hipError_t e = hipSuccess;
    const size_t align_el = esz >= 256 ? 1 : 256 / esz;
    for (int d = 0; d < g && e == hipSuccess; ++d) {
        size_t lo = count * (size_t)d / (size_t)g, hi = count * (size_t)(d + 1) / (size_t)g;
        lo -= lo % align_el;
        if (d + 1 < g) hi -= hi % align_el;
        if (hi <= lo) continue;
        e = hipSetDevice(dev_of(d));
        if (e == hipSuccess && !streams[(size_t)d]) e = hipStreamCreateWithFlags(&streams[(size_t)d], hipStreamNonBlocking);
        void* din = e == hipSuccess ? alias(in) : nullptr;
        void* dio = e == hipSuccess ? alias(inout) : nullptr;
        if (e == hipSuccess && (!din || !dio)) e = hipErrorInvalidValue;
        if (e == hipSuccess)
            e = launch_combine(opidx, k, static_cast<const char*>(din) + lo * esz, static_cast<char*>(dio) + lo * esz,
                               hi - lo, streams[(size_t)d], cfg);
    }
    for (int d = 0; d < g; ++d) {
        if (!streams[(size_t)d]) continue;
        (void)hipSetDevice(dev_of(d));
        hipError_t e2 = hipStreamSynchronize(streams[(size_t)d]);
        if (e == hipSuccess) e = e2;
    }
    (void)hipSetDevice(cur);
    return e == hipSuccess ? MPI_SUCCESS : hip_fail(e, "multi-GPU combine");   // pins released after the syncs
}

namespace {
struct Roctx {
    int (*push)(const char*) = nullptr;
    int (*pop)() = nullptr;
    bool ok = false;
};
const Roctx& roctx()
{
    static const Roctx r = [] {
        Roctx x;
        const char* e = getenv("MSX_TRACE_RANGES");
        if (!e || atoi(e) == 0) return x;
        void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("libroctx64.so.4", RTLD_NOW | RTLD_LOCAL);
        if (!h) return x;
        x.push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
        x.pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
        x.ok = x.push && x.pop;
        return x;
    }();
    return r;
}
}  // namespace

ApiRange::ApiRange(const char* fn) : on_(roctx().ok)
{
    if (on_) roctx().push(fn);
}

ApiRange::~ApiRange()
{
    if (on_) roctx().pop();
}

}  // namespace msx
