// host_path_probe.cpp — how fast can MPI_Reduce_local on PAGEABLE host buffers
// go on this box?  (DESIGN.md §5 "Host-memory rate".)  A measurement, not a test.
//
// 256 MiB fp32 per operand; inout += in must end in the user's pageable inout.
// Variants:
//   serial   : the library's current path — 64 MiB chunks, hipMemcpyAsync
//              H2D(in), H2D(io), combine, D2H(io) on two streams (pageable
//              copies are synchronous, so nothing overlaps)
//   duplex   : same copies, but H2D issued by one host thread and D2H by
//              another, so the two PCIe directions can overlap
//   bounce T : our own pinned bounce ring (4 slots x chunk); T host threads copy
//              pageable -> pinned and back; the kernel reads both operands and
//              writes the result in place in the pinned slot over PCIe (zero copy)
// Also prints raw rates: pageable/pinned H2D and D2H, CPU memcpy with T threads.
//
// build: hipcc -O2 --offload-arch=gfx950 -std=c++17 -pthread scripts/host_path_probe.cpp -o scripts/host_path_probe
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
            exit(2);                                                                            \
        }                                                                                       \
    } while (0)

static double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__global__ void k_add(const float4* __restrict__ a, float4* __restrict__ b, size_t n)
{
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) {
        float4 x = a[i], y = b[i];
        b[i] = make_float4(y.x + x.x, y.y + x.y, y.z + x.z, y.w + x.w);
    }
}

static void add(const void* a, void* b, size_t bytes, hipStream_t s)
{
    size_t n = bytes / 16;
    hipLaunchKernelGGL(k_add, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const float4*)a, (float4*)b, n);
}

// fixed pool of T threads running one parallel memcpy at a time
struct Pool {
    int T;
    std::vector<std::thread> th;
    std::mutex mu;
    std::condition_variable cv, done_cv;
    std::function<void(int)> job;
    long gen = 0;
    int left = 0;
    bool stop = false;
    explicit Pool(int t) : T(t)
    {
        for (int i = 0; i < T; ++i)
            th.emplace_back([this, i] {
                long seen = 0;
                for (;;) {
                    std::function<void(int)> j;
                    {
                        std::unique_lock<std::mutex> g(mu);
                        cv.wait(g, [&] { return stop || gen != seen; });
                        if (stop) return;
                        seen = gen;
                        j = job;
                    }
                    j(i);
                    std::lock_guard<std::mutex> g(mu);
                    if (--left == 0) done_cv.notify_all();
                }
            });
    }
    ~Pool()
    {
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
        }
        cv.notify_all();
        for (auto& t : th) t.join();
    }
    void run(std::function<void(int)> j)
    {
        std::unique_lock<std::mutex> g(mu);
        job = std::move(j);
        left = T;
        ++gen;
        cv.notify_all();
        done_cv.wait(g, [&] { return left == 0; });
    }
    // dst[0..n) = src[0..n) split over the T threads (4 KiB-aligned pieces)
    void copy(void* dst, const void* src, size_t n)
    {
        run([=](int i) {
            size_t per = ((n / T) + 4095) & ~(size_t)4095;
            size_t lo = std::min(n, per * i), hi = std::min(n, per * (i + 1));
            if (hi > lo) memcpy((char*)dst + lo, (const char*)src + lo, hi - lo);
        });
    }
    // two copies at once, each over half the threads
    void copy2(void* d0, const void* s0, size_t n0, void* d1, const void* s1, size_t n1)
    {
        run([=](int i) {
            const int h = T / 2 > 0 ? T / 2 : 1;
            void* d = i < h ? d0 : d1;
            const void* s = i < h ? s0 : s1;
            size_t n = i < h ? n0 : n1;
            int k = i < h ? i : i - h, m = i < h ? h : T - h;
            if (m <= 0) return;
            size_t per = ((n / m) + 4095) & ~(size_t)4095;
            size_t lo = std::min(n, per * k), hi = std::min(n, per * (k + 1));
            if (hi > lo) memcpy((char*)d + lo, (const char*)s + lo, hi - lo);
        });
    }
};

int main(int argc, char** argv)
{
    const size_t N = (size_t)64 << 20;   // fp32 elements per operand
    const size_t B = N * 4;
    CK(hipSetDevice(0));
    float* hin = (float*)aligned_alloc(4096, B);
    float* hio = (float*)aligned_alloc(4096, B);
    float* ref = (float*)aligned_alloc(4096, B);
    for (size_t i = 0; i < N; ++i) {
        hin[i] = (float)((i * 2654435761u) % 1000) * 0.001f;
        hio[i] = (float)((i * 40503u) % 777) * 0.01f;
    }
    memcpy(ref, hio, B);
    void *din, *dio;
    CK(hipMalloc(&din, (size_t)64 << 20));
    CK(hipMalloc(&dio, (size_t)64 << 20));
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    int reps = 0;   // calls of the variant so far (expected result = ref + reps*in)

    auto check = [&](const char* name) {
        size_t bad = 0;
        for (size_t i = 0; i < N; i += 4097) {
            float e = ref[i];
            for (int r = 0; r < reps; ++r) e += hin[i];
            if (hio[i] != e) ++bad;
        }
        if (bad) printf("%s: %zu mismatches\n", name, bad);
        return bad == 0;
    };

    // ---- raw rates ----
    {
        double t = now();
        for (int r = 0; r < 3; ++r) CK(hipMemcpy(din, hin, (size_t)64 << 20, hipMemcpyHostToDevice));
        printf("{\"raw\":\"pageable_h2d\",\"GB_s\":%.1f}\n", 3.0 * (64 << 20) / (now() - t) / 1e9);
        t = now();
        for (int r = 0; r < 3; ++r) CK(hipMemcpy(ref, dio, (size_t)64 << 20, hipMemcpyDeviceToHost));
        printf("{\"raw\":\"pageable_d2h\",\"GB_s\":%.1f}\n", 3.0 * (64 << 20) / (now() - t) / 1e9);
        memcpy(ref, hio, B);
        void* pin;
        CK(hipHostMalloc(&pin, (size_t)64 << 20, 0));
        t = now();
        for (int r = 0; r < 3; ++r) CK(hipMemcpy(din, pin, (size_t)64 << 20, hipMemcpyHostToDevice));
        printf("{\"raw\":\"pinned_h2d\",\"GB_s\":%.1f}\n", 3.0 * (64 << 20) / (now() - t) / 1e9);
        t = now();
        for (int r = 0; r < 3; ++r) CK(hipMemcpy(pin, dio, (size_t)64 << 20, hipMemcpyDeviceToHost));
        printf("{\"raw\":\"pinned_d2h\",\"GB_s\":%.1f}\n", 3.0 * (64 << 20) / (now() - t) / 1e9);
        for (int T : {1, 2, 4, 8, 12, 16}) {
            Pool pool(T);
            pool.copy(pin, hin, (size_t)64 << 20);
            t = now();
            for (int r = 0; r < 5; ++r) pool.copy(pin, hin, (size_t)64 << 20);
            printf("{\"raw\":\"cpu_memcpy_to_pinned\",\"threads\":%d,\"GB_s\":%.1f}\n", T,
                   5.0 * (64 << 20) / (now() - t) / 1e9);
        }
        CK(hipHostFree(pin));
    }
    fflush(stdout);

    // ---- serial (the library's current pageable path) ----
    auto serial = [&] {
        const size_t C = (size_t)64 << 20;
        void* sin[2] = {din, nullptr};
        void* sio[2] = {dio, nullptr};
        static void *din2 = nullptr, *dio2 = nullptr;
        if (!din2) { CK(hipMalloc(&din2, C)); CK(hipMalloc(&dio2, C)); }
        sin[1] = din2; sio[1] = dio2;
        hipStream_t st[2] = {s0, s1};
        int slot = 0;
        for (size_t off = 0; off < B; off += C) {
            size_t n = std::min(C, B - off);
            CK(hipMemcpyAsync(sin[slot], (char*)hin + off, n, hipMemcpyHostToDevice, st[slot]));
            CK(hipMemcpyAsync(sio[slot], (char*)hio + off, n, hipMemcpyHostToDevice, st[slot]));
            add(sin[slot], sio[slot], n, st[slot]);
            CK(hipMemcpyAsync((char*)hio + off, sio[slot], n, hipMemcpyDeviceToHost, st[slot]));
            slot ^= 1;
            if (off + C < B) CK(hipStreamSynchronize(st[slot]));
        }
        CK(hipStreamSynchronize(s0));
        CK(hipStreamSynchronize(s1));
    };

    // ---- duplex: H2D on this thread, D2H on a second thread ----
    auto duplex = [&](size_t C) {
        const int NS = 3;
        static std::vector<void*> bi, bo;
        static size_t cap = 0;
        if (cap < C) {
            for (void* p : bi) CK(hipFree(p));
            for (void* p : bo) CK(hipFree(p));
            bi.assign(NS, nullptr); bo.assign(NS, nullptr);
            for (int i = 0; i < NS; ++i) { CK(hipMalloc(&bi[i], C)); CK(hipMalloc(&bo[i], C)); }
            cap = C;
        }
        const size_t nch = (B + C - 1) / C;
        std::vector<hipEvent_t> ready(nch);
        for (auto& e : ready) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        std::atomic<long> issued{-1}, drained{-1};
        std::thread out([&] {
            hipStream_t so;
            CK(hipStreamCreateWithFlags(&so, hipStreamNonBlocking));
            for (size_t i = 0; i < nch; ++i) {
                while (issued.load() < (long)i) std::this_thread::yield();
                CK(hipStreamWaitEvent(so, ready[i], 0));
                size_t off = i * C, n = std::min(C, B - off);
                CK(hipMemcpyAsync((char*)hio + off, bo[i % NS], n, hipMemcpyDeviceToHost, so));
                CK(hipStreamSynchronize(so));
                drained.store((long)i);
            }
            CK(hipStreamDestroy(so));
        });
        for (size_t i = 0; i < nch; ++i) {
            while (drained.load() < (long)i - NS) std::this_thread::yield();   // slot i%NS free
            size_t off = i * C, n = std::min(C, B - off);
            CK(hipMemcpyAsync(bi[i % NS], (char*)hin + off, n, hipMemcpyHostToDevice, s0));
            CK(hipMemcpyAsync(bo[i % NS], (char*)hio + off, n, hipMemcpyHostToDevice, s0));
            add(bi[i % NS], bo[i % NS], n, s0);
            CK(hipEventRecord(ready[i], s0));
            issued.store((long)i);
        }
        out.join();
        CK(hipStreamSynchronize(s0));
        for (auto& e : ready) CK(hipEventDestroy(e));
    };

    // ---- bounce: pinned ring + T copy threads + zero-copy kernel ----
    auto bounce = [&](Pool& pool, size_t C) {
        const int NS = 3;
        static std::vector<void*> pi, po;
        static size_t cap = 0;
        if (cap < C) {
            for (void* p : pi) CK(hipHostFree(p));
            for (void* p : po) CK(hipHostFree(p));
            pi.assign(NS, nullptr); po.assign(NS, nullptr);
            for (int i = 0; i < NS; ++i) { CK(hipHostMalloc(&pi[i], C, 0)); CK(hipHostMalloc(&po[i], C, 0)); }
            cap = C;
        }
        const size_t nch = (B + C - 1) / C;
        std::vector<hipEvent_t> ev(nch);
        for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        auto cin = [&](size_t i) {
            size_t off = i * C, n = std::min(C, B - off);
            pool.copy2(pi[i % NS], (char*)hin + off, n, po[i % NS], (char*)hio + off, n);
            add(pi[i % NS], po[i % NS], n, s0);
            CK(hipEventRecord(ev[i], s0));
        };
        auto cout = [&](size_t i) {
            size_t off = i * C, n = std::min(C, B - off);
            CK(hipEventSynchronize(ev[i]));
            pool.copy((char*)hio + off, po[i % NS], n);
        };
        cin(0);
        for (size_t i = 1; i < nch; ++i) {
            cin(i);           // CPU fills slot i while the GPU combines slot i-1
            cout(i - 1);
        }
        cout(nch - 1);
        for (auto& e : ev) CK(hipEventDestroy(e));
    };

    // ---- bounce2: copy-in of chunk i+1 and copy-out of chunk i-1 run at the
    // same time on two halves of the pool while the GPU combines chunk i ----
    auto bounce2 = [&](Pool& pool, size_t C) {
        const int NS = 3;
        static std::vector<void*> pi, po;
        static size_t cap = 0;
        if (cap < C) {
            for (void* p : pi) CK(hipHostFree(p));
            for (void* p : po) CK(hipHostFree(p));
            pi.assign(NS, nullptr); po.assign(NS, nullptr);
            for (int i = 0; i < NS; ++i) { CK(hipHostMalloc(&pi[i], C, 0)); CK(hipHostMalloc(&po[i], C, 0)); }
            cap = C;
        }
        const long nch = (long)((B + C - 1) / C);
        std::vector<hipEvent_t> ev(nch);
        for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        const int T = pool.T, h = T / 2 > 0 ? T / 2 : 1;
        auto piece = [](size_t n, int k, int m, size_t* lo, size_t* hi) {
            size_t per = ((n / m) + 4095) & ~(size_t)4095;
            *lo = std::min(n, per * k);
            *hi = std::min(n, per * (k + 1));
        };
        for (long k = -1; k < nch; ++k) {
            const long ci = k + 1, co = k - 1;   // chunk to fill, chunk to drain
            pool.run([&](int t) {
                if (t < h) {
                    if (ci >= nch) return;
                    size_t off = (size_t)ci * C, n = std::min(C, B - off), lo, hi;
                    piece(n, t, h, &lo, &hi);
                    if (hi > lo) {
                        memcpy((char*)pi[ci % NS] + lo, (char*)hin + off + lo, hi - lo);
                        memcpy((char*)po[ci % NS] + lo, (char*)hio + off + lo, hi - lo);
                    }
                } else {
                    if (co < 0) return;
                    CK(hipEventSynchronize(ev[co]));
                    size_t off = (size_t)co * C, n = std::min(C, B - off), lo, hi;
                    piece(n, t - h, T - h, &lo, &hi);
                    if (hi > lo) memcpy((char*)hio + off + lo, (char*)po[co % NS] + lo, hi - lo);
                }
            });
            if (ci < nch) {
                size_t off = (size_t)ci * C, n = std::min(C, B - off);
                add(pi[ci % NS], po[ci % NS], n, s0);
                CK(hipEventRecord(ev[ci], s0));
            }
        }
        // the last chunk
        CK(hipEventSynchronize(ev[nch - 1]));
        {
            size_t off = (size_t)(nch - 1) * C, n = std::min(C, B - off);
            pool.copy((char*)hio + off, po[(nch - 1) % NS], n);
        }
        for (auto& e : ev) CK(hipEventDestroy(e));
    };

    // ---- register: pin the user's pageable buffers for the call ----
    auto reg = [&] {
        CK(hipHostRegister(hin, B, hipHostRegisterMapped));
        CK(hipHostRegister(hio, B, hipHostRegisterMapped));
        void *da, *db;
        CK(hipHostGetDevicePointer(&da, hin, 0));
        CK(hipHostGetDevicePointer(&db, hio, 0));
        add(da, db, B, s0);
        CK(hipStreamSynchronize(s0));
        CK(hipHostUnregister(hin));
        CK(hipHostUnregister(hio));
    };

    auto timeit = [&](const char* name, int T, size_t C, std::function<void()> f) {
        memcpy(hio, ref, B);
        reps = 0;
        f();
        ++reps;
        double best = 1e9;
        for (int r = 0; r < 4; ++r) {
            double t = now();
            f();
            ++reps;
            best = std::min(best, now() - t);
        }
        bool ok = check(name);
        printf("{\"variant\":\"%s\",\"threads\":%d,\"chunk_MiB\":%zu,\"ms\":%.2f,\"payload_GiB_s\":%.2f,\"ok\":%s}\n",
               name, T, C >> 20, best * 1e3, B / best / (1 << 30), ok ? "true" : "false");
        fflush(stdout);
    };
    const bool quick = argc > 1 && !strcmp(argv[1], "quick");
    timeit("serial", 1, 64 << 20, serial);
    timeit("register", 1, 256, reg);
    if (!quick) {
        for (size_t C : {(size_t)16 << 20, (size_t)32 << 20, (size_t)64 << 20})
            timeit("duplex", 2, C, [&] { duplex(C); });
        for (int T : {8, 16})
            for (size_t C : {(size_t)16 << 20, (size_t)32 << 20}) {
                Pool pool(T);
                timeit("bounce", T, C, [&] { bounce(pool, C); });
            }
    }
    for (int T : {4, 8, 12, 16})
        for (size_t C : {(size_t)4 << 20, (size_t)8 << 20, (size_t)16 << 20, (size_t)32 << 20}) {
            Pool pool(T);
            timeit("bounce2", T, C, [&] { bounce2(pool, C); });
        }
    return 0;
}
