// msx_probe.hip — bench-only measurement kernels (libmsx_probe.so).  Not part
// of the product library libmsmpi_mi355x.so: nothing in the MPI path loads
// this.  bench.py and scripts/ use it to put the product kernels' rates next
// to what this GPU's HBM delivers:
//   * msxp_hbm: other stream mixes in the default combine's launch geometry
//     (16 B per lane, 256-lane workgroups, one tile each, XCD-contiguous,
//     non-temporal loads), plus copies with one-wave workgroups in dispatch
//     order (k_copy_dram's) and in XCD runs of 128 tiles (k_combine_dram's),
//     and 16-of-32-byte gapped loads / stores;
//   * msxp_variant_*: the fp32 SUM combine body (msx_combine_dev.h, the exact
//     device code of k_combine / k_combine_dram) in other launch geometries,
//     for the tuning sweep, and the default DRAM-regime body under its own
//     symbol (k_probe_combine<..., 64, ..., -1>) so single cold-cache launches
//     stay out of the headline kernel's rocprof statistics;
//   * msxp_tree8: the product's 8-source DRAM-regime tree (k_tree, fp32 SUM,
//     non-temporal loads, one-wave workgroups) in another tile order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "msx_combine_dev.h"
#include "msx_tree_dev.h"

#define MSXP_EXPORT extern "C" __attribute__((visibility("default")))

namespace msx {
namespace probe {

using namespace dev;

// MODE 0: read a and b (2R)   MODE 1: write b (1W)   MODE 2: copy a -> b (1R1W)
// MODE 3: read a (1R)   MODE 6: write 16 B of every 32 B of b   MODE 7: read
// 16 B of every 32 B of a.  Reads feed a conditional store on a value random
// data essentially never produces (`key`), so the compiler cannot drop them.
template <int MODE>
__global__ __launch_bounds__(256) void k_probe(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t nvec,
                                               unsigned key)
{
    const size_t i = (size_t)xcd_tile(blockIdx.x, gridDim.x) * 256 + threadIdx.x;
    if (i >= nvec) return;
    if constexpr (MODE == 0) {
        u32x4 x = ld<true>(a + i), y = ld<true>(b + i);
        issued_together(x, y);
        const u32x4 r = x ^ y;
        if ((r.x ^ r.y ^ r.z ^ r.w) == key) b[i] = r;
    } else if constexpr (MODE == 1) {
        b[i] = u32x4{key, key ^ (unsigned)i, key, (unsigned)(i >> 32)};
    } else if constexpr (MODE == 2) {
        b[i] = ld<true>(a + i);
    } else if constexpr (MODE == 6) {
        b[2 * i] = u32x4{key, key ^ (unsigned)i, key, (unsigned)(i >> 32)};
    } else if constexpr (MODE == 7) {
        const u32x4 x = ld<true>(a + 2 * i);
        if ((x.x ^ x.y ^ x.z ^ x.w) == key) b[i] = x;
    } else {
        const u32x4 x = ld<true>(a + i);
        if ((x.x ^ x.y ^ x.z ^ x.w) == key) b[i] = x;
    }
}

// copy a -> b with one-wave workgroups in tile order XG (-1 dispatch order,
// k_copy_dram's; 128 = XCD runs of 128 tiles, k_combine_dram's)
template <int XG>
__global__ __launch_bounds__(64) void k_probe_copy_rr(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t nvec)
{
    const size_t i = combine_tile<XG>(blockIdx.x, gridDim.x) * 64 + threadIdx.x;
    if (i < nvec) b[i] = ld<true>(a + i);
}

template <int UNROLL, int BLOCK, bool NTLD, bool NTST, int XG>
__global__ __launch_bounds__(BLOCK) void k_probe_combine(const float* __restrict__ in, float* __restrict__ io,
                                                         size_t head, size_t nvec, size_t tail)
{
    combine_body<O_SUM, float, float, UNROLL, BLOCK, NTLD, NTST, XG>(in, io, head, nvec, tail);
}

// the "LDS staging of the incoming chunk" form: `in` goes global -> LDS ->
// registers.  Each element is used once, so the stage only adds an LDS write
// + read per byte and a barrier (measured, not asserted)
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_probe_combine_lds(const float* __restrict__ in, float* __restrict__ io,
                                                             size_t head, size_t nvec, size_t tail)
{
    __shared__ u32x4 stage[BLOCK];
    const u32x4* __restrict__ vin = reinterpret_cast<const u32x4*>(in + head);
    u32x4* __restrict__ vio = reinterpret_cast<u32x4*>(io + head);
    for (size_t t0 = (size_t)blockIdx.x * BLOCK; t0 < nvec; t0 += (size_t)gridDim.x * BLOCK) {
        const size_t i = t0 + threadIdx.x;
        const bool live = i < nvec;
        u32x4 b = {};
        if (live) {
            stage[threadIdx.x] = ld<true>(vin + i);
            b = ld<true>(vio + i);
        }
        __syncthreads();
        if (live) vio[i] = apply_vec<O_SUM, float>(b, stage[threadIdx.x]);
        __syncthreads();
    }
    const size_t nscalar = head + tail, body_end = head + nvec * 4;
    for (size_t s = (size_t)blockIdx.x * BLOCK + threadIdx.x; s < nscalar; s += (size_t)gridDim.x * BLOCK) {
        const size_t e = s < head ? s : body_end + (s - head);
        io[e] = Fn<O_SUM>::apply(io[e], in[e]);
    }
}

template <int UNROLL, int BLOCK, bool NTLD, bool NTST, int XG>
hipError_t run_variant(const void* in, void* io, size_t count, hipStream_t s)
{
    size_t head, nvec, tail;
    combine_split<float>(in, io, count, head, nvec, tail);
    const size_t tile = (size_t)BLOCK * UNROLL;
    size_t grid = (nvec + tile - 1) / tile;
    const size_t sc = (head + tail + BLOCK - 1) / BLOCK;
    if (grid < sc) grid = sc;
    if (grid == 0) return hipSuccess;
    if (grid > 0x7fffffffu) return hipErrorInvalidValue;
    hipLaunchKernelGGL((k_probe_combine<UNROLL, BLOCK, NTLD, NTST, XG>), dim3((unsigned)grid), dim3(BLOCK), 0, s,
                       static_cast<const float*>(in), static_cast<float*>(io), head, nvec, tail);
    return hipGetLastError();
}

template <int BLOCK>
hipError_t run_variant_lds(const void* in, void* io, size_t count, hipStream_t s)
{
    size_t head, nvec, tail;
    combine_split<float>(in, io, count, head, nvec, tail);
    size_t grid = (nvec + BLOCK - 1) / BLOCK;
    const size_t sc = (head + tail + BLOCK - 1) / BLOCK;
    if (grid < sc) grid = sc;
    if (grid == 0) return hipSuccess;
    if (grid > 0x7fffffffu) return hipErrorInvalidValue;
    hipLaunchKernelGGL((k_probe_combine_lds<BLOCK>), dim3((unsigned)grid), dim3(BLOCK), 0, s,
                       static_cast<const float*>(in), static_cast<float*>(io), head, nvec, tail);
    return hipGetLastError();
}

struct Variant {
    const char* name;
    hipError_t (*fn)(const void*, void*, size_t, hipStream_t);
};

// index 0: the product's default body above 16 MiB per operand (k_combine_dram:
// one-wave workgroups, XCD runs of 128 tiles) under the probe symbol
const Variant kVariants[] = {
    {"default_body_probe", run_variant<1, 64, true, false, 128>},
    {"u1_b64_ntld_rr", run_variant<1, 64, true, false, -1>},          // rounds 4-5 default above 16 MiB
    {"u1_b256_ntld_tiles", run_variant<1, 256, true, false, 0>},      // rounds 1-4 default: XCD-contiguous tiles
    {"u1_b256_ntld_rr", run_variant<1, 256, true, false, -1>},
    {"u1_b128_ntld_rr", run_variant<1, 128, true, false, -1>},
    {"u2_b64_ntld_rr", run_variant<2, 64, true, false, -1>},
    {"u4_b256_ntld_tiles", run_variant<4, 256, true, false, 0>},
    {"u1_b64_ntall_rr", run_variant<1, 64, true, true, -1>},
    {"u1_b64_plain_rr", run_variant<1, 64, false, false, -1>},
    {"u1_b256_ntld_xg8", run_variant<1, 256, true, false, 8>},
    {"u1_b256_ntld_xg32", run_variant<1, 256, true, false, 32>},
    {"u1_b256_ntld_xg128", run_variant<1, 256, true, false, 128>},
    {"u1_b64_ntld_tiles", run_variant<1, 64, true, false, 0>},      // one-wave workgroups, XCD-contiguous eighths
    {"u1_b64_ntld_xg8", run_variant<1, 64, true, false, 8>},
    {"u1_b64_ntld_xg32", run_variant<1, 64, true, false, 32>},
    {"u1_b64_ntld_xg64", run_variant<1, 64, true, false, 64>},
    {"u1_b64_ntld_xg256", run_variant<1, 64, true, false, 256>},
    {"u1_b64_ntld_xg512", run_variant<1, 64, true, false, 512>},
    {"u1_b128_ntld_xg64", run_variant<1, 128, true, false, 64>},
    {"u1_b128_ntld_xg128", run_variant<1, 128, true, false, 128>},
    {"u1_b64_ntall_xg128", run_variant<1, 64, true, true, 128>},
    {"u1_b256_lds", run_variant_lds<256>},
};
constexpr int kNumVariants = (int)(sizeof(kVariants) / sizeof(kVariants[0]));

}  // namespace probe
}  // namespace msx

using namespace msx::probe;

MSXP_EXPORT int msxp_hbm(int mode, const void* a, void* b, int64_t bytes, void* stream)
{
    if (bytes < 0 || !b || (mode != 1 && mode != 6 && !a) || ((((uintptr_t)a | (uintptr_t)b) & 15) != 0)) return 1;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const u32x4* va = static_cast<const u32x4*>(a);
    u32x4* vb = static_cast<u32x4*>(b);
    if (mode == 9 || mode == 10) {
        const size_t nv = (size_t)bytes / 16, grid = (nv + 63) / 64;
        if (grid == 0) return 0;
        if (grid > 0x7fffffffu) return 1;
        if (mode == 9) hipLaunchKernelGGL(k_probe_copy_rr<-1>, dim3((unsigned)grid), dim3(64), 0, s, va, vb, nv);
        else hipLaunchKernelGGL(k_probe_copy_rr<128>, dim3((unsigned)grid), dim3(64), 0, s, va, vb, nv);
        return hipGetLastError() == hipSuccess ? 0 : 2;
    }
    const size_t nvec = (mode >= 6) ? (size_t)bytes / 32 : (size_t)bytes / 16;
    const size_t grid = (nvec + 255) / 256;
    if (grid == 0) return 0;
    if (grid > 0x7fffffffu) return 1;
    const unsigned key = 0x9E3779B9u;
    switch (mode) {
    case 0: hipLaunchKernelGGL(k_probe<0>, dim3((unsigned)grid), dim3(256), 0, s, va, vb, nvec, key); break;
    case 1: hipLaunchKernelGGL(k_probe<1>, dim3((unsigned)grid), dim3(256), 0, s, va, vb, nvec, key); break;
    case 2: hipLaunchKernelGGL(k_probe<2>, dim3((unsigned)grid), dim3(256), 0, s, va, vb, nvec, key); break;
    case 3: hipLaunchKernelGGL(k_probe<3>, dim3((unsigned)grid), dim3(256), 0, s, va, vb, nvec, key); break;
    case 6: hipLaunchKernelGGL(k_probe<6>, dim3((unsigned)grid), dim3(256), 0, s, va, vb, nvec, key); break;
    case 7: hipLaunchKernelGGL(k_probe<7>, dim3((unsigned)grid), dim3(256), 0, s, va, vb, nvec, key); break;
    default: return 1;
    }
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

// device memory with the engine windows' cache type (uncached = 1) or plain
MSXP_EXPORT int msxp_alloc(int64_t bytes, int uncached, void** out)
{
    if (bytes <= 0 || !out) return 1;
    *out = nullptr;
    hipError_t e = uncached ? hipExtMallocWithFlags(out, (size_t)bytes, hipDeviceMallocUncached)
                            : hipMalloc(out, (size_t)bytes);
    return e == hipSuccess ? 0 : 2;
}

MSXP_EXPORT int msxp_free(void* p) { return p && hipFree(p) != hipSuccess ? 2 : 0; }

MSXP_EXPORT int msxp_variant_count(void) { return kNumVariants; }

MSXP_EXPORT const char* msxp_variant_name(int v) { return v >= 0 && v < kNumVariants ? kVariants[v].name : nullptr; }

// inout[i] += in[i] over `count` fp32 (MPI_SUM MPI_FLOAT), variant v, on `stream`
MSXP_EXPORT int msxp_variant_run(int v, const void* in, void* inout, int64_t count, void* stream)
{
    if (v < 0 || v >= kNumVariants || count < 0 || !in || !inout) return 1;
    return kVariants[v].fn(in, inout, (size_t)count, static_cast<hipStream_t>(stream)) == hipSuccess ? 0 : 2;
}

// out[i] = ((s0+s1)+(s2+s3))+((s4+s5)+(s6+s7)) over n fp32 (16-byte aligned
// pointers, n a multiple of 4): the product's k_tree<SUM, float, float, 64,
// NT, 8 leaves> -- the tree above 256 MiB of sources -- with tile order xg
// (-1 dispatch order, the product's; 0 XCD-contiguous; G > 0 XCD runs of G)
MSXP_EXPORT int msxp_tree8(const void* const* srcs, void* out, int64_t n, int xg, void* stream)
{
    using namespace msx::dev;
    if (!srcs || !out || n <= 0 || (n & 3)) return 1;
    TreeArgs a{};
    for (int k = 0; k < 8; ++k) {
        if (!srcs[k] || ((uintptr_t)srcs[k] & 15)) return 1;
        a.s[2 * k] = a.s[2 * k + 1] = srcs[k];
    }
    if ((uintptr_t)out & 15) return 1;
    a.P = 8;
    a.nleaves = 8;
    a.xg = xg;
    a.done_launches = 1;
    const size_t nvec = (size_t)n / 4, grid = (nvec + 63) / 64;
    if (grid > 0x7fffffffu) return 1;
    hipLaunchKernelGGL((k_tree<msx::O_SUM, float, float, 64, true, 8, 1, false, false>), dim3((unsigned)grid), dim3(64), 0,
                       static_cast<hipStream_t>(stream), a, static_cast<float*>(out), nvec, (size_t)0, 1);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

// one workgroup: lane 0 waits `ticks` of s_memrealtime (100 MHz), then stores
// `value` to *flag (page-locked host memory, system-scope release) -- a kernel
// whose completion the host can see directly, to check that a stream or device
// synchronisation returns only after it (scripts/sync_probe.py)
__global__ __launch_bounds__(64) void k_probe_spin_mark(unsigned long long ticks, unsigned* flag, unsigned value)
{
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
    __hip_atomic_store(flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

MSXP_EXPORT int msxp_spin_mark(int64_t ticks, void* flag_dev, unsigned value, void* stream)
{
    if (ticks < 0 || ticks > 100000000 || !flag_dev) return 1;   // at most 1 s
    hipLaunchKernelGGL(k_probe_spin_mark, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream),
                       (unsigned long long)ticks, static_cast<unsigned*>(flag_dev), value);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}
