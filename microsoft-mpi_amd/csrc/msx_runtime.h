// msx_runtime.h — process state, device/stream management, buffer placement.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <memory>
#include <string>

#include "msx_kernels.h"
#include "msx_types.h"

namespace msx {

// Where a user buffer lives, as seen from the current device.
enum class Place { Device, Host };

struct BufInfo {
    Place place = Place::Host;
    void* dev = nullptr;     // device-accessible alias (device/managed/pinned), or nullptr
    int device = -1;
    bool pinned_host = false;   // Device designation of a host buffer's mapped alias
};

// MSX_TRACE=1: timestamped engine trace on stderr
void trace(const char* fmt, ...);

// thread-local error text (msx_last_error)
void set_error(const char* fmt, ...);
const char* last_error();

// A host step that may block on another process or GPU; a watchdog thread
// prints `MSX_STUCK {"rank":..,"phase":..,"peer":..,"seconds":..}` on stderr
// once the step exceeds MSX_STUCK_REPORT_S (default 30 s) -- or, for a
// stream synchronisation (sync = true, which a large call on a loaded GPU may
// legitimately spend long in), MSX_STUCK_SYNC_S (default 300 s, 0 = never).
class PhaseScope {
public:
    PhaseScope(const char* phase, int peer = -1, bool sync = false);
    ~PhaseScope();
    PhaseScope(const PhaseScope&) = delete;
    PhaseScope& operator=(const PhaseScope&) = delete;
private:
    int slot_ = -1;
};
void set_diag_rank(int rank);   // the rank named in MSX_STUCK lines

// Device bring-up.  Returns MPI_SUCCESS or MPI_ERR_OTHER (no usable GPU).
int ensure_device();
hipStream_t internal_stream();
int device_count_noinit();

BufInfo classify(const void* p);

// Call-scoped device aliases of host operands.  Pageable ranges are pinned
// (hipHostRegister, page-rounded) for the lifetime of the hold and listed so
// that classify() on any thread keeps reporting them as pageable: no other
// path of the library launches a kernel on pages this call will unpin.  The
// destructor synchronises the streams registered with sync_before_release()
// before it unpins, so error paths cannot leave work running on them.
class PinHold {
public:
    PinHold();
    ~PinHold();
    PinHold(const PinHold&) = delete;
    PinHold& operator=(const PinHold&) = delete;
    void sync_before_release(hipStream_t s);
    struct Impl;
private:
    std::unique_ptr<Impl> impl_;
    friend bool alias_host_operands(PinHold&, bool, const void*, size_t, BufInfo*, const void*, size_t, BufInfo*);
};

// A pinned host buffer the kernels read and write over PCIe, for small host
// operands: the CPU copies the user's bytes in and out around one launch,
// instead of synchronous pageable DMA copies.  Grows, never shrinks; not
// thread-safe (one owner at a time).
struct Bounce {
    char* host = nullptr;
    char* dev = nullptr;     // device alias of `host`
    size_t cap = 0;
    bool get(size_t bytes);  // false: allocation failed (use another path)
};
// Host operands up to this many bytes go through a bounce buffer
// (256 KiB; the test hook MSX_TEST_HOST_BOUNCE_MAX=0 disables it).
size_t bounce_max_bytes();

// Operands a (na bytes) and b (nb bytes; b may be a, or null): pinned host
// memory is used through its mapped alias; with pin_pageable, pageable memory
// of at least 1 MiB (test hook: MSX_TEST_HOST_PIN_MIN) is pinned for the hold's
// lifetime (one pin when the operands share pages).  Each operand aliased this
// way becomes {Place::Device, alias, pinned_host}.  Returns true when no
// operand is left in host memory.
bool alias_host_operands(PinHold& hold, bool pin_pageable, const void* a, size_t na, BufInfo* ia, const void* b,
                         size_t nb, BufInfo* ib);

void set_staging_chunk(size_t bytes);
// host operands: 0 = pinned memory combined in place by the kernel (zero-copy),
// pageable memory pinned for the call and combined the same way; 1 = every
// host operand staged through HBM; 2 = pinned in place, pageable staged
void set_host_mode(int mode);

// inout = inout (op) in over `count` elements on any combination of host and
// device buffers; blocking (returns after the result is in `inout`).
// Returns an MPI error class.
int reduce_local_any(int opidx, Kind k, const void* in, void* inout, size_t count);

// The same combine split over the node's GPUs (ngpus <= 0: every visible
// one), each range over its own PCIe link; host operands only (device
// operands and small vectors take reduce_local_any).  Blocking.
int reduce_local_multi(int opidx, Kind k, const void* in, void* inout, size_t count, int ngpus);

// Same, stream-ordered, both operands device-accessible.
int reduce_local_device(int opidx, Kind k, const void* in, void* inout, size_t count,
                        hipStream_t s);

// Host <-> device copy that never hands PAGEABLE host memory to the HIP
// runtime's copy path: a pageable side goes through the library's own
// page-locked staging ring (CPU memcpy + DMA from hipHostMalloc'd memory);
// device and page-locked memory are copied directly.  DESIGN.md §2: the
// wrong results of rounds 3-4 were 256-byte holes in pageable transfers of
// the test harness, so the product keeps its own bytes off that path.
// Stream-ordered after earlier work on s, and synchronous: returns after the
// bytes have arrived (the pageable copies it replaces were synchronous too).
// Every hipMemcpy* call site of the product is either this helper or marked
// `// xfer: device/pinned` (tests/test_abi.py audits it).
int xfer_sync(void* dst, const void* src, size_t bytes, hipStream_t s);
// true when p is host memory HIP would treat as pageable (not page-locked)
bool host_pageable(const void* p);

// hipError_t -> MPI error class with the HIP error text recorded.
int hip_fail(hipError_t e, const char* what);

// API entry/exit ranges for `rocprofv3 --marker-trace`: the counterpart of the
// reference's ETW TraceEnter_/TraceLeave_ wrappers around every MPI call
// (api/mpi_reduce.cpp:58,249,271,...).  Off unless MSX_TRACE_RANGES=1; roctx
// is opened with dlopen, so the library has no link-time dependency on it.
class ApiRange {
public:
    explicit ApiRange(const char* fn);
    ~ApiRange();
    ApiRange(const ApiRange&) = delete;
    ApiRange& operator=(const ApiRange&) = delete;
private:
    bool on_;
};

}  // namespace msx
