// msx_runtime.h — process state, device/stream management, buffer placement.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
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
};

// MSX_TRACE=1: timestamped engine trace on stderr
void trace(const char* fmt, ...);

// thread-local error text (msx_last_error)
void set_error(const char* fmt, ...);
const char* last_error();

// Device bring-up.  Returns MPI_SUCCESS or MPI_ERR_OTHER (no usable GPU).
int ensure_device();
int current_device();
hipStream_t internal_stream();
int device_count_noinit();

BufInfo classify(const void* p);

LaunchCfg& launch_cfg();
void set_staging_chunk(size_t bytes);
// host operands: 0 = pinned memory combined in place by the kernel (zero-copy),
// pageable memory pinned for the call and combined the same way; 1 = every
// host operand staged through HBM; 2 = pinned in place, pageable staged
void set_host_mode(int mode);
int host_mode();

// inout = inout (op) in over `count` elements on any combination of host and
// device buffers; blocking (returns after the result is in `inout`).
// Returns an MPI error class.
int reduce_local_any(int opidx, Kind k, const void* in, void* inout, size_t count);

// Same, stream-ordered, both operands device-accessible.
int reduce_local_device(int opidx, Kind k, const void* in, void* inout, size_t count,
                        hipStream_t s);

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
