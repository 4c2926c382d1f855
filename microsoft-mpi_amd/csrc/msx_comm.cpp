// msx_comm.cpp — process state, communicators, local combine, requests.
//
// Reference anchors:
//   MPI_Init -> MpiProcess::Initialize (mpid/env.cpp:1062-1175)
//   MPID_Uop_call / MPIR_Op_c_proxy (include/op.h:171-174, mpid/op.cpp:542-545)
//   NBC requests progressed in MPI_Test/Wait (mpid/request.cpp:780-886)
#include "msx_comm.h"
#include "msx_dtype.h"

#include <atomic>
#include <deque>
#include <thread>
#include <chrono>
#include <functional>
#include <future>
#include <mutex>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>
#include <vector>

#include "msx_runtime.h"
#include "msx_transport.h"

namespace msx {

namespace {

std::atomic<bool> g_init{false};
std::atomic<bool> g_fini{false};
Comm g_world;
Comm g_self;

}  // namespace

bool is_initialized() { return g_init.load(); }
bool is_finalized() { return g_fini.load(); }
Comm* world() { return g_init.load() ? &g_world : nullptr; }

// Derived communicators: direct handles 0x84000000 | index (HANDLE_TYPE_DIRECT,
// kind comm), as MS-MPI numbers them.
namespace {
std::mutex g_comm_mu;
std::vector<Comm*> g_comms;
constexpr unsigned kCommDirect = 0x84000000u;
}  // namespace

Comm* lookup_comm(MPI_Comm c)
{
    if (c == MPI_COMM_WORLD) return &g_world;
    if (c == MPI_COMM_SELF) return &g_self;
    if (((unsigned)c & 0xfc000000u) != kCommDirect) return nullptr;
    std::lock_guard<std::mutex> g(g_comm_mu);
    const size_t idx = (unsigned)c & 0x03ffffffu;
    return idx < g_comms.size() ? g_comms[idx] : nullptr;
}

MPI_Comm comm_register(Comm* c)
{
    std::lock_guard<std::mutex> g(g_comm_mu);
    size_t idx = 0;
    while (idx < g_comms.size() && g_comms[idx]) ++idx;
    if (idx == g_comms.size()) g_comms.push_back(nullptr);
    g_comms[idx] = c;
    c->handle = (MPI_Comm)(kCommDirect | (unsigned)idx);
    return c->handle;
}

void comm_unregister(Comm* c)
{
    std::lock_guard<std::mutex> g(g_comm_mu);
    const size_t idx = (unsigned)c->handle & 0x03ffffffu;
    if (idx < g_comms.size() && g_comms[idx] == c) g_comms[idx] = nullptr;
}

static int env_int(const char* a, const char* b, int dflt)
{
    const char* v = getenv(a);
    if (!v && b) v = getenv(b);
    return v ? atoi(v) : dflt;
}

int world_init()
{
    g_world = Comm{};
    g_world.handle = MPI_COMM_WORLD;
    g_self = Comm{};
    g_self.handle = MPI_COMM_SELF;
    // One process per GPU, launched by torchrun-style env (RANK, WORLD_SIZE,
    // LOCAL_RANK, MASTER_ADDR, MASTER_PORT) or MSX_RANK / MSX_SIZE.
    const int size = env_int("MSX_SIZE", "WORLD_SIZE", 1);
    const int rank = env_int("MSX_RANK", "RANK", 0);
    if (size < 1 || rank < 0 || rank >= size) {
        set_error("bad rank/size from environment (rank=%d size=%d)", rank, size);
        return MPI_ERR_OTHER;
    }
    // A host without a GPU still initialises (argument checking works); every
    // compute call then fails loudly with MPI_ERR_OTHER.
    (void)ensure_device();
    g_world.rank = rank;
    g_world.size = size;
    set_diag_rank(rank);
    g_world.lpid.resize((size_t)size);
    for (int r = 0; r < size; ++r) g_world.lpid[(size_t)r] = r;
    g_self.lpid.assign(1, rank);
    if (size > 1) {
        int rc = transport_create(rank, size, &g_world.tp);
        if (rc == MPI_SUCCESS) rc = engine_mailbox_init(g_world.tp, rank, size);   // MPI_Intercomm_create
        if (rc != MPI_SUCCESS) return rc;
    }
    g_init.store(true);
    return MPI_SUCCESS;
}

int world_finalize()
{
    int rc = MPI_SUCCESS;
    if (g_world.tp) {
        rc = g_world.tp->barrier();
        transport_destroy(g_world.tp);
        g_world.tp = nullptr;
    }
    if (ensure_device() == MPI_SUCCESS) (void)hipDeviceSynchronize();
    g_fini.store(true);
    return rc;
}

// ---------------------------------------------------------------------------
// copies and the local combine
// ---------------------------------------------------------------------------
int copy_any(void* dst, const void* src, size_t bytes)
{
    if (bytes == 0 || dst == src) return MPI_SUCCESS;
    BufInfo bd = classify(dst), bs = classify(src);
    if (bd.place == Place::Host && bs.place == Place::Host) {
        memcpy(dst, src, bytes);   // MPIR_Localcopy memcpy (mpid/pt2pt.cpp:812)
        return MPI_SUCCESS;
    }
    int rc = ensure_device();
    if (rc != MPI_SUCCESS) return rc;
    return xfer_sync(dst, src, bytes, internal_stream());   // pageable sides through the page-locked ring
}

// A derived datatype reaches only user functions (the builtin ops' check
// tables reject it): MPID_Uop_call(op, in, inout, &count, &dt) on the typed
// buffers (api/mpi_reduce.cpp:361).  Device operands are staged through host
// memory over the whole byte span the type map touches, so the bytes between
// the mapped elements of `inout` are written back unchanged.
int local_combine_typed(const OpRef& op, MPI_Datatype dt, const void* in, void* inout, size_t count)
{
    const Dtype* t = dtype_lookup(dt);
    if (!t) { set_error("invalid datatype 0x%x", dt); return MPI_ERR_TYPE; }
    if (count > 0x7fffffff) { set_error("count exceeds the MPI_User_function range"); return MPI_ERR_COUNT; }
    int64_t lo, hi;
    dt_span(t, (int64_t)count, &lo, &hi);
    const size_t span = (size_t)(hi - lo);
    const char* pin = static_cast<const char*>(in);
    char* pio = static_cast<char*>(inout);
    const BufInfo bi = classify(pin + lo), bo = classify(pio + lo);
    std::vector<char> hin, hio;
    int rc = MPI_SUCCESS;
    if (span && bi.place == Place::Device) {
        hin.resize(span);
        if ((rc = copy_any(hin.data(), pin + lo, span)) != MPI_SUCCESS) return rc;
        pin = hin.data() - lo;
    }
    if (span && bo.place == Place::Device) {
        hio.resize(span);
        if ((rc = copy_any(hio.data(), pio + lo, span)) != MPI_SUCCESS) return rc;
        pio = hio.data() - lo;
    }
    int len = (int)count;
    MPI_Datatype d = dt;
    op.user_fn(const_cast<char*>(pin), pio, &len, &d);
    if (span && bo.place == Place::Device) rc = copy_any(static_cast<char*>(inout) + lo, hio.data(), span);
    return rc;
}

int local_combine(const OpRef& op, MPI_Datatype dt, const void* in, void* inout, size_t count)
{
    if (count == 0) return MPI_SUCCESS;
    if (op.opidx != O_NULL) {
        const TypeInfo* t = type_info(dt);
        if (!t) { set_error("datatype 0x%x has no reduction kernel", dt); return MPI_ERR_OP; }
        return reduce_local_any(op.opidx, t->kind, in, inout, count);
    }
    // User-defined op: MPI_User_function is host code (mpi.h:2258-2265), called
    // through the C proxy with int-sized chunks.  Device operands are staged
    // to host memory around the call.
    if (dtype_is_derived(dt)) return local_combine_typed(op, dt, in, inout, count);
    const int esz = type_size(dt);
    if (esz <= 0) { set_error("datatype 0x%x not supported with user ops", dt); return MPI_ERR_TYPE; }
    const size_t bytes = count * (size_t)esz;
    BufInfo bi = classify(in), bo = classify(inout);
    std::vector<char> hin, hio;
    const char* pin = static_cast<const char*>(in);
    char* pio = static_cast<char*>(inout);
    int rc = MPI_SUCCESS;
    if (bi.place == Place::Device) {
        hin.resize(bytes);
        if ((rc = copy_any(hin.data(), in, bytes)) != MPI_SUCCESS) return rc;
        pin = hin.data();
    }
    if (bo.place == Place::Device) {
        hio.resize(bytes);
        if ((rc = copy_any(hio.data(), inout, bytes)) != MPI_SUCCESS) return rc;
        pio = hio.data();
    }
    size_t off = 0;
    while (off < count) {
        size_t n = count - off;
        if (n > 0x7fffffff) n = 0x7fffffff;
        int len = (int)n;
        MPI_Datatype d = dt;
        op.user_fn(const_cast<char*>(pin) + off * esz, pio + off * esz, &len, &d);
        off += n;
    }
    if (bo.place == Place::Device) rc = copy_any(inout, hio.data(), bytes);
    return rc;
}

// ---------------------------------------------------------------------------
// collectives: single-rank forms here, multi-rank forms in the transport engine
// ---------------------------------------------------------------------------
// MPIR_Localcopy (mpid/pt2pt.cpp:770-948): a predefined type is one memcpy,
// a derived one goes through the pack / unpack kernels (non-contiguous copy).
int local_copy(const void* src, void* dst, size_t count, MPI_Datatype dt)
{
    if (dtype_is_derived(dt)) return dt_copy_any(src, (int64_t)count, dt, dst, (int64_t)count, dt);
    return copy_any(dst, src, count * (size_t)type_size(dt));
}

int coll_barrier(Comm* c)
{
    if (c->size == 1 || !c->tp) return MPI_SUCCESS;
    return c->tp->barrier();
}

int coll_allreduce(Comm* c, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
                   const OpRef& op, bool nbc)
{
    if (c->size == 1) {
        if (sendbuf == MPI_IN_PLACE) return MPI_SUCCESS;
        return local_copy(sendbuf, recvbuf, count, dt);
    }
    return engine_allreduce(c, sendbuf, recvbuf, count, dt, op, nbc);
}

int coll_reduce(Comm* c, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
                const OpRef& op, int root, bool nbc)
{
    if (c->size == 1) {
        if (sendbuf == MPI_IN_PLACE) return MPI_SUCCESS;
        return local_copy(sendbuf, recvbuf, count, dt);
    }
    return engine_reduce(c, sendbuf, recvbuf, count, dt, op, root, nbc);
}

bool force_async()
{
    // env_is_on (common/mpiutil.cpp:9-61): a 5-wchar buffer, so values of
    // five or more characters read as unset (the default, off)
    static const bool on = [] {
        const char* v = getenv("MSMPI_FORCE_ASYNC_WORKFLOW");
        if (!v || strlen(v) > 4) return false;
        if (strcmp(v, "1") == 0) return true;
        return strcasecmp(v, "on") == 0 || strcasecmp(v, "yes") == 0 || strcasecmp(v, "true") == 0;
    }();
    return on;
}

int coll_reduce_scatter(Comm* c, const void* sendbuf, void* recvbuf, const int* recvcounts,
                        MPI_Datatype dt, const OpRef& op)
{
    if (c->size == 1) {
        if (sendbuf == MPI_IN_PLACE || recvcounts[0] == 0) return MPI_SUCCESS;
        return local_copy(sendbuf, recvbuf, (size_t)recvcounts[0], dt);
    }
    return engine_reduce_scatter(c, sendbuf, recvbuf, recvcounts, dt, op);
}

int coll_scan(Comm* c, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
              const OpRef& op, bool exclusive)
{
    if (c->size == 1) {
        // Exscan leaves rank 0's recvbuf undefined (unchanged here).
        if (exclusive || sendbuf == MPI_IN_PLACE) return MPI_SUCCESS;
        return local_copy(sendbuf, recvbuf, count, dt);
    }
    return engine_scan(c, sendbuf, recvbuf, count, dt, op, exclusive);
}

// ---------------------------------------------------------------------------
// requests: MPI_Request = 0xAC000000 | slot (type DIRECT, kind MPID_REQUEST)
// ---------------------------------------------------------------------------
struct Request {
    bool live = false;
    bool rma = false;              // request-based RMA operation (MPI_Rput ... MPI_Rget_accumulate)
    bool done = false;
    int rc = MPI_SUCCESS;
    bool has_fut = false;
    std::shared_future<int> fut;   // collective running on the engine worker
};

namespace {
std::mutex g_req_mu;
std::deque<Request> g_reqs;     // deque: a Request* stays valid while other threads add slots
constexpr int kReqBase = (int)0xAC000000;

int req_alloc(MPI_Request* out, Request** r)
{
    std::lock_guard<std::mutex> g(g_req_mu);
    size_t i = 0;
    while (i < g_reqs.size() && g_reqs[i].live) ++i;
    if (i == g_reqs.size()) g_reqs.emplace_back();
    g_reqs[i] = Request{};
    g_reqs[i].live = true;
    *out = kReqBase | (int)i;
    *r = &g_reqs[i];
    return MPI_SUCCESS;
}

Request* req_lookup(MPI_Request h)
{
    std::lock_guard<std::mutex> g(g_req_mu);
    size_t i = (size_t)(h & 0x03ffffff);
    if ((h & (int)0xfc000000) != kReqBase || i >= g_reqs.size() || !g_reqs[i].live) return nullptr;
    return &g_reqs[i];
}

void fill_status(MPI_Status* st, int rc)
{
    if (st == MPI_STATUS_IGNORE || st == nullptr) return;
    st->MPI_SOURCE = MPI_UNDEFINED;
    st->MPI_TAG = MPI_UNDEFINED;
    st->MPI_ERROR = rc;
    st->internal[0] = st->internal[1] = 0;
}

}  // namespace

int request_start_generic(Comm* c, std::function<int()> body, MPI_Request* req, MPI_Datatype hold)
{
    if (dtype_is_derived(hold)) {
        dtype_add_ref(hold);
        body = [body, hold]() {
            const int rc = body();
            MPI_Datatype h = hold;
            dtype_free(&h);
            return rc;
        };
    }
    Request* r;
    if (c->size > 1) {
        // The engine worker runs it behind every earlier collective; the
        // caller overlaps host work until MPI_Test/MPI_Wait.
        std::shared_future<int> f = engine_async(std::move(body));
        req_alloc(req, &r);
        r->fut = f;
        r->has_fut = true;
        return MPI_SUCCESS;
    }
    int rc = body();
    req_alloc(req, &r);
    r->done = true;
    r->rc = rc;
    return MPI_SUCCESS;
}

int request_completed_rma(MPI_Request* req, int rc)
{
    Request* r;
    req_alloc(req, &r);
    r->rma = true;
    r->done = true;
    r->rc = rc;
    return MPI_SUCCESS;
}

int request_free(MPI_Request* req)
{
    Request* r = req_lookup(*req);
    if (!r) { set_error("invalid request handle 0x%x", (unsigned)*req); return MPI_ERR_REQUEST; }
    if (!r->rma) {
        set_error("request 0x%x: invalid kind (a nonblocking collective request cannot be freed)", (unsigned)*req);
        return MPI_ERR_OTHER;
    }
    {
        std::lock_guard<std::mutex> g(g_req_mu);
        r->live = false;
    }
    *req = MPI_REQUEST_NULL;
    return MPI_SUCCESS;
}

int request_start_allreduce(Comm* c, const void* sendbuf, void* recvbuf, size_t count,
                            MPI_Datatype dt, const OpRef& op, MPI_Request* req)
{
    return request_start_generic(
        c, [=] { return count ? coll_allreduce(c, sendbuf, recvbuf, count, dt, op, true) : MPI_SUCCESS; },
        req, dt);
}

int request_test(MPI_Request* req, int* flag, MPI_Status* st)
{
    if (*req == MPI_REQUEST_NULL) { *flag = 1; fill_status(st, MPI_SUCCESS); return MPI_SUCCESS; }
    Request* r = req_lookup(*req);
    if (!r) { set_error("invalid request"); return MPI_ERR_REQUEST; }
    if (!r->done && r->has_fut) {
        if (r->fut.wait_for(std::chrono::seconds(0)) != std::future_status::ready) {
            *flag = 0;
            return MPI_SUCCESS;
        }
        r->done = true;
        r->rc = r->fut.get();
    }
    *flag = 1;
    int rc = r->rc;
    r->fut = std::shared_future<int>();
    {
        std::lock_guard<std::mutex> g(g_req_mu);
        r->live = false;
    }
    *req = MPI_REQUEST_NULL;
    fill_status(st, rc);
    return rc;
}

// MpiaRequestValidate (api/mpi_api.h): a live request handle of this process
int request_validate(MPI_Request h)
{
    if (!req_lookup(h)) {
        set_error("invalid request handle 0x%x", (unsigned)h);
        return MPI_ERR_REQUEST;
    }
    return MPI_SUCCESS;
}

// request_ptr->test_complete(): non-destructive; the request stays live
bool request_done(MPI_Request h)
{
    Request* r = req_lookup(h);
    if (!r) return true;
    if (!r->done && r->has_fut) {
        if (r->fut.wait_for(std::chrono::seconds(0)) != std::future_status::ready) return false;
        r->rc = r->fut.get();
        r->done = true;
    }
    return true;
}

// MPIR_Request_get_error: the completed request's error code
int request_error(MPI_Request h)
{
    Request* r = req_lookup(h);
    return r ? r->rc : MPI_ERR_REQUEST;
}

// MPIR_Status_set_empty (include/mpierror.h): source ANY, tag ANY, no error
void status_set_empty(MPI_Status* st)
{
    if (st == MPI_STATUS_IGNORE || st == nullptr) return;
    st->MPI_SOURCE = -2;    // MPI_ANY_SOURCE
    st->MPI_TAG = -1;       // MPI_ANY_TAG
    st->MPI_ERROR = MPI_SUCCESS;
    st->internal[0] = st->internal[1] = 0;
}

// MPID_Progress_wait: the engine worker makes the progress; the caller
// spins briefly, then yields its core in short sleeps
void progress_pause(int iter)
{
    if (iter < 2000) std::this_thread::yield();
    else std::this_thread::sleep_for(std::chrono::microseconds(20));
}

int request_wait(MPI_Request* req, MPI_Status* st)
{
    if (*req == MPI_REQUEST_NULL) { fill_status(st, MPI_SUCCESS); return MPI_SUCCESS; }
    Request* r = req_lookup(*req);
    if (!r) { set_error("invalid request"); return MPI_ERR_REQUEST; }
    if (!r->done && r->has_fut) {
        r->rc = r->fut.get();
        r->done = true;
    }
    int flag;
    return request_test(req, &flag, st);
}

}  // namespace msx
