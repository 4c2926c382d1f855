// msx_api.cpp — MPI-2.2 C entry points of the reduction path.
//
// Each function keeps the reference's argument-validation ORDER, because the
// first failing check decides which error class a caller sees:
//   MPI_Reduce_local           api/mpi_reduce.cpp:304-385
//   MPI_Reduce                 api/mpi_reduce.cpp:46-273
//   MPI_Allreduce              api/mpi_reduce.cpp:1246-1410
//   MPI_Reduce_scatter(_block) api/mpi_reduce.cpp:422-997
//   MPI_Iallreduce / I*        api/mpi_reduce.cpp:1445-1591, 617-790
//   MPI_Scan / MPI_Exscan      api/mpi_reduce.cpp:1626-1900
//   MPI_Op_create/free/commutative  api/mpi_op.cpp:48-260
//   validators MpiaOpValidate / MpiaDatatypeValidate  api/mpi_api.h:113-212, 707-775
//   error return               mpid/error.cpp:85-134 (ERRORS_ARE_FATAL default)
#include <algorithm>
#include <hip/hip_runtime.h>

#include <atomic>
#include <map>
#include <chrono>
#include <mutex>
#include <thread>
#include <unistd.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "../../include/msx.h"
#include "msx_comm.h"
#include "msx_dtype.h"
#include "msx_transport.h"
#include "msx_kernels.h"
#include "msx_runtime.h"
#include "msx_types.h"

using namespace msx;

#define MSX_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

// ---------------------------------------------------------------------------
// user ops: MPID_Op pool for HANDLE_TYPE_DIRECT op handles (include/op.h:82-134)
// ---------------------------------------------------------------------------
struct UserOp {
    MPI_User_function* fn = nullptr;
    bool commute = true;
    bool live = false;
};
std::mutex g_op_mu;
std::vector<UserOp> g_user_ops;
constexpr int kUserOpBase = (int)0x98000000;   // type DIRECT (2) | kind MPID_OP (6)

const char* class_string(int cls)
{
    switch (cls) {
    case MPI_SUCCESS: return "No MPI error";
    case MPI_ERR_BUFFER: return "Invalid buffer pointer";
    case MPI_ERR_COUNT: return "Invalid count argument";
    case MPI_ERR_TYPE: return "Invalid datatype argument";
    case MPI_ERR_TAG: return "Invalid tag argument";
    case MPI_ERR_COMM: return "Invalid communicator";
    case MPI_ERR_RANK: return "Invalid rank";
    case MPI_ERR_ROOT: return "Invalid root";
    case MPI_ERR_GROUP: return "Invalid group";
    case MPI_ERR_OP: return "Invalid MPI_Op";
    case MPI_ERR_ARG: return "Invalid argument";
    case MPI_ERR_UNKNOWN: return "Unknown error";
    case MPI_ERR_TRUNCATE: return "Message truncated";
    case MPI_ERR_OTHER: return "Other MPI error";
    case MPI_ERR_INTERN: return "Internal MPI error";
    case MPI_ERR_REQUEST: return "Invalid MPI_Request";
    case MPI_ERR_NO_MEM: return "Out of memory";
    case MPI_ERR_INFO: return "Invalid info argument";
    case MPI_ERR_WIN: return "Invalid win argument";
    case MPI_ERR_RMA_SYNC: return "Wrong synchronization of RMA calls";
    case MPI_ERR_SIZE: return "Invalid size argument";
    case MPI_ERR_DISP: return "Invalid disp argument";
    default: return "Unknown error class";
    }
}

void not_initialized_exit(const char* fn)
{
    // MpiaIsInitializedOrExit -> MPIR_Err_preOrPostInit (api/mpi_api.h:27)
    fprintf(stderr,
            "Fatal error in %s: Attempting to use an MPI routine %s MPI_Init\n", fn,
            is_finalized() ? "after finalizing" : "before initializing");
    fflush(stderr);
    exit(1);
}

// Entry of every MPI call: MpiaIsInitializedOrExit, then an API range that
// spans the rest of the call (ApiRange, msx_runtime.h).
#define MSX_REQUIRE_INIT(fn)                                                  \
    if (!is_initialized() || is_finalized()) not_initialized_exit(fn);        \
    ApiRange msx_api_range_(fn)

// MPIR_Err_return_comm (mpid/error.cpp:85-134): default handler is the one on
// MPI_COMM_WORLD; ERRORS_ARE_FATAL aborts the job.
int err_return_h(MPI_Errhandler h, const char* fn, int code)
{
    if (code == MPI_SUCCESS) return code;
    if (h == MPI_ERRORS_ARE_FATAL) {
        const char* detail = last_error();
        fprintf(stderr, "Fatal error in %s: %s, error stack:\n%s  %s\n", fn, class_string(code),
                fn, (detail && *detail) ? detail : "");
        fflush(stderr);
        exit(code);
    }
    return code;
}

int err_return(Comm* c, const char* fn, int code)
{
    if (code == MPI_SUCCESS) return code;
    if (c == nullptr) c = world();
    return err_return_h(c ? c->errhandler : MPI_ERRORS_ARE_FATAL, fn, code);
}

// MpiaCommValidateHandle
int v_comm(MPI_Comm c, Comm** out)
{
    *out = nullptr;
    if (c == MPI_COMM_NULL) { set_error("null communicator"); return MPI_ERR_COMM; }
    Comm* p = lookup_comm(c);
    if (!p) { set_error("invalid communicator 0x%x", c); return MPI_ERR_COMM; }
    *out = p;
    return MPI_SUCCESS;
}

// MpiaCommValidateIntracomm: an intercommunicator is MPI_ERR_COMM (**commnotintra)
int v_intracomm(MPI_Comm c, Comm** out)
{
    int rc = v_comm(c, out);
    if (rc == MPI_SUCCESS && (*out)->inter) {
        set_error("an intercommunicator is not valid here (**commnotintra)");
        rc = MPI_ERR_COMM;
    }
    return rc;
}

bool dtype_known(MPI_Datatype dt) { return type_size(dt) >= 0; }

// MpiaDatatypeValidate (mpi_api.h:113-169), predefined datatypes only.
int v_dtype(const void* buf, long long count, MPI_Datatype dt)
{
    if (count == 0) return MPI_SUCCESS;
    if (count < 0) { set_error("negative count %lld", count); return MPI_ERR_COUNT; }
    if (dt == MPI_DATATYPE_NULL) { set_error("null datatype"); return MPI_ERR_TYPE; }
    if (!dtype_known(dt)) { set_error("invalid datatype 0x%x", dt); return MPI_ERR_TYPE; }
    if (buf == nullptr) { set_error("null buffer"); return MPI_ERR_BUFFER; }
    return MPI_SUCCESS;
}

// MpiaDatatypeValidate (mpi_api.h:113-164) with derived datatypes: the
// one-sided calls and MPI_Reduce_local (user ops) accept committed derived types.
int v_dtype_any(const void* buf, long long count, MPI_Datatype dt)
{
    if (count == 0) return MPI_SUCCESS;
    if (count < 0) { set_error("negative count %lld", count); return MPI_ERR_COUNT; }
    if (dt == MPI_DATATYPE_NULL) { set_error("null datatype"); return MPI_ERR_TYPE; }
    if (!dtype_is_derived(dt)) return v_dtype(buf, count, dt);
    Dtype* t = dtype_lookup(dt);
    if (!t) { set_error("invalid datatype 0x%x", dt); return MPI_ERR_TYPE; }
    if (!t->committed) { set_error("datatype 0x%x is not committed", dt); return MPI_ERR_TYPE; }
    if (buf == nullptr && t->true_lb == 0 && t->size > 0) { set_error("null buffer"); return MPI_ERR_BUFFER; }
    return MPI_SUCCESS;
}

// MpiaDatatypeValidateBuffer (mpi_api.h:190-212)
int v_buffer(MPI_Datatype dt, const void* buf, long long count)
{
    if (dtype_is_derived(dt)) {
        const Dtype* t = dtype_lookup(dt);
        if (buf == nullptr && count > 0 && t && t->true_lb == 0 && t->size > 0) {
            set_error("null buffer");
            return MPI_ERR_BUFFER;
        }
        return MPI_SUCCESS;
    }
    if (buf == nullptr && count > 0 && type_size(dt) > 0) {
        set_error("null buffer");
        return MPI_ERR_BUFFER;
    }
    return MPI_SUCCESS;
}

// MpiaOpValidateHandle (mpi_api.h:707-728)
int v_op_handle(MPI_Op op, OpRef* out)
{
    if (handle_kind(op) != OBJ_OP || handle_type(op) == HT_INVALID) {
        set_error("invalid MPI_Op 0x%x", op);
        return MPI_ERR_OP;
    }
    if (handle_type(op) == HT_BUILTIN) {
        int idx = op & 0xff;
        if (idx < O_MAX || idx > O_NOOP || (op & 0x03ffff00)) {
            set_error("invalid builtin MPI_Op 0x%x", op);
            return MPI_ERR_OP;
        }
        out->opidx = idx;
        out->user_fn = nullptr;
        out->commutative = (idx != O_REPLACE && idx != O_NOOP);
        return MPI_SUCCESS;
    }
    std::lock_guard<std::mutex> g(g_op_mu);
    size_t idx = (size_t)(op & 0x03ffffff);
    if (handle_type(op) != HT_DIRECT || idx >= g_user_ops.size() || !g_user_ops[idx].live) {
        set_error("MPI_Op 0x%x does not name a live operation", op);
        return MPI_ERR_OP;
    }
    out->opidx = O_NULL;
    out->user_fn = g_user_ops[idx].fn;
    out->commutative = g_user_ops[idx].commute;
    return MPI_SUCCESS;
}

// MpiaOpValidate (mpi_api.h:731-775), rmaOp = false
int v_op(MPI_Op op, MPI_Datatype dt, OpRef* out)
{
    int rc = v_op_handle(op, out);
    if (rc != MPI_SUCCESS) return rc;
    if (out->opidx == O_REPLACE) { set_error("MPI_REPLACE not allowed"); return MPI_ERR_OP; }
    if (out->opidx == O_NOOP) { set_error("MPI_NO_OP not allowed"); return MPI_ERR_OP; }
    if (out->opidx != O_NULL) {
        rc = op_check_dtype(out->opidx, dt);
        if (rc != MPI_SUCCESS) {
            set_error("MPI_Op 0x%x is not defined for datatype 0x%x", op, dt);
            return rc;
        }
    }
    return MPI_SUCCESS;
}

}  // namespace

// ---- entry-point helpers shared with msx_dtype_api.cpp -----------------------
namespace msx {
void api_require_init(const char* fn)
{
    if (!is_initialized() || is_finalized()) not_initialized_exit(fn);
}
// (datatype entry points are not traced: no device work of their own except
// MPI_Pack / MPI_Unpack, which open their own range)
int api_err_return(const char* fn, int code) { return err_return(nullptr, fn, code); }
int api_comm_valid(MPI_Comm comm)
{
    Comm* c;
    return v_comm(comm, &c);
}
}  // namespace msx

// ===========================================================================
// environment
// ===========================================================================
namespace {
int g_thread_level = MPI_THREAD_SINGLE;     // Mpi.ThreadLevel
std::thread::id g_main_thread;              // the thread that initialised MPI
}

MSX_EXPORT int MPI_Init(int* argc, char*** argv)
{
    (void)argc; (void)argv;
    if (is_initialized()) {
        set_error("MPI_Init called twice");
        return err_return(nullptr, "MPI_Init", MPI_ERR_OTHER);
    }
    int rc = world_init();
    if (rc != MPI_SUCCESS) {
        fprintf(stderr, "Fatal error in MPI_Init: %s\n", last_error());
        exit(rc);
    }
    g_thread_level = MPI_THREAD_SINGLE;       // mpi_env.cpp:167
    g_main_thread = std::this_thread::get_id();
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Init_thread(int* argc, char*** argv, int required, int* provided)
{
    int rc = MPI_Init(argc, argv);
    // Kernels are reentrant; the host staging path and bootstrap are locked
    // (mid/env.cpp:1071-1078 grants up to MULTIPLE).
    const int level = required > MPI_THREAD_MULTIPLE ? MPI_THREAD_MULTIPLE : required;
    if (rc == MPI_SUCCESS) g_thread_level = level;
    if (provided) *provided = level;
    return rc;
}

MSX_EXPORT int MPI_Finalize(void)
{
    MSX_REQUIRE_INIT("MPI_Finalize");
    return world_finalize();
}

MSX_EXPORT int MPI_Initialized(int* flag)
{
    if (!flag) return MPI_ERR_ARG;
    *flag = is_initialized() ? 1 : 0;
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Finalized(int* flag)
{
    if (!flag) return MPI_ERR_ARG;
    *flag = is_finalized() ? 1 : 0;
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Abort(MPI_Comm comm, int errorcode)
{
    (void)comm;
    fprintf(stderr, "MPI_Abort called with error code %d\n", errorcode);
    fflush(stderr);
    exit(errorcode);
}

MSX_EXPORT double MPI_Wtime(void)
{
    using namespace std::chrono;
    return duration<double>(steady_clock::now().time_since_epoch()).count();
}

// the resolution of MPI_Wtime's clock (mpi_env.cpp:767)
MSX_EXPORT double MPI_Wtick(void)
{
    using namespace std::chrono;
    return duration<double>(steady_clock::duration(1)).count();
}

// mpi_env.cpp:575-610: the level MPI_Init / MPI_Init_thread provided
MSX_EXPORT int MPI_Query_thread(int* provided)
{
    MSX_REQUIRE_INIT("MPI_Query_thread");
    if (!provided) { set_error("**nullptr provided"); return err_return(nullptr, "MPI_Query_thread", MPI_ERR_ARG); }
    *provided = g_thread_level;
    return MPI_SUCCESS;
}

// mpi_env.cpp:463-500: is the caller the thread that initialised MPI
MSX_EXPORT int MPI_Is_thread_main(int* flag)
{
    MSX_REQUIRE_INIT("MPI_Is_thread_main");
    if (!flag) { set_error("**nullptr flag"); return err_return(nullptr, "MPI_Is_thread_main", MPI_ERR_ARG); }
    *flag = std::this_thread::get_id() == g_main_thread ? 1 : 0;
    return MPI_SUCCESS;
}

// mpi_env.cpp:630-680; callable before MPI_Init
MSX_EXPORT int MPI_Get_version(int* version, int* subversion)
{
    if (!version || !subversion) {
        set_error("**nullptr %s", version ? "subversion" : "version");
        return is_initialized() ? err_return(nullptr, "MPI_Get_version", MPI_ERR_ARG) : MPI_ERR_ARG;
    }
    *version = MPI_VERSION;
    *subversion = MPI_SUBVERSION;
    return MPI_SUCCESS;
}

// mpi_env.cpp:1095-1140 (MPID_Get_processor_name: the host name)
MSX_EXPORT int MPI_Get_processor_name(char* name, int* resultlen)
{
    MSX_REQUIRE_INIT("MPI_Get_processor_name");
    if (!name || !resultlen) {
        set_error("**nullptr %s", name ? "resultlen" : "name");
        return err_return(nullptr, "MPI_Get_processor_name", MPI_ERR_ARG);
    }
    char host[MPI_MAX_PROCESSOR_NAME] = {0};
    if (gethostname(host, sizeof(host) - 1) != 0) snprintf(host, sizeof(host), "localhost");
    const size_t n = strnlen(host, MPI_MAX_PROCESSOR_NAME - 1);
    memcpy(name, host, n);
    name[n] = 0;
    *resultlen = (int)n;
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Comm_rank(MPI_Comm comm, int* rank)
{
    MSX_REQUIRE_INIT("MPI_Comm_rank");
    Comm* c;
    int rc = v_comm(comm, &c);
    if (rc == MPI_SUCCESS && !rank) { set_error("null rank"); rc = MPI_ERR_ARG; }
    if (rc != MPI_SUCCESS) return err_return(nullptr, "MPI_Comm_rank", rc);
    *rank = c->rank;
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Comm_size(MPI_Comm comm, int* size)
{
    MSX_REQUIRE_INIT("MPI_Comm_size");
    Comm* c;
    int rc = v_comm(comm, &c);
    if (rc == MPI_SUCCESS && !size) { set_error("null size"); rc = MPI_ERR_ARG; }
    if (rc != MPI_SUCCESS) return err_return(nullptr, "MPI_Comm_size", rc);
    *size = c->size;
    return MPI_SUCCESS;
}

// ---- derived communicators (api/mpi_comm.cpp: MPI_Comm_split / dup / free) ------
// Reductions on sub-communicators need them: each group gets its own
// transport (hub, shared-memory barrier, engine windows) and runs the same
// reference-order schedules over its own ranks.
MSX_EXPORT int MPI_Comm_split(MPI_Comm comm, int color, int key, MPI_Comm* newcomm)
{
    MSX_REQUIRE_INIT("MPI_Comm_split");
    Comm* c;
    int rc = v_intracomm(comm, &c);     // intercommunicator splits are not supported
    if (rc == MPI_SUCCESS && !newcomm) { set_error("null newcomm"); rc = MPI_ERR_ARG; }
    if (rc == MPI_SUCCESS && color < 0 && color != MPI_UNDEFINED) {
        set_error("color %d is negative and not MPI_UNDEFINED", color);
        rc = MPI_ERR_ARG;
    }
    Comm* n = nullptr;
    if (rc == MPI_SUCCESS) rc = engine_comm_split(c, color, key, &n);
    if (rc != MPI_SUCCESS) return err_return(c, "MPI_Comm_split", rc);
    *newcomm = n ? comm_register(n) : MPI_COMM_NULL;
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Comm_dup(MPI_Comm comm, MPI_Comm* newcomm)
{
    MSX_REQUIRE_INIT("MPI_Comm_dup");
    Comm* c;
    int rc = v_comm(comm, &c);
    if (rc == MPI_SUCCESS && !newcomm) { set_error("null newcomm"); rc = MPI_ERR_ARG; }
    Comm* n = nullptr;
    if (rc == MPI_SUCCESS && c->inter) rc = engine_intercomm_dup(c, &n);
    else if (rc == MPI_SUCCESS) rc = engine_comm_split(c, 0, c->rank, &n);   // same group, same order
    if (rc != MPI_SUCCESS) return err_return(c, "MPI_Comm_dup", rc);
    *newcomm = comm_register(n);
    return MPI_SUCCESS;
}

// api/mpi_comm.cpp:184-248, MPIR_Comm_create_intra (mpid/comm.cpp:1027-1128):
// collective over `comm`; members get a communicator ranked in group order,
// the others MPI_COMM_NULL.  A group member outside `comm` is MPI_ERR_GROUP
// (**groupnotincomm, comm.cpp:977) on the members, after the collective step
// every process takes (here the split, there the context id).
MSX_EXPORT int MPI_Comm_create(MPI_Comm comm, MPI_Group group, MPI_Comm* newcomm)
{
    MSX_REQUIRE_INIT("MPI_Comm_create");
    Comm* c;
    int rc = v_intracomm(comm, &c);     // MPIR_Comm_create_inter is not supported
    if (rc != MPI_SUCCESS) return err_return(nullptr, "MPI_Comm_create", rc);
    std::vector<int> members;
    rc = group_members(group, &members);
    if (rc == MPI_SUCCESS && !newcomm) { set_error("null newcomm"); rc = MPI_ERR_ARG; }
    if (rc != MPI_SUCCESS) return err_return(c, "MPI_Comm_create", rc);
    const int me = c->lpid.empty() ? c->rank : c->lpid[(size_t)c->rank];
    int grank = MPI_UNDEFINED;
    bool valid = true;
    for (size_t i = 0; i < members.size(); ++i) {
        if (members[i] == me) grank = (int)i;
        if (std::find(c->lpid.begin(), c->lpid.end(), members[i]) == c->lpid.end()) valid = false;
    }
    Comm* n = nullptr;
    rc = engine_comm_split(c, grank != MPI_UNDEFINED && valid ? 0 : MPI_UNDEFINED, grank, &n);
    if (rc == MPI_SUCCESS && grank != MPI_UNDEFINED && !valid) {
        set_error("**groupnotincomm: a group member is not in the communicator");
        rc = MPI_ERR_GROUP;
    }
    if (rc != MPI_SUCCESS) return err_return(c, "MPI_Comm_create", rc);
    *newcomm = n ? comm_register(n) : MPI_COMM_NULL;
    return MPI_SUCCESS;
}

// api/mpi_comm.cpp:51-157 (intracommunicators): IDENT for the same handle,
// else the groups' relation with IDENT promoted to CONGRUENT
MSX_EXPORT int MPI_Comm_compare(MPI_Comm comm1, MPI_Comm comm2, int* result)
{
    MSX_REQUIRE_INIT("MPI_Comm_compare");
    Comm *c1, *c2 = nullptr;
    int rc = v_comm(comm1, &c1);
    if (rc == MPI_SUCCESS) rc = v_comm(comm2, &c2);
    if (rc == MPI_SUCCESS && !result) { set_error("**nullptr result"); rc = MPI_ERR_ARG; }
    if (rc != MPI_SUCCESS) return err_return(nullptr, "MPI_Comm_compare", rc);
    auto rel = [](const std::vector<int>& x, const std::vector<int>& y) {
        if (x == y) return MPI_IDENT;
        std::vector<int> a = x, b = y;
        std::sort(a.begin(), a.end());
        std::sort(b.begin(), b.end());
        return a == b ? MPI_SIMILAR : MPI_UNEQUAL;
    };
    if (c1->inter != c2->inter) {
        *result = MPI_UNEQUAL;
    } else if (comm1 == comm2) {
        *result = MPI_IDENT;
    } else {
        // groups (and, for intercommunicators, remote groups too: the weaker
        // relation of the two); identical groups under another handle are
        // congruent
        int r = rel(c1->lpid, c2->lpid);
        if (c1->inter) r = std::max(r, rel(c1->remote_lpid, c2->remote_lpid));
        *result = r == MPI_IDENT ? MPI_CONGRUENT : r;
    }
    return MPI_SUCCESS;
}

// api/mpi_comm.cpp:1386-1420
MSX_EXPORT int MPI_Comm_test_inter(MPI_Comm comm, int* flag)
{
    MSX_REQUIRE_INIT("MPI_Comm_test_inter");
    Comm* c;
    int rc = v_comm(comm, &c);
    if (rc == MPI_SUCCESS && !flag) { set_error("**nullptr flag"); rc = MPI_ERR_ARG; }
    if (rc != MPI_SUCCESS) return err_return(nullptr, "MPI_Comm_test_inter", rc);
    *flag = c->inter ? 1 : 0;
    return MPI_SUCCESS;
}

// ---- intercommunicators (api/mpi_comm.cpp:835-960, 1482-1830) ------------------
MSX_EXPORT int MPI_Comm_remote_size(MPI_Comm comm, int* size)
{
    MSX_REQUIRE_INIT("MPI_Comm_remote_size");
    Comm* c;
    int rc = v_comm(comm, &c);
    if (rc == MPI_SUCCESS && !c->inter) { set_error("**commnotinter"); rc = MPI_ERR_COMM; }
    if (rc == MPI_SUCCESS && !size) { set_error("**nullptr size"); rc = MPI_ERR_ARG; }
    if (rc != MPI_SUCCESS) return err_return(c, "MPI_Comm_remote_size", rc);
    *size = (int)c->remote_lpid.size();
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Comm_remote_group(MPI_Comm comm, MPI_Group* group)
{
    MSX_REQUIRE_INIT("MPI_Comm_remote_group");
    Comm* c;
    int rc = v_comm(comm, &c);
    if (rc == MPI_SUCCESS && !c->inter) { set_error("**commnotinter"); rc = MPI_ERR_COMM; }
    if (rc == MPI_SUCCESS && !group) { set_error("**nullptr group"); rc = MPI_ERR_ARG; }
    if (rc == MPI_SUCCESS) rc = group_create(c->remote_lpid, group);
    return err_return(c, "MPI_Comm_remote_group", rc);
}

// The leaders exchange their groups over the world mailbox; both groups then
// join one bootstrap hub (the low group's rank 0), which carries the windows
// and flags of the transfers between the groups.
MSX_EXPORT int MPI_Intercomm_create(MPI_Comm local_comm, int local_leader, MPI_Comm peer_comm, int remote_leader,
                                    int tag, MPI_Comm* newintercomm)
{
    MSX_REQUIRE_INIT("MPI_Intercomm_create");
    Comm *c, *peer = nullptr;
    int rc = v_intracomm(local_comm, &c);
    if (rc == MPI_SUCCESS && (local_leader < 0 || local_leader >= c->size)) {
        set_error("**ranklocal %d %d", local_leader, c->size);
        rc = MPI_ERR_RANK;
    }
    if (rc == MPI_SUCCESS && c->rank == local_leader) {
        rc = v_comm(peer_comm, &peer);
        if (rc == MPI_SUCCESS && peer->inter) {
            set_error("an intercommunicator as peer_comm is not supported");
            rc = MPI_ERR_COMM;
        }
        if (rc == MPI_SUCCESS && (remote_leader < 0 || remote_leader >= peer->size)) {
            set_error("**rankremote %d %d", remote_leader, peer->size);
            rc = MPI_ERR_RANK;
        }
        if (rc == MPI_SUCCESS && peer->rank == remote_leader) {
            set_error("**ranksdistinct");
            rc = MPI_ERR_RANK;
        }
    }
    if (rc == MPI_SUCCESS && !newintercomm) { set_error("**nullptr newintercomm"); rc = MPI_ERR_ARG; }
    Comm* n = nullptr;
    if (rc == MPI_SUCCESS) rc = engine_intercomm_create(c, local_leader, peer, remote_leader, tag, &n);
    if (rc != MPI_SUCCESS) return err_return(c, "MPI_Intercomm_create", rc);
    *newintercomm = comm_register(n);
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Intercomm_merge(MPI_Comm intercomm, int high, MPI_Comm* newintracomm)
{
    MSX_REQUIRE_INIT("MPI_Intercomm_merge");
    Comm* c;
    int rc = v_comm(intercomm, &c);
    if (rc == MPI_SUCCESS && !c->inter) { set_error("**commnotinter"); rc = MPI_ERR_COMM; }
    if (rc == MPI_SUCCESS && !newintracomm) { set_error("**nullptr newintracomm"); rc = MPI_ERR_ARG; }
    Comm* n = nullptr;
    if (rc == MPI_SUCCESS) rc = engine_intercomm_merge(c, high, &n);
    if (rc != MPI_SUCCESS) return err_return(c, "MPI_Intercomm_merge", rc);
    *newintracomm = comm_register(n);
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Comm_free(MPI_Comm* comm)
{
    MSX_REQUIRE_INIT("MPI_Comm_free");
    if (!comm) { set_error("null comm"); return err_return(nullptr, "MPI_Comm_free", MPI_ERR_ARG); }
    Comm* c;
    int rc = v_comm(*comm, &c);
    if (rc != MPI_SUCCESS) return err_return(nullptr, "MPI_Comm_free", rc);
    if (c == lookup_comm(MPI_COMM_WORLD) || c == lookup_comm(MPI_COMM_SELF)) {
        set_error("a predefined communicator cannot be freed (**commperm)");
        return err_return(c, "MPI_Comm_free", MPI_ERR_COMM);
    }
    rc = engine_comm_free(c);
    comm_unregister(c);
    delete c;
    *comm = MPI_COMM_NULL;
    return rc == MPI_SUCCESS ? MPI_SUCCESS : err_return(nullptr, "MPI_Comm_free", rc);
}

MSX_EXPORT int MPI_Barrier(MPI_Comm comm)
{
    MSX_REQUIRE_INIT("MPI_Barrier");
    Comm* c;
    int rc = v_comm(comm, &c);
    if (rc == MPI_SUCCESS) rc = coll_barrier(c->inter ? c->uni : c);   // intercomm: both groups
    return err_return(c, "MPI_Barrier", rc);
}

MSX_EXPORT int MPI_Comm_set_errhandler(MPI_Comm comm, MPI_Errhandler eh)
{
    MSX_REQUIRE_INIT("MPI_Comm_set_errhandler");
    Comm* c;
    int rc = v_comm(comm, &c);
    if (rc == MPI_SUCCESS && eh != MPI_ERRORS_ARE_FATAL && eh != MPI_ERRORS_RETURN) {
        set_error("unsupported errhandler 0x%x", eh);
        rc = MPI_ERR_ARG;
    }
    if (rc != MPI_SUCCESS) return err_return(c, "MPI_Comm_set_errhandler", rc);
    c->errhandler = eh;
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Comm_get_errhandler(MPI_Comm comm, MPI_Errhandler* eh)
{
    MSX_REQUIRE_INIT("MPI_Comm_get_errhandler");
    Comm* c;
    int rc = v_comm(comm, &c);
    if (rc == MPI_SUCCESS && !eh) rc = MPI_ERR_ARG;
    if (rc != MPI_SUCCESS) return err_return(c, "MPI_Comm_get_errhandler", rc);
    *eh = c->errhandler;
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Error_class(int errorcode, int* errorclass)
{
    if (!errorclass) return MPI_ERR_ARG;
    // This library returns error classes as codes.
    *errorclass = errorcode & 0x7f;
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Error_string(int errorcode, char* str, int* len)
{
    if (!str || !len) return MPI_ERR_ARG;
    int n = snprintf(str, MPI_MAX_ERROR_STRING, "%s", class_string(errorcode & 0x7f));
    *len = n < MPI_MAX_ERROR_STRING ? n : MPI_MAX_ERROR_STRING - 1;
    return MPI_SUCCESS;
}

// ===========================================================================
// operations (api/mpi_op.cpp:48-260)
// ===========================================================================
MSX_EXPORT int MPI_Op_create(MPI_User_function* user_fn, int commute, MPI_Op* op)
{
    MSX_REQUIRE_INIT("MPI_Op_create");
    int rc = MPI_SUCCESS;
    if (user_fn == nullptr) { set_error("null user_fn"); rc = MPI_ERR_ARG; }
    else if (op == nullptr) { set_error("null op"); rc = MPI_ERR_ARG; }
    if (rc != MPI_SUCCESS) return err_return(nullptr, "MPI_Op_create", rc);
    std::lock_guard<std::mutex> g(g_op_mu);
    size_t idx = 0;
    while (idx < g_user_ops.size() && g_user_ops[idx].live) ++idx;
    if (idx == g_user_ops.size()) g_user_ops.push_back(UserOp{});
    g_user_ops[idx] = UserOp{user_fn, commute != 0, true};
    *op = kUserOpBase | (int)idx;
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Op_free(MPI_Op* op)
{
    MSX_REQUIRE_INIT("MPI_Op_free");
    int rc = MPI_SUCCESS;
    OpRef r;
    if (op == nullptr) { set_error("null op"); rc = MPI_ERR_ARG; }
    else rc = v_op_handle(*op, &r);
    if (rc == MPI_SUCCESS && r.opidx != O_NULL) {
        set_error("cannot free permanent MPI_Op");   // "**permop" mpi_op.cpp:169-173
        rc = MPI_ERR_OP;
    }
    if (rc != MPI_SUCCESS) return err_return(nullptr, "MPI_Op_free", rc);
    std::lock_guard<std::mutex> g(g_op_mu);
    g_user_ops[(size_t)(*op & 0x03ffffff)].live = false;
    *op = MPI_OP_NULL;
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Op_commutative(MPI_Op op, int* commute)
{
    MSX_REQUIRE_INIT("MPI_Op_commutative");
    OpRef r;
    int rc = v_op_handle(op, &r);
    if (rc == MPI_SUCCESS && commute == nullptr) { set_error("null commute"); rc = MPI_ERR_ARG; }
    if (rc != MPI_SUCCESS) return err_return(nullptr, "MPI_Op_commutative", rc);
    *commute = r.commutative ? 1 : 0;
    return MPI_SUCCESS;
}

// ===========================================================================
// MPI_Reduce_local (api/mpi_reduce.cpp:304-385)
// ===========================================================================
MSX_EXPORT int MPI_Reduce_local(const void* inbuf, void* inoutbuf, int count,
                                MPI_Datatype datatype, MPI_Op op)
{
    MSX_REQUIRE_INIT("MPI_Reduce_local");
    if (count == 0) return MPI_SUCCESS;             // :319-322, before any check
    OpRef r;
    int rc = v_op(op, datatype, &r);                // :324
    if (rc == MPI_SUCCESS && inbuf == MPI_IN_PLACE) { set_error("inbuf is MPI_IN_PLACE"); rc = MPI_ERR_BUFFER; }
    if (rc == MPI_SUCCESS && inoutbuf == MPI_IN_PLACE) { set_error("inoutbuf is MPI_IN_PLACE"); rc = MPI_ERR_BUFFER; }
    if (rc == MPI_SUCCESS) rc = v_dtype_any(inbuf, count, datatype);   // :343
    if (rc == MPI_SUCCESS && inbuf == inoutbuf) { set_error("inbuf aliases inoutbuf"); rc = MPI_ERR_BUFFER; }
    // MSX_REDUCE_LOCAL_GPUS=k (k = 0: every GPU of the node): host operands
    // split over k GPUs' PCIe links (reduce_local_multi); for single-process
    // use -- in a job with one rank per GPU each rank would use them all
    static const int multi = [] {
        const char* e = getenv("MSX_REDUCE_LOCAL_GPUS");
        return e ? atoi(e) : 1;
    }();
    if (rc == MPI_SUCCESS && multi != 1 && r.opidx != O_NULL && type_info(datatype))
        rc = reduce_local_multi(r.opidx, type_info(datatype)->kind, inbuf, inoutbuf, (size_t)count, multi);
    else if (rc == MPI_SUCCESS)
        rc = local_combine(r, datatype, inbuf, inoutbuf, (size_t)count);
    return err_return(nullptr, "MPI_Reduce_local", rc);
}

// ===========================================================================
// reduction collectives
// ===========================================================================
namespace {

// api/mpi_reduce.cpp:1073-1160: recvbuf / sendbuf rules of MPI_Allreduce
// (MPI_IN_PLACE is not allowed on an intercommunicator)
int v_allreduce_bufs(Comm* c, const void* sendbuf, void* recvbuf, int count, MPI_Datatype datatype)
{
    if (recvbuf == MPI_IN_PLACE) { set_error("recvbuf is MPI_IN_PLACE"); return MPI_ERR_BUFFER; }
    if (sendbuf == MPI_IN_PLACE) {
        if (c->inter) { set_error("**sendbuf_inplace on an intercommunicator"); return MPI_ERR_BUFFER; }
        return MPI_SUCCESS;
    }
    int rc = v_buffer(datatype, sendbuf, count);
    if (rc == MPI_SUCCESS && sendbuf == recvbuf) { set_error("sendbuf aliases recvbuf"); rc = MPI_ERR_BUFFER; }
    return rc;
}

// api/mpi_reduce.cpp:46-273: MPI_Reduce's checks; on an intercommunicator the
// root is MPI_ROOT (receives), MPI_PROC_NULL (does nothing) or a remote rank
// (sends).  *skip: nothing to do on this process.
int v_reduce(Comm* c, const void* sendbuf, void* recvbuf, int count, MPI_Datatype datatype, MPI_Op op, int root,
             OpRef* r, bool* skip)
{
    *skip = false;
    if (c->inter) {
        if (root == MPI_PROC_NULL) { *skip = true; return MPI_SUCCESS; }
        if (root == MPI_ROOT) {
            int rc = v_dtype_any(recvbuf, count, datatype);
            return rc == MPI_SUCCESS ? v_op(op, datatype, r) : rc;
        }
        if (root < 0 || root >= (int)c->remote_lpid.size()) { set_error("invalid root %d", root); return MPI_ERR_ROOT; }
        if (count > 0 && sendbuf == MPI_IN_PLACE) { set_error("**sendbuf_inplace"); return MPI_ERR_BUFFER; }
        int rc = v_dtype_any(sendbuf, count, datatype);
        return rc == MPI_SUCCESS ? v_op(op, datatype, r) : rc;
    }
    if (root < 0 || root >= c->size) { set_error("invalid root %d", root); return MPI_ERR_ROOT; }
    int rc = v_dtype_any(sendbuf, count, datatype);
    if (rc == MPI_SUCCESS) rc = v_op(op, datatype, r);
    if (rc != MPI_SUCCESS) return rc;
    if (c->rank == root) {
        if (recvbuf == MPI_IN_PLACE) { set_error("recvbuf is MPI_IN_PLACE"); return MPI_ERR_BUFFER; }
        rc = v_buffer(datatype, recvbuf, count);
        if (rc == MPI_SUCCESS && count > 0 && sendbuf == recvbuf) { set_error("sendbuf aliases recvbuf"); rc = MPI_ERR_BUFFER; }
    } else if (count > 0 && sendbuf == MPI_IN_PLACE) {
        set_error("sendbuf is MPI_IN_PLACE on a non-root rank");
        rc = MPI_ERR_BUFFER;
    }
    return rc;
}

int run_reduce(Comm* c, const void* sendbuf, void* recvbuf, size_t n, MPI_Datatype datatype, const OpRef& r, int root,
               bool nbc)
{
    if (n == 0) return MPI_SUCCESS;
    return c->inter ? engine_inter_reduce(c, sendbuf, recvbuf, n, datatype, r, root)
                    : coll_reduce(c, sendbuf, recvbuf, n, datatype, r, root, nbc);
}

int run_reduce_scatter(Comm* c, const void* sendbuf, void* recvbuf, const int* counts, MPI_Datatype datatype,
                       const OpRef& r)
{
    return c->inter ? engine_inter_reduce_scatter(c, sendbuf, recvbuf, counts, datatype, r)
                    : coll_reduce_scatter(c, sendbuf, recvbuf, counts, datatype, r);
}

}  // namespace

MSX_EXPORT int MPI_Allreduce(const void* sendbuf, void* recvbuf, int count, MPI_Datatype datatype,
                             MPI_Op op, MPI_Comm comm)
{
    MSX_REQUIRE_INIT("MPI_Allreduce");
    Comm* c;
    OpRef r;
    int rc = v_comm(comm, &c);
    if (rc == MPI_SUCCESS) rc = v_dtype_any(recvbuf, count, datatype);
    if (rc == MPI_SUCCESS) rc = v_op(op, datatype, &r);
    if (rc == MPI_SUCCESS && count > 0) rc = v_allreduce_bufs(c, sendbuf, recvbuf, count, datatype);
    if (rc == MPI_SUCCESS && count > 0)
        rc = c->inter ? engine_inter_allreduce(c, sendbuf, recvbuf, (size_t)count, datatype, r)
                      : coll_allreduce(c, sendbuf, recvbuf, (size_t)count, datatype, r, force_async());
    return err_return(c, "MPI_Allreduce", rc);
}

MSX_EXPORT int MPI_Reduce(const void* sendbuf, void* recvbuf, int count, MPI_Datatype datatype,
                          MPI_Op op, int root, MPI_Comm comm)
{
    MSX_REQUIRE_INIT("MPI_Reduce");
    Comm* c;
    OpRef r;
    bool skip = false;
    int rc = v_comm(comm, &c);
    if (rc == MPI_SUCCESS) rc = v_reduce(c, sendbuf, recvbuf, count, datatype, op, root, &r, &skip);
    if (rc == MPI_SUCCESS && !skip) rc = run_reduce(c, sendbuf, recvbuf, (size_t)count, datatype, r, root, force_async());
    return err_return(c, "MPI_Reduce", rc);
}

namespace {

int validate_reduce_scatter(Comm* c, const void* sendbuf, void* recvbuf, const int* recvcounts,
                            MPI_Datatype datatype, MPI_Op op, OpRef* r)
{
    if (!recvcounts) { set_error("null recvcounts"); return MPI_ERR_ARG; }
    int sentinel = 0;
    for (int i = 0; i < c->size; ++i) {
        if (recvcounts[i] < 0) { set_error("negative recvcount %d", recvcounts[i]); return MPI_ERR_COUNT; }
        sentinel |= recvcounts[i];   // the reference's OR trick (mpi_reduce.cpp:833-847)
    }
    int rc = v_dtype_any(sendbuf, sentinel, datatype);
    if (rc == MPI_SUCCESS) rc = v_op(op, datatype, r);
    if (rc == MPI_SUCCESS && recvcounts[c->rank] > 0) {
        if (recvbuf == MPI_IN_PLACE) { set_error("recvbuf is MPI_IN_PLACE"); rc = MPI_ERR_BUFFER; }
        else if (sendbuf != MPI_IN_PLACE) {
            rc = v_buffer(datatype, recvbuf, recvcounts[c->rank]);
            if (rc == MPI_SUCCESS && sendbuf == recvbuf) { set_error("sendbuf aliases recvbuf"); rc = MPI_ERR_BUFFER; }
        } else if (c->inter) {                // mpi_reduce.cpp:893-897
            set_error("**sendbuf_inplace on an intercommunicator");
            rc = MPI_ERR_BUFFER;
        }
    }
    return rc;
}

}  // namespace

MSX_EXPORT int MPI_Reduce_scatter(const void* sendbuf, void* recvbuf, const int recvcounts[],
                                  MPI_Datatype datatype, MPI_Op op, MPI_Comm comm)
{
    MSX_REQUIRE_INIT("MPI_Reduce_scatter");
    Comm* c;
    OpRef r;
    int rc = v_comm(comm, &c);
    if (rc == MPI_SUCCESS) rc = validate_reduce_scatter(c, sendbuf, recvbuf, recvcounts, datatype, op, &r);
    if (rc == MPI_SUCCESS) rc = run_reduce_scatter(c, sendbuf, recvbuf, recvcounts, datatype, r);
    return err_return(c, "MPI_Reduce_scatter", rc);
}

MSX_EXPORT int MPI_Reduce_scatter_block(const void* sendbuf, void* recvbuf, int recvcount,
                                        MPI_Datatype datatype, MPI_Op op, MPI_Comm comm)
{
    MSX_REQUIRE_INIT("MPI_Reduce_scatter_block");
    Comm* c;
    OpRef r;
    int rc = v_comm(comm, &c);
    std::vector<int> counts;
    if (rc == MPI_SUCCESS && recvcount < 0) { set_error("negative recvcount"); rc = MPI_ERR_COUNT; }
    if (rc == MPI_SUCCESS) {
        counts.assign((size_t)c->size, recvcount);
        rc = validate_reduce_scatter(c, sendbuf, recvbuf, counts.data(), datatype, op, &r);
    }
    if (rc == MPI_SUCCESS) rc = run_reduce_scatter(c, sendbuf, recvbuf, counts.data(), datatype, r);
    return err_return(c, "MPI_Reduce_scatter_block", rc);
}

namespace {

// request == nullptr: blocking MPI_(Ex)scan; else MPI_I(ex)scan
// (api/mpi_reduce.cpp:1920-2068 validate like the blocking forms)
int scan_common(const char* fn, const void* sendbuf, void* recvbuf, int count, MPI_Datatype datatype,
                MPI_Op op, MPI_Comm comm, bool exclusive, MPI_Request* request = nullptr,
                bool nonblocking = false)
{
    Comm* c;
    OpRef r;
    int rc = v_intracomm(comm, &c);      // scans are defined on intracommunicators only
    if (rc == MPI_SUCCESS && nonblocking) {
        if (request == nullptr) { set_error("null request"); rc = MPI_ERR_ARG; }
        else *request = MPI_REQUEST_NULL;
    }
    if (rc == MPI_SUCCESS) rc = v_dtype_any(recvbuf, count, datatype);
    if (rc == MPI_SUCCESS) rc = v_op(op, datatype, &r);
    if (rc == MPI_SUCCESS && count > 0) {
        if (recvbuf == MPI_IN_PLACE) { set_error("recvbuf is MPI_IN_PLACE"); rc = MPI_ERR_BUFFER; }
        else if (sendbuf != MPI_IN_PLACE) {
            rc = v_buffer(datatype, sendbuf, count);
            if (rc == MPI_SUCCESS && sendbuf == recvbuf) { set_error("sendbuf aliases recvbuf"); rc = MPI_ERR_BUFFER; }
        }
    }
    if (rc == MPI_SUCCESS && nonblocking) {
        const size_t n = (size_t)count;
        rc = request_start_generic(c, [=] {
            return n ? coll_scan(c, sendbuf, recvbuf, n, datatype, r, exclusive) : MPI_SUCCESS;
        }, request, datatype);
    } else if (rc == MPI_SUCCESS && count > 0) {
        rc = coll_scan(c, sendbuf, recvbuf, (size_t)count, datatype, r, exclusive);
    }
    return err_return(c, fn, rc);
}

}  // namespace

MSX_EXPORT int MPI_Scan(const void* sendbuf, void* recvbuf, int count, MPI_Datatype datatype,
                        MPI_Op op, MPI_Comm comm)
{
    MSX_REQUIRE_INIT("MPI_Scan");
    return scan_common("MPI_Scan", sendbuf, recvbuf, count, datatype, op, comm, false);
}

MSX_EXPORT int MPI_Exscan(const void* sendbuf, void* recvbuf, int count, MPI_Datatype datatype,
                          MPI_Op op, MPI_Comm comm)
{
    MSX_REQUIRE_INIT("MPI_Exscan");
    return scan_common("MPI_Exscan", sendbuf, recvbuf, count, datatype, op, comm, true);
}

MSX_EXPORT int MPI_Iscan(const void* sendbuf, void* recvbuf, int count, MPI_Datatype datatype,
                         MPI_Op op, MPI_Comm comm, MPI_Request* request)
{
    MSX_REQUIRE_INIT("MPI_Iscan");
    return scan_common("MPI_Iscan", sendbuf, recvbuf, count, datatype, op, comm, false, request, true);
}

MSX_EXPORT int MPI_Iexscan(const void* sendbuf, void* recvbuf, int count, MPI_Datatype datatype,
                           MPI_Op op, MPI_Comm comm, MPI_Request* request)
{
    MSX_REQUIRE_INIT("MPI_Iexscan");
    return scan_common("MPI_Iexscan", sendbuf, recvbuf, count, datatype, op, comm, true, request, true);
}

// ---- non-blocking variants: stream-ordered requests -----------------------
MSX_EXPORT int MPI_Iallreduce(const void* sendbuf, void* recvbuf, int count, MPI_Datatype datatype,
                              MPI_Op op, MPI_Comm comm, MPI_Request* request)
{
    MSX_REQUIRE_INIT("MPI_Iallreduce");
    Comm* c;
    OpRef r;
    int rc = v_comm(comm, &c);
    if (rc == MPI_SUCCESS && request == nullptr) { set_error("null request"); rc = MPI_ERR_ARG; }
    if (rc == MPI_SUCCESS) *request = MPI_REQUEST_NULL;
    if (rc == MPI_SUCCESS) rc = v_dtype_any(recvbuf, count, datatype);
    if (rc == MPI_SUCCESS) rc = v_op(op, datatype, &r);
    if (rc == MPI_SUCCESS && count > 0) rc = v_allreduce_bufs(c, sendbuf, recvbuf, count, datatype);
    if (rc == MPI_SUCCESS && c->inter) {
        const size_t n = (size_t)count;
        rc = request_start_generic(c, [=] {
            return n ? engine_inter_allreduce(c, sendbuf, recvbuf, n, datatype, r) : MPI_SUCCESS;
        }, request, datatype);
    } else if (rc == MPI_SUCCESS) {
        rc = request_start_allreduce(c, sendbuf, recvbuf, (size_t)count, datatype, r, request);
    }
    return err_return(c, "MPI_Iallreduce", rc);
}

MSX_EXPORT int MPI_Ireduce(const void* sendbuf, void* recvbuf, int count, MPI_Datatype datatype,
                           MPI_Op op, int root, MPI_Comm comm, MPI_Request* request)
{
    MSX_REQUIRE_INIT("MPI_Ireduce");
    Comm* c;
    OpRef r;
    int rc = v_comm(comm, &c);
    if (rc == MPI_SUCCESS && request == nullptr) { set_error("null request"); rc = MPI_ERR_ARG; }
    if (rc == MPI_SUCCESS) *request = MPI_REQUEST_NULL;
    bool skip = false;
    if (rc == MPI_SUCCESS) rc = v_reduce(c, sendbuf, recvbuf, count, datatype, op, root, &r, &skip);
    if (rc == MPI_SUCCESS) {
        const size_t n = skip ? 0 : (size_t)count;
        rc = request_start_generic(c, [=] { return run_reduce(c, sendbuf, recvbuf, n, datatype, r, root, true); },
                                   request, datatype);
    }
    return err_return(c, "MPI_Ireduce", rc);
}

MSX_EXPORT int MPI_Ireduce_scatter(const void* sendbuf, void* recvbuf, const int recvcounts[],
                                   MPI_Datatype datatype, MPI_Op op, MPI_Comm comm,
                                   MPI_Request* request)
{
    MSX_REQUIRE_INIT("MPI_Ireduce_scatter");
    Comm* c;
    OpRef r;
    int rc = v_comm(comm, &c);
    if (rc == MPI_SUCCESS && request == nullptr) { set_error("null request"); rc = MPI_ERR_ARG; }
    if (rc == MPI_SUCCESS) *request = MPI_REQUEST_NULL;
    if (rc == MPI_SUCCESS) rc = validate_reduce_scatter(c, sendbuf, recvbuf, recvcounts, datatype, op, &r);
    if (rc == MPI_SUCCESS) {
        std::vector<int> counts(recvcounts, recvcounts + c->size);
        rc = request_start_generic(c, [=] {
            return run_reduce_scatter(c, sendbuf, recvbuf, counts.data(), datatype, r);
        }, request, datatype);
    }
    return err_return(c, "MPI_Ireduce_scatter", rc);
}

MSX_EXPORT int MPI_Ireduce_scatter_block(const void* sendbuf, void* recvbuf, int recvcount,
                                         MPI_Datatype datatype, MPI_Op op, MPI_Comm comm,
                                         MPI_Request* request)
{
    MSX_REQUIRE_INIT("MPI_Ireduce_scatter_block");
    Comm* c;
    OpRef r;
    int rc = v_comm(comm, &c);
    if (rc == MPI_SUCCESS && request == nullptr) { set_error("null request"); rc = MPI_ERR_ARG; }
    if (rc == MPI_SUCCESS) *request = MPI_REQUEST_NULL;
    if (rc == MPI_SUCCESS && recvcount < 0) { set_error("negative recvcount"); rc = MPI_ERR_COUNT; }
    std::vector<int> counts;
    if (rc == MPI_SUCCESS) {
        counts.assign((size_t)c->size, recvcount);
        rc = validate_reduce_scatter(c, sendbuf, recvbuf, counts.data(), datatype, op, &r);
    }
    if (rc == MPI_SUCCESS) {
        rc = request_start_generic(c, [=] {
            return run_reduce_scatter(c, sendbuf, recvbuf, counts.data(), datatype, r);
        }, request, datatype);
    }
    return err_return(c, "MPI_Ireduce_scatter_block", rc);
}

MSX_EXPORT int MPI_Wait(MPI_Request* request, MPI_Status* status)
{
    MSX_REQUIRE_INIT("MPI_Wait");
    // mpi_completion.cpp:907-920: MPI_STATUS_IGNORE is not NULL; NULL is an error
    if (!request || !status) {
        set_error("null %s", !request ? "request" : "status");
        return err_return(nullptr, "MPI_Wait", MPI_ERR_ARG);
    }
    return err_return(nullptr, "MPI_Wait", request_wait(request, status));
}

MSX_EXPORT int MPI_Test(MPI_Request* request, int* flag, MPI_Status* status)
{
    MSX_REQUIRE_INIT("MPI_Test");
    if (!request || !flag || !status) {
        set_error("null %s", !request ? "request" : (!flag ? "flag" : "status"));
        return err_return(nullptr, "MPI_Test", MPI_ERR_ARG);
    }
    return err_return(nullptr, "MPI_Test", request_test(request, flag, status));
}

// ---- multi-request completion (api/mpi_completion.cpp, api/mpi_request.cpp) ----
// Argument checks, the handling of MPI_REQUEST_NULL entries, MPI_ERR_IN_STATUS
// / MPI_ERR_PENDING reporting and which outcomes go through the error handler
// follow the reference function by function.
namespace {
MPI_Status* status_at(MPI_Status* statuses, int i)
{
    return statuses == MPI_STATUSES_IGNORE ? MPI_STATUS_IGNORE : &statuses[i];
}
void status_set_error(MPI_Status* st, int rc)
{
    if (st != MPI_STATUS_IGNORE && st != nullptr) st->MPI_ERROR = rc;
}
}  // namespace

// mpi_completion.cpp:1022-1140: an error completes nothing further (the rest
// get MPI_ERR_PENDING); MPI_ERR_IN_STATUS is returned without the handler
MSX_EXPORT int MPI_Waitall(int count, MPI_Request reqs[], MPI_Status statuses[])
{
    MSX_REQUIRE_INIT("MPI_Waitall");
    if (count < 0) { set_error("negative count %d", count); return err_return(nullptr, "MPI_Waitall", MPI_ERR_COUNT); }
    if (count != 0 && (!reqs || !statuses)) {
        set_error("null %s", !reqs ? "array_of_requests" : "array_of_statuses");
        return err_return(nullptr, "MPI_Waitall", MPI_ERR_ARG);
    }
    int rc = MPI_SUCCESS;
    bool have_errors = false;
    for (int i = 0; i < count; ++i) {
        MPI_Status* st = status_at(statuses, i);
        if (reqs[i] == MPI_REQUEST_NULL) { status_set_empty(st); continue; }
        int v = request_validate(reqs[i]);
        if (v != MPI_SUCCESS) {
            rc = MPI_ERR_IN_STATUS;
            status_set_error(st, v);
            have_errors = true;
            continue;
        }
        if (have_errors) { status_set_error(st, MPI_ERR_PENDING); continue; }
        int r = request_wait(&reqs[i], st);
        status_set_error(st, r);
        if (r != MPI_SUCCESS) { rc = MPI_ERR_IN_STATUS; have_errors = true; }
    }
    return rc;
}

// mpi_completion.cpp:226-417
MSX_EXPORT int MPI_Testall(int count, MPI_Request reqs[], int* flag, MPI_Status statuses[])
{
    MSX_REQUIRE_INIT("MPI_Testall");
    if (count < 0) { set_error("negative count %d", count); return err_return(nullptr, "MPI_Testall", MPI_ERR_COUNT); }
    if (!flag) { set_error("null flag"); return err_return(nullptr, "MPI_Testall", MPI_ERR_ARG); }
    if (count != 0 && (!reqs || !statuses)) {
        set_error("null %s", !reqs ? "array_of_requests" : "array_of_statuses");
        return err_return(nullptr, "MPI_Testall", MPI_ERR_ARG);
    }
    for (int i = 0; i < count; ++i)
        if (reqs[i] != MPI_REQUEST_NULL && request_validate(reqs[i]) != MPI_SUCCESS)
            return err_return(nullptr, "MPI_Testall", MPI_ERR_REQUEST);
    int n_completed = 0, rc = MPI_SUCCESS;
    std::vector<char> done((size_t)count, 0);
    for (int i = 0; i < count; ++i) {
        if (reqs[i] == MPI_REQUEST_NULL) { ++n_completed; continue; }
        if (!request_done(reqs[i])) continue;
        done[(size_t)i] = 1;
        ++n_completed;
        if (request_error(reqs[i]) != MPI_SUCCESS) rc = MPI_ERR_IN_STATUS;
    }
    if (n_completed == count || rc == MPI_ERR_IN_STATUS) {
        n_completed = 0;
        for (int i = 0; i < count; ++i) {
            MPI_Status* st = status_at(statuses, i);
            if (reqs[i] == MPI_REQUEST_NULL) {
                ++n_completed;
                status_set_empty(st);
            } else if (done[(size_t)i]) {
                ++n_completed;
                int f = 0;
                const int r = request_test(&reqs[i], &f, st);
                if (rc == MPI_ERR_IN_STATUS) status_set_error(st, r);
            } else if (rc == MPI_ERR_IN_STATUS) {
                status_set_error(st, MPI_ERR_PENDING);
            }
        }
    }
    *flag = n_completed == count;
    return err_return(nullptr, "MPI_Testall", rc);
}

// mpi_completion.cpp:453-625: the completed request's code is returned
// without the handler
MSX_EXPORT int MPI_Testany(int count, MPI_Request reqs[], int* index, int* flag, MPI_Status* status)
{
    MSX_REQUIRE_INIT("MPI_Testany");
    if (count < 0) { set_error("negative count %d", count); return err_return(nullptr, "MPI_Testany", MPI_ERR_COUNT); }
    if ((count != 0 && (!reqs || !status)) || !index || !flag) {
        set_error("null argument");
        return err_return(nullptr, "MPI_Testany", MPI_ERR_ARG);
    }
    int n_inactive = 0;
    for (int i = 0; i < count; ++i) {
        if (reqs[i] == MPI_REQUEST_NULL) { ++n_inactive; continue; }
        if (request_validate(reqs[i]) != MPI_SUCCESS) return err_return(nullptr, "MPI_Testany", MPI_ERR_REQUEST);
    }
    *index = MPI_UNDEFINED;
    if (n_inactive == count) {
        *flag = 1;
        if (status) status_set_empty(status);
        return MPI_SUCCESS;
    }
    *flag = 0;
    for (int i = 0; i < count; ++i) {
        if (reqs[i] == MPI_REQUEST_NULL || !request_done(reqs[i])) continue;
        int f = 0;
        const int r = request_test(&reqs[i], &f, status);
        *flag = 1;
        *index = i;
        return r;
    }
    return MPI_SUCCESS;
}

// mpi_completion.cpp:1176-1333
MSX_EXPORT int MPI_Waitany(int count, MPI_Request reqs[], int* index, MPI_Status* status)
{
    MSX_REQUIRE_INIT("MPI_Waitany");
    if (count < 0) { set_error("negative count %d", count); return err_return(nullptr, "MPI_Waitany", MPI_ERR_COUNT); }
    if ((count != 0 && (!reqs || !status)) || !index) {
        set_error("null argument");
        return err_return(nullptr, "MPI_Waitany", MPI_ERR_ARG);
    }
    int n_inactive = 0;
    for (int i = 0; i < count; ++i) {
        if (reqs[i] == MPI_REQUEST_NULL) { ++n_inactive; continue; }
        if (request_validate(reqs[i]) != MPI_SUCCESS) return err_return(nullptr, "MPI_Waitany", MPI_ERR_REQUEST);
    }
    if (n_inactive == count) {
        *index = MPI_UNDEFINED;
        status_set_empty(status);
        return MPI_SUCCESS;
    }
    for (int it = 0;; ++it) {
        for (int i = 0; i < count; ++i) {
            if (reqs[i] == MPI_REQUEST_NULL || !request_done(reqs[i])) continue;
            int f = 0;
            const int r = request_test(&reqs[i], &f, status);
            *index = i;
            return r;
        }
        progress_pause(it);
    }
}

namespace {
// the completion pass shared by MPI_Testsome and MPI_Waitsome
// (mpi_completion.cpp:765-837, 1491-1566)
int complete_some(int incount, MPI_Request reqs[], int* outcount, int indices[], MPI_Status statuses[],
                  int* n_inactive)
{
    int n_active = 0, rc = MPI_SUCCESS;
    std::vector<int> failed;
    for (int i = 0; i < incount; ++i) {
        if (reqs[i] == MPI_REQUEST_NULL || !request_done(reqs[i])) continue;
        MPI_Status* st = status_at(statuses, n_active);
        int f = 0;
        const int r = request_test(&reqs[i], &f, st);
        indices[n_active] = i;
        if (r != MPI_SUCCESS) {
            rc = MPI_ERR_IN_STATUS;
            status_set_error(st, r);
            failed.push_back(n_active);
        }
        ++n_active;
    }
    (void)n_inactive;
    if (rc == MPI_ERR_IN_STATUS && statuses != MPI_STATUSES_IGNORE)
        for (int k = 0; k < n_active; ++k)
            if (std::find(failed.begin(), failed.end(), k) == failed.end()) statuses[k].MPI_ERROR = MPI_SUCCESS;
    *outcount = n_active;
    return rc;
}
}  // namespace

// mpi_completion.cpp:663-862: MPI_ERR_IN_STATUS goes through the handler
MSX_EXPORT int MPI_Testsome(int incount, MPI_Request reqs[], int* outcount, int indices[], MPI_Status statuses[])
{
    MSX_REQUIRE_INIT("MPI_Testsome");
    if (incount < 0) { set_error("negative count %d", incount); return err_return(nullptr, "MPI_Testsome", MPI_ERR_COUNT); }
    if ((incount != 0 && (!reqs || !indices || !statuses)) || !outcount) {
        set_error("null argument");
        return err_return(nullptr, "MPI_Testsome", MPI_ERR_ARG);
    }
    *outcount = 0;
    int n_inactive = 0;
    for (int i = 0; i < incount; ++i) {
        if (reqs[i] == MPI_REQUEST_NULL) { ++n_inactive; continue; }
        if (request_validate(reqs[i]) != MPI_SUCCESS) return err_return(nullptr, "MPI_Testsome", MPI_ERR_REQUEST);
    }
    if (n_inactive == incount) { *outcount = MPI_UNDEFINED; return MPI_SUCCESS; }
    const int rc = complete_some(incount, reqs, outcount, indices, statuses, &n_inactive);
    return err_return(nullptr, "MPI_Testsome", rc);
}

// mpi_completion.cpp:1385-1595: blocks until at least one completes;
// MPI_ERR_IN_STATUS is returned without the handler
MSX_EXPORT int MPI_Waitsome(int incount, MPI_Request reqs[], int* outcount, int indices[], MPI_Status statuses[])
{
    MSX_REQUIRE_INIT("MPI_Waitsome");
    if (incount < 0) { set_error("negative count %d", incount); return err_return(nullptr, "MPI_Waitsome", MPI_ERR_COUNT); }
    if ((incount != 0 && (!reqs || !indices || !statuses)) || !outcount) {
        set_error("null argument");
        return err_return(nullptr, "MPI_Waitsome", MPI_ERR_ARG);
    }
    *outcount = 0;
    int n_inactive = 0;
    for (int i = 0; i < incount; ++i) {
        if (reqs[i] == MPI_REQUEST_NULL) { ++n_inactive; continue; }
        if (request_validate(reqs[i]) != MPI_SUCCESS) return err_return(nullptr, "MPI_Waitsome", MPI_ERR_REQUEST);
    }
    if (n_inactive == incount) { *outcount = MPI_UNDEFINED; return MPI_SUCCESS; }
    for (int it = 0;; ++it) {
        const int rc = complete_some(incount, reqs, outcount, indices, statuses, &n_inactive);
        if (*outcount > 0) return rc;
        progress_pause(it);
    }
}

// mpi_request.cpp:52-141: the reference frees only point-to-point, RMA,
// persistent and generalized requests; a collective (NBC) request is an
// invalid kind there (MPI_ERR_OTHER, "**request_invalid_kind")
MSX_EXPORT int MPI_Request_free(MPI_Request* request)
{
    MSX_REQUIRE_INIT("MPI_Request_free");
    if (!request) { set_error("null request"); return err_return(nullptr, "MPI_Request_free", MPI_ERR_ARG); }
    int rc = request_validate(*request);
    if (rc == MPI_SUCCESS) rc = request_free(request);
    return err_return(nullptr, "MPI_Request_free", rc);
}

// mpi_request.cpp:170-330: non-destructive; an NBC request's status is left
// as the caller passed it
MSX_EXPORT int MPI_Request_get_status(MPI_Request request, int* flag, MPI_Status* status)
{
    MSX_REQUIRE_INIT("MPI_Request_get_status");
    if (!flag || !status) { set_error("null argument"); return err_return(nullptr, "MPI_Request_get_status", MPI_ERR_ARG); }
    if (request == MPI_REQUEST_NULL) {
        status_set_empty(status);
        *flag = 1;
        return MPI_SUCCESS;
    }
    const int rc = request_validate(request);
    if (rc != MPI_SUCCESS) return err_return(nullptr, "MPI_Request_get_status", rc);
    *flag = request_done(request) ? 1 : 0;
    return MPI_SUCCESS;
}

// ---- PMPI_ profiling aliases (dll/msmpi.def) --------------------------------
#define MSX_ALIAS(name) extern "C" __attribute__((visibility("default"), alias(#name)))
MSX_ALIAS(MPI_Reduce_local) int PMPI_Reduce_local(const void*, void*, int, MPI_Datatype, MPI_Op);
MSX_ALIAS(MPI_Testall) int PMPI_Testall(int, MPI_Request[], int*, MPI_Status[]);
MSX_ALIAS(MPI_Win_post) int PMPI_Win_post(MPI_Group, int, MPI_Win);
MSX_ALIAS(MPI_Comm_create) int PMPI_Comm_create(MPI_Comm, MPI_Group, MPI_Comm*);
MSX_ALIAS(MPI_Comm_compare) int PMPI_Comm_compare(MPI_Comm, MPI_Comm, int*);
MSX_ALIAS(MPI_Intercomm_create) int PMPI_Intercomm_create(MPI_Comm, int, MPI_Comm, int, int, MPI_Comm*);
MSX_ALIAS(MPI_Intercomm_merge) int PMPI_Intercomm_merge(MPI_Comm, int, MPI_Comm*);
MSX_ALIAS(MPI_Win_start) int PMPI_Win_start(MPI_Group, int, MPI_Win);
MSX_ALIAS(MPI_Win_complete) int PMPI_Win_complete(MPI_Win);
MSX_ALIAS(MPI_Win_wait) int PMPI_Win_wait(MPI_Win);
MSX_ALIAS(MPI_Win_test) int PMPI_Win_test(MPI_Win, int*);
MSX_ALIAS(MPI_Win_get_group) int PMPI_Win_get_group(MPI_Win, MPI_Group*);
MSX_ALIAS(MPI_Testany) int PMPI_Testany(int, MPI_Request[], int*, int*, MPI_Status*);
MSX_ALIAS(MPI_Testsome) int PMPI_Testsome(int, MPI_Request[], int*, int[], MPI_Status[]);
MSX_ALIAS(MPI_Waitany) int PMPI_Waitany(int, MPI_Request[], int*, MPI_Status*);
MSX_ALIAS(MPI_Waitsome) int PMPI_Waitsome(int, MPI_Request[], int*, int[], MPI_Status[]);
MSX_ALIAS(MPI_Request_free) int PMPI_Request_free(MPI_Request*);
MSX_ALIAS(MPI_Rput) int PMPI_Rput(const void*, int, MPI_Datatype, int, MPI_Aint, int, MPI_Datatype, MPI_Win,
                                  MPI_Request*);
MSX_ALIAS(MPI_Rget) int PMPI_Rget(void*, int, MPI_Datatype, int, MPI_Aint, int, MPI_Datatype, MPI_Win, MPI_Request*);
MSX_ALIAS(MPI_Raccumulate) int PMPI_Raccumulate(const void*, int, MPI_Datatype, int, MPI_Aint, int, MPI_Datatype,
                                                MPI_Op, MPI_Win, MPI_Request*);
MSX_ALIAS(MPI_Rget_accumulate) int PMPI_Rget_accumulate(const void*, int, MPI_Datatype, void*, int, MPI_Datatype, int,
                                                        MPI_Aint, int, MPI_Datatype, MPI_Op, MPI_Win, MPI_Request*);
MSX_ALIAS(MPI_Request_get_status) int PMPI_Request_get_status(MPI_Request, int*, MPI_Status*);
MSX_ALIAS(MPI_Reduce) int PMPI_Reduce(const void*, void*, int, MPI_Datatype, MPI_Op, int, MPI_Comm);
MSX_ALIAS(MPI_Allreduce) int PMPI_Allreduce(const void*, void*, int, MPI_Datatype, MPI_Op, MPI_Comm);
MSX_ALIAS(MPI_Reduce_scatter_block) int PMPI_Reduce_scatter_block(const void*, void*, int, MPI_Datatype, MPI_Op, MPI_Comm);
MSX_ALIAS(MPI_Reduce_scatter) int PMPI_Reduce_scatter(const void*, void*, const int[], MPI_Datatype, MPI_Op, MPI_Comm);
MSX_ALIAS(MPI_Iallreduce) int PMPI_Iallreduce(const void*, void*, int, MPI_Datatype, MPI_Op, MPI_Comm, MPI_Request*);
MSX_ALIAS(MPI_Iscan) int PMPI_Iscan(const void*, void*, int, MPI_Datatype, MPI_Op, MPI_Comm, MPI_Request*);
MSX_ALIAS(MPI_Iexscan) int PMPI_Iexscan(const void*, void*, int, MPI_Datatype, MPI_Op, MPI_Comm, MPI_Request*);
MSX_ALIAS(MPI_Scan) int PMPI_Scan(const void*, void*, int, MPI_Datatype, MPI_Op, MPI_Comm);
MSX_ALIAS(MPI_Exscan) int PMPI_Exscan(const void*, void*, int, MPI_Datatype, MPI_Op, MPI_Comm);
MSX_ALIAS(MPI_Ireduce) int PMPI_Ireduce(const void*, void*, int, MPI_Datatype, MPI_Op, int, MPI_Comm, MPI_Request*);
MSX_ALIAS(MPI_Ireduce_scatter_block) int PMPI_Ireduce_scatter_block(const void*, void*, int, MPI_Datatype, MPI_Op,
                                                                    MPI_Comm, MPI_Request*);
MSX_ALIAS(MPI_Ireduce_scatter) int PMPI_Ireduce_scatter(const void*, void*, const int*, MPI_Datatype, MPI_Op,
                                                        MPI_Comm, MPI_Request*);
MSX_ALIAS(MPI_Accumulate) int PMPI_Accumulate(const void*, int, MPI_Datatype, int, MPI_Aint, int, MPI_Datatype,
                                              MPI_Op, MPI_Win);
MSX_ALIAS(MPI_Get_accumulate) int PMPI_Get_accumulate(const void*, int, MPI_Datatype, void*, int, MPI_Datatype, int,
                                                      MPI_Aint, int, MPI_Datatype, MPI_Op, MPI_Win);
MSX_ALIAS(MPI_Fetch_and_op) int PMPI_Fetch_and_op(const void*, void*, MPI_Datatype, int, MPI_Aint, MPI_Op, MPI_Win);
MSX_ALIAS(MPI_Op_create) int PMPI_Op_create(MPI_User_function*, int, MPI_Op*);
MSX_ALIAS(MPI_Op_free) int PMPI_Op_free(MPI_Op*);
MSX_ALIAS(MPI_Op_commutative) int PMPI_Op_commutative(MPI_Op, int*);

// ===========================================================================
// one-sided communication (api/mpi_win.cpp, api/mpi_rma.cpp), fence epochs
// ===========================================================================
namespace {

std::mutex g_win_mu;
std::vector<RmaWin*> g_wins;          // direct handles 0xA0000000 | index
constexpr int kWinKindBits = 0xA0000000;

// MpiaWinValidateHandle
int v_win(MPI_Win h, RmaWin** out)
{
    *out = nullptr;
    if (h == MPI_WIN_NULL) { set_error("null window"); return MPI_ERR_WIN; }
    std::lock_guard<std::mutex> g(g_win_mu);
    const unsigned idx = (unsigned)h & 0x03ffffffu;
    if (((unsigned)h & 0xfc000000u) != (unsigned)kWinKindBits || idx >= g_wins.size() || !g_wins[idx]) {
        set_error("invalid window 0x%x", h);
        return MPI_ERR_WIN;
    }
    *out = g_wins[idx];
    return MPI_SUCCESS;
}

int err_win(RmaWin* w, const char* fn, int code)
{
    if (code == MPI_SUCCESS) return code;
    // MPIR_Err_return_win (mpid/error.cpp:142-151): a window without an
    // error handler of its own reports through MPI_COMM_WORLD's
    if (!w || w->errhandler == MPI_ERRHANDLER_NULL) return err_return(nullptr, fn, code);
    return err_return_h(w->errhandler, fn, code);
}

// target datatype checks (MpiaDatatypeValidate with MPI_IN_PLACE as buffer),
// the displacement and the rank, in the order of mpi_rma.cpp:697-735
int v_target(RmaWin* w, int target_count, MPI_Datatype target_dt, int target_rank, MPI_Aint target_disp)
{
    int rc = v_dtype_any(MPI_IN_PLACE, target_count, target_dt);
    if (rc != MPI_SUCCESS) return rc;
    if (target_disp < 0) { set_error("negative target displacement"); return MPI_ERR_DISP; }
    if (target_rank != MPI_PROC_NULL && (target_rank < 0 || target_rank >= w->comm->size)) {
        set_error("invalid target rank %d", target_rank);
        return MPI_ERR_RANK;
    }
    return MPI_SUCCESS;
}

// Origin and target must describe the same data: predefined pairs the same
// type and count; with a derived type on either side the same number of bytes
// of the same basic element type (the type signatures of MPI-2.2 §11.3).
int v_match(int ocount, MPI_Datatype odt, int tcount, MPI_Datatype tdt)
{
    if (!dtype_is_derived(odt) && !dtype_is_derived(tdt)) {
        if (odt != tdt) { set_error("origin and target datatypes differ (0x%x, 0x%x)", odt, tdt); return MPI_ERR_TYPE; }
        if (ocount != tcount) { set_error("origin and target counts differ (%d, %d)", ocount, tcount); return MPI_ERR_COUNT; }
        return MPI_SUCCESS;
    }
    const Dtype* o = dtype_lookup(odt);
    const Dtype* t = dtype_lookup(tdt);
    if ((int64_t)ocount * o->size != (int64_t)tcount * t->size) {
        set_error("origin and target describe %lld and %lld bytes", (long long)((int64_t)ocount * o->size),
                  (long long)((int64_t)tcount * t->size));
        return MPI_ERR_TYPE;
    }
    if (o->eltype != t->eltype && o->size > 0) {
        set_error("origin and target element types differ (0x%x, 0x%x)", o->eltype, t->eltype);
        return MPI_ERR_TYPE;
    }
    return MPI_SUCCESS;
}

// Device temporary holding `count` instances of `dt` from `src`, packed.
int pack_to_device(const void* src, int64_t count, MPI_Datatype dt, void** out)
{
    *out = nullptr;
    const Dtype* t = dtype_lookup(dt);
    const size_t bytes = (size_t)(count * t->size);
    if (bytes == 0) return MPI_SUCCESS;
    int rc = ensure_device();
    if (rc != MPI_SUCCESS) return rc;
    if (hipMalloc(out, bytes) != hipSuccess) { *out = nullptr; set_error("rma temporary"); return MPI_ERR_NO_MEM; }
    rc = dt_pack_any(t, count, src, *out);
    if (rc != MPI_SUCCESS) { (void)hipFree(*out); *out = nullptr; }
    return rc;
}

// Queue a remote operation, or apply it now when the target is this rank
// (win.cpp:1570-1590: MPIDI_Win_local_accumulate / MPIR_Localcopy).
// Derived origin / result types are packed / unpacked on the origin's GPU; a
// derived target type travels as its flattened layout.
int rma_issue(RmaWin* w, RmaKind kind, int target, MPI_Aint disp, int opidx, const void* origin, int ocount,
              MPI_Datatype odt, void* result, int rcount, MPI_Datatype rdt, int tcount, MPI_Datatype tdt,
              const void* compare)
{
    RmaDesc d;
    d.kind = kind;
    d.target = target;
    d.opidx = opidx;
    d.tdisp = (int64_t)disp * w->disp_units[(size_t)target];    // the TARGET's disp_unit
    const bool self = target == w->comm->rank;
    const Dtype* T = nullptr;
    if (dtype_is_derived(tdt)) {
        T = dtype_lookup(tdt);
        d.dt = T->eltype;
        d.count = tcount;
        d.usize = T->size;
        d.uext = T->extent;
        dt_span(T, tcount, &d.span_lo, &d.span_hi);
        if (T->size == 0) return MPI_SUCCESS;
        if (!self) {
            d.layout = (int32_t)w->blob.size();
            dtype_serialize(T, w->blob);
        }
    } else {
        d.dt = tdt;
        d.count = tcount;
        d.usize = d.uext = type_size(tdt);
    }
    RmaLocal l;
    l.origin = origin;
    l.result = result;
    l.compare = compare;
    int rc = MPI_SUCCESS;
    const bool sends = kind == RMA_PUT || ((kind == RMA_ACC || kind == RMA_GACC) && opidx != O_NOOP);
    const bool fetches = kind == RMA_GET || kind == RMA_GACC;
    // the typed kernels read the payload and write fetched bytes in device memory
    if (sends && (dtype_is_derived(odt) || (T && classify(origin).place != Place::Device))) {
        rc = pack_to_device(origin, ocount, odt, &l.tmp_origin);
        l.origin = l.tmp_origin;
    }
    if (rc == MPI_SUCCESS && fetches && (dtype_is_derived(rdt) || (T && classify(result).place != Place::Device))) {
        const size_t bytes = (size_t)(rcount * dtype_lookup(rdt)->size);
        if (bytes && hipMalloc(&l.tmp_result, bytes) != hipSuccess) {
            l.tmp_result = nullptr;
            set_error("rma temporary");
            rc = MPI_ERR_NO_MEM;
        }
        l.result = l.tmp_result;
        l.result_user = result;
        l.result_dt = rdt;
        l.result_count = rcount;
        if (l.tmp_result) dtype_add_ref(rdt);      // released by rma_local_complete
    }
    if (rc != MPI_SUCCESS) {
        rma_local_complete(l);
        return rc;
    }
    if (self) {
        engine_rma_self_guard(w, true);      // not concurrently with the window's service thread
        rc = rma_apply_self(w, d, l, T);
        engine_rma_self_guard(w, false);
        const int r2 = rma_local_complete(l);
        return rc != MPI_SUCCESS ? rc : r2;
    }
    w->q.push_back(d);
    w->ql.push_back(l);
    return MPI_SUCCESS;
}

int rma_op(MPI_Op op, OpRef* r, bool allow_noop)
{
    int rc = v_op_handle(op, r);       // MpiaOpValidate(rmaOp = true): handle only
    if (rc != MPI_SUCCESS) return rc;
    if (!allow_noop && r->opidx == O_NOOP) { set_error("MPI_NO_OP not allowed"); return MPI_ERR_OP; }
    if (r->opidx == O_NULL) {
        // do_accumulate_op: **opnotpredefined (packethandling.cpp:2934-2937)
        set_error("user-defined operations are not allowed in RMA");
        return MPI_ERR_OP;
    }
    return MPI_SUCCESS;
}

}  // namespace

// ---- MPI_Alloc_mem / MPI_Free_mem (api/mpi_env.cpp:841-945) ---------------------
// The reference returns heap memory (MPID_Alloc_mem, mpid/env.cpp:1745).  Here
// it is pinned host memory when a GPU is present: still ordinary CPU memory,
// and the combine kernels read and write it in place over PCIe (the zero-copy
// host path), instead of staging pageable pages.
namespace {
std::mutex g_mem_mu;
std::map<void*, bool> g_mem;          // base -> pinned (hipHostMalloc) or heap

int alloc_mem(MPI_Aint size, void** out)
{
    const size_t n = size > 0 ? (size_t)size : 1;
    void* p = nullptr;
    bool pinned = false;
    if (device_count_noinit() > 0 && ensure_device() == MPI_SUCCESS &&
        hipHostMalloc(&p, n, hipHostMallocDefault) == hipSuccess) {
        pinned = true;
    } else {
        (void)hipGetLastError();
        p = malloc(n);
    }
    if (!p) { set_error("MPI_Alloc_mem: %lld bytes not available (**allocmem)", (long long)size); return MPI_ERR_NO_MEM; }
    std::lock_guard<std::mutex> g(g_mem_mu);
    g_mem[p] = pinned;
    *out = p;
    return MPI_SUCCESS;
}

int free_mem(void* base)
{
    bool pinned;
    {
        std::lock_guard<std::mutex> g(g_mem_mu);
        auto it = g_mem.find(base);
        if (it == g_mem.end()) { set_error("memory %p was not allocated by MPI_Alloc_mem", base); return MPI_ERR_BASE; }
        pinned = it->second;
        g_mem.erase(it);
    }
    if (pinned) (void)hipHostFree(base);
    else free(base);
    return MPI_SUCCESS;
}
}  // namespace

MSX_EXPORT int MPI_Alloc_mem(MPI_Aint size, MPI_Info info, void* baseptr)
{
    MSX_REQUIRE_INIT("MPI_Alloc_mem");
    int rc = MPI_SUCCESS;
    if (size < 0) { set_error("negative size %lld (**argneg)", (long long)size); rc = MPI_ERR_ARG; }
    else if (!baseptr) { set_error("null baseptr"); rc = MPI_ERR_ARG; }
    else if (info != MPI_INFO_NULL) { set_error("only MPI_INFO_NULL is supported"); rc = MPI_ERR_INFO; }
    void* p = nullptr;
    if (rc == MPI_SUCCESS) rc = alloc_mem(size, &p);
    if (rc == MPI_SUCCESS) *static_cast<void**>(baseptr) = p;
    return err_return(nullptr, "MPI_Alloc_mem", rc);
}

// mpi_env.cpp:920-945: errors are returned, not raised through a handler
MSX_EXPORT int MPI_Free_mem(void* base)
{
    MSX_REQUIRE_INIT("MPI_Free_mem");
    if (!base) { set_error("null base"); return MPI_ERR_BASE; }
    return free_mem(base);
}

MSX_EXPORT int MPI_Win_create(void* base, MPI_Aint size, int disp_unit, MPI_Info info, MPI_Comm comm,
                              MPI_Win* win)
{
    MSX_REQUIRE_INIT("MPI_Win_create");
    Comm* c;
    int rc = v_intracomm(comm, &c);
    if (rc == MPI_SUCCESS && info != MPI_INFO_NULL) { set_error("only MPI_INFO_NULL is supported"); rc = MPI_ERR_INFO; }
    if (rc == MPI_SUCCESS && size < 0) { set_error("negative window size"); rc = MPI_ERR_SIZE; }
    if (rc == MPI_SUCCESS && disp_unit <= 0) { set_error("disp_unit must be positive"); rc = MPI_ERR_ARG; }
    if (rc == MPI_SUCCESS && win == nullptr) { set_error("null win"); rc = MPI_ERR_ARG; }
    if (rc != MPI_SUCCESS) return err_return(c, "MPI_Win_create", rc);
    auto* w = new RmaWin();
    w->comm = c;
    w->base = static_cast<char*>(base);
    w->size = size;
    w->disp_unit = disp_unit;
    w->lock_mode.assign((size_t)c->size, 0);
    w->lock_held.assign((size_t)c->size, 0);
    rc = engine_rma_create(w);
    if (rc != MPI_SUCCESS) {
        delete w;
        return err_return(c, "MPI_Win_create", rc);
    }
    std::lock_guard<std::mutex> g(g_win_mu);
    size_t idx = 0;
    while (idx < g_wins.size() && g_wins[idx]) ++idx;
    if (idx == g_wins.size()) g_wins.push_back(nullptr);
    g_wins[idx] = w;
    w->handle = kWinKindBits | (int)idx;
    *win = w->handle;
    return MPI_SUCCESS;
}

// MPI_Win_allocate (api/mpi_win.cpp:295-380): MPI_Alloc_mem + MPI_Win_create,
// the memory freed by MPI_Win_free
MSX_EXPORT int MPI_Win_allocate(MPI_Aint size, int disp_unit, MPI_Info info, MPI_Comm comm, void* baseptr,
                                MPI_Win* win)
{
    MSX_REQUIRE_INIT("MPI_Win_allocate");
    Comm* c;
    int rc = v_intracomm(comm, &c);
    if (rc == MPI_SUCCESS && info != MPI_INFO_NULL) { set_error("only MPI_INFO_NULL is supported"); rc = MPI_ERR_INFO; }
    if (rc == MPI_SUCCESS && size < 0) { set_error("negative window size (**rmasize)"); rc = MPI_ERR_SIZE; }
    if (rc == MPI_SUCCESS && disp_unit <= 0) { set_error("disp_unit must be positive"); rc = MPI_ERR_ARG; }
    if (rc == MPI_SUCCESS && (win == nullptr || baseptr == nullptr)) { set_error("null win / baseptr"); rc = MPI_ERR_ARG; }
    void* p = nullptr;
    if (rc == MPI_SUCCESS) rc = alloc_mem(size, &p);
    if (rc != MPI_SUCCESS) return err_return(c, "MPI_Win_allocate", rc);
    rc = MPI_Win_create(p, size, disp_unit, info, comm, win);
    if (rc != MPI_SUCCESS) {
        (void)free_mem(p);
        return rc;                    // already reported by MPI_Win_create
    }
    RmaWin* w;
    (void)v_win(*win, &w);
    w->owned = p;
    *static_cast<void**>(baseptr) = p;
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Win_free(MPI_Win* win)
{
    MSX_REQUIRE_INIT("MPI_Win_free");
    if (!win) { set_error("null win"); return err_return(nullptr, "MPI_Win_free", MPI_ERR_ARG); }
    RmaWin* w;
    int rc = v_win(*win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Win_free", rc);
    if (!w->q.empty()) { set_error("MPI_Win_free with operations pending (no closing fence)"); return err_win(w, "MPI_Win_free", MPI_ERR_RMA_SYNC); }
    for (int m : w->lock_mode)
        if (m) { set_error("MPI_Win_free inside a passive-target epoch"); return err_win(w, "MPI_Win_free", MPI_ERR_RMA_SYNC); }
    if (w->access_epoch || w->exposure_epoch) {
        set_error("MPI_Win_free inside a post-start-complete-wait epoch");
        return err_win(w, "MPI_Win_free", MPI_ERR_RMA_SYNC);
    }
    rc = coll_barrier(w->comm);       // every rank is done with the window
    if (rc != MPI_SUCCESS) return err_win(w, "MPI_Win_free", rc);
    engine_rma_free(w);               // no request can be in flight after the barrier
    if (w->owned) (void)free_mem(w->owned);
    {
        std::lock_guard<std::mutex> g(g_win_mu);
        g_wins[(size_t)(*win & 0x03ffffff)] = nullptr;
    }
    delete w;
    *win = MPI_WIN_NULL;
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Win_fence(int assert_, MPI_Win win)
{
    MSX_REQUIRE_INIT("MPI_Win_fence");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Win_fence", rc);
    (void)assert_;                    // hints only
    return err_win(w, "MPI_Win_fence", engine_rma_fence(w));
}

// ---- passive target (api/mpi_win.cpp:1153-1990, mpid/win.cpp:4090-4500) ----------
namespace {
// MpiaCommValidateSendRank: a rank of the window's group or MPI_PROC_NULL
int v_lock_rank(RmaWin* w, int rank)
{
    if (rank == MPI_PROC_NULL || (rank >= 0 && rank < w->comm->size)) return MPI_SUCCESS;
    set_error("invalid rank %d", rank);
    return MPI_ERR_RANK;
}

// MPID_Win_lock: a lock on this rank itself is acquired now (blocking); on
// another rank it is requested lazily, granted at the first flush / unlock
int win_lock(RmaWin* w, int lock_type, int rank, int assert_)
{
    (void)assert_;                    // MPI_MODE_NOCHECK: a hint
    if (rank == MPI_PROC_NULL) return MPI_SUCCESS;
    if (w->lock_mode[(size_t)rank]) {
        set_error("rank %d is already locked in this window (**rmasyncq)", rank);
        return MPI_ERR_OTHER;
    }
    if (rank == w->comm->rank) {
        const int rc = engine_rma_lock(w, rank, lock_type);
        if (rc != MPI_SUCCESS) return rc;
        w->lock_held[(size_t)rank] = 1;
    }
    w->lock_mode[(size_t)rank] = lock_type;
    return MPI_SUCCESS;
}

int win_unlock(RmaWin* w, int rank)
{
    if (rank == MPI_PROC_NULL) return MPI_SUCCESS;
    if (!w->lock_mode[(size_t)rank]) {
        set_error("MPI_Win_unlock without MPI_Win_lock on rank %d (**rmasync)", rank);
        return MPI_ERR_OTHER;
    }
    const int rc = engine_rma_flush(w, rank);
    engine_rma_unlock_target(w, rank);
    w->lock_mode[(size_t)rank] = 0;
    w->lock_held[(size_t)rank] = 0;
    return rc;
}
}  // namespace

MSX_EXPORT int MPI_Win_lock(int lock_type, int rank, int assert_, MPI_Win win)
{
    MSX_REQUIRE_INIT("MPI_Win_lock");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Win_lock", rc);
    if (lock_type != MPI_LOCK_SHARED && lock_type != MPI_LOCK_EXCLUSIVE) {
        set_error("invalid lock type %d (**locktype)", lock_type);
        rc = MPI_ERR_OTHER;
    }
    if (rc == MPI_SUCCESS) rc = v_lock_rank(w, rank);
    if (rc == MPI_SUCCESS) rc = win_lock(w, lock_type, rank, assert_);
    return err_win(w, "MPI_Win_lock", rc);
}

MSX_EXPORT int MPI_Win_unlock(int rank, MPI_Win win)
{
    MSX_REQUIRE_INIT("MPI_Win_unlock");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Win_unlock", rc);
    rc = v_lock_rank(w, rank);
    if (rc == MPI_SUCCESS) rc = win_unlock(w, rank);
    return err_win(w, "MPI_Win_unlock", rc);
}

// ---- post-start-complete-wait (api/mpi_win.cpp:28-70,979-1030,1331-1381,
// 1487-1537,1566-1613,1769-1808; mpid/win.cpp:2001-2012,3689-4088) -------------
namespace {
// The window ranks of a group's members (MpiaGroupValidateHandle, then
// MPIR_Group_translate_ranks into the window's communicator).  A member outside
// the window's communicator is an invalid group here (the reference would
// address rank MPI_UNDEFINED).
int group_window_ranks(RmaWin* w, MPI_Group g, std::vector<int>* ranks)
{
    std::vector<int> lp;
    int rc = group_members(g, &lp);
    if (rc != MPI_SUCCESS) return rc;
    ranks->clear();
    for (int id : lp) {
        const auto& cl = w->comm->lpid;
        const auto it = std::find(cl.begin(), cl.end(), id);
        if (it == cl.end()) {
            set_error("group member (process %d) is not in the window's communicator", id);
            return MPI_ERR_GROUP;
        }
        ranks->push_back((int)(it - cl.begin()));
    }
    return MPI_SUCCESS;
}
void pscw_sizes(RmaWin* w)
{
    const size_t p = (size_t)w->comm->size;
    if (w->starts.size() != p) w->starts.assign(p, 0);
    if (w->posts.size() != p) w->posts.assign(p, 0);
}
}  // namespace

// Exposure epoch: every origin of `group` may access this window until MPI_Win_wait
MSX_EXPORT int MPI_Win_post(MPI_Group group, int assert_, MPI_Win win)
{
    MSX_REQUIRE_INIT("MPI_Win_post");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Win_post", rc);
    std::vector<int> origins;
    rc = group_window_ranks(w, group, &origins);
    if (rc == MPI_SUCCESS && w->exposure_epoch) {
        set_error("MPI_Win_post inside an exposure epoch (**rmasync)");
        rc = MPI_ERR_RMA_SYNC;
    }
    (void)assert_;                    // MPI_MODE_NOCHECK / NOSTORE / NOPUT: hints here
    if (rc == MPI_SUCCESS) {
        pscw_sizes(w);
        w->exposure_origins = origins;
        w->exposure_epoch = true;
        rc = engine_rma_post(w);
    }
    return err_win(w, "MPI_Win_post", rc);
}

// Access epoch: operations to `group`'s members are queued until
// MPI_Win_complete, which waits for their posts (MPID_Win_start only records
// the group, win.cpp:3775-3801)
MSX_EXPORT int MPI_Win_start(MPI_Group group, int assert_, MPI_Win win)
{
    MSX_REQUIRE_INIT("MPI_Win_start");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Win_start", rc);
    std::vector<int> targets;
    rc = group_window_ranks(w, group, &targets);
    if (rc == MPI_SUCCESS && w->access_epoch) {
        set_error("MPI_Win_start inside an access epoch (**rmasync)");
        rc = MPI_ERR_RMA_SYNC;
    }
    if (rc == MPI_SUCCESS) {
        pscw_sizes(w);
        w->access_targets = targets;
        w->access_assert = assert_;
        w->access_epoch = true;
    }
    return err_win(w, "MPI_Win_start", rc);
}

// Every operation of the access epoch is applied at its target before the
// target's MPI_Win_wait can return.  Without a matching MPI_Win_start the
// reference dereferences a null group; here it is MPI_ERR_RMA_SYNC.
MSX_EXPORT int MPI_Win_complete(MPI_Win win)
{
    MSX_REQUIRE_INIT("MPI_Win_complete");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Win_complete", rc);
    if (!w->access_epoch) {
        set_error("MPI_Win_complete without MPI_Win_start (**rmasync)");
        return err_win(w, "MPI_Win_complete", MPI_ERR_RMA_SYNC);
    }
    rc = engine_rma_complete(w);
    w->access_epoch = false;
    w->access_targets.clear();
    return err_win(w, "MPI_Win_complete", rc);
}

// MPID_Win_wait (win.cpp:4077-4088): returns once every origin of the posted
// group completed; with no exposure epoch open there is nothing to wait for
MSX_EXPORT int MPI_Win_wait(MPI_Win win)
{
    MSX_REQUIRE_INIT("MPI_Win_wait");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Win_wait", rc);
    if (!w->exposure_epoch) return MPI_SUCCESS;
    int flag = 0;
    rc = engine_rma_wait(w, true, &flag);
    if (rc == MPI_SUCCESS) {
        w->exposure_epoch = false;
        w->exposure_origins.clear();
    }
    return err_win(w, "MPI_Win_wait", rc);
}

// MPID_Win_test (win.cpp:2001-2012): the non-blocking MPI_Win_wait
MSX_EXPORT int MPI_Win_test(MPI_Win win, int* flag)
{
    MSX_REQUIRE_INIT("MPI_Win_test");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Win_test", rc);
    if (!flag) { set_error("null flag"); return err_win(w, "MPI_Win_test", MPI_ERR_ARG); }
    if (!w->exposure_epoch) { *flag = 1; return MPI_SUCCESS; }
    rc = engine_rma_wait(w, false, flag);
    if (rc == MPI_SUCCESS && *flag) {
        w->exposure_epoch = false;
        w->exposure_origins.clear();
    }
    return err_win(w, "MPI_Win_test", rc);
}

// api/mpi_win.cpp:979-1030: the group of the window's communicator
MSX_EXPORT int MPI_Win_get_group(MPI_Win win, MPI_Group* group)
{
    MSX_REQUIRE_INIT("MPI_Win_get_group");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Win_get_group", rc);
    if (!group) { set_error("null group"); return err_win(w, "MPI_Win_get_group", MPI_ERR_ARG); }
    return err_win(w, "MPI_Win_get_group", group_create(w->comm->lpid, group));
}

// MPID_Win_lock_all: a shared lock on every rank (mpid/win.cpp:4133-4150)
MSX_EXPORT int MPI_Win_lock_all(int assert_, MPI_Win win)
{
    MSX_REQUIRE_INIT("MPI_Win_lock_all");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Win_lock_all", rc);
    for (int r = 0; rc == MPI_SUCCESS && r < w->comm->size; ++r) rc = win_lock(w, MPI_LOCK_SHARED, r, assert_);
    if (rc == MPI_SUCCESS) w->lock_all = true;
    return err_win(w, "MPI_Win_lock_all", rc);
}

MSX_EXPORT int MPI_Win_unlock_all(MPI_Win win)
{
    MSX_REQUIRE_INIT("MPI_Win_unlock_all");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Win_unlock_all", rc);
    if (!w->lock_all) {
        set_error("MPI_Win_unlock_all without MPI_Win_lock_all (**rmasync)");
        return err_win(w, "MPI_Win_unlock_all", MPI_ERR_OTHER);
    }
    for (int r = 0; r < w->comm->size; ++r) {
        const int r2 = w->lock_mode[(size_t)r] ? win_unlock(w, r) : MPI_SUCCESS;
        if (rc == MPI_SUCCESS) rc = r2;
    }
    w->lock_all = false;
    return err_win(w, "MPI_Win_unlock_all", rc);
}

// Flush: every operation this rank issued to `rank` is complete at origin and
// target (a fetch has landed; an update is visible to the target's next
// access).  flush_local needs only origin completion, which is the same here.
MSX_EXPORT int MPI_Win_flush(int rank, MPI_Win win)
{
    MSX_REQUIRE_INIT("MPI_Win_flush");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Win_flush", rc);
    rc = v_lock_rank(w, rank);
    if (rc == MPI_SUCCESS && rank != MPI_PROC_NULL) rc = engine_rma_flush(w, rank);
    return err_win(w, "MPI_Win_flush", rc);
}

MSX_EXPORT int MPI_Win_flush_local(int rank, MPI_Win win)
{
    MSX_REQUIRE_INIT("MPI_Win_flush_local");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Win_flush_local", rc);
    rc = v_lock_rank(w, rank);
    if (rc == MPI_SUCCESS && rank != MPI_PROC_NULL) rc = engine_rma_flush(w, rank);
    return err_win(w, "MPI_Win_flush_local", rc);
}

namespace {
int flush_all(RmaWin* w)
{
    int rc = MPI_SUCCESS;
    for (int r = 0; r < w->comm->size; ++r) {
        const int r2 = engine_rma_flush(w, r);
        if (rc == MPI_SUCCESS) rc = r2;
    }
    return rc;
}
}  // namespace

MSX_EXPORT int MPI_Win_flush_all(MPI_Win win)
{
    MSX_REQUIRE_INIT("MPI_Win_flush_all");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Win_flush_all", rc);
    return err_win(w, "MPI_Win_flush_all", flush_all(w));
}

MSX_EXPORT int MPI_Win_flush_local_all(MPI_Win win)
{
    MSX_REQUIRE_INIT("MPI_Win_flush_local_all");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Win_flush_local_all", rc);
    return err_win(w, "MPI_Win_flush_local_all", flush_all(w));
}

// MPI_Win_sync: public and private copies of the window agree.  Remote
// updates are applied by this rank's own service thread on this GPU and are
// complete (stream-synchronised) before their origin's flush returns, so
// a memory fence for the host-side view is all that is left.
MSX_EXPORT int MPI_Win_sync(MPI_Win win)
{
    MSX_REQUIRE_INIT("MPI_Win_sync");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Win_sync", rc);
    std::atomic_thread_fence(std::memory_order_seq_cst);
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Win_set_errhandler(MPI_Win win, MPI_Errhandler eh)
{
    MSX_REQUIRE_INIT("MPI_Win_set_errhandler");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc == MPI_SUCCESS && eh != MPI_ERRORS_ARE_FATAL && eh != MPI_ERRORS_RETURN) {
        set_error("unsupported errhandler 0x%x", eh);
        rc = MPI_ERR_ARG;
    }
    if (rc != MPI_SUCCESS) return err_win(w, "MPI_Win_set_errhandler", rc);
    w->errhandler = eh;
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Win_get_errhandler(MPI_Win win, MPI_Errhandler* eh)
{
    MSX_REQUIRE_INIT("MPI_Win_get_errhandler");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc == MPI_SUCCESS && !eh) rc = MPI_ERR_ARG;
    if (rc != MPI_SUCCESS) return err_win(w, "MPI_Win_get_errhandler", rc);
    *eh = w->errhandler == MPI_ERRHANDLER_NULL ? MPI_ERRORS_ARE_FATAL : w->errhandler;
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Put(const void* origin_addr, int origin_count, MPI_Datatype origin_datatype, int target_rank,
                       MPI_Aint target_disp, int target_count, MPI_Datatype target_datatype, MPI_Win win)
{
    MSX_REQUIRE_INIT("MPI_Put");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Put", rc);
    rc = v_dtype_any(origin_addr, origin_count, origin_datatype);
    if (rc == MPI_SUCCESS) rc = v_target(w, target_count, target_datatype, target_rank, target_disp);
    if (rc == MPI_SUCCESS && target_rank != MPI_PROC_NULL && origin_count > 0)
        rc = v_match(origin_count, origin_datatype, target_count, target_datatype);
    if (rc == MPI_SUCCESS && target_rank != MPI_PROC_NULL && origin_count > 0)
        rc = rma_issue(w, RMA_PUT, target_rank, target_disp, O_REPLACE, origin_addr, origin_count, origin_datatype,
                       nullptr, 0, MPI_DATATYPE_NULL, target_count, target_datatype, nullptr);
    return err_win(w, "MPI_Put", rc);
}

MSX_EXPORT int MPI_Get(void* origin_addr, int origin_count, MPI_Datatype origin_datatype, int target_rank,
                       MPI_Aint target_disp, int target_count, MPI_Datatype target_datatype, MPI_Win win)
{
    MSX_REQUIRE_INIT("MPI_Get");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Get", rc);
    rc = v_dtype_any(origin_addr, origin_count, origin_datatype);
    if (rc == MPI_SUCCESS) rc = v_target(w, target_count, target_datatype, target_rank, target_disp);
    if (rc == MPI_SUCCESS && target_rank != MPI_PROC_NULL && origin_count > 0)
        rc = v_match(origin_count, origin_datatype, target_count, target_datatype);
    if (rc == MPI_SUCCESS && target_rank != MPI_PROC_NULL && origin_count > 0)
        rc = rma_issue(w, RMA_GET, target_rank, target_disp, O_NOOP, nullptr, 0, MPI_DATATYPE_NULL, origin_addr,
                       origin_count, origin_datatype, target_count, target_datatype, nullptr);
    return err_win(w, "MPI_Get", rc);
}

MSX_EXPORT int MPI_Accumulate(const void* origin_addr, int origin_count, MPI_Datatype origin_datatype,
                              int target_rank, MPI_Aint target_disp, int target_count,
                              MPI_Datatype target_datatype, MPI_Op op, MPI_Win win)
{
    MSX_REQUIRE_INIT("MPI_Accumulate");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Accumulate", rc);
    OpRef r;
    rc = v_dtype_any(origin_addr, origin_count, origin_datatype);
    if (rc == MPI_SUCCESS) rc = rma_op(op, &r, false);
    if (rc == MPI_SUCCESS) rc = v_target(w, target_count, target_datatype, target_rank, target_disp);
    if (rc == MPI_SUCCESS && target_rank != MPI_PROC_NULL && origin_count > 0)
        rc = v_match(origin_count, origin_datatype, target_count, target_datatype);
    if (rc == MPI_SUCCESS && target_rank != MPI_PROC_NULL && origin_count > 0)
        rc = rma_issue(w, RMA_ACC, target_rank, target_disp, r.opidx, origin_addr, origin_count, origin_datatype,
                       nullptr, 0, MPI_DATATYPE_NULL, target_count, target_datatype, nullptr);
    return err_win(w, "MPI_Accumulate", rc);
}

MSX_EXPORT int MPI_Get_accumulate(const void* origin_addr, int origin_count, MPI_Datatype origin_datatype,
                                  void* result_addr, int result_count, MPI_Datatype result_datatype,
                                  int target_rank, MPI_Aint target_disp, int target_count,
                                  MPI_Datatype target_datatype, MPI_Op op, MPI_Win win)
{
    MSX_REQUIRE_INIT("MPI_Get_accumulate");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Get_accumulate", rc);
    OpRef r;
    rc = v_op_handle(op, &r);
    const bool noop = rc == MPI_SUCCESS && r.opidx == O_NOOP;
    if (rc == MPI_SUCCESS && !noop) rc = v_dtype_any(origin_addr, origin_count, origin_datatype);
    if (rc == MPI_SUCCESS) rc = v_dtype_any(result_addr, result_count, result_datatype);
    if (rc == MPI_SUCCESS) rc = v_target(w, target_count, target_datatype, target_rank, target_disp);
    if (rc == MPI_SUCCESS) rc = rma_op(op, &r, true);
    if (rc == MPI_SUCCESS && target_rank != MPI_PROC_NULL && result_count > 0) {
        rc = v_match(result_count, result_datatype, target_count, target_datatype);
        if (rc == MPI_SUCCESS && !noop) rc = v_match(origin_count, origin_datatype, target_count, target_datatype);
    }
    if (rc == MPI_SUCCESS && target_rank != MPI_PROC_NULL && target_count > 0)
        rc = rma_issue(w, noop ? RMA_GET : RMA_GACC, target_rank, target_disp, r.opidx, origin_addr, origin_count,
                       origin_datatype, result_addr, result_count, result_datatype, target_count, target_datatype,
                       nullptr);
    return err_win(w, "MPI_Get_accumulate", rc);
}

MSX_EXPORT int MPI_Fetch_and_op(const void* origin_addr, void* result_addr, MPI_Datatype datatype,
                                int target_rank, MPI_Aint target_disp, MPI_Op op, MPI_Win win)
{
    MSX_REQUIRE_INIT("MPI_Fetch_and_op");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Fetch_and_op", rc);
    OpRef r;
    rc = v_op_handle(op, &r);
    const bool noop = rc == MPI_SUCCESS && r.opidx == O_NOOP;
    if (rc == MPI_SUCCESS && !noop) rc = v_dtype(origin_addr, 1, datatype);
    if (rc == MPI_SUCCESS) rc = v_dtype(result_addr, 1, datatype);
    if (rc == MPI_SUCCESS) rc = v_target(w, 1, datatype, target_rank, target_disp);
    if (rc == MPI_SUCCESS) rc = rma_op(op, &r, true);
    if (rc == MPI_SUCCESS && target_rank != MPI_PROC_NULL)
        rc = rma_issue(w, noop ? RMA_GET : RMA_GACC, target_rank, target_disp, r.opidx, origin_addr, 1, datatype,
                       result_addr, 1, datatype, 1, datatype, nullptr);
    return err_win(w, "MPI_Fetch_and_op", rc);
}

MSX_EXPORT int MPI_Compare_and_swap(const void* origin_addr, const void* compare_addr, void* result_addr,
                                    MPI_Datatype datatype, int target_rank, MPI_Aint target_disp, MPI_Win win)
{
    MSX_REQUIRE_INIT("MPI_Compare_and_swap");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Compare_and_swap", rc);
    rc = v_dtype(origin_addr, 1, datatype);
    if (rc == MPI_SUCCESS) rc = v_dtype(compare_addr, 1, datatype);
    if (rc == MPI_SUCCESS) rc = v_dtype(result_addr, 1, datatype);
    if (rc == MPI_SUCCESS) rc = v_target(w, 1, datatype, target_rank, target_disp);
    if (rc == MPI_SUCCESS && target_rank != MPI_PROC_NULL)
        rc = rma_issue(w, RMA_CAS, target_rank, target_disp, O_REPLACE, origin_addr, 1, datatype, result_addr, 1,
                       datatype, 1, datatype, compare_addr);
    return err_win(w, "MPI_Compare_and_swap", rc);
}

// ---- request-based RMA (api/mpi_rma.cpp:187 MPI_Rput, 486 MPI_Rget, 813
// MPI_Raccumulate, 1215 MPI_Rget_accumulate; MPID_Win_R* mpid/win.cpp:1324-1900).
// The operation is validated and queued exactly as its plain form.  Its request
// must complete without a synchronisation call, so the target's queue is
// flushed at once (the reference completes the request when its queued
// operation has gone out, at the latest at the next flush / unlock) and a
// complete request is returned.  Passive-target epochs only (MPI-3 11.3.5):
// in a fence or PSCW epoch the call fails with MPI_ERR_RMA_SYNC.
namespace {
int rma_request_pre(RmaWin* w, MPI_Request* request, int target)
{
    if (!request) { set_error("**nullptr request"); return MPI_ERR_ARG; }
    *request = MPI_REQUEST_NULL;
    if (target != MPI_PROC_NULL && target >= 0 && target < w->comm->size && !w->lock_all &&
        !w->lock_mode[(size_t)target]) {
        set_error("request-based RMA outside a passive-target epoch on rank %d (**rmasync)", target);
        return MPI_ERR_RMA_SYNC;
    }
    return MPI_SUCCESS;
}

int rma_request_post(RmaWin* w, int target, int rc, MPI_Request* request)
{
    if (rc == MPI_SUCCESS && target != MPI_PROC_NULL) rc = engine_rma_flush(w, target);
    if (rc == MPI_SUCCESS) rc = request_completed_rma(request, MPI_SUCCESS);
    return rc;
}
}  // namespace

MSX_EXPORT int MPI_Rput(const void* origin_addr, int origin_count, MPI_Datatype origin_datatype, int target_rank,
                        MPI_Aint target_disp, int target_count, MPI_Datatype target_datatype, MPI_Win win,
                        MPI_Request* request)
{
    MSX_REQUIRE_INIT("MPI_Rput");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Rput", rc);
    rc = rma_request_pre(w, request, target_rank);
    if (rc == MPI_SUCCESS) rc = v_dtype_any(origin_addr, origin_count, origin_datatype);
    if (rc == MPI_SUCCESS) rc = v_target(w, target_count, target_datatype, target_rank, target_disp);
    if (rc == MPI_SUCCESS && target_rank != MPI_PROC_NULL && origin_count > 0)
        rc = v_match(origin_count, origin_datatype, target_count, target_datatype);
    if (rc == MPI_SUCCESS && target_rank != MPI_PROC_NULL && origin_count > 0)
        rc = rma_issue(w, RMA_PUT, target_rank, target_disp, O_REPLACE, origin_addr, origin_count, origin_datatype,
                       nullptr, 0, MPI_DATATYPE_NULL, target_count, target_datatype, nullptr);
    if (rc == MPI_SUCCESS) rc = rma_request_post(w, target_rank, rc, request);
    return err_win(w, "MPI_Rput", rc);
}

MSX_EXPORT int MPI_Rget(void* origin_addr, int origin_count, MPI_Datatype origin_datatype, int target_rank,
                        MPI_Aint target_disp, int target_count, MPI_Datatype target_datatype, MPI_Win win,
                        MPI_Request* request)
{
    MSX_REQUIRE_INIT("MPI_Rget");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Rget", rc);
    rc = rma_request_pre(w, request, target_rank);
    if (rc == MPI_SUCCESS) rc = v_dtype_any(origin_addr, origin_count, origin_datatype);
    if (rc == MPI_SUCCESS) rc = v_target(w, target_count, target_datatype, target_rank, target_disp);
    if (rc == MPI_SUCCESS && target_rank != MPI_PROC_NULL && origin_count > 0)
        rc = v_match(origin_count, origin_datatype, target_count, target_datatype);
    if (rc == MPI_SUCCESS && target_rank != MPI_PROC_NULL && origin_count > 0)
        rc = rma_issue(w, RMA_GET, target_rank, target_disp, O_NOOP, nullptr, 0, MPI_DATATYPE_NULL, origin_addr,
                       origin_count, origin_datatype, target_count, target_datatype, nullptr);
    if (rc == MPI_SUCCESS) rc = rma_request_post(w, target_rank, rc, request);
    return err_win(w, "MPI_Rget", rc);
}

MSX_EXPORT int MPI_Raccumulate(const void* origin_addr, int origin_count, MPI_Datatype origin_datatype,
                               int target_rank, MPI_Aint target_disp, int target_count,
                               MPI_Datatype target_datatype, MPI_Op op, MPI_Win win, MPI_Request* request)
{
    MSX_REQUIRE_INIT("MPI_Raccumulate");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Raccumulate", rc);
    OpRef r;
    rc = rma_request_pre(w, request, target_rank);
    if (rc == MPI_SUCCESS) rc = v_dtype_any(origin_addr, origin_count, origin_datatype);
    if (rc == MPI_SUCCESS) rc = rma_op(op, &r, false);        // MPI_NO_OP: **noopnotallowed
    if (rc == MPI_SUCCESS) rc = v_target(w, target_count, target_datatype, target_rank, target_disp);
    if (rc == MPI_SUCCESS && target_rank != MPI_PROC_NULL && origin_count > 0)
        rc = v_match(origin_count, origin_datatype, target_count, target_datatype);
    if (rc == MPI_SUCCESS && target_rank != MPI_PROC_NULL && origin_count > 0)
        rc = rma_issue(w, RMA_ACC, target_rank, target_disp, r.opidx, origin_addr, origin_count, origin_datatype,
                       nullptr, 0, MPI_DATATYPE_NULL, target_count, target_datatype, nullptr);
    if (rc == MPI_SUCCESS) rc = rma_request_post(w, target_rank, rc, request);
    return err_win(w, "MPI_Raccumulate", rc);
}

MSX_EXPORT int MPI_Rget_accumulate(const void* origin_addr, int origin_count, MPI_Datatype origin_datatype,
                                   void* result_addr, int result_count, MPI_Datatype result_datatype,
                                   int target_rank, MPI_Aint target_disp, int target_count,
                                   MPI_Datatype target_datatype, MPI_Op op, MPI_Win win, MPI_Request* request)
{
    MSX_REQUIRE_INIT("MPI_Rget_accumulate");
    RmaWin* w;
    int rc = v_win(win, &w);
    if (rc != MPI_SUCCESS) return err_win(nullptr, "MPI_Rget_accumulate", rc);
    OpRef r;
    rc = rma_request_pre(w, request, target_rank);
    if (rc == MPI_SUCCESS) rc = v_op_handle(op, &r);
    const bool noop = rc == MPI_SUCCESS && r.opidx == O_NOOP;
    if (rc == MPI_SUCCESS && !noop) rc = v_dtype_any(origin_addr, origin_count, origin_datatype);
    if (rc == MPI_SUCCESS) rc = v_dtype_any(result_addr, result_count, result_datatype);
    if (rc == MPI_SUCCESS) rc = v_target(w, target_count, target_datatype, target_rank, target_disp);
    if (rc == MPI_SUCCESS) rc = rma_op(op, &r, true);
    if (rc == MPI_SUCCESS && target_rank != MPI_PROC_NULL && result_count > 0) {
        rc = v_match(result_count, result_datatype, target_count, target_datatype);
        if (rc == MPI_SUCCESS && !noop) rc = v_match(origin_count, origin_datatype, target_count, target_datatype);
    }
    if (rc == MPI_SUCCESS && target_rank != MPI_PROC_NULL && target_count > 0)
        rc = rma_issue(w, noop ? RMA_GET : RMA_GACC, target_rank, target_disp, r.opidx, origin_addr, origin_count,
                       origin_datatype, result_addr, result_count, result_datatype, target_count, target_datatype,
                       nullptr);
    if (rc == MPI_SUCCESS) rc = rma_request_post(w, target_rank, rc, request);
    return err_win(w, "MPI_Rget_accumulate", rc);
}

// ===========================================================================
// device-side extension ABI (include/msx.h)
// ===========================================================================
// Build provenance: MSX_SOURCE_HASH is the SHA-256 prefix of the library's
// sources and headers at build time (Makefile), so a test can tell whether a
// prebuilt .so was compiled from the tree it ships with (tests/test_abi.py).
#ifndef MSX_SOURCE_HASH
#define MSX_SOURCE_HASH "unknown"
#endif
MSX_EXPORT const char* msx_version(void) { return "msmpi-mi355x 0.1 (gfx950) src=" MSX_SOURCE_HASH; }

MSX_EXPORT const char* msx_engine_transport(void)
{
    Comm* c = world();
    return engine_transport_name(c ? c->tp : nullptr);
}
MSX_EXPORT int msx_engine_gpu_shared(void)
{
    Comm* c = world();
    if (!c) return -1;
    return c->tp && c->tp->gpu_shared ? 1 : 0;
}
MSX_EXPORT int msx_engine_stats(double* out, int n, int reset)
{
    if (!out || n < 0) return -1;
    return engine_stats(out, n, reset);
}
MSX_EXPORT int msx_peer_write_bandwidth(int64_t bytes_per_peer, int reps, double* seconds, int64_t* bytes_used)
{
    MSX_REQUIRE_INIT("msx_peer_write_bandwidth");
    if (!seconds || !bytes_used || bytes_per_peer <= 0 || reps <= 0) return MPI_ERR_ARG;
    Comm* c = world();
    return engine_peer_write_probe(c, (size_t)bytes_per_peer, reps, seconds, bytes_used);
}
MSX_EXPORT int msx_device_count(void) { return device_count_noinit(); }
MSX_EXPORT const char* msx_last_error(void) { return last_error(); }

MSX_EXPORT int msx_op_check(MPI_Op op, MPI_Datatype dt)
{
    OpRef r;
    return v_op(op, dt, &r);
}

MSX_EXPORT int msx_type_size(MPI_Datatype dt) { return type_size(dt); }

// ---- the builtin op table (MPIR_Op_table, mpid/op.cpp:618-622, :703-1923) ----
// Each entry has the MPI_User_function shape the reference's internal callers
// bind to: NBC reduce tasks (mpid/tasks.cpp:667,680), RMA accumulate
// (mpid/win.cpp:1435, packethandling.cpp:2938,3046), the Fortran proxy
// (fortran/mpif.cpp:963-976) and MPID_Uop_call (include/op.h:171-174).  Like
// MPIR_Op_<op> they validate nothing up front: `*len` <= 0 does nothing (the
// reference loops `while(--len >= 0)`), and a datatype outside the op's table
// leaves inout untouched and sets the calling thread's op_errno to MPI_ERR_OP
// (op.cpp:732,...,1791; Mpi.CallState->op_errno, include/MpiCallState.h:13).
// Device operands (or pinned / pageable host memory, offloaded like
// MPI_Reduce_local) are combined by the gfx950 kernels; the call returns with
// the result in `inout`.  A failure of the GPU path also lands in op_errno.
namespace {
thread_local int t_op_errno = 0;

void op_entry(int opidx, void* in, void* inout, int* len, MPI_Datatype* dt)
{
    if (!len || !dt || *len <= 0) return;
    if (op_check_dtype(opidx, *dt) != MPI_SUCCESS) {
        set_error("**opundefined: builtin op %d on datatype 0x%x", opidx, *dt);
        t_op_errno = MPI_ERR_OP;
        return;
    }
    const int rc = reduce_local_any(opidx, type_info(*dt)->kind, in, inout, (size_t)*len);
    if (rc != MPI_SUCCESS) t_op_errno = rc;
}
}  // namespace

#define MSX_OP_ENTRY(fn, idx) \
    MSX_EXPORT void fn(void* in, void* inout, int* len, MPI_Datatype* dt) { op_entry(idx, in, inout, len, dt); }
MSX_OP_ENTRY(msx_op_max, O_MAX)
MSX_OP_ENTRY(msx_op_min, O_MIN)
MSX_OP_ENTRY(msx_op_sum, O_SUM)
MSX_OP_ENTRY(msx_op_prod, O_PROD)
MSX_OP_ENTRY(msx_op_land, O_LAND)
MSX_OP_ENTRY(msx_op_band, O_BAND)
MSX_OP_ENTRY(msx_op_lor, O_LOR)
MSX_OP_ENTRY(msx_op_bor, O_BOR)
MSX_OP_ENTRY(msx_op_lxor, O_LXOR)
MSX_OP_ENTRY(msx_op_bxor, O_BXOR)
MSX_OP_ENTRY(msx_op_minloc, O_MINLOC)
MSX_OP_ENTRY(msx_op_maxloc, O_MAXLOC)
#undef MSX_OP_ENTRY

// MPIR_Op_replace (op.cpp:1886-1903): MPIR_Localcopy(in -> inout), any datatype
MSX_EXPORT void msx_op_replace(void* in, void* inout, int* len, MPI_Datatype* dt)
{
    if (!len || !dt || *len <= 0) return;
    const int rc = local_copy(in, inout, (size_t)*len, *dt);
    if (rc != MPI_SUCCESS) t_op_errno = rc;
}

// MPIR_Op_noop (op.cpp:1906-1923)
MSX_EXPORT void msx_op_noop(void*, void*, int*, MPI_Datatype*) {}

// MPIR_Op_table[op % 16 - 1]: the entry of a builtin op handle
// (MPI_MAX .. MPI_NO_OP, 0x58000001 .. 0x5800000e), NULL for anything else.
MSX_EXPORT MPI_User_function* msx_op_table(MPI_Op op)
{
    static MPI_User_function* const kTable[] = {
        msx_op_max, msx_op_min, msx_op_sum, msx_op_prod, msx_op_land, msx_op_band, msx_op_lor,
        msx_op_bor, msx_op_lxor, msx_op_bxor, msx_op_minloc, msx_op_maxloc, msx_op_replace, msx_op_noop};
    static_assert(sizeof(kTable) / sizeof(kTable[0]) == O_NOOP, "one entry per builtin op");
    const int idx = op & 0xff;
    if ((op & ~0xff) != (MPI_MAX & ~0xff) || idx < O_MAX || idx > O_NOOP) return nullptr;
    return kTable[idx - 1];
}

// The routing test of the table binding: both operands in
// device memory.  Host operands stay on the reference's own MPIR_Op_<op> loop,
// which the offload beats only above ~1 MiB (bench.py host_path.crossover);
// the library itself has no CPU combine.  No GPU -> 0, without initialising one.
MSX_EXPORT int msx_operands_on_device(const void* in, const void* inout)
{
    if (!in || !inout || device_count_noinit() <= 0) return 0;
    return classify(in).place == Place::Device && classify(inout).place == Place::Device ? 1 : 0;
}

// Mpi.CallState->op_errno of the calling thread: read it, and clear it before
// a sequence of calls (the collectives do `op_errno = 0`, reduce.cpp:97,3794).
MSX_EXPORT int msx_op_errno(void) { return t_op_errno; }
MSX_EXPORT void msx_op_errno_reset(void) { t_op_errno = 0; }

MSX_EXPORT int msx_reduce_local_dev(const void* in, void* inout, int64_t count, MPI_Datatype dt,
                                    MPI_Op op, void* stream)
{
    if (count == 0) return MPI_SUCCESS;
    OpRef r;
    int rc = v_op(op, dt, &r);
    if (rc != MPI_SUCCESS) return rc;
    if (r.opidx == O_NULL) { set_error("device entry point takes builtin ops only"); return MPI_ERR_OP; }
    if (count < 0) { set_error("negative count"); return MPI_ERR_COUNT; }
    if (!in || !inout) { set_error("null buffer"); return MPI_ERR_BUFFER; }
    if (in == inout) { set_error("inbuf aliases inoutbuf"); return MPI_ERR_BUFFER; }
    rc = ensure_device();
    if (rc != MPI_SUCCESS) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);   // NULL = the HIP null stream
    return reduce_local_device(r.opidx, type_info(dt)->kind, in, inout, (size_t)count, s);
}

// one MPI_Reduce_local-sized vector split over the node's GPUs
// (ngpus <= 0: all visible), host operands over each GPU's own PCIe link;
// MPI_Reduce_local's checks, error codes returned (no error handler).
MSX_EXPORT int msx_reduce_local_multi(const void* in, void* inout, int64_t count, MPI_Datatype dt, MPI_Op op,
                                      int ngpus)
{
    if (count == 0) return MPI_SUCCESS;
    OpRef r;
    int rc = v_op(op, dt, &r);
    if (rc != MPI_SUCCESS) return rc;
    if (r.opidx == O_NULL || !type_info(dt)) { set_error("multi-GPU entry point takes builtin ops only"); return MPI_ERR_OP; }
    if (count < 0) { set_error("negative count"); return MPI_ERR_COUNT; }
    if (!in || !inout) { set_error("null buffer"); return MPI_ERR_BUFFER; }
    if (in == inout) { set_error("inbuf aliases inoutbuf"); return MPI_ERR_BUFFER; }
    return reduce_local_multi(r.opidx, type_info(dt)->kind, in, inout, (size_t)count, ngpus);
}

MSX_EXPORT int msx_reduce_tree_dev(const void* const* srcs, int p, void* out, int64_t count,
                                   MPI_Datatype dt, MPI_Op op, void* stream)
{
    if (count == 0) return MPI_SUCCESS;
    OpRef r;
    int rc = v_op(op, dt, &r);
    if (rc != MPI_SUCCESS) return rc;
    if (r.opidx == O_NULL) { set_error("device entry point takes builtin ops only"); return MPI_ERR_OP; }
    if (count < 0) { set_error("negative count"); return MPI_ERR_COUNT; }
    if (!srcs || !out || !(p == 1 || p == 2 || p == 4 || p == 8 || p == 16)) {
        set_error("bad tree arguments (p=%d)", p);
        return MPI_ERR_ARG;
    }
    rc = ensure_device();
    if (rc != MPI_SUCCESS) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);   // NULL = the HIP null stream
    hipError_t e = launch_tree(r.opidx, type_info(dt)->kind, srcs, p, out, (size_t)count, s);
    return e == hipSuccess ? MPI_SUCCESS : hip_fail(e, "tree kernel launch");
}

// Any reference-order tree the engine evaluates (TreeSpec): P leaves (a power
// of two <= 16) over srcs[2k] (leaf k) and srcs[2k+1] (its fold pair when bit
// k of pairmask is set), leaves >= nleaves absent (0 = all present); or, with
// chain set, the left-deep chain over srcs[0..P-1].  Stream-ordered, device
// pointers.  For tests and probes of the tree kernels outside a collective.
MSX_EXPORT int msx_reduce_tree_spec_dev(const void* const* srcs, int P, unsigned pairmask, int nleaves, int chain,
                                        void* out, int64_t count, MPI_Datatype dt, MPI_Op op, void* stream)
{
    if (count == 0) return MPI_SUCCESS;
    OpRef r;
    int rc = v_op(op, dt, &r);
    if (rc != MPI_SUCCESS) return rc;
    if (r.opidx == O_NULL) { set_error("device entry point takes builtin ops only"); return MPI_ERR_OP; }
    if (count < 0) { set_error("negative count"); return MPI_ERR_COUNT; }
    const bool pow2 = P >= 1 && P <= 16 && (P & (P - 1)) == 0;
    if (!srcs || !out || (chain ? (P < 1 || P > 16) : !pow2) || nleaves < 0 || nleaves > P ||
        (!chain && (pairmask >> P) != 0)) {
        set_error("bad tree spec (P=%d pairmask=0x%x nleaves=%d chain=%d)", P, pairmask, nleaves, chain);
        return MPI_ERR_ARG;
    }
    rc = ensure_device();
    if (rc != MPI_SUCCESS) return rc;
    TreeSpec t;
    t.P = P;
    t.chain = chain != 0;
    t.pairmask = chain ? 0 : pairmask;
    t.nleaves = chain ? 0 : nleaves;
    const int ns = chain ? P : 2 * P;
    for (int i = 0; i < ns; ++i) t.src[i] = srcs[i];
    hipError_t e = launch_tree_spec(r.opidx, type_info(dt)->kind, t, out, (size_t)count, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? MPI_SUCCESS : hip_fail(e, "tree kernel launch");
}

// The engine's local copy (the collect step of the collectives, MPIR_Localcopy
// of device data, mpid/pt2pt.cpp:929-948): k_copy_segs' XCD-contiguous 4-KiB
// tiles up to 16 MiB, k_copy_dram's one-wave dispatch-order grid above.
// Stream-ordered, device pointers (tests of the copy kernels).
MSX_EXPORT int msx_copy_dev(void* dst, const void* src, int64_t bytes, void* stream)
{
    if (bytes < 0 || (bytes > 0 && (!dst || !src))) return MPI_ERR_ARG;
    if (bytes == 0) return MPI_SUCCESS;
    int rc = ensure_device();
    if (rc != MPI_SUCCESS) return rc;
    const void* ps = src;
    void* pd = dst;
    size_t n = (size_t)bytes;
    hipError_t e = launch_copy_segs(&ps, &pd, &n, 1, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? MPI_SUCCESS : hip_fail(e, "copy kernel launch");
}

// Test hook: the pack/unpack/accumulate kernel geometry (0 = by size, the
// default; 1 = grid-stride form; 2 = tile form at every size), so small test
// cases run the kernels the default takes at large sizes.
MSX_EXPORT int msx_tune_pack(int mode)
{
    return pack_tune_set(mode) == 0 ? MPI_SUCCESS : MPI_ERR_ARG;
}

MSX_EXPORT int msx_set_staging_chunk(int64_t bytes)
{
    if (bytes <= 0) return MPI_ERR_ARG;
    set_staging_chunk((size_t)bytes);
    return MPI_SUCCESS;
}

MSX_EXPORT int msx_set_host_mode(int mode)
{
    if (mode < 0 || mode > 2) { set_error("host mode must be 0, 1 or 2"); return MPI_ERR_ARG; }
    set_host_mode(mode);
    return MPI_SUCCESS;
}

// ---- schedule introspection (host-side tests of the collective engine) ------
#include "msx_transport.h"

// which: 0 = allreduce tree of newrank n, 1 = reduce_scatter (recursive
// halving) tree of newrank n, 2 = pairwise chain of real rank n.
// src32 receives real ranks per kernel slot (-1 = unused).
MSX_EXPORT int msx_schedule_tree(int which, int p, int n, int* src32, int* P, unsigned* pairmask,
                                 int* chain)
{
    if (p < 1 || p > 16 || !src32 || !P || !pairmask || !chain) return MPI_ERR_ARG;
    RankTree t;
    if (which == 0) t = tree_allreduce(p, n);
    else if (which == 1) t = tree_reduce_scatter(p, n);
    else if (which == 2) t = tree_pairwise(p, n);
    else if (which == 3) t = tree_reduce_rsag(p, n);
    else if (which == 4) t = tree_reduce_binomial(p, n);
    else return MPI_ERR_ARG;
    for (int i = 0; i < 32; ++i) src32[i] = t.src[i];
    *P = t.P;
    if (t.nleaves) {   // absent leaves are reported as -1
        for (int i = 2 * t.nleaves; i < 32; ++i) src32[i] = -1;
    }
    *pairmask = t.pairmask;
    *chain = t.chain ? 1 : 0;
    return MPI_SUCCESS;
}

// which: 0 = allreduce algorithm, 1 = reduce_scatter algorithm (Algo enum)
MSX_EXPORT int msx_schedule_algo(int which, int p, int64_t count, int type_size)
{
    if (which == 0) return allreduce_algo(p, (size_t)count, type_size, true);
    if (which == 2) return reduce_algo(p, (size_t)count, type_size, true);
    return reduce_scatter_algo(p, (size_t)count, type_size, true);
}

// The same, with the gate's bytes per element taken from the datatype as the
// reference does: MPI_Type_size for the blocking calls and every reduce_scatter,
// the extent for the NBC task lists of MPI_Iallreduce / MPI_Ireduce (nbc = 1).
MSX_EXPORT int msx_schedule_algo_dt(int which, int p, int64_t count, MPI_Datatype dt, int nbc)
{
    if (!dtype_lookup(dt)) return -1;
    const int gate = gate_type_size(dt, which != 1 && nbc != 0);
    return msx_schedule_algo(which, p, count, gate);
}

// MPI_Ireduce's Rabenseifner tree of newrank n for `root` (root-relative ranks,
// reduce.cpp:6267-6670); same reporting as msx_schedule_tree
MSX_EXPORT int msx_schedule_ireduce_tree(int p, int n, int root, int* src32, int* P, unsigned* pairmask,
                                         int* chain)
{
    if (p < 1 || p > 16 || root < 0 || root >= p || !src32 || !P || !pairmask || !chain) return MPI_ERR_ARG;
    const RankTree t = tree_ireduce_rsag(p, n, root);
    for (int i = 0; i < 32; ++i) src32[i] = t.src[i];
    *P = t.P;
    *pairmask = t.pairmask;
    *chain = 0;
    return MPI_SUCCESS;
}

// newrank of `rank`, and the allreduce block owned by newrank n
MSX_EXPORT int msx_schedule_newrank(int rank, int p) { return newrank_of(rank, p); }
// The pipelined two-step allreduce / reduce's plan for one rank (tests): the
// chunk length in elements, and every range of that rank's pieces over all
// chunks as (first element, end element, owner newrank) triples in out[3i..];
// returns the number of ranges, or -1 when `cap` triples do not suffice.
MSX_EXPORT int64_t msx_schedule_two_step(int p, int64_t count, int esz, int rank, int64_t* chunk_el, int64_t* out,
                                         int64_t cap)
{
    if (p < 2 || p > 32 || count <= 0 || esz <= 0 || rank < 0 || rank >= p || !chunk_el || !out) return -1;
    const size_t pc = two_step_chunk_el(p, (size_t)esz);
    *chunk_el = (int64_t)pc;
    if (pc == 0) return 0;
    std::vector<TwoStepRange> ranges;
    int64_t n = 0;
    for (size_t ci = 0; ci * pc < (size_t)count; ++ci) {
        size_t plo, phi, len;
        two_step_plan(p, (size_t)count, pc, ci, rank, &ranges, &plo, &phi, &len);
        for (const TwoStepRange& g : ranges) {
            if (n >= cap) return -1;
            out[3 * n] = (int64_t)(ci * pc + g.e0);
            out[3 * n + 1] = (int64_t)(ci * pc + g.e1);
            out[3 * n + 2] = g.owner;
            ++n;
        }
    }
    return n;
}

MSX_EXPORT int msx_schedule_block(int p, int64_t count, int n, int64_t* start, int64_t* len)
{
    size_t s, l;
    allreduce_block(p, (size_t)count, allreduce_block_of_newrank(p, n), &s, &l);
    *start = (int64_t)s;
    *len = (int64_t)l;
    return MPI_SUCCESS;
}
