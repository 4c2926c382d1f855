// msx_comm.h — communicators, user ops and the collective engine interface.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <functional>
#include <vector>

#include "msx_types.h"

namespace msx {

class Transport;   // msx_transport.h

struct Comm {
    MPI_Comm handle = MPI_COMM_NULL;
    int rank = 0;
    int size = 1;
    MPI_Errhandler errhandler = MPI_ERRORS_ARE_FATAL;
    Transport* tp = nullptr;   // null when size == 1
    // process id (MPI_COMM_WORLD rank) of every member, by rank in this
    // communicator: the lrank_to_lpid map of the comm's group (mpid/group.cpp)
    std::vector<int> lpid;
    // Intercommunicator (MPI_Intercomm_create): rank / size / lpid describe
    // the local group; `local` is the local group as an intracommunicator of
    // its own (the reference's inter.local_comm), `uni` both groups in one
    // intracommunicator, the low group first -- the data plane between the
    // groups (point-to-point transfers over its windows).
    bool inter = false;
    bool is_low = false;              // this group is first in `uni`
    std::vector<int> remote_lpid;     // the remote group
    Comm* local = nullptr;
    Comm* uni = nullptr;
};

// MPI_COMM_WORLD, MPI_COMM_SELF or a derived communicator; nullptr otherwise.
Comm* lookup_comm(MPI_Comm c);
MPI_Comm comm_register(Comm* c);      // assigns c->handle
void comm_unregister(Comm* c);

// Groups (msx_group.cpp): ordered lists of process ids.  MpiaGroupValidateHandle:
// MPI_SUCCESS and *lpid = the members, or MPI_ERR_GROUP.
int group_members(MPI_Group g, std::vector<int>* lpid);
// A new group handle for the members (MPI_GROUP_EMPTY when empty).
int group_create(const std::vector<int>& lpid, MPI_Group* out);

// Resolved op (builtin kernel or user function), MPID_Op (include/op.h:82-134).
struct OpRef {
    int opidx = O_NULL;                 // builtin index, or O_NULL for user ops
    MPI_User_function* user_fn = nullptr;
    bool commutative = true;
};

// MSMPI_FORCE_ASYNC_WORKFLOW (mpid/env.cpp:1381-1384, read at MPI_Init with
// env_is_on: "1", or "on" / "yes" / "true" in any case, at most 4
// characters): blocking MPI_Reduce / MPI_Allreduce / MPI_Reduce_scatter[_block]
// run the NBC builders and wait (api/mpi_reduce.cpp:129,508,903,1317).
bool force_async();

// Process state (init/finalize, world bootstrap).
bool is_initialized();
bool is_finalized();
int world_init();          // MPI_Init body: device + (multi-rank) bootstrap
int world_finalize();
Comm* world();

// Reduction collectives over `comm` (arguments already validated).
// `kind` is the element class of `dt` (K_NONE for user ops on non-reducible types).
// nbc: follow the reference's NBC task list (MPI_Iallreduce / MPI_Ireduce,
// or the blocking call under MSMPI_FORCE_ASYNC_WORKFLOW, force_async()).
int coll_allreduce(Comm* c, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
                   const OpRef& op, bool nbc = false);
int coll_reduce(Comm* c, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
                const OpRef& op, int root, bool nbc = false);
int coll_reduce_scatter(Comm* c, const void* sendbuf, void* recvbuf, const int* recvcounts,
                        MPI_Datatype dt, const OpRef& op);
int coll_scan(Comm* c, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
              const OpRef& op, bool exclusive);
int coll_barrier(Comm* c);

// Local combine with any op (builtin -> GPU kernel; user fn -> host call).
int local_combine(const OpRef& op, MPI_Datatype dt, const void* in, void* inout, size_t count);

// Copy `bytes` between any two buffers (host or device), blocking.
int copy_any(void* dst, const void* src, size_t bytes);
// MPIR_Localcopy: count elements of dt (derived types through the pack kernels).
int local_copy(const void* src, void* dst, size_t count, MPI_Datatype dt);

// Non-blocking requests (stream/event backed).
struct Request;
int request_start_allreduce(Comm* c, const void* sendbuf, void* recvbuf, size_t count,
                            MPI_Datatype dt, const OpRef& op, MPI_Request* req);
// Start `body` as a request: on the engine worker when c->size > 1 (true
// overlap with the caller), inline otherwise.  A derived datatype named by
// `hold` keeps a reference until the request completes (MPI_Type_free of a
// type in use by a pending operation defers its destruction).
int request_start_generic(Comm* c, std::function<int()> body, MPI_Request* req,
                          MPI_Datatype hold = MPI_DATATYPE_NULL);
// A complete request of a request-based RMA call (its operation already
// flushed); MPI_Request_free releases these, and refuses collective requests.
int request_completed_rma(MPI_Request* req, int rc);
int request_free(MPI_Request* req);
int request_wait(MPI_Request* req, MPI_Status* st);
int request_test(MPI_Request* req, int* flag, MPI_Status* st);
// completion helpers of the multi-request calls (api/mpi_completion.cpp)
int request_validate(MPI_Request h);         // MPI_SUCCESS or MPI_ERR_REQUEST
bool request_done(MPI_Request h);            // non-destructive completion test
int request_error(MPI_Request h);            // error code of a completed request
void status_set_empty(MPI_Status* st);
void progress_pause(int iter);

}  // namespace msx
