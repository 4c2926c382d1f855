/*
 * mpi.h — MPI-2.2 C API subset for the MI355X-native MS-MPI reduction path.
 *
 * This header is written for this project.  It keeps the numeric ABI of
 * MS-MPI (handle values, error classes, typedef widths) so that code compiled
 * against MS-MPI's reduction API keeps its meaning when linked against
 * libmsmpi_mi355x.so.  Values are cited against the reference header
 * /root/reference/src/include/mpi.h (file:line).
 *
 * Scope: the local-reduction path (MPI_Op kernels) and the reduction
 * collectives that call it.  See DESIGN.md.
 */
#ifndef MSX_MPI_H_INCLUDED
#define MSX_MPI_H_INCLUDED

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* mpi.h:185 — __stdcall is a no-op on x64; keep the spelling for drop-in. */
#define MPIAPI
/* mpi.h:515 */
#define MPI_METHOD int MPIAPI

#define MPI_VERSION    2      /* mpi.h:4070-4071: MS-MPI reports 2.0 */
#define MPI_SUBVERSION 0

/* ---- error classes (mpi.h:192-250) -------------------------------------- */
#define MPI_SUCCESS          0
#define MPI_ERR_BUFFER       1
#define MPI_ERR_COUNT        2
#define MPI_ERR_TYPE         3
#define MPI_ERR_TAG          4
#define MPI_ERR_COMM         5
#define MPI_ERR_RANK         6
#define MPI_ERR_ROOT         7
#define MPI_ERR_GROUP        8
#define MPI_ERR_OP           9
#define MPI_ERR_TOPOLOGY    10
#define MPI_ERR_DIMS        11
#define MPI_ERR_ARG         12
#define MPI_ERR_UNKNOWN     13
#define MPI_ERR_TRUNCATE    14
#define MPI_ERR_OTHER       15
#define MPI_ERR_INTERN      16
#define MPI_ERR_IN_STATUS   17
#define MPI_ERR_PENDING     18
#define MPI_ERR_REQUEST     19
#define MPI_ERR_INFO        28
#define MPI_ERR_NO_MEM      34
#define MPI_ERR_NOT_SAME    35
#define MPI_ERR_WIN         45
#define MPI_ERR_BASE        46
#define MPI_ERR_LOCKTYPE    47
#define MPI_ERR_RMA_CONFLICT 49
#define MPI_ERR_RMA_SYNC    50
#define MPI_ERR_SIZE        51
#define MPI_ERR_DISP        52
#define MPI_ERR_ASSERT      53
/* classes of the MPI-2 subsystems outside the reduction path (I/O, dynamic
 * processes, attributes): values as the reference header, so code that names
 * them compiles unchanged */
#define MPI_ERR_ACCESS      20
#define MPI_ERR_AMODE       21
#define MPI_ERR_BAD_FILE    22
#define MPI_ERR_CONVERSION  23
#define MPI_ERR_DUP_DATAREP 24
#define MPI_ERR_FILE_EXISTS 25
#define MPI_ERR_FILE_IN_USE 26
#define MPI_ERR_FILE        27
#define MPI_ERR_INFO_KEY    29
#define MPI_ERR_INFO_VALUE  30
#define MPI_ERR_INFO_NOKEY  31
#define MPI_ERR_IO          32
#define MPI_ERR_NAME        33
#define MPI_ERR_NO_SPACE    36
#define MPI_ERR_NO_SUCH_FILE 37
#define MPI_ERR_PORT        38
#define MPI_ERR_QUOTA       39
#define MPI_ERR_READ_ONLY   40
#define MPI_ERR_SERVICE     41
#define MPI_ERR_SPAWN       42
#define MPI_ERR_UNSUPPORTED_DATAREP 43
#define MPI_ERR_UNSUPPORTED_OPERATION 44
#define MPI_ERR_KEYVAL      48
#define MPI_ERR_LASTCODE    0x3fffffff
#define MPICH_ERR_LAST_CLASS 53

#define MPI_MAX_ERROR_STRING 512
#define MPI_MAX_PROCESSOR_NAME 128

/* ---- basic integer types (mpi.h:258-270, Win64 / LLP64) ------------------ */
typedef int64_t MPI_Aint;
typedef int     MPI_Fint;
typedef int64_t MPI_Offset;
typedef int64_t MPI_Count;

/* ---- MPI_Datatype (mpi.h:281-368): 0x4c00SSII, SS = element bytes -------- */
typedef int MPI_Datatype;
#define MPI_DATATYPE_NULL           ((MPI_Datatype)0x0c000000)

#define MPI_CHAR                    ((MPI_Datatype)0x4c000101)
#define MPI_UNSIGNED_CHAR           ((MPI_Datatype)0x4c000102)
#define MPI_SHORT                   ((MPI_Datatype)0x4c000203)
#define MPI_UNSIGNED_SHORT          ((MPI_Datatype)0x4c000204)
#define MPI_INT                     ((MPI_Datatype)0x4c000405)
#define MPI_UNSIGNED                ((MPI_Datatype)0x4c000406)
#define MPI_LONG                    ((MPI_Datatype)0x4c000407)   /* LLP64: 4 bytes */
#define MPI_UNSIGNED_LONG           ((MPI_Datatype)0x4c000408)   /* LLP64: 4 bytes */
#define MPI_LONG_LONG_INT           ((MPI_Datatype)0x4c000809)
#define MPI_LONG_LONG               MPI_LONG_LONG_INT
#define MPI_FLOAT                   ((MPI_Datatype)0x4c00040a)
#define MPI_DOUBLE                  ((MPI_Datatype)0x4c00080b)
#define MPI_LONG_DOUBLE             ((MPI_Datatype)0x4c00080c)   /* MSVC: 8 bytes */
#define MPI_BYTE                    ((MPI_Datatype)0x4c00010d)
#define MPI_WCHAR                   ((MPI_Datatype)0x4c00020e)
#define MPI_PACKED                  ((MPI_Datatype)0x4c00010f)
#define MPI_LB                      ((MPI_Datatype)0x4c000010)
#define MPI_UB                      ((MPI_Datatype)0x4c000011)
#define MPI_C_COMPLEX               ((MPI_Datatype)0x4c000812)
#define MPI_C_FLOAT_COMPLEX         ((MPI_Datatype)0x4c000813)
#define MPI_C_DOUBLE_COMPLEX        ((MPI_Datatype)0x4c001014)
#define MPI_C_LONG_DOUBLE_COMPLEX   ((MPI_Datatype)0x4c001015)
#define MPI_2INT                    ((MPI_Datatype)0x4c000816)
#define MPI_C_BOOL                  ((MPI_Datatype)0x4c000117)
#define MPI_SIGNED_CHAR             ((MPI_Datatype)0x4c000118)
#define MPI_UNSIGNED_LONG_LONG      ((MPI_Datatype)0x4c000819)
#define MPI_CHARACTER               ((MPI_Datatype)0x4c00011a)
#define MPI_INTEGER                 ((MPI_Datatype)0x4c00041b)
#define MPI_REAL                    ((MPI_Datatype)0x4c00041c)
#define MPI_LOGICAL                 ((MPI_Datatype)0x4c00041d)
#define MPI_COMPLEX                 ((MPI_Datatype)0x4c00081e)
#define MPI_DOUBLE_PRECISION        ((MPI_Datatype)0x4c00081f)
#define MPI_2INTEGER                ((MPI_Datatype)0x4c000820)
#define MPI_2REAL                   ((MPI_Datatype)0x4c000821)
#define MPI_DOUBLE_COMPLEX          ((MPI_Datatype)0x4c001022)
#define MPI_2DOUBLE_PRECISION       ((MPI_Datatype)0x4c001023)
#define MPI_2COMPLEX                ((MPI_Datatype)0x4c001024)
#define MPI_2DOUBLE_COMPLEX         ((MPI_Datatype)0x4c002025)
#define MPI_REAL2                   MPI_DATATYPE_NULL
#define MPI_REAL4                   ((MPI_Datatype)0x4c000427)
#define MPI_COMPLEX8                ((MPI_Datatype)0x4c000828)
#define MPI_REAL8                   ((MPI_Datatype)0x4c000829)
#define MPI_COMPLEX16               ((MPI_Datatype)0x4c00102a)
#define MPI_REAL16                  MPI_DATATYPE_NULL
#define MPI_COMPLEX32               MPI_DATATYPE_NULL
#define MPI_INTEGER1                ((MPI_Datatype)0x4c00012d)
#define MPI_COMPLEX4                MPI_DATATYPE_NULL
#define MPI_INTEGER2                ((MPI_Datatype)0x4c00022f)
#define MPI_INTEGER4                ((MPI_Datatype)0x4c000430)
#define MPI_INTEGER8                ((MPI_Datatype)0x4c000831)
#define MPI_INTEGER16               MPI_DATATYPE_NULL
#define MPI_INT8_T                  ((MPI_Datatype)0x4c000133)
#define MPI_INT16_T                 ((MPI_Datatype)0x4c000234)
#define MPI_INT32_T                 ((MPI_Datatype)0x4c000435)
#define MPI_INT64_T                 ((MPI_Datatype)0x4c000836)
#define MPI_UINT8_T                 ((MPI_Datatype)0x4c000137)
#define MPI_UINT16_T                ((MPI_Datatype)0x4c000238)
#define MPI_UINT32_T                ((MPI_Datatype)0x4c000439)
#define MPI_UINT64_T                ((MPI_Datatype)0x4c00083a)
#define MPI_AINT                    ((MPI_Datatype)0x4c00083b)   /* _WIN64 value */
#define MPI_OFFSET                  ((MPI_Datatype)0x4c00083c)
#define MPI_COUNT                   ((MPI_Datatype)0x4c00083d)
/* value/location pair types (mpi.h:364-368) */
#define MPI_FLOAT_INT               ((MPI_Datatype)0x8c000000)
#define MPI_DOUBLE_INT              ((MPI_Datatype)0x8c000001)
#define MPI_LONG_INT                ((MPI_Datatype)0x8c000002)
#define MPI_SHORT_INT               ((MPI_Datatype)0x8c000003)
#define MPI_LONG_DOUBLE_INT         ((MPI_Datatype)0x8c000004)

/* ---- MPI_Comm (mpi.h:375-379) ------------------------------------------- */
typedef int MPI_Comm;
#define MPI_COMM_NULL  ((MPI_Comm)0x04000000)
#define MPI_COMM_WORLD ((MPI_Comm)0x44000000)
#define MPI_COMM_SELF  ((MPI_Comm)0x44000001)

/* ---- MPI_Group (mpi.h:450-452, 2957-2960) -------------------------------- */
typedef int MPI_Group;
#define MPI_GROUP_NULL  ((MPI_Group)0x08000000)
#define MPI_GROUP_EMPTY ((MPI_Group)0x48000000)
#define MPI_IDENT       0
#define MPI_CONGRUENT   1
#define MPI_SIMILAR     2
#define MPI_UNEQUAL     3

/* ---- MPI_Op (mpi.h:410-426) --------------------------------------------- */
typedef int MPI_Op;
#define MPI_OP_NULL ((MPI_Op)0x18000000)
#define MPI_MAX     ((MPI_Op)0x58000001)
#define MPI_MIN     ((MPI_Op)0x58000002)
#define MPI_SUM     ((MPI_Op)0x58000003)
#define MPI_PROD    ((MPI_Op)0x58000004)
#define MPI_LAND    ((MPI_Op)0x58000005)
#define MPI_BAND    ((MPI_Op)0x58000006)
#define MPI_LOR     ((MPI_Op)0x58000007)
#define MPI_BOR     ((MPI_Op)0x58000008)
#define MPI_LXOR    ((MPI_Op)0x58000009)
#define MPI_BXOR    ((MPI_Op)0x5800000a)
#define MPI_MINLOC  ((MPI_Op)0x5800000b)
#define MPI_MAXLOC  ((MPI_Op)0x5800000c)
#define MPI_REPLACE ((MPI_Op)0x5800000d)
#define MPI_NO_OP   ((MPI_Op)0x5800000e)

/* ---- MPI_Request / MPI_Errhandler / MPI_Status (mpi.h:441-489) ----------- */
typedef int MPI_Request;
#define MPI_REQUEST_NULL ((MPI_Request)0x2c000000)

typedef int MPI_Errhandler;
#define MPI_ERRHANDLER_NULL  ((MPI_Errhandler)0x14000000)
#define MPI_ERRORS_ARE_FATAL ((MPI_Errhandler)0x54000000)
#define MPI_ERRORS_RETURN    ((MPI_Errhandler)0x54000001)

typedef struct MPI_Status
{
    int internal[2];
    int MPI_SOURCE;
    int MPI_TAG;
    int MPI_ERROR;
} MPI_Status;

#define MPI_STATUS_IGNORE   ((MPI_Status*)(MPI_Aint)1)
#define MPI_STATUSES_IGNORE ((MPI_Status*)(MPI_Aint)1)

#define MPI_UNDEFINED   (-32766)
#define MPI_BOTTOM      ((void*)0)
/* mpi.h:1956 */
#define MPI_IN_PLACE    ((void*)(MPI_Aint)-1)

/* thread levels */
#define MPI_THREAD_SINGLE     0
#define MPI_THREAD_FUNNELED   1
#define MPI_THREAD_SERIALIZED 2
#define MPI_THREAD_MULTIPLE   3

/* ---- user reduction function (mpi.h:2258-2265) --------------------------- */
typedef void (MPIAPI MPI_User_function)(void* invec, void* inoutvec, int* len,
                                         MPI_Datatype* datatype);

/* ---- environment ---------------------------------------------------------- */
MPI_METHOD MPI_Init(int* argc, char*** argv);
MPI_METHOD MPI_Init_thread(int* argc, char*** argv, int required, int* provided);
MPI_METHOD MPI_Finalize(void);
MPI_METHOD MPI_Initialized(int* flag);
MPI_METHOD MPI_Finalized(int* flag);
MPI_METHOD MPI_Abort(MPI_Comm comm, int errorcode);
double MPIAPI MPI_Wtime(void);
double MPIAPI MPI_Wtick(void);
MPI_METHOD MPI_Query_thread(int* provided);
MPI_METHOD MPI_Is_thread_main(int* flag);
MPI_METHOD MPI_Get_version(int* version, int* subversion);
MPI_METHOD MPI_Get_processor_name(char* name, int* resultlen);
MPI_METHOD MPI_Comm_rank(MPI_Comm comm, int* rank);
MPI_METHOD MPI_Comm_size(MPI_Comm comm, int* size);
MPI_METHOD MPI_Barrier(MPI_Comm comm);
MPI_METHOD MPI_Comm_split(MPI_Comm comm, int color, int key, MPI_Comm* newcomm);
MPI_METHOD MPI_Comm_dup(MPI_Comm comm, MPI_Comm* newcomm);
MPI_METHOD MPI_Comm_free(MPI_Comm* comm);
MPI_METHOD MPI_Comm_set_errhandler(MPI_Comm comm, MPI_Errhandler errhandler);
MPI_METHOD MPI_Comm_get_errhandler(MPI_Comm comm, MPI_Errhandler* errhandler);
MPI_METHOD MPI_Error_class(int errorcode, int* errorclass);
MPI_METHOD MPI_Error_string(int errorcode, char* string, int* resultlen);
MPI_METHOD MPI_Type_size(MPI_Datatype datatype, int* size);

/* ---- reduction operations (mpi.h:2266-2300) ------------------------------ */
MPI_METHOD MPI_Op_commutative(MPI_Op op, int* commute);
MPI_METHOD MPI_Op_create(MPI_User_function* user_fn, int commute, MPI_Op* op);
MPI_METHOD MPI_Op_free(MPI_Op* op);

/* ---- reduction collectives (mpi.h:2305-2560) ----------------------------- */
MPI_METHOD MPI_Reduce(const void* sendbuf, void* recvbuf, int count,
                      MPI_Datatype datatype, MPI_Op op, int root, MPI_Comm comm);
MPI_METHOD MPI_Allreduce(const void* sendbuf, void* recvbuf, int count,
                         MPI_Datatype datatype, MPI_Op op, MPI_Comm comm);
MPI_METHOD MPI_Reduce_local(const void* inbuf, void* inoutbuf, int count,
                            MPI_Datatype datatype, MPI_Op op);
MPI_METHOD MPI_Reduce_scatter_block(const void* sendbuf, void* recvbuf, int recvcount,
                                    MPI_Datatype datatype, MPI_Op op, MPI_Comm comm);
MPI_METHOD MPI_Reduce_scatter(const void* sendbuf, void* recvbuf, const int recvcounts[],
                              MPI_Datatype datatype, MPI_Op op, MPI_Comm comm);
MPI_METHOD MPI_Scan(const void* sendbuf, void* recvbuf, int count,
                    MPI_Datatype datatype, MPI_Op op, MPI_Comm comm);
MPI_METHOD MPI_Exscan(const void* sendbuf, void* recvbuf, int count,
                      MPI_Datatype datatype, MPI_Op op, MPI_Comm comm);
MPI_METHOD MPI_Iallreduce(const void* sendbuf, void* recvbuf, int count,
                          MPI_Datatype datatype, MPI_Op op, MPI_Comm comm,
                          MPI_Request* request);
MPI_METHOD MPI_Iscan(const void* sendbuf, void* recvbuf, int count,
                     MPI_Datatype datatype, MPI_Op op, MPI_Comm comm,
                     MPI_Request* request);
MPI_METHOD MPI_Iexscan(const void* sendbuf, void* recvbuf, int count,
                       MPI_Datatype datatype, MPI_Op op, MPI_Comm comm,
                       MPI_Request* request);
MPI_METHOD MPI_Ireduce(const void* sendbuf, void* recvbuf, int count,
                       MPI_Datatype datatype, MPI_Op op, int root, MPI_Comm comm,
                       MPI_Request* request);
MPI_METHOD MPI_Ireduce_scatter_block(const void* sendbuf, void* recvbuf, int recvcount,
                                     MPI_Datatype datatype, MPI_Op op, MPI_Comm comm,
                                     MPI_Request* request);
MPI_METHOD MPI_Ireduce_scatter(const void* sendbuf, void* recvbuf, const int recvcounts[],
                               MPI_Datatype datatype, MPI_Op op, MPI_Comm comm,
                               MPI_Request* request);

/* ---- request completion --------------------------------------------------- */
MPI_METHOD MPI_Wait(MPI_Request* request, MPI_Status* status);
MPI_METHOD MPI_Test(MPI_Request* request, int* flag, MPI_Status* status);
MPI_METHOD MPI_Waitall(int count, MPI_Request array_of_requests[],
                       MPI_Status array_of_statuses[]);
/* api/mpi_completion.cpp:226,453,663,1176,1385; api/mpi_request.cpp:52,170 */
MPI_METHOD MPI_Testall(int count, MPI_Request array_of_requests[], int* flag,
                       MPI_Status array_of_statuses[]);
MPI_METHOD MPI_Testany(int count, MPI_Request array_of_requests[], int* index, int* flag,
                       MPI_Status* status);
MPI_METHOD MPI_Testsome(int incount, MPI_Request array_of_requests[], int* outcount,
                        int array_of_indices[], MPI_Status array_of_statuses[]);
MPI_METHOD MPI_Waitany(int count, MPI_Request array_of_requests[], int* index,
                       MPI_Status* status);
MPI_METHOD MPI_Waitsome(int incount, MPI_Request array_of_requests[], int* outcount,
                        int array_of_indices[], MPI_Status array_of_statuses[]);
MPI_METHOD MPI_Request_free(MPI_Request* request);
MPI_METHOD MPI_Request_get_status(MPI_Request request, int* flag, MPI_Status* status);

/* ---- one-sided communication, fence synchronisation (mpi.h:394-395,
 *      434, 500, 5246-5250; api/mpi_win.cpp, api/mpi_rma.cpp) ------------- */
typedef int MPI_Win;
#define MPI_WIN_NULL        ((MPI_Win)0x20000000)
typedef int MPI_Info;
#define MPI_INFO_NULL       ((MPI_Info)0x1c000000)
#define MPI_PROC_NULL       (-1)
#define MPI_ANY_SOURCE      (-2)
#define MPI_ROOT            (-3)
#define MPI_ANY_TAG         (-1)
#define MPI_MODE_NOCHECK    1024
#define MPI_MODE_NOSTORE    2048
#define MPI_MODE_NOPUT      4096
#define MPI_MODE_NOPRECEDE  8192
#define MPI_MODE_NOSUCCEED 16384
/* passive-target lock types (mpi.h:5324-5325) */
#define MPI_LOCK_EXCLUSIVE  234
#define MPI_LOCK_SHARED     235

MPI_METHOD MPI_Win_create(void* base, MPI_Aint size, int disp_unit, MPI_Info info,
                          MPI_Comm comm, MPI_Win* win);
MPI_METHOD MPI_Win_free(MPI_Win* win);
MPI_METHOD MPI_Win_allocate(MPI_Aint size, int disp_unit, MPI_Info info, MPI_Comm comm, void* baseptr,
                            MPI_Win* win);
/* memory for RMA and staging (api/mpi_env.cpp:841-945): pinned host memory,
   which the GPU reads and writes in place over PCIe */
MPI_METHOD MPI_Alloc_mem(MPI_Aint size, MPI_Info info, void* baseptr);
MPI_METHOD MPI_Free_mem(void* base);
MPI_METHOD MPI_Win_fence(int assert, MPI_Win win);
/* passive-target synchronisation (api/mpi_win.cpp:1153-1990) */
MPI_METHOD MPI_Win_lock(int lock_type, int rank, int assert, MPI_Win win);
MPI_METHOD MPI_Win_unlock(int rank, MPI_Win win);
MPI_METHOD MPI_Win_lock_all(int assert, MPI_Win win);
MPI_METHOD MPI_Win_unlock_all(MPI_Win win);
MPI_METHOD MPI_Win_flush(int rank, MPI_Win win);
MPI_METHOD MPI_Win_flush_all(MPI_Win win);
MPI_METHOD MPI_Win_flush_local(int rank, MPI_Win win);
MPI_METHOD MPI_Win_flush_local_all(MPI_Win win);
MPI_METHOD MPI_Win_sync(MPI_Win win);
/* post-start-complete-wait synchronisation (api/mpi_win.cpp:28,979,1331,1487,1566,1769) */
MPI_METHOD MPI_Win_post(MPI_Group group, int assert, MPI_Win win);
MPI_METHOD MPI_Win_start(MPI_Group group, int assert, MPI_Win win);
MPI_METHOD MPI_Win_complete(MPI_Win win);
MPI_METHOD MPI_Win_wait(MPI_Win win);
MPI_METHOD MPI_Win_test(MPI_Win win, int* flag);
MPI_METHOD MPI_Win_get_group(MPI_Win win, MPI_Group* group);
MPI_METHOD MPI_Win_set_errhandler(MPI_Win win, MPI_Errhandler errhandler);
MPI_METHOD MPI_Win_get_errhandler(MPI_Win win, MPI_Errhandler* errhandler);
MPI_METHOD MPI_Put(const void* origin_addr, int origin_count, MPI_Datatype origin_datatype,
                   int target_rank, MPI_Aint target_disp, int target_count,
                   MPI_Datatype target_datatype, MPI_Win win);
MPI_METHOD MPI_Get(void* origin_addr, int origin_count, MPI_Datatype origin_datatype,
                   int target_rank, MPI_Aint target_disp, int target_count,
                   MPI_Datatype target_datatype, MPI_Win win);
MPI_METHOD MPI_Accumulate(const void* origin_addr, int origin_count, MPI_Datatype origin_datatype,
                          int target_rank, MPI_Aint target_disp, int target_count,
                          MPI_Datatype target_datatype, MPI_Op op, MPI_Win win);
MPI_METHOD MPI_Get_accumulate(const void* origin_addr, int origin_count,
                              MPI_Datatype origin_datatype, void* result_addr, int result_count,
                              MPI_Datatype result_datatype, int target_rank, MPI_Aint target_disp,
                              int target_count, MPI_Datatype target_datatype, MPI_Op op,
                              MPI_Win win);
MPI_METHOD MPI_Fetch_and_op(const void* origin_addr, void* result_addr, MPI_Datatype datatype,
                            int target_rank, MPI_Aint target_disp, MPI_Op op, MPI_Win win);
MPI_METHOD MPI_Compare_and_swap(const void* origin_addr, const void* compare_addr,
                                void* result_addr, MPI_Datatype datatype, int target_rank,
                                MPI_Aint target_disp, MPI_Win win);
/* request-based RMA (api/mpi_rma.cpp:187,486,813,1215): passive-target
 * epochs; the operation is flushed to its target and the request returned
 * complete */
MPI_METHOD MPI_Rput(const void* origin_addr, int origin_count, MPI_Datatype origin_datatype,
                    int target_rank, MPI_Aint target_disp, int target_count,
                    MPI_Datatype target_datatype, MPI_Win win, MPI_Request* request);
MPI_METHOD MPI_Rget(void* origin_addr, int origin_count, MPI_Datatype origin_datatype,
                    int target_rank, MPI_Aint target_disp, int target_count,
                    MPI_Datatype target_datatype, MPI_Win win, MPI_Request* request);
MPI_METHOD MPI_Raccumulate(const void* origin_addr, int origin_count, MPI_Datatype origin_datatype,
                           int target_rank, MPI_Aint target_disp, int target_count,
                           MPI_Datatype target_datatype, MPI_Op op, MPI_Win win,
                           MPI_Request* request);
MPI_METHOD MPI_Rget_accumulate(const void* origin_addr, int origin_count,
                               MPI_Datatype origin_datatype, void* result_addr, int result_count,
                               MPI_Datatype result_datatype, int target_rank, MPI_Aint target_disp,
                               int target_count, MPI_Datatype target_datatype, MPI_Op op,
                               MPI_Win win, MPI_Request* request);

/* ---- groups (api/mpi_group.cpp, api/mpi_comm.cpp:677) -------------------- */
MPI_METHOD MPI_Comm_group(MPI_Comm comm, MPI_Group* group);
MPI_METHOD MPI_Comm_create(MPI_Comm comm, MPI_Group group, MPI_Comm* newcomm);
MPI_METHOD MPI_Comm_compare(MPI_Comm comm1, MPI_Comm comm2, int* result);
MPI_METHOD MPI_Comm_test_inter(MPI_Comm comm, int* flag);
MPI_METHOD MPI_Comm_remote_size(MPI_Comm comm, int* size);
MPI_METHOD MPI_Comm_remote_group(MPI_Comm comm, MPI_Group* group);
MPI_METHOD MPI_Intercomm_create(MPI_Comm local_comm, int local_leader, MPI_Comm peer_comm, int remote_leader,
                                int tag, MPI_Comm* newintercomm);
MPI_METHOD MPI_Intercomm_merge(MPI_Comm intercomm, int high, MPI_Comm* newintracomm);
MPI_METHOD MPI_Group_size(MPI_Group group, int* size);
MPI_METHOD MPI_Group_rank(MPI_Group group, int* rank);
MPI_METHOD MPI_Group_free(MPI_Group* group);
MPI_METHOD MPI_Group_incl(MPI_Group group, int n, const int ranks[], MPI_Group* newgroup);
MPI_METHOD MPI_Group_excl(MPI_Group group, int n, const int ranks[], MPI_Group* newgroup);
MPI_METHOD MPI_Group_range_incl(MPI_Group group, int n, int ranges[][3], MPI_Group* newgroup);
MPI_METHOD MPI_Group_range_excl(MPI_Group group, int n, int ranges[][3], MPI_Group* newgroup);
MPI_METHOD MPI_Group_union(MPI_Group group1, MPI_Group group2, MPI_Group* newgroup);
MPI_METHOD MPI_Group_intersection(MPI_Group group1, MPI_Group group2, MPI_Group* newgroup);
MPI_METHOD MPI_Group_difference(MPI_Group group1, MPI_Group group2, MPI_Group* newgroup);
MPI_METHOD MPI_Group_translate_ranks(MPI_Group group1, int n, const int ranks1[], MPI_Group group2,
                                     int ranks2[]);
MPI_METHOD MPI_Group_compare(MPI_Group group1, MPI_Group group2, int* result);

/* ---- derived datatypes (mpi.h:1340-1822) and pack/unpack (mpi.h:1823-1887)
 * Constructors, queries and MPI_Pack/MPI_Unpack; the bytes are moved by the
 * gfx950 pack kernels.  Derived types are accepted by MPI_Pack/MPI_Unpack and
 * the one-sided calls; the reduction collectives take predefined types. */
#define MPI_ORDER_C         56
#define MPI_ORDER_FORTRAN   57

#define MPI_DISTRIBUTE_BLOCK        121     /* mpi.h:1513-1516 */
#define MPI_DISTRIBUTE_CYCLIC       122
#define MPI_DISTRIBUTE_NONE         123
#define MPI_DISTRIBUTE_DFLT_DARG    (-49767)

enum {                                  /* mpi.h:1758-1778 */
    MPI_COMBINER_NAMED            = 1,
    MPI_COMBINER_DUP              = 2,
    MPI_COMBINER_CONTIGUOUS       = 3,
    MPI_COMBINER_VECTOR           = 4,
    MPI_COMBINER_HVECTOR_INTEGER  = 5,
    MPI_COMBINER_HVECTOR          = 6,
    MPI_COMBINER_INDEXED          = 7,
    MPI_COMBINER_HINDEXED_INTEGER = 8,
    MPI_COMBINER_HINDEXED         = 9,
    MPI_COMBINER_INDEXED_BLOCK    = 10,
    MPI_COMBINER_STRUCT_INTEGER   = 11,
    MPI_COMBINER_STRUCT           = 12,
    MPI_COMBINER_SUBARRAY         = 13,
    MPI_COMBINER_DARRAY           = 14,
    MPI_COMBINER_F90_REAL         = 15,
    MPI_COMBINER_F90_COMPLEX      = 16,
    MPI_COMBINER_F90_INTEGER      = 17,
    MPI_COMBINER_RESIZED          = 18,
    MPI_COMBINER_HINDEXED_BLOCK   = 19
};

MPI_METHOD MPI_Type_contiguous(int count, MPI_Datatype oldtype, MPI_Datatype* newtype);
MPI_METHOD MPI_Type_vector(int count, int blocklength, int stride, MPI_Datatype oldtype,
                           MPI_Datatype* newtype);
MPI_METHOD MPI_Type_create_hvector(int count, int blocklength, MPI_Aint stride,
                                   MPI_Datatype oldtype, MPI_Datatype* newtype);
MPI_METHOD MPI_Type_hvector(int count, int blocklength, MPI_Aint stride, MPI_Datatype oldtype,
                            MPI_Datatype* newtype);
MPI_METHOD MPI_Type_indexed(int count, const int array_of_blocklengths[],
                            const int array_of_displacements[], MPI_Datatype oldtype,
                            MPI_Datatype* newtype);
MPI_METHOD MPI_Type_create_hindexed(int count, const int array_of_blocklengths[],
                                    const MPI_Aint array_of_displacements[],
                                    MPI_Datatype oldtype, MPI_Datatype* newtype);
MPI_METHOD MPI_Type_hindexed(int count, const int array_of_blocklengths[],
                             const MPI_Aint array_of_displacements[], MPI_Datatype oldtype,
                             MPI_Datatype* newtype);
MPI_METHOD MPI_Type_create_indexed_block(int count, int blocklength,
                                         const int array_of_displacements[],
                                         MPI_Datatype oldtype, MPI_Datatype* newtype);
MPI_METHOD MPI_Type_create_hindexed_block(int count, int blocklength,
                                          const MPI_Aint array_of_displacements[],
                                          MPI_Datatype oldtype, MPI_Datatype* newtype);
MPI_METHOD MPI_Type_create_struct(int count, const int array_of_blocklengths[],
                                  const MPI_Aint array_of_displacements[],
                                  const MPI_Datatype array_of_types[], MPI_Datatype* newtype);
MPI_METHOD MPI_Type_struct(int count, const int array_of_blocklengths[],
                           const MPI_Aint array_of_displacements[],
                           const MPI_Datatype array_of_types[], MPI_Datatype* newtype);
MPI_METHOD MPI_Type_create_subarray(int ndims, const int array_of_sizes[],
                                    const int array_of_subsizes[], const int array_of_starts[],
                                    int order, MPI_Datatype oldtype, MPI_Datatype* newtype);
MPI_METHOD MPI_Type_create_darray(int size, int rank, int ndims, const int array_of_gsizes[],
                                  const int array_of_distribs[], const int array_of_dargs[],
                                  const int array_of_psizes[], int order, MPI_Datatype oldtype,
                                  MPI_Datatype* newtype);
MPI_METHOD MPI_Type_create_resized(MPI_Datatype oldtype, MPI_Aint lb, MPI_Aint extent,
                                   MPI_Datatype* newtype);
MPI_METHOD MPI_Type_dup(MPI_Datatype oldtype, MPI_Datatype* newtype);
MPI_METHOD MPI_Type_commit(MPI_Datatype* datatype);
MPI_METHOD MPI_Type_free(MPI_Datatype* datatype);
MPI_METHOD MPI_Type_size_x(MPI_Datatype datatype, MPI_Count* size);
MPI_METHOD MPI_Type_get_extent(MPI_Datatype datatype, MPI_Aint* lb, MPI_Aint* extent);
MPI_METHOD MPI_Type_get_extent_x(MPI_Datatype datatype, MPI_Count* lb, MPI_Count* extent);
MPI_METHOD MPI_Type_get_true_extent(MPI_Datatype datatype, MPI_Aint* true_lb,
                                    MPI_Aint* true_extent);
MPI_METHOD MPI_Type_get_true_extent_x(MPI_Datatype datatype, MPI_Count* true_lb,
                                      MPI_Count* true_extent);
MPI_METHOD MPI_Type_extent(MPI_Datatype datatype, MPI_Aint* extent);
MPI_METHOD MPI_Type_lb(MPI_Datatype datatype, MPI_Aint* displacement);
MPI_METHOD MPI_Type_ub(MPI_Datatype datatype, MPI_Aint* displacement);
MPI_METHOD MPI_Type_get_envelope(MPI_Datatype datatype, int* num_integers, int* num_addresses,
                                 int* num_datatypes, int* combiner);
MPI_METHOD MPI_Type_get_contents(MPI_Datatype datatype, int max_integers, int max_addresses,
                                 int max_datatypes, int array_of_integers[],
                                 MPI_Aint array_of_addresses[],
                                 MPI_Datatype array_of_datatypes[]);
MPI_METHOD MPI_Get_address(const void* location, MPI_Aint* address);
MPI_METHOD MPI_Address(void* location, MPI_Aint* address);
MPI_METHOD MPI_Pack(const void* inbuf, int incount, MPI_Datatype datatype, void* outbuf,
                    int outsize, int* position, MPI_Comm comm);
MPI_METHOD MPI_Unpack(const void* inbuf, int insize, int* position, void* outbuf, int outcount,
                      MPI_Datatype datatype, MPI_Comm comm);
MPI_METHOD MPI_Pack_size(int incount, MPI_Datatype datatype, MPI_Comm comm, int* size);

/* ---- Fortran handle conversion (mpi.h:6816-6876): handles are already ints - */
#define MPI_Comm_c2f(comm)         (MPI_Fint)(comm)
#define MPI_Comm_f2c(comm)         (MPI_Comm)(comm)
#define MPI_Type_c2f(datatype)     (MPI_Fint)(datatype)
#define MPI_Type_f2c(datatype)     (MPI_Datatype)(datatype)
#define MPI_Op_c2f(op)             (MPI_Fint)(op)
#define MPI_Op_f2c(op)             (MPI_Op)(op)
#define MPI_Request_c2f(request)   (MPI_Fint)(request)
#define MPI_Request_f2c(request)   (MPI_Request)(request)
#define MPI_Win_c2f(win)           (MPI_Fint)(win)
#define MPI_Win_f2c(win)           (MPI_Win)(win)
#define MPI_Group_c2f(group)       (MPI_Fint)(group)
#define MPI_Group_f2c(group)       (MPI_Group)(group)
#define MPI_Info_c2f(info)         (MPI_Fint)(info)
#define MPI_Info_f2c(info)         (MPI_Info)(info)
#define MPI_Errhandler_c2f(errhandler) (MPI_Fint)(errhandler)
#define MPI_Errhandler_f2c(errhandler) (MPI_Errhandler)(errhandler)
#define PMPI_Comm_c2f(comm)        (MPI_Fint)(comm)
#define PMPI_Comm_f2c(comm)        (MPI_Comm)(comm)
#define PMPI_Type_c2f(datatype)    (MPI_Fint)(datatype)
#define PMPI_Type_f2c(datatype)    (MPI_Datatype)(datatype)
#define PMPI_Op_c2f(op)            (MPI_Fint)(op)
#define PMPI_Op_f2c(op)            (MPI_Op)(op)
#define PMPI_Request_c2f(request)  (MPI_Fint)(request)
#define PMPI_Request_f2c(request)  (MPI_Request)(request)
#define PMPI_Win_c2f(win)          (MPI_Fint)(win)
#define PMPI_Win_f2c(win)          (MPI_Win)(win)
#define PMPI_Group_c2f(group)      (MPI_Fint)(group)
#define PMPI_Group_f2c(group)      (MPI_Group)(group)
/* The Fortran bindings (mpif.h, include/mpif.h) are exported by the library
   as mpi_<name>_ with the MPI_<NAME>, mpi_<name>, mpi_<name>__ and PMPI_ aliases
   (microsoft-mpi_amd/csrc/msx_fortran.cpp). */

/* ---- profiling interface aliases (msmpi.def:101-102,422-423,478-483,...) -- */
MPI_METHOD PMPI_Reduce_local(const void* inbuf, void* inoutbuf, int count,
                             MPI_Datatype datatype, MPI_Op op);
MPI_METHOD PMPI_Reduce(const void* sendbuf, void* recvbuf, int count,
                       MPI_Datatype datatype, MPI_Op op, int root, MPI_Comm comm);
MPI_METHOD PMPI_Allreduce(const void* sendbuf, void* recvbuf, int count,
                          MPI_Datatype datatype, MPI_Op op, MPI_Comm comm);
MPI_METHOD PMPI_Reduce_scatter_block(const void* sendbuf, void* recvbuf, int recvcount,
                                     MPI_Datatype datatype, MPI_Op op, MPI_Comm comm);
MPI_METHOD PMPI_Reduce_scatter(const void* sendbuf, void* recvbuf, const int recvcounts[],
                               MPI_Datatype datatype, MPI_Op op, MPI_Comm comm);
MPI_METHOD PMPI_Iallreduce(const void* sendbuf, void* recvbuf, int count,
                           MPI_Datatype datatype, MPI_Op op, MPI_Comm comm,
                           MPI_Request* request);
MPI_METHOD PMPI_Iscan(const void* sendbuf, void* recvbuf, int count,
                      MPI_Datatype datatype, MPI_Op op, MPI_Comm comm,
                      MPI_Request* request);
MPI_METHOD PMPI_Iexscan(const void* sendbuf, void* recvbuf, int count,
                        MPI_Datatype datatype, MPI_Op op, MPI_Comm comm,
                        MPI_Request* request);
MPI_METHOD PMPI_Scan(const void* sendbuf, void* recvbuf, int count,
                     MPI_Datatype datatype, MPI_Op op, MPI_Comm comm);
MPI_METHOD PMPI_Exscan(const void* sendbuf, void* recvbuf, int count,
                       MPI_Datatype datatype, MPI_Op op, MPI_Comm comm);
MPI_METHOD PMPI_Ireduce(const void* sendbuf, void* recvbuf, int count,
                        MPI_Datatype datatype, MPI_Op op, int root, MPI_Comm comm,
                        MPI_Request* request);
MPI_METHOD PMPI_Ireduce_scatter_block(const void* sendbuf, void* recvbuf, int recvcount,
                                      MPI_Datatype datatype, MPI_Op op, MPI_Comm comm,
                                      MPI_Request* request);
MPI_METHOD PMPI_Ireduce_scatter(const void* sendbuf, void* recvbuf, const int recvcounts[],
                                MPI_Datatype datatype, MPI_Op op, MPI_Comm comm,
                                MPI_Request* request);
MPI_METHOD PMPI_Accumulate(const void* origin_addr, int origin_count,
                           MPI_Datatype origin_datatype, int target_rank, MPI_Aint target_disp,
                           int target_count, MPI_Datatype target_datatype, MPI_Op op,
                           MPI_Win win);
MPI_METHOD PMPI_Get_accumulate(const void* origin_addr, int origin_count,
                               MPI_Datatype origin_datatype, void* result_addr, int result_count,
                               MPI_Datatype result_datatype, int target_rank,
                               MPI_Aint target_disp, int target_count,
                               MPI_Datatype target_datatype, MPI_Op op, MPI_Win win);
MPI_METHOD PMPI_Fetch_and_op(const void* origin_addr, void* result_addr, MPI_Datatype datatype,
                             int target_rank, MPI_Aint target_disp, MPI_Op op, MPI_Win win);
MPI_METHOD PMPI_Rput(const void* origin_addr, int origin_count, MPI_Datatype origin_datatype,
                     int target_rank, MPI_Aint target_disp, int target_count,
                     MPI_Datatype target_datatype, MPI_Win win, MPI_Request* request);
MPI_METHOD PMPI_Rget(void* origin_addr, int origin_count, MPI_Datatype origin_datatype,
                     int target_rank, MPI_Aint target_disp, int target_count,
                     MPI_Datatype target_datatype, MPI_Win win, MPI_Request* request);
MPI_METHOD PMPI_Raccumulate(const void* origin_addr, int origin_count, MPI_Datatype origin_datatype,
                            int target_rank, MPI_Aint target_disp, int target_count,
                            MPI_Datatype target_datatype, MPI_Op op, MPI_Win win,
                            MPI_Request* request);
MPI_METHOD PMPI_Rget_accumulate(const void* origin_addr, int origin_count,
                                MPI_Datatype origin_datatype, void* result_addr, int result_count,
                                MPI_Datatype result_datatype, int target_rank,
                                MPI_Aint target_disp, int target_count,
                                MPI_Datatype target_datatype, MPI_Op op, MPI_Win win,
                                MPI_Request* request);
MPI_METHOD PMPI_Comm_group(MPI_Comm comm, MPI_Group* group);
MPI_METHOD PMPI_Comm_create(MPI_Comm comm, MPI_Group group, MPI_Comm* newcomm);
MPI_METHOD PMPI_Comm_compare(MPI_Comm comm1, MPI_Comm comm2, int* result);
MPI_METHOD PMPI_Intercomm_create(MPI_Comm local_comm, int local_leader, MPI_Comm peer_comm, int remote_leader,
                                 int tag, MPI_Comm* newintercomm);
MPI_METHOD PMPI_Intercomm_merge(MPI_Comm intercomm, int high, MPI_Comm* newintracomm);
MPI_METHOD PMPI_Group_size(MPI_Group group, int* size);
MPI_METHOD PMPI_Group_rank(MPI_Group group, int* rank);
MPI_METHOD PMPI_Group_free(MPI_Group* group);
MPI_METHOD PMPI_Group_incl(MPI_Group group, int n, const int ranks[], MPI_Group* newgroup);
MPI_METHOD PMPI_Group_excl(MPI_Group group, int n, const int ranks[], MPI_Group* newgroup);
MPI_METHOD PMPI_Group_range_incl(MPI_Group group, int n, int ranges[][3], MPI_Group* newgroup);
MPI_METHOD PMPI_Group_range_excl(MPI_Group group, int n, int ranges[][3], MPI_Group* newgroup);
MPI_METHOD PMPI_Group_union(MPI_Group group1, MPI_Group group2, MPI_Group* newgroup);
MPI_METHOD PMPI_Group_intersection(MPI_Group group1, MPI_Group group2, MPI_Group* newgroup);
MPI_METHOD PMPI_Group_difference(MPI_Group group1, MPI_Group group2, MPI_Group* newgroup);
MPI_METHOD PMPI_Group_translate_ranks(MPI_Group group1, int n, const int ranks1[], MPI_Group group2,
                                      int ranks2[]);
MPI_METHOD PMPI_Group_compare(MPI_Group group1, MPI_Group group2, int* result);
MPI_METHOD PMPI_Win_post(MPI_Group group, int assert, MPI_Win win);
MPI_METHOD PMPI_Win_start(MPI_Group group, int assert, MPI_Win win);
MPI_METHOD PMPI_Win_complete(MPI_Win win);
MPI_METHOD PMPI_Win_wait(MPI_Win win);
MPI_METHOD PMPI_Win_test(MPI_Win win, int* flag);
MPI_METHOD PMPI_Win_get_group(MPI_Win win, MPI_Group* group);
MPI_METHOD PMPI_Testall(int count, MPI_Request array_of_requests[], int* flag,
                        MPI_Status array_of_statuses[]);
MPI_METHOD PMPI_Testany(int count, MPI_Request array_of_requests[], int* index, int* flag,
                        MPI_Status* status);
MPI_METHOD PMPI_Testsome(int incount, MPI_Request array_of_requests[], int* outcount,
                         int array_of_indices[], MPI_Status array_of_statuses[]);
MPI_METHOD PMPI_Waitany(int count, MPI_Request array_of_requests[], int* index,
                        MPI_Status* status);
MPI_METHOD PMPI_Waitsome(int incount, MPI_Request array_of_requests[], int* outcount,
                         int array_of_indices[], MPI_Status array_of_statuses[]);
MPI_METHOD PMPI_Request_free(MPI_Request* request);
MPI_METHOD PMPI_Request_get_status(MPI_Request request, int* flag, MPI_Status* status);
MPI_METHOD PMPI_Op_create(MPI_User_function* user_fn, int commute, MPI_Op* op);
MPI_METHOD PMPI_Op_free(MPI_Op* op);
MPI_METHOD PMPI_Op_commutative(MPI_Op op, int* commute);

#ifdef __cplusplus
}
#endif

#endif /* MSX_MPI_H_INCLUDED */
