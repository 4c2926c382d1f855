// msx_fortran.cpp — Fortran (mpif.h) bindings of the reduction path.
//
// Reference: src/mpi/msmpi/fortran/mpif.cpp (one cdecl entry per MPI call,
// every argument by reference, the error code in a trailing `ierr`) and the
// symbol aliases of fortran/amd64.cdecl.alias (MPI_X, mpi_x, mpi_x_, mpi_x__
// and the PMPI_ forms all name one function).  Only the calls this library
// implements are bound: the reductions and their non-blocking forms, user
// ops, requests, the datatype engine, MPI_Pack and one-sided accumulate.
//
// Fortran sentinels.  MPI_BOTTOM, MPI_IN_PLACE and MPI_STATUS_IGNORE are
// variables of COMMON /MPIPRIV1/ (MPI_STATUSES_IGNORE, MPI_ERRCODES_IGNORE of
// /MPIPRIV2/, include/mpif.h); a Fortran program passes their ADDRESS.  The
// reference learns those addresses from MPIRINITC, called by the Fortran
// routine MPIRINITF (mpif.cpp:43-56, setbotf.f).  Here the common blocks are
// also defined by the library (symbols mpipriv1_/mpipriv2_); when a Fortran
// executable carries its own copy of the block, the dynamic linker's lookup
// (dlsym(RTLD_DEFAULT)) finds the executable's, which is the one its code
// passes.  MPIRINITC is exported too, so a program built with the reference's
// MPIRINITF registers its addresses the reference's way.
//
// Calling convention: on x86-64 SysV a Fortran subroutine with by-reference
// arguments has exactly the C MPI_User_function shape, so MPI_OP_CREATE
// stores the Fortran procedure as is (the reference needs MPIR_Op_f_proxy,
// mpif.cpp:963-976, only because Win32 Fortran is __stdcall).  Fortran
// LOGICAL .TRUE. is 1 (include/mpi_fortlogical.h:14, MPIR_TO_FLOG).
// Hidden CHARACTER lengths are size_t (gfortran >= 8, flang).
#include "../../include/mpi.h"

#include <dlfcn.h>
#include <stddef.h>
#include <string.h>

#include <atomic>
#include <vector>

#define FAPI extern "C" __attribute__((visibility("default")))

// The eight names of one Fortran entry (fortran/amd64.cdecl.alias): the
// definition is mpi_<lc>_; the others are assembler aliases of it.
#define FNAMES(lc, UC)                                         \
    __asm__(".globl MPI_" #UC "\n.set MPI_" #UC ", mpi_" #lc "_\n"     \
            ".globl mpi_" #lc "\n.set mpi_" #lc ", mpi_" #lc "_\n"     \
            ".globl mpi_" #lc "__\n.set mpi_" #lc "__, mpi_" #lc "_\n" \
            ".globl PMPI_" #UC "\n.set PMPI_" #UC ", mpi_" #lc "_\n"   \
            ".globl pmpi_" #lc "\n.set pmpi_" #lc ", mpi_" #lc "_\n"   \
            ".globl pmpi_" #lc "_\n.set pmpi_" #lc "_, mpi_" #lc "_\n" \
            ".globl pmpi_" #lc "__\n.set pmpi_" #lc "__, mpi_" #lc "_\n");

extern "C" {
struct MsxFortranPriv1 {
    MPI_Fint bottom, in_place, status_ignore[5];
};
struct MsxFortranPriv2 {
    MPI_Fint statuses_ignore[5], errcodes_ignore[1];
};
__attribute__((visibility("default"))) MsxFortranPriv1 mpipriv1_;
__attribute__((visibility("default"))) MsxFortranPriv2 mpipriv2_;
}

namespace {

struct Sentinels {
    const void* bottom;
    const void* in_place;
    const void* status_ignore;
    const void* statuses_ignore;
};

std::atomic<const void*> g_reg_bottom{nullptr}, g_reg_in_place{nullptr}, g_reg_status{nullptr},
    g_reg_statuses{nullptr};

const Sentinels& common_blocks()
{
    static const Sentinels s = [] {
        auto* p1 = static_cast<MsxFortranPriv1*>(dlsym(RTLD_DEFAULT, "mpipriv1_"));
        auto* p2 = static_cast<MsxFortranPriv2*>(dlsym(RTLD_DEFAULT, "mpipriv2_"));
        if (!p1) p1 = &mpipriv1_;
        if (!p2) p2 = &mpipriv2_;
        return Sentinels{&p1->bottom, &p1->in_place, p1->status_ignore, p2->statuses_ignore};
    }();
    return s;
}

bool is_sentinel(const void* p, const std::atomic<const void*>& reg, const void* common)
{
    const void* r = reg.load(std::memory_order_relaxed);
    return p && (p == common || (r && p == r));
}

// Fortran MPI_IN_PLACE -> C MPI_IN_PLACE (the reference converts every
// buffer argument of the reductions, e.g. mpif.cpp:692-703)
void* buf(void* p)
{
    return is_sentinel(p, g_reg_in_place, common_blocks().in_place) ? MPI_IN_PLACE : p;
}

MPI_Status* status(MPI_Fint* s)
{
    return is_sentinel(s, g_reg_status, common_blocks().status_ignore) ? MPI_STATUS_IGNORE
                                                                       : reinterpret_cast<MPI_Status*>(s);
}

MPI_Status* statuses(MPI_Fint* s)
{
    return is_sentinel(s, g_reg_statuses, common_blocks().statuses_ignore) ? MPI_STATUSES_IGNORE
                                                                           : reinterpret_cast<MPI_Status*>(s);
}

// addresses are relative to MPI_BOTTOM (mpif.cpp:3800-3808)
MPI_Aint bottom_addr()
{
    const void* r = g_reg_bottom.load(std::memory_order_relaxed);
    return (MPI_Aint)(r ? r : common_blocks().bottom);
}

MPI_Fint to_flog(int v) { return v ? 1 : 0; }

}  // namespace

// ---- MPIRINITC (mpif.cpp:43-56) -----------------------------------------------
FAPI void mpirinitc_(void* a, void* b, void* c, void* d, void* e, void* f, void* g, void* h, MPI_Fint)
{
    (void)e, (void)f, (void)g, (void)h;
    g_reg_bottom.store(a);
    g_reg_in_place.store(b);
    g_reg_status.store(c);
    g_reg_statuses.store(d);
}
FAPI void mpirinitc2_(char* a, size_t) { *a = ' '; }
__asm__(".globl mpirinitc\n.set mpirinitc, mpirinitc_\n"
        ".globl MPIRINITC\n.set MPIRINITC, mpirinitc_\n"
        ".globl mpirinitc2\n.set mpirinitc2, mpirinitc2_\n"
        ".globl MPIRINITC2\n.set MPIRINITC2, mpirinitc2_\n");

// ---- environment ----------------------------------------------------------------
FAPI void mpi_init_(MPI_Fint* ierr) { *ierr = MPI_Init(nullptr, nullptr); }
FNAMES(init, INIT)
FAPI void mpi_init_thread_(const MPI_Fint* required, MPI_Fint* provided, MPI_Fint* ierr)
{
    *ierr = MPI_Init_thread(nullptr, nullptr, *required, provided);
}
FNAMES(init_thread, INIT_THREAD)
FAPI void mpi_finalize_(MPI_Fint* ierr) { *ierr = MPI_Finalize(); }
FNAMES(finalize, FINALIZE)
FAPI void mpi_initialized_(MPI_Fint* flag, MPI_Fint* ierr)
{
    int f = 0;
    *ierr = MPI_Initialized(&f);
    *flag = to_flog(f);
}
FNAMES(initialized, INITIALIZED)
FAPI void mpi_finalized_(MPI_Fint* flag, MPI_Fint* ierr)
{
    int f = 0;
    *ierr = MPI_Finalized(&f);
    *flag = to_flog(f);
}
FNAMES(finalized, FINALIZED)
FAPI void mpi_abort_(const MPI_Fint* comm, const MPI_Fint* code, MPI_Fint* ierr) { *ierr = MPI_Abort(*comm, *code); }
FNAMES(abort, ABORT)
FAPI double mpi_wtime_() { return MPI_Wtime(); }
FNAMES(wtime, WTIME)
FAPI double mpi_wtick_() { return MPI_Wtick(); }
FNAMES(wtick, WTICK)
FAPI void mpi_query_thread_(MPI_Fint* provided, MPI_Fint* ierr) { *ierr = MPI_Query_thread(provided); }
FNAMES(query_thread, QUERY_THREAD)
FAPI void mpi_is_thread_main_(MPI_Fint* flag, MPI_Fint* ierr)
{
    int f = 0;
    *ierr = MPI_Is_thread_main(&f);
    *flag = to_flog(f);
}
FNAMES(is_thread_main, IS_THREAD_MAIN)
FAPI void mpi_get_version_(MPI_Fint* version, MPI_Fint* subversion, MPI_Fint* ierr)
{
    *ierr = MPI_Get_version(version, subversion);
}
FNAMES(get_version, GET_VERSION)
// CHARACTER*(*) name, blank-padded like mpi_error_string_
FAPI void mpi_get_processor_name_(char* name, MPI_Fint* resultlen, MPI_Fint* ierr, size_t len)
{
    char tmp[MPI_MAX_PROCESSOR_NAME] = {0};
    int n = 0;
    *ierr = MPI_Get_processor_name(tmp, &n);
    size_t k = strnlen(tmp, sizeof(tmp));
    if (k > len) k = len;
    memcpy(name, tmp, k);
    if (len > k) memset(name + k, ' ', len - k);
    *resultlen = n;
}
FNAMES(get_processor_name, GET_PROCESSOR_NAME)
FAPI void mpi_comm_rank_(const MPI_Fint* comm, MPI_Fint* rank, MPI_Fint* ierr) { *ierr = MPI_Comm_rank(*comm, rank); }
FNAMES(comm_rank, COMM_RANK)
FAPI void mpi_comm_size_(const MPI_Fint* comm, MPI_Fint* size, MPI_Fint* ierr) { *ierr = MPI_Comm_size(*comm, size); }
FNAMES(comm_size, COMM_SIZE)
FAPI void mpi_barrier_(const MPI_Fint* comm, MPI_Fint* ierr) { *ierr = MPI_Barrier(*comm); }
FNAMES(barrier, BARRIER)
FAPI void mpi_comm_split_(const MPI_Fint* comm, const MPI_Fint* color, const MPI_Fint* key, MPI_Fint* newcomm,
                          MPI_Fint* ierr)
{
    *ierr = MPI_Comm_split(*comm, *color, *key, newcomm);
}
FNAMES(comm_split, COMM_SPLIT)
FAPI void mpi_comm_dup_(const MPI_Fint* comm, MPI_Fint* newcomm, MPI_Fint* ierr) { *ierr = MPI_Comm_dup(*comm, newcomm); }
FNAMES(comm_dup, COMM_DUP)
FAPI void mpi_comm_free_(MPI_Fint* comm, MPI_Fint* ierr) { *ierr = MPI_Comm_free(comm); }
FNAMES(comm_free, COMM_FREE)
// groups (api/mpi_group.cpp): ranks are ranks, not Fortran indices
FAPI void mpi_comm_group_(const MPI_Fint* comm, MPI_Fint* group, MPI_Fint* ierr) { *ierr = MPI_Comm_group(*comm, group); }
FNAMES(comm_group, COMM_GROUP)
FAPI void mpi_comm_create_(const MPI_Fint* comm, const MPI_Fint* group, MPI_Fint* newcomm, MPI_Fint* ierr)
{
    *ierr = MPI_Comm_create(*comm, *group, newcomm);
}
FNAMES(comm_create, COMM_CREATE)
FAPI void mpi_comm_compare_(const MPI_Fint* a, const MPI_Fint* b, MPI_Fint* result, MPI_Fint* ierr)
{
    *ierr = MPI_Comm_compare(*a, *b, result);
}
FNAMES(comm_compare, COMM_COMPARE)
FAPI void mpi_comm_test_inter_(const MPI_Fint* comm, MPI_Fint* flag, MPI_Fint* ierr)
{
    int f = 0;
    *ierr = MPI_Comm_test_inter(*comm, &f);
    *flag = to_flog(f);
}
FNAMES(comm_test_inter, COMM_TEST_INTER)
FAPI void mpi_comm_remote_size_(const MPI_Fint* comm, MPI_Fint* size, MPI_Fint* ierr)
{
    *ierr = MPI_Comm_remote_size(*comm, size);
}
FNAMES(comm_remote_size, COMM_REMOTE_SIZE)
FAPI void mpi_comm_remote_group_(const MPI_Fint* comm, MPI_Fint* group, MPI_Fint* ierr)
{
    *ierr = MPI_Comm_remote_group(*comm, group);
}
FNAMES(comm_remote_group, COMM_REMOTE_GROUP)
FAPI void mpi_intercomm_create_(const MPI_Fint* local_comm, const MPI_Fint* local_leader, const MPI_Fint* peer_comm,
                                const MPI_Fint* remote_leader, const MPI_Fint* tag, MPI_Fint* newintercomm,
                                MPI_Fint* ierr)
{
    *ierr = MPI_Intercomm_create(*local_comm, *local_leader, *peer_comm, *remote_leader, *tag, newintercomm);
}
FNAMES(intercomm_create, INTERCOMM_CREATE)
FAPI void mpi_intercomm_merge_(const MPI_Fint* intercomm, const MPI_Fint* high, MPI_Fint* newintracomm, MPI_Fint* ierr)
{
    *ierr = MPI_Intercomm_merge(*intercomm, *high, newintracomm);   // LOGICAL: nonzero = .TRUE.
}
FNAMES(intercomm_merge, INTERCOMM_MERGE)
FAPI void mpi_group_size_(const MPI_Fint* group, MPI_Fint* size, MPI_Fint* ierr) { *ierr = MPI_Group_size(*group, size); }
FNAMES(group_size, GROUP_SIZE)
FAPI void mpi_group_rank_(const MPI_Fint* group, MPI_Fint* rank, MPI_Fint* ierr) { *ierr = MPI_Group_rank(*group, rank); }
FNAMES(group_rank, GROUP_RANK)
FAPI void mpi_group_incl_(const MPI_Fint* group, const MPI_Fint* n, const MPI_Fint* ranks, MPI_Fint* out, MPI_Fint* ierr)
{
    *ierr = MPI_Group_incl(*group, *n, ranks, out);
}
FNAMES(group_incl, GROUP_INCL)
FAPI void mpi_group_excl_(const MPI_Fint* group, const MPI_Fint* n, const MPI_Fint* ranks, MPI_Fint* out, MPI_Fint* ierr)
{
    *ierr = MPI_Group_excl(*group, *n, ranks, out);
}
FNAMES(group_excl, GROUP_EXCL)
// ranges: INTEGER RANGES(3, N), column-major = n consecutive (first, last, stride) triples
FAPI void mpi_group_range_incl_(const MPI_Fint* group, const MPI_Fint* n, MPI_Fint* ranges, MPI_Fint* out,
                                MPI_Fint* ierr)
{
    *ierr = MPI_Group_range_incl(*group, *n, reinterpret_cast<int (*)[3]>(ranges), out);
}
FNAMES(group_range_incl, GROUP_RANGE_INCL)
FAPI void mpi_group_range_excl_(const MPI_Fint* group, const MPI_Fint* n, MPI_Fint* ranges, MPI_Fint* out,
                                MPI_Fint* ierr)
{
    *ierr = MPI_Group_range_excl(*group, *n, reinterpret_cast<int (*)[3]>(ranges), out);
}
FNAMES(group_range_excl, GROUP_RANGE_EXCL)
FAPI void mpi_group_union_(const MPI_Fint* a, const MPI_Fint* b, MPI_Fint* out, MPI_Fint* ierr)
{
    *ierr = MPI_Group_union(*a, *b, out);
}
FNAMES(group_union, GROUP_UNION)
FAPI void mpi_group_intersection_(const MPI_Fint* a, const MPI_Fint* b, MPI_Fint* out, MPI_Fint* ierr)
{
    *ierr = MPI_Group_intersection(*a, *b, out);
}
FNAMES(group_intersection, GROUP_INTERSECTION)
FAPI void mpi_group_difference_(const MPI_Fint* a, const MPI_Fint* b, MPI_Fint* out, MPI_Fint* ierr)
{
    *ierr = MPI_Group_difference(*a, *b, out);
}
FNAMES(group_difference, GROUP_DIFFERENCE)
FAPI void mpi_group_translate_ranks_(const MPI_Fint* a, const MPI_Fint* n, const MPI_Fint* ranks, const MPI_Fint* b,
                                     MPI_Fint* out, MPI_Fint* ierr)
{
    *ierr = MPI_Group_translate_ranks(*a, *n, ranks, *b, out);
}
FNAMES(group_translate_ranks, GROUP_TRANSLATE_RANKS)
FAPI void mpi_group_compare_(const MPI_Fint* a, const MPI_Fint* b, MPI_Fint* result, MPI_Fint* ierr)
{
    *ierr = MPI_Group_compare(*a, *b, result);
}
FNAMES(group_compare, GROUP_COMPARE)
FAPI void mpi_group_free_(MPI_Fint* group, MPI_Fint* ierr) { *ierr = MPI_Group_free(group); }
FNAMES(group_free, GROUP_FREE)
FAPI void mpi_comm_set_errhandler_(const MPI_Fint* comm, const MPI_Fint* eh, MPI_Fint* ierr)
{
    *ierr = MPI_Comm_set_errhandler(*comm, *eh);
}
FNAMES(comm_set_errhandler, COMM_SET_ERRHANDLER)
FAPI void mpi_comm_get_errhandler_(const MPI_Fint* comm, MPI_Fint* eh, MPI_Fint* ierr)
{
    *ierr = MPI_Comm_get_errhandler(*comm, eh);
}
FNAMES(comm_get_errhandler, COMM_GET_ERRHANDLER)
FAPI void mpi_error_class_(const MPI_Fint* code, MPI_Fint* cls, MPI_Fint* ierr) { *ierr = MPI_Error_class(*code, cls); }
FNAMES(error_class, ERROR_CLASS)
// CHARACTER*(*) string: copied and blank-padded to its declared length
// (mpif.cpp mpi_error_string__)
FAPI void mpi_error_string_(const MPI_Fint* code, char* str, MPI_Fint* resultlen, MPI_Fint* ierr, size_t len)
{
    char tmp[MPI_MAX_ERROR_STRING + 1];
    tmp[0] = 0;
    int n = 0;
    *ierr = MPI_Error_string(*code, tmp, &n);
    size_t k = strnlen(tmp, sizeof(tmp));
    if (k > len) k = len;
    memcpy(str, tmp, k);
    if (len > k) memset(str + k, ' ', len - k);
    *resultlen = n;
}
FNAMES(error_string, ERROR_STRING)

// ---- user ops (mpif.cpp:963-989) ------------------------------------------------
FAPI void mpi_op_create_(MPI_User_function* fn, const MPI_Fint* commute, MPI_Fint* op, MPI_Fint* ierr)
{
    *ierr = MPI_Op_create(fn, *commute, op);
}
FNAMES(op_create, OP_CREATE)
FAPI void mpi_op_commutative_(const MPI_Fint* op, MPI_Fint* commute, MPI_Fint* ierr)
{
    int c = 0;
    *ierr = MPI_Op_commutative(*op, &c);
    *commute = to_flog(c);
}
FNAMES(op_commutative, OP_COMMUTATIVE)
FAPI void mpi_op_free_(MPI_Fint* op, MPI_Fint* ierr) { *ierr = MPI_Op_free(op); }
FNAMES(op_free, OP_FREE)

// ---- reductions (mpif.cpp:692-1047) ---------------------------------------------
FAPI void mpi_reduce_local_(void* in, void* inout, const MPI_Fint* count, const MPI_Fint* dt, const MPI_Fint* op,
                            MPI_Fint* ierr)
{
    *ierr = MPI_Reduce_local(buf(in), buf(inout), *count, *dt, *op);
}
FNAMES(reduce_local, REDUCE_LOCAL)
FAPI void mpi_reduce_(void* s, void* r, const MPI_Fint* count, const MPI_Fint* dt, const MPI_Fint* op,
                      const MPI_Fint* root, const MPI_Fint* comm, MPI_Fint* ierr)
{
    *ierr = MPI_Reduce(buf(s), buf(r), *count, *dt, *op, *root, *comm);
}
FNAMES(reduce, REDUCE)
FAPI void mpi_ireduce_(void* s, void* r, const MPI_Fint* count, const MPI_Fint* dt, const MPI_Fint* op,
                       const MPI_Fint* root, const MPI_Fint* comm, MPI_Fint* req, MPI_Fint* ierr)
{
    *ierr = MPI_Ireduce(buf(s), buf(r), *count, *dt, *op, *root, *comm, req);
}
FNAMES(ireduce, IREDUCE)
FAPI void mpi_allreduce_(void* s, void* r, const MPI_Fint* count, const MPI_Fint* dt, const MPI_Fint* op,
                         const MPI_Fint* comm, MPI_Fint* ierr)
{
    *ierr = MPI_Allreduce(buf(s), buf(r), *count, *dt, *op, *comm);
}
FNAMES(allreduce, ALLREDUCE)
FAPI void mpi_iallreduce_(void* s, void* r, const MPI_Fint* count, const MPI_Fint* dt, const MPI_Fint* op,
                          const MPI_Fint* comm, MPI_Fint* req, MPI_Fint* ierr)
{
    *ierr = MPI_Iallreduce(buf(s), buf(r), *count, *dt, *op, *comm, req);
}
FNAMES(iallreduce, IALLREDUCE)
FAPI void mpi_reduce_scatter_(void* s, void* r, const MPI_Fint* counts, const MPI_Fint* dt, const MPI_Fint* op,
                              const MPI_Fint* comm, MPI_Fint* ierr)
{
    *ierr = MPI_Reduce_scatter(buf(s), buf(r), counts, *dt, *op, *comm);
}
FNAMES(reduce_scatter, REDUCE_SCATTER)
FAPI void mpi_ireduce_scatter_(void* s, void* r, const MPI_Fint* counts, const MPI_Fint* dt, const MPI_Fint* op,
                               const MPI_Fint* comm, MPI_Fint* req, MPI_Fint* ierr)
{
    *ierr = MPI_Ireduce_scatter(buf(s), buf(r), counts, *dt, *op, *comm, req);
}
FNAMES(ireduce_scatter, IREDUCE_SCATTER)
FAPI void mpi_reduce_scatter_block_(void* s, void* r, const MPI_Fint* count, const MPI_Fint* dt, const MPI_Fint* op,
                                    const MPI_Fint* comm, MPI_Fint* ierr)
{
    *ierr = MPI_Reduce_scatter_block(buf(s), buf(r), *count, *dt, *op, *comm);
}
FNAMES(reduce_scatter_block, REDUCE_SCATTER_BLOCK)
FAPI void mpi_ireduce_scatter_block_(void* s, void* r, const MPI_Fint* count, const MPI_Fint* dt,
                                     const MPI_Fint* op, const MPI_Fint* comm, MPI_Fint* req, MPI_Fint* ierr)
{
    *ierr = MPI_Ireduce_scatter_block(buf(s), buf(r), *count, *dt, *op, *comm, req);
}
FNAMES(ireduce_scatter_block, IREDUCE_SCATTER_BLOCK)
FAPI void mpi_scan_(void* s, void* r, const MPI_Fint* count, const MPI_Fint* dt, const MPI_Fint* op,
                    const MPI_Fint* comm, MPI_Fint* ierr)
{
    *ierr = MPI_Scan(buf(s), buf(r), *count, *dt, *op, *comm);
}
FNAMES(scan, SCAN)
FAPI void mpi_iscan_(void* s, void* r, const MPI_Fint* count, const MPI_Fint* dt, const MPI_Fint* op,
                     const MPI_Fint* comm, MPI_Fint* req, MPI_Fint* ierr)
{
    *ierr = MPI_Iscan(buf(s), buf(r), *count, *dt, *op, *comm, req);
}
FNAMES(iscan, ISCAN)
FAPI void mpi_exscan_(void* s, void* r, const MPI_Fint* count, const MPI_Fint* dt, const MPI_Fint* op,
                      const MPI_Fint* comm, MPI_Fint* ierr)
{
    *ierr = MPI_Exscan(buf(s), buf(r), *count, *dt, *op, *comm);
}
FNAMES(exscan, EXSCAN)
FAPI void mpi_iexscan_(void* s, void* r, const MPI_Fint* count, const MPI_Fint* dt, const MPI_Fint* op,
                       const MPI_Fint* comm, MPI_Fint* req, MPI_Fint* ierr)
{
    *ierr = MPI_Iexscan(buf(s), buf(r), *count, *dt, *op, *comm, req);
}
FNAMES(iexscan, IEXSCAN)

// ---- requests (mpif.cpp:164-225) ------------------------------------------------
FAPI void mpi_wait_(MPI_Fint* req, MPI_Fint* st, MPI_Fint* ierr) { *ierr = MPI_Wait(req, status(st)); }
FNAMES(wait, WAIT)
FAPI void mpi_test_(MPI_Fint* req, MPI_Fint* flag, MPI_Fint* st, MPI_Fint* ierr)
{
    int f = 0;
    *ierr = MPI_Test(req, &f, status(st));
    *flag = to_flog(f);
}
FNAMES(test, TEST)
FAPI void mpi_waitall_(const MPI_Fint* n, MPI_Fint* reqs, MPI_Fint* sts, MPI_Fint* ierr)
{
    *ierr = MPI_Waitall(*n, reqs, statuses(sts));
}
FNAMES(waitall, WAITALL)
FAPI void mpi_testall_(const MPI_Fint* n, MPI_Fint* reqs, MPI_Fint* flag, MPI_Fint* sts, MPI_Fint* ierr)
{
    int f = 0;
    *ierr = MPI_Testall(*n, reqs, &f, statuses(sts));
    *flag = to_flog(f);
}
FNAMES(testall, TESTALL)
// indices are 1-based in Fortran (mpif.cpp:190-263); MPI_UNDEFINED stays as is
FAPI void mpi_waitany_(const MPI_Fint* n, MPI_Fint* reqs, MPI_Fint* index, MPI_Fint* st, MPI_Fint* ierr)
{
    int i = 0;
    *ierr = MPI_Waitany(*n, reqs, &i, status(st));
    *index = i >= 0 ? i + 1 : i;
}
FNAMES(waitany, WAITANY)
FAPI void mpi_testany_(const MPI_Fint* n, MPI_Fint* reqs, MPI_Fint* index, MPI_Fint* flag, MPI_Fint* st,
                       MPI_Fint* ierr)
{
    int i = 0, f = 0;
    *ierr = MPI_Testany(*n, reqs, &i, &f, status(st));
    *index = i >= 0 ? i + 1 : i;
    *flag = to_flog(f);
}
FNAMES(testany, TESTANY)
FAPI void mpi_waitsome_(const MPI_Fint* n, MPI_Fint* reqs, MPI_Fint* outcount, MPI_Fint* indices, MPI_Fint* sts,
                        MPI_Fint* ierr)
{
    *ierr = MPI_Waitsome(*n, reqs, outcount, indices, statuses(sts));
    for (int k = 0; k < *outcount; ++k)
        if (indices[k] >= 0) indices[k] += 1;
}
FNAMES(waitsome, WAITSOME)
FAPI void mpi_testsome_(const MPI_Fint* n, MPI_Fint* reqs, MPI_Fint* outcount, MPI_Fint* indices, MPI_Fint* sts,
                        MPI_Fint* ierr)
{
    *ierr = MPI_Testsome(*n, reqs, outcount, indices, statuses(sts));
    for (int k = 0; k < *outcount; ++k)
        if (indices[k] >= 0) indices[k] += 1;
}
FNAMES(testsome, TESTSOME)
FAPI void mpi_request_free_(MPI_Fint* req, MPI_Fint* ierr) { *ierr = MPI_Request_free(req); }
FNAMES(request_free, REQUEST_FREE)
FAPI void mpi_request_get_status_(const MPI_Fint* req, MPI_Fint* flag, MPI_Fint* st, MPI_Fint* ierr)
{
    int f = 0;
    *ierr = MPI_Request_get_status(*req, &f, status(st));
    *flag = to_flog(f);
}
FNAMES(request_get_status, REQUEST_GET_STATUS)

// ---- datatypes (mpif.cpp:401-548, 3253-3300, 3800-3815) ---------------------------
FAPI void mpi_type_size_(const MPI_Fint* dt, MPI_Fint* size, MPI_Fint* ierr) { *ierr = MPI_Type_size(*dt, size); }
FNAMES(type_size, TYPE_SIZE)
FAPI void mpi_type_size_x_(const MPI_Fint* dt, MPI_Count* size, MPI_Fint* ierr) { *ierr = MPI_Type_size_x(*dt, size); }
FNAMES(type_size_x, TYPE_SIZE_X)
FAPI void mpi_type_contiguous_(const MPI_Fint* count, const MPI_Fint* old, MPI_Fint* nt, MPI_Fint* ierr)
{
    *ierr = MPI_Type_contiguous(*count, *old, nt);
}
FNAMES(type_contiguous, TYPE_CONTIGUOUS)
FAPI void mpi_type_vector_(const MPI_Fint* count, const MPI_Fint* blen, const MPI_Fint* stride, const MPI_Fint* old,
                           MPI_Fint* nt, MPI_Fint* ierr)
{
    *ierr = MPI_Type_vector(*count, *blen, *stride, *old, nt);
}
FNAMES(type_vector, TYPE_VECTOR)
// MPI-1 form: the byte stride is a default INTEGER
FAPI void mpi_type_hvector_(const MPI_Fint* count, const MPI_Fint* blen, const MPI_Fint* stride, const MPI_Fint* old,
                            MPI_Fint* nt, MPI_Fint* ierr)
{
    *ierr = MPI_Type_create_hvector(*count, *blen, (MPI_Aint)*stride, *old, nt);
}
FNAMES(type_hvector, TYPE_HVECTOR)
FAPI void mpi_type_create_hvector_(const MPI_Fint* count, const MPI_Fint* blen, const MPI_Aint* stride,
                                   const MPI_Fint* old, MPI_Fint* nt, MPI_Fint* ierr)
{
    *ierr = MPI_Type_create_hvector(*count, *blen, *stride, *old, nt);
}
FNAMES(type_create_hvector, TYPE_CREATE_HVECTOR)
FAPI void mpi_type_indexed_(const MPI_Fint* count, const MPI_Fint* blens, const MPI_Fint* displs, const MPI_Fint* old,
                            MPI_Fint* nt, MPI_Fint* ierr)
{
    *ierr = MPI_Type_indexed(*count, blens, displs, *old, nt);
}
FNAMES(type_indexed, TYPE_INDEXED)
namespace {
std::vector<MPI_Aint> widen(const MPI_Fint* v, MPI_Fint n)
{
    std::vector<MPI_Aint> out(n > 0 ? (size_t)n : 0);
    for (MPI_Fint i = 0; i < n; ++i) out[(size_t)i] = v[i];
    return out;
}
}  // namespace
// MPI-1 forms with default-INTEGER byte displacements, widened to MPI_Aint
// (mpif.cpp mpi_type_hindexed__ / mpi_type_struct__, HAVE_AINT_LARGER_THAN_FINT)
FAPI void mpi_type_hindexed_(const MPI_Fint* count, const MPI_Fint* blens, const MPI_Fint* displs,
                             const MPI_Fint* old, MPI_Fint* nt, MPI_Fint* ierr)
{
    const std::vector<MPI_Aint> d = widen(displs, *count);
    *ierr = MPI_Type_create_hindexed(*count, blens, d.data(), *old, nt);
}
FNAMES(type_hindexed, TYPE_HINDEXED)
FAPI void mpi_type_create_hindexed_(const MPI_Fint* count, const MPI_Fint* blens, const MPI_Aint* displs,
                                    const MPI_Fint* old, MPI_Fint* nt, MPI_Fint* ierr)
{
    *ierr = MPI_Type_create_hindexed(*count, blens, displs, *old, nt);
}
FNAMES(type_create_hindexed, TYPE_CREATE_HINDEXED)
FAPI void mpi_type_create_indexed_block_(const MPI_Fint* count, const MPI_Fint* blen, const MPI_Fint* displs,
                                         const MPI_Fint* old, MPI_Fint* nt, MPI_Fint* ierr)
{
    *ierr = MPI_Type_create_indexed_block(*count, *blen, displs, *old, nt);
}
FNAMES(type_create_indexed_block, TYPE_CREATE_INDEXED_BLOCK)
FAPI void mpi_type_create_hindexed_block_(const MPI_Fint* count, const MPI_Fint* blen, const MPI_Aint* displs,
                                          const MPI_Fint* old, MPI_Fint* nt, MPI_Fint* ierr)
{
    *ierr = MPI_Type_create_hindexed_block(*count, *blen, displs, *old, nt);
}
FNAMES(type_create_hindexed_block, TYPE_CREATE_HINDEXED_BLOCK)
FAPI void mpi_type_struct_(const MPI_Fint* count, const MPI_Fint* blens, const MPI_Fint* displs, const MPI_Fint* types,
                           MPI_Fint* nt, MPI_Fint* ierr)
{
    const std::vector<MPI_Aint> d = widen(displs, *count);
    *ierr = MPI_Type_create_struct(*count, blens, d.data(), types, nt);
}
FNAMES(type_struct, TYPE_STRUCT)
FAPI void mpi_type_create_struct_(const MPI_Fint* count, const MPI_Fint* blens, const MPI_Aint* displs,
                                  const MPI_Fint* types, MPI_Fint* nt, MPI_Fint* ierr)
{
    *ierr = MPI_Type_create_struct(*count, blens, displs, types, nt);
}
FNAMES(type_create_struct, TYPE_CREATE_STRUCT)
FAPI void mpi_type_create_subarray_(const MPI_Fint* ndims, const MPI_Fint* sizes, const MPI_Fint* subsizes,
                                    const MPI_Fint* starts, const MPI_Fint* order, const MPI_Fint* old, MPI_Fint* nt,
                                    MPI_Fint* ierr)
{
    *ierr = MPI_Type_create_subarray(*ndims, sizes, subsizes, starts, *order, *old, nt);
}
FNAMES(type_create_subarray, TYPE_CREATE_SUBARRAY)
FAPI void mpi_type_create_darray_(const MPI_Fint* size, const MPI_Fint* rank, const MPI_Fint* ndims,
                                  const MPI_Fint* gsizes, const MPI_Fint* distribs, const MPI_Fint* dargs,
                                  const MPI_Fint* psizes, const MPI_Fint* order, const MPI_Fint* old, MPI_Fint* nt,
                                  MPI_Fint* ierr)
{
    *ierr = MPI_Type_create_darray(*size, *rank, *ndims, gsizes, distribs, dargs, psizes, *order, *old, nt);
}
FNAMES(type_create_darray, TYPE_CREATE_DARRAY)
FAPI void mpi_type_create_resized_(const MPI_Fint* old, const MPI_Aint* lb, const MPI_Aint* extent, MPI_Fint* nt,
                                   MPI_Fint* ierr)
{
    *ierr = MPI_Type_create_resized(*old, *lb, *extent, nt);
}
FNAMES(type_create_resized, TYPE_CREATE_RESIZED)
FAPI void mpi_type_dup_(const MPI_Fint* old, MPI_Fint* nt, MPI_Fint* ierr) { *ierr = MPI_Type_dup(*old, nt); }
FNAMES(type_dup, TYPE_DUP)
FAPI void mpi_type_commit_(MPI_Fint* dt, MPI_Fint* ierr) { *ierr = MPI_Type_commit(dt); }
FNAMES(type_commit, TYPE_COMMIT)
FAPI void mpi_type_free_(MPI_Fint* dt, MPI_Fint* ierr) { *ierr = MPI_Type_free(dt); }
FNAMES(type_free, TYPE_FREE)
FAPI void mpi_type_get_extent_(const MPI_Fint* dt, MPI_Aint* lb, MPI_Aint* extent, MPI_Fint* ierr)
{
    *ierr = MPI_Type_get_extent(*dt, lb, extent);
}
FNAMES(type_get_extent, TYPE_GET_EXTENT)
FAPI void mpi_type_get_extent_x_(const MPI_Fint* dt, MPI_Count* lb, MPI_Count* extent, MPI_Fint* ierr)
{
    *ierr = MPI_Type_get_extent_x(*dt, lb, extent);
}
FNAMES(type_get_extent_x, TYPE_GET_EXTENT_X)
FAPI void mpi_type_get_true_extent_(const MPI_Fint* dt, MPI_Aint* lb, MPI_Aint* extent, MPI_Fint* ierr)
{
    *ierr = MPI_Type_get_true_extent(*dt, lb, extent);
}
FNAMES(type_get_true_extent, TYPE_GET_TRUE_EXTENT)
FAPI void mpi_type_get_true_extent_x_(const MPI_Fint* dt, MPI_Count* lb, MPI_Count* extent, MPI_Fint* ierr)
{
    *ierr = MPI_Type_get_true_extent_x(*dt, lb, extent);
}
FNAMES(type_get_true_extent_x, TYPE_GET_TRUE_EXTENT_X)
// MPI-1 queries return default INTEGERs (mpif.cpp mpi_type_extent__/lb__/ub__)
FAPI void mpi_type_extent_(const MPI_Fint* dt, MPI_Fint* extent, MPI_Fint* ierr)
{
    MPI_Aint lb = 0, ext = 0;
    *ierr = MPI_Type_get_extent(*dt, &lb, &ext);
    *extent = (MPI_Fint)ext;
}
FNAMES(type_extent, TYPE_EXTENT)
FAPI void mpi_type_lb_(const MPI_Fint* dt, MPI_Fint* lbout, MPI_Fint* ierr)
{
    MPI_Aint lb = 0, ext = 0;
    *ierr = MPI_Type_get_extent(*dt, &lb, &ext);
    *lbout = (MPI_Fint)lb;
}
FNAMES(type_lb, TYPE_LB)
FAPI void mpi_type_ub_(const MPI_Fint* dt, MPI_Fint* ubout, MPI_Fint* ierr)
{
    MPI_Aint lb = 0, ext = 0;
    *ierr = MPI_Type_get_extent(*dt, &lb, &ext);
    *ubout = (MPI_Fint)(lb + ext);
}
FNAMES(type_ub, TYPE_UB)
FAPI void mpi_type_get_envelope_(const MPI_Fint* dt, MPI_Fint* ni, MPI_Fint* na, MPI_Fint* nd, MPI_Fint* comb,
                                 MPI_Fint* ierr)
{
    *ierr = MPI_Type_get_envelope(*dt, ni, na, nd, comb);
}
FNAMES(type_get_envelope, TYPE_GET_ENVELOPE)
FAPI void mpi_type_get_contents_(const MPI_Fint* dt, const MPI_Fint* mi, const MPI_Fint* ma, const MPI_Fint* md,
                                 MPI_Fint* ints, MPI_Aint* addrs, MPI_Fint* types, MPI_Fint* ierr)
{
    *ierr = MPI_Type_get_contents(*dt, *mi, *ma, *md, ints, addrs, types);
}
FNAMES(type_get_contents, TYPE_GET_CONTENTS)
FAPI void mpi_get_address_(void* loc, MPI_Aint* addr, MPI_Fint* ierr)
{
    MPI_Aint a = 0;
    *ierr = MPI_Get_address(loc, &a);
    *addr = a - bottom_addr();
}
FNAMES(get_address, GET_ADDRESS)
// MPI-1 MPI_ADDRESS: a default INTEGER; truncation is MPI_ERR_ARG
FAPI void mpi_address_(void* loc, MPI_Fint* addr, MPI_Fint* ierr)
{
    MPI_Aint a = 0;
    *ierr = MPI_Get_address(loc, &a);
    const MPI_Aint b = a - bottom_addr();
    *addr = (MPI_Fint)b;
    if (*ierr == MPI_SUCCESS && (MPI_Aint)*addr != b) *ierr = MPI_ERR_ARG;
}
FNAMES(address, ADDRESS)
FAPI void mpi_pack_(void* in, const MPI_Fint* incount, const MPI_Fint* dt, void* out, const MPI_Fint* outsize,
                    MPI_Fint* position, const MPI_Fint* comm, MPI_Fint* ierr)
{
    *ierr = MPI_Pack(in, *incount, *dt, out, *outsize, position, *comm);
}
FNAMES(pack, PACK)
FAPI void mpi_unpack_(void* in, const MPI_Fint* insize, MPI_Fint* position, void* out, const MPI_Fint* outcount,
                      const MPI_Fint* dt, const MPI_Fint* comm, MPI_Fint* ierr)
{
    *ierr = MPI_Unpack(in, *insize, position, out, *outcount, *dt, *comm);
}
FNAMES(unpack, UNPACK)
FAPI void mpi_pack_size_(const MPI_Fint* incount, const MPI_Fint* dt, const MPI_Fint* comm, MPI_Fint* size,
                         MPI_Fint* ierr)
{
    *ierr = MPI_Pack_size(*incount, *dt, *comm, size);
}
FNAMES(pack_size, PACK_SIZE)

// ---- one-sided (mpif.cpp:2032-2175) -----------------------------------------------
FAPI void mpi_win_create_(void* base, const MPI_Aint* size, const MPI_Fint* disp_unit, const MPI_Fint* info,
                          const MPI_Fint* comm, MPI_Fint* win, MPI_Fint* ierr)
{
    *ierr = MPI_Win_create(base, *size, *disp_unit, *info, *comm, win);
}
FNAMES(win_create, WIN_CREATE)
FAPI void mpi_win_free_(MPI_Fint* win, MPI_Fint* ierr) { *ierr = MPI_Win_free(win); }
FNAMES(win_free, WIN_FREE)
FAPI void mpi_win_fence_(const MPI_Fint* assert_, const MPI_Fint* win, MPI_Fint* ierr)
{
    *ierr = MPI_Win_fence(*assert_, *win);
}
FNAMES(win_fence, WIN_FENCE)
FAPI void mpi_win_lock_(const MPI_Fint* lock_type, const MPI_Fint* rank, const MPI_Fint* assert_, const MPI_Fint* win,
                        MPI_Fint* ierr)
{
    *ierr = MPI_Win_lock(*lock_type, *rank, *assert_, *win);
}
FNAMES(win_lock, WIN_LOCK)
FAPI void mpi_win_unlock_(const MPI_Fint* rank, const MPI_Fint* win, MPI_Fint* ierr) { *ierr = MPI_Win_unlock(*rank, *win); }
FNAMES(win_unlock, WIN_UNLOCK)
FAPI void mpi_win_lock_all_(const MPI_Fint* assert_, const MPI_Fint* win, MPI_Fint* ierr)
{
    *ierr = MPI_Win_lock_all(*assert_, *win);
}
FNAMES(win_lock_all, WIN_LOCK_ALL)
FAPI void mpi_win_unlock_all_(const MPI_Fint* win, MPI_Fint* ierr) { *ierr = MPI_Win_unlock_all(*win); }
FNAMES(win_unlock_all, WIN_UNLOCK_ALL)
FAPI void mpi_win_flush_(const MPI_Fint* rank, const MPI_Fint* win, MPI_Fint* ierr) { *ierr = MPI_Win_flush(*rank, *win); }
FNAMES(win_flush, WIN_FLUSH)
FAPI void mpi_win_flush_all_(const MPI_Fint* win, MPI_Fint* ierr) { *ierr = MPI_Win_flush_all(*win); }
FNAMES(win_flush_all, WIN_FLUSH_ALL)
FAPI void mpi_win_flush_local_(const MPI_Fint* rank, const MPI_Fint* win, MPI_Fint* ierr)
{
    *ierr = MPI_Win_flush_local(*rank, *win);
}
FNAMES(win_flush_local, WIN_FLUSH_LOCAL)
FAPI void mpi_win_flush_local_all_(const MPI_Fint* win, MPI_Fint* ierr) { *ierr = MPI_Win_flush_local_all(*win); }
FNAMES(win_flush_local_all, WIN_FLUSH_LOCAL_ALL)
FAPI void mpi_win_sync_(const MPI_Fint* win, MPI_Fint* ierr) { *ierr = MPI_Win_sync(*win); }
FNAMES(win_sync, WIN_SYNC)
FAPI void mpi_win_post_(const MPI_Fint* group, const MPI_Fint* assert_, const MPI_Fint* win, MPI_Fint* ierr)
{
    *ierr = MPI_Win_post(*group, *assert_, *win);
}
FNAMES(win_post, WIN_POST)
FAPI void mpi_win_start_(const MPI_Fint* group, const MPI_Fint* assert_, const MPI_Fint* win, MPI_Fint* ierr)
{
    *ierr = MPI_Win_start(*group, *assert_, *win);
}
FNAMES(win_start, WIN_START)
FAPI void mpi_win_complete_(const MPI_Fint* win, MPI_Fint* ierr) { *ierr = MPI_Win_complete(*win); }
FNAMES(win_complete, WIN_COMPLETE)
FAPI void mpi_win_wait_(const MPI_Fint* win, MPI_Fint* ierr) { *ierr = MPI_Win_wait(*win); }
FNAMES(win_wait, WIN_WAIT)
FAPI void mpi_win_test_(const MPI_Fint* win, MPI_Fint* flag, MPI_Fint* ierr)
{
    int f = 0;
    *ierr = MPI_Win_test(*win, &f);
    *flag = to_flog(f);
}
FNAMES(win_test, WIN_TEST)
FAPI void mpi_win_get_group_(const MPI_Fint* win, MPI_Fint* group, MPI_Fint* ierr)
{
    *ierr = MPI_Win_get_group(*win, group);
}
FNAMES(win_get_group, WIN_GET_GROUP)
FAPI void mpi_win_set_errhandler_(const MPI_Fint* win, const MPI_Fint* eh, MPI_Fint* ierr)
{
    *ierr = MPI_Win_set_errhandler(*win, *eh);
}
FNAMES(win_set_errhandler, WIN_SET_ERRHANDLER)
FAPI void mpi_win_get_errhandler_(const MPI_Fint* win, MPI_Fint* eh, MPI_Fint* ierr)
{
    *ierr = MPI_Win_get_errhandler(*win, eh);
}
FNAMES(win_get_errhandler, WIN_GET_ERRHANDLER)
FAPI void mpi_put_(void* o, const MPI_Fint* ocount, const MPI_Fint* odt, const MPI_Fint* target, const MPI_Aint* disp,
                   const MPI_Fint* tcount, const MPI_Fint* tdt, const MPI_Fint* win, MPI_Fint* ierr)
{
    *ierr = MPI_Put(o, *ocount, *odt, *target, *disp, *tcount, *tdt, *win);
}
FNAMES(put, PUT)
FAPI void mpi_get_(void* o, const MPI_Fint* ocount, const MPI_Fint* odt, const MPI_Fint* target, const MPI_Aint* disp,
                   const MPI_Fint* tcount, const MPI_Fint* tdt, const MPI_Fint* win, MPI_Fint* ierr)
{
    *ierr = MPI_Get(o, *ocount, *odt, *target, *disp, *tcount, *tdt, *win);
}
FNAMES(get, GET)
FAPI void mpi_accumulate_(void* o, const MPI_Fint* ocount, const MPI_Fint* odt, const MPI_Fint* target,
                          const MPI_Aint* disp, const MPI_Fint* tcount, const MPI_Fint* tdt, const MPI_Fint* op,
                          const MPI_Fint* win, MPI_Fint* ierr)
{
    *ierr = MPI_Accumulate(o, *ocount, *odt, *target, *disp, *tcount, *tdt, *op, *win);
}
FNAMES(accumulate, ACCUMULATE)
FAPI void mpi_get_accumulate_(void* o, const MPI_Fint* ocount, const MPI_Fint* odt, void* r, const MPI_Fint* rcount,
                              const MPI_Fint* rdt, const MPI_Fint* target, const MPI_Aint* disp,
                              const MPI_Fint* tcount, const MPI_Fint* tdt, const MPI_Fint* op, const MPI_Fint* win,
                              MPI_Fint* ierr)
{
    *ierr = MPI_Get_accumulate(o, *ocount, *odt, r, *rcount, *rdt, *target, *disp, *tcount, *tdt, *op, *win);
}
FNAMES(get_accumulate, GET_ACCUMULATE)
FAPI void mpi_fetch_and_op_(void* o, void* r, const MPI_Fint* dt, const MPI_Fint* target, const MPI_Aint* disp,
                            const MPI_Fint* op, const MPI_Fint* win, MPI_Fint* ierr)
{
    *ierr = MPI_Fetch_and_op(o, r, *dt, *target, *disp, *op, *win);
}
FNAMES(fetch_and_op, FETCH_AND_OP)
FAPI void mpi_compare_and_swap_(void* o, void* c, void* r, const MPI_Fint* dt, const MPI_Fint* target,
                                const MPI_Aint* disp, const MPI_Fint* win, MPI_Fint* ierr)
{
    *ierr = MPI_Compare_and_swap(o, c, r, *dt, *target, *disp, *win);
}
FNAMES(compare_and_swap, COMPARE_AND_SWAP)
FAPI void mpi_rput_(void* o, const MPI_Fint* ocount, const MPI_Fint* odt, const MPI_Fint* target, const MPI_Aint* disp,
                    const MPI_Fint* tcount, const MPI_Fint* tdt, const MPI_Fint* win, MPI_Fint* req, MPI_Fint* ierr)
{
    *ierr = MPI_Rput(o, *ocount, *odt, *target, *disp, *tcount, *tdt, *win, req);
}
FNAMES(rput, RPUT)
FAPI void mpi_rget_(void* o, const MPI_Fint* ocount, const MPI_Fint* odt, const MPI_Fint* target, const MPI_Aint* disp,
                    const MPI_Fint* tcount, const MPI_Fint* tdt, const MPI_Fint* win, MPI_Fint* req, MPI_Fint* ierr)
{
    *ierr = MPI_Rget(o, *ocount, *odt, *target, *disp, *tcount, *tdt, *win, req);
}
FNAMES(rget, RGET)
FAPI void mpi_raccumulate_(void* o, const MPI_Fint* ocount, const MPI_Fint* odt, const MPI_Fint* target,
                           const MPI_Aint* disp, const MPI_Fint* tcount, const MPI_Fint* tdt, const MPI_Fint* op,
                           const MPI_Fint* win, MPI_Fint* req, MPI_Fint* ierr)
{
    *ierr = MPI_Raccumulate(o, *ocount, *odt, *target, *disp, *tcount, *tdt, *op, *win, req);
}
FNAMES(raccumulate, RACCUMULATE)
FAPI void mpi_rget_accumulate_(void* o, const MPI_Fint* ocount, const MPI_Fint* odt, void* r, const MPI_Fint* rcount,
                               const MPI_Fint* rdt, const MPI_Fint* target, const MPI_Aint* disp,
                               const MPI_Fint* tcount, const MPI_Fint* tdt, const MPI_Fint* op, const MPI_Fint* win,
                               MPI_Fint* req, MPI_Fint* ierr)
{
    *ierr = MPI_Rget_accumulate(o, *ocount, *odt, r, *rcount, *rdt, *target, *disp, *tcount, *tdt, *op, *win, req);
}
FNAMES(rget_accumulate, RGET_ACCUMULATE)
