"""Fortran bindings (mpif.h, fortran/mpif.cpp) without a GPU.

* include/mpif.h is the generator's output for the current include/mpi.h;
* the library exports the eight names of every Fortran entry
  (fortran/amd64.cdecl.alias: MPI_X, mpi_x, mpi_x_, mpi_x__, PMPI_X, pmpi_x,
  pmpi_x_, pmpi_x__), all at one address;
* a Fortran program built with flang against include/mpif.h drives the
  environment, datatype constructors/queries (checked against the oracle's
  type maps), user ops (host functions, so no GPU), and the sentinel path:
  the Fortran MPI_IN_PLACE must reach MPI_Reduce_local as the C MPI_IN_PLACE
  (rejected there with MPI_ERR_BUFFER, mpi_reduce.cpp:304-385).
"""
import os
import subprocess
import sys

import pytest

import msx
from oracle import msx_dtype_oracle as O

C = msx.C
REPO = msx.REPO_ROOT
FDIR = os.path.join(REPO, "tests", "fortran")
FLANG = "/opt/rocm/lib/llvm/bin/flang"

ENTRIES = [
    "init", "init_thread", "finalize", "initialized", "finalized", "abort", "wtime", "comm_rank",
    "comm_size", "barrier", "comm_split", "comm_dup", "comm_free", "comm_set_errhandler", "comm_get_errhandler", "error_class", "error_string",
    "op_create", "op_commutative", "op_free",
    "reduce_local", "reduce", "ireduce", "allreduce", "iallreduce", "reduce_scatter", "ireduce_scatter",
    "reduce_scatter_block", "ireduce_scatter_block", "scan", "iscan", "exscan", "iexscan",
    "wait", "test", "waitall", "waitany", "waitsome", "testall", "testany", "testsome", "request_free",
    "request_get_status",
    "comm_group", "group_size", "group_rank", "group_incl", "group_excl", "group_range_incl",
    "group_range_excl", "group_union", "group_intersection", "group_difference", "group_translate_ranks",
    "group_compare", "group_free",
    "wtick", "query_thread", "is_thread_main", "get_version", "get_processor_name", "comm_create",
    "comm_compare", "comm_test_inter", "comm_remote_size", "comm_remote_group", "intercomm_create",
    "intercomm_merge", "rput", "rget", "raccumulate", "rget_accumulate",
    "win_post", "win_start", "win_complete", "win_wait", "win_test", "win_get_group",
    "type_size", "type_size_x", "type_contiguous", "type_vector", "type_hvector", "type_create_hvector",
    "type_indexed", "type_hindexed", "type_create_hindexed", "type_create_indexed_block",
    "type_create_hindexed_block", "type_struct", "type_create_struct", "type_create_subarray",
    "type_create_darray", "type_create_resized", "type_dup", "type_commit", "type_free", "type_get_extent",
    "type_get_extent_x", "type_get_true_extent", "type_get_true_extent_x", "type_extent", "type_lb",
    "type_ub", "type_get_envelope", "type_get_contents", "get_address", "address", "pack", "unpack",
    "pack_size",
    "win_create", "win_free", "win_fence", "win_set_errhandler", "win_get_errhandler", "put", "get",
    "win_lock", "win_unlock", "win_lock_all", "win_unlock_all", "win_flush", "win_flush_all", "win_flush_local",
    "win_flush_local_all", "win_sync",
    "accumulate", "get_accumulate", "fetch_and_op", "compare_and_swap",
]


def _names(e):
    return [f"MPI_{e.upper()}", f"mpi_{e}", f"mpi_{e}_", f"mpi_{e}__",
            f"PMPI_{e.upper()}", f"pmpi_{e}", f"pmpi_{e}_", f"pmpi_{e}__"]


def test_mpif_h_is_generated_from_mpi_h():
    r = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "gen_mpif.py"), "--check"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def test_mpif_h_values():
    text = open(os.path.join(REPO, "include", "mpif.h")).read()
    vals = {}
    for line in text.splitlines():
        line = line.strip()
        if line.startswith("PARAMETER ("):
            k, v = line[len("PARAMETER ("):-1].split("=")
            vals[k] = int(v)
    # ABI values of the reference's mpif.h / mpi.h (signed 32-bit)
    assert vals["MPI_COMM_WORLD"] == 0x44000000
    assert vals["MPI_SUM"] == 0x58000003
    assert vals["MPI_INTEGER"] == 0x4C00041B
    assert vals["MPI_DOUBLE_PRECISION"] == 0x4C00081F
    assert vals["MPI_2INTEGER"] == 0x4C000820
    assert vals["MPI_STATUS_SIZE"] == 5 and vals["MPI_SOURCE"] == 3 and vals["MPI_ERROR"] == 5
    assert vals["MPI_ADDRESS_KIND"] == 8
    for k, v in vals.items():
        if hasattr(C, k):
            assert getattr(C, k) == v, k
    assert "COMMON /MPIPRIV1/ MPI_BOTTOM, MPI_IN_PLACE, MPI_STATUS_IGNORE" in text
    assert all(len(l) <= 72 for l in text.splitlines())


def test_every_fortran_entry_and_alias_is_exported():
    import ctypes
    L = msx.lib()
    for e in ENTRIES:
        addrs = set()
        for n in _names(e):
            addrs.add(ctypes.cast(getattr(L, n), ctypes.c_void_p).value)
        assert len(addrs) == 1, (e, addrs)
    for n in ("mpirinitc_", "MPIRINITC", "mpipriv1_", "mpipriv2_"):
        assert hasattr(L, n), n


def _build(prog):
    exe = os.path.join(FDIR, "build", prog)
    if not os.path.exists(FLANG):
        pytest.skip("flang not in this image")
    r = subprocess.run(["make", "-C", FDIR, f"build/{prog}"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return exe


def _run(exe, env_extra=None):
    env = dict(os.environ)
    for k in ("MSX_SIZE", "MSX_RANK"):
        env.pop(k, None)
    env.update(env_extra or {})
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = {}
    for line in r.stdout.splitlines():
        parts = line.split()
        if parts:
            out[parts[0]] = parts[1:]
    return out


def test_fortran_program_without_gpu():
    out = _run(_build("f_cpu"))
    as_int = lambda k: [int(x) for x in out[k]]
    assert as_int("INIT") == [0]
    assert out["INITIALIZED"] == ["T"]
    assert as_int("RANK_SIZE") == [0, 1]
    v = O.vector(3, 2, 5, O.predefined(C.MPI_DOUBLE_PRECISION))
    assert as_int("VECTOR") == [v.size, v.lb, v.extent]
    assert as_int("VECTOR_SIZE_X") == [v.size]
    assert as_int("ENVELOPE") == [3, 0, 1, C.MPI_COMBINER_VECTOR]
    assert as_int("CONTENTS") == [3, 2, 5, C.MPI_DOUBLE_PRECISION]
    h = O.hvector(2, 1, 24, O.predefined(C.MPI_INTEGER))
    # MPI_TYPE_HVECTOR from Fortran builds through MPI_Type_create_hvector
    # (mpif.cpp mpi_type_hvector__), so the combiner is HVECTOR
    assert as_int("HVECTOR") == [h.extent, C.MPI_COMBINER_HVECTOR]
    s = O.struct([1, 1], [0, 8], [O.predefined(C.MPI_INTEGER), O.predefined(C.MPI_DOUBLE_PRECISION)])
    assert as_int("STRUCT") == [s.size, s.extent, s.extent]
    sa = O.subarray([6, 5, 4], [2, 3, 2], [1, 2, 1], False, O.predefined(C.MPI_REAL))
    assert as_int("SUBARRAY") == [sa.size, sa.lb, sa.extent, sa.true_lb, sa.true_ub - sa.true_lb]
    assert as_int("ADDRESS_DIFF") == [8, 8]
    assert out["OP_CREATE"] == ["0", "T"]
    assert out["OP2_COMMUTATIVE"] == ["F"]
    assert out["USER_REDUCE_LOCAL"] == ["0", "T", "10", "T"]
    assert as_int("IN_PLACE_CLASS") == [C.MPI_ERR_BUFFER]
    assert as_int("BAND_DOUBLE_CLASS") == [C.MPI_ERR_OP]
    assert as_int("COUNT0") == [0]
    assert as_int("WAITANY") == [0, 1]
    assert out["TESTANY"] == ["0", "3", "T"]
    assert out["TESTANY_NONE"] == [str(-32766), "T"]
    assert out["TESTALL"] == ["0", "T", "T"]
    assert as_int("WAITSOME") == [0, 1, 3]
    assert out["GET_STATUS"] == ["0", "T", "T"]
    assert as_int("REQUEST_FREE_CLASS") == [C.MPI_ERR_OTHER]
    assert as_int("TESTSOME") == [0, 1, 1]
    assert as_int("TESTSOME_NONE") == [-32766]
    assert as_int("GROUP") == [0, 1, 0]
    assert out["RANGE_INCL"] == ["0", "T"]
    assert as_int("RANGE_DUP_CLASS") == [C.MPI_ERR_ARG]     # **rangedup, mpid/group.cpp:372-390
    assert as_int("EXCL") == [0, 0, -32766]
    # group2 is empty: even MPI_PROC_NULL stays MPI_UNDEFINED (api/mpi_group.cpp:1351-1368)
    assert as_int("TRANSLATE") == [0, -32766, -32766]
    assert out["UNION_IDENT"] == ["T"]
    assert out["INTERSECTION_EMPTY"] == ["T"]
    assert as_int("DIFFERENCE") == [0]
    assert out["VERSION"] == ["2", "0", str(C.MPI_THREAD_SINGLE), "T"]
    assert out["PROCNAME"] == ["0", "T", "T"]
    assert out["WTICK"] == ["T"]
    assert out["COMM_CREATE"] == ["0", "T", "F"]
    assert out["PSCW"] == ["0", "T", "T"]
    assert as_int("COMPLETE_CLASS") == [C.MPI_ERR_RMA_SYNC]
    assert out["GROUP_FREE"] == ["0", "T"]
    assert out["ERROR_STRING"] == ["0", "T", "T"]
    assert as_int("PACK_SIZE") == [12]
    assert out["WTIME"] == ["T"]
    assert out["OP_FREE"] == ["T"]
    assert as_int("FREE_BUILTIN_CLASS") == [C.MPI_ERR_OP]
    assert out["TYPE_FREE"] == ["T"]
    assert out["FINALIZE"] == ["0", "T"]


def test_registered_sentinels_are_honoured():
    """A program built with the reference's MPIRINITF registers its own
    sentinel addresses through MPIRINITC (mpif.cpp:43-56); those are then
    recognised as MPI_IN_PLACE exactly like the common block's."""
    import ctypes
    L = msx.init(errors_return=True)
    fint = ctypes.c_int
    block = (fint * 8)()
    L.mpirinitc_.argtypes = [ctypes.c_void_p] * 8 + [fint]
    L.mpirinitc_(ctypes.addressof(block), ctypes.addressof(block) + 4, ctypes.addressof(block) + 8,
                 None, None, None, None, None, 0)
    a = (fint * 4)(1, 2, 3, 4)
    cnt, dt, op, ierr = fint(4), fint(C.MPI_INT), fint(C.MPI_SUM), fint(-1)
    L.mpi_reduce_local_.argtypes = [ctypes.c_void_p] * 6
    L.mpi_reduce_local_(ctypes.addressof(block) + 4, a, ctypes.byref(cnt), ctypes.byref(dt), ctypes.byref(op),
                        ctypes.byref(ierr))
    cls = fint()
    L.MPI_Error_class(ierr.value, ctypes.byref(cls))
    assert cls.value == C.MPI_ERR_BUFFER
    # the library's own common block is recognised too
    own = ctypes.addressof(fint.in_dll(L, "mpipriv1_")) + 4
    L.mpi_reduce_local_(own, a, ctypes.byref(cnt), ctypes.byref(dt), ctypes.byref(op), ctypes.byref(ierr))
    L.MPI_Error_class(ierr.value, ctypes.byref(cls))
    assert cls.value == C.MPI_ERR_BUFFER
    # unregister (this process's later callers must not match a dead block)
    L.mpirinitc_(None, None, None, None, None, None, None, None, 0)
