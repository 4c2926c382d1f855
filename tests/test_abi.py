"""CPU: the C-ABI library loads, exports every symbol the headers declare, keeps
MS-MPI's handle values, and reproduces MPI_Reduce_local's argument checks in
the reference's order (api/mpi_reduce.cpp:304-385, api/mpi_api.h:113-212,
707-775).  No compute call here needs a GPU."""
import ctypes
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

import msx
import oracle
from _cases import KIND, NON_REDUCIBLE, OPS, h

C = msx.C


def test_library_exports_every_declared_symbol():
    L = msx.lib()
    missing = [s for s in msx.exported_symbols() if not hasattr(L, s)]
    assert not missing, missing
    assert len(msx.exported_symbols()) >= 50


def test_handle_values_match_msmpi_abi():
    # src/include/mpi.h:192-250, 281-368, 410-426, 441-463, 1956
    assert (C.MPI_SUCCESS, C.MPI_ERR_BUFFER, C.MPI_ERR_COUNT, C.MPI_ERR_TYPE, C.MPI_ERR_OP,
            C.MPI_ERR_ARG, C.MPI_ERR_OTHER) == (0, 1, 2, 3, 9, 12, 15)
    u = lambda v: v & 0xFFFFFFFF
    assert u(C.MPI_SUM) == 0x58000003 and u(C.MPI_MAXLOC) == 0x5800000C and u(C.MPI_OP_NULL) == 0x18000000
    assert u(C.MPI_FLOAT) == 0x4C00040A and u(C.MPI_LONG) == 0x4C000407 and u(C.MPI_UINT64_T) == 0x4C00083A
    assert u(C.MPI_LONG_DOUBLE) == 0x4C00080C and u(C.MPI_AINT) == 0x4C00083B
    assert u(C.MPI_FLOAT_INT) == 0x8C000000 and u(C.MPI_LONG_DOUBLE_INT) == 0x8C000004
    assert u(C.MPI_COMM_WORLD) == 0x44000000 and u(C.MPI_ERRORS_RETURN) == 0x54000001
    assert C.MPI_IN_PLACE == -1 and C.MPI_REAL2 == C.MPI_DATATYPE_NULL
    # element size lives in byte 1 of the handle (include/datatype.h:36)
    L = msx.lib()
    for name, kind in KIND.items():
        hv = u(h(name))
        if hv >> 24 == 0x4C:
            assert L.msx_type_size(h(name)) == (hv >> 8) & 0xFF, name


# Constants of the reference header that name subsystems outside the reduction
# path (MPI-IO, point-to-point / buffered sends, attributes and window
# attributes, dynamic processes, matched probes): not declared by include/mpi.h.
_OUT_OF_PATH_CONSTANTS = {
    "MPI_APPNUM", "MPI_BSEND_OVERHEAD", "MPI_DISPLACEMENT_CURRENT", "MPI_FILE_NULL", "MPI_HOST", "MPI_IO",
    "MPI_KEYVAL_INVALID", "MPI_LASTUSEDCODE", "MPI_MAX_DATAREP_STRING", "MPI_MAX_INFO_KEY", "MPI_MAX_INFO_VAL",
    "MPI_MAX_LIBRARY_VERSION_STRING", "MPI_MAX_OBJECT_NAME", "MPI_MAX_PORT_NAME", "MPI_MESSAGE_NO_PROC",
    "MPI_MESSAGE_NULL", "MPI_MODE_APPEND", "MPI_MODE_CREATE", "MPI_MODE_DELETE_ON_CLOSE", "MPI_MODE_EXCL",
    "MPI_MODE_RDONLY", "MPI_MODE_RDWR", "MPI_MODE_SEQUENTIAL", "MPI_MODE_UNIQUE_OPEN", "MPI_MODE_WRONLY",
    "MPI_SEEK_CUR", "MPI_SEEK_END", "MPI_SEEK_SET", "MPI_TAG_UB", "MPI_TYPECLASS_COMPLEX", "MPI_TYPECLASS_INTEGER",
    "MPI_TYPECLASS_REAL", "MPI_UNIVERSE_SIZE", "MPI_WIN_BASE", "MPI_WIN_CREATE_FLAVOR", "MPI_WIN_DISP_UNIT",
    "MPI_WIN_FLAVOR_ALLOCATE", "MPI_WIN_FLAVOR_CREATE", "MPI_WIN_FLAVOR_DYNAMIC", "MPI_WIN_FLAVOR_SHARED",
    "MPI_WIN_MODEL", "MPI_WIN_SEPARATE", "MPI_WIN_SIZE", "MPI_WIN_UNIFIED", "MPI_WTIME_IS_GLOBAL",
    "MSMPI_BSEND_OVERHEAD_V1", "MSMPI_BSEND_OVERHEAD_V2", "MSMPI_MODE_HIDDEN", "MSMPI_VER"}


def test_header_constants_match_the_reference_header():
    """Every integer constant of include/mpi.h that the reference's
    src/include/mpi.h also defines has the reference's value (x64 branch), and
    every reference constant is declared except the out-of-path list above.
    The reference values are the data fixture tests/golden/mpi_h_constants.json
    (229 constants), made by tests/golden/gen_mpi_h_constants.py from the
    reference header in the survey container."""
    import json
    sys.path.insert(0, os.path.join(msx.REPO_ROOT, "tests", "golden"))
    import gen_mpi_h_constants as gen
    with open(os.path.join(msx.REPO_ROOT, "tests", "golden", "mpi_h_constants.json")) as f:
        ref = json.load(f)["constants"]
    with open(os.path.join(msx.REPO_ROOT, "include", "mpi.h")) as f:
        ours = gen.parse(f.read(), defined={"_WIN64", "MSMPI_NO_SAL"})
    shared = sorted(set(ref) & set(ours))
    assert len(shared) >= 180
    wrong = [(k, hex(ref[k]), hex(ours[k])) for k in shared if ref[k] != ours[k]]
    assert not wrong, wrong
    missing = sorted(set(ref) - set(ours) - _OUT_OF_PATH_CONSTANTS)
    assert not missing, missing
    # and the values the library itself reports (msx.C is read from the same header)
    for k in shared:
        if hasattr(C, k):
            assert getattr(C, k) & 0xFFFFFFFF == ref[k] & 0xFFFFFFFF, k


def test_type_sizes_llp64():
    L = msx.lib()
    assert L.msx_type_size(C.MPI_LONG) == 4 and L.msx_type_size(C.MPI_UNSIGNED_LONG) == 4
    assert L.msx_type_size(C.MPI_LONG_DOUBLE) == 8
    assert L.msx_type_size(C.MPI_SHORT_INT) == 8 and L.msx_type_size(C.MPI_DOUBLE_INT) == 16


def test_op_check_matches_oracle_everywhere():
    L = msx.lib()
    for op in OPS:
        for dt in list(KIND) + NON_REDUCIBLE + ["MPI_DATATYPE_NULL"]:
            assert L.msx_op_check(h(op), h(dt)) == oracle.op_check(h(op), h(dt)), (op, dt)
    for bad in (C.MPI_REPLACE, C.MPI_NO_OP, C.MPI_OP_NULL, 0x12345678, C.MPI_FLOAT):
        assert L.msx_op_check(bad, C.MPI_INT) == C.MPI_ERR_OP


def test_reduce_local_validation_order(msxlib):
    L = msxlib
    a = np.arange(8, dtype=np.int32)
    b = np.ones(8, dtype=np.int32)
    pa, pb = a.ctypes.data, b.ctypes.data
    IN_PLACE = ctypes.c_void_p(-1 & 0xFFFFFFFFFFFFFFFF).value
    # count == 0 returns success before any check (:319-322), even with bad op/type
    assert L.MPI_Reduce_local(None, None, 0, 0x1234, 0x42) == 0
    # op checked first (:324)
    assert L.MPI_Reduce_local(None, None, 5, C.MPI_INT, C.MPI_OP_NULL) == C.MPI_ERR_OP
    assert L.MPI_Reduce_local(pa, pb, 5, C.MPI_BYTE, C.MPI_SUM) == C.MPI_ERR_OP
    assert L.MPI_Reduce_local(pa, pb, -1, C.MPI_BYTE, C.MPI_SUM) == C.MPI_ERR_OP
    assert L.MPI_Reduce_local(pa, pb, 5, C.MPI_INT, C.MPI_REPLACE) == C.MPI_ERR_OP
    assert L.MPI_Reduce_local(pa, pb, 5, C.MPI_INT, C.MPI_NO_OP) == C.MPI_ERR_OP
    assert L.MPI_Reduce_local(pa, pb, 5, C.MPI_DATATYPE_NULL, C.MPI_SUM) == C.MPI_ERR_OP
    # then IN_PLACE on either side (:331-341)
    assert L.MPI_Reduce_local(IN_PLACE, pb, 5, C.MPI_INT, C.MPI_SUM) == C.MPI_ERR_BUFFER
    assert L.MPI_Reduce_local(pa, IN_PLACE, 5, C.MPI_INT, C.MPI_SUM) == C.MPI_ERR_BUFFER
    # then count / null buffer (:343, mpi_api.h:113-169)
    assert L.MPI_Reduce_local(pa, pb, -3, C.MPI_INT, C.MPI_SUM) == C.MPI_ERR_COUNT
    assert L.MPI_Reduce_local(None, pb, 5, C.MPI_INT, C.MPI_SUM) == C.MPI_ERR_BUFFER
    # then aliasing (:349-358)
    assert L.MPI_Reduce_local(pb, pb, 5, C.MPI_INT, C.MPI_SUM) == C.MPI_ERR_BUFFER
    assert (b == 1).all()


def test_user_ops_and_commutativity(msxlib):
    L = msxlib
    c = ctypes.c_int(-1)
    for op in OPS:
        assert L.MPI_Op_commutative(h(op), ctypes.byref(c)) == 0 and c.value == 1
    assert L.MPI_Op_commutative(C.MPI_REPLACE, ctypes.byref(c)) == 0 and c.value == 0
    UF = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                          ctypes.POINTER(ctypes.c_int))

    def sub(invec, inoutvec, n, dt):      # inout = in - inout (non-commutative)
        x = np.ctypeslib.as_array((ctypes.c_int * n[0]).from_address(invec))
        y = np.ctypeslib.as_array((ctypes.c_int * n[0]).from_address(inoutvec))
        y[:] = x - y

    fn = UF(sub)
    op = ctypes.c_int(0)
    assert L.MPI_Op_create(fn, 0, ctypes.byref(op)) == 0
    assert L.MPI_Op_commutative(op.value, ctypes.byref(c)) == 0 and c.value == 0
    a = np.arange(6, dtype=np.int32)
    b = np.full(6, 10, dtype=np.int32)
    # user functions are host code: host buffers call it directly, no GPU needed
    assert L.MPI_Reduce_local(a.ctypes.data, b.ctypes.data, 6, C.MPI_INT, op.value) == 0
    assert b.tolist() == [-10, -9, -8, -7, -6, -5]
    # freeing a builtin is an error ("**permop", mpi_op.cpp:169-173)
    perm = ctypes.c_int(C.MPI_SUM)
    assert L.MPI_Op_free(ctypes.byref(perm)) == C.MPI_ERR_OP
    assert L.MPI_Op_free(ctypes.byref(op)) == 0 and op.value == C.MPI_OP_NULL
    assert L.MPI_Op_free(ctypes.byref(op)) == C.MPI_ERR_OP


def test_no_gpu_fails_loudly_not_silently(msxlib):
    if msxlib.msx_device_count() > 0:
        pytest.skip("GPU present")
    a = np.arange(8, dtype=np.float32)
    b = np.ones(8, dtype=np.float32)
    rc = msxlib.MPI_Reduce_local(a.ctypes.data, b.ctypes.data, 8, C.MPI_FLOAT, C.MPI_SUM)
    assert rc == C.MPI_ERR_OTHER and "no usable MI355X" in msx.last_error()
    assert (b == 1).all()    # nothing computed on the CPU
    assert msxlib.msx_reduce_local_dev(a.ctypes.data, b.ctypes.data, 8, C.MPI_FLOAT, C.MPI_SUM,
                                       None) == C.MPI_ERR_OTHER


def test_config1_cpu_plumbing_and_oracle(msxlib):
    """BASELINE configs[0] ("MPI_Reduce_local MPI_SUM MPI_INT, 1 MiB, single
    process on CPU: plumbing + bit-exact oracle, no GPU").  Plumbing: MPI_Init,
    the reference's checks and the (op, type) table pass for the 1 MiB call,
    which then reaches the device dispatch and, with no GPU, returns
    MPI_ERR_OTHER without touching inoutbuf -- the product has no CPU combine.
    Oracle: the C restatement of Op<int>::Sum (op.cpp:42-52) on the same
    1 MiB equals two's-complement wrap arithmetic bit for bit (the survey's
    recorded int32 SUM answer over 1 MiB is test_oracle's known-answer case).
    On the GPU box the same call runs through the product: test_gpu_local's
    examples/reduce_local_demo.c test."""
    n = (1 << 20) // 4
    rng = np.random.default_rng(20)
    a = rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)
    b0 = rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)
    b = b0.copy()
    assert msxlib.msx_op_check(C.MPI_SUM, C.MPI_INT) == 0
    if msxlib.msx_device_count() == 0:
        rc = msxlib.MPI_Reduce_local(a.ctypes.data, b.ctypes.data, n, C.MPI_INT, C.MPI_SUM)
        assert rc == C.MPI_ERR_OTHER and "no usable MI355X" in msx.last_error()
        assert np.array_equal(b, b0)
    want = ((a.astype(np.int64) + b0.astype(np.int64) + 2**31) % 2**32 - 2**31).astype(np.int32)
    got = b0.copy()
    assert oracle.reduce_local(C.MPI_SUM, C.MPI_INT, a, got) == 0
    assert np.array_equal(got, want)


def test_op_table_entries_without_gpu(msxlib):
    """msx_op_table / msx_op_<op> (the MPIR_Op_table replacement, op.cpp:618-622,
    703-1923): lookups, the MPI_User_function shape, op_errno semantics
    (illegal pair -> MPI_ERR_OP with inout untouched, op.cpp:1791; len <= 0 does
    nothing), and on a GPU-less host a loud MPI_ERR_OTHER instead of a CPU result."""
    L = msxlib
    UF = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                          ctypes.POINTER(ctypes.c_int))
    L.msx_op_table.restype = ctypes.c_void_p
    L.msx_op_table.argtypes = [ctypes.c_int]
    names = ["max", "min", "sum", "prod", "land", "band", "lor", "bor", "lxor", "bxor", "minloc", "maxloc",
             "replace", "noop"]
    for k, nm in enumerate(names):
        assert L.msx_op_table(0x58000001 + k) == ctypes.cast(getattr(L, "msx_op_" + nm), ctypes.c_void_p).value, nm
    for bad in (C.MPI_OP_NULL, 0x5800000F, 0x58000000, 0x58000103, C.MPI_FLOAT):
        assert L.msx_op_table(bad) is None, hex(bad)
    L.msx_op_errno.restype = ctypes.c_int
    a = np.arange(8, dtype=np.uint8)
    b = np.full(8, 5, dtype=np.uint8)
    n, dt = ctypes.c_int(8), ctypes.c_int(C.MPI_BYTE)
    fsum = UF(L.msx_op_table(C.MPI_SUM))
    L.msx_op_errno_reset()
    fsum(a.ctypes.data, b.ctypes.data, ctypes.byref(n), ctypes.byref(dt))     # SUM on MPI_BYTE
    assert L.msx_op_errno() == C.MPI_ERR_OP and (b == 5).all()
    L.msx_op_errno_reset()
    z = ctypes.c_int(0)
    fsum(a.ctypes.data, b.ctypes.data, ctypes.byref(z), ctypes.byref(ctypes.c_int(C.MPI_INT)))
    assert L.msx_op_errno() == 0 and (b == 5).all()
    # noop / replace (host memcpy, no GPU needed)
    fr = UF(L.msx_op_table(C.MPI_REPLACE))
    fr(a.ctypes.data, b.ctypes.data, ctypes.byref(n), ctypes.byref(dt))
    assert L.msx_op_errno() == 0 and (b == a).all()
    # the binding's routing test: host operands stay on the
    # reference's own loop, NULL is never "device"
    assert L.msx_operands_on_device(a.ctypes.data, b.ctypes.data) == 0
    assert L.msx_operands_on_device(None, b.ctypes.data) == 0
    if L.msx_device_count() == 0:
        x = np.ones(8, np.float32)
        y = np.full(8, 2, np.float32)
        fsum(x.ctypes.data, y.ctypes.data, ctypes.byref(n), ctypes.byref(ctypes.c_int(C.MPI_FLOAT)))
        assert L.msx_op_errno() == C.MPI_ERR_OTHER and (y == 2).all()
        assert "no usable MI355X" in msx.last_error()


class _Status(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_int * 2), ("MPI_SOURCE", ctypes.c_int), ("MPI_TAG", ctypes.c_int),
                ("MPI_ERROR", ctypes.c_int)]


def test_request_completion_semantics(msxlib):
    """MPI_Waitall/Testall/Waitany/Testany/Waitsome/Testsome/Request_free/
    Request_get_status as api/mpi_completion.cpp and api/mpi_request.cpp
    define them: REQUEST_NULL entries, MPI_UNDEFINED results, 1 request
    completed per *any call, MPI_ERR_IN_STATUS with MPI_ERR_PENDING for the
    entries after a bad handle, argument errors.  One-rank nonblocking
    collectives complete at the call (host buffers: no GPU involved)."""
    L = msxlib
    UNDEF, NULLREQ = -32766, C.MPI_REQUEST_NULL
    src = np.arange(4, dtype=np.int32)
    outs = []

    def start():
        out = np.zeros(4, np.int32)
        outs.append(out)
        r = ctypes.c_int()
        assert L.MPI_Iallreduce(src.ctypes.data, out.ctypes.data, 4, C.MPI_INT, C.MPI_SUM, C.MPI_COMM_WORLD,
                                ctypes.byref(r)) == 0
        return r.value

    IGN = ctypes.c_void_p(1)                  # MPI_STATUS(ES)_IGNORE
    reqs = (ctypes.c_int * 3)(start(), NULLREQ, start())
    sts = (_Status * 3)()
    assert L.MPI_Waitall(3, reqs, sts) == 0
    assert list(reqs) == [NULLREQ] * 3
    assert (sts[1].MPI_SOURCE, sts[1].MPI_TAG, sts[1].MPI_ERROR) == (-2, -1, 0)
    assert all((o == src).all() for o in outs)
    # a bad handle: MPI_ERR_IN_STATUS, later entries MPI_ERR_PENDING and untouched
    reqs = (ctypes.c_int * 3)(start(), 0x2C00FFF0, start())
    live = reqs[2]
    assert L.MPI_Waitall(3, reqs, sts) == C.MPI_ERR_IN_STATUS
    assert reqs[0] == NULLREQ and sts[0].MPI_ERROR == 0
    assert sts[1].MPI_ERROR == C.MPI_ERR_REQUEST and sts[2].MPI_ERROR == 18 and reqs[2] == live
    r = ctypes.c_int(live)
    assert L.MPI_Wait(ctypes.byref(r), IGN) == 0 and r.value == NULLREQ
    # Testall: flag and all handles released
    reqs = (ctypes.c_int * 2)(start(), start())
    flag = ctypes.c_int(-1)
    assert L.MPI_Testall(2, reqs, ctypes.byref(flag), IGN) == 0 and flag.value == 1
    assert list(reqs) == [NULLREQ] * 2
    # Testany / Waitany: one request per call, MPI_UNDEFINED when none is active
    reqs = (ctypes.c_int * 3)(NULLREQ, start(), start())
    idx, st = ctypes.c_int(-1), _Status()
    assert L.MPI_Testany(3, reqs, ctypes.byref(idx), ctypes.byref(flag), ctypes.byref(st)) == 0
    assert (idx.value, flag.value, reqs[1]) == (1, 1, NULLREQ) and reqs[2] != NULLREQ
    assert L.MPI_Waitany(3, reqs, ctypes.byref(idx), ctypes.byref(st)) == 0 and idx.value == 2
    assert L.MPI_Waitany(3, reqs, ctypes.byref(idx), ctypes.byref(st)) == 0 and idx.value == UNDEF
    assert (st.MPI_SOURCE, st.MPI_TAG, st.MPI_ERROR) == (-2, -1, 0)
    assert L.MPI_Testany(3, reqs, ctypes.byref(idx), ctypes.byref(flag), ctypes.byref(st)) == 0
    assert (idx.value, flag.value) == (UNDEF, 1)
    # Testsome / Waitsome: every completed request, outcount MPI_UNDEFINED when none active
    reqs = (ctypes.c_int * 3)(start(), NULLREQ, start())
    n, ind = ctypes.c_int(-1), (ctypes.c_int * 3)()
    assert L.MPI_Testsome(3, reqs, ctypes.byref(n), ind, IGN) == 0
    assert n.value == 2 and list(ind)[:2] == [0, 2] and list(reqs) == [NULLREQ] * 3
    assert L.MPI_Waitsome(3, reqs, ctypes.byref(n), ind, IGN) == 0 and n.value == UNDEF
    reqs[0] = start()
    assert L.MPI_Waitsome(3, reqs, ctypes.byref(n), ind, sts) == 0 and n.value == 1 and ind[0] == 0
    # Request_get_status is non-destructive; Request_free refuses an NBC request
    r = ctypes.c_int(start())
    h0 = r.value
    assert L.MPI_Request_get_status(r.value, ctypes.byref(flag), ctypes.byref(st)) == 0
    assert flag.value == 1 and r.value == h0
    assert L.MPI_Request_free(ctypes.byref(r)) == C.MPI_ERR_OTHER and r.value == h0
    assert L.MPI_Test(ctypes.byref(r), ctypes.byref(flag), IGN) == 0 and r.value == NULLREQ
    assert L.MPI_Request_get_status(NULLREQ, ctypes.byref(flag), ctypes.byref(st)) == 0 and flag.value == 1
    assert L.MPI_Request_get_status(h0, ctypes.byref(flag), ctypes.byref(st)) == C.MPI_ERR_REQUEST
    # argument errors
    assert L.MPI_Waitall(-1, reqs, sts) == C.MPI_ERR_COUNT
    assert L.MPI_Waitall(1, None, sts) == C.MPI_ERR_ARG
    assert L.MPI_Testall(1, reqs, None, sts) == C.MPI_ERR_ARG
    assert L.MPI_Waitany(1, reqs, None, ctypes.byref(st)) == C.MPI_ERR_ARG
    assert L.MPI_Testsome(1, reqs, None, ind, sts) == C.MPI_ERR_ARG
    assert L.MPI_Request_free(None) == C.MPI_ERR_ARG
    bad = (ctypes.c_int * 1)(0x2C00FFF0)
    assert L.MPI_Testany(1, bad, ctypes.byref(idx), ctypes.byref(flag), ctypes.byref(st)) == C.MPI_ERR_REQUEST


def _run_py(code, env=None):
    e = dict(os.environ)
    e.update(env or {})
    pre = f"import sys; sys.path.insert(0, {os.path.join(msx.REPO_ROOT, 'microsoft-mpi_amd')!r})\n"
    return subprocess.run([sys.executable, "-c", pre + textwrap.dedent(code)], capture_output=True,
                          text=True, env=e, timeout=120)


def test_errors_are_fatal_by_default_and_require_init():
    r = _run_py("""
        import msx
        L = msx.lib()
        L.MPI_Init(None, None)
        L.MPI_Reduce_local(None, None, 4, msx.C.MPI_BYTE, msx.C.MPI_SUM)
        print("not reached")
    """)
    assert r.returncode == C.MPI_ERR_OP and "not reached" not in r.stdout
    assert "Fatal error in MPI_Reduce_local" in r.stderr
    r = _run_py("""
        import msx
        msx.lib().MPI_Reduce_local(None, None, 4, msx.C.MPI_INT, msx.C.MPI_SUM)
        print("not reached")
    """)
    assert r.returncode != 0 and "before initializing" in r.stderr


def test_rma_window_validation(msxlib):
    """MPI_Win_create / MPI_Put / MPI_Accumulate argument checks in the order of
    api/mpi_win.cpp:96-170 and api/mpi_rma.cpp:640-735 (no GPU needed)."""
    L = msxlib
    buf = np.zeros(64, np.int32)
    win = ctypes.c_int()
    assert L.MPI_Win_create(buf.ctypes.data, -1, 4, C.MPI_INFO_NULL, C.MPI_COMM_WORLD, ctypes.byref(win)) == C.MPI_ERR_SIZE
    assert L.MPI_Win_create(buf.ctypes.data, 256, 0, C.MPI_INFO_NULL, C.MPI_COMM_WORLD, ctypes.byref(win)) == C.MPI_ERR_ARG
    assert L.MPI_Win_create(buf.ctypes.data, 256, 4, 0x1c000001, C.MPI_COMM_WORLD, ctypes.byref(win)) == C.MPI_ERR_INFO
    assert L.MPI_Win_create(buf.ctypes.data, 256, 4, C.MPI_INFO_NULL, C.MPI_COMM_NULL, ctypes.byref(win)) == C.MPI_ERR_COMM
    assert L.MPI_Win_create(buf.ctypes.data, 256, 4, C.MPI_INFO_NULL, C.MPI_COMM_WORLD, ctypes.byref(win)) == 0
    assert (win.value & 0xFC000000) == 0xA0000000
    eh = ctypes.c_int()
    assert L.MPI_Win_get_errhandler(win, ctypes.byref(eh)) == 0 and eh.value == C.MPI_ERRORS_ARE_FATAL
    assert L.MPI_Win_set_errhandler(win, C.MPI_ERRORS_RETURN) == 0
    src = np.arange(8, dtype=np.int32)
    I = C.MPI_INT
    # displacement, rank, MPI_PROC_NULL, zero count
    assert L.MPI_Put(src.ctypes.data, 8, I, 0, -1, 8, I, win) == C.MPI_ERR_DISP
    assert L.MPI_Put(src.ctypes.data, 8, I, 1, 0, 8, I, win) == C.MPI_ERR_RANK
    assert L.MPI_Put(src.ctypes.data, 8, I, C.MPI_PROC_NULL, 0, 8, I, win) == 0
    assert L.MPI_Put(src.ctypes.data, 0, I, 0, 0, 0, I, win) == 0
    assert L.MPI_Put(src.ctypes.data, -1, I, 0, 0, 8, I, win) == C.MPI_ERR_COUNT
    assert L.MPI_Put(src.ctypes.data, 8, I, 0, 0, 8, C.MPI_FLOAT, win) == C.MPI_ERR_TYPE
    # ops: NO_OP and user ops are not accumulate operations; REPLACE is
    assert L.MPI_Accumulate(src.ctypes.data, 8, I, 0, 0, 8, I, C.MPI_NO_OP, win) == C.MPI_ERR_OP
    assert L.MPI_Accumulate(src.ctypes.data, 8, I, 0, 0, 8, I, C.MPI_OP_NULL, win) == C.MPI_ERR_OP
    UF = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                          ctypes.POINTER(ctypes.c_int))
    fn = UF(lambda a, b, n, d: None)
    op = ctypes.c_int()
    assert L.MPI_Op_create(fn, 1, ctypes.byref(op)) == 0
    assert L.MPI_Accumulate(src.ctypes.data, 8, I, 0, 0, 8, I, op.value, win) == C.MPI_ERR_OP
    assert L.MPI_Op_free(ctypes.byref(op)) == 0
    assert L.MPI_Accumulate(src.ctypes.data, 8, I, C.MPI_PROC_NULL, 0, 8, I, C.MPI_REPLACE, win) == 0
    # a real transfer needs the GPU: without one it fails loudly
    if L.msx_device_count() == 0:
        assert L.MPI_Accumulate(src.ctypes.data, 8, I, 0, 0, 8, I, C.MPI_SUM, win) == C.MPI_ERR_OTHER
    assert L.MPI_Win_fence(0, win) == 0
    assert L.MPI_Win_free(ctypes.byref(win)) == 0 and win.value == C.MPI_WIN_NULL
    bad = ctypes.c_int(0xA0000000 | 77)
    assert L.MPI_Win_fence(0, bad) == C.MPI_ERR_WIN


def test_pscw_synchronisation_state(msxlib):
    """Post-start-complete-wait epoch rules on one rank (api/mpi_win.cpp:1331-1381,
    1487-1537, 1566-1613, 1769-1808; no GPU needed, no transfers): a second post or
    start inside an open epoch and complete without start are MPI_ERR_RMA_SYNC,
    wait / test without an exposure epoch succeed at once, an invalid group is
    MPI_ERR_GROUP, MPI_Win_get_group is the communicator's group, and a window
    with an open epoch cannot be freed."""
    L = msxlib
    buf = np.zeros(64, np.int32)
    win = ctypes.c_int()
    assert L.MPI_Win_create(buf.ctypes.data, 256, 4, C.MPI_INFO_NULL, C.MPI_COMM_WORLD, ctypes.byref(win)) == 0
    W = win.value
    assert L.MPI_Win_set_errhandler(W, C.MPI_ERRORS_RETURN) == 0
    wg, g2 = ctypes.c_int(), ctypes.c_int()
    assert L.MPI_Comm_group(C.MPI_COMM_WORLD, ctypes.byref(wg)) == 0
    assert L.MPI_Win_get_group(W, ctypes.byref(g2)) == 0
    res = ctypes.c_int()
    assert L.MPI_Group_compare(wg.value, g2.value, ctypes.byref(res)) == 0 and res.value == C.MPI_IDENT
    flag = ctypes.c_int(-1)
    assert L.MPI_Win_wait(W) == 0
    assert L.MPI_Win_test(W, ctypes.byref(flag)) == 0 and flag.value == 1
    assert L.MPI_Win_complete(W) == C.MPI_ERR_RMA_SYNC
    assert L.MPI_Win_post(C.MPI_GROUP_NULL, 0, W) == C.MPI_ERR_GROUP
    assert L.MPI_Win_start(0x48000077, 0, W) == C.MPI_ERR_GROUP
    # exposure and access to self
    assert L.MPI_Win_post(wg.value, C.MPI_MODE_NOPUT, W) == 0
    assert L.MPI_Win_post(wg.value, 0, W) == C.MPI_ERR_RMA_SYNC
    assert L.MPI_Win_start(wg.value, 0, W) == 0
    assert L.MPI_Win_start(wg.value, 0, W) == C.MPI_ERR_RMA_SYNC
    assert L.MPI_Win_free(ctypes.byref(win)) == C.MPI_ERR_RMA_SYNC
    assert L.MPI_Put(buf.ctypes.data, 0, C.MPI_INT, 0, 0, 0, C.MPI_INT, W) == 0
    assert L.MPI_Win_complete(W) == 0
    assert L.MPI_Win_test(W, ctypes.byref(flag)) == 0 and flag.value == 1
    assert L.MPI_Win_wait(W) == 0
    # the empty group: an epoch with nobody in it
    assert L.MPI_Win_post(C.MPI_GROUP_EMPTY, 0, W) == 0 and L.MPI_Win_wait(W) == 0
    assert L.MPI_Win_start(C.MPI_GROUP_EMPTY, C.MPI_MODE_NOCHECK, W) == 0 and L.MPI_Win_complete(W) == 0
    for g in (wg, g2):
        assert L.MPI_Group_free(ctypes.byref(g)) == 0
    assert L.MPI_Win_free(ctypes.byref(win)) == 0


def test_environment_queries_and_communicator_relations(msxlib):
    """MPI_Get_version (2.0, mpi.h:4070), MPI_Query_thread / MPI_Is_thread_main /
    MPI_Get_processor_name / MPI_Wtick (api/mpi_env.cpp), MPI_Comm_compare
    (api/mpi_comm.cpp:51-157), MPI_Comm_test_inter and MPI_Comm_create
    (api/mpi_comm.cpp:184-248) on one rank; no GPU needed."""
    L = msxlib
    v, sv = ctypes.c_int(), ctypes.c_int()
    assert L.MPI_Get_version(ctypes.byref(v), ctypes.byref(sv)) == 0 and (v.value, sv.value) == (2, 0)
    assert L.MPI_Get_version(None, ctypes.byref(sv)) == C.MPI_ERR_ARG
    lvl, flag = ctypes.c_int(-1), ctypes.c_int(-1)
    assert L.MPI_Query_thread(ctypes.byref(lvl)) == 0 and lvl.value in (C.MPI_THREAD_SINGLE, C.MPI_THREAD_MULTIPLE)
    assert L.MPI_Is_thread_main(ctypes.byref(flag)) == 0 and flag.value == 1
    import threading
    other = []
    th = threading.Thread(target=lambda: other.append((L.MPI_Is_thread_main(ctypes.byref(flag)), flag.value)))
    th.start(); th.join()
    assert other == [(0, 0)]
    name, n = ctypes.create_string_buffer(C.MPI_MAX_PROCESSOR_NAME), ctypes.c_int()
    assert L.MPI_Get_processor_name(name, ctypes.byref(n)) == 0
    import socket
    assert name.value.decode() == socket.gethostname()[:127] and n.value == len(name.value)
    L.MPI_Wtick.restype = ctypes.c_double
    assert 0 < L.MPI_Wtick() <= 1e-6
    res = ctypes.c_int(-1)
    W, S = C.MPI_COMM_WORLD, C.MPI_COMM_SELF
    assert L.MPI_Comm_compare(W, W, ctypes.byref(res)) == 0 and res.value == C.MPI_IDENT
    d = ctypes.c_int()
    assert L.MPI_Comm_dup(W, ctypes.byref(d)) == 0
    assert L.MPI_Comm_compare(W, d.value, ctypes.byref(res)) == 0 and res.value == C.MPI_CONGRUENT
    assert L.MPI_Comm_compare(W, S, ctypes.byref(res)) == 0 and res.value == C.MPI_CONGRUENT
    assert L.MPI_Comm_compare(W, C.MPI_COMM_NULL, ctypes.byref(res)) == C.MPI_ERR_COMM
    assert L.MPI_Comm_compare(W, W, None) == C.MPI_ERR_ARG
    assert L.MPI_Comm_test_inter(W, ctypes.byref(flag)) == 0 and flag.value == 0
    wg, nc = ctypes.c_int(), ctypes.c_int()
    assert L.MPI_Comm_group(W, ctypes.byref(wg)) == 0
    assert L.MPI_Comm_create(d.value, wg.value, ctypes.byref(nc)) == 0 and nc.value != C.MPI_COMM_NULL
    sz, rk = ctypes.c_int(), ctypes.c_int()
    L.MPI_Comm_size(nc.value, ctypes.byref(sz)); L.MPI_Comm_rank(nc.value, ctypes.byref(rk))
    assert (sz.value, rk.value) == (1, 0)
    assert L.MPI_Comm_compare(nc.value, W, ctypes.byref(res)) == 0 and res.value == C.MPI_CONGRUENT
    assert L.MPI_Comm_free(ctypes.byref(nc)) == 0
    assert L.MPI_Comm_create(W, C.MPI_GROUP_EMPTY, ctypes.byref(nc)) == 0 and nc.value == C.MPI_COMM_NULL
    assert L.MPI_Comm_create(W, C.MPI_GROUP_NULL, ctypes.byref(nc)) == C.MPI_ERR_GROUP
    assert L.MPI_Comm_create(C.MPI_COMM_NULL, wg.value, ctypes.byref(nc)) == C.MPI_ERR_COMM
    assert L.MPI_Group_free(ctypes.byref(wg)) == 0
    assert L.MPI_Comm_free(ctypes.byref(d)) == 0


def _build_c_demo(tmp_path):
    exe = str(tmp_path / "reduce_local_demo")
    libdir = os.path.join(msx.REPO_ROOT, "microsoft-mpi_amd", "lib")
    subprocess.run(["gcc", "-O2", "-Wall", "-Werror", "-I", os.path.join(msx.REPO_ROOT, "include"),
                    os.path.join(msx.REPO_ROOT, "examples", "reduce_local_demo.c"), "-L", libdir,
                    "-lmsmpi_mi355x", f"-Wl,-rpath,{libdir}", "-o", exe], check=True)
    return exe


def test_plain_c_program_builds_against_the_headers(tmp_path):
    """Link-level drop-in: a C MPI program compiles with gcc against include/mpi.h
    and links the library; without a GPU its first reduction aborts loudly with
    the MPI error class (MPI_ERR_OTHER), never a silent CPU result."""
    exe = _build_c_demo(tmp_path)
    if msx.lib().msx_device_count() > 0:
        pytest.skip("GPU present: covered by tests/test_gpu_local.py")
    r = subprocess.run([exe], capture_output=True, text=True, env={**os.environ, "MSX_SIZE": "1"})
    assert r.returncode == C.MPI_ERR_OTHER
    assert "no usable MI355X" in r.stderr


def test_collectives_demo_compiles_as_plain_c(tmp_path):
    """examples/collectives_demo.c (the whole API surface an MPI application of
    this path touches) compiles warning-free with gcc against include/mpi.h and
    links the library; it runs in tests/test_gpu_c_demo.py."""
    exe = str(tmp_path / "collectives_demo")
    libdir = os.path.join(msx.REPO_ROOT, "microsoft-mpi_amd", "lib")
    subprocess.run(["gcc", "-O2", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(msx.REPO_ROOT, "include"),
                    os.path.join(msx.REPO_ROOT, "examples", "collectives_demo.c"), "-L", libdir,
                    "-lmsmpi_mi355x", f"-Wl,-rpath,{libdir}", "-o", exe], check=True)
    assert os.path.exists(exe)


def test_alloc_mem_validation_without_gpu():
    """MPI_Alloc_mem / MPI_Free_mem argument checks (api/mpi_env.cpp:841-945):
    negative size -> MPI_ERR_ARG, null or foreign base -> MPI_ERR_BASE; the
    memory itself is plain host memory the caller can use."""
    import ctypes
    L = msx.init(errors_return=True)
    p = ctypes.c_void_p()
    assert L.MPI_Alloc_mem(-1, C.MPI_INFO_NULL, ctypes.byref(p)) == C.MPI_ERR_ARG
    assert L.MPI_Alloc_mem(64, C.MPI_INFO_NULL, None) == C.MPI_ERR_ARG
    assert L.MPI_Alloc_mem(4096, C.MPI_INFO_NULL, ctypes.byref(p)) == 0 and p.value
    buf = (ctypes.c_char * 4096).from_address(p.value)
    buf[:] = b"\x5a" * 4096
    assert bytes(buf[:4]) == b"ZZZZ"
    assert L.MPI_Free_mem(None) == C.MPI_ERR_BASE
    other = ctypes.create_string_buffer(16)
    assert L.MPI_Free_mem(ctypes.addressof(other)) == C.MPI_ERR_BASE
    assert L.MPI_Free_mem(p) == 0
    assert L.MPI_Free_mem(p) == C.MPI_ERR_BASE          # not twice


def test_library_was_built_from_these_sources(msxlib):
    """Build provenance: msx_version() carries the SHA-256 prefix of every
    library source and header at build time (microsoft-mpi_amd/Makefile), so
    a prebuilt libmsmpi_mi355x.so shipped with the tree must match it."""
    import glob
    import hashlib
    pkg = os.path.join(msx.REPO_ROOT, "microsoft-mpi_amd")
    files = sorted(glob.glob(os.path.join(pkg, "csrc", "*.hip")) + glob.glob(os.path.join(pkg, "csrc", "*.cpp")) +
                   glob.glob(os.path.join(pkg, "csrc", "*.h")), key=lambda f: os.path.relpath(f, pkg))
    files += [os.path.join(msx.REPO_ROOT, "include", "mpi.h"), os.path.join(msx.REPO_ROOT, "include", "msx.h")]
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    msxlib.msx_version.restype = ctypes.c_char_p
    v = msxlib.msx_version().decode()
    assert v.endswith("src=" + h.hexdigest()[:16]), (v, h.hexdigest()[:16])


def test_no_pageable_memory_reaches_hip_copies():
    """the wrong results of rounds 3-4 are best explained by
    256-byte holes in pageable host transfers (the test harness's; a
    hypothesis no run has reproduced).  The product keeps user bytes off HIP's
    pageable-copy path: every hipMemcpy* call in csrc/ is
    either inside xfer_sync's page-locked ring or marked as a device / page-
    locked copy (`xfer: device/pinned`); pageable sides go through xfer_sync."""
    import re
    csrc = os.path.join(msx.REPO_ROOT, "microsoft-mpi_amd", "csrc")
    unmarked = []
    for f in sorted(os.listdir(csrc)):
        if not f.endswith((".cpp", ".hip", ".h")):
            continue
        text = open(os.path.join(csrc, f)).read()
        for m in re.finditer(r"\bhipMemcpy\w*\s*\(", text):
            line_start = text.rfind("\n", 0, m.start()) + 1
            if text[line_start:m.start()].lstrip().startswith("//"):
                continue                                  # a comment mentioning it
            end = text.find(";", m.end())
            stmt_end = text.find("\n", end)
            stmt = text[m.start():stmt_end if stmt_end >= 0 else len(text)]
            if "xfer: device/pinned" not in stmt:
                unmarked.append(f"{f}:{text.count(chr(10), 0, m.start()) + 1}")
    assert not unmarked, unmarked


def test_measurement_code_stays_out_of_the_product_library():
    """VERDICT r05 'Next' 4: the HBM probes and the combine / tree tuning
    variants live in the bench-only libmsx_probe.so; the product library holds
    the default geometries only (no probe or tuning kernel symbols, no tuning
    exports) and never loads the probe library."""
    so = os.path.join(msx.REPO_ROOT, "microsoft-mpi_amd", "lib", "libmsmpi_mi355x.so")
    blob = open(so, "rb").read()
    for name in (b"k_probe", b"k_combine_rr", b"k_combine_kt", b"k_combine_lds", b"msx_tune_set",
                 b"msx_tune_tree", b"msx_probe_hbm", b"libmsx_probe"):
        assert name not in blob, name
    L = msx.lib()
    for sym in ("msx_tune_set", "msx_tune_tree", "msx_tune_shift", "msx_probe_hbm", "msx_probe_alloc"):
        assert not hasattr(L, sym), sym
    csrc = os.path.join(msx.REPO_ROOT, "microsoft-mpi_amd", "csrc")
    for f in os.listdir(csrc):
        assert "dlopen(\"libmsx_probe" not in open(os.path.join(csrc, f), errors="replace").read(), f


# The environment the product reads (VERDICT r05 'Next' 3): launcher, tuning
# and diagnostics variables documented in INTEGRATION.md section 1, and test
# hooks under one MSX_TEST_ prefix.  A new getenv needs a line here and there.
PRODUCT_ENV = {"MSX_SIZE", "MSX_RANK", "MSX_DEVICE", "MSX_BOOTSTRAP_ADDR", "MSX_BOOTSTRAP_PORT",
               "MSX_BOOTSTRAP_TIMEOUT", "MSX_TRANSPORT", "MSX_CHUNK_BYTES", "MSX_TWO_STEP_MAX", "MSX_RMA_BYTES",
               "MSX_REDUCE_LOCAL_GPUS", "MSX_FLAG_TIMEOUT_MS", "MSX_STUCK_REPORT_S", "MSX_STUCK_SYNC_S",
               "MSX_TRACE", "MSX_TRACE_RANGES"}


def test_every_environment_variable_is_documented_or_a_test_hook():
    import re
    csrc = os.path.join(msx.REPO_ROOT, "microsoft-mpi_amd", "csrc")
    seen = set()
    for f in os.listdir(csrc):
        seen |= set(re.findall(r'getenv\("(MSX_[A-Z0-9_]+)"\)', open(os.path.join(csrc, f)).read()))
    unknown = sorted(v for v in seen if v not in PRODUCT_ENV and not v.startswith("MSX_TEST_"))
    assert not unknown, unknown
    doc = open(os.path.join(msx.REPO_ROOT, "INTEGRATION.md")).read()
    undocumented = sorted(v for v in seen if v not in doc)
    assert not undocumented, undocumented
