! Fortran bindings without a GPU: environment, datatype engine queries,
! user ops (run on host), validation through the Fortran sentinels.
! Prints KEY value lines that tests/test_fortran_cpu.py checks.
subroutine uadd(invec, inoutvec, n, dtype)
  implicit none
  integer n, dtype, i
  integer invec(n), inoutvec(n)
  integer seen_len, seen_type
  common /useen/ seen_len, seen_type
  seen_len = n
  seen_type = dtype
  do i = 1, n
    inoutvec(i) = inoutvec(i) + invec(i)
  end do
end subroutine

program fcpu
  implicit none
  include 'mpif.h'
  integer ierr, rank, nprocs, dt, dt2, dt3, dt4, sz, op, op2, i, cls, rlen
  integer ni, na, nd, comb, ints(8), types(4), blens(2), fdispls(2), ftypes(2)
  integer sizes(3), subsizes(3), starts(3), a1i, a3i
  integer(kind=MPI_ADDRESS_KIND) lb, ext, a1, a3, addrs(4)
  integer(kind=MPI_COUNT_KIND) szx
  integer a(10), b(10), c(10)
  integer reqs(3), idx, nout, idxs(3), st(MPI_STATUS_SIZE)
  logical flag, comm
  integer wg, g1, g2, g3, ranges(3, 2), tin(2), tout(2), gres, win
  integer(kind=MPI_ADDRESS_KIND) wsize
  integer ver, subver, newc
  character(len=MPI_MAX_PROCESSOR_NAME) pname
  double precision t
  character(len=600) msg
  integer seen_len, seen_type
  common /useen/ seen_len, seen_type
  external uadd

  call MPI_INIT(ierr)
  print '(A,I0)', 'INIT ', ierr
  call MPI_INITIALIZED(flag, ierr)
  print '(A,L1)', 'INITIALIZED ', flag
  call MPI_COMM_RANK(MPI_COMM_WORLD, rank, ierr)
  call MPI_COMM_SIZE(MPI_COMM_WORLD, nprocs, ierr)
  print '(A,I0,1X,I0)', 'RANK_SIZE ', rank, nprocs
  call MPI_COMM_SET_ERRHANDLER(MPI_COMM_WORLD, MPI_ERRORS_RETURN, ierr)

  ! vector(3, 2, 5) of DOUBLE PRECISION
  call MPI_TYPE_VECTOR(3, 2, 5, MPI_DOUBLE_PRECISION, dt, ierr)
  call MPI_TYPE_COMMIT(dt, ierr)
  call MPI_TYPE_SIZE(dt, sz, ierr)
  call MPI_TYPE_GET_EXTENT(dt, lb, ext, ierr)
  print '(A,I0,1X,I0,1X,I0)', 'VECTOR ', sz, lb, ext
  call MPI_TYPE_SIZE_X(dt, szx, ierr)
  print '(A,I0)', 'VECTOR_SIZE_X ', szx
  call MPI_TYPE_GET_ENVELOPE(dt, ni, na, nd, comb, ierr)
  print '(A,4(I0,1X))', 'ENVELOPE ', ni, na, nd, comb
  call MPI_TYPE_GET_CONTENTS(dt, 8, 4, 4, ints, addrs, types, ierr)
  print '(A,3(I0,1X),I0)', 'CONTENTS ', ints(1), ints(2), ints(3), types(1)
  call MPI_TYPE_FREE(types(1), ierr)

  ! MPI-1 forms: default-INTEGER byte stride / displacements
  call MPI_TYPE_HVECTOR(2, 1, 24, MPI_INTEGER, dt2, ierr)
  call MPI_TYPE_GET_EXTENT(dt2, lb, ext, ierr)
  call MPI_TYPE_GET_ENVELOPE(dt2, ni, na, nd, comb, ierr)
  print '(A,I0,1X,I0)', 'HVECTOR ', ext, comb
  blens = (/ 1, 1 /)
  fdispls = (/ 0, 8 /)
  ftypes = (/ MPI_INTEGER, MPI_DOUBLE_PRECISION /)
  call MPI_TYPE_STRUCT(2, blens, fdispls, ftypes, dt3, ierr)
  call MPI_TYPE_SIZE(dt3, sz, ierr)
  call MPI_TYPE_GET_EXTENT(dt3, lb, ext, ierr)
  call MPI_TYPE_EXTENT(dt3, i, ierr)
  print '(A,I0,1X,I0,1X,I0)', 'STRUCT ', sz, ext, i

  ! Fortran-order 3-D subarray of REAL
  sizes = (/ 6, 5, 4 /)
  subsizes = (/ 2, 3, 2 /)
  starts = (/ 1, 2, 1 /)
  call MPI_TYPE_CREATE_SUBARRAY(3, sizes, subsizes, starts, MPI_ORDER_FORTRAN, MPI_REAL, dt4, ierr)
  call MPI_TYPE_COMMIT(dt4, ierr)
  call MPI_TYPE_SIZE(dt4, sz, ierr)
  call MPI_TYPE_GET_EXTENT(dt4, lb, ext, ierr)
  call MPI_TYPE_GET_TRUE_EXTENT(dt4, a1, a3, ierr)
  print '(A,I0,1X,I0,1X,I0,1X,I0,1X,I0)', 'SUBARRAY ', sz, lb, ext, a1, a3

  ! addresses relative to MPI_BOTTOM
  call MPI_GET_ADDRESS(a(1), a1, ierr)
  call MPI_GET_ADDRESS(a(3), a3, ierr)
  call MPI_ADDRESS(a(1), a1i, ierr)
  call MPI_ADDRESS(a(3), a3i, ierr)
  print '(A,I0,1X,I0)', 'ADDRESS_DIFF ', a3 - a1, a3i - a1i

  ! user ops
  call MPI_OP_CREATE(uadd, .true., op, ierr)
  call MPI_OP_COMMUTATIVE(op, comm, ierr)
  print '(A,I0,1X,L1)', 'OP_CREATE ', ierr, comm
  call MPI_OP_CREATE(uadd, .false., op2, ierr)
  call MPI_OP_COMMUTATIVE(op2, comm, ierr)
  print '(A,L1)', 'OP2_COMMUTATIVE ', comm
  do i = 1, 10
    a(i) = i * 7
    b(i) = 1000 - i
    c(i) = a(i) + b(i)
  end do
  seen_len = -1
  seen_type = -1
  call MPI_REDUCE_LOCAL(a, b, 10, MPI_INTEGER, op, ierr)
  print '(A,I0,1X,L1,1X,I0,1X,L1)', 'USER_REDUCE_LOCAL ', ierr, all(b == c), seen_len, seen_type == MPI_INTEGER

  ! the Fortran MPI_IN_PLACE is recognised: the reference's Reduce_local
  ! rejects it as inbuf (MPI_ERR_BUFFER) -- a plain buffer would pass
  call MPI_REDUCE_LOCAL(MPI_IN_PLACE, b, 10, MPI_INTEGER, op, ierr)
  call MPI_ERROR_CLASS(ierr, cls, i)
  print '(A,I0)', 'IN_PLACE_CLASS ', cls
  ! illegal (op, type) pair: MPI_ERR_OP at validation, before any device work
  call MPI_REDUCE_LOCAL(a, b, 10, MPI_DOUBLE_PRECISION, MPI_BAND, ierr)
  call MPI_ERROR_CLASS(ierr, cls, i)
  print '(A,I0)', 'BAND_DOUBLE_CLASS ', cls
  ! count 0 succeeds before op validation
  call MPI_REDUCE_LOCAL(a, b, 0, MPI_DOUBLE_PRECISION, MPI_BAND, ierr)
  print '(A,I0)', 'COUNT0 ', ierr

  ! request completion (mpif.cpp:186-263): one-rank nonblocking calls complete
  ! at the call; indices come back 1-based, MPI_UNDEFINED stays as is
  call MPI_IALLREDUCE(a, c, 10, MPI_INTEGER, MPI_SUM, MPI_COMM_WORLD, reqs(1), ierr)
  reqs(2) = MPI_REQUEST_NULL
  call MPI_IALLREDUCE(a, c, 10, MPI_INTEGER, MPI_SUM, MPI_COMM_WORLD, reqs(3), ierr)
  call MPI_WAITANY(3, reqs, idx, st, ierr)
  print '(A,I0,1X,I0)', 'WAITANY ', ierr, idx
  call MPI_TESTANY(3, reqs, idx, flag, st, ierr)
  print '(A,I0,1X,I0,1X,L1)', 'TESTANY ', ierr, idx, flag
  call MPI_TESTANY(3, reqs, idx, flag, st, ierr)
  print '(A,I0,1X,L1)', 'TESTANY_NONE ', idx, flag
  call MPI_IALLREDUCE(a, c, 10, MPI_INTEGER, MPI_SUM, MPI_COMM_WORLD, reqs(2), ierr)
  call MPI_TESTALL(3, reqs, flag, MPI_STATUSES_IGNORE, ierr)
  print '(A,I0,1X,L1,1X,L1)', 'TESTALL ', ierr, flag, reqs(2) == MPI_REQUEST_NULL
  call MPI_IALLREDUCE(a, c, 10, MPI_INTEGER, MPI_SUM, MPI_COMM_WORLD, reqs(3), ierr)
  call MPI_WAITSOME(3, reqs, nout, idxs, MPI_STATUSES_IGNORE, ierr)
  print '(A,I0,1X,I0,1X,I0)', 'WAITSOME ', ierr, nout, idxs(1)
  call MPI_IALLREDUCE(a, c, 10, MPI_INTEGER, MPI_SUM, MPI_COMM_WORLD, reqs(1), ierr)
  call MPI_REQUEST_GET_STATUS(reqs(1), flag, st, ierr)
  print '(A,I0,1X,L1,1X,L1)', 'GET_STATUS ', ierr, flag, reqs(1) /= MPI_REQUEST_NULL
  call MPI_REQUEST_FREE(reqs(1), ierr)
  call MPI_ERROR_CLASS(ierr, cls, i)
  print '(A,I0)', 'REQUEST_FREE_CLASS ', cls
  call MPI_TESTSOME(3, reqs, nout, idxs, MPI_STATUSES_IGNORE, ierr)
  print '(A,I0,1X,I0,1X,I0)', 'TESTSOME ', ierr, nout, idxs(1)
  call MPI_TESTSOME(3, reqs, nout, idxs, MPI_STATUSES_IGNORE, ierr)
  print '(A,I0)', 'TESTSOME_NONE ', nout

  ! groups (one process): range (0, 0, 1) twice is a duplicate (MPI_ERR_ARG)
  call MPI_COMM_GROUP(MPI_COMM_WORLD, wg, ierr)
  call MPI_GROUP_SIZE(wg, sz, ierr)
  call MPI_GROUP_RANK(wg, i, ierr)
  print '(A,I0,1X,I0,1X,I0)', 'GROUP ', ierr, sz, i
  ranges(:, 1) = (/ 0, 0, 1 /)
  call MPI_GROUP_RANGE_INCL(wg, 1, ranges, g1, ierr)
  call MPI_GROUP_COMPARE(g1, wg, gres, ierr)
  print '(A,I0,1X,L1)', 'RANGE_INCL ', ierr, gres == MPI_IDENT
  ranges(:, 2) = (/ 0, 0, 1 /)
  call MPI_GROUP_RANGE_INCL(wg, 2, ranges, g3, ierr)
  call MPI_ERROR_CLASS(ierr, cls, i)
  print '(A,I0)', 'RANGE_DUP_CLASS ', cls
  call MPI_GROUP_EXCL(wg, 1, (/ 0 /), g2, ierr)
  call MPI_GROUP_SIZE(g2, sz, ierr)
  call MPI_GROUP_RANK(g2, i, ierr)
  print '(A,I0,1X,I0,1X,I0)', 'EXCL ', ierr, sz, i
  tin = (/ 0, MPI_PROC_NULL /)
  call MPI_GROUP_TRANSLATE_RANKS(wg, 2, tin, g2, tout, ierr)
  print '(A,I0,1X,I0,1X,I0)', 'TRANSLATE ', ierr, tout(1), tout(2)
  call MPI_GROUP_UNION(g2, wg, g3, ierr)
  call MPI_GROUP_COMPARE(g3, wg, gres, ierr)
  print '(A,L1)', 'UNION_IDENT ', gres == MPI_IDENT
  call MPI_GROUP_FREE(g3, ierr)
  call MPI_GROUP_INTERSECTION(g2, wg, g3, ierr)
  call MPI_GROUP_COMPARE(g3, MPI_GROUP_EMPTY, gres, ierr)
  print '(A,L1)', 'INTERSECTION_EMPTY ', gres == MPI_IDENT
  call MPI_GROUP_FREE(g3, ierr)
  call MPI_GROUP_DIFFERENCE(wg, g1, g3, ierr)
  call MPI_GROUP_SIZE(g3, sz, ierr)
  print '(A,I0)', 'DIFFERENCE ', sz
  call MPI_GROUP_FREE(g3, ierr)

  ! environment queries, communicator relations
  call MPI_GET_VERSION(ver, subver, ierr)
  call MPI_QUERY_THREAD(i, ierr)
  call MPI_IS_THREAD_MAIN(flag, ierr)
  print '(A,I0,1X,I0,1X,I0,1X,L1)', 'VERSION ', ver, subver, i, flag
  call MPI_GET_PROCESSOR_NAME(pname, rlen, ierr)
  print '(A,I0,1X,L1,1X,L1)', 'PROCNAME ', ierr, rlen > 0, len_trim(pname) == rlen
  print '(A,L1)', 'WTICK ', MPI_WTICK() > 0.0d0
  call MPI_COMM_CREATE(MPI_COMM_WORLD, wg, newc, ierr)
  call MPI_COMM_COMPARE(MPI_COMM_WORLD, newc, gres, ierr)
  call MPI_COMM_TEST_INTER(newc, flag, ierr)
  print '(A,I0,1X,L1,1X,L1)', 'COMM_CREATE ', ierr, gres == MPI_CONGRUENT, flag
  call MPI_COMM_FREE(newc, ierr)

  ! post-start-complete-wait on a one-rank window (no transfers)
  wsize = 40
  call MPI_WIN_CREATE(a, wsize, 4, MPI_INFO_NULL, MPI_COMM_WORLD, win, ierr)
  call MPI_WIN_SET_ERRHANDLER(win, MPI_ERRORS_RETURN, ierr)
  call MPI_WIN_GET_GROUP(win, g3, ierr)
  call MPI_GROUP_COMPARE(g3, wg, gres, ierr)
  call MPI_WIN_POST(wg, 0, win, ierr)
  call MPI_WIN_START(wg, MPI_MODE_NOCHECK, win, ierr)
  call MPI_WIN_COMPLETE(win, ierr)
  call MPI_WIN_TEST(win, flag, ierr)
  print '(A,I0,1X,L1,1X,L1)', 'PSCW ', ierr, flag, gres == MPI_IDENT
  call MPI_WIN_COMPLETE(win, ierr)
  call MPI_ERROR_CLASS(ierr, cls, i)
  print '(A,I0)', 'COMPLETE_CLASS ', cls
  call MPI_WIN_WAIT(win, ierr)
  call MPI_WIN_FREE(win, ierr)
  call MPI_GROUP_FREE(g1, ierr)
  call MPI_GROUP_FREE(g2, ierr)
  call MPI_GROUP_FREE(g3, ierr)
  call MPI_GROUP_FREE(wg, ierr)
  print '(A,I0,1X,L1)', 'GROUP_FREE ', ierr, wg == MPI_GROUP_NULL

  msg = 'x'
  call MPI_ERROR_STRING(MPI_ERR_OP, msg, rlen, ierr)
  print '(A,I0,1X,L1,1X,L1)', 'ERROR_STRING ', ierr, rlen > 0, len_trim(msg) == rlen

  call MPI_PACK_SIZE(3, MPI_INTEGER, MPI_COMM_WORLD, sz, ierr)
  print '(A,I0)', 'PACK_SIZE ', sz
  t = MPI_WTIME()
  print '(A,L1)', 'WTIME ', t > 0.0d0

  call MPI_OP_FREE(op, ierr)
  call MPI_OP_FREE(op2, ierr)
  print '(A,L1)', 'OP_FREE ', op == MPI_OP_NULL
  call MPI_OP_FREE(MPI_SUM, ierr)
  call MPI_ERROR_CLASS(ierr, cls, i)
  print '(A,I0)', 'FREE_BUILTIN_CLASS ', cls
  call MPI_TYPE_FREE(dt, ierr)
  call MPI_TYPE_FREE(dt2, ierr)
  call MPI_TYPE_FREE(dt3, ierr)
  call MPI_TYPE_FREE(dt4, ierr)
  print '(A,L1)', 'TYPE_FREE ', dt == MPI_DATATYPE_NULL
  call MPI_FINALIZE(ierr)
  call MPI_FINALIZED(flag, ierr)
  print '(A,I0,1X,L1)', 'FINALIZE ', ierr, flag
end program
