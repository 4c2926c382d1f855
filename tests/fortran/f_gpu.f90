! Fortran bindings on the GPU path: host arrays from a Fortran program go
! through the HIP combine / collective / pack / RMA engines.  Run with 1..3
! ranks (MSX_SIZE / MSX_RANK); every expected value is computed here exactly
! (integer arithmetic, or one IEEE operation per element).  Prints
! "FRESULT rank nprocs nfail" and one FAIL line per failed check.
subroutine imax(invec, inoutvec, n, dtype)
  implicit none
  integer n, dtype, i
  integer invec(n), inoutvec(n)
  do i = 1, n
    inoutvec(i) = max(inoutvec(i), invec(i)) + 1
  end do
end subroutine

module chk
  implicit none
  integer :: nfail = 0
contains
  subroutine check(ok, tag)
    logical, intent(in) :: ok
    character(len=*), intent(in) :: tag
    if (.not. ok) then
      nfail = nfail + 1
      print '(A,A)', 'FAIL ', tag
    end if
  end subroutine
end module

program fgpu
  use chk
  implicit none
  include 'mpif.h'
  integer, parameter :: n = 100003, m = 4099
  integer ierr, rank, p, i, r, op, req, reqs(2), dt, pos, win, root, cls
  integer st(MPI_STATUS_SIZE)
  real, allocatable :: fa(:), fb(:), fexp(:)
  double precision, allocatable :: da(:), db(:), dexp(:)
  integer, allocatable :: ia(:), ib(:), iexp(:), ired(:), irs(:), isc(:), iwin(:), iacc(:)
  integer loc_a(2, 8), loc_b(2, 8), loc_e(2, 8)
  integer packed(64), vec(40), vout(40)
  integer(kind=MPI_ADDRESS_KIND) wsize, disp
  integer one, fetched
  logical flag
  external imax

  call MPI_INIT(ierr)
  call MPI_COMM_RANK(MPI_COMM_WORLD, rank, ierr)
  call MPI_COMM_SIZE(MPI_COMM_WORLD, p, ierr)
  call MPI_COMM_SET_ERRHANDLER(MPI_COMM_WORLD, MPI_ERRORS_RETURN, ierr)

  ! ---- MPI_REDUCE_LOCAL on host arrays (the HIP combine kernels) ----
  allocate(fa(n), fb(n), fexp(n), da(n), db(n), dexp(n), ia(n), ib(n), iexp(n))
  do i = 1, n
    fa(i) = real(mod(i * 37, 1009)) / 64.0 - 7.5
    fb(i) = real(mod(i * 11, 997)) / 32.0 + 0.25
    fexp(i) = fb(i) + fa(i)
    da(i) = dble(mod(i * 13, 1013)) - 500.5d0
    db(i) = dble(mod(i * 29, 1019)) - 510.25d0
    dexp(i) = max(db(i), da(i))
    ia(i) = i * 2654435 + 12345
    ib(i) = ieor(i * 40503, 987654321)
    iexp(i) = iand(ib(i), ia(i))
  end do
  call MPI_REDUCE_LOCAL(fa, fb, n, MPI_REAL, MPI_SUM, ierr)
  call check(ierr == 0 .and. all(fb == fexp), 'reduce_local SUM REAL')
  call MPI_REDUCE_LOCAL(da, db, n, MPI_DOUBLE_PRECISION, MPI_MAX, ierr)
  call check(ierr == 0 .and. all(db == dexp), 'reduce_local MAX DOUBLE PRECISION')
  call MPI_REDUCE_LOCAL(ia, ib, n, MPI_INTEGER, MPI_BAND, ierr)
  call check(ierr == 0 .and. all(ib == iexp), 'reduce_local BAND INTEGER')
  ! MAXLOC over 2INTEGER pairs (value, location); ties keep the smaller location
  do i = 1, 8
    loc_a(1, i) = mod(i * 5, 7)
    loc_a(2, i) = 100 + i
    loc_b(1, i) = mod(i * 3, 7)
    loc_b(2, i) = 200 - i
    if (loc_a(1, i) > loc_b(1, i)) then
      loc_e(:, i) = loc_a(:, i)
    else if (loc_a(1, i) < loc_b(1, i)) then
      loc_e(:, i) = loc_b(:, i)
    else
      loc_e(1, i) = loc_a(1, i)
      loc_e(2, i) = min(loc_a(2, i), loc_b(2, i))
    end if
  end do
  call MPI_REDUCE_LOCAL(loc_a, loc_b, 8, MPI_2INTEGER, MPI_MAXLOC, ierr)
  call check(ierr == 0 .and. all(loc_b == loc_e), 'reduce_local MAXLOC 2INTEGER')
  ! an illegal pair still fails at validation
  call MPI_REDUCE_LOCAL(da, db, n, MPI_DOUBLE_PRECISION, MPI_BXOR, ierr)
  call MPI_ERROR_CLASS(ierr, cls, i)
  call check(cls == MPI_ERR_OP, 'BXOR on DOUBLE PRECISION is MPI_ERR_OP')

  ! ---- MPI_PACK / MPI_UNPACK of vector(5, 3, 8) of INTEGER ----
  do i = 1, 40
    vec(i) = 1000 * rank + i
  end do
  call MPI_TYPE_VECTOR(5, 3, 8, MPI_INTEGER, dt, ierr)
  call MPI_TYPE_COMMIT(dt, ierr)
  pos = 0
  call MPI_PACK(vec, 1, dt, packed, 256, pos, MPI_COMM_WORLD, ierr)
  call check(ierr == 0 .and. pos == 60, 'pack position')
  flag = .true.
  do i = 0, 4
    do r = 1, 3
      flag = flag .and. packed(3 * i + r) == vec(8 * i + r)
    end do
  end do
  call check(flag, 'pack contents')
  vout = -1
  pos = 0
  call MPI_UNPACK(packed, 256, pos, vout, 1, dt, MPI_COMM_WORLD, ierr)
  flag = ierr == 0 .and. pos == 60
  do i = 1, 37
    if (mod(i - 1, 8) < 3) then
      flag = flag .and. vout(i) == vec(i)
    else
      flag = flag .and. vout(i) == -1
    end if
  end do
  call check(flag, 'unpack keeps the gaps')
  call MPI_TYPE_FREE(dt, ierr)

  ! ---- collectives over all ranks (integer data: exact under any order) ----
  allocate(ired(m), irs(m * p), isc(m), iwin(m), iacc(m))
  do i = 1, m
    ired(i) = rank * 100000 + i
  end do
  call MPI_ALLREDUCE(MPI_IN_PLACE, ired, m, MPI_INTEGER, MPI_SUM, MPI_COMM_WORLD, ierr)
  flag = ierr == 0
  do i = 1, m
    flag = flag .and. ired(i) == 100000 * (p * (p - 1) / 2) + p * i
  end do
  call check(flag, 'allreduce SUM in place')

  root = p - 1
  do i = 1, m
    isc(i) = rank + 3 * i
  end do
  iwin = -5
  call MPI_REDUCE(isc, iwin, m, MPI_INTEGER, MPI_MAX, root, MPI_COMM_WORLD, ierr)
  if (rank == root) then
    flag = ierr == 0
    do i = 1, m
      flag = flag .and. iwin(i) == p - 1 + 3 * i
    end do
    call check(flag, 'reduce MAX at root')
  end if

  do i = 1, m * p
    irs(i) = i + rank
  end do
  iacc = 0
  call MPI_REDUCE_SCATTER_BLOCK(irs, iacc, m, MPI_INTEGER, MPI_SUM, MPI_COMM_WORLD, ierr)
  flag = ierr == 0
  do i = 1, m
    flag = flag .and. iacc(i) == p * (rank * m + i) + p * (p - 1) / 2
  end do
  call check(flag, 'reduce_scatter_block SUM')

  do i = 1, m
    ired(i) = (rank + 1) * i
  end do
  call MPI_SCAN(ired, isc, m, MPI_INTEGER, MPI_SUM, MPI_COMM_WORLD, ierr)
  flag = ierr == 0
  do i = 1, m
    flag = flag .and. isc(i) == i * (rank + 1) * (rank + 2) / 2
  end do
  call check(flag, 'scan SUM')
  isc = -9
  call MPI_EXSCAN(ired, isc, m, MPI_INTEGER, MPI_SUM, MPI_COMM_WORLD, ierr)
  if (rank > 0) then
    flag = ierr == 0
    do i = 1, m
      flag = flag .and. isc(i) == i * rank * (rank + 1) / 2
    end do
    call check(flag, 'exscan SUM')
  end if

  ! non-blocking: Iallreduce + Wait(MPI_STATUS_IGNORE), Test loop, Waitall
  do i = 1, m
    ired(i) = ieor(i, rank * 7919)
  end do
  call MPI_IALLREDUCE(ired, isc, m, MPI_INTEGER, MPI_BXOR, MPI_COMM_WORLD, req, ierr)
  call MPI_WAIT(req, MPI_STATUS_IGNORE, ierr)
  flag = ierr == 0 .and. req == MPI_REQUEST_NULL
  do i = 1, m
    iexp(i) = 0
    do r = 0, p - 1
      iexp(i) = ieor(iexp(i), ieor(i, r * 7919))
    end do
    flag = flag .and. isc(i) == iexp(i)
  end do
  call check(flag, 'iallreduce BXOR + wait')
  call MPI_IALLREDUCE(ired, iwin, m, MPI_INTEGER, MPI_BXOR, MPI_COMM_WORLD, req, ierr)
  flag = .false.
  do while (.not. flag)
    call MPI_TEST(req, flag, st, ierr)
  end do
  call check(ierr == 0 .and. all(iwin(1:m) == iexp(1:m)), 'iallreduce + test loop')
  call MPI_IREDUCE(ired, iwin, m, MPI_INTEGER, MPI_BXOR, 0, MPI_COMM_WORLD, reqs(1), ierr)
  call MPI_ISCAN(ired, iacc, m, MPI_INTEGER, MPI_BOR, MPI_COMM_WORLD, reqs(2), ierr)
  call MPI_WAITALL(2, reqs, MPI_STATUSES_IGNORE, ierr)
  flag = ierr == 0
  if (rank == 0) flag = flag .and. all(iwin(1:m) == iexp(1:m))
  call check(flag, 'ireduce + iscan + waitall')

  ! a Fortran user op in a collective (commutative: max(a,b)+1 per step is
  ! not associative, so only the value at p <= 2 is closed-form)
  call MPI_OP_CREATE(imax, .true., op, ierr)
  do i = 1, m
    ired(i) = rank * 3 + i
  end do
  call MPI_ALLREDUCE(ired, isc, m, MPI_INTEGER, op, MPI_COMM_WORLD, ierr)
  if (p <= 2) then
    flag = ierr == 0
    do i = 1, m
      if (p == 1) then
        flag = flag .and. isc(i) == i
      else
        flag = flag .and. isc(i) == 3 + i + 1
      end if
    end do
    call check(flag, 'allreduce with a Fortran user op')
  else
    call check(ierr == 0, 'allreduce with a Fortran user op (p>2)')
  end if
  call MPI_OP_FREE(op, ierr)

  ! ---- one-sided accumulate into the next rank's window ----
  iwin = 10
  wsize = 4 * m
  call MPI_WIN_CREATE(iwin, wsize, 4, MPI_INFO_NULL, MPI_COMM_WORLD, win, ierr)
  call check(ierr == 0, 'win_create')
  call MPI_WIN_FENCE(0, win, ierr)
  do i = 1, m
    iacc(i) = rank * 1000 + i
  end do
  disp = 0
  call MPI_ACCUMULATE(iacc, m, MPI_INTEGER, mod(rank + 1, p), disp, m, MPI_INTEGER, MPI_SUM, win, ierr)
  call MPI_WIN_FENCE(0, win, ierr)
  r = mod(rank + p - 1, p)
  flag = ierr == 0
  do i = 1, m
    flag = flag .and. iwin(i) == 10 + r * 1000 + i
  end do
  call check(flag, 'accumulate SUM + fence')
  one = 1
  disp = 5
  call MPI_FETCH_AND_OP(one, fetched, MPI_INTEGER, 0, disp, MPI_SUM, win, ierr)
  call MPI_WIN_FENCE(0, win, ierr)
  call check(ierr == 0 .and. fetched >= 10, 'fetch_and_op')
  if (rank == 0) call check(iwin(6) == 10 + mod(p - 1, p) * 1000 + 6 + p, 'fetch_and_op total')
  call MPI_WIN_FREE(win, ierr)

  print '(A,I0,1X,I0,1X,I0)', 'FRESULT ', rank, p, nfail
  call MPI_FINALIZE(ierr)
end program
