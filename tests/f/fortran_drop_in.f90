! A Fortran caller written to the reference's Fortran interface (SRC/dsaupd.f:182,
! SRC/dseupd.f:218, SRC/dnaupd.f; the EXAMPLES/SIMPLE driver pattern), linked
! against libarpack_hip.so instead of libarpack.  Every argument by reference,
! CHARACTER lengths as the hidden trailing arguments of the gfortran/flang ABI.
!   1. dsaupd/dseupd: 1-D Laplacian tridiag(-1,2,-1), n = 200, the 4 largest
!      eigenvalues 2 - 2 cos(k pi/(n+1)) and their residuals;
!   2. dnaupd/dneupd: the non-normal upper bidiagonal diag(1..n) + c*superdiag,
!      whose eigenvalues are its diagonal: the 4 of largest magnitude n .. n-3.
! Exit status 0 on success (stop 1..8 name the failing check).
program fortran_drop_in
  implicit none
  integer, parameter :: n = 200, nev = 4, ncv = 20, ldv = n
  double precision, parameter :: pi = 3.14159265358979323846d0, conv = 0.3d0
  double precision :: v(ldv, ncv), workd(3*n), resid(n), ax(n), d(nev), z(ldv, nev)
  double precision :: workl(3*ncv*ncv + 6*ncv), dr(nev+1), di(nev+1), zn(ldv, nev+1)
  double precision :: workev(3*ncv), tol, sigma, sigmai, want, err, rmax
  logical :: sel(ncv), rvec
  integer :: iparam(11), ipntr(14), ido, info, ierr, j, k, lworkl
  character(len=1) :: bmat
  character(len=2) :: which

  ! ---------------------------------------------------------- dsaupd / dseupd
  bmat = 'I'
  which = 'LA'
  tol = 0d0
  lworkl = ncv*(ncv + 8)
  iparam = 0
  iparam(1) = 1
  iparam(3) = 300
  iparam(7) = 1
  ido = 0
  info = 0
  do
    call dsaupd(ido, bmat, n, which, nev, tol, resid, ncv, v, ldv, iparam, ipntr, &
                workd, workl, lworkl, info)
    if (ido /= -1 .and. ido /= 1) exit
    call lap(n, 0d0, workd(ipntr(1)), workd(ipntr(2)))
  end do
  if (info /= 0 .or. iparam(5) /= nev) then
    print *, 'dsaupd info', info, ' nconv', iparam(5), ' cycles', iparam(3)
    stop 1
  end if
  rvec = .true.
  call dseupd(rvec, 'A', sel, d, z, ldv, sigma, bmat, n, which, nev, tol, resid, ncv, v, &
              ldv, iparam, ipntr, workd, workl, lworkl, ierr)
  if (ierr /= 0) stop 2
  rmax = 0d0
  do j = 1, nev
    k = n - nev + j          ! d ascending: the 4 largest, smallest first
    want = 2d0 - 2d0*cos(k*pi/(n + 1))
    if (abs(d(j) - want) > 1d-10) stop 3
    call lap(n, 0d0, z(1, j), ax)
    err = sqrt(sum((ax - d(j)*z(:, j))**2))
    rmax = max(rmax, err)
  end do
  if (rmax > 1d-9) stop 4
  print '(a,i4,a,i6,a,es9.2)', 'dsaupd ok: cycles', iparam(3), '  OP*x', iparam(9), &
        '  max residual', rmax

  ! ---------------------------------------------------------- dnaupd / dneupd
  which = 'LM'
  tol = 0d0
  lworkl = 3*ncv*ncv + 6*ncv
  iparam = 0
  iparam(1) = 1
  iparam(3) = 300
  iparam(7) = 1
  ido = 0
  info = 0
  do
    call dnaupd(ido, bmat, n, which, nev, tol, resid, ncv, v, ldv, iparam, ipntr, &
                workd, workl, lworkl, info)
    if (ido /= -1 .and. ido /= 1) exit
    call bidiag(n, conv, workd(ipntr(1)), workd(ipntr(2)))
  end do
  if (info /= 0 .or. iparam(5) < nev) then
    print *, 'dnaupd info', info, ' nconv', iparam(5), ' cycles', iparam(3)
    stop 5
  end if
  sigma = 0d0
  sigmai = 0d0
  call dneupd(rvec, 'A', sel, dr, di, zn, ldv, sigma, sigmai, workev, bmat, n, which, nev, &
              tol, resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl, ierr)
  if (ierr /= 0) stop 6
  do j = 1, nev
    if (abs(di(j)) > 1d-8) stop 7
    err = 1d300
    do k = n - nev + 1, n
      err = min(err, abs(dr(j) - dble(k)))
    end do
    if (err > 1d-8*n) stop 8
  end do
  print '(a,i4,a,i6)', 'dnaupd ok: cycles', iparam(3), '  OP*x', iparam(9)
end program fortran_drop_in

! y = (diag(1..n) + c * superdiag) x
subroutine bidiag(n, c, x, y)
  implicit none
  integer, intent(in) :: n
  double precision, intent(in) :: c, x(n)
  double precision, intent(out) :: y(n)
  integer :: i
  do i = 1, n
    y(i) = dble(i)*x(i)
    if (i < n) y(i) = y(i) + c*x(i + 1)
  end do
end subroutine bidiag

! y = tridiag(-1-c, 2, -1+c) x
subroutine lap(n, c, x, y)
  implicit none
  integer, intent(in) :: n
  double precision, intent(in) :: c, x(n)
  double precision, intent(out) :: y(n)
  integer :: i
  do i = 1, n
    y(i) = 2d0*x(i)
    if (i > 1) y(i) = y(i) - (1d0 + c)*x(i - 1)
    if (i < n) y(i) = y(i) - (1d0 - c)*x(i + 1)
  end do
end subroutine lap
