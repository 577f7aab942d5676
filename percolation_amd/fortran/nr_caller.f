c     nr_caller.f -- a Fortran 77 caller of libperc's Numerical-Recipes
c     layer, written for the tests (tests/test_nr_symbols.py).  It calls
c     every NR entry point the reference programs embed
c     (Fortran/Square/bondc.f:723-917) exactly the way those programs do:
c     the matrix lives in COMMON /mat/ sa(NMAX), ija(NMAX) with NMAX =
c     20000 (bondc.f:59,753,845,859), arguments by reference, and the
c     routines are resolved at link time from libperc.so instead of the
c     copies each reference program carries.
c
c     Inputs (raw little-endian stream files written by the test):
c       dense.bin   n, np (int32), thresh (real*8), a(np,np) column-major
c       vec.bin     n (int32), x(n)
c       system.bin  n, k (int32), sa(1..k), ija(1..k), b(n), itol (int32),
c                   tol (real*8), itmax (int32)
c     Outputs:
c       sprsin.bin  status, k, sa(1..k), ija(1..k)
c       ops.bin     status, dsprsax, dsprstx, atimes(0), atimes(1),
c                   asolve, snrm(itol=1), snrm(itol=2), snrm(itol=4)
c       linbcg.bin  status, iter, err, x(n)
      program nrcall
      implicit none
      integer NMAX, NPMAX
      parameter (NMAX=20000, NPMAX=600)
      double precision sa(NMAX)
      integer ija(NMAX)
      common /mat/ sa, ija
      double precision a(NPMAX,NPMAX), thresh
      double precision x(NMAX), b(NMAX), r1(NMAX), r2(NMAX)
      double precision r3(NMAX), r4(NMAX), r5(NMAX), s1, s2, s4
      double precision tol, err, snrm
      integer n, np, k, i, j, nmx, itol, itmax, iter, st
      integer perc_nr_status
      external snrm, perc_nr_status

c     ---- sprsin: dense -> row-indexed storage (bondc.f:723-746)
      open(10, file='dense.bin', access='stream', form='unformatted',
     &     status='old')
      read(10) n, np, thresh
      read(10) ((a(i,j), i=1,np), j=1,np)
      close(10)
      nmx = NMAX
      call sprsin(a, n, NPMAX, thresh, nmx, sa, ija)
      st = perc_nr_status()
      k = ija(ija(1)-1) - 1
      open(11, file='sprsin.bin', access='stream', form='unformatted',
     &     status='replace')
      write(11) st, k
      write(11) (sa(i), i=1,k)
      write(11) (ija(i), i=1,k)
      close(11)

c     ---- products and norms on that storage (bondc.f:841-899, 902-917)
      open(12, file='vec.bin', access='stream', form='unformatted',
     &     status='old')
      read(12) n
      read(12) (x(i), i=1,n)
      close(12)
      call dsprsax(sa, ija, x, r1, n)
      call dsprstx(sa, ija, x, r2, n)
      call atimes(n, x, r3, 0)
      call atimes(n, x, r4, 1)
      call asolve(n, x, r5, 0)
      st = perc_nr_status()
      s1 = snrm(n, x, 1)
      s2 = snrm(n, x, 2)
      s4 = snrm(n, x, 4)
      open(13, file='ops.bin', access='stream', form='unformatted',
     &     status='replace')
      write(13) st
      write(13) (r1(i), i=1,n)
      write(13) (r2(i), i=1,n)
      write(13) (r3(i), i=1,n)
      write(13) (r4(i), i=1,n)
      write(13) (r5(i), i=1,n)
      write(13) s1, s2, s4
      close(13)

c     ---- linbcg on COMMON /mat/ (bondc.f:545, 750-838)
      open(14, file='system.bin', access='stream', form='unformatted',
     &     status='old')
      read(14) n, k
      read(14) (sa(i), i=1,k)
      read(14) (ija(i), i=1,k)
      read(14) (b(i), i=1,n)
      read(14) itol, tol, itmax
      close(14)
      do 20 i = 1, n
        x(i) = 0.0d0
20    continue
      call linbcg(n, b, x, itol, tol, itmax, iter, err)
      st = perc_nr_status()
      open(15, file='linbcg.bin', access='stream', form='unformatted',
     &     status='replace')
      write(15) st, iter, err
      write(15) (x(i), i=1,n)
      close(15)
      end
