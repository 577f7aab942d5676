c     nn_caller.f -- a Fortran 77 caller of libperc's nearestn_ written for
c     the tests (tests/test_nr_symbols.py): the blank COMMON of the
c     reference programs (Square/bondc.f:58), call nearestn(i) for every
c     site as bondc.f:140 does, resolved at link time from libperc.so.
c     Input nn.in: m, n, pbc, scn (list-directed).  Output nn.bin (stream):
c     status, then nn(1..scn) of sites 1..m*n.
      program nncall
      implicit none
      integer m, n, t, pbc, nn(10), scn
      common m, n, t, pbc, nn, scn
      integer i, z, st
      integer perc_nr_status
      external perc_nr_status
      open(10, file='nn.in', status='old')
      read(10, *) m, n, pbc, scn
      close(10)
      t = m*n
      open(11, file='nn.bin', access='stream', form='unformatted',
     &     status='replace')
      st = 0
      do i = 1, t
         call nearestn(i)
         if (perc_nr_status() .ne. 0) st = perc_nr_status()
         write(11) (nn(z), z=1,scn)
      end do
      write(11) st
      close(11)
      end
