! Fortran caller of GJKEPA_COLLIDE (MODULE GCLIB_GJKEPA): reads a hull pool (same file format as
! test_broadphase), prints  N <hits> <info>  then one line per colliding pair:
!   C a b colliType status depth nx ny nz px py pz    (1-based hull indices, reals as ES25.17)
PROGRAM test_collide
    USE GCLIB_GJKEPA
    IMPLICIT NONE
    REAL*8, ALLOCATABLE :: pts(:,:), pool(:), npts(:,:,:), nrm(:,:), cpt(:,:), dep(:)
    INTEGER*8, ALLOCATABLE :: off(:)
    INTEGER*4, ALLOCATABLE :: cnt(:), pairs(:,:), typ(:), st(:)
    INTEGER*4 :: nh, h, n, i, info, tot
    CHARACTER(256) :: path
    CALL GET_COMMAND_ARGUMENT(1, path)
    OPEN(10, FILE=TRIM(path), STATUS='OLD')
    READ(10, *) nh
    ALLOCATE(off(nh), cnt(nh), pool(0))
    tot = 0
    DO h = 1, nh
        READ(10, *) n
        ALLOCATE(pts(n, 3))
        DO i = 1, n
            READ(10, *) pts(i, :)
        END DO
        off(h) = tot + 1; cnt(h) = n
        pool = [pool, RESHAPE(pts, [3 * n])]
        tot = tot + 3 * n
        DEALLOCATE(pts)
    END DO
    CLOSE(10)
    CALL GJKEPA_COLLIDE(2, 1.D0, pool, off, cnt, pairs, typ, npts, nrm, cpt, dep, st, info)
    WRITE(*, '(A, 1X, I0, 1X, I0)') 'N', SIZE(pairs, 2), info
    DO i = 1, SIZE(pairs, 2)
        WRITE(*, '(A, 4(1X, I0), 7(1X, ES25.17))') 'C', pairs(1, i), pairs(2, i), typ(i), st(i), dep(i), &
            nrm(:, i), cpt(:, i)
    END DO
END PROGRAM test_collide
