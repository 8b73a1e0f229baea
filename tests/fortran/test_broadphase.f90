! Fortran caller of GJKEPA_BROADPHASE (MODULE GCLIB_GJKEPA): reads a hull pool from the file named
! on the command line (line 1: number of hulls; per hull: n, then n lines x y z), prints
!   N <number of pairs>   then one "P a b" line per pair (1-based hull indices)
PROGRAM test_broadphase
    USE GCLIB_GJKEPA
    IMPLICIT NONE
    REAL*8, ALLOCATABLE :: pts(:,:), pool(:)
    INTEGER*8, ALLOCATABLE :: off(:)
    INTEGER*4, ALLOCATABLE :: cnt(:), pairs(:,:)
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
    CALL GJKEPA_BROADPHASE(pool, off, cnt, pairs, info)
    WRITE(*, '(A, 1X, I0, 1X, I0)') 'N', SIZE(pairs, 2), info
    DO i = 1, SIZE(pairs, 2)
        WRITE(*, '(A, 1X, I0, 1X, I0)') 'P', pairs(1, i), pairs(2, i)
    END DO
END PROGRAM test_broadphase
