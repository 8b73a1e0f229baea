! Fortran caller of the hull modules written against the reference's call sites
! (GCLIB_GJKEPA.f90:920, :950): USE GCLIB_QuickHull / GCLIB_DeHull, CALL QuickHull(...),
! CALL getHullMeshesVertex(...).  Reads clouds from the file named on the command line
! (line 1: number of clouds; per cloud: n, then n lines x y z), prints per cloud
!   Q <cloud> <info> <nfaces> <nverts>   then one "F" line per face (9 coordinates)
! and the batched entry's result as   B <cloud> <status> <nfaces> <nverts> <face index triples...>
PROGRAM test_quickhull
    USE GCLIB_QuickHull
    USE GCLIB_DeHull
    IMPLICIT NONE
    REAL*8, ALLOCATABLE :: pts(:,:), poly(:,:,:), verts(:,:), pool(:), hv(:)
    INTEGER*8, ALLOCATABLE :: off(:), foff(:)
    INTEGER*4, ALLOCATABLE :: cnt(:), faces(:,:), nf(:), nv(:), st(:)
    INTEGER*4 :: info, info2, nc, c, n, i, f, tot, totf
    CHARACTER(256) :: path
    CALL GET_COMMAND_ARGUMENT(1, path)
    OPEN(10, FILE=TRIM(path), STATUS='OLD')
    READ(10, *) nc
    ALLOCATE(off(nc), foff(nc), cnt(nc), nf(nc), nv(nc), st(nc))
    ALLOCATE(pool(0))
    tot = 0; totf = 0
    DO c = 1, nc
        READ(10, *) n
        ALLOCATE(pts(n, 3))
        DO i = 1, n
            READ(10, *) pts(i, :)
        END DO
        CALL QuickHull(pts, poly, info)
        CALL getHullMeshesVertex(poly, verts, info2)
        WRITE(*, '(A, 1X, I0, 1X, I0, 1X, I0, 1X, I0)') 'Q', c, info, SIZE(poly, 1), SIZE(verts, 1)
        DO f = 1, SIZE(poly, 1)
            WRITE(*, '(A, 9(1X, ES24.16E3))') 'F', poly(f, 1, :), poly(f, 2, :), poly(f, 3, :)
        END DO
        off(c) = tot + 1; cnt(c) = n; foff(c) = totf + 1
        pool = [pool, RESHAPE(pts, [3 * n])]
        tot = tot + 3 * n
        totf = totf + MAX(2 * n - 4, 0)
        DEALLOCATE(pts)
    END DO
    CLOSE(10)
    ALLOCATE(faces(3, MAX(totf, 1)), hv(tot))
    CALL QUICKHULL_BATCH(pool, off, cnt, foff, faces, nf, nv, st, hv)
    DO c = 1, nc
        WRITE(*, '(A, 1X, I0, 1X, I0, 1X, I0, 1X, I0)', ADVANCE='NO') 'B', c, st(c), nf(c), nv(c)
        DO f = 0, nf(c) - 1
            WRITE(*, '(3(1X, I0))', ADVANCE='NO') faces(:, foff(c) + f)
        END DO
        WRITE(*, *)
    END DO
END PROGRAM test_quickhull
