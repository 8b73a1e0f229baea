! The reference's caller pattern, timed (VERDICT r1 "Missing #6"): N pairs of 32-vertex hulls (unit
! vectors about the centre, hull B offset r ~ U[0, 2.5], the C2 distribution from a small LCG),
!   OMP    !$OMP PARALLEL DO over pairs, each iteration one CALL GJKEPA (GCLIB_GJKEPA.f90:39-52), the
!          way a caller of the reference parallelises it (THREADPRIVATE state, :9, :16, :55-60)
!   BATCH  one CALL GJKEPA_BATCH over the same pairs (one GPU submission)
! and checks that both agree.  Usage: bench_callpattern [n_pairs]; prints one line per mode.
PROGRAM bench_callpattern
    USE GCLIB_GJKEPA
    USE OMP_LIB
    IMPLICIT NONE
    INTEGER, PARAMETER :: NV = 32
    INTEGER :: n, i, k, j, nthr, nfail
    CHARACTER(32) :: arg
    REAL*8, ALLOCATABLE :: verts(:), od(:), bd(:), bn(:,:), bp(:,:), bnp(:,:,:)
    INTEGER*8, ALLOCATABLE :: hoff(:)
    INTEGER*4, ALLOCATABLE :: hcnt(:), prs(:,:), btyp(:), bst(:)
    LOGICAL*1, ALLOCATABLE :: oh(:), bh(:)
    REAL*8 :: A(NV,3), B(NV,3), npt(2,3), nrm(3), cpt(3), dep, t0, t1, t2, u(3), r, c(3)
    INTEGER*4 :: typ
    LOGICAL*1 :: hit
    INTEGER*8 :: s

    n = 20000
    IF (COMMAND_ARGUMENT_COUNT() >= 1) THEN
        CALL GET_COMMAND_ARGUMENT(1, arg)
        READ(arg, *) n
    END IF
    ALLOCATE(verts(6 * NV * n), hoff(2 * n), hcnt(2 * n), prs(2, n), oh(n), od(n), bh(n), bd(n), &
             bn(3, n), bp(3, n), bnp(2, 3, n), btyp(n), bst(n))
    s = 1234567_8
    DO i = 1, n
        DO k = 0, 1
            c = 0.D0
            IF (k == 1) THEN
                CALL unitvec(s, u)
                r = 2.5D0 * rnd(s)
                c = r * u
            END IF
            hoff(2*i-1+k) = INT(2*i-2+k, 8) * 3 * NV + 1
            hcnt(2*i-1+k) = NV
            DO j = 1, NV
                CALL unitvec(s, u)
                verts(hoff(2*i-1+k) + j - 1) = c(1) + u(1)
                verts(hoff(2*i-1+k) + NV + j - 1) = c(2) + u(2)
                verts(hoff(2*i-1+k) + 2*NV + j - 1) = c(3) + u(3)
            END DO
        END DO
        prs(1, i) = 2*i - 1; prs(2, i) = 2*i
    END DO
    nthr = OMP_GET_MAX_THREADS()

    CALL GJKEPA_BATCH(2, 1.D0, verts, hoff, hcnt, prs(:, 1:1), bh(1:1), btyp(1:1), bnp(:,:,1:1), bn(:,1:1), &
                      bp(:,1:1), bd(1:1), bst(1:1))                        ! device warm-up
    DO j = 1, 3                                                                ! query path set-up
        A(:, j) = verts(hoff(1) + (j-1)*NV : hoff(1) + j*NV - 1)
        B(:, j) = verts(hoff(2) + (j-1)*NV : hoff(2) + j*NV - 1)
    END DO
    CALL GJKEPA(2, 1.D0, A, B, hit, typ, npt, nrm, cpt, dep)
    t0 = OMP_GET_WTIME()
    !$OMP PARALLEL DO PRIVATE(A, B, hit, typ, npt, nrm, cpt, dep, j) SCHEDULE(DYNAMIC, 16)
    DO i = 1, n
        DO j = 1, 3
            A(:, j) = verts(hoff(2*i-1) + (j-1)*NV : hoff(2*i-1) + j*NV - 1)
            B(:, j) = verts(hoff(2*i) + (j-1)*NV : hoff(2*i) + j*NV - 1)
        END DO
        CALL GJKEPA(2, 1.D0, A, B, hit, typ, npt, nrm, cpt, dep)
        oh(i) = hit; od(i) = dep
    END DO
    !$OMP END PARALLEL DO
    t1 = OMP_GET_WTIME()
    CALL GJKEPA_BATCH(2, 1.D0, verts, hoff, hcnt, prs, bh, btyp, bnp, bn, bp, bd, bst)
    t2 = OMP_GET_WTIME()
    nfail = 0
    DO i = 1, n
        IF ((oh(i) .NEQV. bh(i)) .OR. od(i) /= bd(i)) nfail = nfail + 1
    END DO
    WRITE(*, '(A,I8,A,I4,A,F12.4,A,F10.3,A)') 'OMP ', n, ' pairs ', nthr, ' threads ', n / (t1 - t0) / 1.D6, &
        ' M/s ', 1.D6 * (t1 - t0) / n, ' us/pair'
    WRITE(*, '(A,I8,A,F12.4,A,F10.3,A)') 'BATCH ', n, ' pairs ', n / (t2 - t1) / 1.D6, ' M/s ', &
        1.D6 * (t2 - t1) / n, ' us/pair'
    WRITE(*, '(A,I8)') 'MISMATCH ', nfail

CONTAINS
    REAL*8 FUNCTION rnd(st)            ! 64-bit LCG, top 53 bits
        INTEGER*8, INTENT(INOUT) :: st
        st = st * 6364136223846793005_8 + 1442695040888963407_8
        rnd = REAL(ISHFT(st, -11), 8) / 9007199254740992.D0
    END FUNCTION rnd
    SUBROUTINE unitvec(st, v)
        INTEGER*8, INTENT(INOUT) :: st
        REAL*8, INTENT(OUT) :: v(3)
        REAL*8 :: zz, ph
        zz = 2.D0 * rnd(st) - 1.D0
        ph = 6.283185307179586D0 * rnd(st)
        v = [SQRT(1.D0 - zz * zz) * COS(ph), SQRT(1.D0 - zz * zz) * SIN(ph), zz]
    END SUBROUTINE unitvec
END PROGRAM bench_callpattern
