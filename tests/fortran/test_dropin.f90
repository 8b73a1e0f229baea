! Drop-in check for MODULE GCLIB_GJKEPA: a caller written against the reference's interface
! (USE GCLIB_GJKEPA; CALL GJKEPA(...), src/GCLIB_GJKEPA.f90:39-52) — unchanged — plus the batched
! entry and the reference's intended caller pattern, an OpenMP loop over pairs calling GJKEPA.
! Prints one parseable line per query; tests/test_fortran_dropin.py compares them with the oracle.
PROGRAM test_dropin
    USE GCLIB_GJKEPA
    IMPLICIT NONE
    REAL*8 :: A(8,3), B(8,3), offs(12,3)
    LOGICAL*1 :: hit
    INTEGER*4 :: typ, v, i, k, nfail
    REAL*8 :: npt(2,3), nrm(3), cpt(3), dep
    ! batch
    REAL*8, ALLOCATABLE :: verts(:)
    INTEGER*8 :: hoff(24)
    INTEGER*4 :: hcnt(24), prs(2,12), btyp(12), bst(12)
    LOGICAL*1 :: bhit(12)
    REAL*8 :: bnp(2,3,12), bn(3,12), bp(3,12), bd(12)
    ! omp
    LOGICAL*1 :: ohit(12)
    REAL*8 :: odep(12), on(3,12)

    ! unit cube [0,1]^3, x fastest (SURVEY.md §8d row d2)
    k = 0
    DO i = 0, 7
        A(i+1, 1) = MOD(i, 2); A(i+1, 2) = MOD(i/2, 2); A(i+1, 3) = i/4
    END DO
    offs = RESHAPE([0.5D0, 1.D0, 1.D0+1.D-9, 0.D0, 0.5D0, 0.3D0, 0.9D0, 0.9D0, 3.D0, 0.D0, 0.3D0, 1.D0, &
                    0.2D0, 0.D0, 0.D0,       0.D0, 0.5D0, 0.2D0, 0.8D0, 0.25D0, 0.D0, 0.D0, 0.3D0, 1.D0, &
                    0.1D0, 0.D0, 0.D0,     1.D-3, 0.1D0, 0.1D0, 0.7D0, 0.D0,   0.D0, 0.D0, 0.3D0, 1.D0], [12, 3])
    DO v = 1, 3
        DO i = 1, 12
            B(:, 1) = A(:, 1) + offs(i, 1); B(:, 2) = A(:, 2) + offs(i, 2); B(:, 3) = A(:, 3) + offs(i, 3)
            CALL GJKEPA(v, 1.D-3, A, B, hit, typ, npt, nrm, cpt, dep)
            WRITE(*, '(A,2I4,L2,2I3,13ES26.17)') 'Q', v, i, hit, typ, GJKEPA_LAST_STATUS(), dep, nrm, cpt, &
                npt(1,:), npt(2,:)
        END DO
    END DO

    ! batched entry: the same 12 pairs in one submission (1-based offsets / hull indices)
    ALLOCATE(verts(24 * 24))
    DO i = 1, 12
        B(:, 1) = A(:, 1) + offs(i, 1); B(:, 2) = A(:, 2) + offs(i, 2); B(:, 3) = A(:, 3) + offs(i, 3)
        hoff(2*i-1) = (2*i-2) * 24 + 1; hcnt(2*i-1) = 8
        hoff(2*i)   = (2*i-1) * 24 + 1; hcnt(2*i) = 8
        verts(hoff(2*i-1) : hoff(2*i-1) + 23) = RESHAPE(A, [24])
        verts(hoff(2*i) : hoff(2*i) + 23) = RESHAPE(B, [24])
        prs(1, i) = 2*i - 1; prs(2, i) = 2*i
    END DO
    CALL GJKEPA_BATCH(2, 1.D-3, verts, hoff, hcnt, prs, bhit, btyp, bnp, bn, bp, bd, bst)
    DO i = 1, 12
        WRITE(*, '(A,2I4,L2,2I3,13ES26.17)') 'B', 2, i, bhit(i), btyp(i), bst(i), bd(i), bn(:, i), bp(:, i), &
            bnp(1, :, i), bnp(2, :, i)
    END DO

    ! the device-list form (gjkepa_batch_multi): same records as the one-device submission
    CALL GJKEPA_BATCH(2, 1.D-3, verts, hoff, hcnt, prs, ohit, btyp, bnp, on, bp, odep, bst, devices_=[0])
    nfail = 0
    DO i = 1, 12
        IF (ohit(i) .NEQV. bhit(i)) nfail = nfail + 1
        IF (odep(i) /= bd(i) .OR. ANY(on(:, i) /= bn(:, i))) nfail = nfail + 1
    END DO
    WRITE(*, '(A,I4)') 'MULTI_MISMATCH', nfail

    ! the reference's caller pattern: OpenMP loop over pairs, each thread calling GJKEPA
    !$OMP PARALLEL DO PRIVATE(B, hit, typ, npt, nrm, cpt, dep) SCHEDULE(DYNAMIC)
    DO i = 1, 12
        B(:, 1) = A(:, 1) + offs(i, 1); B(:, 2) = A(:, 2) + offs(i, 2); B(:, 3) = A(:, 3) + offs(i, 3)
        CALL GJKEPA(2, 1.D-3, A, B, hit, typ, npt, nrm, cpt, dep)
        ohit(i) = hit; odep(i) = dep; on(:, i) = nrm
    END DO
    !$OMP END PARALLEL DO
    nfail = 0
    DO i = 1, 12
        IF (ohit(i) .NEQV. bhit(i)) nfail = nfail + 1
        IF (odep(i) /= bd(i)) nfail = nfail + 1
    END DO
    WRITE(*, '(A,I4)') 'OMP_MISMATCH', nfail
END PROGRAM test_dropin
