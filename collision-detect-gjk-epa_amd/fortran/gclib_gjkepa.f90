!---------------------------------------------------------------------------------------------
! MODULE GCLIB_GJKEPA — MI355X drop-in for the reference module of the same name
! (xiejihong0306/collision-detect-GJK-EPA, src/GCLIB_GJKEPA.f90:12).
!
!   GJKEPA        unchanged public signature (GCLIB_GJKEPA.f90:39-52).  One pair, answered by
!                 the HIP kernels through the C-ABI (include/gjkepa.h: gjkepa_query).
!   GJKEPA_BATCH  the batched form: a pooled hull set and a pair list, replacing the caller's
!                 `!$OMP PARALLEL DO ... CALL GJKEPA` loop with one GPU submission; with the
!                 optional devices_ list, one submission per GPU of the node (contiguous shards).
!   GJKEPA_LAST_STATUS  per-thread status of the last GJKEPA call (the reference PAUSEs/STOPs
!                 instead, :300-301, :337-339, :1370-1372; here the call returns and reports).
!   GJKEPA_BROADPHASE  the pairs (a < b) of a pooled hull set that pass the reference's own first
!                 test, RoughCollisionDetection_SphericalEnvelope (:76-77, :1165-1188), computed on
!                 the GPU: the list a caller's all-pairs GJKEPA loop reduces to.
!   GJKEPA_COLLIDE  the whole all-pairs loop in one call: broad phase, GJKEPA on every candidate,
!                 and only the colliding pairs returned with their GJKEPA outputs.
!   GJKEPA_SERVICE_STOP  drain the resident grid that answers GJKEPA calls (include/gjkepa.h:
!                 gjkepa_query_service_stop) before a device-wide synchronisation.
!
! Only ISO_C_BINDING is used (no hipfort).  Hulls are REAL*8 p(n,3) exactly like the reference.
!---------------------------------------------------------------------------------------------
MODULE GCLIB_GJKEPA
    USE, INTRINSIC :: ISO_C_BINDING
    IMPLICIT NONE
    PRIVATE
    PUBLIC :: GJKEPA, GJKEPA_BATCH, GJKEPA_LAST_STATUS, GJKEPA_SET_DEVICE, GJKEPA_BROADPHASE, GJKEPA_COLLIDE
    PUBLIC :: GJKEPA_SERVICE_STOP
    PUBLIC :: GJKEPA_STATUS_OK, GJKEPA_STATUS_EPA_MAXITER, GJKEPA_STATUS_DEGENERATE
    PUBLIC :: GJKEPA_STATUS_BAD_VERSION, GJKEPA_STATUS_BAD_INPUT

    INTEGER*4, PARAMETER :: GJKEPA_STATUS_OK = 0, GJKEPA_STATUS_EPA_MAXITER = 1
    INTEGER*4, PARAMETER :: GJKEPA_STATUS_DEGENERATE = 2, GJKEPA_STATUS_BAD_VERSION = 3
    INTEGER*4, PARAMETER :: GJKEPA_STATUS_BAD_INPUT = 4

    ! mirror of gjkepa_contact_f64 (include/gjkepa.h), 128 bytes
    TYPE, BIND(C) :: contact_f64
        REAL(C_DOUBLE)     :: penetration_depth
        REAL(C_DOUBLE)     :: collision_normal(3)
        REAL(C_DOUBLE)     :: collision_point(3)
        REAL(C_DOUBLE)     :: nearest_points(6)
        INTEGER(C_INT8_T)  :: collision, colli_type, status, reserved
        INTEGER(C_INT32_T) :: diag
        INTEGER(C_INT32_T) :: pad(4)
    END TYPE contact_f64

    INTEGER(C_INT32_T), SAVE :: last_status = 0
    INTEGER(C_INT32_T), SAVE :: device = 0
    !$OMP THREADPRIVATE(last_status)

    INTERFACE
        FUNCTION c_gjkepa_query(version, tol_ff, p1, n1, p2, n2, collision, colli_type, nearest, &
                                normal, point, depth, status, dev) BIND(C, NAME="gjkepa_query")
            IMPORT :: C_INT32_T, C_INT8_T, C_DOUBLE, C_INT
            INTEGER(C_INT32_T), VALUE :: version, n1, n2, dev
            REAL(C_DOUBLE), VALUE     :: tol_ff
            REAL(C_DOUBLE), INTENT(IN) :: p1(*), p2(*)
            INTEGER(C_INT8_T), INTENT(OUT) :: collision
            INTEGER(C_INT32_T), INTENT(OUT) :: colli_type, status
            REAL(C_DOUBLE), INTENT(OUT) :: nearest(6), normal(3), point(3), depth
            INTEGER(C_INT) :: c_gjkepa_query
        END FUNCTION c_gjkepa_query

        FUNCTION c_gjkepa_batch(version, tol_ff, vert_dtype, precision, verts, n_vert_scalars, &
                                hull_off, hull_cnt, n_hulls, pairs, n_pairs, out, dev) &
                                BIND(C, NAME="gjkepa_batch")
            IMPORT :: C_INT32_T, C_INT64_T, C_DOUBLE, C_INT, contact_f64
            INTEGER(C_INT32_T), VALUE :: version, vert_dtype, precision, dev
            REAL(C_DOUBLE), VALUE     :: tol_ff
            REAL(C_DOUBLE), INTENT(IN) :: verts(*)
            INTEGER(C_INT64_T), VALUE :: n_vert_scalars, n_hulls, n_pairs
            INTEGER(C_INT64_T), INTENT(IN) :: hull_off(*)
            INTEGER(C_INT32_T), INTENT(IN) :: hull_cnt(*), pairs(*)
            TYPE(contact_f64), INTENT(OUT) :: out(*)
            INTEGER(C_INT) :: c_gjkepa_batch
        END FUNCTION c_gjkepa_batch

        FUNCTION c_gjkepa_batch_multi(version, tol_ff, vert_dtype, precision, verts, n_vert_scalars, &
                                      hull_off, hull_cnt, n_hulls, pairs, n_pairs, out, devices, ndev) &
                                      BIND(C, NAME="gjkepa_batch_multi")
            IMPORT :: C_INT32_T, C_INT64_T, C_DOUBLE, C_INT, contact_f64
            INTEGER(C_INT32_T), VALUE :: version, vert_dtype, precision, ndev
            REAL(C_DOUBLE), VALUE     :: tol_ff
            REAL(C_DOUBLE), INTENT(IN) :: verts(*)
            INTEGER(C_INT64_T), VALUE :: n_vert_scalars, n_hulls, n_pairs
            INTEGER(C_INT64_T), INTENT(IN) :: hull_off(*)
            INTEGER(C_INT32_T), INTENT(IN) :: hull_cnt(*), pairs(*), devices(*)
            TYPE(contact_f64), INTENT(OUT) :: out(*)
            INTEGER(C_INT) :: c_gjkepa_batch_multi
        END FUNCTION c_gjkepa_batch_multi

        FUNCTION c_gjkepa_broadphase(vert_dtype, verts, n_vert_scalars, hull_off, hull_cnt, n_hulls, &
                                     pairs, max_pairs, n_pairs, dev) BIND(C, NAME="gjkepa_broadphase")
            IMPORT :: C_INT32_T, C_INT64_T, C_DOUBLE, C_INT
            INTEGER(C_INT32_T), VALUE :: vert_dtype, dev
            REAL(C_DOUBLE), INTENT(IN) :: verts(*)
            INTEGER(C_INT64_T), VALUE :: n_vert_scalars, n_hulls, max_pairs
            INTEGER(C_INT64_T), INTENT(IN) :: hull_off(*)
            INTEGER(C_INT32_T), INTENT(IN) :: hull_cnt(*)
            INTEGER(C_INT32_T), INTENT(OUT) :: pairs(*)
            INTEGER(C_INT64_T), INTENT(OUT) :: n_pairs
            INTEGER(C_INT) :: c_gjkepa_broadphase
        END FUNCTION c_gjkepa_broadphase

        FUNCTION c_gjkepa_collide(version, tol_ff, vert_dtype, precision, verts, n_vert_scalars, &
                                  hull_off, hull_cnt, n_hulls, pairs, out, max_contacts, n_contacts, &
                                  n_candidates, dev) BIND(C, NAME="gjkepa_collide")
            IMPORT :: C_INT32_T, C_INT64_T, C_DOUBLE, C_INT, contact_f64
            INTEGER(C_INT32_T), VALUE :: version, vert_dtype, precision, dev
            REAL(C_DOUBLE), VALUE     :: tol_ff
            REAL(C_DOUBLE), INTENT(IN) :: verts(*)
            INTEGER(C_INT64_T), VALUE :: n_vert_scalars, n_hulls, max_contacts
            INTEGER(C_INT64_T), INTENT(IN) :: hull_off(*)
            INTEGER(C_INT32_T), INTENT(IN) :: hull_cnt(*)
            INTEGER(C_INT32_T), INTENT(OUT) :: pairs(*)
            TYPE(contact_f64), INTENT(OUT) :: out(*)
            INTEGER(C_INT64_T), INTENT(OUT) :: n_contacts, n_candidates
            INTEGER(C_INT) :: c_gjkepa_collide
        END FUNCTION c_gjkepa_collide

        FUNCTION c_gjkepa_query_service_stop(dev) BIND(C, NAME="gjkepa_query_service_stop")
            IMPORT :: C_INT32_T, C_INT
            INTEGER(C_INT32_T), VALUE :: dev
            INTEGER(C_INT) :: c_gjkepa_query_service_stop
        END FUNCTION c_gjkepa_query_service_stop

        FUNCTION c_gjkepa_last_error() BIND(C, NAME="gjkepa_last_error")
            IMPORT :: C_PTR
            TYPE(C_PTR) :: c_gjkepa_last_error
        END FUNCTION c_gjkepa_last_error
    END INTERFACE

CONTAINS

    !-----------------------------------------------------------------------------------------
    ! GJKEPA — same arguments and meaning as the reference (GCLIB_GJKEPA.f90:39-52)
    !-----------------------------------------------------------------------------------------
    SUBROUTINE GJKEPA(version_, TOL_FF_, p1_, p2_, collision_, colliType_, &
                      nearest_points_, collision_normal_, collision_point_, penetration_depth_)
        INTEGER*4, INTENT(IN)  :: version_
        REAL*8,    INTENT(IN)  :: TOL_FF_
        REAL*8,    INTENT(IN)  :: p1_(:,:), p2_(:,:)
        LOGICAL*1, INTENT(OUT) :: collision_
        INTEGER*4, INTENT(OUT) :: colliType_
        REAL*8,    INTENT(OUT) :: nearest_points_(2,3)
        REAL*8,    INTENT(OUT) :: collision_normal_(3)
        REAL*8,    INTENT(OUT) :: collision_point_(3)
        REAL*8,    INTENT(OUT) :: penetration_depth_
        REAL*8 :: a(SIZE(p1_,1), 3), b(SIZE(p2_,1), 3), np(6)
        INTEGER(C_INT8_T)  :: hit
        INTEGER(C_INT32_T) :: typ, st
        INTEGER(C_INT)     :: rc
        a = p1_                    ! contiguous column-major copies (p(n,3), as the reference)
        b = p2_
        rc = c_gjkepa_query(INT(version_, C_INT32_T), TOL_FF_, a, INT(SIZE(p1_,1), C_INT32_T), &
                            b, INT(SIZE(p2_,1), C_INT32_T), hit, typ, np, collision_normal_, &
                            collision_point_, penetration_depth_, st, device)
        IF (rc /= 0) THEN
            CALL report(rc, "GJKEPA")
            collision_ = .FALSE.; colliType_ = 0
            nearest_points_ = 0.D0; collision_normal_ = 0.D0; collision_point_ = 0.D0
            penetration_depth_ = 0.D0
            last_status = GJKEPA_STATUS_BAD_INPUT
            RETURN
        END IF
        collision_ = hit /= 0
        colliType_ = typ
        nearest_points_ = RESHAPE(np, [2, 3])
        last_status = st
    END SUBROUTINE GJKEPA

    !-----------------------------------------------------------------------------------------
    ! GJKEPA_SERVICE_STOP — drain the grid that answers GJKEPA calls on the current device (all
    ! devices with all_ = .TRUE.); later GJKEPA calls relaunch it.  rc_ (optional): 0 or GJKEPA_E_*.
    !-----------------------------------------------------------------------------------------
    SUBROUTINE GJKEPA_SERVICE_STOP(all_, rc_)
        LOGICAL, INTENT(IN), OPTIONAL    :: all_
        INTEGER*4, INTENT(OUT), OPTIONAL :: rc_
        INTEGER(C_INT) :: rc
        INTEGER(C_INT32_T) :: dev
        dev = device
        IF (PRESENT(all_)) THEN
            IF (all_) dev = -1
        END IF
        rc = c_gjkepa_query_service_stop(dev)
        IF (rc /= 0) CALL report(rc, "GJKEPA_SERVICE_STOP")
        IF (PRESENT(rc_)) rc_ = rc
    END SUBROUTINE GJKEPA_SERVICE_STOP

    !-----------------------------------------------------------------------------------------
    ! GJKEPA_BATCH — npairs queries in one submission.
    !   verts_(:)        REAL*8 hull pool; hull h occupies verts_(hull_off_(h) : hull_off_(h)+3n-1)
    !                    as x(1:n), y(1:n), z(1:n)  (1-based offsets, n = hull_cnt_(h))
    !   pairs_(2,np)     1-based hull indices (p1_, p2_) of each pair
    !   outputs          per pair, same meaning as GJKEPA's INTENT(OUT) arguments, plus status_
    !   devices_         OPTIONAL 0-based GPU list: the pairs split into SIZE(devices_) contiguous
    !                    shards, one per device, run concurrently (gjkepa_batch_multi); results are
    !                    identical to one device.  Absent: the device of GJKEPA_SET_DEVICE.
    !-----------------------------------------------------------------------------------------
    SUBROUTINE GJKEPA_BATCH(version_, TOL_FF_, verts_, hull_off_, hull_cnt_, pairs_, &
                            collision_, colliType_, nearest_points_, collision_normal_, &
                            collision_point_, penetration_depth_, status_, devices_)
        INTEGER*4, INTENT(IN)  :: version_
        REAL*8,    INTENT(IN)  :: TOL_FF_
        REAL*8,    INTENT(IN)  :: verts_(:)
        INTEGER*8, INTENT(IN)  :: hull_off_(:)
        INTEGER*4, INTENT(IN)  :: hull_cnt_(:)
        INTEGER*4, INTENT(IN)  :: pairs_(:,:)
        LOGICAL*1, INTENT(OUT) :: collision_(:)
        INTEGER*4, INTENT(OUT) :: colliType_(:)
        REAL*8,    INTENT(OUT) :: nearest_points_(:,:,:)     ! (2,3,np)
        REAL*8,    INTENT(OUT) :: collision_normal_(:,:)     ! (3,np)
        REAL*8,    INTENT(OUT) :: collision_point_(:,:)      ! (3,np)
        REAL*8,    INTENT(OUT) :: penetration_depth_(:)
        INTEGER*4, INTENT(OUT) :: status_(:)
        INTEGER*4, INTENT(IN), OPTIONAL :: devices_(:)
        TYPE(contact_f64), ALLOCATABLE :: rec(:)
        REAL(C_DOUBLE), ALLOCATABLE :: v(:)
        INTEGER(C_INT64_T), ALLOCATABLE :: off(:)
        INTEGER(C_INT32_T), ALLOCATABLE :: cnt(:), prs(:)
        INTEGER(C_INT64_T) :: np, nh
        INTEGER :: k
        INTEGER(C_INT) :: rc
        np = SIZE(pairs_, 2)
        nh = SIZE(hull_cnt_)
        ALLOCATE(rec(MAX(np, 1_C_INT64_T)), v(SIZE(verts_)), off(nh), cnt(nh), prs(2 * np))
        v = verts_
        off = hull_off_ - 1                     ! 0-based scalar offsets for the C-ABI
        cnt = hull_cnt_
        prs = RESHAPE(pairs_ - 1, [INT(2 * np)])
        IF (PRESENT(devices_)) THEN
            rc = c_gjkepa_batch_multi(INT(version_, C_INT32_T), TOL_FF_, 1_C_INT32_T, 1_C_INT32_T, v, &
                                      INT(SIZE(verts_), C_INT64_T), off, cnt, nh, prs, np, rec, &
                                      INT(devices_, C_INT32_T), INT(SIZE(devices_), C_INT32_T))
        ELSE
            rc = c_gjkepa_batch(INT(version_, C_INT32_T), TOL_FF_, 1_C_INT32_T, 1_C_INT32_T, v, &
                                INT(SIZE(verts_), C_INT64_T), off, cnt, nh, prs, np, rec, device)
        END IF
        IF (rc /= 0) THEN
            CALL report(rc, "GJKEPA_BATCH")
            collision_ = .FALSE.; colliType_ = 0; nearest_points_ = 0.D0
            collision_normal_ = 0.D0; collision_point_ = 0.D0; penetration_depth_ = 0.D0
            status_ = GJKEPA_STATUS_BAD_INPUT
            RETURN
        END IF
        DO k = 1, INT(np)
            collision_(k) = rec(k)%collision /= 0
            colliType_(k) = rec(k)%colli_type
            nearest_points_(1, :, k) = rec(k)%nearest_points(1:3)
            nearest_points_(2, :, k) = rec(k)%nearest_points(4:6)
            collision_normal_(:, k) = rec(k)%collision_normal
            collision_point_(:, k) = rec(k)%collision_point
            penetration_depth_(k) = rec(k)%penetration_depth
            status_(k) = rec(k)%status
        END DO
    END SUBROUTINE GJKEPA_BATCH

    !-----------------------------------------------------------------------------------------
    ! GJKEPA_BROADPHASE — candidate pairs of a pooled hull set (same pool layout as GJKEPA_BATCH).
    !   pairs_(2, n)  ALLOCATABLE out: 1-based hull indices (a < b), ascending (a, b), exactly the
    !                 pairs whose GJKEPA call would pass RoughCollisionDetection_SphericalEnvelope
    !   info_         0, or a negative GJKEPA_E_* code (pairs_ then has size 0)
    !-----------------------------------------------------------------------------------------
    SUBROUTINE GJKEPA_BROADPHASE(verts_, hull_off_, hull_cnt_, pairs_, info_)
        REAL*8,    INTENT(IN)  :: verts_(:)
        INTEGER*8, INTENT(IN)  :: hull_off_(:)
        INTEGER*4, INTENT(IN)  :: hull_cnt_(:)
        INTEGER*4, ALLOCATABLE, INTENT(OUT) :: pairs_(:,:)
        INTEGER*4, INTENT(OUT) :: info_
        INTEGER(C_INT64_T), ALLOCATABLE :: off(:)
        INTEGER(C_INT32_T), ALLOCATABLE :: buf(:)
        INTEGER(C_INT64_T) :: nh, cap, nfound
        INTEGER(C_INT) :: rc
        nh = SIZE(hull_cnt_)
        ALLOCATE(off(nh))
        off = hull_off_ - 1
        cap = MAX(8_C_INT64_T * nh, 1024_C_INT64_T)
        DO
            ALLOCATE(buf(2 * cap))
            rc = c_gjkepa_broadphase(1_C_INT32_T, verts_, INT(SIZE(verts_), C_INT64_T), off, hull_cnt_, nh, &
                                     buf, cap, nfound, device)
            IF (rc /= 0 .OR. nfound <= cap) EXIT
            cap = nfound                     ! the list was cut: call again with room for all of it
            DEALLOCATE(buf)
        END DO
        IF (rc /= 0) THEN
            CALL report(rc, "GJKEPA_BROADPHASE")
            ALLOCATE(pairs_(2, 0))
            info_ = rc
            RETURN
        END IF
        ALLOCATE(pairs_(2, nfound))
        pairs_ = RESHAPE(buf(1:2 * nfound), [2, INT(nfound)]) + 1
        info_ = 0
    END SUBROUTINE GJKEPA_BROADPHASE

    !-----------------------------------------------------------------------------------------
    ! GJKEPA_COLLIDE — every colliding pair of a pooled hull set (same pool layout as GJKEPA_BATCH),
    ! i.e. the caller's `DO a; DO b = a+1; CALL GJKEPA(...); IF (collision_) ...` loop in one call.
    !   pairs_(2, n)           ALLOCATABLE out: 1-based (a < b), ascending, only pairs with collision_
    !   outputs (…, n)          ALLOCATABLE out: GJKEPA's INTENT(OUT) values for those pairs
    !   info_                  0, or a negative GJKEPA_E_* code (everything then has size 0)
    !-----------------------------------------------------------------------------------------
    SUBROUTINE GJKEPA_COLLIDE(version_, TOL_FF_, verts_, hull_off_, hull_cnt_, pairs_, colliType_, &
                              nearest_points_, collision_normal_, collision_point_, penetration_depth_, &
                              status_, info_)
        INTEGER*4, INTENT(IN)  :: version_
        REAL*8,    INTENT(IN)  :: TOL_FF_
        REAL*8,    INTENT(IN)  :: verts_(:)
        INTEGER*8, INTENT(IN)  :: hull_off_(:)
        INTEGER*4, INTENT(IN)  :: hull_cnt_(:)
        INTEGER*4, ALLOCATABLE, INTENT(OUT) :: pairs_(:,:), colliType_(:), status_(:)
        REAL*8,    ALLOCATABLE, INTENT(OUT) :: nearest_points_(:,:,:), collision_normal_(:,:)
        REAL*8,    ALLOCATABLE, INTENT(OUT) :: collision_point_(:,:), penetration_depth_(:)
        INTEGER*4, INTENT(OUT) :: info_
        TYPE(contact_f64), ALLOCATABLE :: rec(:)
        INTEGER(C_INT64_T), ALLOCATABLE :: off(:)
        INTEGER(C_INT32_T), ALLOCATABLE :: buf(:)
        INTEGER(C_INT64_T) :: nh, cap, nhit, ncand
        INTEGER(C_INT) :: rc
        INTEGER :: k, n
        nh = SIZE(hull_cnt_)
        ALLOCATE(off(nh))
        off = hull_off_ - 1
        cap = MAX(4_C_INT64_T * nh, 1024_C_INT64_T)
        DO
            ALLOCATE(buf(2 * cap), rec(cap))
            rc = c_gjkepa_collide(INT(version_, C_INT32_T), TOL_FF_, 1_C_INT32_T, 1_C_INT32_T, verts_, &
                                  INT(SIZE(verts_), C_INT64_T), off, hull_cnt_, nh, buf, rec, cap, nhit, &
                                  ncand, device)
            IF (rc /= 0 .OR. nhit <= cap) EXIT
            cap = nhit                       ! more hits than room: call again with room for all
            DEALLOCATE(buf, rec)
        END DO
        n = 0
        IF (rc == 0) n = INT(nhit)
        ALLOCATE(pairs_(2, n), colliType_(n), status_(n), nearest_points_(2, 3, n), collision_normal_(3, n), &
                 collision_point_(3, n), penetration_depth_(n))
        info_ = rc
        IF (rc /= 0) THEN
            CALL report(rc, "GJKEPA_COLLIDE")
            RETURN
        END IF
        DO k = 1, n
            pairs_(:, k) = buf(2 * k - 1 : 2 * k) + 1
            colliType_(k) = rec(k)%colli_type
            nearest_points_(1, :, k) = rec(k)%nearest_points(1:3)
            nearest_points_(2, :, k) = rec(k)%nearest_points(4:6)
            collision_normal_(:, k) = rec(k)%collision_normal
            collision_point_(:, k) = rec(k)%collision_point
            penetration_depth_(k) = rec(k)%penetration_depth
            status_(k) = rec(k)%status
        END DO
    END SUBROUTINE GJKEPA_COLLIDE

    INTEGER*4 FUNCTION GJKEPA_LAST_STATUS()
        GJKEPA_LAST_STATUS = last_status
    END FUNCTION GJKEPA_LAST_STATUS

    SUBROUTINE GJKEPA_SET_DEVICE(dev_)
        INTEGER*4, INTENT(IN) :: dev_
        device = dev_
    END SUBROUTINE GJKEPA_SET_DEVICE

    SUBROUTINE report(rc, where)
        INTEGER(C_INT), INTENT(IN) :: rc
        CHARACTER(*), INTENT(IN) :: where
        CHARACTER(KIND=C_CHAR), POINTER :: msg(:)
        TYPE(C_PTR) :: p
        INTEGER :: n
        p = c_gjkepa_last_error()
        CALL C_F_POINTER(p, msg, [512])
        n = 0
        DO WHILE (n < 512)
            IF (msg(n + 1) == C_NULL_CHAR) EXIT
            n = n + 1
        END DO
        WRITE(0, '(A, A, I0, A, 512A1)') where, "(): gjkepa error ", rc, ": ", msg(1:n)
    END SUBROUTINE report

END MODULE GCLIB_GJKEPA
