!---------------------------------------------------------------------------------------------
! MODULE GCLIB_QuickHull / MODULE GCLIB_DeHull — MI355X versions of the two hull routines the
! reference USEs but does not vendor (xiejihong0306/collision-detect-GJK-EPA,
! src/GCLIB_GJKEPA.f90:14-15), with the argument lists of its call sites:
!
!   CALL QuickHull(scatPoints, polytope_2_, info)           (GCLIB_GJKEPA.f90:950)
!       points(n,3) REAL*8 -> polytope(F,3,3) REAL*8 ALLOCATABLE (face, vertex, xyz), outward
!       wound triangles; info = GJKEPA status (0 OK, 2 degenerate cloud, 4 bad input).  Runs on the
!       GPU through the C-ABI (include/gjkepa.h: gjkepa_hull_batch).
!   CALL getHullMeshesVertex(polytope_1_, scatPoints, info) (GCLIB_GJKEPA.f90:920)
!       the distinct vertices of a triangle soup, in order of first appearance (host code).
!   QUICKHULL_BATCH  every cloud of a pool in one GPU submission (1-based offsets / indices).
!
! Only ISO_C_BINDING is used.  Clouds are REAL*8 p(n,3), column major, like the reference.
!---------------------------------------------------------------------------------------------
MODULE GCLIB_QuickHull
    USE, INTRINSIC :: ISO_C_BINDING
    IMPLICIT NONE
    PRIVATE
    PUBLIC :: QuickHull, QUICKHULL_BATCH

    INTERFACE
        FUNCTION c_gjkepa_hull_batch(vert_dtype, points, n_point_scalars, cloud_off, cloud_cnt, n_clouds, &
                                     face_off, n_face_slots, faces, n_faces, n_verts, status, hull_verts, &
                                     vert_idx, dev) BIND(C, NAME="gjkepa_hull_batch")
            IMPORT :: C_INT32_T, C_INT64_T, C_INT8_T, C_DOUBLE, C_INT, C_PTR
            INTEGER(C_INT32_T), VALUE :: vert_dtype, dev
            REAL(C_DOUBLE), INTENT(IN) :: points(*)
            INTEGER(C_INT64_T), VALUE :: n_point_scalars, n_clouds, n_face_slots
            INTEGER(C_INT64_T), INTENT(IN) :: cloud_off(*), face_off(*)
            INTEGER(C_INT32_T), INTENT(IN) :: cloud_cnt(*)
            INTEGER(C_INT32_T), INTENT(OUT) :: faces(*), n_faces(*), n_verts(*)
            INTEGER(C_INT8_T), INTENT(OUT) :: status(*)
            REAL(C_DOUBLE), INTENT(OUT) :: hull_verts(*)
            TYPE(C_PTR), VALUE :: vert_idx
            INTEGER(C_INT) :: c_gjkepa_hull_batch
        END FUNCTION c_gjkepa_hull_batch
    END INTERFACE

    INTEGER*4, PARAMETER :: BAD_INPUT = 4

CONTAINS

    SUBROUTINE QuickHull(points_, polytope_, info_)
        REAL*8, INTENT(IN) :: points_(:,:)
        REAL*8, ALLOCATABLE, INTENT(OUT) :: polytope_(:,:,:)
        INTEGER*4, INTENT(OUT) :: info_
        REAL(C_DOUBLE) :: p(SIZE(points_, 1) * 3), hv(SIZE(points_, 1) * 3)
        INTEGER(C_INT32_T) :: faces(3, MAX(2 * SIZE(points_, 1) - 4, 1)), nf(1), nv(1), cnt(1)
        INTEGER(C_INT64_T) :: off(1), foff(1)
        INTEGER(C_INT8_T) :: st(1)
        INTEGER(C_INT) :: rc
        INTEGER :: n, f, v
        n = SIZE(points_, 1)
        p = RESHAPE(points_(:, 1:3), [3 * n])      ! x(1:n), y(1:n), z(1:n)
        off = 0; foff = 0; cnt = n
        rc = c_gjkepa_hull_batch(1_C_INT32_T, p, INT(3 * n, C_INT64_T), off, cnt, 1_C_INT64_T, foff, &
                                 INT(SIZE(faces, 2), C_INT64_T), faces, nf, nv, st, hv, C_NULL_PTR, 0_C_INT32_T)
        IF (rc /= 0) THEN
            ALLOCATE(polytope_(0, 3, 3))
            info_ = BAD_INPUT
            RETURN
        END IF
        ALLOCATE(polytope_(nf(1), 3, 3))
        DO f = 1, nf(1)
            DO v = 1, 3
                polytope_(f, v, :) = points_(faces(v, f) + 1, 1:3)
            END DO
        END DO
        info_ = st(1)
    END SUBROUTINE QuickHull

    !-----------------------------------------------------------------------------------------
    ! QUICKHULL_BATCH — hulls of every cloud of a pool.
    !   points_(:)        REAL*8 pool; cloud c occupies points_(cloud_off_(c) : +3n-1) as x, y, z
    !   face_off_(c)      1-based first triangle of cloud c in faces_(3,:) (room for 2n-4)
    !   faces_(3,:)       1-based point indices (within the cloud) of each outward triangle
    !   hull_verts_(:)    cloud c's hull vertices at cloud_off_(c), stride n_verts_(c)
    !-----------------------------------------------------------------------------------------
    SUBROUTINE QUICKHULL_BATCH(points_, cloud_off_, cloud_cnt_, face_off_, faces_, n_faces_, n_verts_, &
                               status_, hull_verts_)
        REAL*8,    INTENT(IN)  :: points_(:)
        INTEGER*8, INTENT(IN)  :: cloud_off_(:), face_off_(:)
        INTEGER*4, INTENT(IN)  :: cloud_cnt_(:)
        INTEGER*4, INTENT(OUT) :: faces_(:,:), n_faces_(:), n_verts_(:), status_(:)
        REAL*8,    INTENT(OUT) :: hull_verts_(:)
        INTEGER(C_INT64_T), ALLOCATABLE :: off(:), foff(:)
        INTEGER(C_INT32_T), ALLOCATABLE :: fc(:,:)
        INTEGER(C_INT8_T), ALLOCATABLE :: st(:)
        INTEGER(C_INT) :: rc
        INTEGER :: c, f
        ALLOCATE(off(SIZE(cloud_cnt_)), foff(SIZE(cloud_cnt_)), st(SIZE(cloud_cnt_)))
        ALLOCATE(fc(3, MAX(SIZE(faces_, 2), 1)))
        off = cloud_off_ - 1
        foff = face_off_ - 1
        rc = c_gjkepa_hull_batch(1_C_INT32_T, points_, INT(SIZE(points_), C_INT64_T), off, cloud_cnt_, &
                                 INT(SIZE(cloud_cnt_), C_INT64_T), foff, INT(SIZE(faces_, 2), C_INT64_T), fc, &
                                 n_faces_, n_verts_, st, hull_verts_, C_NULL_PTR, 0_C_INT32_T)
        IF (rc /= 0) THEN
            n_faces_ = 0; n_verts_ = 0; status_ = BAD_INPUT
            RETURN
        END IF
        status_ = st
        DO c = 1, SIZE(cloud_cnt_)
            DO f = 0, n_faces_(c) - 1
                faces_(:, face_off_(c) + f) = fc(:, foff(c) + f + 1) + 1
            END DO
        END DO
    END SUBROUTINE QUICKHULL_BATCH

END MODULE GCLIB_QuickHull


MODULE GCLIB_DeHull
    IMPLICIT NONE
    PRIVATE
    PUBLIC :: getHullMeshesVertex

CONTAINS

    SUBROUTINE getHullMeshesVertex(polytope_, points_, info_)
        REAL*8, INTENT(IN) :: polytope_(:,:,:)
        REAL*8, ALLOCATABLE, INTENT(OUT) :: points_(:,:)
        INTEGER*4, INTENT(OUT) :: info_
        REAL*8 :: buf(3 * SIZE(polytope_, 1), 3)
        INTEGER :: f, v, k, m
        LOGICAL :: seen
        m = 0
        DO f = 1, SIZE(polytope_, 1)
            DO v = 1, 3
                seen = .FALSE.
                DO k = 1, m
                    IF (ALL(buf(k, :) == polytope_(f, v, :))) THEN
                        seen = .TRUE.
                        EXIT
                    END IF
                END DO
                IF (.NOT. seen) THEN
                    m = m + 1
                    buf(m, :) = polytope_(f, v, :)
                END IF
            END DO
        END DO
        ALLOCATE(points_(m, 3))
        points_ = buf(1:m, :)
        info_ = 0
    END SUBROUTINE getHullMeshesVertex

END MODULE GCLIB_DeHull
