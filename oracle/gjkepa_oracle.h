/*
 * gjkepa_oracle.h — TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference GJK/EPA path
 * (src/GCLIB_GJKEPA.f90 of xiejihong0306/collision-detect-GJK-EPA), used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker.  The product
 * (libgjkepa_hip.so and the Fortran drop-in) never links or calls this code.
 *
 * PARITY UNPINNED against the reference's own outputs: the reference ships no tests or golden
 * vectors, and it cannot be built here (it USEs the unvendored GCLIB_List / GCLIB_QuickHull /
 * GCLIB_DeHull modules, GCLIB_GJKEPA.f90:13-15, and ifort-only extensions).  The restatement is
 * cross-checked instead against (a) the known-answer cube cases recorded in SURVEY.md
 * Appendix C and (b) independent geometric ground truth (scipy Qhull of the Minkowski difference).
 * See DESIGN.md §Oracle.
 */
#ifndef GJKEPA_ORACLE_H
#define GJKEPA_ORACLE_H
#include <stdint.h>
#include "../include/gjkepa.h"

#ifdef __cplusplus
extern "C" {
#endif

/* One pair, fp64.  p1/p2 column-major (n,3).  Fills a gjkepa_contact_f64 record. */
int oracle_gjkepa(int32_t version, double tol_ff,
                  const double* p1, int32_t n1, const double* p2, int32_t n2,
                  gjkepa_contact_f64* out);

/* Batch over a hull pool (same layout as gjkepa_batch); OpenMP over pairs with `nthreads`
 * threads (<= 0: OpenMP default).  vert_dtype F32 pools are upcast to fp64. */
int oracle_gjkepa_batch(int32_t version, double tol_ff, int32_t vert_dtype,
                        const void* verts, const int64_t* hull_off, const int32_t* hull_cnt,
                        const int32_t* pairs, int64_t n_pairs,
                        gjkepa_contact_f64* out, int32_t nthreads);

/* Branch coverage.  oracle_gjkepa_batch_cov also writes, per pair, the mask of reference branches
 * the pair took (bit ORC_BR_x; cov may be NULL).  The fixtures' histogram of these bits is the
 * evidence that the GPU parity tests exercise the reference's rare paths (tests/test_branch_cov.py). */
enum {
    ORC_BR_SPHERE_MISS = 0,     /* :76-77  RoughCollisionDetection_SphericalEnvelope rejects */
    ORC_BR_INIT_RETRY,          /* :106-112 s1 ~ s2: next table direction */
    ORC_BR_INIT_CAP,            /* :86-89  99 directions exhausted */
    ORC_BR_INIT_S3_COINCIDE,    /* :123-127 third support coincides: miss */
    ORC_BR_INIT_TRI_HIT,        /* :139-148 origin on the initial triangle: hit */
    ORC_BR_INIT_TRI_PLANE,      /* :140    origin within 1e-8 of the triangle plane, IS_INSIDE_PF false */
    ORC_BR_INIT_COPLANAR,       /* :157-160 fourth support coplanar: miss */
    ORC_BR_INIT_TETRA_HIT,      /* :164-170 initial tetrahedron holds the origin (strictly) */
    ORC_BR_INIT_TETRA_ONFACE,   /* :164 via isPointInSimplex's on-face branch (:1246-1256) */
    ORC_BR_LOOP_CAP,            /* :186    50 tetrahedron iterations */
    ORC_BR_LOOP_COLLINEAR,      /* :199-201 */
    ORC_BR_LOOP_COPLANAR,       /* :203-206 */
    ORC_BR_LOOP_HIT,            /* :210-216 tetrahedron holds the origin (strictly, :1260) */
    ORC_BR_LOOP_ONFACE,         /* :210-216 via the on-face branch (:1246-1256) */
    ORC_BR_LOOP_CYCLE,          /* :219-234 simplex repeats one of the last two */
    ORC_BR_IPF_XZ,              /* :1310-1322 IS_INSIDE_PF falls back to the XZ projection */
    ORC_BR_EPA_CENTROID,        /* :905-908 orientation from the polytope mean */
    ORC_BR_EPA_FLIP,            /* :910    direction flipped */
    ORC_BR_EPA_TWO,             /* :935-944 origin on a face: second support along -dir */
    ORC_BR_EPA_SWALLOW,         /* :1005   QuickHull swallowed the new point (hull unchanged) */
    ORC_BR_EPA_STOP_EQUAL,      /* :994    same face count, sorted distances equal */
    ORC_BR_EPA_STOP_SHRINK,     /* :1010   fewer faces than before */
    ORC_BR_EPA_CAP,             /* :299-302 99 EPA iterations: zeros */
    ORC_BR_DEGENERATE,          /* :1369-1373 (and the other STOPs): status DEGENERATE */
    ORC_BR_BAD_VERSION,         /* :336-339 version_ not in {1,2,3} on a hit: status BAD_VERSION */
    ORC_BR_BAD_INPUT,           /* hull size outside 1..GJKEPA_MAX_HULL_VERTS */
    ORC_BR_V1_MID,              /* get_collisionPoint_01 :754-756 midpoint of two single supports */
    ORC_BR_V1_B,                /* :759-760 contact on p2 */
    ORC_BR_V1_A,                /* :761-762 contact on p1 */
    ORC_BR_V1_MEAN,             /* :766-803 mean of p1's supports within 0.1 */
    ORC_BR_V2_CASE01,           /* get_collisionPoint_02 case_01 (1,1) */
    ORC_BR_V2_CASE02,           /* case_02 (1, >=2) */
    ORC_BR_V2_CASE02B,          /* case_02 (>=2, 1) */
    ORC_BR_V2_CASE03,           /* case_03 (2,2) FOOT_LL */
    ORC_BR_V2_CASE04,           /* case_04 (2, >=3) */
    ORC_BR_V2_CASE04B,          /* case_04 (>=3, 2) */
    ORC_BR_V2_CASE04_1,         /* branch_case_04 C = 0: FOOT_PL of the centroid */
    ORC_BR_V2_CASE04_2,         /* C = 2 */
    ORC_BR_V2_CASE04_3,         /* C = 1 */
    ORC_BR_V2_CASE05,           /* case_05 (>=3, >=3) */
    ORC_BR_V2_OVERLAP,          /* SORT_CLOCK on coincident points (OVERLAP, :1399-1418) */
    ORC_BR_FOOTLL_PARALLEL,     /* FOOT_LL parallel lines (:1474) */
    ORC_BR_V3_NAN,              /* get_collisionPoint_03 normal = +-z: NaN normal (:447) */
    ORC_BR_TYPE1,               /* get_info_collisionType -> 1 */
    ORC_BR_TYPE2,               /* -> 2 */
    ORC_BR_COUNT
};
int oracle_gjkepa_batch_cov(int32_t version, double tol_ff, int32_t vert_dtype,
                            const void* verts, const int64_t* hull_off, const int32_t* hull_cnt,
                            const int32_t* pairs, int64_t n_pairs,
                            gjkepa_contact_f64* out, uint64_t* cov, int32_t nthreads);

/* Batched convex hulls (include/gjkepa.h: gjkepa_hull_batch semantics, host buffers, OpenMP over
 * clouds).  Same arguments as gjkepa_hull_batch minus the size bounds and the device. */
int oracle_hull_batch(int32_t vert_dtype, const void* points, const int64_t* cloud_off,
                      const int32_t* cloud_cnt, int64_t n_clouds, const int64_t* face_off,
                      int32_t* faces, int32_t* n_faces, int32_t* n_verts, int8_t* status,
                      void* hull_verts, int32_t* vert_idx, int32_t nthreads);

/* Broad phase (include/gjkepa.h: gjkepa_broadphase semantics): every pair a < b passing the
 * reference's sphere test, ascending (a, b); *n_pairs = number found, first max_pairs written. */
int oracle_broadphase(int32_t vert_dtype, const void* verts, const int64_t* hull_off, const int32_t* hull_cnt,
                      int64_t n_hulls, int32_t* pairs, int64_t max_pairs, int64_t* n_pairs, int32_t nthreads);

/* Number of OpenMP threads the batch call would use for nthreads <= 0. */
int oracle_max_threads(void);

#ifdef __cplusplus
}
#endif
#endif
