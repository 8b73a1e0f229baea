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
