/*
 * gjkepa.h — C-ABI drop-in boundary of the MI355X batched GJK/EPA narrow phase.
 *
 * The reference (xiejihong0306/collision-detect-GJK-EPA) exposes exactly one public entry,
 * SUBROUTINE GJKEPA in MODULE GCLIB_GJKEPA (src/GCLIB_GJKEPA.f90:12, :39-52).  It answers one
 * convex-pair query: hit flag, contact type, nearest points, normal, contact point and
 * penetration depth.  The entries below are what an ISO_C_BINDING interface for that path binds:
 *
 *   gjkepa_query         one pair, same arguments / meaning as GJKEPA (GCLIB_GJKEPA.f90:39-52);
 *                        host buffers, blocking.  The Fortran drop-in module
 *                        (collision-detect-gjk-epa_amd/fortran/gclib_gjkepa.f90) wraps it
 *                        under the unchanged GJKEPA signature.
 *   gjkepa_batch         N pairs over a pooled hull set, host buffers, blocking.  This replaces
 *                        the caller-side `!$OMP PARALLEL DO ... CALL GJKEPA` loop implied by the
 *                        THREADPRIVATE design (GCLIB_GJKEPA.f90:9, :16, :55-60).
 *   gjkepa_batch_device  the same with every buffer already resident in device memory (HBM),
 *                        asynchronous on a caller stream; no allocation, no synchronisation,
 *                        so it can be captured into a hipGraph.
 *
 * Error behaviour.  The reference has no return codes: it writes to unit 6 and then PAUSEs or
 * STOPs (GCLIB_GJKEPA.f90:300-301, :337-339, :499-501, :635-637, :1370-1372).  Here every
 * pair carries a status code instead (GJKEPA_STATUS_*), outputs are left at the values the
 * reference would have returned (EPA cap: all zero with collision = 1, :299-302) or zeroed
 * where the reference would have aborted, and the process never blocks.  Functions return
 * 0 on success or a negative GJKEPA_E_* code.
 *
 * Data layout.  A hull is stored exactly like the reference's REAL*8 p(n,3) argument: column
 * major, i.e. x[0..n-1], y[0..n-1], z[0..n-1] (structure of arrays per hull).  Hulls are pooled:
 * hull h starts at scalar offset hull_off[h] of `verts` and has hull_cnt[h] vertices.  A pair
 * is two hull indices (pairs[2k], pairs[2k+1]) = (p1_, p2_).
 *
 * Plain pointers and sizes only; no torch or HIP types in any signature.
 */
#ifndef GJKEPA_H
#define GJKEPA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- per-pair status (replaces PAUSE / STOP) ---------------------------------------------- */
#define GJKEPA_STATUS_OK          0  /* normal return */
#define GJKEPA_STATUS_EPA_MAXITER 1  /* EPA hit its 99-iteration cap (:299-302): outputs 0, colli_type 0 */
#define GJKEPA_STATUS_DEGENERATE  2  /* reference would STOP: degenerate plane (:1369-1373) etc. */
#define GJKEPA_STATUS_BAD_VERSION 3  /* version_ not in {1,2,3} on a hit (:336-339) */
#define GJKEPA_STATUS_BAD_INPUT   4  /* hull with < 1 vertex or above GJKEPA_MAX_HULL_VERTS */

/* ---- API return codes ---------------------------------------------------------------------- */
#define GJKEPA_E_OK          0
#define GJKEPA_E_ARG        -1  /* invalid argument (null pointer, bad enum, bad size) */
#define GJKEPA_E_HIP        -2  /* HIP runtime error (see gjkepa_last_error) */
#define GJKEPA_E_NODEVICE   -3  /* no usable gfx950 device */
#define GJKEPA_E_WORKSPACE  -4  /* device workspace too small */
#define GJKEPA_E_COMM       -5  /* RCCL unavailable or a collective failed (see gjkepa_last_error) */

/* ---- enums --------------------------------------------------------------------------------- */
#define GJKEPA_DTYPE_F32 0      /* vertex storage dtype */
#define GJKEPA_DTYPE_F64 1
#define GJKEPA_PREC_F64  1      /* compute precision: fp64 = the reference's REAL*8 semantics */
#define GJKEPA_PREC_F32  0      /* compute precision: fp32, opt-in; an fp32 answer is kept only when certified to
                                   1e-6 relative depth (else recomputed in fp64), which makes it slower than F64 */

#define GJKEPA_MAX_HULL_VERTS 256   /* largest hull the kernels accept (config C4: 8..256) */

/* ---- contact records (one per pair) ---------------------------------------------------------
 * Field meaning follows GJKEPA's INTENT(OUT) arguments (GCLIB_GJKEPA.f90:47-52):
 *   penetration_depth  <- penetration_depth_
 *   collision_normal   <- collision_normal_(3)
 *   collision_point    <- collision_point_(3)
 *   nearest_points     <- nearest_points_(2,3), stored row-wise: p1 xyz then p2 xyz
 *   collision          <- collision_ (LOGICAL*1)
 *   colli_type         <- colliType_ (0 no hit / 1 other / 2 face-face)
 *   status             <- GJKEPA_STATUS_*
 *   diag               <- (gjk_iters) | (epa_iters << 8) | (final_faces << 16); diagnostics only
 */
typedef struct gjkepa_contact_f64 {
    double   penetration_depth;
    double   collision_normal[3];
    double   collision_point[3];
    double   nearest_points[6];
    int8_t   collision;
    int8_t   colli_type;
    int8_t   status;
    int8_t   reserved;
    uint32_t diag;
    uint32_t pad[4];
} gjkepa_contact_f64;            /* 128 bytes */

typedef struct gjkepa_contact_f32 {
    float    penetration_depth;
    float    collision_normal[3];
    float    collision_point[3];
    float    nearest_points[6];
    int8_t   collision;
    int8_t   colli_type;
    int8_t   status;
    int8_t   reserved;
    uint32_t diag;
    uint32_t pad;
} gjkepa_contact_f32;            /* 64 bytes */

/* Size in bytes of one contact record for a compute precision (128 for F64, 64 for F32). */
int gjkepa_record_bytes(int32_t precision);

/* ---- single pair: the GJKEPA drop-in (GCLIB_GJKEPA.f90:39-52) ---------------------------------
 * p1, p2: REAL*8 (n,3) column-major, exactly the memory of the Fortran assumed-shape actuals.
 * nearest_points: REAL*8 (2,3) column-major (Fortran layout: p1x p2x p1y p2y p1z p2z).
 * status may be NULL.  Runs on device `device` (batch of one); blocking; thread-safe. */
int gjkepa_query(int32_t version, double tol_ff,
                 const double* p1, int32_t n1,
                 const double* p2, int32_t n2,
                 int8_t* collision, int32_t* colli_type,
                 double* nearest_points, double* collision_normal,
                 double* collision_point, double* penetration_depth,
                 int32_t* status, int32_t device);

/* ---- the resident query service behind gjkepa_query ------------------------------------------
 * gjkepa_query posts each pair to a persistent grid of 64 one-wave workgroups (one per request slot
 * in host-mapped memory) instead of launching kernels per call.  The grid runs on the library's own
 * stream and leaves by itself once no call arrived for 2 ms, or after 20 ms of residency even under
 * steady traffic (the next call relaunches it at once).  While it is resident:
 *   - a device-wide synchronisation in the caller's process (hipDeviceSynchronize,
 *     torch.cuda.synchronize() without a stream, a legacy default-stream sync) waits for the grid
 *     to leave, i.e. up to 2 ms after the last call, or up to 20 ms while other threads keep calling;
 *   - work the process enqueues on a stream that shares the grid's hardware queue (streams are
 *     spread over GPU_MAX_HW_QUEUES queues) starts only after the grid leaves, within those bounds.
 * Callers that synchronise the whole device, or want it idle, drain the grid first: */
/* Drain the service grid of `device` (device < 0: every device) now; returns after it has left.
 * Calls that arrive later relaunch it.  Returns 0 or GJKEPA_E_HIP. */
int gjkepa_query_service_stop(int32_t device);
/* Turn the service on (1) or off (0) for later gjkepa_query calls; off also drains every grid.  Off,
 * single-pair calls of concurrent threads are combined into one batch launch (no resident grid).
 * The initial setting is on unless the environment sets GJKEPA_QUERY_SERVICE=0.  Returns the
 * previous setting (0/1) or a negative GJKEPA_E_* code. */
int gjkepa_query_service_set(int32_t enabled);
/* Diagnostic: 1 while a service grid of `device` (device < 0: any device) is still on the GPU, 0 when
 * none is, or a negative GJKEPA_E_* code.  Non-blocking. */
int gjkepa_query_service_resident(int32_t device);

/* ---- batch over host buffers (blocking) ------------------------------------------------------
 * verts:     hull vertex pool, dtype `vert_dtype`, n_vert_scalars scalars in total.
 * hull_off:  [n_hulls] scalar offset of each hull's x[0] in `verts`.
 * hull_cnt:  [n_hulls] vertex count of each hull (1..GJKEPA_MAX_HULL_VERTS).
 * pairs:     [2*n_pairs] hull indices (p1_, p2_) per pair.
 * out:       [n_pairs] records, gjkepa_contact_f64 (precision F64) or _f32 (precision F32). */
int gjkepa_batch(int32_t version, double tol_ff, int32_t vert_dtype, int32_t precision,
                 const void* verts, int64_t n_vert_scalars,
                 const int64_t* hull_off, const int32_t* hull_cnt, int64_t n_hulls,
                 const int32_t* pairs, int64_t n_pairs,
                 void* out, int32_t device);

/* ---- batch over device buffers (asynchronous on `stream`, a hipStream_t or NULL) -------------
 * All pointers are device pointers on the current device.  `workspace` (256-byte aligned) should hold
 * gjkepa_workspace_bytes(n_pairs) bytes: a 512-byte header of per-kernel work counters and route
 * tallies (reset by the call itself), one routing byte per pair (which GJK / EPA / contact kernel
 * tier owns the pair next), and park slots of 2880 bytes for one pair in 8: an EPA tier whose
 * polytope is about to outgrow it parks the polytope there and the next tier resumes it instead of
 * restarting from the GJK simplex (results identical either way).  The minimum is the header plus
 * the route bytes rounded up to 256; park slots are used as far as the workspace provides them.  It
 * may be reused between calls on the same stream. */
int64_t gjkepa_workspace_bytes(int64_t n_pairs);
/* The same with park slots for one in 8 of `n_large_pairs`: the pairs with a hull above 32 vertices,
 * the only ones that can reach the parking EPA tiers (0 for a batch of small hulls such as config C2:
 * header and route bytes only).  gjkepa_workspace_bytes(n) = gjkepa_workspace_bytes_for(n, n). */
int64_t gjkepa_workspace_bytes_for(int64_t n_pairs, int64_t n_large_pairs);

/* ---- per-launch timing (diagnostics; bench.py's dominant-kernel roofline) ---------------------
 * gjkepa_launch_timing(1): every later chain the calling thread enqueues (gjkepa_batch_device and the
 * entries built on it) records a timing event at its head on the caller's stream and one before and
 * after each kernel launch, on the stream that launch goes to (the caller's or an internal one).
 * gjkepa_launch_timing_read waits for those events and writes up to `max` entries, one per launch in
 * enqueue order; it returns the number written and forgets every recorded launch.  Returns the
 * previous setting / a GJKEPA_E_* code.  Not for graph capture. */
typedef struct gjkepa_launch_time {
    char     kernel[16];    /* "reset", "gjk", "epa", "contact", "redo" or "query" */
    int32_t  tier;          /* kernel tier (contact tier for "contact") */
    int32_t  part;          /* part index of a tier launched over consecutive pair ranges, else 0 */
    int32_t  route_code;    /* the pairs it serves (-1: every pair) */
    int32_t  chain;         /* enqueue call, counted from 0 since the last read */
    int32_t  stream;        /* 0: the caller's stream; 1..: the chain's internal streams, by first use */
    int32_t  pad;
    int64_t  first_pair;    /* pair range the launch scans */
    int64_t  n_pairs;
    float    start_ms;      /* events before / after the launch, ms after the chain's head event */
    float    end_ms;
} gjkepa_launch_time;
int gjkepa_launch_timing(int32_t enable);
int gjkepa_launch_timing_read(gjkepa_launch_time* out, int32_t max);
int gjkepa_batch_device(int32_t version, double tol_ff, int32_t vert_dtype, int32_t precision,
                        const void* verts, const int64_t* hull_off, const int32_t* hull_cnt,
                        const int32_t* pairs, int64_t n_pairs,
                        void* out, void* workspace, int64_t workspace_bytes,
                        void* stream);

/* ---- batched convex hulls ----------------------------------------------
 * The reference rebuilds a convex hull every EPA iteration with
 *   CALL QuickHull(scatPoints, polytope_2_, info)           (GCLIB_GJKEPA.f90:950)
 *   CALL getHullMeshesVertex(polytope_1_, scatPoints, info) (GCLIB_GJKEPA.f90:920)
 * from the unvendored modules GCLIB_QuickHull / GCLIB_DeHull (:14-15, no version pin).  These
 * entries expose the same two operations as a first-class batched device module: the hull of
 * every point cloud of a pool as outward triangles (QuickHull) plus the hull's vertex set
 * (getHullMeshesVertex), so callers can reduce raw point clouds to hulls before the narrow phase.
 *
 * Algorithm (restated bit for bit by oracle/gjkepa_oracle.c: oracle_hull_batch): QuickHull with a
 * global furthest-point order, fp64 arithmetic, absolute epsilon GJKEPA_HULL_EPS.
 *   1. initial tetrahedron: i0 = first argmin x; i1 = first argmax |p - p_i0|^2;
 *      i2 = first argmax |(p_i1 - p_i0) x (p - p_i0)|^2; i3 = first argmax |(p - p_i0).n|,
 *      n = (p_i1 - p_i0) x (p_i2 - p_i0).  Collinear / coplanar / coincident clouds (distance
 *      <= eps at any step) are GJKEPA_STATUS_DEGENERATE.
 *   2. every other point is assigned to the face it is furthest above (first face on ties) when
 *      that distance exceeds eps, otherwise discarded as interior.
 *   3. repeat: the eye is the assigned point furthest above its face (lowest index on ties); every
 *      face the eye is more than eps above is removed; each horizon edge (u, w) is coned to the
 *      eye as face (u, w, eye); points of removed faces are re-assigned among the new faces only.
 * Face slots: new faces take the removed faces' slots in slot order, then append; faces are
 * reported in slot order.  Outward winding: normal = (b - a) x (c - b) points out of the hull.
 * Vertex set (getHullMeshesVertex): the points the faces reference, in ascending point index.
 *
 * Layout.  Input clouds use the hull-pool layout above (cloud c: cloud_cnt[c] points, SoA at
 * scalar offset cloud_off[c]).  Cloud c's faces are written as int32 (a, b, c) point-index
 * triples at triangle offset face_off[c] of `faces`, with room for gjkepa_hull_face_capacity(
 * cloud_cnt[c]) = 2n - 4 triangles.  Optional outputs (NULL to skip), both at cloud_off[c]:
 * `hull_verts` (same dtype as the input) receives the hull as a pool entry of n_verts[c] points,
 * SoA with stride n_verts[c], directly usable as a gjkepa_batch hull with hull_cnt = n_verts;
 * `vert_idx` (int32) receives the hull vertices' point indices.
 * status[c]: GJKEPA_STATUS_OK, _DEGENERATE (flat cloud, zero-area cone face or a non-manifold
 * horizon that overflows 2n - 4 face slots) or _BAD_INPUT (n < 4, n > GJKEPA_HULL_MAX_POINTS,
 * non-finite coordinates); n_faces = n_verts = 0 unless OK. */
#define GJKEPA_HULL_MAX_POINTS 256
#define GJKEPA_HULL_EPS 1.0e-10

/* Triangle slots cloud c needs in `faces`: 2n - 4 (0 for n < 4). */
int64_t gjkepa_hull_face_capacity(int32_t n_points);

/* Host buffers, blocking.  n_point_scalars / n_face_slots bound the pool and face buffers. */
int gjkepa_hull_batch(int32_t vert_dtype, const void* points, int64_t n_point_scalars,
                      const int64_t* cloud_off, const int32_t* cloud_cnt, int64_t n_clouds,
                      const int64_t* face_off, int64_t n_face_slots, int32_t* faces,
                      int32_t* n_faces, int32_t* n_verts, int8_t* status,
                      void* hull_verts, int32_t* vert_idx, int32_t device);

/* Device buffers, asynchronous on `stream` (hipStream_t or NULL); no allocation, no sync. */
int gjkepa_hull_batch_device(int32_t vert_dtype, const void* points,
                             const int64_t* cloud_off, const int32_t* cloud_cnt, int64_t n_clouds,
                             const int64_t* face_off, int32_t* faces,
                             int32_t* n_faces, int32_t* n_verts, int8_t* status,
                             void* hull_verts, int32_t* vert_idx, void* stream);

/* ---- device broad phase -------------------------------------------------
 * Emits the candidate pair list a narrow-phase batch consumes: every pair of hulls (a < b) of a
 * pool whose bounding spheres pass the reference's own rough test,
 * RoughCollisionDetection_SphericalEnvelope (GCLIB_GJKEPA.f90:1165-1188):
 *   m = SUM(p(:,k)) / n (sequential sums), r = MAXVAL(NORM2(p_i - m)),
 *   pair iff NORM2(m_a - m_b) <= r_a + r_b + 1.0      (fp64, the oracle's arithmetic, bit-exact)
 * i.e. exactly the pairs whose GJKEPA call would get past its first test (:76-77); a caller's
 * double loop over all pairs collapses to this list.  Hulls with a bad vertex count or non-finite
 * coordinates take part in no pair.
 *
 * Method (MI355X): per-hull sphere kernel; uniform grid of cell edge 2 r_max + 1 with a radix
 * sort of the cell keys (rocPRIM) and a hash table from cell to first sorted hull; count / scan /
 * emit kernels test each hull against the later-indexed hulls of its 27 neighbouring cells; a final
 * radix sort of the emitted (a << 32 | b) keys leaves the list in ascending (a, b) order — the
 * order of `DO a = 1, N; DO b = a+1, N`.
 * Output: pairs[2k], pairs[2k+1] = (a, b) for k < min(n_found, max_pairs); *n_pairs = n_found
 * (device int64 for the device entry).  n_found > max_pairs means the list was cut: enlarge it and
 * call again.  The device entry never synchronises (graph-capturable): the final sort runs over
 * max_pairs keys padded with all-ones, so size max_pairs near the expected count. */
int64_t gjkepa_broadphase_workspace_bytes(int64_t n_hulls, int64_t max_pairs);

/* Host buffers, blocking.  *n_pairs = pairs found (the list holds the first max_pairs of them). */
int gjkepa_broadphase(int32_t vert_dtype, const void* verts, int64_t n_vert_scalars,
                      const int64_t* hull_off, const int32_t* hull_cnt, int64_t n_hulls,
                      int32_t* pairs, int64_t max_pairs, int64_t* n_pairs, int32_t device);

/* Device buffers, asynchronous on `stream`; n_pairs is a device int64. */
int gjkepa_broadphase_device(int32_t vert_dtype, const void* verts, const int64_t* hull_off,
                             const int32_t* hull_cnt, int64_t n_hulls,
                             int32_t* pairs, int64_t max_pairs, int64_t* n_pairs,
                             void* workspace, int64_t workspace_bytes, void* stream);

/* ---- contact-list compaction -------------------------------------
 * Turns a batch's records (gjkepa_batch_device output, one per pair) into the dense list a device
 * consumer needs: hit_idx[k] = index of the k-th pair whose collision flag is set (ascending), and,
 * when `hits` is not NULL, that pair's record copied to hits[k].  *n_hits (device int64) = count.
 * Deterministic (no atomics), asynchronous on `stream`, graph-capturable; records stay in HBM.
 * workspace: gjkepa_compact_workspace_bytes(n_pairs) bytes (tile counts, offsets, scan scratch). */
int64_t gjkepa_compact_workspace_bytes(int64_t n_pairs);
int gjkepa_compact_hits_device(int32_t precision, const void* records, int64_t n_pairs,
                               int32_t* hit_idx, void* hits, int64_t* n_hits,
                               void* workspace, int64_t workspace_bytes, void* stream);

/* ---- warm start for persistent pairs -------------------------------------
 * gjkepa_batch_device plus `warm`: a device uint32[4 * n_pairs] array, one slot per pair, carried
 * from call to call (e.g. simulation frames; the same pair at the same index).  On entry a slot holds
 * the support codes (ia | ib << 16) of the simplex the pair's previous call ended GJK with, or
 * 0xFFFFFFFF (fill the array with 0xFF bytes for a first call).  When that simplex, rebuilt from the
 * current vertices, holds the origin strictly inside (every face more than 1e-6 from it), the pair
 * is a hit and EPA starts from it, skipping GJK; otherwise the reference GJK runs.  A pair that
 * missed is marked 0xFFFFFFFE (first word) and runs the reference GJK on its next call.  On exit
 * every slot holds this call's simplex (hits), the miss mark, or 0xFFFFFFFF (errors).  Pairs that
 * are not warm-started are bit-exact with gjkepa_batch_device (hit flags always are); warm-started
 * hits agree with a cold call within EPA's own tolerance (a different start polytope), not bit for
 * bit. */
int gjkepa_batch_warm_device(int32_t version, double tol_ff, int32_t vert_dtype, int32_t precision,
                             const void* verts, const int64_t* hull_off, const int32_t* hull_cnt,
                             const int32_t* pairs, int64_t n_pairs,
                             void* out, void* workspace, int64_t workspace_bytes,
                             uint32_t* warm, void* stream);

/* ---- whole collision step (host buffers, blocking) ---------------------------------------------
 * The reference caller's `DO a; DO b = a+1; CALL GJKEPA(...)` over a pooled hull set in one call:
 * gjkepa_broadphase_device -> gjkepa_batch_device on the candidate list -> gjkepa_compact_hits_device.
 * Writes the first min(n, max_contacts) hits: pairs[2k], pairs[2k+1] = (a, b) (a < b, ascending)
 * and out[k] = that pair's record (gjkepa_contact_f64 / _f32 by precision), bit-exact with GJKEPA
 * on (p_a, p_b).  *n_contacts = hits found; *n_candidates (may be NULL) = pairs past the sphere test. */
int gjkepa_collide(int32_t version, double tol_ff, int32_t vert_dtype, int32_t precision,
                   const void* verts, int64_t n_vert_scalars,
                   const int64_t* hull_off, const int32_t* hull_cnt, int64_t n_hulls,
                   int32_t* pairs, void* out, int64_t max_contacts,
                   int64_t* n_contacts, int64_t* n_candidates, int32_t device);

/* ---- multi-GPU (SURVEY.md §8 row e) ---------------------------------------------------------------
 * Pairs are independent: a job splits into contiguous shards of pairs, one per device, with no
 * exchange during compute.  The reference's own parallelism is the caller's OpenMP loop over GJKEPA
 * (GCLIB_GJKEPA.f90:9, :16, :55-60); these entries replace it across the GPUs of a node.
 *
 * gjkepa_shard_range: rank r of `world` owns pairs [first, first + count); shards differ by at most
 * one pair (the first n_pairs % world ranks get one more). */
int gjkepa_shard_range(int64_t n_pairs, int32_t world, int32_t rank, int64_t* first, int64_t* count);

/* One process, several devices (host buffers, blocking): gjkepa_batch's arguments plus a device list.
 * Shard s (gjkepa_shard_range over ndev) runs on devices[s] from its own host thread; only the hulls
 * the shard references are copied to that device; its records land at out[first .. first + count),
 * so `out` holds every record in pair order — bit-identical to one gjkepa_batch call.  The argument
 * checks are gjkepa_batch's, over the whole job, before any shard runs.  A device may appear more
 * than once: its shards then run one after the other. */
int gjkepa_batch_multi(int32_t version, double tol_ff, int32_t vert_dtype, int32_t precision,
                       const void* verts, int64_t n_vert_scalars,
                       const int64_t* hull_off, const int32_t* hull_cnt, int64_t n_hulls,
                       const int32_t* pairs, int64_t n_pairs,
                       void* out, const int32_t* devices, int32_t ndev);

/* One process per device (config C3): an RCCL communicator for the contact-record exchange.
 * Rank 0 creates the id (gjkepa_comm_unique_id), the caller broadcasts its GJKEPA_COMM_ID_BYTES bytes
 * (MPI_Bcast, torch.distributed, a file ...), every rank calls gjkepa_comm_init.  RCCL is bound at
 * run time (the copy already in the process, else librccl.so.1); GJKEPA_E_COMM if it is absent. */
#define GJKEPA_COMM_ID_BYTES 128
typedef struct gjkepa_comm gjkepa_comm;
int gjkepa_comm_unique_id(void* id);
int gjkepa_comm_init(gjkepa_comm** comm, int32_t world, int32_t rank, const void* id, int32_t device);
int gjkepa_comm_destroy(gjkepa_comm* comm);
/* Which RCCL the library bound ("process (...)", "librccl.so.1", or "unavailable"). */
const char* gjkepa_comm_backend(void);

/* All-gather of every rank's `count` contact records (device buffers; equal shards) into
 * all_records[world * count] in rank order: one ncclAllGather on `stream` (asynchronous; xGMI).
 * In place when shard_records == all_records + rank * count records. */
int gjkepa_allgather_records_device(gjkepa_comm* comm, int32_t precision, const void* shard_records,
                                    void* all_records, int64_t count, void* stream);

/* Last error message of the calling thread ("" if none). */
const char* gjkepa_last_error(void);

/* Library build string (kernels' target, caps, compile flags). */
const char* gjkepa_version_string(void);

/* ---- synthetic workload generator (deterministic, counter-based SplitMix64) ----
 * Fills a hull pool for `n_pairs` pairs with two private hulls per pair (hull 2k = p1_, 2k+1 = p2_):
 * vertices are unit vectors about the hull centre (all extreme), hull A centred at 0, hull B at
 * u*r with u uniform on S^2 and r ~ U[0, r_max].  Hull sizes are n_min..n_max (uniform integer;
 * n_min == n_max for fixed-size configs).  Values are rounded to fp32 so the fp32 and fp64 pools
 * hold identical numbers.  `first_pair` offsets the counter so shards of one logical job agree.
 * hull_off/hull_cnt/pairs are written for the generated pool (pairs are global hull indices of
 * this pool, i.e. 2k, 2k+1).  Pass verts == NULL to only compute sizes: returns the number of
 * vertex scalars the pool needs. */
int64_t gjkepa_synth_pairs(uint64_t seed, int64_t first_pair, int64_t n_pairs,
                           int32_t n_min, int32_t n_max, double r_max,
                           int32_t vert_dtype, void* verts,
                           int64_t* hull_off, int32_t* hull_cnt, int32_t* pairs);

/* Synthetic point clouds for the hull module: n ~ U{n_min..n_max} points per cloud, uniform in the
 * unit ball (shape 0) or on the unit sphere (shape 1); same conventions as gjkepa_synth_pairs
 * (counter-based per global cloud index, fp32-rounded; verts == NULL returns the scalar count). */
int64_t gjkepa_synth_clouds(uint64_t seed, int64_t first_cloud, int64_t n_clouds,
                            int32_t n_min, int32_t n_max, int32_t shape,
                            int32_t vert_dtype, void* verts,
                            int64_t* cloud_off, int32_t* cloud_cnt);

/* Synthetic scene for the broad phase: n_hulls hulls of n ~ U{n_min..n_max} unit-sphere vertices
 * (as gjkepa_synth_pairs' hull A) centred uniformly in the cube [0, box)^3; counter-based per
 * global hull index, fp32-rounded; verts == NULL returns the scalar count. */
int64_t gjkepa_synth_scene(uint64_t seed, int64_t first_hull, int64_t n_hulls,
                           int32_t n_min, int32_t n_max, double box,
                           int32_t vert_dtype, void* verts, int64_t* hull_off, int32_t* hull_cnt);

#ifdef __cplusplus
}
#endif
#endif /* GJKEPA_H */
