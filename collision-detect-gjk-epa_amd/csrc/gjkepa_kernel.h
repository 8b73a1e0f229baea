// gjkepa_kernel.h — host-side interface of the tiered GJK/EPA kernels (internal, not the C-ABI).
//
// Tiers: every pair first runs in tier 0 (hulls up to G*K vertices, EPA polytope up to
// VCAP vertices / FCAP faces).  A pair that does not fit is appended, on the device, to the next
// tier's work list, and so on; the last tier holds the worst case the reference allows
// (6 + 2*99 EPA points, 2*V-4 faces), so it never defers.  Deferral recomputes the pair from
// scratch, so results do not depend on which tier produced them.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

// tier t: G lanes per pair (64/G pairs per wave), K vertices per lane per hull (hull <= G*K),
// EPA polytope capacity VCAP vertices / FCAP faces
#ifndef GJKEPA_T0_G
#define GJKEPA_T0_G 16
#endif
#ifndef GJKEPA_T0_K
#define GJKEPA_T0_K 2
#endif
#ifndef GJKEPA_T0_VCAP
#define GJKEPA_T0_VCAP 40
#endif
#ifndef GJKEPA_T0_FCAP
#define GJKEPA_T0_FCAP 64
#endif
#ifndef GJKEPA_T1_G
#define GJKEPA_T1_G 64
#endif
#ifndef GJKEPA_T1_K
#define GJKEPA_T1_K 1
#endif
#ifndef GJKEPA_T1_VCAP
#define GJKEPA_T1_VCAP 64
#endif
#ifndef GJKEPA_T1_FCAP
#define GJKEPA_T1_FCAP 128
#endif
#ifndef GJKEPA_T2_G
#define GJKEPA_T2_G 64
#endif
#ifndef GJKEPA_T2_K
#define GJKEPA_T2_K 4
#endif
#ifndef GJKEPA_T2_VCAP
#define GJKEPA_T2_VCAP 104
#endif
#ifndef GJKEPA_T2_FCAP
#define GJKEPA_T2_FCAP 208
#endif
#ifndef GJKEPA_T3_G
#define GJKEPA_T3_G 64
#endif
#ifndef GJKEPA_T3_K
#define GJKEPA_T3_K 4
#endif
#ifndef GJKEPA_T3_VCAP
#define GJKEPA_T3_VCAP 208
#endif
#ifndef GJKEPA_T3_FCAP
#define GJKEPA_T3_FCAP 416
#endif
#define GJKEPA_NUM_TIERS 4

struct gjkepa_tier_args {
    int version;
    double tol_ff;
    const void* verts;
    const int64_t* hull_off;
    const int32_t* hull_cnt;
    const int32_t* pairs;
    int64_t n_pairs;
    const int32_t* in_list;    // null: process pairs [0, n_pairs)
    const int32_t* in_count;   // device count of in_list
    int32_t* out_list;         // null on the last tier
    int32_t* out_count;
    void* out;                 // contact records
    int grid;                  // <= 0: occupancy x CUs
    int num_cus;
};

hipError_t gjkepa_launch_tier(int tier, int vert_dtype, int precision, const gjkepa_tier_args& a, hipStream_t s);
