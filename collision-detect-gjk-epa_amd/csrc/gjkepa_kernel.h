// gjkepa_kernel.h — host-side interface of the tiered GJK/EPA kernels (internal, not the C-ABI).
//
// Tiers: every pair first runs in tier 0 (hulls up to 64*T0_K vertices, EPA polytope up to
// T0_VCAP vertices / T0_FCAP faces).  A pair that does not fit is appended, on the device, to
// tier 1's work list, and so on; tier 2 holds the worst case the reference allows
// (6 + 2*99 EPA points, 2*V-4 faces), so it never defers.  Deferral recomputes the pair from
// scratch, so results do not depend on which tier produced them.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#define GJKEPA_T0_K 1
#define GJKEPA_T0_VCAP 64
#define GJKEPA_T0_FCAP 128
#define GJKEPA_T1_K 4
#define GJKEPA_T1_VCAP 96
#define GJKEPA_T1_FCAP 192
#define GJKEPA_T2_K 4
#define GJKEPA_T2_VCAP 208
#define GJKEPA_T2_FCAP 416
#define GJKEPA_NUM_TIERS 3

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
size_t gjkepa_tier_lds_bytes(int tier, int precision);
