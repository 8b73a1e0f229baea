// hull_kernel.h — host-side interface of the batched convex-hull kernels (internal, not the C-ABI).
//
// Two tiers over the same cloud list: tier 0 (G0 lanes per cloud, clouds of <= G0*K0 points, plus
// every BAD_INPUT cloud) and tier 1 (one wave per cloud, up to GJKEPA_HULL_MAX_POINTS points).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#ifndef GJKEPA_H0_G
#define GJKEPA_H0_G 16
#endif
#ifndef GJKEPA_H0_K
#define GJKEPA_H0_K 4
#endif
#define GJKEPA_H1_G 64
#define GJKEPA_H1_K 4

struct gjkepa_hull_args {
    const void* points;
    const int64_t* cloud_off;
    const int32_t* cloud_cnt;
    int64_t n_clouds;
    const int64_t* face_off;
    int32_t* faces;
    int32_t* n_faces;
    int32_t* n_verts;
    int8_t* status;
    void* hull_verts;           // optional
    int32_t* vert_idx;          // optional
    int num_cus;
    int tier;                   // set by the launcher
    int lo;                     // tier 1: clouds with lo < n
};

hipError_t gjkepa_launch_hull(int vert_dtype, const gjkepa_hull_args& a, hipStream_t s);
