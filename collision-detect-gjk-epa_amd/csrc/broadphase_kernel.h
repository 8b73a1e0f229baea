// broadphase_kernel.h — host-side interface of the device broad phase (internal, not the C-ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

// workspace bytes for n hulls and a max_pairs-long pair list (-1 when the device query fails)
int64_t gjkepa_broadphase_ws_bytes(int64_t n_hulls, int64_t max_pairs);

// enqueue the sphere / sort / sweep / sort / unpack pipeline on `s`; sets *ws_too_small (and
// enqueues nothing) when ws_bytes is below gjkepa_broadphase_ws_bytes(n, max_pairs)
hipError_t gjkepa_enqueue_broadphase(int vert_dtype, const void* verts, const int64_t* hull_off, const int32_t* hull_cnt,
                                     int64_t n, int32_t* pairs, int64_t max_pairs, int64_t* n_pairs, void* ws,
                                     int64_t ws_bytes, hipStream_t s, bool* ws_too_small);
