// contacts_kernel.h — host-side interface of the contact-list compaction (internal, not the C-ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

// workspace bytes for compacting n records (-1 when the device query fails)
int64_t gjkepa_compact_ws_bytes(int64_t n);

// enqueue count / scan / write on `s` (n >= 1); hits may be null (indices only)
hipError_t gjkepa_enqueue_compact(const void* records, int64_t n, int rec_bytes, int flag_off, int32_t* hit_idx,
                                  void* hits, int64_t* n_hits, void* ws, hipStream_t s);
