// contacts_kernel.hip — CDNA4 (gfx950) contact-list compaction.
//
// A narrow-phase batch leaves one fixed-size record per pair, hit or not.  A device consumer (an
// integrator, a contact solver) or a multi-GPU exchange wants only the hits: this pass turns the
// records into a dense, order-preserving list — the indices of the pairs whose collision_ flag is
// set (GJKEPA's collision_ output, GCLIB_GJKEPA.f90:47) and, optionally, their records packed
// contiguously.  Records never leave HBM.
//
// Deterministic two-pass stream compaction, no atomics: count_kernel — one block per 4096-record
// tile, each lane reads the flag byte of its records (a 1-byte load per 64/128-byte record: the pass
// is bound by the record lines it touches) and the block sums them; an exclusive scan of the tile
// counts (rocPRIM via hipCUB); write_kernel — each tile re-reads its flags, ranks them with
// ballot + mbcnt across waves (LDS wave offsets) and writes indices (and records, 16 bytes per lane
// per step) in pair order.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdint>

#include "../../include/gjkepa.h"
#include "contacts_kernel.h"

namespace gk {
namespace ct {

constexpr int BLOCK = 256;
constexpr int PER_THREAD = 16;
constexpr int TILE = BLOCK * PER_THREAD;   // records per tile

__global__ __launch_bounds__(BLOCK) void count_kernel(const uint8_t* __restrict__ rec, int64_t n, int rec_bytes,
                                                      int flag_off, int64_t* __restrict__ tile_counts) {
    __shared__ int wsum[BLOCK / 64];
    const int64_t t0 = (int64_t)blockIdx.x * TILE;
    int c = 0;
#pragma unroll
    for (int j = 0; j < PER_THREAD; ++j) {
        const int64_t k = t0 + (int64_t)j * BLOCK + threadIdx.x;
        if (k < n) c += rec[k * rec_bytes + flag_off] != 0;
    }
    for (int m = 32; m >= 1; m /= 2) c += __shfl_xor(c, m, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x / 64] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        int s = 0;
        for (int w = 0; w < BLOCK / 64; ++w) s += wsum[w];
        tile_counts[blockIdx.x] = s;
    }
}

__global__ __launch_bounds__(BLOCK) void write_kernel(const uint8_t* __restrict__ rec, int64_t n, int rec_bytes,
                                                      int flag_off, const int64_t* __restrict__ tile_offs,
                                                      int64_t n_tiles, int32_t* __restrict__ hit_idx,
                                                      uint8_t* __restrict__ hits, int64_t* __restrict__ n_hits) {
    __shared__ int wcnt[BLOCK / 64];
    const int64_t t0 = (int64_t)blockIdx.x * TILE;
    const int lane = threadIdx.x & 63, wave = threadIdx.x / 64;
    int64_t run = tile_offs[blockIdx.x];
    for (int j = 0; j < PER_THREAD; ++j) {           // step j: records t0 + j*BLOCK .. + BLOCK-1, in order
        const int64_t k = t0 + (int64_t)j * BLOCK + threadIdx.x;
        const bool hit = k < n && rec[k * rec_bytes + flag_off] != 0;
        const uint64_t m = __ballot(hit);
        const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (lane == 0) wcnt[wave] = __popcll(m);
        __syncthreads();
        int before = 0, total = 0;
        for (int w = 0; w < BLOCK / 64; ++w) { before += w < wave ? wcnt[w] : 0; total += wcnt[w]; }
        if (hit) {
            const int64_t pos = run + before + below;
            hit_idx[pos] = (int32_t)k;
            if (hits) {
                const uint4* src = (const uint4*)(rec + k * rec_bytes);
                uint4* dst = (uint4*)(hits + pos * rec_bytes);
                for (int q = 0; q < rec_bytes / 16; ++q) dst[q] = src[q];
            }
        }
        run += total;
        __syncthreads();
    }
    if (blockIdx.x == n_tiles - 1 && threadIdx.x == 0) *n_hits = run;
}

}  // namespace ct
}  // namespace gk

int64_t gjkepa_compact_ws_bytes(int64_t n) {
    const int64_t tiles = (n + gk::ct::TILE - 1) / gk::ct::TILE;
    size_t scan = 0;
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, scan, (const int64_t*)nullptr, (int64_t*)nullptr, (int)(tiles > 0 ? tiles : 1)) != hipSuccess)
        return -1;
    return 2 * ((tiles * 8 + 255) / 256 * 256) + (int64_t)((scan + 255) / 256 * 256);
}

hipError_t gjkepa_enqueue_compact(const void* records, int64_t n, int rec_bytes, int flag_off, int32_t* hit_idx,
                                  void* hits, int64_t* n_hits, void* ws, hipStream_t s) {
    using namespace gk::ct;
    const int64_t tiles = (n + TILE - 1) / TILE;
    const size_t tb = (size_t)((tiles * 8 + 255) / 256 * 256);
    int64_t* counts = (int64_t*)ws;
    int64_t* offs = (int64_t*)((char*)ws + tb);
    void* temp = (char*)ws + 2 * tb;
    size_t scan = 0;
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, scan, counts, offs, (int)tiles, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(count_kernel, dim3((unsigned)tiles), dim3(BLOCK), 0, s, (const uint8_t*)records, n, rec_bytes,
                       flag_off, counts);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipcub::DeviceScan::ExclusiveSum(temp, scan, counts, offs, (int)tiles, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(write_kernel, dim3((unsigned)tiles), dim3(BLOCK), 0, s, (const uint8_t*)records, n, rec_bytes,
                       flag_off, (const int64_t*)offs, tiles, hit_idx, (uint8_t*)hits, n_hits);
    return hipGetLastError();
}
