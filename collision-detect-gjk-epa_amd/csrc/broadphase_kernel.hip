// broadphase_kernel.hip — CDNA4 (gfx950) device broad phase.
//
// What it computes: the list of hull pairs (a < b) that pass the reference's rough test
// RoughCollisionDetection_SphericalEnvelope (src/GCLIB_GJKEPA.f90:1165-1188): centre = the
// sequential mean of the vertices, radius = max vertex distance from it, pair iff
// NORM2(m_a - m_b) <= r_a + r_b + 1.0.  Same fp64 arithmetic as oracle/gjkepa_oracle.c
// (hull_mean, sphere_test), so the list is identical to the oracle's, in ascending (a, b) order.
//
// Pipeline on one stream, no host synchronisation (graph-capturable):
//   1. sphere_kernel  16 lanes per hull (LDS-staged coalesced loads): centre, radius, validity;
//                     the largest radius (atomicMax on the bit pattern, one atomic per block).
//   2. key_kernel     uniform grid of edge 2 r_max + 1 (every passing pair lies in neighbouring
//                     cells); 63-bit cell keys (iz, iy, ix), coordinates wrapped at 2^21.
//   3. radix sort of (cell key, hull) pairs (rocPRIM via hipCUB); gather of the spheres into cell
//      order, so neighbouring threads read neighbouring entries.
//   4. cell_table_kernel: hash table (cell key -> first sorted position) from the segment starts;
//      grid_kernel<count>: thread p walks the 9 cell rows around its cell (ix-1..ix+1 is one key
//      range: first non-empty cell by table lookup, then forward) and tests the hulls there with a
//      larger index; exclusive scan of the counts; grid_kernel<emit> writes (a << 32 | b) keys.
//   5. radix sort of the max_pairs keys (padded with all-ones); unpack to int32 (a, b) pairs.
// Memory-latency-bound integer / fp64 work (binary searches, short candidate runs), no MFMA.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cfloat>
#include <cmath>
#include <cstdint>

#include "../../include/gjkepa.h"
#include "broadphase_kernel.h"

#define DEV_BP __device__ __forceinline__

namespace gk {
namespace bp {

constexpr double kTol = 1.0;               // TOL of RoughCollisionDetection_SphericalEnvelope (:1172)
constexpr uint64_t kMask = (1ull << 21) - 1;
constexpr uint64_t kInvalid = ~0ull;

DEV_BP uint64_t cell_key(uint64_t ix, uint64_t iy, uint64_t iz) { return ((iz & kMask) << 42) | ((iy & kMask) << 21) | (ix & kMask); }

// centre, radius and validity of every hull; the largest radius via one atomic per block.
// A group of SG lanes owns a hull: the group stages the hull's 3n scalars in LDS with coalesced
// loads, three lanes form the x / y / z sums sequentially in index order (the reference's SUM, so
// the centre is bit-exact), then every lane takes vertices gl, gl+SG, ... for the radius (a max,
// order-free).  One thread per hull instead would issue 64 scattered loads per instruction.
constexpr int SG = 16;
constexpr int SPHERE_BLOCK = 128;   // 8 hulls per block
constexpr int SPHERE_STAGE = 64;    // hulls of up to 64 vertices are staged: 6 KB (fp32) of LDS per block
template <typename TIn>
__global__ __launch_bounds__(SPHERE_BLOCK) void sphere_kernel(const TIn* __restrict__ verts, const int64_t* __restrict__ hull_off,
                                                              const int32_t* __restrict__ hull_cnt, int64_t n_hulls,
                                                              double* __restrict__ cx, double* __restrict__ cy,
                                                              double* __restrict__ cz, double* __restrict__ cr,
                                                              unsigned long long* __restrict__ rmax_bits) {
    constexpr int GPB = SPHERE_BLOCK / SG;
    __shared__ TIn stage[GPB][3 * SPHERE_STAGE];
    __shared__ double cen[GPB][3];
    __shared__ unsigned long long blk;
    const int gl = threadIdx.x % SG, grp = threadIdx.x / SG;
    if (threadIdx.x == 0) blk = 0;
    __syncthreads();
    unsigned long long mine = 0;
    for (int64_t base = blockIdx.x * (int64_t)GPB; base < n_hulls; base += (int64_t)gridDim.x * GPB) {
        const int64_t h = base + grp;
        const int n = h < n_hulls ? hull_cnt[h] : 0;
        const bool in = h < n_hulls && n >= 1 && n <= GJKEPA_MAX_HULL_VERTS;
        const TIn* p = in ? verts + hull_off[h] : verts;
        if (in && n <= SPHERE_STAGE)
            for (int i = gl; i < 3 * n; i += SG) stage[grp][i] = p[i];
        __syncthreads();
        const TIn* q = n <= SPHERE_STAGE ? stage[grp] : p;   // larger hulls are read in place
        if (in && gl < 3) {   // SUM(p(:,k)) / SIZE(p,1), sequential in index order (:1175-1176)
            const TIn* col = q + gl * n;
            double sum = 0.0;
            int i = 0;
            for (; i + 8 <= n; i += 8) {   // loads batched ahead of the in-order adds
                TIn v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = col[i + u];
#pragma unroll
                for (int u = 0; u < 8; ++u) sum += (double)v[u];
            }
            for (; i < n; ++i) sum += (double)col[i];
            cen[grp][gl] = sum / (double)n;
        }
        __syncthreads();
        double r = -DBL_MAX;
        const double mx = cen[grp][0], my = cen[grp][1], mz = cen[grp][2];
        if (in) {             // MAXVAL(NORM2(p(i,:) - mp)) (:1179-1182)
            for (int i = gl; i < n; i += SG) {
                const double dx = (double)q[i] - mx, dy = (double)q[n + i] - my, dz = (double)q[2 * n + i] - mz;
                const double t = ::sqrt(dx * dx + dy * dy + dz * dz);
                r = t > r ? t : r;
            }
        }
#pragma unroll
        for (int m = SG / 2; m >= 1; m /= 2) {
            const double o = __shfl_xor(r, m, SG);
            r = o > r ? o : r;
        }
        if (h < n_hulls && gl == 0) {
            const bool ok = in && isfinite(mx) && isfinite(my) && isfinite(mz) && isfinite(r);
            cx[h] = in ? mx : NAN; cy[h] = in ? my : NAN; cz[h] = in ? mz : NAN; cr[h] = ok ? r : NAN;
            if (ok) {   // r >= 0: the bit patterns of non-negative doubles order like the values
                const unsigned long long b = (unsigned long long)__double_as_longlong(r);
                mine = b > mine ? b : mine;
            }
        }
        __syncthreads();
    }
    atomicMax(&blk, mine);
    __syncthreads();
    if (threadIdx.x == 0 && blk) atomicMax(rmax_bits, blk);
}

// grid cell of every hull: edge 2 r_max + 1 (widened by a relative margin), so every pair that can
// pass the test lies in neighbouring cells; cell coordinates wrap at 2^21 (aliasing only adds
// candidates).  Key = (iz, iy, ix) with ix fastest: a cell row ix-1..ix+1 is one key range.
__global__ __launch_bounds__(256) void key_kernel(int64_t n, const double* __restrict__ cx, const double* __restrict__ cy,
                                                  const double* __restrict__ cz, const double* __restrict__ cr,
                                                  const unsigned long long* __restrict__ rmax_bits,
                                                  double* __restrict__ cell_out, uint64_t* __restrict__ keys,
                                                  int32_t* __restrict__ idx) {
    const double rmax = __longlong_as_double((long long)*rmax_bits);
    const double cell = (2.0 * rmax + kTol) * (1.0 + 1e-9) + 1e-9;
    for (int64_t h = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; h < n; h += (int64_t)gridDim.x * blockDim.x) {
        uint64_t k = kInvalid;
        if (!isnan(cr[h]))
            k = cell_key((uint64_t)(int64_t)floor(cx[h] / cell), (uint64_t)(int64_t)floor(cy[h] / cell),
                         (uint64_t)(int64_t)floor(cz[h] / cell));
        keys[h] = k;
        idx[h] = (int32_t)h;
        if (h == 0) *cell_out = cell;
    }
}

__global__ __launch_bounds__(256) void gather_kernel(int64_t n, const int32_t* __restrict__ order,
                                                     const double* __restrict__ cx, const double* __restrict__ cy,
                                                     const double* __restrict__ cz, const double* __restrict__ cr,
                                                     double* __restrict__ sx, double* __restrict__ sy,
                                                     double* __restrict__ sz, double* __restrict__ sr) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const int32_t h = order[p];
        sx[p] = cx[h]; sy[p] = cy[h]; sz[p] = cz[h]; sr[p] = cr[h];
    }
}

// Cell table: open-addressing hash (linear probing) from a cell key to the first sorted position
// of that cell, built from the segment starts of the sorted keys; a lookup costs ~1 probe instead of
// a 20-step binary search over the whole key array.
DEV_BP uint64_t mix64(uint64_t x) {
    x ^= x >> 31; x *= 0x7FB5D329728EA185ull; x ^= x >> 27; x *= 0x81DADEF4BC2DD44Dull; x ^= x >> 33;
    return x;
}

__global__ __launch_bounds__(256) void cell_table_kernel(int64_t n, const uint64_t* __restrict__ keys,
                                                         unsigned long long* __restrict__ tkeys,
                                                         int32_t* __restrict__ tstart, uint64_t tmask) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t k = keys[p];
        if (k == kInvalid || (p > 0 && keys[p - 1] == k)) continue;
        for (uint64_t h = mix64(k) & tmask;; h = (h + 1) & tmask) {
            const unsigned long long prev = atomicCAS(&tkeys[h], (unsigned long long)kInvalid, (unsigned long long)k);
            if (prev == (unsigned long long)kInvalid) { tstart[h] = (int32_t)p; break; }
        }
    }
}

// first sorted position of cell k, -1 when the cell is empty
DEV_BP int64_t cell_start(const unsigned long long* __restrict__ tkeys, const int32_t* __restrict__ tstart,
                          uint64_t tmask, uint64_t k) {
    for (uint64_t h = mix64(k) & tmask;; h = (h + 1) & tmask) {
        const uint64_t t = tkeys[h];
        if (t == k) return tstart[h];
        if (t == kInvalid) return -1;
    }
}

// the hulls q from sorted position q0 on while their cell key is <= kh that form a passing pair with hull a
// (larger index); returns how many, writing their keys from out[o] on when EMIT
template <bool EMIT>
DEV_BP int64_t visit_range(int64_t q0, uint64_t kh, int64_t n, const uint64_t* __restrict__ keys,
                           const double* __restrict__ sx, const double* __restrict__ sy, const double* __restrict__ sz,
                           const double* __restrict__ sr, const int32_t* __restrict__ order, int32_t a, double x,
                           double y, double z, double r, uint64_t* __restrict__ out, int64_t o, int64_t max_pairs) {
    int64_t c = 0;
    for (int64_t q = q0; q < n && keys[q] <= kh; ++q) {
        const int32_t b = order[q];
        if (b <= a) continue;
        // NORM2(mp1 - mp2) <= r1 + r2 + TOL (:1185), mp1 = hull a
        const double dx = x - sx[q], dy = y - sy[q], dz = z - sz[q];
        if (!(::sqrt(dx * dx + dy * dy + dz * dz) <= r + sr[q] + kTol)) continue;
        if constexpr (EMIT) {
            if (o + c < max_pairs) out[o + c] = ((uint64_t)(uint32_t)a << 32) | (uint32_t)b;
        }
        ++c;
    }
    return c;
}

// thread p (cell-sorted hull): the hulls of the 27 neighbouring cells with a larger index that
// pass the exact test; EMIT = false counts, true writes (a << 32 | b) keys at the thread's offset
template <bool EMIT>
__global__ __launch_bounds__(256) void grid_kernel(int64_t n, const uint64_t* __restrict__ keys,
                                                   const double* __restrict__ sx, const double* __restrict__ sy,
                                                   const double* __restrict__ sz, const double* __restrict__ sr,
                                                   const int32_t* __restrict__ order,
                                                   const unsigned long long* __restrict__ tkeys,
                                                   const int32_t* __restrict__ tstart, uint64_t tmask,
                                                   int64_t* __restrict__ counts, const int64_t* __restrict__ offs,
                                                   uint64_t* __restrict__ out, int64_t max_pairs) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t k = keys[p];
        int64_t c = 0;
        if (k != kInvalid) {
            const double x = sx[p], y = sy[p], z = sz[p], r = sr[p];
            const int32_t a = order[p];
            const int64_t o = EMIT ? offs[p] : 0;
            const uint64_t ix = k & kMask, iy = (k >> 21) & kMask, iz = k >> 42;
            const bool row = ix >= 1 && ix + 1 <= kMask;          // ix-1..ix+1 contiguous in key order
            for (int t = 0; t < 9; ++t) {
                const uint64_t jy = iy + (uint64_t)(t % 3) - 1, jz = iz + (uint64_t)(t / 3) - 1;
                if (row) {   // the row's first non-empty cell, then forward through the row
                    int64_t q0 = -1;
                    for (uint64_t jx = ix - 1; jx != ix + 2 && q0 < 0; ++jx) q0 = cell_start(tkeys, tstart, tmask, cell_key(jx, jy, jz));
                    if (q0 >= 0)
                        c += visit_range<EMIT>(q0, cell_key(ix + 1, jy, jz), n, keys, sx, sy, sz, sr, order, a, x, y, z,
                                               r, out, o + c, max_pairs);
                } else {     // the row wraps at 2^21: its three cells separately
                    for (uint64_t jx = ix - 1; jx != ix + 2; ++jx) {
                        const uint64_t kc = cell_key(jx, jy, jz);
                        const int64_t q0 = cell_start(tkeys, tstart, tmask, kc);
                        if (q0 >= 0)
                            c += visit_range<EMIT>(q0, kc, n, keys, sx, sy, sz, sr, order, a, x, y, z, r, out, o + c,
                                                   max_pairs);
                    }
                }
            }
        }
        if constexpr (!EMIT) counts[p] = c;
    }
}

__global__ void total_kernel(const int64_t* __restrict__ offs, int64_t n, int64_t* __restrict__ n_pairs) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *n_pairs = offs[n];
}

__global__ __launch_bounds__(256) void unpack_kernel(const uint64_t* __restrict__ keys, const int64_t* __restrict__ n_pairs,
                                                     int64_t max_pairs, int32_t* __restrict__ pairs) {
    const int64_t m = *n_pairs < max_pairs ? *n_pairs : max_pairs;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t v = keys[k];
        pairs[2 * k] = (int32_t)(v >> 32);
        pairs[2 * k + 1] = (int32_t)(v & 0xffffffffu);
    }
}

}  // namespace bp
}  // namespace gk

namespace {

constexpr size_t kAlign = 256;
size_t up(size_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

struct Layout {
    size_t cx, cy, cz, cr, rmax, cell, keys0, idx, skeys, order, sx, sy, sz, sr, counts, offs, tkeys, tstart, pk, pk2,
        temp, total;
    uint64_t tsize;
    size_t sort1, scan, sort2;
};

hipError_t temp_sizes(int64_t n, int64_t max_pairs, size_t& sort1, size_t& scan, size_t& sort2) {
    hipError_t e;
    sort1 = scan = sort2 = 0;
    if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, sort1, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                                (const int32_t*)nullptr, (int32_t*)nullptr, (int)n)) != hipSuccess)
        return e;
    if ((e = hipcub::DeviceScan::ExclusiveSum(nullptr, scan, (const int64_t*)nullptr, (int64_t*)nullptr, (int)(n + 1))) != hipSuccess)
        return e;
    return hipcub::DeviceRadixSort::SortKeys(nullptr, sort2, (const uint64_t*)nullptr, (uint64_t*)nullptr, (int)max_pairs);
}

Layout layout(int64_t n, int64_t max_pairs, size_t sort1, size_t scan, size_t sort2) {
    Layout L{};
    size_t o = 0;
    auto take = [&](size_t bytes) { const size_t at = o; o += up(bytes); return at; };
    const size_t d = (size_t)n * 8, i = (size_t)n * 4;
    L.cx = take(d); L.cy = take(d); L.cz = take(d); L.cr = take(d); L.rmax = take(8); L.cell = take(8);
    L.keys0 = take(d); L.idx = take(i); L.skeys = take(d); L.order = take(i);
    L.sx = take(d); L.sy = take(d); L.sz = take(d); L.sr = take(d);
    L.counts = take((size_t)(n + 1) * 8); L.offs = take((size_t)(n + 1) * 8);
    L.tsize = 1024;
    while (L.tsize < 2 * (uint64_t)n) L.tsize *= 2;           // load factor <= 1/2
    L.tkeys = take(L.tsize * 8); L.tstart = take(L.tsize * 4);
    L.pk = take((size_t)max_pairs * 8); L.pk2 = take((size_t)max_pairs * 8);
    L.sort1 = sort1; L.scan = scan; L.sort2 = sort2;
    L.temp = take(std::max(sort1, std::max(scan, sort2)));
    L.total = o;
    return L;
}

template <typename T> T* at(void* ws, size_t off) { return (T*)((char*)ws + off); }

int blocks_for(int64_t n) {
    const int64_t b = (n + 255) / 256;
    return (int)(b < 1 ? 1 : b > 65536 ? 65536 : b);
}

}  // namespace

int64_t gjkepa_broadphase_ws_bytes(int64_t n_hulls, int64_t max_pairs) {
    size_t s1, sc, s2;
    if (temp_sizes(n_hulls, max_pairs, s1, sc, s2) != hipSuccess) return -1;
    return (int64_t)layout(n_hulls, max_pairs, s1, sc, s2).total;
}

hipError_t gjkepa_enqueue_broadphase(int vert_dtype, const void* verts, const int64_t* hull_off, const int32_t* hull_cnt,
                                     int64_t n, int32_t* pairs, int64_t max_pairs, int64_t* n_pairs, void* ws,
                                     int64_t ws_bytes, hipStream_t s, bool* ws_too_small) {
    using namespace gk::bp;
    size_t s1, sc, s2;
    hipError_t e = temp_sizes(n, max_pairs, s1, sc, s2);
    if (e != hipSuccess) return e;
    const Layout L = layout(n, max_pairs, s1, sc, s2);
    *ws_too_small = (int64_t)L.total > ws_bytes;
    if (*ws_too_small) return hipSuccess;
    const int nb = blocks_for(n);
    if ((e = hipMemsetAsync(at<void>(ws, L.rmax), 0, 8, s)) != hipSuccess) return e;
    auto* rmax = at<unsigned long long>(ws, L.rmax);
    const int nbs = blocks_for((n + SPHERE_BLOCK / SG - 1) / (SPHERE_BLOCK / SG) * 256);   // one block per SPHERE_BLOCK / SG hulls
    if (vert_dtype == GJKEPA_DTYPE_F32)
        hipLaunchKernelGGL(sphere_kernel<float>, dim3(nbs), dim3(SPHERE_BLOCK), 0, s, (const float*)verts, hull_off, hull_cnt, n,
                           at<double>(ws, L.cx), at<double>(ws, L.cy), at<double>(ws, L.cz), at<double>(ws, L.cr), rmax);
    else
        hipLaunchKernelGGL(sphere_kernel<double>, dim3(nbs), dim3(SPHERE_BLOCK), 0, s, (const double*)verts, hull_off, hull_cnt, n,
                           at<double>(ws, L.cx), at<double>(ws, L.cy), at<double>(ws, L.cz), at<double>(ws, L.cr), rmax);
    hipLaunchKernelGGL(key_kernel, dim3(nb), dim3(256), 0, s, n, at<double>(ws, L.cx), at<double>(ws, L.cy),
                       at<double>(ws, L.cz), at<double>(ws, L.cr), (const unsigned long long*)rmax, at<double>(ws, L.cell),
                       at<uint64_t>(ws, L.keys0), at<int32_t>(ws, L.idx));
    if ((e = hipGetLastError()) != hipSuccess) return e;
    size_t tb = L.sort1;
    if ((e = hipcub::DeviceRadixSort::SortPairs(at<void>(ws, L.temp), tb, at<uint64_t>(ws, L.keys0),
                                                at<uint64_t>(ws, L.skeys), at<int32_t>(ws, L.idx),
                                                at<int32_t>(ws, L.order), (int)n, 0, 64, s)) != hipSuccess)
        return e;
    hipLaunchKernelGGL(gather_kernel, dim3(nb), dim3(256), 0, s, n, at<int32_t>(ws, L.order), at<double>(ws, L.cx),
                       at<double>(ws, L.cy), at<double>(ws, L.cz), at<double>(ws, L.cr), at<double>(ws, L.sx),
                       at<double>(ws, L.sy), at<double>(ws, L.sz), at<double>(ws, L.sr));
    if ((e = hipMemsetAsync(at<int64_t>(ws, L.counts) + n, 0, 8, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(at<void>(ws, L.tkeys), 0xFF, L.tsize * 8, s)) != hipSuccess) return e;
    const uint64_t tmask = L.tsize - 1;
    hipLaunchKernelGGL(cell_table_kernel, dim3(nb), dim3(256), 0, s, n, (const uint64_t*)at<uint64_t>(ws, L.skeys),
                       at<unsigned long long>(ws, L.tkeys), at<int32_t>(ws, L.tstart), tmask);
    hipLaunchKernelGGL(grid_kernel<false>, dim3(nb), dim3(256), 0, s, n, at<uint64_t>(ws, L.skeys), at<double>(ws, L.sx),
                       at<double>(ws, L.sy), at<double>(ws, L.sz), at<double>(ws, L.sr), at<int32_t>(ws, L.order),
                       (const unsigned long long*)at<unsigned long long>(ws, L.tkeys), (const int32_t*)at<int32_t>(ws, L.tstart),
                       tmask, at<int64_t>(ws, L.counts), (const int64_t*)nullptr, (uint64_t*)nullptr, max_pairs);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    tb = L.scan;
    if ((e = hipcub::DeviceScan::ExclusiveSum(at<void>(ws, L.temp), tb, at<int64_t>(ws, L.counts),
                                              at<int64_t>(ws, L.offs), (int)(n + 1), s)) != hipSuccess)
        return e;
    hipLaunchKernelGGL(total_kernel, dim3(1), dim3(64), 0, s, at<int64_t>(ws, L.offs), n, n_pairs);
    if (max_pairs > 0) {
        if ((e = hipMemsetAsync(at<uint64_t>(ws, L.pk), 0xFF, (size_t)max_pairs * 8, s)) != hipSuccess) return e;
        hipLaunchKernelGGL(grid_kernel<true>, dim3(nb), dim3(256), 0, s, n, at<uint64_t>(ws, L.skeys), at<double>(ws, L.sx),
                           at<double>(ws, L.sy), at<double>(ws, L.sz), at<double>(ws, L.sr), at<int32_t>(ws, L.order),
                           (const unsigned long long*)at<unsigned long long>(ws, L.tkeys),
                           (const int32_t*)at<int32_t>(ws, L.tstart), tmask, (int64_t*)nullptr, at<int64_t>(ws, L.offs),
                           at<uint64_t>(ws, L.pk), max_pairs);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        tb = L.sort2;
        if ((e = hipcub::DeviceRadixSort::SortKeys(at<void>(ws, L.temp), tb, at<uint64_t>(ws, L.pk),
                                                   at<uint64_t>(ws, L.pk2), (int)max_pairs, 0, 64, s)) != hipSuccess)
            return e;
        hipLaunchKernelGGL(unpack_kernel, dim3(blocks_for(max_pairs)), dim3(256), 0, s, at<uint64_t>(ws, L.pk2),
                           (const int64_t*)n_pairs, max_pairs, pairs);
    }
    return hipGetLastError();
}
