// broadphase_kernel.hip — CDNA4 (gfx950) device broad phase.
//
// What it computes: the list of hull pairs (a < b) that pass the reference's rough test
// RoughCollisionDetection_SphericalEnvelope (src/GCLIB_GJKEPA.f90:1165-1188): centre = the
// sequential mean of the vertices, radius = max vertex distance from it, pair iff
// NORM2(m_a - m_b) <= r_a + r_b + 1.0.  Same fp64 arithmetic as oracle/gjkepa_oracle.c
// (hull_mean, sphere_test), so the list is identical to the oracle's, in ascending (a, b) order.
//
// Pipeline on one stream, no host synchronisation (graph-capturable):
//   1. sphere_kernel   one thread per hull: centre, radius, x-extent [lo, hi] widened by 0.5 + a
//                      relative margin (the sweep only has to be conservative; the exact test
//                      decides); invalid hulls get lo = +inf so they sort last and match nothing.
//   2. radix sort of (lo, hull) pairs (rocPRIM via hipCUB), then gather of the spheres into
//      x order so the sweep reads consecutive entries.
//   3. sweep_kernel<count>  thread p tests the spheres after it in x order while lo_q <= hi_p;
//      exclusive scan of the counts; sweep_kernel<emit> writes (a << 32 | b) keys at the offsets.
//   4. radix sort of the max_pairs keys (padded with all-ones), unpack to int32 (a, b) pairs.
// The sweep is HBM/L2-streaming integer-and-fp64 work, no MFMA: each thread walks a contiguous
// run of the sorted arrays, so neighbouring threads share cache lines.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cfloat>
#include <cmath>
#include <cstdint>

#include "../../include/gjkepa.h"
#include "broadphase_kernel.h"

namespace gk {
namespace bp {

constexpr double kTol = 1.0;   // TOL of RoughCollisionDetection_SphericalEnvelope (:1172)

template <typename TIn>
__global__ __launch_bounds__(256) void sphere_kernel(const TIn* __restrict__ verts, const int64_t* __restrict__ hull_off,
                                                     const int32_t* __restrict__ hull_cnt, int64_t n_hulls,
                                                     double* __restrict__ cx, double* __restrict__ cy,
                                                     double* __restrict__ cz, double* __restrict__ cr,
                                                     double* __restrict__ lo, double* __restrict__ hi,
                                                     int32_t* __restrict__ idx) {
    for (int64_t h = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; h < n_hulls; h += (int64_t)gridDim.x * blockDim.x) {
        const int n = hull_cnt[h];
        double mx = NAN, my = NAN, mz = NAN, r = NAN;
        if (n >= 1 && n <= GJKEPA_MAX_HULL_VERTS) {
            const TIn* p = verts + hull_off[h];
            // SUM(p(:,k)) / SIZE(p,1), sequential in index order (:1175-1176)
            double sx = 0.0, sy = 0.0, sz = 0.0;
            for (int i = 0; i < n; ++i) { sx += (double)p[i]; sy += (double)p[n + i]; sz += (double)p[2 * n + i]; }
            const double dn = (double)n;
            mx = sx / dn; my = sy / dn; mz = sz / dn;
            // MAXVAL(NORM2(p(i,:) - mp)) (:1179-1182)
            r = -DBL_MAX;
            for (int i = 0; i < n; ++i) {
                const double dx = (double)p[i] - mx, dy = (double)p[n + i] - my, dz = (double)p[2 * n + i] - mz;
                const double t = ::sqrt(dx * dx + dy * dy + dz * dz);
                r = t > r ? t : r;
            }
        }
        cx[h] = mx; cy[h] = my; cz[h] = mz; cr[h] = r;
        const bool ok = isfinite(mx) && isfinite(my) && isfinite(mz) && isfinite(r);
        // conservative x extent: rounding of the exact test is ~1e-16 relative, the margin 1e-9
        const double half = 0.5 * kTol + r, e = 1e-9 * (1.0 + fabs(mx) + r);
        lo[h] = ok ? (mx - half) - e : INFINITY;
        hi[h] = ok ? (mx + half) + e : -INFINITY;
        idx[h] = (int32_t)h;
    }
}

__global__ __launch_bounds__(256) void gather_kernel(int64_t n, const int32_t* __restrict__ order,
                                                     const double* __restrict__ cx, const double* __restrict__ cy,
                                                     const double* __restrict__ cz, const double* __restrict__ cr,
                                                     const double* __restrict__ hi, double* __restrict__ sx,
                                                     double* __restrict__ sy, double* __restrict__ sz,
                                                     double* __restrict__ sr, double* __restrict__ shi) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const int32_t h = order[p];
        sx[p] = cx[h]; sy[p] = cy[h]; sz[p] = cz[h]; sr[p] = cr[h]; shi[p] = hi[h];
    }
}

// thread p: spheres q > p in x order while slo[q] <= shi[p]; EMIT = false counts, true writes keys
template <bool EMIT>
__global__ __launch_bounds__(256) void sweep_kernel(int64_t n, const double* __restrict__ slo,
                                                    const double* __restrict__ shi, const double* __restrict__ sx,
                                                    const double* __restrict__ sy, const double* __restrict__ sz,
                                                    const double* __restrict__ sr, const int32_t* __restrict__ order,
                                                    int64_t* __restrict__ counts, const int64_t* __restrict__ offs,
                                                    uint64_t* __restrict__ keys, int64_t max_pairs) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const double h = shi[p], x = sx[p], y = sy[p], z = sz[p], r = sr[p];
        int64_t c = 0, o = EMIT ? offs[p] : 0;
        const uint32_t a0 = EMIT ? (uint32_t)order[p] : 0u;
        for (int64_t q = p + 1; q < n && slo[q] <= h; ++q) {
            // NORM2(mp1 - mp2) <= r1 + r2 + TOL (:1185); symmetric bit for bit in (p, q)
            const double dx = x - sx[q], dy = y - sy[q], dz = z - sz[q];
            if (!(::sqrt(dx * dx + dy * dy + dz * dz) <= r + sr[q] + kTol)) continue;
            if constexpr (EMIT) {
                if (o + c < max_pairs) {
                    const uint32_t b0 = (uint32_t)order[q];
                    const uint32_t a = a0 < b0 ? a0 : b0, b = a0 < b0 ? b0 : a0;
                    keys[o + c] = ((uint64_t)a << 32) | b;
                }
            }
            ++c;
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
    size_t cx, cy, cz, cr, lo, hi, idx, slo, order, sx, sy, sz, sr, shi, counts, offs, keys, keys2, temp, total;
    size_t sort1, scan, sort2;
};

hipError_t temp_sizes(int64_t n, int64_t max_pairs, size_t& sort1, size_t& scan, size_t& sort2) {
    hipError_t e;
    sort1 = scan = sort2 = 0;
    if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, sort1, (const double*)nullptr, (double*)nullptr,
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
    L.cx = take(d); L.cy = take(d); L.cz = take(d); L.cr = take(d); L.lo = take(d); L.hi = take(d);
    L.idx = take(i); L.slo = take(d); L.order = take(i);
    L.sx = take(d); L.sy = take(d); L.sz = take(d); L.sr = take(d); L.shi = take(d);
    L.counts = take((size_t)(n + 1) * 8); L.offs = take((size_t)(n + 1) * 8);
    L.keys = take((size_t)max_pairs * 8); L.keys2 = take((size_t)max_pairs * 8);
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
    if (vert_dtype == GJKEPA_DTYPE_F32)
        hipLaunchKernelGGL(sphere_kernel<float>, dim3(nb), dim3(256), 0, s, (const float*)verts, hull_off, hull_cnt, n,
                           at<double>(ws, L.cx), at<double>(ws, L.cy), at<double>(ws, L.cz), at<double>(ws, L.cr),
                           at<double>(ws, L.lo), at<double>(ws, L.hi), at<int32_t>(ws, L.idx));
    else
        hipLaunchKernelGGL(sphere_kernel<double>, dim3(nb), dim3(256), 0, s, (const double*)verts, hull_off, hull_cnt, n,
                           at<double>(ws, L.cx), at<double>(ws, L.cy), at<double>(ws, L.cz), at<double>(ws, L.cr),
                           at<double>(ws, L.lo), at<double>(ws, L.hi), at<int32_t>(ws, L.idx));
    if ((e = hipGetLastError()) != hipSuccess) return e;
    size_t tb = L.sort1;
    if ((e = hipcub::DeviceRadixSort::SortPairs(at<void>(ws, L.temp), tb, at<double>(ws, L.lo), at<double>(ws, L.slo),
                                                at<int32_t>(ws, L.idx), at<int32_t>(ws, L.order), (int)n, 0, 64, s)) != hipSuccess)
        return e;
    hipLaunchKernelGGL(gather_kernel, dim3(nb), dim3(256), 0, s, n, at<int32_t>(ws, L.order), at<double>(ws, L.cx),
                       at<double>(ws, L.cy), at<double>(ws, L.cz), at<double>(ws, L.cr), at<double>(ws, L.hi),
                       at<double>(ws, L.sx), at<double>(ws, L.sy), at<double>(ws, L.sz), at<double>(ws, L.sr),
                       at<double>(ws, L.shi));
    if ((e = hipMemsetAsync(at<int64_t>(ws, L.counts) + n, 0, 8, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(sweep_kernel<false>, dim3(nb), dim3(256), 0, s, n, at<double>(ws, L.slo), at<double>(ws, L.shi),
                       at<double>(ws, L.sx), at<double>(ws, L.sy), at<double>(ws, L.sz), at<double>(ws, L.sr),
                       at<int32_t>(ws, L.order), at<int64_t>(ws, L.counts), (const int64_t*)nullptr, (uint64_t*)nullptr,
                       max_pairs);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    tb = L.scan;
    if ((e = hipcub::DeviceScan::ExclusiveSum(at<void>(ws, L.temp), tb, at<int64_t>(ws, L.counts),
                                              at<int64_t>(ws, L.offs), (int)(n + 1), s)) != hipSuccess)
        return e;
    hipLaunchKernelGGL(total_kernel, dim3(1), dim3(64), 0, s, at<int64_t>(ws, L.offs), n, n_pairs);
    if (max_pairs > 0) {
        if ((e = hipMemsetAsync(at<uint64_t>(ws, L.keys), 0xFF, (size_t)max_pairs * 8, s)) != hipSuccess) return e;
        hipLaunchKernelGGL(sweep_kernel<true>, dim3(nb), dim3(256), 0, s, n, at<double>(ws, L.slo), at<double>(ws, L.shi),
                           at<double>(ws, L.sx), at<double>(ws, L.sy), at<double>(ws, L.sz), at<double>(ws, L.sr),
                           at<int32_t>(ws, L.order), (int64_t*)nullptr, at<int64_t>(ws, L.offs), at<uint64_t>(ws, L.keys),
                           max_pairs);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        tb = L.sort2;
        if ((e = hipcub::DeviceRadixSort::SortKeys(at<void>(ws, L.temp), tb, at<uint64_t>(ws, L.keys),
                                                   at<uint64_t>(ws, L.keys2), (int)max_pairs, 0, 64, s)) != hipSuccess)
            return e;
        hipLaunchKernelGGL(unpack_kernel, dim3(blocks_for(max_pairs)), dim3(256), 0, s, at<uint64_t>(ws, L.keys2),
                           (const int64_t*)n_pairs, max_pairs, pairs);
    }
    return hipGetLastError();
}
