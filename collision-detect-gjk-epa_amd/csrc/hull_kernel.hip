// hull_kernel.hip — CDNA4 (gfx950) batched convex hulls.
//
// What it computes: for every point cloud of a pool, the convex hull the reference obtains from
// GCLIB_QuickHull::QuickHull and the vertex set GCLIB_DeHull::getHullMeshesVertex reads back
// (GCLIB_GJKEPA.f90:920, :950; unvendored modules).  The algorithm is fixed in include/gjkepa.h
// (QuickHull in global furthest-point order, fp64, absolute eps) and restated scalar by
// oracle/gjkepa_oracle.c (qh_cloud), which this file follows operation for operation, so results
// compare bit for bit (faces, their order, vertex sets, statuses).
//
// Mapping onto the wavefront.  A group of G lanes owns one cloud (64/G clouds per wave):
//   * points: lane l owns points l, l+G, ... (K per lane): coordinates, assigned face slot and
//     distance above it in registers; an LDS copy of the coordinates for random access.
//   * faces: slot s (packed vertex ids + unit normal) in the group's LDS slice, up to 2*G*K - 4.
//     Visibility is lane-parallel over slots (row r = slots r*G .. r*G+G-1); the visible list
//     is built in slot order with ballot + mbcnt; horizon edges are lane-parallel over
//     (visible face, edge) items with a twin search over the visible list (LDS broadcasts).
//   * eye selection and the initial tetrahedron's extreme points are group (value, index)
//     reductions on DPP / permlane butterflies with the lowest index winning ties (gk_common.h).
// Work distribution: a wave takes 64-cloud chunks (grid-stride), ballots the clouds whose size
// fits this tier and hands them to its groups in cloud order.  Tier 0 (G = 16, <= 64 points) also
// answers BAD_INPUT clouds; tier 1 (G = 64, <= 256 points) takes the rest.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdint>

#include "../../include/gjkepa.h"
#include "gk_common.h"
#include "hull_kernel.h"

namespace gk {
namespace qh {

constexpr uint32_t DEAD = 0xFFFFFFFFu;
DEV uint32_t pack3(int a, int b, int c) { return (uint32_t)a | ((uint32_t)b << 10) | ((uint32_t)c << 20); }
DEV int id0(uint32_t f) { return (int)(f & 1023u); }
DEV int id1(uint32_t f) { return (int)((f >> 10) & 1023u); }
DEV int id2(uint32_t f) { return (int)((f >> 20) & 1023u); }

// wave-scope ordering point between LDS writes of some lanes and reads of others
DEV void lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

template <typename TP, int G, int K> struct HullLds {
    static constexpr int NP = G * K;
    static constexpr int FC = 2 * NP - 4;
    TP px[NP], py[NP], pz[NP];          // points at storage precision (widened exactly on use)
    double fnx[FC], fny[FC], fnz[FC];   // unit normals (UNINML of the stored order)
    uint32_t fv[FC];                    // packed vertex ids; DEAD = removed slot with no successor
    uint32_t hl[FC];                    // horizon edges u | w << 10, in (visible face, edge) order
    uint16_t vl[FC];                    // visible slots, ascending
    uint8_t vis[FC];                    // visible flag by slot (this iteration)
    uint8_t used[NP];                   // point referenced by a live face (output pass)
};

template <typename TP, int G, int K> struct Cloud {
    using L_t = HullLds<TP, G, K>;
    static constexpr int FC = L_t::FC;
    static constexpr int R = (FC + G - 1) / G;
    L_t& L;
    Grp<G> g;
    double x[K], y[K], z[K];
    int st[K];                          // assigned face slot, -1 = interior / processed / absent
    double ds[K];                       // distance above the assigned face
    int n;
    DEV V3<double> P(int i) const { return vmk<double>((double)L.px[i], (double)L.py[i], (double)L.pz[i]); }
    DEV V3<double> mine(int k) const { return vmk<double>(x[k], y[k], z[k]); }
    DEV double fdist(int f, V3<double> p) const {   // qh_dist: dot(p - p_a, n_f)
        const V3<double> a = P(id0(L.fv[f]));
        return dot(vsub(p, a), vmk<double>(L.fnx[f], L.fny[f], L.fnz[f]));
    }
};

// group-wide (value, index) argmax over the lane's own points; `val(k, i)` gives point i's value,
// or -DBL_MAX when it does not take part.  First index wins ties (lower k first within a lane,
// since index k*G+gl grows with k; lowest index across lanes).
template <typename TP, int G, int K, typename F> DEV void point_argmax(const Cloud<TP, G, K>& c, F val, double& v, int& idx) {
    v = -DBL_MAX;
    idx = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int i = k * G + c.g.gl;
        const double t = val(k, i);
        if (t > v) { v = t; idx = i; }
    }
    gargmax<G>(v, idx);
    idx = c.g.uni(idx);
}

// the cloud's hull; returns a GJKEPA_STATUS_* code.  On OK, hwm is the face high-water mark.
template <typename TP, int G, int K> DEV int build(Cloud<TP, G, K>& c, int& hwm_out) {
    using C = Cloud<TP, G, K>;
    auto& L = c.L;
    const int gl = c.g.gl, n = c.n, fcap = 2 * n - 4;
    const double eps = GJKEPA_HULL_EPS;
    // 1. initial tetrahedron (qh_cloud step 1)
    double v;
    int i0, i1, i2, i3;
    {
        double m = DBL_MAX;
        i0 = 0x7fffffff;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int i = k * G + gl;
            if (i < n && (i0 == 0x7fffffff || c.x[k] < m)) { m = c.x[k]; i0 = i; }
        }
        gargmin<G>(m, i0);
        i0 = c.g.uni(i0);
    }
    const V3<double> p0 = c.P(i0);
    point_argmax(c, [&](int k, int i) { const V3<double> d = vsub(c.mine(k), p0); return i < n ? dot(d, d) : -DBL_MAX; }, v, i1);
    const V3<double> e1 = vsub(c.P(i1), p0);
    const double l1 = norm2(e1);
    if (!(l1 > eps)) return GJKEPA_STATUS_DEGENERATE;
    point_argmax(c, [&](int k, int i) { const V3<double> q = cross(e1, vsub(c.mine(k), p0)); return i < n ? dot(q, q) : -DBL_MAX; }, v, i2);
    const V3<double> pn = cross(e1, vsub(c.P(i2), p0));
    const double lp = norm2(pn);
    if (!(lp / l1 > eps)) return GJKEPA_STATUS_DEGENERATE;
    point_argmax(c, [&](int k, int i) { return i < n ? fabs(dot(vsub(c.mine(k), p0), pn)) : -DBL_MAX; }, v, i3);
    if (!(v / lp > eps)) return GJKEPA_STATUS_DEGENERATE;
    {
        const int t[4] = {i0, i1, i2, i3};
        const V3<double> cen = centroid4(c.P(i0), c.P(i1), c.P(i2), c.P(i3));
        // SEED = {0,1,2}, {0,2,3}, {0,1,3}, {1,2,3}; every lane computes, lane f < 4 stores face f
        bool bad = false;
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            int a = t[f == 3 ? 1 : 0], b = t[f == 0 ? 1 : f == 1 ? 2 : f == 2 ? 1 : 2], cc = t[f == 0 ? 2 : 3];
            const V3<double> nn = cross(vsub(c.P(b), c.P(a)), vsub(c.P(cc), c.P(b)));
            if (dot(nn, vsub(c.P(a), cen)) < 0.0) { const int s = b; b = cc; cc = s; }
            const V3<double> un = uninml(c.P(a), c.P(b), c.P(cc));
            bad |= is_zero_nml(un);
            if (gl == f) {
                L.fv[f] = pack3(a, b, cc);
                L.fnx[f] = un.x; L.fny[f] = un.y; L.fnz[f] = un.z;
                L.vis[f] = 0;
            }
        }
        if (bad) return GJKEPA_STATUS_DEGENERATE;
        lds_sync();
        // 2. initial assignment
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int i = k * G + gl;
            c.st[k] = -1;
            if (i >= n || i == i0 || i == i1 || i == i2 || i == i3) continue;
            double best = -DBL_MAX;
            int bf = -1;
            for (int f = 0; f < 4; ++f) {
                const double d = c.fdist(f, c.mine(k));
                if (d > best) { best = d; bf = f; }
            }
            if (best > eps) { c.st[k] = bf; c.ds[k] = best; }
        }
    }
    int hwm = 4;
    // 3. furthest-point expansion
    for (;;) {
        int eye;
        point_argmax(c, [&](int k, int) { return c.st[k] >= 0 ? c.ds[k] : -DBL_MAX; }, v, eye);
        if (!(v > 0.0)) break;                          // no assigned point left (dist > eps > 0)
        const V3<double> pe = c.P(eye);
        // visible faces, in slot order
        int nvis = 0;
        for (int r = 0; r * G < hwm; ++r) {
            const int s = r * G + gl;
            bool vz = false;
            if (s < hwm && L.fv[s] != DEAD) vz = c.fdist(s, pe) > eps;
            if (s < hwm) L.vis[s] = vz;
            const uint64_t m = c.g.ballot(vz);
            if (vz) L.vl[nvis + mbcnt(m)] = (uint16_t)s;
            nvis += popc(m);
        }
        lds_sync();
        // horizon edges, in (visible face, edge) order
        int nh = 0;
        bool over = false;
        for (int base = 0; base < 3 * nvis; base += G) {
            const int t = base + gl;
            bool hz = false;
            int u = 0, w = 0;
            if (t < 3 * nvis) {
                const int j = t / 3, e = t - 3 * j;
                const uint32_t f = L.fv[L.vl[j]];
                u = e == 0 ? id0(f) : e == 1 ? id1(f) : id2(f);
                w = e == 0 ? id1(f) : e == 1 ? id2(f) : id0(f);
                bool twin = false;
                for (int m = 0; m < nvis; ++m) {
                    const uint32_t h = L.fv[L.vl[m]];
                    const int a = id0(h), b = id1(h), cc = id2(h);
                    twin |= (a == w && b == u) || (b == w && cc == u) || (cc == w && a == u);
                }
                hz = !twin;
            }
            const uint64_t m = c.g.ballot(hz);
            const int pos = nh + mbcnt(m);
            if (hz && pos < C::FC) L.hl[pos] = (uint32_t)u | ((uint32_t)w << 10);
            nh += popc(m);
            over |= nh > fcap;
        }
        if (over || nh == 0 || hwm + (nh > nvis ? nh - nvis : 0) > fcap) return GJKEPA_STATUS_DEGENERATE;
        lds_sync();
        // cone faces (u, w, eye) into the removed slots in slot order, then appended
        bool bad = false;
        for (int base = 0; base < (nh > nvis ? nh : nvis); base += G) {
            const int k = base + gl;
            if (k < nh) {
                const uint32_t e = L.hl[k];
                const int u = (int)(e & 1023u), w = (int)(e >> 10);
                const V3<double> un = uninml(c.P(u), c.P(w), pe);
                bad |= is_zero_nml(un);
                const int s = k < nvis ? (int)L.vl[k] : hwm + (k - nvis);
                L.fv[s] = pack3(u, w, eye);
                L.fnx[s] = un.x; L.fny[s] = un.y; L.fnz[s] = un.z;
            } else if (k < nvis) {
                L.fv[L.vl[k]] = DEAD;                   // removed slots left over
            }
        }
        if (c.g.any(bad)) return GJKEPA_STATUS_DEGENERATE;
        lds_sync();
        // re-assign the points of removed faces among the new faces (old visibility flags)
        bool cand[K];
        bool anyc = false;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int i = k * G + gl;
            if (i == eye) c.st[k] = -1;
            cand[k] = c.st[k] >= 0 && L.vis[c.st[k]];
            anyc |= cand[k];
        }
        if (c.g.any(anyc)) {
            double best[K];
            int bk[K];
#pragma unroll
            for (int k = 0; k < K; ++k) { best[k] = -DBL_MAX; bk[k] = 0; }
            for (int kk = 0; kk < nh; ++kk) {
                const int s = kk < nvis ? (int)L.vl[kk] : hwm + (kk - nvis);
                const V3<double> a = c.P((int)(L.hl[kk] & 1023u));   // new face kk = (u, w, eye)
                const V3<double> nn = vmk<double>(L.fnx[s], L.fny[s], L.fnz[s]);
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const double d = dot(vsub(c.mine(k), a), nn);
                    if (cand[k] && d > best[k]) { best[k] = d; bk[k] = s; }
                }
            }
#pragma unroll
            for (int k = 0; k < K; ++k) {
                if (!cand[k]) continue;
                if (best[k] > eps) { c.st[k] = bk[k]; c.ds[k] = best[k]; } else c.st[k] = -1;
            }
        }
        lds_sync();
        for (int base = 0; base < nvis; base += G)
            if (base + gl < nvis) L.vis[L.vl[base + gl]] = 0;
        if (nh > nvis) hwm += nh - nvis;
        lds_sync();
    }
    hwm_out = hwm;
    return GJKEPA_STATUS_OK;
}

template <typename TIn, int G, int K> DEV void run_cloud(Cloud<TIn, G, K>& c, const gjkepa_hull_args& a, int64_t ci) {
    auto& L = c.L;
    const int gl = c.g.gl;
    const int n = a.cloud_cnt[ci];
    c.n = n;
    int st = GJKEPA_STATUS_BAD_INPUT, hwm = 0;
    const int64_t off = a.cloud_off[ci];
    const TIn* src = (const TIn*)a.points + off;
    if (n >= 4 && n <= G * K) {
        bool finite = true;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int i = k * G + gl;
            if (i < n) {
                c.x[k] = (double)src[i]; c.y[k] = (double)src[n + i]; c.z[k] = (double)src[2 * n + i];
                finite &= isfinite(c.x[k]) && isfinite(c.y[k]) && isfinite(c.z[k]);
                L.px[i] = src[i]; L.py[i] = src[n + i]; L.pz[i] = src[2 * n + i];
            } else {
                c.x[k] = c.y[k] = c.z[k] = 0.0;
            }
            L.used[k * G + gl] = 0;
        }
        lds_sync();
        if (c.g.all(finite)) st = build(c, hwm);
    }
    int nf = 0, nv = 0;
    if (st == GJKEPA_STATUS_OK) {
        // live faces in slot order; mark their vertices
        int32_t* fo = a.faces + 3 * a.face_off[ci];
        for (int r = 0; r * G < hwm; ++r) {
            const int s = r * G + gl;
            const bool live = s < hwm && L.fv[s] != DEAD;
            const uint64_t m = c.g.ballot(live);
            if (live) {
                const uint32_t f = L.fv[s];
                const int p = nf + mbcnt(m);
                fo[3 * p] = id0(f); fo[3 * p + 1] = id1(f); fo[3 * p + 2] = id2(f);
                L.used[id0(f)] = 1; L.used[id1(f)] = 1; L.used[id2(f)] = 1;
            }
            nf += popc(m);
        }
        lds_sync();
        // vertex set in ascending point index (getHullMeshesVertex)
        bool u[K];
        int base[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int i = k * G + gl;
            u[k] = i < n && L.used[i];
            const uint64_t m = c.g.ballot(u[k]);
            base[k] = nv + mbcnt(m);
            nv += popc(m);
        }
        TIn* hv = a.hull_verts ? (TIn*)a.hull_verts + off : nullptr;
        int32_t* vi = a.vert_idx ? a.vert_idx + off : nullptr;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (!u[k]) continue;
            const int i = k * G + gl, p = base[k];
            if (vi) vi[p] = i;
            if (hv) { hv[p] = src[i]; hv[nv + p] = src[n + i]; hv[2 * nv + p] = src[2 * n + i]; }
        }
    }
    if (gl == 0) {
        a.n_faces[ci] = nf;
        a.n_verts[ci] = nv;
        a.status[ci] = (int8_t)st;
    }
    lds_sync();
}

// clouds this tier answers: lo < n <= hi (tier 0 also takes every BAD_INPUT size)
template <typename TIn, int G, int K>
__global__ __launch_bounds__(64, 1) void hull_kernel(const gjkepa_hull_args a) {
    constexpr int GPW = 64 / G;
    extern __shared__ __align__(16) unsigned char smem[];
    const int lane = lane_id();
    const int grp = lane / G;
    HullLds<TIn, G, K>* Ls = reinterpret_cast<HullLds<TIn, G, K>*>(smem);
    Cloud<TIn, G, K> c{Ls[grp]};
    const bool tier0 = a.tier == 0;
    for (int64_t chunk = blockIdx.x; chunk * 64 < a.n_clouds; chunk += gridDim.x) {
        const int64_t ci = chunk * 64 + lane;
        bool mine = false;
        if (ci < a.n_clouds) {
            const int n = a.cloud_cnt[ci];
            const bool bad = n < 4 || n > GJKEPA_HULL_MAX_POINTS;
            mine = tier0 ? (bad || n <= G * K) : (!bad && n > a.lo);
        }
        uint64_t m = __ballot(mine);
        // the j-th selected cloud of the chunk goes to group j % GPW
        const int cnt = popc(m);
        for (int j = grp; j < cnt; j += GPW) {
            uint64_t mm = m;
            for (int s = 0; s < j; ++s) mm &= mm - 1;
            const int64_t cj = chunk * 64 + __builtin_ctzll(mm);
            run_cloud<TIn, G, K>(c, a, cj);
        }
    }
}

}  // namespace qh
}  // namespace gk

namespace {
template <typename TIn, int G, int K> hipError_t launch_tier(gjkepa_hull_args a, int lo, hipStream_t s) {
    auto kfn = gk::qh::hull_kernel<TIn, G, K>;
    constexpr int GPW = 64 / G;
    const size_t lds = sizeof(gk::qh::HullLds<TIn, G, K>) * GPW;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, 64, lds) != hipSuccess || per_cu < 1) per_cu = 1;
    const int64_t chunks = (a.n_clouds + 63) / 64;
    int64_t grid = (int64_t)per_cu * a.num_cus;
    if (chunks < grid) grid = chunks;
    if (grid < 1) return hipSuccess;
    a.lo = lo;
    hipLaunchKernelGGL(kfn, dim3((unsigned)grid), dim3(64), lds, s, a);
    return hipGetLastError();
}
template <typename TIn> hipError_t launch_all(gjkepa_hull_args a, hipStream_t s) {
    a.tier = 0;
    hipError_t e = launch_tier<TIn, GJKEPA_H0_G, GJKEPA_H0_K>(a, 0, s);
    if (e != hipSuccess) return e;
    a.tier = 1;
    return launch_tier<TIn, GJKEPA_H1_G, GJKEPA_H1_K>(a, GJKEPA_H0_G * GJKEPA_H0_K, s);
}
}  // namespace

static_assert(GJKEPA_H1_G * GJKEPA_H1_K >= GJKEPA_HULL_MAX_POINTS, "the last hull tier must hold every cloud");
static_assert(GJKEPA_HULL_MAX_POINTS <= 1024, "vertex ids are packed in 10 bits");

hipError_t gjkepa_launch_hull(int vert_dtype, const gjkepa_hull_args& a, hipStream_t s) {
    return vert_dtype == GJKEPA_DTYPE_F32 ? launch_all<float>(a, s) : launch_all<double>(a, s);
}
