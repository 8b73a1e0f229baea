// gjkepa_kernel.hip — CDNA4 (gfx950) batched GJK/EPA narrow phase: one wavefront per pair.
//
// What it computes: SUBROUTINE GJKEPA of src/GCLIB_GJKEPA.f90 (:39-239) for every pair of a
// pooled hull set; each device function cites the reference lines it follows.  The numerical
// recipe (operation order, no FMA contraction, sequential sums, first-index tie rules) is the
// same as oracle/gjkepa_oracle.c so fp64 results can be compared bit for bit.
//
// Mapping onto the wavefront (64 lanes):
//   * hull vertices: lane l owns vertices l, l+64, ... of both hulls in registers (K per hull),
//     with an LDS copy for random access; loaded with coalesced SoA loads (x[], y[], z[]).
//   * support mapping (:1030-1062): per-lane dot + argmax, then a 6-step butterfly
//     (value, index) reduction across the wave — the lowest index wins ties like the
//     reference's strict '>' scan.
//   * GJK simplex logic (:82-236): wave-uniform scalar code (every lane holds the same values).
//   * EPA polytope (:863-1022 + the re-supplied hull): vertices and faces (plane, |distance|,
//     packed vertex ids) in LDS; face f lives on lane f % 64.  MINLOC, visibility, horizon
//     extraction, compaction and new-face construction are lane-parallel; order-preserving
//     compaction uses ballot + mbcnt prefix counts.
//   * capacities are template parameters; a pair that does not fit a tier (hull larger than
//     64*K vertices, polytope beyond VCAP/FCAP) is appended to the next tier's work list.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdint>

#include "../../include/gjkepa.h"
#include "gjkepa_kernel.h"

namespace gk {

#define DEV __device__ __forceinline__

constexpr int kWave = 64;
constexpr int ST_DEFER = 100;   // internal: does not fit this tier

// GET_RANDOM_UNIT_VECTOR table (:1578-1689)
__constant__ double kDirTab[100][3] = {
#include "dirtab.inc"
};

// ---------------------------------------------------------------- precision-dependent constants
template <typename T> struct Tol;
template <> struct Tol<double> {
    static constexpr double PT = 1.0e-8;     // :106, :123, :140, :157, :199, :203, :994, :1248
    static constexpr double Z = 1.0e-12;     // UTZVEC / UNINML / DIST_PF_SIGN zero (:1350, :1392, :1369)
    static constexpr double ZO = 1.0e-12;    // EPA orientation & origin-on-face (:905, :910, :935)
    static constexpr double POS = 1.0e-15;   // IS_INSIDE_PF positive (:1306)
    static constexpr double HULL = 1.0e-10;  // re-supplied QuickHull visibility
    static constexpr double BIG = DBL_MAX;   // HUGE(1.0D0)
};
template <> struct Tol<float> {              // fp32 throughput path: tolerances scaled to fp32 noise
    static constexpr float PT = 1.0e-6f;
    static constexpr float Z = 1.0e-12f;
    static constexpr float ZO = 1.0e-6f;
    static constexpr float POS = 1.0e-15f;
    static constexpr float HULL = 2.0e-6f;
    static constexpr float BIG = FLT_MAX;
};

DEV double tsqrt(double x) { return ::sqrt(x); }
DEV float tsqrt(float x) { return ::sqrtf(x); }
DEV double tatan2(double y, double x) { return ::atan2(y, x); }
DEV float tatan2(float y, float x) { return ::atan2f(y, x); }
DEV double tfmod(double a, double b) { return ::fmod(a, b); }
DEV float tfmod(float a, float b) { return ::fmodf(a, b); }

// ---------------------------------------------------------------- 3-vectors (oracle arithmetic)
template <typename T> struct V3 { T x, y, z; };
template <typename T> DEV V3<T> vmk(T x, T y, T z) { V3<T> r; r.x = x; r.y = y; r.z = z; return r; }
template <typename T> DEV V3<T> vsub(V3<T> a, V3<T> b) { return vmk<T>(a.x - b.x, a.y - b.y, a.z - b.z); }
template <typename T> DEV V3<T> vadd(V3<T> a, V3<T> b) { return vmk<T>(a.x + b.x, a.y + b.y, a.z + b.z); }
template <typename T> DEV V3<T> vneg(V3<T> a) { return vmk<T>(-a.x, -a.y, -a.z); }
template <typename T> DEV V3<T> vscl(T s, V3<T> a) { return vmk<T>(s * a.x, s * a.y, s * a.z); }
template <typename T> DEV V3<T> vdiv(V3<T> a, T s) { return vmk<T>(a.x / s, a.y / s, a.z / s); }
template <typename T> DEV T dot(V3<T> a, V3<T> b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
template <typename T> DEV T norm2(V3<T> a) { return tsqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
template <typename T> DEV V3<T> zero3() { return vmk<T>(T(0), T(0), T(0)); }
// CROSS_PRODUCT_3D (:1201-1212)
template <typename T> DEV V3<T> cross(V3<T> a, V3<T> b) {
    return vmk<T>(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
// UTZVEC (:1343-1352)
template <typename T> DEV V3<T> utzvec(V3<T> a) {
    T md = norm2(a);
    if (md < Tol<T>::Z) return zero3<T>();
    return vdiv(a, md);
}
// UNINML (:1382-1394)
template <typename T> DEV V3<T> uninml(V3<T> p1, V3<T> p2, V3<T> p3) {
    V3<T> c = cross(vsub(p2, p1), vsub(p3, p2));
    if (fabs(c.x) > Tol<T>::Z || fabs(c.y) > Tol<T>::Z || fabs(c.z) > Tol<T>::Z) return vdiv(c, norm2(c));
    return zero3<T>();
}
template <typename T> DEV bool is_zero_nml(V3<T> n) {
    return fabs(n.x) < Tol<T>::Z && fabs(n.y) < Tol<T>::Z && fabs(n.z) < Tol<T>::Z;
}
template <typename T> DEV bool allclose8(V3<T> a, V3<T> b) {
    return fabs(a.x - b.x) < Tol<T>::PT && fabs(a.y - b.y) < Tol<T>::PT && fabs(a.z - b.z) < Tol<T>::PT;
}

// ---------------------------------------------------------------- wave primitives
DEV int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
DEV int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
DEV bool unib(bool b) { return __builtin_amdgcn_readfirstlane((int)b) != 0; }
DEV uint64_t ballot(bool p) { return __ballot(p); }
DEV int prefix_in(uint64_t m) {   // set bits of m below this lane
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
DEV int popc(uint64_t m) { return __popcll(m); }

template <typename T> DEV T shfl_xor(T v, int m) { return __shfl_xor(v, m, kWave); }

// (value, index) butterfly: max value, lowest index among equal values
template <typename T> DEV void wave_argmax(T& v, int& i) {
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        T ov = shfl_xor(v, o);
        int oi = shfl_xor(i, o);
        bool take = (ov > v) || (ov == v && oi < i);
        v = take ? ov : v;
        i = take ? oi : i;
    }
}
// min value, lowest index among equal values
template <typename T> DEV void wave_argmin(T& v, int& i) {
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        T ov = shfl_xor(v, o);
        int oi = shfl_xor(i, o);
        bool take = (ov < v) || (ov == v && oi < i);
        v = take ? ov : v;
        i = take ? oi : i;
    }
}
template <typename T> DEV T wave_max(T v) {
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) { T ov = shfl_xor(v, o); v = ov > v ? ov : v; }
    return v;
}

// ---------------------------------------------------------------- per-wave LDS image
template <typename T, int K, int VCAP, int FCAP> struct Lds {
    static constexpr int NH = K * kWave;
    T hx[2][NH], hy[2][NH], hz[2][NH];   // hull A (0) / B (1) vertices, compute precision
    T vx[VCAP], vy[VCAP], vz[VCAP];      // EPA polytope vertices
    T fnx[FCAP], fny[FCAP], fnz[FCAP];   // face unit normal UNINML(stored order), outward
    T fd[FCAP];                          // |DIST_PF_SIGN(O, face)|
    T dsv[FCAP];                         // previous iteration's distances (termination test)
    T srt[FCAP];                         // sorted distances scratch
    uint32_t fv[FCAP];                   // vertex ids v0 | v1<<8 | v2<<16
    uint32_t visf[FCAP];                 // visible face list
    uint32_t hor[FCAP];                  // horizon edges u | w<<8
    T sx[NH], sy[NH], sz[NH];            // support-set / sort scratch for contact points
    T pol[NH];                           // polygon coordinate exchange (SORT_CLOCK / IS_INSIDE_PF)
    uint32_t ord[NH];                    // SORT_CLOCK order
    uint32_t rec[32];                    // staged output record
};

template <typename T, int K> struct Hull {
    T ax[K], ay[K], az[K], bx[K], by[K], bz[K];
    int na, nb;
};

template <typename T, int K, int VCAP, int FCAP> struct Ctx {
    Lds<T, K, VCAP, FCAP>& L;
    Hull<T, K> h;
    int lane;
    DEV V3<T> A(int i) const { return vmk<T>(L.hx[0][i], L.hy[0][i], L.hz[0][i]); }
    DEV V3<T> B(int i) const { return vmk<T>(L.hx[1][i], L.hy[1][i], L.hz[1][i]); }
    DEV V3<T> vert(int i) const { return vmk<T>(L.vx[i], L.vy[i], L.vz[i]); }
    DEV V3<T> fn(int f) const { return vmk<T>(L.fnx[f], L.fny[f], L.fnz[f]); }
};

// ---------------------------------------------------------------- support mapping (:1030-1062)
// indices: argmax_i d.a_i (first), argmax_j (-d).b_j (first); -dot(d,b) == dot(-d,b) bit for bit.
template <typename T, int K, int VC, int FC>
DEV void support_idx(const Ctx<T, K, VC, FC>& c, V3<T> d, int& ia, int& ib) {
    T va = -Tol<T>::BIG, vb = -Tol<T>::BIG;
    int xa = 0x7fffffff, xb = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        int i = k * kWave + c.lane;
        T ta = d.x * c.h.ax[k] + d.y * c.h.ay[k] + d.z * c.h.az[k];
        if (i < c.h.na && ta > va) { va = ta; xa = i; }
        T tb = -(d.x * c.h.bx[k] + d.y * c.h.by[k] + d.z * c.h.bz[k]);
        if (i < c.h.nb && tb > vb) { vb = tb; xb = i; }
    }
    wave_argmax(va, xa);
    wave_argmax(vb, xb);
    ia = uni(xa == 0x7fffffff ? 0 : xa);
    ib = uni(xb == 0x7fffffff ? 0 : xb);
}
template <typename T, int K, int VC, int FC>
DEV V3<T> support(const Ctx<T, K, VC, FC>& c, V3<T> d) {
    int ia, ib;
    support_idx(c, d, ia, ib);
    return vsub(c.A(ia), c.B(ib));
}

// ---------------------------------------------------------------- GJK helpers
// VEC_PL (:1423-1440)
template <typename T> DEV V3<T> vec_pl(V3<T> C, V3<T> A, V3<T> B) {
    V3<T> AB = vsub(B, A), AC = vsub(C, A);
    T k = dot(AC, AB) / norm2(AB);
    V3<T> D = vadd(A, vscl(k, utzvec(AB)));
    return utzvec(vsub(D, C));
}
// IS_INSIDE_PF for a triangle, scalar (:1271-1337)
template <typename T> DEV bool inside_tri(V3<T> V0, V3<T> V1, V3<T> V2, V3<T> P) {
    V3<T> V[3] = {V0, V1, V2};
    T cp[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        int j = (i == 2) ? 0 : i + 1;
        cp[i] = (V[j].x - V[i].x) * (P.y - V[i].y) - (V[j].y - V[i].y) * (P.x - V[i].x);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) if (fabs(cp[i]) < Tol<T>::Z) cp[i] = T(0);
    bool anypos = cp[0] > Tol<T>::POS || cp[1] > Tol<T>::POS || cp[2] > Tol<T>::POS;
    if (!anypos) {
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            int j = (i == 2) ? 0 : i + 1;
            cp[i] = (V[j].x - V[i].x) * (P.z - V[i].z) - (V[j].z - V[i].z) * (P.x - V[i].x);
        }
    }
    return !(cp[0] * cp[0] < T(0) || cp[0] * cp[1] < T(0) || cp[0] * cp[2] < T(0));
}

template <typename T> DEV V3<T> centroid4(const V3<T>* S) {   // SUM(simplex_(:,k)) / 4
    return vmk<T>((((S[0].x + S[1].x) + S[2].x) + S[3].x) / T(4),
                  (((S[0].y + S[1].y) + S[2].y) + S[3].y) / T(4),
                  (((S[0].z + S[1].z) + S[2].z) + S[3].z) / T(4));
}
template <typename T> DEV V3<T> tet_face_nml(const V3<T>* S, int i) {
    int f0 = i == 3 ? 1 : 0;
    int f1 = i == 0 ? 2 : (i == 3 ? 2 : 1);
    int f2 = i == 2 ? 2 : 3;
    V3<T> AB = vsub(S[f0], S[f1]);
    V3<T> BC = vsub(S[f1], S[f2]);
    return utzvec(cross(AB, BC));
}
// isPointInSimplex (:1217-1265) for P = origin
template <typename T> DEV bool origin_in_simplex(const V3<T>* S) {
    V3<T> M = centroid4(S);
    V3<T> O = zero3<T>();
    T dist[4];
    V3<T> nml[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        nml[i] = tet_face_nml(S, i);
        if (dot(nml[i], vsub(S[i], M)) < T(0)) nml[i] = vneg(nml[i]);
        dist[i] = dot(vsub(S[i], O), nml[i]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (fabs(dist[i]) < Tol<T>::PT) {
            int f0 = i == 3 ? 1 : 0;
            int f1 = i == 0 ? 2 : (i == 3 ? 2 : 1);
            int f2 = i == 2 ? 2 : 3;
            if (inside_tri(S[f0], S[f1], S[f2], O)) return true;
        }
    }
    return dist[0] > T(0) && dist[1] > T(0) && dist[2] > T(0) && dist[3] > T(0);
}
// update_simplex_GJK (:1070-1157)
template <typename T, int K, int VC, int FC>
DEV void update_simplex(const Ctx<T, K, VC, FC>& c, V3<T>* S) {
    V3<T> M = centroid4(S);
    V3<T> O = zero3<T>();
    V3<T> nml[4];
    T dst[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        V3<T> R = (i == 3) ? S[1] : S[0];
        nml[i] = tet_face_nml(S, i);
        if (dot(nml[i], vsub(R, M)) < T(0)) nml[i] = vneg(nml[i]);
        dst[i] = dot(vneg(nml[i]), vsub(R, O));
    }
    int k = 0;
#pragma unroll
    for (int i = 1; i < 4; ++i) if (dst[i] > dst[k]) k = i;
    k = uni(k);
    V3<T> dir = nml[0];
    if (k == 1) dir = nml[1];
    if (k == 2) dir = nml[2];
    if (k == 3) dir = nml[3];
    V3<T> SM = support(c, dir);
    V3<T> s0 = S[0], s1 = S[1], s2 = S[2], s3 = S[3];
    if (k == 0) { S[0] = s0; S[1] = s2; S[2] = s3; }
    else if (k == 1) { S[0] = s0; S[1] = s1; S[2] = s3; }
    else if (k == 2) { S[0] = s0; S[1] = s1; S[2] = s2; }
    else { S[0] = s1; S[1] = s2; S[2] = s3; }
    S[3] = SM;
}

// ---------------------------------------------------------------- EPA polytope (re-supplied hull)
template <typename T, int K, int VC, int FC>
DEV void write_face(Ctx<T, K, VC, FC>& c, int f, int a, int b, int d, V3<T> n, T dist) {
    c.L.fv[f] = (uint32_t)a | ((uint32_t)b << 8) | ((uint32_t)d << 16);
    c.L.fnx[f] = n.x; c.L.fny[f] = n.y; c.L.fnz[f] = n.z;
    c.L.fd[f] = dist;
}

// Add point p (vertex id k; appended at nv when `append`) — visible faces (signed distance >
// HULL) removed, horizon coned to k.  Order: survivors, then new faces by (visible face, edge).
template <typename T, int K, int VC, int FC>
DEV int hull_add(Ctx<T, K, VC, FC>& c, int& nv, int& nf, V3<T> p, bool append, int kexist) {
    constexpr int R = (FC + kWave - 1) / kWave;
    auto& L = c.L;
    const int lane = c.lane;
    uint64_t vm[R];
    int nvis = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        int f = r * kWave + lane;
        bool vis = false;
        if (f < nf) {
            int a = (int)(L.fv[f] & 0xffu);
            vis = dot(vsub(p, c.vert(a)), c.fn(f)) > Tol<T>::HULL;
        }
        vm[r] = ballot(vis);
        nvis += popc(vm[r]);
    }
    nvis = uni(nvis);
    if (nvis == 0) return 0;
    int k = kexist;
    if (append) {
        if (nv >= VC) return ST_DEFER;
        k = nv;
        if (lane == 0) { L.vx[k] = p.x; L.vy[k] = p.y; L.vz[k] = p.z; }
        nv = nv + 1;
    }
    // visible face list, in face order
    {
        int base = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if ((vm[r] >> lane) & 1ull) L.visf[base + prefix_in(vm[r])] = (uint32_t)(r * kWave + lane);
            base += popc(vm[r]);
        }
    }
    __builtin_amdgcn_wave_barrier();
    // horizon edges: edge (u,w) of a visible face whose twin (w,u) is on no visible face
    int nh = 0;
    const int ne = 3 * nvis;
    for (int e0 = 0; e0 < ne; e0 += kWave) {
        int e = e0 + lane;
        bool hz = false;
        uint32_t uw = 0;
        if (e < ne) {
            int fi = e / 3, s = e - 3 * fi;
            uint32_t fv = L.fv[L.visf[fi]];
            uint32_t u = (fv >> (8 * s)) & 0xffu;
            uint32_t w = (fv >> (8 * (s == 2 ? 0 : s + 1))) & 0xffu;
            bool twin = false;
            for (int j = 0; j < nvis && !twin; ++j) {
                uint32_t g = L.fv[L.visf[j]];
                uint32_t g0 = g & 0xffu, g1 = (g >> 8) & 0xffu, g2 = (g >> 16) & 0xffu;
                twin = (g0 == w && g1 == u) || (g1 == w && g2 == u) || (g2 == w && g0 == u);
            }
            hz = !twin;
            uw = u | (w << 8);
        }
        uint64_t m = ballot(hz);
        if (hz) {
            int pos = nh + prefix_in(m);
            if (pos < FC) L.hor[pos] = uw;
        }
        nh += popc(m);
    }
    nh = uni(nh);
    const int nf2 = nf - nvis + nh;
    if (nh > FC || nf2 > FC) return ST_DEFER;
    // compact surviving faces (order preserved; in place is safe: new index <= old index)
    int base = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        int f = r * kWave + lane;
        bool keep = f < nf && !((vm[r] >> lane) & 1ull);
        uint32_t fv = 0;
        T nx = 0, ny = 0, nz = 0, d = 0;
        if (keep) { fv = L.fv[f]; nx = L.fnx[f]; ny = L.fny[f]; nz = L.fnz[f]; d = L.fd[f]; }
        uint64_t m = ballot(keep);
        __builtin_amdgcn_wave_barrier();
        if (keep) {
            int pos = base + prefix_in(m);
            L.fv[pos] = fv; L.fnx[pos] = nx; L.fny[pos] = ny; L.fnz[pos] = nz; L.fd[pos] = d;
        }
        base += popc(m);
        __builtin_amdgcn_wave_barrier();
    }
    // cone the horizon to k
    const V3<T> P = c.vert(k);
    bool bad = false;
    for (int h0 = 0; h0 < nh; h0 += kWave) {
        int h = h0 + lane;
        if (h < nh) {
            uint32_t uw = L.hor[h];
            int u = (int)(uw & 0xffu), w = (int)((uw >> 8) & 0xffu);
            V3<T> U = c.vert(u), W = c.vert(w);
            V3<T> n = uninml(U, W, P);
            if (is_zero_nml(n)) bad = true;
            T d = fabs(dot(vsub(zero3<T>(), U), n));
            write_face(c, base + h, u, w, k, n, d);
        }
    }
    __builtin_amdgcn_wave_barrier();
    nf = nf2;
    if (unib(ballot(bad) != 0)) return GJKEPA_STATUS_DEGENERATE;
    return 0;
}

// Hull of <= 6 points from scratch (EPA iteration 1): the points are vertex ids 0..m-1 of the
// LDS polytope.  First non-degenerate tetrahedron in list order, faces in the seed pattern of
// :279-293 wound outward, then the remaining points in order.
template <typename T, int K, int VC, int FC>
DEV int hull_build(Ctx<T, K, VC, FC>& c, int& nv, int& nf, int m) {
    nv = m;
    nf = 0;
    const V3<T> P0 = c.vert(0);
    int i1 = -1, i2 = -1, i3 = -1;
    for (int j = 1; j < m; ++j) if (unib(norm2(vsub(c.vert(j), P0)) > Tol<T>::HULL)) { i1 = j; break; }
    if (i1 < 0) return GJKEPA_STATUS_DEGENERATE;
    const V3<T> P1 = c.vert(i1);
    const V3<T> e1 = vsub(P1, P0);
    const T l1 = norm2(e1);
    for (int j = i1 + 1; j < m; ++j)
        if (unib(norm2(cross(e1, vsub(c.vert(j), P0))) / l1 > Tol<T>::HULL)) { i2 = j; break; }
    if (i2 < 0) return GJKEPA_STATUS_DEGENERATE;
    const V3<T> P2 = c.vert(i2);
    const V3<T> pn = utzvec(cross(e1, vsub(P2, P0)));
    for (int j = i2 + 1; j < m; ++j)
        if (unib(fabs(dot(vsub(c.vert(j), P0), pn)) > Tol<T>::HULL)) { i3 = j; break; }
    if (i3 < 0) return GJKEPA_STATUS_DEGENERATE;
    const V3<T> P3 = c.vert(i3);
    const int t[4] = {0, i1, i2, i3};
    const V3<T> Tt[4] = {P0, P1, P2, P3};
    const V3<T> cen = centroid4(Tt);
    const int SEED[4][3] = {{0, 1, 2}, {0, 2, 3}, {0, 1, 3}, {1, 2, 3}};
    bool bad = false;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
        int a = t[SEED[f][0]], b = t[SEED[f][1]], d = t[SEED[f][2]];
        V3<T> Pa = Tt[SEED[f][0]], Pb = Tt[SEED[f][1]], Pd = Tt[SEED[f][2]];
        V3<T> n0 = cross(vsub(Pb, Pa), vsub(Pd, Pb));
        if (dot(n0, vsub(Pa, cen)) < T(0)) { int s = b; b = d; d = s; V3<T> q = Pb; Pb = Pd; Pd = q; }
        V3<T> n = uninml(Pa, Pb, Pd);
        if (is_zero_nml(n)) bad = true;
        T dist = fabs(dot(vsub(zero3<T>(), Pa), n));
        if (c.lane == f) write_face(c, f, a, b, d, n, dist);
    }
    __builtin_amdgcn_wave_barrier();
    if (unib(bad)) return GJKEPA_STATUS_DEGENERATE;
    nf = 4;
    for (int j = 1; j < m; ++j) {
        if (j == i1 || j == i2 || j == i3) continue;
        int st = hull_add(c, nv, nf, c.vert(j), false, j);
        if (st) return st;
    }
    return 0;
}

// first-index argmin of fd[0..nf)
template <typename T, int K, int VC, int FC>
DEV int face_argmin(Ctx<T, K, VC, FC>& c, int nf) {
    constexpr int R = (FC + kWave - 1) / kWave;
    T v = Tol<T>::BIG;
    int idx = 0x7fffffff;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        int f = r * kWave + c.lane;
        if (f < nf) { T d = c.L.fd[f]; if (idx == 0x7fffffff || d < v) { v = d; idx = f; } }
    }
    wave_argmin(v, idx);
    return uni(idx == 0x7fffffff ? 0 : idx);
}

// ALL(|sort(d1) - sort(d2)| < 1e-8), d1 = dsv[0..n), d2 = fd[0..n)  (:972-1004)
template <typename T, int K, int VC, int FC>
DEV bool sorted_equal(Ctx<T, K, VC, FC>& c, int n) {
    auto& L = c.L;
    for (int i0 = 0; i0 < n; i0 += kWave) {
        int i = i0 + c.lane;
        if (i < n) {
            T x = L.fd[i];
            int r = 0;
            for (int j = 0; j < n; ++j) { T y = L.fd[j]; r += (y < x) || (y == x && j < i); }
            L.srt[r] = x;
        }
    }
    __builtin_amdgcn_wave_barrier();
    bool ok = true;
    for (int i0 = 0; i0 < n; i0 += kWave) {
        int i = i0 + c.lane;
        if (i < n) {
            T x = L.dsv[i];
            int r = 0;
            for (int j = 0; j < n; ++j) { T y = L.dsv[j]; r += (y < x) || (y == x && j < i); }
            if (!(fabs(x - L.srt[r]) < Tol<T>::PT)) ok = false;
        }
    }
    return unib(ballot(!ok) == 0);
}

// EPA_solu loop (:274-323) + update_expandingPolytope_EPA (:863-1022)
template <typename T, int K, int VC, int FC>
DEV int epa(Ctx<T, K, VC, FC>& c, const V3<T>* S, T& depth, V3<T>& normal, int& iters, int& nf) {
    constexpr int R = (FC + kWave - 1) / kWave;
    auto& L = c.L;
    const int SOUP[4][3] = {{0, 1, 2}, {0, 2, 3}, {0, 1, 3}, {1, 2, 3}};
    const V3<T> O = zero3<T>();
    int nv = 0;
    nf = 0;
    for (int iter = 1;; ++iter) {
        iters = iter;
        if (iter > 99) return GJKEPA_STATUS_EPA_MAXITER;
        int F1;
        T minv;
        V3<T> dir, a1;
        if (iter == 1) {
            T d[4];
            bool bad = false;
#pragma unroll
            for (int f = 0; f < 4; ++f) {
                V3<T> n = uninml(S[SOUP[f][0]], S[SOUP[f][1]], S[SOUP[f][2]]);
                if (is_zero_nml(n)) bad = true;
                d[f] = fabs(dot(vsub(O, S[SOUP[f][0]]), n));
            }
            if (bad) return GJKEPA_STATUS_DEGENERATE;
            int ml = 0;
#pragma unroll
            for (int f = 1; f < 4; ++f) if (d[f] < d[ml]) ml = f;
            ml = uni(ml);
            minv = d[0];
            V3<T> q0 = S[0], q1 = S[1], q2 = S[2];
#pragma unroll
            for (int f = 1; f < 4; ++f)
                if (ml == f) { minv = d[f]; q0 = S[SOUP[f][0]]; q1 = S[SOUP[f][1]]; q2 = S[SOUP[f][2]]; }
            dir = uninml(q0, q1, q2);
            a1 = q0;
            if (c.lane < 4) {
                T dl = d[0];
                for (int f = 1; f < 4; ++f) if (c.lane == f) dl = d[f];
                L.dsv[c.lane] = dl;
            }
            F1 = 4;
        } else {
            F1 = nf;
            int ml = face_argmin(c, nf);
            minv = L.fd[ml];
            dir = c.fn(ml);
            a1 = c.vert((int)(L.fv[ml] & 0xffu));
#pragma unroll
            for (int r = 0; r < R; ++r) {
                int f = r * kWave + c.lane;
                if (f < nf) L.dsv[f] = L.fd[f];
            }
        }
        T dt = dot(vsub(a1, O), dir);
        if (unib(fabs(dt) < Tol<T>::ZO)) {                        // :905-908 polytope centroid
            T sx = 0, sy = 0, sz = 0;
            for (int j = 0; j < 3; ++j)
                for (int f = 0; f < F1; ++f) {
                    V3<T> q;
                    if (iter == 1) {
                        int vi = SOUP[0][j];
                        if (f == 1) vi = SOUP[1][j];
                        if (f == 2) vi = SOUP[2][j];
                        if (f == 3) vi = SOUP[3][j];
                        q = S[0];
                        if (vi == 1) q = S[1];
                        if (vi == 2) q = S[2];
                        if (vi == 3) q = S[3];
                    } else {
                        q = c.vert((int)((L.fv[f] >> (8 * j)) & 0xffu));
                    }
                    sx += q.x; sy += q.y; sz += q.z;
                }
            T cnt = (T)(F1 * 3);
            V3<T> M = vmk<T>(sx / cnt, sy / cnt, sz / cnt);
            dt = dot(vsub(a1, M), dir);
        }
        if (unib(dt <= -Tol<T>::ZO)) dir = vneg(dir);             // :910
        V3<T> sp = support(c, dir);                               // :914
        const bool two = unib(fabs(minv) < Tol<T>::ZO);           // :935
        int st;
        if (iter == 1) {
            // unique polytope vertices (getHullMeshesVertex, :920) + new point(s) -> LDS ids 0..m-1
            int m = 0;
#pragma unroll
            for (int f = 0; f < 4; ++f)
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    V3<T> q = S[SOUP[f][j]];
                    bool dup = false;
                    for (int i = 0; i < m; ++i) {
                        V3<T> p = c.vert(i);
                        dup = dup || (p.x == q.x && p.y == q.y && p.z == q.z);
                    }
                    if (!unib(dup)) {
                        if (c.lane == 0) { L.vx[m] = q.x; L.vy[m] = q.y; L.vz[m] = q.z; }
                        __builtin_amdgcn_wave_barrier();
                        ++m;
                    }
                }
            if (c.lane == 0) { L.vx[m] = sp.x; L.vy[m] = sp.y; L.vz[m] = sp.z; }
            ++m;
            if (two) {
                V3<T> sq = support(c, vneg(dir));
                if (c.lane == 0) { L.vx[m] = sq.x; L.vy[m] = sq.y; L.vz[m] = sq.z; }
                ++m;
            }
            __builtin_amdgcn_wave_barrier();
            st = hull_build(c, nv, nf, m);
        } else {
            st = hull_add(c, nv, nf, sp, true, 0);
            if (!st && two) st = hull_add(c, nv, nf, support(c, vneg(dir)), true, 0);
        }
        if (st) return st;
        const int F2 = nf;                                        // :956-969
        const int ml2 = face_argmin(c, nf);
        const T minv2 = L.fd[ml2];
        V3<T> dir2 = c.fn(ml2);
        if (unib(dot(vsub(c.vert((int)(L.fv[ml2] & 0xffu)), O), dir2) < T(0))) dir2 = vneg(dir2);
        bool stop;                                                // :972-1015
        if (F1 == F2) stop = sorted_equal(c, F1);
        else stop = F1 > F2;
        if (stop) { depth = minv2; normal = dir2; return 0; }
    }
}

// ---------------------------------------------------------------- contact features
// sequential "> max - 1e-8" scans (:722-747, :438-444): the running max may decrease
template <typename T, int K, int VC, int FC>
DEV void scan_top2(Ctx<T, K, VC, FC>& c, int side, V3<T> n, int idx[2]) {
    T mx = -Tol<T>::BIG;
    idx[0] = -1; idx[1] = -1;
    const int cnt = side ? c.h.nb : c.h.na;
    for (int i = 0; i < cnt; ++i) {
        V3<T> p = side ? c.B(i) : c.A(i);
        T t = dot(n, p);
        if (t > mx - Tol<T>::PT) { mx = t; idx[1] = idx[0]; idx[0] = i; }
    }
    if (idx[1] == -1) idx[1] = idx[0];
}

// lane-parallel max of dot(n, p_i) over one hull
template <typename T, int K, int VC, int FC>
DEV T hull_dot_max(Ctx<T, K, VC, FC>& c, int side, V3<T> n) {
    T mx = -Tol<T>::BIG;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        int i = k * kWave + c.lane;
        T t = side ? n.x * c.h.bx[k] + n.y * c.h.by[k] + n.z * c.h.bz[k]
                   : n.x * c.h.ax[k] + n.y * c.h.ay[k] + n.z * c.h.az[k];
        if (i < (side ? c.h.nb : c.h.na) && t > mx) mx = t;
    }
    return wave_max(mx);
}
// members with dot(n,p) > mx - band (index order) → LDS sx/sy/sz; returns count
template <typename T, int K, int VC, int FC>
DEV int hull_band_set(Ctx<T, K, VC, FC>& c, int side, V3<T> n, T mx, T band, bool store) {
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        int i = k * kWave + c.lane;
        T px = side ? c.h.bx[k] : c.h.ax[k], py = side ? c.h.by[k] : c.h.ay[k], pz = side ? c.h.bz[k] : c.h.az[k];
        T t = n.x * px + n.y * py + n.z * pz;
        bool in = i < (side ? c.h.nb : c.h.na) && t > mx - band;
        uint64_t m = ballot(in);
        if (store && in) { int pos = cnt + prefix_in(m); c.L.sx[pos] = px; c.L.sy[pos] = py; c.L.sz[pos] = pz; }
        cnt += popc(m);
    }
    __builtin_amdgcn_wave_barrier();
    return uni(cnt);
}

// get_info_collisionType (:353-413)
template <typename T, int K, int VC, int FC>
DEV int collision_type(Ctx<T, K, VC, FC>& c, V3<T> n, T tol) {
    T m1 = hull_dot_max(c, 0, n);
    int C = hull_band_set(c, 0, n, m1, tol, false);
    V3<T> nn = vneg(n);
    T m2 = hull_dot_max(c, 1, nn);
    int D = hull_band_set(c, 1, nn, m2, tol, false);
    return (C >= 3 && D >= 3) ? 2 : 1;
}

// get_collisionPoint_01 (:700-806)
template <typename T, int K, int VC, int FC>
DEV int contact_v1(Ctx<T, K, VC, FC>& c, V3<T> n, V3<T>& res) {
    int i1[2], i2[2];
    scan_top2(c, 0, n, i1);
    scan_top2(c, 1, vneg(n), i2);
    if (i1[0] < 0 || i2[0] < 0) return GJKEPA_STATUS_DEGENERATE;
    res = zero3<T>();
    if (i1[0] == i1[1] && i2[0] == i2[1]) res = vdiv(vadd(c.A(i1[0]), c.B(i2[0])), T(2));
    if (i1[0] != i1[1] && i2[0] == i2[1]) res = c.B(i2[0]);
    else if (i1[0] == i1[1] && i2[0] != i2[1]) res = c.A(i1[0]);
    if (i1[0] != i1[1] && i2[0] != i2[1]) {
        T mx = hull_dot_max(c, 0, n);
        int C = hull_band_set(c, 0, n, mx, T(0.1), true);
        T sx = 0, sy = 0, sz = 0;
        for (int i = 0; i < C; ++i) { sx += c.L.sx[i]; sy += c.L.sy[i]; sz += c.L.sz[i]; }
        T dc = (T)C;
        res = vmk<T>(sx / dc, sy / dc, sz / dc);
    }
    return 0;
}

// FOOT_PL (:1492-1505)
template <typename T> DEV V3<T> foot_pl(V3<T> P, V3<T> V1, V3<T> V2) {
    V3<T> u = utzvec(vsub(V2, V1));
    return vadd(V1, vscl(dot(vsub(P, V1), u), u));
}
// FOOT_LL (:1446-1487)
template <typename T> DEV void foot_ll(V3<T> P1, V3<T> Q1, V3<T> P2, V3<T> Q2, V3<T>& f1, V3<T>& f2) {
    V3<T> d1 = vsub(Q1, P1), d2 = vsub(Q2, P2), r = vsub(P1, P2);
    T a = dot(d1, d1), b = dot(d1, d2), cc = dot(d1, r), e = dot(d2, d2), f = dot(d2, r);
    T d = a * e - b * b;
    if (fabs(d) < Tol<T>::Z) {
        f1 = vdiv(vadd(P1, Q1), T(2));
        f2 = foot_pl(f1, P2, Q2);
    } else {
        T s = (b * f - cc * e) / d;
        T t = (a * f - b * cc) / d;
        f1 = vadd(P1, vscl(s, vsub(Q1, P1)));
        f2 = vadd(P2, vscl(t, vsub(Q2, P2)));
    }
}

// case_04 (:575-669) on the set in L.s*[0..na) with the 2-point set Bp; SORT_CLOCK (:1513-1575)
// writes the ordered polygon back into L.s* (lane-parallel angle argmin per step).
template <typename T, int K, int VC, int FC>
DEV int contact_case04(Ctx<T, K, VC, FC>& c, int na, const V3<T>* Bp, V3<T>& res) {
    auto& L = c.L;
    constexpr int NH = K * kWave;
    const T TWO_PI_SP = (T)(2.0f * 3.14159274101257324f);
    // OVERLAP (:1399-1418): all points pairwise within 1e-12 -> order unchanged
    bool diff = false;
    for (int i0 = 0; i0 < na; i0 += kWave) {
        int i = i0 + c.lane;
        if (i < na) {
            for (int j = 0; j < na; ++j)
                diff = diff || fabs(L.sx[i] - L.sx[j]) > Tol<T>::Z || fabs(L.sy[i] - L.sy[j]) > Tol<T>::Z ||
                       fabs(L.sz[i] - L.sz[j]) > Tol<T>::Z;
        }
    }
    const bool ovl = unib(ballot(diff) == 0);
    // polygon lives in lanes: lane q holds element q (na <= NH, up to K per lane)
    T px[K], py[K], pz[K];
    bool used[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        int i = k * kWave + c.lane;
        px[k] = i < na ? L.sx[i] : T(0); py[k] = i < na ? L.sy[i] : T(0); pz[k] = i < na ? L.sz[i] : T(0);
        used[k] = false;
    }
    if (!ovl) {
        T sx = 0, sy = 0, sz = 0;
        for (int i = 0; i < na; ++i) { sx += L.sx[i]; sy += L.sy[i]; sz += L.sz[i]; }
        T dn = (T)na;
        V3<T> cen = vmk<T>(sx / dn, sy / dn, sz / dn);
        V3<T> p0 = vmk<T>(L.sx[0], L.sy[0], L.sz[0]);
        V3<T> nrm = cross(vsub(vmk<T>(L.sx[1], L.sy[1], L.sz[1]), p0), vsub(vmk<T>(L.sx[2], L.sy[2], L.sz[2]), p0));
        V3<T> prev = p0;
        // ordered list goes to hor[] as indices (reuse), ordered coords rebuilt after
        __builtin_amdgcn_wave_barrier();
        if (c.lane == 0) L.ord[0] = 0u;
        // element equal to an already-ordered point is skipped (exact compare, :1560-1573)
#pragma unroll
        for (int k = 0; k < K; ++k) {
            int i = k * kWave + c.lane;
            used[k] = i < na && px[k] == p0.x && py[k] == p0.y && pz[k] == p0.z;
        }
        for (int s = 1; s < na; ++s) {
            T best = Tol<T>::BIG;
            int bi = 0x7fffffff;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                int j = k * kWave + c.lane;
                if (j < na && !used[k]) {
                    V3<T> w1 = vsub(vmk<T>(px[k], py[k], pz[k]), cen), w2 = vsub(prev, cen);
                    T ang = tatan2(dot(nrm, cross(w2, w1)), dot(w1, w2));
                    ang = tfmod(ang + TWO_PI_SP, TWO_PI_SP);
                    if (ang < best) { best = ang; bi = j; }
                }
            }
            wave_argmin(best, bi);
            bi = uni(bi);
            if (bi == 0x7fffffff) return GJKEPA_STATUS_DEGENERATE;
            prev = vmk<T>(L.sx[bi], L.sy[bi], L.sz[bi]);
            if (c.lane == 0) L.ord[s] = (uint32_t)bi;
#pragma unroll
            for (int k = 0; k < K; ++k)
                used[k] = used[k] || (px[k] == prev.x && py[k] == prev.y && pz[k] == prev.z);
        }
        __builtin_amdgcn_wave_barrier();
        // permute polygon into lane order q -> element hor[q]
#pragma unroll
        for (int k = 0; k < K; ++k) {
            int q = k * kWave + c.lane;
            if (q < na) { int src = (int)L.ord[q]; px[k] = L.sx[src]; py[k] = L.sy[src]; pz[k] = L.sz[src]; }
        }
    }
    (void)NH;
    // IS_INSIDE_PF(sorted polygon, Bp[i]) for i = 0, 1 (lane-parallel over polygon edges)
    int C = 0;
    for (int t = 0; t < 2; ++t) {
        const V3<T> P = Bp[t];
        // edge i: (V_i, V_{i+1}) — neighbour fetched by shuffle-free LDS write/read of the polygon
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int k = 0; k < K; ++k) {
            int q = k * kWave + c.lane;
            if (q < na) { L.pol[q] = px[k]; }
        }
        __builtin_amdgcn_wave_barrier();
        T nxv[K], nyv[K], nzv[K];
#pragma unroll
        for (int k = 0; k < K; ++k) { int q = k * kWave + c.lane; int j = (q == na - 1) ? 0 : q + 1; nxv[k] = q < na ? L.pol[j] : T(0); }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int k = 0; k < K; ++k) { int q = k * kWave + c.lane; if (q < na) L.pol[q] = py[k]; }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int k = 0; k < K; ++k) { int q = k * kWave + c.lane; int j = (q == na - 1) ? 0 : q + 1; nyv[k] = q < na ? L.pol[j] : T(0); }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int k = 0; k < K; ++k) { int q = k * kWave + c.lane; if (q < na) L.pol[q] = pz[k]; }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int k = 0; k < K; ++k) { int q = k * kWave + c.lane; int j = (q == na - 1) ? 0 : q + 1; nzv[k] = q < na ? L.pol[j] : T(0); }
        __builtin_amdgcn_wave_barrier();
        T cp[K];
        bool pos = false;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            int q = k * kWave + c.lane;
            cp[k] = (nxv[k] - px[k]) * (P.y - py[k]) - (nyv[k] - py[k]) * (P.x - px[k]);
            if (fabs(cp[k]) < Tol<T>::Z) cp[k] = T(0);
            pos = pos || (q < na && cp[k] > Tol<T>::POS);
        }
        if (unib(ballot(pos) == 0)) {
#pragma unroll
            for (int k = 0; k < K; ++k)
                cp[k] = (nxv[k] - px[k]) * (P.z - pz[k]) - (nzv[k] - pz[k]) * (P.x - px[k]);
        }
        T c0 = __shfl(cp[0], 0, kWave);
        bool neg = false;
#pragma unroll
        for (int k = 0; k < K; ++k) { int q = k * kWave + c.lane; neg = neg || (q < na && c0 * cp[k] < T(0)); }
        if (unib(ballot(neg) == 0)) ++C;
    }
    if (C == 0) {                                                  // case_04_1
        T sx = 0, sy = 0, sz = 0;
        // centroid of the unsorted set, SUM over sprt1 (:650); sx/sy/sz still hold it
        for (int i = 0; i < na; ++i) { sx += L.sx[i]; sy += L.sy[i]; sz += L.sz[i]; }
        T dn = (T)na;
        res = foot_pl(vmk<T>(sx / dn, sy / dn, sz / dn), Bp[0], Bp[1]);
    } else {
        res = vscl(T(0.5), vadd(Bp[0], Bp[1]));                    // case_04_2 / case_04_3
    }
    return 0;
}

// get_collisionPoint_02 (:457-696)
template <typename T, int K, int VC, int FC>
DEV int contact_v2(Ctx<T, K, VC, FC>& c, V3<T> n, V3<T>& res) {
    auto& L = c.L;
    const T band = T(0.1);
    V3<T> nn = vneg(n);
    T m1 = hull_dot_max(c, 0, n);
    T m2 = hull_dot_max(c, 1, nn);
    int n1 = hull_band_set(c, 0, n, m1, band, false);
    int n2 = hull_band_set(c, 1, nn, m2, band, false);
    res = zero3<T>();
    if (n1 == 1 && n2 == 1) {
        hull_band_set(c, 0, n, m1, band, true);
        V3<T> a = vmk<T>(L.sx[0], L.sy[0], L.sz[0]);
        hull_band_set(c, 1, nn, m2, band, true);
        V3<T> b = vmk<T>(L.sx[0], L.sy[0], L.sz[0]);
        res = vdiv(vadd(a, b), T(2));
    } else if (n1 == 1 && n2 >= 2) {
        hull_band_set(c, 0, n, m1, band, true);
        res = vmk<T>(L.sx[0], L.sy[0], L.sz[0]);
    } else if (n1 >= 2 && n2 == 1) {
        hull_band_set(c, 1, nn, m2, band, true);
        res = vmk<T>(L.sx[0], L.sy[0], L.sz[0]);
    } else if (n1 == 2 && n2 == 2) {
        hull_band_set(c, 0, n, m1, band, true);
        V3<T> a0 = vmk<T>(L.sx[0], L.sy[0], L.sz[0]), a1 = vmk<T>(L.sx[1], L.sy[1], L.sz[1]);
        hull_band_set(c, 1, nn, m2, band, true);
        V3<T> b0 = vmk<T>(L.sx[0], L.sy[0], L.sz[0]), b1 = vmk<T>(L.sx[1], L.sy[1], L.sz[1]);
        V3<T> f1, f2;
        foot_ll(a0, a1, b0, b1, f1, f2);
        res = vdiv(vadd(f1, f2), T(2));
    } else if (n1 == 2 && n2 >= 3) {
        hull_band_set(c, 0, n, m1, band, true);
        V3<T> Bp[2] = {vmk<T>(L.sx[0], L.sy[0], L.sz[0]), vmk<T>(L.sx[1], L.sy[1], L.sz[1])};
        __builtin_amdgcn_wave_barrier();
        hull_band_set(c, 1, nn, m2, band, true);
        return contact_case04(c, n2, Bp, res);
    } else if (n1 >= 3 && n2 == 2) {
        hull_band_set(c, 1, nn, m2, band, true);
        V3<T> Bp[2] = {vmk<T>(L.sx[0], L.sy[0], L.sz[0]), vmk<T>(L.sx[1], L.sy[1], L.sz[1])};
        __builtin_amdgcn_wave_barrier();
        hull_band_set(c, 0, n, m1, band, true);
        return contact_case04(c, n1, Bp, res);
    } else if (n1 >= 3 && n2 >= 3) {                               // case_05
        hull_band_set(c, 0, n, m1, band, true);
        T sx = 0, sy = 0, sz = 0;
        for (int i = 0; i < n1; ++i) { sx += L.sx[i]; sy += L.sy[i]; sz += L.sz[i]; }
        T dn = (T)n1;
        res = vmk<T>(sx / dn, sy / dn, sz / dn);
    } else {
        return GJKEPA_STATUS_DEGENERATE;                           // :498-501
    }
    return 0;
}

// get_collisionPoint_03 (:426-452)
template <typename T, int K, int VC, int FC>
DEV int contact_v3(Ctx<T, K, VC, FC>& c, V3<T> n, V3<T>& res, V3<T>& nnew) {
    V3<T> nn = vneg(n);
    T mx = -Tol<T>::BIG;
    int idx = -1;
    for (int i = 0; i < c.h.nb; ++i) {
        T t = dot(nn, c.B(i));
        if (t > mx - Tol<T>::PT) { mx = t; idx = i; }
    }
    if (idx < 0) return GJKEPA_STATUS_DEGENERATE;
    T sz = 0;
    for (int i = 0; i < c.h.na; ++i) sz += c.L.hz[0][i];
    res = c.B(idx);
    res.z = sz / (T)(float)c.h.na;
    V3<T> q = vmk<T>(n.x, n.y, T(0));
    T nq = norm2(q);
    nnew = vdiv(q, nq);
    return 0;
}

// ---------------------------------------------------------------- one pair (GJKEPA :39-239)
struct Out { int status; int hit; };

template <typename T, int K, int VC, int FC>
DEV int gjkepa_pair(Ctx<T, K, VC, FC>& c, int version, T tol_ff, T* o13, int& hit, uint32_t& diag) {
    const V3<T> O = zero3<T>();
    hit = 0;
    diag = 0;
#pragma unroll
    for (int i = 0; i < 13; ++i) o13[i] = T(0);
    auto& L = c.L;
    // --- RoughCollisionDetection_SphericalEnvelope (:1165-1188)
    {
        T s0 = 0, s1 = 0, s2 = 0, t0 = 0, t1 = 0, t2 = 0;
        for (int i = 0; i < c.h.na; ++i) { s0 += L.hx[0][i]; s1 += L.hy[0][i]; s2 += L.hz[0][i]; }
        for (int i = 0; i < c.h.nb; ++i) { t0 += L.hx[1][i]; t1 += L.hy[1][i]; t2 += L.hz[1][i]; }
        T dna = (T)c.h.na, dnb = (T)c.h.nb;
        V3<T> m1 = vmk<T>(s0 / dna, s1 / dna, s2 / dna), m2 = vmk<T>(t0 / dnb, t1 / dnb, t2 / dnb);
        T r1 = -Tol<T>::BIG, r2 = -Tol<T>::BIG;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            int i = k * kWave + c.lane;
            T ta = norm2(vsub(vmk<T>(c.h.ax[k], c.h.ay[k], c.h.az[k]), m1));
            if (i < c.h.na && ta > r1) r1 = ta;
            T tb = norm2(vsub(vmk<T>(c.h.bx[k], c.h.by[k], c.h.bz[k]), m2));
            if (i < c.h.nb && tb > r2) r2 = tb;
        }
        r1 = wave_max(r1);
        r2 = wave_max(r2);
        if (!unib(norm2(vsub(m1, m2)) <= r1 + r2 + T(1))) return 0;
    }
    // --- initial simplex (:82-170)
    V3<T> S[4] = {O, O, O, O};   // fresh SAVE state: stale row 4 = 0
    int iter = 0;
    V3<T> dir;
    for (;;) {
        ++iter;
        if (iter > 99) return 0;
        dir = vmk<T>((T)kDirTab[iter - 1][0], (T)kDirTab[iter - 1][1], (T)kDirTab[iter - 1][2]);
        S[0] = support(c, dir);
        dir = vneg(dir);
        S[1] = support(c, dir);
        if (!unib(allclose8(S[0], S[1]))) break;
    }
    dir = vec_pl(O, S[0], S[1]);
    S[2] = support(c, dir);
    if (unib(allclose8(S[2], S[0]) || allclose8(S[2], S[1]))) return 0;
    dir = utzvec(cross(vsub(S[1], S[0]), vsub(S[2], S[1])));
    const V3<T> VO = vsub(O, S[2]);
    const T vd = dot(VO, dir);
    int gjk_it = 0;
    bool enter = false;
    if (unib(fabs(vd) < Tol<T>::PT)) {
        if (unib(inside_tri(S[0], S[1], S[2], O))) enter = true;
    }
    if (!enter) {
        if (unib(vd < T(0))) dir = vneg(dir);
        S[3] = support(c, dir);
        {
            V3<T> n = uninml(S[0], S[1], S[2]);                         // DIST_PF_SIGN (:157)
            if (unib(is_zero_nml(n))) { hit = 1; return GJKEPA_STATUS_DEGENERATE; }
            if (unib(fabs(dot(vsub(S[3], S[0]), n)) < Tol<T>::PT)) return 0;
        }
        if (unib(origin_in_simplex(S))) enter = true;
    }
    if (!enter) {
        V3<T> L1[4] = {O, O, O, O}, L2[4] = {O, O, O, O};
        for (int it = 1;; ++it) {                                           // :182-236
            gjk_it = it;
            if (it > 50) return 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) { L2[i] = L1[i]; L1[i] = S[i]; }
            update_simplex(c, S);
            if (unib(norm2(cross(vsub(S[1], S[0]), vsub(S[2], S[1]))) < Tol<T>::PT)) return 0;
            V3<T> n = uninml(S[0], S[1], S[2]);
            if (unib(is_zero_nml(n))) { hit = 1; diag = (uint32_t)gjk_it; return GJKEPA_STATUS_DEGENERATE; }
            if (unib(fabs(dot(vsub(S[3], S[0]), n)) < Tol<T>::PT)) return 0;
            if (unib(origin_in_simplex(S))) break;
            bool over = true;
#pragma unroll
            for (int i = 0; i < 4; ++i) over = over && (allclose8(S[i], L1[i]) || allclose8(S[i], L2[i]));
            if (unib(over)) return 0;
        }
    }
    // --- EPA_solu (:242-346)
    hit = 1;
    T depth = 0;
    V3<T> n = O;
    int eit = 0, nf = 0;
    int st = epa(c, S, depth, n, eit, nf);
    diag = (uint32_t)(gjk_it & 0xff) | ((uint32_t)(eit & 0xff) << 8) | ((uint32_t)(nf & 0xffff) << 16);
    if (st) return st;
    int ia, ib;
    support_idx(c, n, ia, ib);                                              // get_nearest_points (:813-855)
    V3<T> q1 = c.A(ia), q2 = c.B(ib);
    V3<T> pt = O;
    if (version == 1) st = contact_v1(c, n, pt);
    else if (version == 2) st = contact_v2(c, n, pt);
    else if (version == 3) { V3<T> nw; st = contact_v3(c, n, pt, nw); n = nw; }
    else st = GJKEPA_STATUS_BAD_VERSION;
    if (st) return st;
    int type = collision_type(c, n, tol_ff);                                // :343
    o13[0] = depth;
    o13[1] = n.x; o13[2] = n.y; o13[3] = n.z;
    o13[4] = pt.x; o13[5] = pt.y; o13[6] = pt.z;
    o13[7] = q1.x; o13[8] = q1.y; o13[9] = q1.z;
    o13[10] = q2.x; o13[11] = q2.y; o13[12] = q2.z;
    return -type;   // negative: OK with colli_type
}

// ---------------------------------------------------------------- kernel
template <typename T> struct RecWords { static constexpr int N = sizeof(T) == 8 ? 32 : 16; };

template <typename TIn, typename T, int K, int VC, int FC>
__global__ __launch_bounds__(64) void gjkepa_tier_kernel(
    int version, double tol_ff, const TIn* __restrict__ verts, const int64_t* __restrict__ hull_off,
    const int32_t* __restrict__ hull_cnt, const int32_t* __restrict__ pairs, int64_t n_pairs,
    const int32_t* __restrict__ in_list, const int32_t* __restrict__ in_count,
    int32_t* __restrict__ out_list, int32_t* __restrict__ out_count, void* __restrict__ out) {
    extern __shared__ __align__(16) unsigned char smem[];
    auto& L = *reinterpret_cast<Lds<T, K, VC, FC>*>(smem);
    const int lane = lane_id();
    const int64_t total = in_list ? (int64_t)(*in_count) : n_pairs;
    for (int64_t w = blockIdx.x; w < total; w += gridDim.x) {
        const int64_t pair = in_list ? (int64_t)in_list[w] : w;
        Ctx<T, K, VC, FC> c{L, {}, lane};
        const int32_t ha = pairs[2 * pair], hb = pairs[2 * pair + 1];
        const int na = uni(hull_cnt[ha]), nb = uni(hull_cnt[hb]);
        int status = 0, hit = 0, type = 0;
        uint32_t diag = 0;
        T o13[13];
#pragma unroll
        for (int i = 0; i < 13; ++i) o13[i] = T(0);
        bool defer = false;
        if (na < 1 || nb < 1 || na > GJKEPA_MAX_HULL_VERTS || nb > GJKEPA_MAX_HULL_VERTS) {
            status = GJKEPA_STATUS_BAD_INPUT;
        } else if (na > K * kWave || nb > K * kWave) {
            defer = true;
        } else {
            const TIn* pa = verts + hull_off[ha];
            const TIn* pb = verts + hull_off[hb];
            c.h.na = na;
            c.h.nb = nb;
            bool nonfinite = false;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                int i = k * kWave + lane;
                T ax = 0, ay = 0, az = 0, bx = 0, by = 0, bz = 0;
                if (i < na) { ax = (T)pa[i]; ay = (T)pa[na + i]; az = (T)pa[2 * na + i]; }
                if (i < nb) { bx = (T)pb[i]; by = (T)pb[nb + i]; bz = (T)pb[2 * nb + i]; }
                nonfinite = nonfinite || !isfinite(ax) || !isfinite(ay) || !isfinite(az) ||
                            !isfinite(bx) || !isfinite(by) || !isfinite(bz);
                c.h.ax[k] = ax; c.h.ay[k] = ay; c.h.az[k] = az;
                c.h.bx[k] = bx; c.h.by[k] = by; c.h.bz[k] = bz;
                L.hx[0][i] = ax; L.hy[0][i] = ay; L.hz[0][i] = az;
                L.hx[1][i] = bx; L.hy[1][i] = by; L.hz[1][i] = bz;
            }
            __builtin_amdgcn_wave_barrier();
            if (unib(ballot(nonfinite) != 0)) {
                status = GJKEPA_STATUS_BAD_INPUT;
            } else {
                const int r = gjkepa_pair(c, version, (T)tol_ff, o13, hit, diag);
                if (r == ST_DEFER) {
                    defer = true;
                } else if (r < 0) {
                    type = -r;                      // OK hit, colli_type
                } else if (r > 0) {                 // error status: outputs zero, collision = 1
                    status = r;
                    hit = 1;
#pragma unroll
                    for (int i = 0; i < 13; ++i) o13[i] = T(0);
                }
            }
        }
        if (defer && !out_list) {                   // last tier: capacity exhausted
            defer = false;
            status = GJKEPA_STATUS_DEGENERATE;
            hit = 1;
#pragma unroll
            for (int i = 0; i < 13; ++i) o13[i] = T(0);
        }
        if (defer) {
            if (lane == 0) {
                int pos = atomicAdd(out_count, 1);
                out_list[pos] = (int32_t)pair;
            }
            continue;
        }
        // stage the record: 13 T fields, then int8 collision, type, status, reserved, uint32 diag
        if (lane == 0) {
            T* tf = reinterpret_cast<T*>(L.rec);
#pragma unroll
            for (int i = 0; i < 13; ++i) tf[i] = o13[i];
            uint32_t* w = L.rec + (13 * sizeof(T)) / 4;
            w[0] = (uint32_t)(hit & 0xff) | ((type & 0xffu) << 8) | ((uint32_t)(status & 0xff) << 16);
            w[1] = diag;
            for (int i = (13 * (int)sizeof(T)) / 4 + 2; i < RecWords<T>::N; ++i) L.rec[i] = 0u;
        }
        __builtin_amdgcn_wave_barrier();
        uint32_t* dst = reinterpret_cast<uint32_t*>(out) + pair * RecWords<T>::N;
        if (lane < RecWords<T>::N) dst[lane] = L.rec[lane];
        __builtin_amdgcn_wave_barrier();
    }
}

}  // namespace gk

// ---------------------------------------------------------------- host-side launch table
namespace {

template <typename TIn, typename T, int K, int VC, int FC>
hipError_t launch_tier(const gjkepa_tier_args& a, hipStream_t s) {
    using Img = gk::Lds<T, K, VC, FC>;
    auto kfn = gk::gjkepa_tier_kernel<TIn, T, K, VC, FC>;
    const size_t lds = sizeof(Img);
    int grid = a.grid;
    if (grid <= 0) {
        int per_cu = 0;
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, 64, lds);
        if (e != hipSuccess) return e;
        if (per_cu < 1) per_cu = 1;
        grid = per_cu * a.num_cus;
    }
    if (!a.in_list && a.n_pairs < grid) grid = (int)(a.n_pairs > 0 ? a.n_pairs : 1);
    hipLaunchKernelGGL(kfn, dim3(grid), dim3(64), lds, s, a.version, a.tol_ff, (const TIn*)a.verts,
                       a.hull_off, a.hull_cnt, a.pairs, a.n_pairs, a.in_list, a.in_count, a.out_list,
                       a.out_count, a.out);
    return hipGetLastError();
}

template <typename TIn, typename T>
hipError_t launch_any(int tier, const gjkepa_tier_args& a, hipStream_t s) {
    switch (tier) {
        case 0: return launch_tier<TIn, T, GJKEPA_T0_K, GJKEPA_T0_VCAP, GJKEPA_T0_FCAP>(a, s);
        case 1: return launch_tier<TIn, T, GJKEPA_T1_K, GJKEPA_T1_VCAP, GJKEPA_T1_FCAP>(a, s);
        default: return launch_tier<TIn, T, GJKEPA_T2_K, GJKEPA_T2_VCAP, GJKEPA_T2_FCAP>(a, s);
    }
}

}  // namespace

hipError_t gjkepa_launch_tier(int tier, int vert_dtype, int precision, const gjkepa_tier_args& a, hipStream_t s) {
    if (vert_dtype == GJKEPA_DTYPE_F32) {
        return precision == GJKEPA_PREC_F64 ? launch_any<float, double>(tier, a, s) : launch_any<float, float>(tier, a, s);
    }
    return precision == GJKEPA_PREC_F64 ? launch_any<double, double>(tier, a, s) : launch_any<double, float>(tier, a, s);
}

size_t gjkepa_tier_lds_bytes(int tier, int precision) {
    if (precision == GJKEPA_PREC_F64) {
        switch (tier) {
            case 0: return sizeof(gk::Lds<double, GJKEPA_T0_K, GJKEPA_T0_VCAP, GJKEPA_T0_FCAP>);
            case 1: return sizeof(gk::Lds<double, GJKEPA_T1_K, GJKEPA_T1_VCAP, GJKEPA_T1_FCAP>);
            default: return sizeof(gk::Lds<double, GJKEPA_T2_K, GJKEPA_T2_VCAP, GJKEPA_T2_FCAP>);
        }
    }
    switch (tier) {
        case 0: return sizeof(gk::Lds<float, GJKEPA_T0_K, GJKEPA_T0_VCAP, GJKEPA_T0_FCAP>);
        case 1: return sizeof(gk::Lds<float, GJKEPA_T1_K, GJKEPA_T1_VCAP, GJKEPA_T1_FCAP>);
        default: return sizeof(gk::Lds<float, GJKEPA_T2_K, GJKEPA_T2_VCAP, GJKEPA_T2_FCAP>);
    }
}
