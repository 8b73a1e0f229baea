// gk_common.h — device primitives shared by the CDNA4 kernels of this library (GJK/EPA narrow
// phase in gjkepa_kernel.hip, batched convex hulls in hull_kernel.hip): tolerance tables, 3-vector
// arithmetic in the oracle's operation order (oracle/gjkepa_oracle.c), and wave64 group
// primitives (lane ids, DPP / permlane butterflies, group argmax/argmin).
#pragma once
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdint>

#ifndef GJKEPA_FMAX_REDUCE
#define GJKEPA_FMAX_REDUCE 1
#endif

namespace gk {

#define DEV __device__ __forceinline__

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
    // fp32 certificate (gjkepa_kernel.hip, epa_close), relative to the depth d (the north star's 1e-6
    // relative): the polytope's MINLOC distance may not drop by more than CERT_DROP x d between
    // iterations, and at termination the support gap h_M(n) - d plus the fp32 evaluation noise of both terms,
    // CERT_NOISE x (|A| + |B|) (|A|: hull A's largest |coordinate|; the Minkowski point's coordinates carry
    // one rounding of a - b, its dot product three more), must stay within CERT_GAP x d.  Everything else is
    // recomputed in fp64.  CPU model sweep (tools/fp32_cert_sweep.py, 65,536 C2 pairs): noise allowance
    // 0 / 2 / 4 / 8 ulps of |A| + |B| -> 0.9% / 30% / 51% / 73% of the pairs recomputed, 160 / 0 / 0 / 0
    // depths outside 1e-6 relative; 4 ulps is the shipped margin.  At C2's scale every pair shallower than
    // about 1 is recomputed: fp32 coordinates cannot resolve its depth to 1e-6 relative.
    static constexpr float CERT_DROP = 5.0e-7f;
    static constexpr float CERT_GAP = 5.0e-7f;
    static constexpr float CERT_NOISE = 2.384185791015625e-07f;   // 4 x 2^-24
    // and the final face's unit normal: its fp32 rounding error, bounded from the face's edges e1, e2 by
    // (2 sqrt3 u (|A| + |B|) (|e1| + |e2|) + 3 u |e1| |e2|) / |e1 x e2| + 2 u (u = 2^-24: the Minkowski
    // points' coordinate error propagated through the cross product, then the normalisation), must stay
    // within CERT_ANGLE radians, half the gate's 1e-5 (CPU model sweep, 65,536 pairs: C5's largest non-tie
    // angle 3.4e-6 -> 1.1e-6 rad, 0.3% -> 2.3% of its pairs recomputed; C2 / C4 +0.2 / +1.9 points)
    static constexpr float CERT_ANGLE = 5.0e-6f;
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
template <typename T> DEV bool veq(V3<T> a, V3<T> b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
template <typename T> DEV V3<T> vsel(bool c, V3<T> a, V3<T> b) { return vmk<T>(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z); }
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
template <typename T> DEV V3<T> centroid4(V3<T> s0, V3<T> s1, V3<T> s2, V3<T> s3) {   // SUM(simplex_(:,k)) / 4
    return vmk<T>((((s0.x + s1.x) + s2.x) + s3.x) / T(4), (((s0.y + s1.y) + s2.y) + s3.y) / T(4),
                  (((s0.z + s1.z) + s2.z) + s3.z) / T(4));
}
template <typename T> DEV bool allclose8(V3<T> a, V3<T> b) {
    return fabs(a.x - b.x) < Tol<T>::PT && fabs(a.y - b.y) < Tol<T>::PT && fabs(a.z - b.z) < Tol<T>::PT;
}

// ---------------------------------------------------------------- group primitives
DEV int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
DEV int mbcnt(uint64_t m) {   // set bits of m below this lane
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
DEV int popc(uint64_t m) { return __popcll(m); }

// cross-lane exchange with the butterfly partner of step S (lane ^ 1, ^2, within 8, within 16,
// across 16-lane rows, across 32-lane halves).  After steps 0..S-1 every 2^S-lane block holds a
// uniform value, so the mirror steps act as xor steps for reductions.
template <int S> DEV uint32_t xchg32(uint32_t x) {
    if constexpr (S == 0) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    else if constexpr (S == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    else if constexpr (S == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, false); // row_half_mirror
    else if constexpr (S == 3) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, false); // row_mirror
    else if constexpr (S == 4) {
        auto p = __builtin_amdgcn_permlane16_swap(x, x, false, false);   // odd rows <-> even rows
        return ((lane_id() >> 4) & 1) ? p[0] : p[1];
    } else {
        auto p = __builtin_amdgcn_permlane32_swap(x, x, false, false);   // upper half <-> lower half
        return (lane_id() >> 5) ? p[0] : p[1];
    }
}
template <int S> DEV int xchg(int v) { return (int)xchg32<S>((uint32_t)v); }
template <int S> DEV float xchg(float v) { return __builtin_bit_cast(float, xchg32<S>(__builtin_bit_cast(uint32_t, v))); }
template <int S> DEV double xchg(double v) {
    uint64_t u = __builtin_bit_cast(uint64_t, v);
    uint64_t lo = xchg32<S>((uint32_t)u), hi = xchg32<S>((uint32_t)(u >> 32));
    return __builtin_bit_cast(double, (hi << 32) | lo);
}

template <int G> struct Grp {
    static constexpr int kSteps = G == 64 ? 6 : G == 32 ? 5 : G == 16 ? 4 : G == 8 ? 3 : G == 4 ? 2 : G == 2 ? 1 : 0;
    int lane, gl;
    uint64_t gmask;
    DEV Grp() : lane(lane_id()) {
        gl = lane & (G - 1);
        gmask = G == 64 ? ~0ull : (((1ull << (G & 63)) - 1ull) << (lane & ~(G - 1)));
    }
    // group-uniform value as a scalar when the group is the whole wave
    DEV int uni(int x) const { if constexpr (G == 64) return __builtin_amdgcn_readfirstlane(x); else return x; }
    DEV bool unib(bool b) const { if constexpr (G == 64) return __builtin_amdgcn_readfirstlane((int)b) != 0; else return b; }
    DEV uint64_t ballot(bool p) const { return __ballot(p) & gmask; }
    DEV bool any(bool p) const { return unib(ballot(p) != 0); }
    DEV bool all(bool p) const { return unib(ballot(!p) == 0); }
    DEV bool bit(uint64_t m) const { return (m >> lane) & 1ull; }
};

template <int S, int N, typename T> DEV void argmax_steps(T& v, int& i) {
    if constexpr (S < N) {
        T ov = xchg<S>(v);
        int oi = xchg<S>(i);
        bool take = (ov > v) || (ov == v && oi < i);
        v = take ? ov : v;
        i = take ? oi : i;
        argmax_steps<S + 1, N>(v, i);
    }
}
template <int S, int N, typename T> DEV void argmin_steps(T& v, int& i) {
    if constexpr (S < N) {
        T ov = xchg<S>(v);
        int oi = xchg<S>(i);
        bool take = (ov < v) || (ov == v && oi < i);
        v = take ? ov : v;
        i = take ? oi : i;
        argmin_steps<S + 1, N>(v, i);
    }
}
// Value-only max / min reductions.  Floating values take v_max_f64 / v_min_f64 (one instruction a
// step instead of compare + two selects): the callers only compare against the result or use values
// that cannot be -0 (squared norms, |distances|), and a NaN operand never wins — as in the
// reference's sequential `IF (t > mx)` scans.  (GJKEPA_FMAX_REDUCE=0: the select form, for A/B.)
template <typename T> DEV T red_max(T a, T b) {
    if constexpr (GJKEPA_FMAX_REDUCE && (sizeof(T) == 8 || sizeof(T) == 4) && T(0.5) != T(0)) return __builtin_fmax(a, b);
    else return a > b ? a : b;
}
template <typename T> DEV T red_min(T a, T b) {
    if constexpr (GJKEPA_FMAX_REDUCE && (sizeof(T) == 8 || sizeof(T) == 4) && T(0.5) != T(0)) return __builtin_fmin(a, b);
    else return a < b ? a : b;
}
template <int S, int N, typename T> DEV void max_steps(T& v) {
    if constexpr (S < N) {
        T ov = xchg<S>(v);
        v = red_max(ov, v);
        max_steps<S + 1, N>(v);
    }
}
// quad (4-lane) broadcast of lane j, DPP quad_perm [j,j,j,j]
template <int J> DEV uint32_t qb32(uint32_t x) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, J * 0x55, 0xF, 0xF, false); }
template <int J> DEV double qbcast(double v) {
    uint64_t u = __builtin_bit_cast(uint64_t, v);
    return __builtin_bit_cast(double, ((uint64_t)qb32<J>((uint32_t)(u >> 32)) << 32) | qb32<J>((uint32_t)u));
}
template <int J> DEV float qbcast(float v) { return __builtin_bit_cast(float, qb32<J>(__builtin_bit_cast(uint32_t, v))); }
DEV bool quad_all(bool b) { int x = b; x &= xchg<0>(x); x &= xchg<1>(x); return x != 0; }
// the value of the one quad lane where `mine` holds, on every lane of the quad (bitwise OR of the
// quad's masked values: exact, signed zeros included)
DEV double quad_pick(bool mine, double v) {
    uint64_t u = mine ? __builtin_bit_cast(uint64_t, v) : 0ull;
    uint32_t lo = (uint32_t)u, hi = (uint32_t)(u >> 32);
    lo |= xchg32<0>(lo); hi |= xchg32<0>(hi);
    lo |= xchg32<1>(lo); hi |= xchg32<1>(hi);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
DEV float quad_pick(bool mine, float v) {
    uint32_t u = mine ? __builtin_bit_cast(uint32_t, v) : 0u;
    u |= xchg32<0>(u);
    u |= xchg32<1>(u);
    return __builtin_bit_cast(float, u);
}
template <typename T> DEV V3<T> quad_pick(bool mine, V3<T> v) {
    return vmk<T>(quad_pick(mine, v.x), quad_pick(mine, v.y), quad_pick(mine, v.z));
}
DEV bool quad_any(bool b) { int x = b; x |= xchg<0>(x); x |= xchg<1>(x); return x != 0; }

// group-wide (value, index) argmax / argmin with lowest-index tie break; max
template <int G, typename T> DEV void gargmax(T& v, int& i) { argmax_steps<0, Grp<G>::kSteps>(v, i); }
template <int G, typename T> DEV void gargmin(T& v, int& i) { argmin_steps<0, Grp<G>::kSteps>(v, i); }
template <int G, typename T> DEV T gmax(T v) { max_steps<0, Grp<G>::kSteps>(v); return v; }
template <int S, int N, typename T> DEV void min_steps(T& v) {
    if constexpr (S < N) {
        T ov = xchg<S>(v);
        v = red_min(ov, v);
        min_steps<S + 1, N>(v);
    }
}
template <int G, typename T> DEV T gmin(T v) { min_steps<0, Grp<G>::kSteps>(v); return v; }

}  // namespace gk
