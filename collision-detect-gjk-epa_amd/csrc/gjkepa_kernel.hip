// gjkepa_kernel.hip — CDNA4 (gfx950) batched GJK/EPA narrow phase.
//
// What it computes: SUBROUTINE GJKEPA of src/GCLIB_GJKEPA.f90 (:39-239) for every pair of a
// pooled hull set; each device function cites the reference lines it follows.  The numerical
// recipe (operation order, no FMA contraction, sequential sums, first-index tie rules) is the
// same as oracle/gjkepa_oracle.c, so fp64 results compare bit for bit.
//
// Mapping onto the wavefront.  A *group* of G consecutive lanes (G = 16, 32 or 64) owns one pair,
// so a wave64 works on 64/G pairs at once; everything below is written for one group:
//   * hull vertices: lane l of the group owns vertices l, l+G, ... (K per hull) in registers, with
//     an LDS copy (storage precision) for random access; loaded with coalesced SoA loads.
//   * support mapping (:1030-1062): per-lane dot + argmax, then a log2(G)-step (value, index)
//     butterfly on DPP (quad_perm, row_half_mirror, row_mirror) and the gfx950 permlane16/32 swaps —
//     no LDS round trips; the lowest index wins ties like the reference's strict '>' scan.
//   * GJK simplex logic (:82-236): group-uniform scalar code (the group's lanes hold equal values;
//     groups of one wave diverge independently under EXEC masking).
//   * EPA polytope (:863-1022 + the re-supplied hull): vertices and faces (plane, |distance|,
//     packed vertex ids) in the group's LDS slice; face f lives on group lane f % G.  MINLOC,
//     visibility, horizon extraction, order-preserving compaction (ballot + mbcnt) and new-face
//     construction are lane-parallel.
//   * capacities are template parameters; a pair that does not fit a tier (hull above G*K
//     vertices, polytope beyond VC/FC) is appended to the next tier's work list and recomputed.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <type_traits>

#include "../../include/gjkepa.h"
#include "gjkepa_kernel.h"
#include "gk_common.h"

// Parts of the product build (the host-side launch table below): GK_IN(p) is true when this object
// compiles part p.
#ifdef GK_PART
#define GK_IN(p) (GK_PART == (p))
#else
#define GK_IN(p) 1
#endif

namespace gk {

constexpr int ST_DEFER = 100;   // internal: does not fit this tier
constexpr int ST_REDO = 103;    // internal (fp32 compute): answer not certified, recompute in fp64
constexpr int ST_PARKED = 104;  // internal: polytope parked for the next tier (gjkepa_kernel.h "Polytope parking")

// A compiler-only memory fence (no instruction): LDS reads after it are not hoisted above it.  Without
// it the scheduler issues a whole hull's K vertex loads (3K VGPRs in fp64: 6 per vertex) ahead of the
// dot products, and for hull B while hull A's are still live, which is where most of the GJK / EPA
// tiers' register peaks and scratch spills came from.
DEV void gk_lds_fence() { asm volatile("" ::: "memory"); }
// Per group width: the small-hull tiers (G < 32) lose by a fence (the hoisted loads are their memory-level
// parallelism: C2 -3 to -4% in round 5), the wide large-hull tiers spill without one.  A/B r6 (2 rounds):
// GJK tier 2's screen fenced (65 -> 14 spilled VGPRs) C4 42.55 -> 42.90; with EPA tier 3's dots too (52 -> 0)
// 42.98; the dots fence in GJK tier 1 or the 64-lane contact tier costs C5 0.7% / 0.3%, so it is EPA only.
#ifndef GJKEPA_SCREEN_FENCE_MIN_G
#define GJKEPA_SCREEN_FENCE_MIN_G 32  // fence between hull A's and hull B's fp32-screened scans in tiers with G >= this (0: none)
#endif
#ifndef GJKEPA_DOTS_FENCE_MIN_G
#define GJKEPA_DOTS_FENCE_MIN_G 64    // support_dots: fence between the two hulls' reads in EPA tiers with G >= this and K >= 4 (0: none)
#endif

// fp32 certificate.  An fp32 EPA can build an invalid polytope from inconsistent visibility decisions
// on near-coplanar faces (the fp32 rounding of a sliver's normal), after which its MINLOC distance
// drops and it may stop far from the penetration depth (C5: 20% low, normal off by 0.4 rad on one
// pair in 2^20).  In exact arithmetic EPA's MINLOC distance never decreases (each polytope contains
// the last) and at termination the support along the final normal lies on the final face, so the
// fp32 path checks both: a drop of more than CERT_DROP * d between iterations, or a support gap
// h_M(n) - d plus its fp32 evaluation noise (CERT_NOISE * (|A| + |B|)) above CERT_GAP * d when EPA stops,
// sends the pair to the redo launch, which recomputes it whole in fp64 (so do fp32 error statuses that
// fp64 may not share, and a polytope the origin is not strictly inside).  A certified answer has
// d <= h_M(n) <= d + gap, and d cannot exceed the depth of the polytope it came from.
template <typename T> DEV constexpr bool certify() { return sizeof(T) == 4; }
// fp32 compute: an EPA / contact outcome the fp64 recomputation may answer differently
template <typename T> DEV bool redo_status(int r, bool last_tier) {
    if constexpr (!certify<T>()) return false;
    return r == ST_REDO || r == GJKEPA_STATUS_EPA_MAXITER || r == GJKEPA_STATUS_DEGENERATE || (r == ST_DEFER && last_tier);
}

// GET_RANDOM_UNIT_VECTOR table (:1578-1689)
[[maybe_unused]] static __constant__ double kDirTab[100][3] = {
#include "dirtab.inc"
};

// ---------------------------------------------------------------- diagnostic phase stamps
// Built only with -DGJKEPA_DIAG_STAMPS (tools/build_variant.sh): wave time between consecutive
// stamps is charged to the phase that ends at the stamp (s_memtime ticks, summed over waves).
#ifdef GJKEPA_DIAG_STAMPS
constexpr int kStamps = 32;
__device__ unsigned long long g_stamps[kStamps];
__shared__ unsigned long long s_stamp[kStamps + 1];
DEV void stamp(int id) {
    const uint64_t t = __builtin_amdgcn_s_memtime();
    const uint64_t act = __ballot(1);
    if ((uint64_t)lane_id() == (uint64_t)__builtin_ctzll(act)) { s_stamp[id] += t - s_stamp[kStamps]; s_stamp[kStamps] = t; }
}
DEV void stamp_begin() {
    if (lane_id() == 0) {
        for (int i = 0; i < kStamps; ++i) s_stamp[i] = 0;
        s_stamp[kStamps] = __builtin_amdgcn_s_memtime();
    }
}
DEV void stamp_end() {
    if (lane_id() == 0)
        for (int i = 0; i < kStamps; ++i) if (s_stamp[i]) atomicAdd(&g_stamps[i], s_stamp[i]);
}
#define GK_STAMP(id) stamp(id)
#define GK_STAMP_BEGIN() stamp_begin()
#define GK_STAMP_END() stamp_end()
#elif defined(GJKEPA_DIAG_MARKERS)   // ISA region markers for static instruction counts (tools/isa_regions.py)
#define GK_STAMP(id) asm volatile("; GKMARK %0" ::"n"(id))
#define GK_STAMP_BEGIN() ((void)0)
#define GK_STAMP_END() ((void)0)
#else
#define GK_STAMP(id) ((void)0)
#define GK_STAMP_BEGIN() ((void)0)
#define GK_STAMP_END() ((void)0)
#endif
// ---------------------------------------------------------------- diagnostic argument guard
// Built only with -DGJKEPA_DIAG_GUARD: every kernel recomputes its argument block's checksum
// (gjkepa_guard_of) at entry; on a mismatch it counts the event in g_guard (read by
// gjkepa_diag_guard) and returns before any memory access the arguments describe.
#ifdef GJKEPA_DIAG_GUARD
__device__ uint32_t g_guard[8];   // [0] mismatches, [1] kernel id << 8 | route code, [2] expected, [3] recomputed
DEV void guard_report(uint32_t kid, uint32_t want, uint32_t got) {
    if (lane_id() == 0) {
        atomicAdd(&g_guard[0], 1u);
        atomicExch(&g_guard[1], kid);
        atomicExch(&g_guard[2], want);
        atomicExch(&g_guard[3], got);
    }
}
#define GK_GUARD(kid, code)                                                                   \
    do {                                                                                     \
        const uint32_t g_ = gjkepa_guard_of(a);                                              \
        if (g_ != a.guard) { guard_report(((uint32_t)(kid) << 8) | ((uint32_t)(code) & 0xffu), a.guard, g_); return; } \
    } while (0)
#else
#define GK_GUARD(kid, code) ((void)0)
#endif

enum { SG_LOAD = 0, SG_SPHERE, SG_INIT, SG_UPD, SG_CHK, SG_STORE, SG_ROUTE,
       SE_LOAD = 10, SE_IT1, SE_DIR, SE_SUP, SE_VIS, SE_HOR, SE_CMP, SE_CONE, SE_TERM, SE_NEAR, SE_CONT, SE_TYPE,
       SE_STORE, SE_ROUTE, SC_ROUTE, SC_LOAD, SC_STORE };


// ---------------------------------------------------------------- per-group LDS image
// Sized for the kernel that uses it: VC > 0 is the EPA polytope (VC vertices, FC face slots);
// VC == 0 is the GJK kernel (FC == 0) or the contact kernel (FC == 1), which carry only their own
// scratch, so a 16-pair GJK wave does not pay for polytope or contact arrays.
// FUSED: the one-kernel query path (query_kernel) keeps the contact arrays beside the polytope.
// One hull vertex in LDS (GJKEPA_HULL_AOS): x, y, z and a zero pad, so a lane fetches a whole
// vertex with one ds_read_b128 (fp32 storage) instead of three ds_read_b32 from three columns.
template <typename TH> struct alignas(16) HV { TH x, y, z, w; };

template <typename T, typename TH, int G, int K, int VC_, int FC_, bool FUSED = false> struct Lds {
    static constexpr int NH = G * K;
    // Coordinate columns are NH + 1 elements apart, so the six columns (hull A/B x, y, z) start on
    // six different banks: the sphere test reads element i of all six at once (one lane each).
    static constexpr int NHP = NH + GJKEPA_LDS_SKEW;
    static constexpr int VC = VC_ > 0 ? VC_ : 1, FC = VC_ > 0 ? FC_ : 1, GS = VC_ > 0 && !GJKEPA_EPA_PLACE ? G : 1;
    static constexpr int NC = ((VC_ == 0 && FC_ == 1) || FUSED) ? NH : 1;
    // Horizon list packing (GJKEPA_EPA_HPACK): a horizon edge is one word u | w << HVB | key << 2 HVB
    // (HVB bits per vertex id) where every face key fits the rest (kbase grows by at most 3 FC per hull
    // insertion, two insertions per iteration, <= 100 iterations), and the list holds FC / 2 edges
    // (hull_add defers a pair whose horizon is longer: at most VC edges, so only tiers with VC > FC / 2
    // can, and a 33-edge horizon on a polytope of at most 40 vertices is not seen).  EPA tiers 0 and 4
    // then fit a twelfth wave per CU.  Tiers whose polytopes are larger than that and whose occupancy
    // is set by registers (1 and 2, 72 / 128) keep the two-word list: packed, C5 lost 0.9%.
    static constexpr int HVB = VC_ <= 128 ? 7 : 8;
    static constexpr bool HPACK = GJKEPA_EPA_HPACK && VC_ > 0 && VC_ <= (1 << HVB) && (VC_ <= 40 || 2 * VC_ <= FC_) &&
                                  4 + 600LL * FC_ < (1LL << (32 - 2 * HVB));
    static constexpr int HC = HPACK ? FC / 2 : FC;
#if GJKEPA_HULL_AOS
    HV<TH> hv[2][NH];                       // hull A (0) / B (1) vertex i, storage precision
#else
    TH hx[2][NHP], hy[2][NHP], hz[2][NHP];  // hull A (0) / B (1) vertices, storage precision
#endif
    struct None {};
    struct E {                           // EPA polytope (faces themselves are in registers)
            T vx[VC], vy[VC], vz[VC];    // vertices by id
            T dsv[FC];                   // saved face distances by slot (termination test), NaN = none
            T best[3];                   // MINLOC face broadcast: normal, first vertex id
            uint32_t bestv;
            union X {
                struct H {                                                                 // hull_add lists
                    uint64_t visl[FC];                       // visible faces: ids | key << 32
                    uint32_t horu[HC], hork[HPACK ? 1 : FC]; // horizon edges: u | w << 8 (| new face key << 16 if HPACK), new face key
#if !GJKEPA_EPA_PLACE
                    T sn[GS][4];                             // new faces of one round: normal, |distance|
                    uint32_t sv[GS], sk[GS];                 //   ids, key
#endif
                } h;
                struct S { T srt[FC]; } s;                                                 // sorted_equal
                struct O { uint32_t key[FC]; uint32_t ord[FC]; } o;                       // centroid order
            } x;
    };
    // contact features: a point set (SPT) is a list of hull vertices, kept as vertex index | side << 15
    // and read back from the hull image (the same fp32 -> T conversion as when it was selected)
    struct C { T pol[NC]; uint32_t ord[NC]; uint16_t si[NC]; };
    // the GJK tiers (VC_ = FC_ = 0) carry nothing but the hulls, so GJK tier 0's 16 images fit 12 waves/CU
    union U {
        std::conditional_t<(VC_ > 0), E, None> e;
        std::conditional_t<(VC_ > 0 || FC_ > 0), C, None> c;
    } u;
};

// Byte distance between the LDS images of consecutive groups of a wave.  The images of the groups
// that share a 32-lane half (the unit ds_read/ds_write banks over) are skewed by an odd multiple of G dwords modulo
// the 32 four-byte banks, so group g's lane l and group g+1's lane l, touching the same field, hit
// different banks; an unpadded image size is often a multiple of 16 or 32 dwords, which puts every
// group of a half on the same banks (GJK tier 0: 16 groups, 8 per half, two distinct bank offsets).
// With GJKEPA_HULL_AOS the images are 16-byte aligned and, for G < 16, skewed by 4G dwords modulo
// 64 banks: the G lanes of a group read G consecutive 16-byte vertex records, so the 16-lane groups
// of a ds_read_b128 (16 / G groups) then cover 256 distinct bytes of banks.
template <typename L_t, int G> constexpr size_t lds_stride() {
    if constexpr (GJKEPA_HULL_AOS) {
        size_t dw = (sizeof(L_t) + 15) / 16 * 4;            // 16-byte aligned, in dwords
        if (GJKEPA_LDS_SKEW && G < 16)
            while (dw % 64 != (size_t)(4 * G)) dw += 4;
        return dw * 4;
    } else {
        size_t dw = (sizeof(L_t) + 7) / 8 * 2;              // 8-byte aligned, in dwords
        if (GJKEPA_LDS_SKEW && G < 32)                      // dw = G x odd (mod 32): the 32 / G groups
            while ((dw % 32) % G != 0 || ((dw % 32) / G) % 2 == 0) dw += 2;   // of a half on distinct banks
        return dw * 4;
    }
}

template <typename T, typename TH, int G, int K, int VC, int FC, int LH> struct Ctx {
    using L_t = Lds<T, TH, G, K, VC, FC, (LH == 2)>;
    L_t& L;
    Grp<G> g;
    // Hull vertex k*G + gl of each hull: in registers, or (LH 1: the tier's GJKEPA_*_LH; 2: the fused
    // query kernel, whose LDS image also holds the contact arrays) read from the
    // group's LDS copy at each use, which frees 6K registers per lane so the tier fits one more wave
    // per SIMD.  Same values either way (LDS holds the storage precision).
    static constexpr bool kRegHull = !LH;
    T ax[kRegHull ? K : 1], ay[kRegHull ? K : 1], az[kRegHull ? K : 1];
    T bx[kRegHull ? K : 1], by[kRegHull ? K : 1], bz[kRegHull ? K : 1];
    int na, nb;
    float vmax_a = 0, vmax_b = 0;   // largest |coordinate| of each hull (fp32 support screen)
#if GJKEPA_HULL_AOS
    // vertex i of hull h in storage precision, fetched whole (one 16-byte LDS read for fp32)
    DEV V3<TH> raw(int h, int i) const {
        if constexpr (sizeof(TH) == 4) {
            typedef float f4 __attribute__((ext_vector_type(4)));
            const f4 v = *reinterpret_cast<const f4*>(&L.hv[h][i]);
            return vmk<TH>(v.x, v.y, v.z);
        } else {
            const HV<TH> v = L.hv[h][i];
            return vmk<TH>(v.x, v.y, v.z);
        }
    }
    DEV TH rawc(int h, int i, int ax) const { return ax == 0 ? L.hv[h][i].x : ax == 1 ? L.hv[h][i].y : L.hv[h][i].z; }
#else
    DEV V3<TH> raw(int h, int i) const { return vmk<TH>(L.hx[h][i], L.hy[h][i], L.hz[h][i]); }
    DEV TH rawc(int h, int i, int ax) const { return ax == 0 ? L.hx[h][i] : ax == 1 ? L.hy[h][i] : L.hz[h][i]; }
#endif
    DEV V3<T> A(int i) const { const V3<TH> v = raw(0, i); return vmk<T>((T)v.x, (T)v.y, (T)v.z); }
    DEV V3<T> B(int i) const { const V3<TH> v = raw(1, i); return vmk<T>((T)v.x, (T)v.y, (T)v.z); }
    // this lane's k-th vertex (k*G + gl) of hull A / B as a whole vector
    DEV V3<T> AV(int k) const { if constexpr (kRegHull) return vmk<T>(ax[k], ay[k], az[k]); else return A(k * G + g.gl); }
    DEV V3<T> BV(int k) const { if constexpr (kRegHull) return vmk<T>(bx[k], by[k], bz[k]); else return B(k * G + g.gl); }
    DEV T Ax(int k) const { if constexpr (kRegHull) return ax[k]; else return (T)rawc(0, k * G + g.gl, 0); }
    DEV T Ay(int k) const { if constexpr (kRegHull) return ay[k]; else return (T)rawc(0, k * G + g.gl, 1); }
    DEV T Az(int k) const { if constexpr (kRegHull) return az[k]; else return (T)rawc(0, k * G + g.gl, 2); }
    DEV T Bx(int k) const { if constexpr (kRegHull) return bx[k]; else return (T)rawc(1, k * G + g.gl, 0); }
    DEV T By(int k) const { if constexpr (kRegHull) return by[k]; else return (T)rawc(1, k * G + g.gl, 1); }
    DEV T Bz(int k) const { if constexpr (kRegHull) return bz[k]; else return (T)rawc(1, k * G + g.gl, 2); }
    DEV V3<T> vert(int i) const { return vmk<T>(L.u.e.vx[i], L.u.e.vy[i], L.u.e.vz[i]); }
};
#define CTX_T template <typename T, typename TH, int G, int K, int VC, int FC, int LH>
#define CTX Ctx<T, TH, G, K, VC, FC, LH>

// ---------------------------------------------------------------- support mapping (:1030-1062)
// indices: argmax_i d.a_i (first), argmax_j (-d).b_j (first); -dot(d,b) == dot(-d,b) bit for bit.
// The group max of the values is reduced alone; the lowest index holding it is then found with
// one ballot per register slot k (index k*G + lane: lower k first, then lower lane).
// fp32-screened support (GJKEPA_SCREEN_MIN_K; fp64 compute over fp32-stored hulls): the dots are
// first taken in fp32 from the stored coordinates (no conversions, half-rate-free arithmetic).  With
// S = |d|_1 max|v| (vmax: the hull's largest |coordinate|), every fp32 dot is within 4.0001 * 2^-24 S
// of the exact dot and every fp64 dot within 2^-51 S, so a vertex whose fp32 dot is below the fp32
// maximum by more than 2E = 2^-18 |d|_1 vmax (E = 32 * 2^-24 * S: 8x margin) has a strictly smaller
// fp64 dot than the fp32 maximum's vertex and cannot be the fp64 argmax.  Only the remaining
// candidates (usually one per group) get the fp64 dot, in this lane's index order, and the group
// takes the largest value, lowest index on ties: the same index as the plain scan.  A non-finite
// screen (overflow, NaN direction) makes every vertex a candidate.
template <int K> struct ScreenOn {
    static constexpr bool value = GJKEPA_SCREEN_MIN_K > 0 && K >= GJKEPA_SCREEN_MIN_K;
};
CTX_T DEV void screened_idx(const CTX& c, V3<T> d, int h, float vmax, int& out) {
    const float fx = (float)d.x, fy = (float)d.y, fz = (float)d.z;
    const float sg = h ? -1.0f : 1.0f;
    const int n = h ? c.nb : c.na;
    float sv[K];
    float m = -FLT_MAX;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int i = k * G + c.g.gl;
        // GJKEPA_PAD_V0: slots past the count hold vertex 0 again, whose screen value can only make
        // vertex 0's duplicates candidates too (then the full path below takes the lowest index)
        const V3<TH> v = c.raw(h, GJKEPA_PAD_V0 || i < n ? i : 0);
        const float t = sg * fmaf(fz, v.z, fmaf(fy, v.y, fx * v.x));
        sv[k] = GJKEPA_PAD_V0 || i < n ? t : -FLT_MAX;
        m = fmaxf(m, sv[k]);
    }
    m = gmax<G>(m);
    // a bound below 2^-90 may have lost terms to fp32 underflow (|d_i| |v| flushed): then every vertex
    // is a candidate (the plain fp64 scan), as for a non-finite screen
    const float bnd = (fabsf(fx) + fabsf(fy) + fabsf(fz)) * vmax;
    const float thr = bnd >= 0x1p-90f ? m - 0x1p-18f * bnd : -INFINITY;
    uint32_t cand = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int i = k * G + c.g.gl;
        if ((GJKEPA_PAD_V0 || i < n) && !(sv[k] < thr)) cand |= 1u << k;      // NaN threshold or value: candidate
    }
    if constexpr (GJKEPA_SCREEN_SINGLE) {
        // one candidate in the whole group (the usual case): it is the fp64 argmax, so its index is
        // the answer without its fp64 dot or the fp64 group reduction (an int group min only)
        const uint64_t lanes = c.g.ballot(cand != 0);
        if (!c.g.any(__builtin_popcount(cand) > 1) && popc(lanes) <= 1) {
            const int key = gmin<G>(cand ? (int)__builtin_ctz(cand) * G + c.g.gl : 0x7FFFFFFF);
            out = c.g.uni(key == 0x7FFFFFFF ? 0 : key);
            return;
        }
    }
    T best = -Tol<T>::BIG;
    int bi = 0x7FFFFFFF;
    while (cand) {                                          // this lane's candidates in index order
        const int k = __builtin_ctz(cand);
        cand &= cand - 1u;
        const int i = k * G + c.g.gl;
        const V3<T> v = h ? c.B(i) : c.A(i);
        const T t = h ? -(d.x * v.x + d.y * v.y + d.z * v.z) : d.x * v.x + d.y * v.y + d.z * v.z;
        if (t > best) { best = t; bi = i; }
    }
    const T vm = gmax<G>(best);
    const int key = gmin<G>(best == vm ? bi : 0x7FFFFFFF);
    out = c.g.uni(key == 0x7FFFFFFF ? 0 : key);
}

// This lane's dots with one direction d over both hulls: t[0][k] = d.a_(kG+gl), t[1][k] = -(d.b_(kG+gl))
// (= (-d).b bit for bit up to a zero's sign), -BIG past the hull, and the group maxima m[0], m[1]:
// get_nearest_points' argmax values, and get_info_collisionType's / the contact points' HUGE-start
// max scans (:381, :401, :471-472) for the same direction.
template <typename T, int K> struct DotSet { T t[2][K]; T m[2]; };

// GJKEPA_PAD_V0: the hull slots past a hull's count hold copies of its vertex 0 (load_hulls), whose dot
// can tie only with vertex 0 itself at a higher index, so the lowest-index argmax and the maxima are the
// plain scan's without masking the padding (three VALU per vertex and hull); the contact band sets,
// which count members, still mask by index.
CTX_T DEV T dot_slot(int i, int n, T t) {
    if constexpr (GJKEPA_PAD_V0) return t;
    else return i < n ? t : -Tol<T>::BIG;
}
// this lane's running maximum of the dots: v_max_f64 (red_max) instead of compare + two selects
template <typename T> DEV T dots_max(T t, T v) {
    if constexpr (GJKEPA_DOTS_FMAX) return red_max(t, v);
    else return t > v ? t : v;
}
CTX_T DEV void support_dots(const CTX& c, V3<T> d, DotSet<T, K>& D, int& ia, int& ib) {
    T (&ta)[K] = D.t[0];
    T (&tb)[K] = D.t[1];
    T va = -Tol<T>::BIG, vb = -Tol<T>::BIG;
    if constexpr (GJKEPA_DOTS_FENCE_MIN_G > 0 && G >= GJKEPA_DOTS_FENCE_MIN_G && K >= 4 && VC > 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int i = k * G + c.g.gl;
        const V3<T> a = c.AV(k);
        ta[k] = dot_slot<T, TH, G, K, VC, FC, LH>(i, c.na, d.x * a.x + d.y * a.y + d.z * a.z);
        va = dots_max(ta[k], va);
    }
    gk_lds_fence();                      // hull B's vertices are read after hull A's dots
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int i = k * G + c.g.gl;
        const V3<T> b = c.BV(k);
        tb[k] = dot_slot<T, TH, G, K, VC, FC, LH>(i, c.nb, -(d.x * b.x + d.y * b.y + d.z * b.z));
        vb = dots_max(tb[k], vb);
    }
    } else {
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int i = k * G + c.g.gl;
        const V3<T> a = c.AV(k), b = c.BV(k);
        ta[k] = dot_slot<T, TH, G, K, VC, FC, LH>(i, c.na, d.x * a.x + d.y * a.y + d.z * a.z);
        tb[k] = dot_slot<T, TH, G, K, VC, FC, LH>(i, c.nb, -(d.x * b.x + d.y * b.y + d.z * b.z));
        va = dots_max(ta[k], va);
        vb = dots_max(tb[k], vb);
    }
    }
    va = gmax<G>(va);
    vb = gmax<G>(vb);
    const int sh = c.g.lane & ~(G - 1);
    int xa = -1, xb = -1;
#pragma unroll
    for (int k = K - 1; k >= 0; --k) {
        const uint64_t ma = (__ballot(ta[k] == va) >> sh) & (G == 64 ? ~0ull : ((1ull << (G & 63)) - 1ull));
        const uint64_t mb = (__ballot(tb[k] == vb) >> sh) & (G == 64 ? ~0ull : ((1ull << (G & 63)) - 1ull));
        if (ma) xa = k * G + (int)__builtin_ctzll(ma);
        if (mb) xb = k * G + (int)__builtin_ctzll(mb);
    }
    ia = c.g.uni(xa < 0 ? 0 : xa);
    ib = c.g.uni(xb < 0 ? 0 : xb);
    D.m[0] = va;
    D.m[1] = vb;
}

CTX_T DEV void support_idx(const CTX& c, V3<T> d, int& ia, int& ib) {
    if constexpr (ScreenOn<K>::value && sizeof(T) == 8 && sizeof(TH) == 4) {
        screened_idx(c, d, 0, c.vmax_a, ia);
        if constexpr (GJKEPA_SCREEN_FENCE_MIN_G > 0 && G >= GJKEPA_SCREEN_FENCE_MIN_G)
            gk_lds_fence();              // hull B's screen reads its vertices after hull A's is done
        screened_idx(c, d, 1, c.vmax_b, ib);
        return;
    }
    DotSet<T, K> D;
    support_dots(c, d, D, ia, ib);
}
CTX_T DEV V3<T> support(const CTX& c, V3<T> d) {
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
    T c0 = (V1.x - V0.x) * (P.y - V0.y) - (V1.y - V0.y) * (P.x - V0.x);
    T c1 = (V2.x - V1.x) * (P.y - V1.y) - (V2.y - V1.y) * (P.x - V1.x);
    T c2 = (V0.x - V2.x) * (P.y - V2.y) - (V0.y - V2.y) * (P.x - V2.x);
    if (fabs(c0) < Tol<T>::Z) c0 = T(0);
    if (fabs(c1) < Tol<T>::Z) c1 = T(0);
    if (fabs(c2) < Tol<T>::Z) c2 = T(0);
    if (!(c0 > Tol<T>::POS || c1 > Tol<T>::POS || c2 > Tol<T>::POS)) {
        c0 = (V1.x - V0.x) * (P.z - V0.z) - (V1.z - V0.z) * (P.x - V0.x);
        c1 = (V2.x - V1.x) * (P.z - V1.z) - (V2.z - V1.z) * (P.x - V1.x);
        c2 = (V0.x - V2.x) * (P.z - V2.z) - (V0.z - V2.z) * (P.x - V2.x);
    }
    return !(c0 * c0 < T(0) || c0 * c1 < T(0) || c0 * c2 < T(0));
}

// candidate normal UTZVEC((a-b)x(b-c)) of the tetra faces idFc = [1,3,4],[1,2,4],[1,2,3],[2,3,4]
template <typename T> DEV V3<T> face_nml(V3<T> a, V3<T> b, V3<T> cc) { return utzvec(cross(vsub(a, b), vsub(b, cc))); }

// Lane-parallel tetrahedron faces: quad lane q = gl & 3 owns face q of idFc ([1,3,4], [1,2,4],
// [1,2,3], [2,3,4]) with vertices (a, b, c) in idFc order.  Its raw normal UTZVEC((a-b)x(b-c)) is
// computed once per simplex and serves both isPointInSimplex and the next update_simplex_GJK.
template <typename T> DEV void quad_face(int q, V3<T> s0, V3<T> s1, V3<T> s2, V3<T> s3, V3<T>& a, V3<T>& b, V3<T>& cc) {
    a = vsel(q == 3, s1, s0);
    b = vsel(q == 0 || q == 3, s2, s1);
    cc = vsel(q == 2, s2, s3);
}
template <typename T> DEV V3<T> quad_normal(int q, V3<T> s0, V3<T> s1, V3<T> s2, V3<T> s3, T& md) {
    V3<T> a, b, cc;
    quad_face(q, s0, s1, s2, s3, a, b, cc);
    const V3<T> cr = cross(vsub(a, b), vsub(b, cc));
    md = norm2(cr);
    return md < Tol<T>::Z ? zero3<T>() : vdiv(cr, md);
}
// isPointInSimplex (:1217-1265) for P = origin from the quad's raw normals (same booleans as
// origin_in_simplex: any boundary hit, else all four distances positive)
template <typename T> DEV bool quad_inside(int q, V3<T> s0, V3<T> s1, V3<T> s2, V3<T> s3, V3<T> nq) {
    const V3<T> M = centroid4(s0, s1, s2, s3);
    const V3<T> ref = q == 0 ? s0 : q == 1 ? s1 : q == 2 ? s2 : s3;
    if (dot(nq, vsub(ref, M)) < T(0)) nq = vneg(nq);
    const T d = dot(vsub(ref, zero3<T>()), nq);
    bool bnd = false;
    if (fabs(d) < Tol<T>::PT) {
        V3<T> a, b, cc;
        quad_face(q, s0, s1, s2, s3, a, b, cc);
        bnd = inside_tri(a, b, cc, zero3<T>());
    }
    return quad_any(bnd) || quad_all(d > T(0));
}
// simplex coordinate j (point j/3, axis j%3) for the cycle history lanes
template <typename T> DEV T simplex_coord(int j, V3<T> s0, V3<T> s1, V3<T> s2, V3<T> s3) {
    const int pt = j / 3, ax = j - 3 * (j / 3);
    const V3<T> q = pt == 0 ? s0 : pt == 1 ? s1 : pt == 2 ? s2 : s3;
    return ax == 0 ? q.x : ax == 1 ? q.y : q.z;
}

// isPointInSimplex (:1217-1265) for P = origin
template <typename T> DEV bool origin_in_simplex(V3<T> s0, V3<T> s1, V3<T> s2, V3<T> s3) {
    const V3<T> M = centroid4(s0, s1, s2, s3), O = zero3<T>();
    V3<T> n0 = face_nml(s0, s2, s3), n1 = face_nml(s0, s1, s3), n2 = face_nml(s0, s1, s2), n3 = face_nml(s1, s2, s3);
    if (dot(n0, vsub(s0, M)) < T(0)) n0 = vneg(n0);
    if (dot(n1, vsub(s1, M)) < T(0)) n1 = vneg(n1);
    if (dot(n2, vsub(s2, M)) < T(0)) n2 = vneg(n2);
    if (dot(n3, vsub(s3, M)) < T(0)) n3 = vneg(n3);
    const T d0 = dot(vsub(s0, O), n0), d1 = dot(vsub(s1, O), n1), d2 = dot(vsub(s2, O), n2), d3 = dot(vsub(s3, O), n3);
    if (fabs(d0) < Tol<T>::PT && inside_tri(s0, s2, s3, O)) return true;
    if (fabs(d1) < Tol<T>::PT && inside_tri(s0, s1, s3, O)) return true;
    if (fabs(d2) < Tol<T>::PT && inside_tri(s0, s1, s2, O)) return true;
    if (fabs(d3) < Tol<T>::PT && inside_tri(s1, s2, s3, O)) return true;
    return d0 > T(0) && d1 > T(0) && d2 > T(0) && d3 > T(0);
}
// ---------------------------------------------------------------- EPA polytope (re-supplied hull)
// Faces live in registers: face slot f = r*G + lane is row r of group lane f % G (R = FC/G rows).
// A face holds its unit normal UNINML (stored order, outward), |DIST_PF_SIGN(O, face)|, its
// vertex ids and a creation key; vertex coordinates are read from the LDS vertex list.  The reference's face list order
// (survivors in order, then new faces by (visible face, edge)) is the order of creation, so the
// key stands in for the list position: MINLOC's "first index" is the lowest key, and faces never
// move.  New faces take the lowest free slots; holes are reused.
constexpr uint32_t kEmpty = 0x80000000u;

template <typename T, int R> struct Faces {
    T nx[R], ny[R], nz[R];     // unit normal
    T d[R];                    // DIST_PF_SIGN(O, face) (signed: the EPA distance is |d|, the plane offset -d)
    uint32_t fv[R];            // v0 | v1 << 8 | v2 << 16, kEmpty = free slot
    uint32_t key[R];           // creation order
};
#define FACES_T Faces<T, (FC + G - 1) / G>

// A free slot: kEmpty, and with GJKEPA_EMPTY_INF a distance of -inf, so that |d| = +inf never wins MINLOC
// and dot(p, n) + d never passes the visibility test: the MINLOC scan needs no validity mask
template <typename T, int R> DEV void free_slot(Faces<T, R>& F, int r) {
    F.fv[r] = kEmpty;
    if constexpr (GJKEPA_EMPTY_INF) F.d[r] = -__builtin_inf();
}

template <typename T> DEV T qnan() { return __builtin_nan(""); }

// Add point p (vertex id k; appended at nv when `append`): faces it sees (signed distance >
// HULL) are removed and the horizon is coned to k.  `changed` reports whether the hull changed;
// with `save_eq` the current distances are saved to dsv[] when the face count will not change
// (the only case the termination test reads them).
CTX_T DEV int hull_add(CTX& c, FACES_T& F, uint32_t& kbase, int& hw, int& nv, int& nf, V3<T> p, bool append,
                       int kexist, bool& changed, bool save_eq) {
    constexpr int R = (FC + G - 1) / G;
    using L_t = typename CTX::L_t;
    auto& E = c.L.u.e;
    const int gl = c.g.gl;
    uint64_t vm[R];
    bool live[R];            // some face of this row is valid somewhere in the wave
    int nvis = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const bool valid = !(F.fv[r] & kEmpty);
        bool vis = false;
        live[r] = __ballot(valid) != 0;
        if (live[r]) {
            // signed distance of p above the face plane: n.p - n.v0 = dot(p, n) + DIST_PF_SIGN(O, face)
            vis = valid && dot(p, vmk<T>(F.nx[r], F.ny[r], F.nz[r])) + F.d[r] > Tol<T>::HULL;
        }
        vm[r] = c.g.ballot(vis);
        nvis += popc(vm[r]);
    }
    nvis = c.g.uni(nvis);
    changed = nvis > 0;
    GK_STAMP(SE_VIS);
    if (nvis == 0) return 0;
    int k = kexist;
    if (append) {
        if (nv >= VC) return ST_DEFER;
        k = nv;
        if (gl == 0) { E.vx[k] = p.x; E.vy[k] = p.y; E.vz[k] = p.z; }
        nv = nv + 1;
    }
    int vp[R];               // position of this slot's face in the visible list, -1 if not visible
    {   // visible faces (ids, key) in slot order
        int base = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            vp[r] = -1;
            if (!live[r]) continue;
            if (c.g.bit(vm[r])) {
                vp[r] = base + mbcnt(vm[r]);
                // GJKEPA_HORIZON_W16: v0 repeated in byte 3, so the face's three directed edges are
                // the 16-bit windows at bytes 0, 1 and 2 (v0v1, v1v2, v2v0)
                const uint32_t fw = GJKEPA_HORIZON_W16 ? F.fv[r] | ((F.fv[r] & 0xffu) << 24) : F.fv[r];
                E.x.h.visl[vp[r]] = (uint64_t)fw | ((uint64_t)F.key[r] << 32);
            }
            base += popc(vm[r]);
        }
    }
    __builtin_amdgcn_wave_barrier();
    GK_STAMP(SE_VIS);
    // horizon edges: edge s = (v_s, v_s+1) of a visible face whose twin (w,u) is on no visible
    // face.  Its new face's key follows the reference order: (rank of the face among the visible
    // ones by key, s).
    int nh = 0;
    const int ne = 3 * nvis;
    for (int e0 = 0; e0 < ne; e0 += G) {
        const int e = e0 + gl;
        bool hz = false;
        uint32_t uw = 0, nkey = 0;
        if (e < ne) {
            const int fi = e / 3, s = e - 3 * fi;
            const uint64_t me = E.x.h.visl[fi];
            const uint32_t fv = (uint32_t)me, kk = (uint32_t)(me >> 32);
            const uint32_t u = (fv >> (8 * s)) & 0xffu;
            const uint32_t w = (fv >> (8 * (s == 2 ? 0 : s + 1))) & 0xffu;
            bool twin = false;
            int rank = 0;
            if constexpr (GJKEPA_HORIZON_W16) {
                // the twin (w, u) is a directed edge of face j iff it is one of its three 16-bit windows
                const uint32_t t = w | (u << 8);
                for (int j = 0; j < nvis; ++j) {
                    const uint64_t qj = E.x.h.visl[j];
                    const uint32_t q = (uint32_t)qj;
                    twin = twin || (q & 0xffffu) == t || ((q >> 8) & 0xffffu) == t || (q >> 16) == t;
                    rank += (uint32_t)(qj >> 32) < kk;
                }
            } else {
                for (int j = 0; j < nvis; ++j) {
                    const uint64_t qj = E.x.h.visl[j];
                    const uint32_t q = (uint32_t)qj;
                    const uint32_t q0 = q & 0xffu, q1 = (q >> 8) & 0xffu, q2 = (q >> 16) & 0xffu;
                    twin = twin || (q0 == w && q1 == u) || (q1 == w && q2 == u) || (q2 == w && q0 == u);
                    rank += (uint32_t)(qj >> 32) < kk;
                }
            }
            hz = !twin;
            uw = u | (w << L_t::HVB);
            nkey = kbase + 3u * (uint32_t)rank + (uint32_t)s;
        }
        const uint64_t m = c.g.ballot(hz);
        if (hz) {
            const int pos = nh + mbcnt(m);
            if (pos < L_t::HC) {
                if constexpr (L_t::HPACK) E.x.h.horu[pos] = uw | (nkey << (2 * L_t::HVB));
                else { E.x.h.horu[pos] = uw; E.x.h.hork[pos] = nkey; }
            }
        }
        nh += popc(m);
    }
    nh = c.g.uni(nh);
    GK_STAMP(SE_HOR);
    const int nf2 = nf - nvis + nh;
    if (nh > L_t::HC || nf2 > FC) return ST_DEFER;
    kbase += 3u * (uint32_t)nvis;
    if (save_eq && nf2 == nf) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int f = r * G + gl;
            if (f < FC) E.dsv[f] = (F.fv[r] & kEmpty) ? qnan<T>() : fabs(F.d[r]);
        }
    }
    __builtin_amdgcn_wave_barrier();
    GK_STAMP(SE_CMP);
#if GJKEPA_EPA_PLACE
    // New faces (horizon edge h coned to k) are built on the lane whose slot receives them, straight
    // into its face registers.  Placement does not change results (the keys carry the order).  The
    // visible faces' slots are freed first; each round, the group lanes that still have a free slot
    // (lowest free row) take the next new faces in lane order, one per lane.  nf2 <= FC guarantees
    // enough free slots in total, so the rounds end; usually one round places every new face.
    const V3<T> P = c.vert(k);
    bool bad = false;
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (vp[r] >= 0) free_slot(F, r);
    int top = 0;
    for (int placed = 0; placed < nh;) {
        int row = -1;
#pragma unroll
        for (int r = R - 1; r >= 0; --r)
            if ((F.fv[r] & kEmpty) && r * G + gl < FC) row = r;
        const uint64_t fl = c.g.ballot(row >= 0);
        const int h = placed + mbcnt(fl);
        if (row >= 0 && h < nh) {
            const uint32_t uw = E.x.h.horu[h];
            constexpr uint32_t vm_ = (1u << L_t::HVB) - 1u;
            const int u = (int)(uw & vm_), w = (int)((uw >> L_t::HVB) & vm_);
            const V3<T> U = c.vert(u), W = c.vert(w);
            const V3<T> n = uninml(U, W, P);
            bad = bad || is_zero_nml(n);
            const T dd = dot(vsub(zero3<T>(), U), n);
            const uint32_t fv = (uint32_t)u | ((uint32_t)w << 8) | ((uint32_t)k << 16);
            const uint32_t kk = L_t::HPACK ? uw >> (2 * L_t::HVB) : E.x.h.hork[h];
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (r == row) { F.nx[r] = n.x; F.ny[r] = n.y; F.nz[r] = n.z; F.d[r] = dd; F.fv[r] = fv; F.key[r] = kk; }
            const int sl = row * G + gl + 1;
            top = top > sl ? top : sl;
        }
        placed += c.g.uni(popc(fl));
    }
    top = gmax<G>(top);
    hw = hw > top ? hw : top;
#else
    // New faces (horizon edge h coned to k) are built G at a time on group lane h % G and staged
    // in LDS, then copied into their slots.  Placement (results do not depend on it: the keys
    // carry the order): new face h takes the slot of visible face h, the ones beyond nvis are
    // appended at the high-water mark hw; a visible slot left over becomes a hole.  When the
    // append would pass FC, the new faces take the first nh free slots (holes included).
    const V3<T> P = c.vert(k);
    bool bad = false;
    int tj[R];               // index of the new face this slot receives, -1 if none
    const int app = nh - nvis;
    if (hw + (app > 0 ? app : 0) <= FC) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int slot = r * G + gl;
            int h = vp[r];
            if (h < 0 && slot >= hw && slot < hw + app) h = nvis + slot - hw;
            tj[r] = h < nh ? h : -1;
            if (vp[r] >= 0) free_slot(F, r);
        }
        if (app > 0) hw += app;
    } else {
        int fbase = 0, top = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const bool vis = vp[r] >= 0;
            const bool fre = ((F.fv[r] & kEmpty) || vis) && (r * G + gl < FC);
            const uint64_t fm = c.g.ballot(fre);
            const int fr = fbase + mbcnt(fm);
            fbase += popc(fm);
            tj[r] = fre && fr < nh ? fr : -1;
            if (tj[r] >= 0) top = r * G + gl + 1;
            if (vis) free_slot(F, r);
        }
        top = gmax<G>(top);
        hw = hw > top ? hw : top;
    }
    for (int h0 = 0; h0 < nh; h0 += G) {
        const int h = h0 + gl;
        if (h < nh) {
            const uint32_t uw = E.x.h.horu[h];
            constexpr uint32_t vm_ = (1u << L_t::HVB) - 1u;
            const int u = (int)(uw & vm_), w = (int)((uw >> L_t::HVB) & vm_);
            const V3<T> U = c.vert(u), W = c.vert(w);
            const V3<T> n = uninml(U, W, P);
            bad = bad || is_zero_nml(n);
            E.x.h.sn[gl][0] = n.x; E.x.h.sn[gl][1] = n.y; E.x.h.sn[gl][2] = n.z;
            E.x.h.sn[gl][3] = dot(vsub(zero3<T>(), U), n);
            E.x.h.sv[gl] = (uint32_t)u | ((uint32_t)w << 8) | ((uint32_t)k << 16);
            E.x.h.sk[gl] = L_t::HPACK ? uw >> (2 * L_t::HVB) : E.x.h.hork[h];
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int j = tj[r] - h0;
            const bool tgt = j >= 0 && j < G;
            if (__ballot(tgt)) {
                if (tgt) {
                    F.nx[r] = E.x.h.sn[j][0]; F.ny[r] = E.x.h.sn[j][1]; F.nz[r] = E.x.h.sn[j][2];
                    F.d[r] = E.x.h.sn[j][3];
                    F.fv[r] = E.x.h.sv[j];
                    F.key[r] = E.x.h.sk[j];
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
#endif
    GK_STAMP(SE_CONE);
    nf = nf2;
    if (c.g.any(bad)) return GJKEPA_STATUS_DEGENERATE;
    return 0;
}

// Hull of <= 6 points from scratch (EPA iteration 1): the points are vertex ids 0..m-1 of the
// polytope.  First non-degenerate tetrahedron in list order, faces in the seed pattern of
// :279-293 wound outward (slots / keys 0..3), then the remaining points in order.
CTX_T DEV int hull_build(CTX& c, FACES_T& F, uint32_t& kbase, int& hw, int& nv, int& nf, int m) {
    constexpr int R = (FC + G - 1) / G;
    nv = m;
    nf = 0;
    const V3<T> P0 = c.vert(0);
    int i1 = -1, i2 = -1, i3 = -1;
    for (int j = 1; j < m; ++j) if (c.g.unib(norm2(vsub(c.vert(j), P0)) > Tol<T>::HULL)) { i1 = j; break; }
    if (i1 < 0) return GJKEPA_STATUS_DEGENERATE;
    const V3<T> P1 = c.vert(i1);
    const V3<T> e1 = vsub(P1, P0);
    const T l1 = norm2(e1);
    for (int j = i1 + 1; j < m; ++j)
        if (c.g.unib(norm2(cross(e1, vsub(c.vert(j), P0))) / l1 > Tol<T>::HULL)) { i2 = j; break; }
    if (i2 < 0) return GJKEPA_STATUS_DEGENERATE;
    const V3<T> P2 = c.vert(i2);
    const V3<T> pn = utzvec(cross(e1, vsub(P2, P0)));
    for (int j = i2 + 1; j < m; ++j)
        if (c.g.unib(fabs(dot(vsub(c.vert(j), P0), pn)) > Tol<T>::HULL)) { i3 = j; break; }
    if (i3 < 0) return GJKEPA_STATUS_DEGENERATE;
    const V3<T> P3 = c.vert(i3);
    const V3<T> cen = centroid4(P0, P1, P2, P3);
    // seed faces over tetra slots (0,1,2),(0,2,3),(0,1,3),(1,2,3); group lane f owns face f
    const int gl = c.g.gl;
    bool bad = false;
#pragma unroll
    for (int r = 0; r < R; ++r) free_slot(F, r);
    if (gl < 4) {
        int a = gl == 3 ? i1 : 0, b = (gl == 0 || gl == 2) ? i1 : i2, d = gl == 0 ? i2 : i3;
        V3<T> Pa = vsel(gl == 3, P1, P0);
        V3<T> Pb = vsel(gl == 0 || gl == 2, P1, P2);
        V3<T> Pd = vsel(gl == 0, P2, P3);
        const V3<T> n0 = cross(vsub(Pb, Pa), vsub(Pd, Pb));
        if (dot(n0, vsub(Pa, cen)) < T(0)) { int s = b; b = d; d = s; V3<T> q = Pb; Pb = Pd; Pd = q; }
        const V3<T> n = uninml(Pa, Pb, Pd);
        bad = is_zero_nml(n);
        F.nx[0] = n.x; F.ny[0] = n.y; F.nz[0] = n.z;
        F.d[0] = dot(vsub(zero3<T>(), Pa), n);
        F.fv[0] = (uint32_t)a | ((uint32_t)b << 8) | ((uint32_t)d << 16);
        F.key[0] = (uint32_t)gl;
    }
    if (c.g.any(bad)) return GJKEPA_STATUS_DEGENERATE;
    nf = 4;
    kbase = 4;
    hw = 4;
    for (int j = 1; j < m; ++j) {
        if (j == i1 || j == i2 || j == i3) continue;
        bool ch;
        int st = hull_add(c, F, kbase, hw, nv, nf, c.vert(j), false, j, ch, false);
        if (st) return st;
    }
    return 0;
}

// MINLOC of the face distances (first in list order = lowest key): value-only group min, then
// the key breaks a tie between lanes.  The winner's normal, first vertex and distance are
// broadcast through the group's LDS slot.
CTX_T DEV void face_argmin(CTX& c, const FACES_T& F, T& dmin, V3<T>& n, bool& neg, int& av) {
    constexpr int R = (FC + G - 1) / G;
    auto& E = c.L.u.e;
    T v = Tol<T>::BIG;
    uint32_t kk = 0xFFFFFFFFu;
    int rr = -1;
    T vmin;
    if constexpr (GJKEPA_EMPTY_INF) {
        // free slots hold |d| = +inf: the value-only minimum over every row, then this lane's lowest key
        // among its rows at the group minimum
#pragma unroll
        for (int r = 0; r < R; ++r) v = red_min(fabs(F.d[r]), v);
        vmin = gmin<G>(v);
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (fabs(F.d[r]) == vmin && F.key[r] < kk) { kk = F.key[r]; rr = r; }
        v = vmin;
    } else {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const bool valid = !(F.fv[r] & kEmpty);
            if (!__ballot(valid)) continue;
            const T ad = fabs(F.d[r]);
            if (valid && (ad < v || (ad == v && F.key[r] < kk))) { v = ad; kk = F.key[r]; rr = r; }
        }
        vmin = gmin<G>(v);
    }
    const bool tie = rr >= 0 && v == vmin;
    uint64_t m = c.g.ballot(tie);
    if (c.g.unib(popc(m) > 1)) {
        const uint32_t kmin = (uint32_t)gmin<G>((int)(tie ? kk : 0x7FFFFFFFu));
        m = c.g.ballot(tie && kk == kmin);
    }
    if (c.g.bit(m)) {
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (rr == r) {
                E.best[0] = F.nx[r]; E.best[1] = F.ny[r]; E.best[2] = F.nz[r];
                // fp32: all three vertex ids (the certificate's normal bound reads them); fp64: the first
                E.bestv = (F.fv[r] & (certify<T>() ? 0xffffffu : 0xffu)) | (F.d[r] < T(0) ? 0x80000000u : 0u);
            }
    }
    __builtin_amdgcn_wave_barrier();
    dmin = vmin;
    n = vmk<T>(E.best[0], E.best[1], E.best[2]);
    const uint32_t bv = E.bestv;
    neg = (bv >> 31) != 0;
    av = (int)(bv & 0xffu);
    __builtin_amdgcn_wave_barrier();
}

// ALL(|sort(d1) - sort(d2)| < 1e-8), d1 = dsv[] (saved, NaN = no face), d2 = the current faces
// (:972-1004).  Both lists hold n values.  Slots at or above the high-water mark hw are empty now
// and were when dsv[] was saved (hw never decreases), so the rank loops stop at hw.
CTX_T DEV bool sorted_equal(CTX& c, const FACES_T& F, int hw) {
    constexpr int R = (FC + G - 1) / G;
    auto& E = c.L.u.e;
    const int gl = c.g.gl;
    // the saved list, sorted (rank among the saved values, ties by slot) into srt[]
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int i = r * G + gl;
        if (i < FC) {
            const T x = E.dsv[i];
            if (x == x) {
                int rk = 0;
                for (int j = 0; j < hw; ++j) { const T y = E.dsv[j]; rk += (y < x) || (y == x && j < i); }
                E.x.s.srt[rk] = x;
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    // dsv[] is read again only after the next save (hull_add / epa_grow save it in every iteration
    // whose termination test compares it), so the current values are ranked in its place
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int f = r * G + gl;
        if (f < FC) E.dsv[f] = (F.fv[r] & kEmpty) ? qnan<T>() : fabs(F.d[r]);
    }
    __builtin_amdgcn_wave_barrier();
    bool ok = true;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int i = r * G + gl;
        if (i < FC && !(F.fv[r] & kEmpty)) {
            const T x = fabs(F.d[r]);
            int rk = 0;
            for (int j = 0; j < hw; ++j) { const T y = E.dsv[j]; rk += (y < x) || (y == x && j < i); }
            if (!(fabs(x - E.x.s.srt[rk]) < Tol<T>::PT)) ok = false;
        }
    }
    __builtin_amdgcn_wave_barrier();
    return c.g.all(ok);
}

// SUM(polytope) / (3 F) over the face list in order (:905-908): faces sorted by key, then the
// sequential sum over vertex slot j = 0..2 and face f (column-major polytope(F,3,3)).  Slots at or
// above the high-water mark hw are empty.
CTX_T DEV V3<T> polytope_centroid(CTX& c, const FACES_T& F, int nf, int hw) {
    constexpr int R = (FC + G - 1) / G;
    auto& E = c.L.u.e;
    const int gl = c.g.gl;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int f = r * G + gl;
        if (f < FC) E.x.o.key[f] = (F.fv[r] & kEmpty) ? 0xFFFFFFFFu : F.key[r];
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int f = r * G + gl;
        if (f < FC && !(F.fv[r] & kEmpty)) {
            int rk = 0;
            for (int j = 0; j < hw; ++j) rk += E.x.o.key[j] < F.key[r];
            E.x.o.ord[rk] = F.fv[r];
        }
    }
    __builtin_amdgcn_wave_barrier();
    T sx = 0, sy = 0, sz = 0;
    for (int j = 0; j < 3; ++j)
        for (int f = 0; f < nf; ++f) {
            const V3<T> q = c.vert((int)((E.x.o.ord[f] >> (8 * j)) & 0xffu));
            sx += q.x; sy += q.y; sz += q.z;
        }
    __builtin_amdgcn_wave_barrier();
    const T cnt = (T)(nf * 3);
    return vmk<T>(sx / cnt, sy / cnt, sz / cnt);
}

// EPA_solu loop (:274-323) + update_expandingPolytope_EPA (:863-1022) as a resumable state
// machine: epa_begin runs iteration 1 (seed soup and hull from scratch), epa_step closes the
// current iteration (MINLOC of the new polytope, termination rules) and, unless it stopped, runs
// the next one.  A group can therefore be refilled with a new pair between any two iterations.
constexpr int ST_CONT = 101;     // internal: EPA continues

template <typename T, int R> struct EpaState {
    Faces<T, R> F;
    int nv, hw, nf, F1, iters;
    uint32_t kbase;
    T minv;
    V3<T> dir;                     // MINLOC face of the current polytope: normal,
    bool neg;                      //   DIST_PF_SIGN(O, face) < 0,
    int av;                        //   first vertex id
    bool unchanged;
    T hsup;                        // fp32 certificate: support value along dir of the last support step
};
#define EPAST_T EpaState<T, (FC + G - 1) / G>

CTX_T DEV int epa_begin(CTX& c, EPAST_T& S, V3<T> s0, V3<T> s1, V3<T> s2, V3<T> s3) {
    constexpr int R = (FC + G - 1) / G;
    auto& E = c.L.u.e;
    const V3<T> O = zero3<T>();
    const int gl = c.g.gl;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        free_slot(S.F, r);
        const int f = r * G + gl;
        if (f < FC) E.dsv[f] = qnan<T>();
    }
    S.nv = 0; S.hw = 0; S.nf = 0; S.kbase = 0; S.iters = 1; S.F1 = 4; S.unchanged = false;
    // seed soup [1,2,3],[1,3,4],[1,2,4],[2,3,4] (:279-293), distances via DIST_PF_SIGN: quad lane q
    // builds face q (its first vertex is the distance reference), the quad shares the results
    const int fq = gl & 3;
    const V3<T> fa = fq == 3 ? s1 : s0, fb = (fq == 0 || fq == 2) ? s1 : s2, fc = fq == 0 ? s2 : s3;
    const V3<T> nq = uninml(fa, fb, fc);
    if (c.g.unib(quad_any(is_zero_nml(nq)))) return GJKEPA_STATUS_DEGENERATE;
    const T dq = fabs(dot(vsub(O, fa), nq));
    const T d0 = qbcast<0>(dq), d1 = qbcast<1>(dq), d2 = qbcast<2>(dq), d3 = qbcast<3>(dq);
    T minv = d0;                                              // MINLOC, first index
    int kmin = 0;
    if (d1 < minv) { minv = d1; kmin = 1; }
    if (d2 < minv) { minv = d2; kmin = 2; }
    if (d3 < minv) { minv = d3; kmin = 3; }
    V3<T> dir = quad_pick(fq == kmin, nq);
    const V3<T> a1 = kmin == 3 ? s1 : s0;
    if (gl < 4) E.dsv[gl] = dq;
    T dt = dot(vsub(a1, O), dir);
    if (c.g.unib(fabs(dt) < Tol<T>::ZO)) {                    // :905-908 polytope centroid
        // SUM over polytope(:,:,k), slot-major over faces: [s0 s0 s0 s1][s1 s2 s1 s2][s2 s3 s3 s3]
        const T sx = ((((((((((s0.x + s0.x) + s0.x) + s1.x) + s1.x) + s2.x) + s1.x) + s2.x) + s2.x) + s3.x) + s3.x) + s3.x;
        const T sy = ((((((((((s0.y + s0.y) + s0.y) + s1.y) + s1.y) + s2.y) + s1.y) + s2.y) + s2.y) + s3.y) + s3.y) + s3.y;
        const T sz = ((((((((((s0.z + s0.z) + s0.z) + s1.z) + s1.z) + s2.z) + s1.z) + s2.z) + s2.z) + s3.z) + s3.z) + s3.z;
        const T cnt = (T)12;
        dt = dot(vsub(a1, vmk<T>(sx / cnt, sy / cnt, sz / cnt)), dir);
    }
    if (c.g.unib(dt <= -Tol<T>::ZO)) dir = vneg(dir);         // :910
    GK_STAMP(SE_IT1);
    const V3<T> sp = support(c, dir);                          // :914
    if constexpr (certify<T>()) { S.minv = minv; S.hsup = dot(sp, dir); }
    const bool two = c.g.unib(fabs(minv) < Tol<T>::ZO);        // :935
    // unique polytope vertices (getHullMeshesVertex, :920) + new point(s) -> ids 0..m-1
    const bool u1 = !veq(s1, s0);
    const bool u2 = !veq(s2, s0) && !veq(s2, s1);
    const bool u3 = !veq(s3, s0) && !veq(s3, s1) && !veq(s3, s2);
    const int i1 = 1, i2 = u1 ? 2 : 1, i3 = i2 + (u2 ? 1 : 0), isp = i3 + (u3 ? 1 : 0);
    int m = isp + 1;
    V3<T> sq = zero3<T>();
    if (two) { sq = support(c, vneg(dir)); ++m; }
    V3<T> q = s0;                                  // group lane j writes point j
    bool w = gl == 0;
    if (u1 && gl == i1) { q = s1; w = true; }
    if (u2 && gl == i2) { q = s2; w = true; }
    if (u3 && gl == i3) { q = s3; w = true; }
    if (gl == isp) { q = sp; w = true; }
    if (two && gl == isp + 1) { q = sq; w = true; }
    if (w) { E.vx[gl] = q.x; E.vy[gl] = q.y; E.vz[gl] = q.z; }
    __builtin_amdgcn_wave_barrier();
    GK_STAMP(SE_IT1);
    return hull_build(c, S.F, S.kbase, S.hw, S.nv, S.nf, m);
}

// EPA iteration 1 up to the support step, for the usual case where hull_build's first tetrahedron is
// the GJK simplex itself (four distinct points, non-degenerate at the hull epsilon): the seed soup's
// MINLOC and orientation as in epa_begin (direction in S.dir), the tetrahedron's faces wound outward
// as hull_build does (slots / keys 0..3) and its points as vertices 0..3.  epa_grow(first = true) then
// adds the support point(s) as hull_build adds them, in the same pass as the other groups' steps.
// ST_FALLBACK: the tetrahedron is not the simplex (duplicate or near-degenerate points): epa_begin.
constexpr int ST_FALLBACK = 102;
CTX_T DEV int epa_seed(CTX& c, EPAST_T& S, V3<T> s0, V3<T> s1, V3<T> s2, V3<T> s3) {
    constexpr int R = (FC + G - 1) / G;
    auto& E = c.L.u.e;
    const V3<T> O = zero3<T>();
    const int gl = c.g.gl;
    // hull_build's tetrahedron search (first non-degenerate one in list order) must give (0, 1, 2, 3)
    const bool distinct = !veq(s1, s0) && !veq(s2, s0) && !veq(s2, s1) && !veq(s3, s0) && !veq(s3, s1) && !veq(s3, s2);
    if (!c.g.unib(distinct)) return ST_FALLBACK;
    const V3<T> e1 = vsub(s1, s0);
    const T l1 = norm2(e1);
    if (!c.g.unib(l1 > Tol<T>::HULL)) return ST_FALLBACK;
    const V3<T> c2 = cross(e1, vsub(s2, s0));
    if (!c.g.unib(norm2(c2) / l1 > Tol<T>::HULL)) return ST_FALLBACK;
    const V3<T> pn = utzvec(c2);
    if (!c.g.unib(fabs(dot(vsub(s3, s0), pn)) > Tol<T>::HULL)) return ST_FALLBACK;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        free_slot(S.F, r);
        const int f = r * G + gl;
        if (f < FC) E.dsv[f] = qnan<T>();
    }
    S.iters = 1; S.F1 = 4; S.unchanged = false;
    // seed soup [1,2,3],[1,3,4],[1,2,4],[2,3,4] (:279-293) on the quad lanes, as in epa_begin
    const int fq = gl & 3;
    const V3<T> fa = fq == 3 ? s1 : s0, fb = (fq == 0 || fq == 2) ? s1 : s2, fc = fq == 0 ? s2 : s3;
    const V3<T> nq = uninml(fa, fb, fc);
    if (c.g.unib(quad_any(is_zero_nml(nq)))) return GJKEPA_STATUS_DEGENERATE;
    const T dq = fabs(dot(vsub(O, fa), nq));
    const T d0 = qbcast<0>(dq), d1 = qbcast<1>(dq), d2 = qbcast<2>(dq), d3 = qbcast<3>(dq);
    T minv = d0;                                              // MINLOC, first index
    int kmin = 0;
    if (d1 < minv) { minv = d1; kmin = 1; }
    if (d2 < minv) { minv = d2; kmin = 2; }
    if (d3 < minv) { minv = d3; kmin = 3; }
    V3<T> dir = quad_pick(fq == kmin, nq);
    const V3<T> a1 = kmin == 3 ? s1 : s0;
    if (gl < 4) E.dsv[gl] = dq;
    T dt = dot(vsub(a1, O), dir);
    if (c.g.unib(fabs(dt) < Tol<T>::ZO)) {                    // :905-908 polytope centroid
        const T sx = ((((((((((s0.x + s0.x) + s0.x) + s1.x) + s1.x) + s2.x) + s1.x) + s2.x) + s2.x) + s3.x) + s3.x) + s3.x;
        const T sy = ((((((((((s0.y + s0.y) + s0.y) + s1.y) + s1.y) + s2.y) + s1.y) + s2.y) + s2.y) + s3.y) + s3.y) + s3.y;
        const T sz = ((((((((((s0.z + s0.z) + s0.z) + s1.z) + s1.z) + s2.z) + s1.z) + s2.z) + s2.z) + s3.z) + s3.z) + s3.z;
        const T cnt = (T)12;
        dt = dot(vsub(a1, vmk<T>(sx / cnt, sy / cnt, sz / cnt)), dir);
    }
    if (c.g.unib(dt <= -Tol<T>::ZO)) dir = vneg(dir);         // :910
    S.dir = dir;                                              // epa_grow's support direction
    S.minv = minv;                                            // epa_grow's two-point test (:935)
    // vertices 0..3 and the tetrahedron's faces wound outward (hull_build with i1, i2, i3 = 1, 2, 3)
    if (gl < 4) {
        const V3<T> q = gl == 0 ? s0 : gl == 1 ? s1 : gl == 2 ? s2 : s3;
        E.vx[gl] = q.x; E.vy[gl] = q.y; E.vz[gl] = q.z;
    }
    const V3<T> cen = centroid4(s0, s1, s2, s3);
    bool bad = false;
    if (gl < 4) {
        int a = gl == 3 ? 1 : 0, b = (gl == 0 || gl == 2) ? 1 : 2, d = gl == 0 ? 2 : 3;
        const V3<T> Pa = vsel(gl == 3, s1, s0);
        V3<T> Pb = vsel(gl == 0 || gl == 2, s1, s2);
        V3<T> Pd = vsel(gl == 0, s2, s3);
        const V3<T> n0 = cross(vsub(Pb, Pa), vsub(Pd, Pb));
        if (dot(n0, vsub(Pa, cen)) < T(0)) { int t = b; b = d; d = t; const V3<T> q = Pb; Pb = Pd; Pd = q; }
        const V3<T> n = uninml(Pa, Pb, Pd);
        bad = is_zero_nml(n);
        S.F.nx[0] = n.x; S.F.ny[0] = n.y; S.F.nz[0] = n.z;
        S.F.d[0] = dot(vsub(zero3<T>(), Pa), n);
        S.F.fv[0] = (uint32_t)a | ((uint32_t)b << 8) | ((uint32_t)d << 16);
        S.F.key[0] = (uint32_t)gl;
    }
    __builtin_amdgcn_wave_barrier();
    if (c.g.any(bad)) return GJKEPA_STATUS_DEGENERATE;
    S.nv = 4; S.nf = 4; S.kbase = 4; S.hw = 4;
    GK_STAMP(SE_IT1);
    return 0;
}

// Closes iteration S.iters (MINLOC of the polytope, termination :956-1015); if EPA goes on, the
// next iteration's direction (:888-910) replaces S.dir.  ST_CONT, 0 (depth and normal set) or a status.
CTX_T DEV int epa_close(CTX& c, EPAST_T& S, T& depth, V3<T>& normal) {
    const int F2 = S.nf;                                      // :956-969
    const T prev = S.minv;
    face_argmin(c, S.F, S.minv, S.dir, S.neg, S.av);
    if constexpr (certify<T>()) {                             // fp32 certificate: MINLOC never drops
        if (c.g.unib(S.minv < prev - Tol<T>::CERT_DROP * prev)) return ST_REDO;
    }
    // dot(a1 - O, n) is -DIST_PF_SIGN(O, face) (exact negation; a zero's sign never matters here):
    // negative iff the face's signed distance is positive
    V3<T> dir2 = S.dir;
    if (c.g.unib(!S.neg && S.minv > T(0))) dir2 = vneg(dir2);
    bool stop;                                                // :972-1015
    if (S.F1 == F2) stop = S.unchanged || sorted_equal(c, S.F, S.hw);   // unchanged hull: identical sorted lists
    else stop = S.F1 > F2;
    GK_STAMP(SE_TERM);
    if constexpr (certify<T>()) {
        // fp32 certificate at termination: support gap plus its evaluation noise within CERT_GAP x d (a
        // touching pair, d below the noise, never passes); the origin strictly below every face (a hit
        // the polytope itself proves)
        if (stop) {
            constexpr int R = (FC + G - 1) / G;
            bool out = false;
#pragma unroll
            for (int r = 0; r < R; ++r) out = out || (!(S.F.fv[r] & kEmpty) && !(S.F.d[r] < T(0)));
            const float sc = c.vmax_a + c.vmax_b;
            // the final face's normal rounding bound (Tol<float>::CERT_ANGLE), from its vertices
            const uint32_t bw = c.L.u.e.bestv;
            const V3<T> U = c.vert((int)(bw & 0xffu)), W = c.vert((int)((bw >> 8) & 0xffu)), P = c.vert((int)((bw >> 16) & 0xffu));
            const V3<T> e1 = vsub(W, U), e2 = vsub(P, W);
            const T l1 = norm2(e1), l2 = norm2(e2), lc = norm2(cross(e1, e2));
            const T u = T(5.9604644775390625e-08), k = T(3.4641016151377544), three = T(3), two = T(2);
            const T th = ((((k * u) * sc) * (l1 + l2)) + (((three * u) * l1) * l2)) / lc + two * u;
            if (c.g.any(out) || c.g.unib(!(S.hsup - S.minv + Tol<T>::CERT_NOISE * sc <= Tol<T>::CERT_GAP * S.minv)) ||
                c.g.unib(!(th <= Tol<T>::CERT_ANGLE)))
                return ST_REDO;
        }
    }
    if (stop) { depth = S.minv; normal = dir2; return 0; }
    // ---- next iteration: same faces as this iteration's F2, so its MINLOC carries over
    S.iters = S.iters + 1;
    if (S.iters > 99) return GJKEPA_STATUS_EPA_MAXITER;
    S.F1 = S.nf;
    T dt = S.neg ? S.minv : -S.minv;                           // dot(a1 - O, dir)
    if (c.g.unib(S.minv < Tol<T>::ZO))                        // :905-908
        dt = dot(vsub(c.vert(S.av), polytope_centroid(c, S.F, S.F1, S.hw)), S.dir);
    if (c.g.unib(dt <= -Tol<T>::ZO)) S.dir = vneg(S.dir);     // :910
    GK_STAMP(SE_DIR);
    return ST_CONT;
}

// The rest of an iteration along dir = S.dir: support point(s) (:914, :935-944) and the hull of the polytope
// vertices and the new point(s) (:918-950).  `first`: iteration 1 after epa_seed, which adds the
// points to the simplex's tetrahedron exactly as hull_build does (no distance save, no unchanged
// short cut: iteration 1's termination test compares the seed soup's distances).
CTX_T DEV int epa_grow(CTX& c, EPAST_T& S, bool first) {
    constexpr int R = (FC + G - 1) / G;
    auto& E = c.L.u.e;
    const int gl = c.g.gl;
    const V3<T> dir = S.dir;
    const V3<T> sp = support(c, dir);                          // :914
    if constexpr (certify<T>()) S.hsup = dot(sp, dir);
    GK_STAMP(SE_SUP);
    const bool two = c.g.unib(fabs(S.minv) < Tol<T>::ZO);      // :935
    if (two && !first) {                  // net face count of two insertions unknown: save now
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int f = r * G + gl;
            if (f < FC) E.dsv[f] = (S.F.fv[r] & kEmpty) ? qnan<T>() : fabs(S.F.d[r]);
        }
    }
    bool ch1 = false, ch2 = false;
    int st = hull_add(c, S.F, S.kbase, S.hw, S.nv, S.nf, sp, true, 0, ch1, !two && !first);
    if (!st && two) st = hull_add(c, S.F, S.kbase, S.hw, S.nv, S.nf, support(c, vneg(dir)), true, 0, ch2, false);
    S.unchanged = !first && !ch1 && !ch2;
    return st ? st : ST_CONT;
}

// Closes iteration S.iters; if EPA goes on, runs the next iteration.  ST_CONT, 0 (depth and
// normal set) or an error status / ST_DEFER.
CTX_T DEV int epa_step(CTX& c, EPAST_T& S, T& depth, V3<T>& normal) {
    const int r = epa_close(c, S, depth, normal);
    if (r != ST_CONT) return r;
    return epa_grow(c, S, false);
}

// ---- polytope parking (gjkepa_kernel.h): park slot layout
//   u32 [0..15]   nv, hw, nf, F1, iters, kbase, neg, av, gjk_it
//   T   @64       dir.x, dir.y, dir.z, minv, hsup
//   T   @HDR      vx[PARK_VC], vy[PARK_VC], vz[PARK_VC]      (vertex coordinates by id)
//   u32 @HDR+3*8*PARK_VC   fv[PARK_FC], key[PARK_FC]        (face slots below hw; kEmpty = hole)
struct ParkCtl {
    unsigned char* base;     // park slots
    uint32_t* ctr;           // slots taken
    uint32_t cap;            // slots available
    uint32_t gjk_it;         // GJK iterations of the pair (kept in the parked state)
    uint32_t* slot;          // the pair's record slot: word 5 <- park slot + 1
};
constexpr int kParkFaces = GJKEPA_PARK_HDR + 3 * 8 * GJKEPA_PARK_VC;

// At the start of an iteration: park the polytope when the next iteration could outgrow this tier
// (two insertions add at most two vertices and four faces to a valid polytope), if a slot is free.
CTX_T DEV bool park_now(CTX& c, const EPAST_T& S, const ParkCtl& pk) {
    static_assert(VC <= GJKEPA_PARK_VC && FC <= GJKEPA_PARK_FC, "parked polytope larger than a park slot");
    constexpr int R = (FC + G - 1) / G;
    if (!c.g.unib(S.nv + 2 > VC || S.nf + 4 > FC)) return false;
    const int gl = c.g.gl;
    uint32_t idx = 0;
    if (gl == 0) idx = atomicAdd(pk.ctr, 1u);
    idx = (uint32_t)__shfl((int)idx, c.g.lane & ~(G - 1));
    if (c.g.unib(idx >= pk.cap)) return false;                 // slots used up: run on, restart later
    unsigned char* rec = pk.base + (size_t)idx * GJKEPA_PARK_BYTES;
    auto& E = c.L.u.e;
    uint32_t* hdr = reinterpret_cast<uint32_t*>(rec);
    T* tv = reinterpret_cast<T*>(rec + 64);
    T* vx = reinterpret_cast<T*>(rec + GJKEPA_PARK_HDR);
    uint32_t* fv = reinterpret_cast<uint32_t*>(rec + kParkFaces);
    if (gl < 9) {
        const uint32_t h[9] = {(uint32_t)S.nv, (uint32_t)S.hw, (uint32_t)S.nf, (uint32_t)S.F1, (uint32_t)S.iters, S.kbase,
                               (uint32_t)S.neg, (uint32_t)S.av, pk.gjk_it};
        uint32_t w = h[0];
#pragma unroll
        for (int j = 1; j < 9; ++j) w = gl == j ? h[j] : w;
        hdr[gl] = w;
    }
    if (gl < 5) {
        const T hs = certify<T>() ? S.hsup : T(0);
        tv[gl] = gl == 0 ? S.dir.x : gl == 1 ? S.dir.y : gl == 2 ? S.dir.z : gl == 3 ? S.minv : hs;
    }
    for (int i = gl; i < S.nv; i += G) {
        vx[i] = E.vx[i];
        vx[GJKEPA_PARK_VC + i] = E.vy[i];
        vx[2 * GJKEPA_PARK_VC + i] = E.vz[i];
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int f = r * G + gl;
        if (f < S.hw) { fv[f] = S.F.fv[r]; fv[GJKEPA_PARK_FC + f] = S.F.key[r]; }
    }
    if (gl == 0) pk.slot[5] = idx + 1;
    return true;
}

// Resume a parked polytope (the next tier's first step is epa_grow): vertices back into LDS, each
// face's plane recomputed from its vertex ids exactly as it was built (UNINML of the stored order,
// DIST_PF_SIGN from its first vertex), slot f in slot f (holes stay holes).
CTX_T DEV void epa_resume(CTX& c, EPAST_T& S, const unsigned char* rec, uint32_t& gjk_it) {
    constexpr int R = (FC + G - 1) / G;
    auto& E = c.L.u.e;
    const int gl = c.g.gl;
    const uint32_t* hdr = reinterpret_cast<const uint32_t*>(rec);
    const T* tv = reinterpret_cast<const T*>(rec + 64);
    const T* vx = reinterpret_cast<const T*>(rec + GJKEPA_PARK_HDR);
    const uint32_t* fv = reinterpret_cast<const uint32_t*>(rec + kParkFaces);
    S.nv = c.g.uni((int)hdr[0]); S.hw = c.g.uni((int)hdr[1]); S.nf = c.g.uni((int)hdr[2]); S.F1 = c.g.uni((int)hdr[3]);
    S.iters = c.g.uni((int)hdr[4]); S.kbase = hdr[5]; S.neg = hdr[6] != 0; S.av = (int)hdr[7]; gjk_it = hdr[8];
    S.dir = vmk<T>(tv[0], tv[1], tv[2]);
    S.minv = tv[3];
    S.hsup = tv[4];
    S.unchanged = false;
    for (int i = gl; i < S.nv; i += G) {
        E.vx[i] = vx[i];
        E.vy[i] = vx[GJKEPA_PARK_VC + i];
        E.vz[i] = vx[2 * GJKEPA_PARK_VC + i];
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int f = r * G + gl;
        free_slot(S.F, r);
        if (f < S.hw) {
            const uint32_t w = fv[f];
            if (!(w & kEmpty)) {
                const V3<T> U = c.vert((int)(w & 0xffu)), W = c.vert((int)((w >> 8) & 0xffu)), P = c.vert((int)((w >> 16) & 0xffu));
                const V3<T> n = uninml(U, W, P);
                S.F.nx[r] = n.x; S.F.ny[r] = n.y; S.F.nz[r] = n.z;
                S.F.d[r] = dot(vsub(zero3<T>(), U), n);
                S.F.fv[r] = w;
                S.F.key[r] = fv[GJKEPA_PARK_FC + f];
            }
        }
    }
}

// EPA from the simplex (or, with `rec`, from a parked polytope); with `park`, the polytope is parked
// through `pk` (ST_PARKED) when it could outgrow this tier and a park slot is free.  `pk` is passed by
// value with a flag, not as a maybe-null pointer: a pointer to the caller's copy selected against null
// keeps that copy in scratch memory (one 32-byte store per lane and pair).
CTX_T DEV int epa(CTX& c, V3<T> s0, V3<T> s1, V3<T> s2, V3<T> s3, T& depth, V3<T>& normal, int& iters, int& nf,
                  bool park = false, ParkCtl pk = {}, const unsigned char* rec = nullptr, uint32_t* gjk_it = nullptr) {
    EPAST_T S;
    int st;
    if (rec) {
        epa_resume(c, S, rec, *gjk_it);
        st = epa_grow(c, S, false);
    } else {
        st = epa_begin(c, S, s0, s1, s2, s3);     // iteration 1 up to its hull; it closes in the loop
        if (st == 0) st = ST_CONT;
    }
    while (st == ST_CONT) {
        st = epa_close(c, S, depth, normal);
        if (st != ST_CONT) break;
        if constexpr (VC <= GJKEPA_PARK_VC && FC <= GJKEPA_PARK_FC) {
            if (park && park_now(c, S, pk)) { st = ST_PARKED; break; }
        }
        st = epa_grow(c, S, false);
    }
    iters = S.iters;
    nf = S.nf;
    return st;
}

// ---------------------------------------------------------------- contact features
// sequential "> max - 1e-8" scans (:722-747, :438-444): the running max may decrease
CTX_T DEV void scan_top2(CTX& c, int side, V3<T> n, int& i0, int& i1) {
    T mx = -Tol<T>::BIG;
    i0 = -1; i1 = -1;
    const int cnt = side ? c.nb : c.na;
    for (int i = 0; i < cnt; ++i) {
        T t = dot(n, side ? c.B(i) : c.A(i));
        if (t > mx - Tol<T>::PT) { mx = t; i1 = i0; i0 = i; }
    }
    if (i1 == -1) i1 = i0;
}

// group-parallel max of dot(n, p_i) over one hull
CTX_T DEV T hull_dot_max(CTX& c, int side, V3<T> n) {
    T mx = -Tol<T>::BIG;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        int i = k * G + c.g.gl;
        const V3<T> p = side ? c.BV(k) : c.AV(k);
        T t = n.x * p.x + n.y * p.y + n.z * p.z;
        if (i < (side ? c.nb : c.na) && t > mx) mx = t;
    }
    return gmax<G>(mx);
}
// members with dot(n,p) > mx - band (index order) -> LDS sx/sy/sz when `store`; returns count
// element i of the contact point set: its hull vertex, converted as when it was selected
CTX_T DEV V3<T> set_pt(const CTX& c, int i) {
    const uint32_t w = c.L.u.c.si[i];
    const V3<TH> v = c.raw((int)(w >> 15), (int)(w & 0x7fffu));
    return vmk<T>((T)v.x, (T)v.y, (T)v.z);
}

CTX_T DEV int hull_band_set(CTX& c, int side, V3<T> n, T mx, T band, bool store) {
    int cnt = 0;
    auto& C = c.L.u.c;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        int i = k * G + c.g.gl;
        const V3<T> p = side ? c.BV(k) : c.AV(k);
        T px = p.x, py = p.y, pz = p.z;
        T t = n.x * px + n.y * py + n.z * pz;
        bool in = i < (side ? c.nb : c.na) && t > mx - band;
        uint64_t m = c.g.ballot(in);
        if (store && in) { int pos = cnt + mbcnt(m); C.si[pos] = (uint16_t)(i | (side << 15)); }
        cnt += popc(m);
    }
    __builtin_amdgcn_wave_barrier();
    return c.g.uni(cnt);
}

// hull_band_set on precomputed dots: members t > thr (index order) -> LDS sx/sy/sz when `store`
CTX_T DEV int band_set(CTX& c, int side, const DotSet<T, K>& D, T thr, bool store) {
    int cnt = 0;
    auto& C = c.L.u.c;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int i = k * G + c.g.gl;
        const bool in = i < (side ? c.nb : c.na) && D.t[side][k] > thr;
        const uint64_t m = c.g.ballot(in);
        if (store && in) {
            const int pos = cnt + mbcnt(m);
            C.si[pos] = (uint16_t)(i | (side << 15));
        }
        cnt += popc(m);
    }
    __builtin_amdgcn_wave_barrier();
    return c.g.uni(cnt);
}

// get_info_collisionType (:353-413)
CTX_T DEV int collision_type(CTX& c, V3<T> n, T tol) {
    const T m1 = hull_dot_max(c, 0, n);
    const int C = hull_band_set(c, 0, n, m1, tol, false);
    const V3<T> nn = vneg(n);
    const T m2 = hull_dot_max(c, 1, nn);
    const int D = hull_band_set(c, 1, nn, m2, tol, false);
    return (C >= 3 && D >= 3) ? 2 : 1;
}
// the same from the dots of n already taken (get_nearest_points' pass)
CTX_T DEV int collision_type(CTX& c, const DotSet<T, K>& D, T tol) {
    const int na = band_set(c, 0, D, D.m[0] - tol, false);
    const int nb = band_set(c, 1, D, D.m[1] - tol, false);
    return (na >= 3 && nb >= 3) ? 2 : 1;
}

// get_collisionPoint_01 (:700-806)
CTX_T DEV int contact_v1(CTX& c, V3<T> n, const DotSet<T, K>& D, V3<T>& res) {
    int a0, a1, b0, b1;
    scan_top2(c, 0, n, a0, a1);
    scan_top2(c, 1, vneg(n), b0, b1);
    if (a0 < 0 || b0 < 0) return GJKEPA_STATUS_DEGENERATE;
    res = zero3<T>();
    if (a0 == a1 && b0 == b1) res = vdiv(vadd(c.A(a0), c.B(b0)), T(2));
    if (a0 != a1 && b0 == b1) res = c.B(b0);
    else if (a0 == a1 && b0 != b1) res = c.A(a0);
    if (a0 != a1 && b0 != b1) {
        const int C = band_set(c, 0, D, D.m[0] - T(0.1), true);
        T sx = 0, sy = 0, sz = 0;
        for (int i = 0; i < C; ++i) { const V3<T> q = set_pt(c, i); sx += q.x; sy += q.y; sz += q.z; }
        const T dc = (T)C;
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

// case_04 (:575-669) on the set in sx/sy/sz[0..na) and the 2-point set (b0, b1):
// SORT_CLOCK (:1513-1575) with a group-parallel angle argmin per step, then IS_INSIDE_PF of the
// ordered polygon for b0 and b1 (group-parallel over edges).
CTX_T DEV int contact_case04(CTX& c, int na, V3<T> b0, V3<T> b1, V3<T>& res) {
    auto& C = c.L.u.c;
    const int gl = c.g.gl;
    const T TWO_PI_SP = (T)(2.0f * 3.14159274101257324f);
    // OVERLAP (:1399-1418): all points pairwise within 1e-12 -> order unchanged
    bool diff = false;
    for (int i0 = 0; i0 < na; i0 += G) {
        int i = i0 + gl;
        if (i < na) {
            const V3<T> pi = set_pt(c, i);
            for (int j = 0; j < na; ++j) {
                const V3<T> pj = set_pt(c, j);
                diff = diff || fabs(pi.x - pj.x) > Tol<T>::Z || fabs(pi.y - pj.y) > Tol<T>::Z || fabs(pi.z - pj.z) > Tol<T>::Z;
            }
        }
    }
    const bool ovl = !c.g.any(diff);
    T px[K], py[K], pz[K];
    bool used[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        int i = k * G + gl;
        const V3<T> q = set_pt(c, i < na ? i : 0);
        px[k] = q.x; py[k] = q.y; pz[k] = q.z;
        used[k] = false;
    }
    if (!ovl) {
        T sx = 0, sy = 0, sz = 0;
        for (int i = 0; i < na; ++i) { const V3<T> q = set_pt(c, i); sx += q.x; sy += q.y; sz += q.z; }
        const T dn = (T)na;
        const V3<T> cen = vmk<T>(sx / dn, sy / dn, sz / dn);
        const V3<T> p0 = set_pt(c, 0);
        const V3<T> nrm = cross(vsub(set_pt(c, 1), p0), vsub(set_pt(c, 2), p0));
        V3<T> prev = p0;
        if (gl == 0) C.ord[0] = 0u;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            int i = k * G + gl;
            used[k] = i < na && px[k] == p0.x && py[k] == p0.y && pz[k] == p0.z;
        }
        for (int s = 1; s < na; ++s) {
            T best = Tol<T>::BIG;
            int bi = 0x7fffffff;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                int j = k * G + gl;
                if (j < na && !used[k]) {
                    V3<T> w1 = vsub(vmk<T>(px[k], py[k], pz[k]), cen), w2 = vsub(prev, cen);
                    T ang = tatan2(dot(nrm, cross(w2, w1)), dot(w1, w2));
                    ang = tfmod(ang + TWO_PI_SP, TWO_PI_SP);
                    if (ang < best) { best = ang; bi = j; }
                }
            }
            gargmin<G>(best, bi);
            bi = c.g.uni(bi);
            if (bi == 0x7fffffff) return GJKEPA_STATUS_DEGENERATE;
            prev = set_pt(c, bi);
            if (gl == 0) C.ord[s] = (uint32_t)bi;
#pragma unroll
            for (int k = 0; k < K; ++k) used[k] = used[k] || (px[k] == prev.x && py[k] == prev.y && pz[k] == prev.z);
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int k = 0; k < K; ++k) {
            int q = k * G + gl;
            if (q < na) { const V3<T> p = set_pt(c, (int)C.ord[q]); px[k] = p.x; py[k] = p.y; pz[k] = p.z; }
        }
    }
    // next polygon vertex of each lane's element, through the pol[] exchange
    T nxv[K], nyv[K], nzv[K];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < K; ++k) { int q = k * G + gl; if (q < na) C.pol[q] = px[k]; }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < K; ++k) { int q = k * G + gl; int j = (q == na - 1) ? 0 : q + 1; nxv[k] = q < na ? C.pol[j] : T(0); }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < K; ++k) { int q = k * G + gl; if (q < na) C.pol[q] = py[k]; }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < K; ++k) { int q = k * G + gl; int j = (q == na - 1) ? 0 : q + 1; nyv[k] = q < na ? C.pol[j] : T(0); }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < K; ++k) { int q = k * G + gl; if (q < na) C.pol[q] = pz[k]; }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < K; ++k) { int q = k * G + gl; int j = (q == na - 1) ? 0 : q + 1; nzv[k] = q < na ? C.pol[j] : T(0); }
    __builtin_amdgcn_wave_barrier();
    // IS_INSIDE_PF(sorted polygon, b_t) for t = 0, 1
    int cnt_in = 0;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const V3<T> P = t ? b1 : b0;
        T cp[K];
        bool pos = false;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            int q = k * G + gl;
            cp[k] = (nxv[k] - px[k]) * (P.y - py[k]) - (nyv[k] - py[k]) * (P.x - px[k]);
            if (fabs(cp[k]) < Tol<T>::Z) cp[k] = T(0);
            pos = pos || (q < na && cp[k] > Tol<T>::POS);
        }
        if (!c.g.any(pos)) {
#pragma unroll
            for (int k = 0; k < K; ++k) cp[k] = (nxv[k] - px[k]) * (P.z - pz[k]) - (nzv[k] - pz[k]) * (P.x - px[k]);
        }
        if (gl == 0) C.pol[0] = cp[0];     // element 0 lives on group lane 0, slot 0
        __builtin_amdgcn_wave_barrier();
        const T c0 = C.pol[0];
        __builtin_amdgcn_wave_barrier();
        bool neg = false;
#pragma unroll
        for (int k = 0; k < K; ++k) { int q = k * G + gl; neg = neg || (q < na && c0 * cp[k] < T(0)); }
        if (!c.g.any(neg)) ++cnt_in;
    }
    if (cnt_in == 0) {                                             // case_04_1
        T sx = 0, sy = 0, sz = 0;
        for (int i = 0; i < na; ++i) { const V3<T> q = set_pt(c, i); sx += q.x; sy += q.y; sz += q.z; }
        const T dn = (T)na;
        res = foot_pl(vmk<T>(sx / dn, sy / dn, sz / dn), b0, b1);
    } else {
        res = vscl(T(0.5), vadd(b0, b1));                          // case_04_2 / case_04_3
    }
    return 0;
}

// case_04 with the point sets left in LDS (GJKEPA_CASE04_LDS): the same arithmetic as contact_case04,
// but each lane reads its set elements (sx/sy/sz[i]), the ordered polygon (sx[ord[q]]) and its next
// vertex from the group's LDS image at each use instead of holding K-element copies in registers, so
// the contact kernel does not carry 60 VGPRs for the quarter of its pairs that take case_04.
CTX_T DEV int contact_case04_lds(CTX& c, int na, V3<T> b0, V3<T> b1, V3<T>& res) {
    auto& C = c.L.u.c;
    const int gl = c.g.gl;
    const T TWO_PI_SP = (T)(2.0f * 3.14159274101257324f);
    auto pt = [&](int i) { return set_pt(c, i); };
    // OVERLAP (:1399-1418): all points pairwise within 1e-12 -> order unchanged
    bool diff = false;
    for (int i0 = 0; i0 < na; i0 += G) {
        int i = i0 + gl;
        if (i < na) {
            const V3<T> pi = set_pt(c, i);
            for (int j = 0; j < na; ++j) {
                const V3<T> pj = set_pt(c, j);
                diff = diff || fabs(pi.x - pj.x) > Tol<T>::Z || fabs(pi.y - pj.y) > Tol<T>::Z || fabs(pi.z - pj.z) > Tol<T>::Z;
            }
        }
    }
    const bool ovl = !c.g.any(diff);
    if (!ovl) {
        T sx = 0, sy = 0, sz = 0;
        for (int i = 0; i < na; ++i) { const V3<T> q = set_pt(c, i); sx += q.x; sy += q.y; sz += q.z; }
        const T dn = (T)na;
        const V3<T> cen = vmk<T>(sx / dn, sy / dn, sz / dn);
        const V3<T> p0 = pt(0);
        const V3<T> nrm = cross(vsub(pt(1), p0), vsub(pt(2), p0));
        V3<T> prev = p0;
        if (gl == 0) C.ord[0] = 0u;
        uint32_t used = 0;                                         // bit k: element k*G + gl is placed
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int i = k * G + gl;
            if (i < na) { const V3<T> q = pt(i); if (q.x == p0.x && q.y == p0.y && q.z == p0.z) used |= 1u << k; }
        }
        for (int s = 1; s < na; ++s) {
            gk_lds_fence();
            T best = Tol<T>::BIG;
            int bi = 0x7fffffff;
#pragma unroll 1
            for (int k = 0; k < K && k * G < na; ++k) {             // one atan2 / fmod instance, not K
                const int j = k * G + gl;
                if (j < na && !((used >> k) & 1u)) {
                    const V3<T> w1 = vsub(pt(j), cen), w2 = vsub(prev, cen);
                    T ang = tatan2(dot(nrm, cross(w2, w1)), dot(w1, w2));
                    ang = tfmod(ang + TWO_PI_SP, TWO_PI_SP);
                    if (ang < best) { best = ang; bi = j; }
                }
            }
            gargmin<G>(best, bi);
            bi = c.g.uni(bi);
            if (bi == 0x7fffffff) return GJKEPA_STATUS_DEGENERATE;
            prev = pt(bi);
            if (gl == 0) C.ord[s] = (uint32_t)bi;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int j = k * G + gl;
                if (j < na) { const V3<T> q = pt(j); if (q.x == prev.x && q.y == prev.y && q.z == prev.z) used |= 1u << k; }
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    // ordered polygon vertex q (SORT_CLOCK's order, or the input order when the points overlap)
    auto opt = [&](int q) { return pt(ovl ? q : (int)C.ord[q]); };
    // IS_INSIDE_PF(sorted polygon, b_t) for t = 0, 1: edge q = (vertex q, vertex q + 1 mod na)
    int cnt_in = 0;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const V3<T> P = t ? b1 : b0;
        auto cp_xy = [&](int q) {
            const V3<T> a = opt(q), b = opt(q == na - 1 ? 0 : q + 1);
            T v = (b.x - a.x) * (P.y - a.y) - (b.y - a.y) * (P.x - a.x);
            if (fabs(v) < Tol<T>::Z) v = T(0);
            return v;
        };
        auto cp_xz = [&](int q) {
            const V3<T> a = opt(q), b = opt(q == na - 1 ? 0 : q + 1);
            return (b.x - a.x) * (P.z - a.z) - (b.z - a.z) * (P.x - a.x);
        };
        bool pos = false;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int q = k * G + gl;
            if (q < na) pos = pos || cp_xy(q) > Tol<T>::POS;
        }
        const bool xz = !c.g.any(pos);
        gk_lds_fence();
        const T c0 = xz ? cp_xz(0) : cp_xy(0);                   // element 0's cross product, on every lane
        bool neg = false;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int q = k * G + gl;
            if (q < na) neg = neg || c0 * (xz ? cp_xz(q) : cp_xy(q)) < T(0);
        }
        if (!c.g.any(neg)) ++cnt_in;
    }
    if (cnt_in == 0) {                                             // case_04_1
        T sx = 0, sy = 0, sz = 0;
        for (int i = 0; i < na; ++i) { const V3<T> q = set_pt(c, i); sx += q.x; sy += q.y; sz += q.z; }
        const T dn = (T)na;
        res = foot_pl(vmk<T>(sx / dn, sy / dn, sz / dn), b0, b1);
    } else {
        res = vscl(T(0.5), vadd(b0, b1));                          // case_04_2 / case_04_3
    }
    return 0;
}
#ifndef GJKEPA_CASE04_LDS
#define GJKEPA_CASE04_LDS 1      // case_04 reads its point sets from LDS (0: register copies, A/B)
#endif

// get_collisionPoint_02 (:457-696)
CTX_T DEV int contact_v2(CTX& c, const DotSet<T, K>& D, V3<T>& res) {
    const T band = T(0.1);
    const T t1 = D.m[0] - band, t2 = D.m[1] - band;                 // :471-472
    const int n1 = band_set(c, 0, D, t1, false);
    const int n2 = band_set(c, 1, D, t2, false);
    res = zero3<T>();
    if (n1 == 1 && n2 == 1) {                                      // case_01
        band_set(c, 0, D, t1, true);
        const V3<T> a = set_pt(c, 0);
        __builtin_amdgcn_wave_barrier();
        band_set(c, 1, D, t2, true);
        res = vdiv(vadd(a, set_pt(c, 0)), T(2));
    } else if (n1 == 1 && n2 >= 2) {                               // case_02
        band_set(c, 0, D, t1, true);
        res = set_pt(c, 0);
    } else if (n1 >= 2 && n2 == 1) {
        band_set(c, 1, D, t2, true);
        res = set_pt(c, 0);
    } else if (n1 == 2 && n2 == 2) {                               // case_03
        band_set(c, 0, D, t1, true);
        const V3<T> a0 = set_pt(c, 0), a1 = set_pt(c, 1);
        __builtin_amdgcn_wave_barrier();
        band_set(c, 1, D, t2, true);
        V3<T> f1, f2;
        foot_ll(a0, a1, set_pt(c, 0), set_pt(c, 1), f1, f2);
        res = vdiv(vadd(f1, f2), T(2));
    } else if (n1 == 2 && n2 >= 3) {                               // case_04(SPT_p2, SPT_p1)
        band_set(c, 0, D, t1, true);
        const V3<T> q0 = set_pt(c, 0), q1 = set_pt(c, 1);
        __builtin_amdgcn_wave_barrier();
        band_set(c, 1, D, t2, true);
        return GJKEPA_CASE04_LDS ? contact_case04_lds(c, n2, q0, q1, res) : contact_case04(c, n2, q0, q1, res);
    } else if (n1 >= 3 && n2 == 2) {                               // case_04(SPT_p1, SPT_p2)
        band_set(c, 1, D, t2, true);
        const V3<T> q0 = set_pt(c, 0), q1 = set_pt(c, 1);
        __builtin_amdgcn_wave_barrier();
        band_set(c, 0, D, t1, true);
        return GJKEPA_CASE04_LDS ? contact_case04_lds(c, n1, q0, q1, res) : contact_case04(c, n1, q0, q1, res);
    } else if (n1 >= 3 && n2 >= 3) {                               // case_05
        band_set(c, 0, D, t1, true);
        T sx = 0, sy = 0, sz = 0;
        for (int i = 0; i < n1; ++i) { const V3<T> q = set_pt(c, i); sx += q.x; sy += q.y; sz += q.z; }
        const T dn = (T)n1;
        res = vmk<T>(sx / dn, sy / dn, sz / dn);
    } else {
        return GJKEPA_STATUS_DEGENERATE;                           // :498-501
    }
    return 0;
}

// get_collisionPoint_03 (:426-452)
CTX_T DEV int contact_v3(CTX& c, V3<T> n, V3<T>& res, V3<T>& nnew) {
    const V3<T> nn = vneg(n);
    T mx = -Tol<T>::BIG;
    int idx = -1;
    for (int i = 0; i < c.nb; ++i) {
        T t = dot(nn, c.B(i));
        if (t > mx - Tol<T>::PT) { mx = t; idx = i; }
    }
    if (idx < 0) return GJKEPA_STATUS_DEGENERATE;
    T sz = 0;
    for (int i = 0; i < c.na; ++i) sz += (T)c.rawc(0, i, 2);
    res = c.B(idx);
    res.z = sz / (T)(float)c.na;
    const V3<T> q = vmk<T>(n.x, n.y, T(0));
    const T nq = norm2(q);
    nnew = vdiv(q, nq);
    return 0;
}

// ---------------------------------------------------------------- GJK phase (GJKEPA :39-239)
// A simplex vertex is a Minkowski point A[ia] - B[ib]; it is carried as the code ia | ib << 16 so
// the EPA kernel can rebuild it bit for bit.  kStale encodes the never-assigned row 4 (= 0).
constexpr uint32_t kStale = 0xFFFFFFFFu;
constexpr int PH_MISS = 0, PH_HIT = -1;

CTX_T DEV V3<T> support_pt(const CTX& c, V3<T> d, uint32_t& code) {
    int ia, ib;
    support_idx(c, d, ia, ib);
    code = (uint32_t)ia | ((uint32_t)ib << 16);
    return vsub(c.A(ia), c.B(ib));
}
CTX_T DEV V3<T> decode_pt(const CTX& c, uint32_t code) {
    if (code == kStale) return zero3<T>();
    return vsub(c.A((int)(code & 0xffffu)), c.B((int)(code >> 16)));
}

// update_simplex_GJK (:1070-1157) with vertex codes carried along
// The four faces are evaluated on the quad lanes (raw normal nq of this lane's face q); the
// first-index MAXLOC is a two-step quad butterfly that carries the winning normal along.
CTX_T DEV void update_simplex_c(const CTX& c, V3<T> nq, V3<T>& s0, V3<T>& s1, V3<T>& s2, V3<T>& s3,
                                uint32_t& k0, uint32_t& k1, uint32_t& k2, uint32_t& k3) {
    const V3<T> M = centroid4(s0, s1, s2, s3), O = zero3<T>();
    const int q = c.g.gl & 3;
    const V3<T> ref = q == 3 ? s1 : s0;
    if (dot(nq, vsub(ref, M)) < T(0)) nq = vneg(nq);
    T best = dot(vneg(nq), vsub(ref, O));
    int k = q;
    V3<T> dir = nq;
#pragma unroll
    for (int st = 0; st < 2; ++st) {
        const T ob = st == 0 ? xchg<0>(best) : xchg<1>(best);
        const int ok = st == 0 ? xchg<0>(k) : xchg<1>(k);
        const V3<T> od = st == 0 ? vmk<T>(xchg<0>(dir.x), xchg<0>(dir.y), xchg<0>(dir.z))
                                 : vmk<T>(xchg<1>(dir.x), xchg<1>(dir.y), xchg<1>(dir.z));
        const bool take = ob > best || (ob == best && ok < k);
        best = take ? ob : best;
        k = take ? ok : k;
        dir = vsel(take, od, dir);
    }
    k = c.g.uni(k);
    uint32_t km;
    const V3<T> SM = support_pt(c, dir, km);
    const V3<T> o0 = s0, o1 = s1, o2 = s2;
    const uint32_t c0 = k0, c1 = k1, c2 = k2, c3 = k3;
    s0 = vsel(k == 3, o1, o0);
    s1 = vsel(k == 0 || k == 3, o2, o1);
    s2 = vsel(k == 2, o2, s3);
    s3 = SM;
    k0 = k == 3 ? c1 : c0;
    k1 = (k == 0 || k == 3) ? c2 : c1;
    k2 = k == 2 ? c2 : c3;
    k3 = km;
}

// Warm start: the simplex a previous call ended GJK with, as support codes
// (ia | ib << 16).  Rebuilt from the current vertices; when the origin lies strictly inside it (every
// face more than kWarmMargin from the origin, so the hulls certainly overlap and a flat or touching
// tetrahedron never qualifies), the pair is a hit and EPA starts from it: GJK's iterations are
// skipped.  Otherwise the call runs the reference GJK from scratch.  Results then agree with a cold
// call to EPA's tolerance rather than bit for bit (a different start polytope).
// A pair that missed is marked kWarmMiss; its next call runs the reference GJK (a shortcut for
// misses is not parity-safe: the reference reports hits on some separated hulls).
constexpr double kWarmMargin = 1e-6;
constexpr uint32_t kWarmMiss = 0xFFFFFFFEu;
CTX_T DEV bool warm_start(CTX& c, const uint32_t* w, uint32_t* kc) {
    uint32_t code[4];
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        code[i] = w[i];
        ok = ok && code[i] != kStale && (int)(code[i] & 0xffffu) < c.na && (int)(code[i] >> 16) < c.nb;
    }
    if (!c.g.unib(ok)) return false;
    const V3<T> s0 = decode_pt(c, code[0]), s1 = decode_pt(c, code[1]), s2 = decode_pt(c, code[2]), s3 = decode_pt(c, code[3]);
    const V3<T> M = centroid4(s0, s1, s2, s3), O = zero3<T>();
    const V3<T> P[4] = {s0, s1, s2, s3};
    const int F[4][3] = {{0, 2, 3}, {0, 1, 3}, {0, 1, 2}, {1, 2, 3}};
    bool inside = true;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
        V3<T> n = face_nml(P[F[f][0]], P[F[f][1]], P[F[f][2]]);
        if (dot(n, vsub(P[F[f][0]], M)) < T(0)) n = vneg(n);
        inside = inside && dot(vsub(P[F[f][0]], O), n) > T(kWarmMargin);
    }
    if (!c.g.unib(inside)) return false;
#pragma unroll
    for (int i = 0; i < 4; ++i) kc[i] = code[i];
    return true;
}

// Sphere pre-test + GJK.  Returns PH_MISS, PH_HIT (codes k0..k3 filled) or an error status.
CTX_T DEV int gjk_phase(CTX& c, uint32_t* kc, int& gjk_it, bool try_axis = false) {
    const V3<T> O = zero3<T>();
    auto& L = c.L;
    const int gl = c.g.gl;
    gjk_it = 0;
    bool axis_sep = false;
    {   // RoughCollisionDetection_SphericalEnvelope (:1165-1188)
        // the six sequential coordinate sums run on group lanes (sum j on lane j % G: hull j/3, axis j%3)
        T cs[(6 + G - 1) / G];           // centroid coordinate j0 + gl of pass j0 / G (hull j / 3, axis j % 3)
#pragma unroll
        for (int j0 = 0; j0 < 6; j0 += G) {
            const int j = j0 + gl;
            cs[j0 / G] = T(0);
            if (j < 6) {
                const int h = j / 3, ax = j - 3 * (j / 3);
#if GJKEPA_HULL_AOS
                const TH* col = &L.hv[h][0].x + ax;  // coordinate ax of vertex i at col[4 i]
                constexpr int CS = 4;
#else
                const TH* col = ax == 0 ? L.hx[h] : ax == 1 ? L.hy[h] : L.hz[h];
                constexpr int CS = 1;
#endif
                const int n = h ? c.nb : c.na;
                T sum = 0;
                int i = 0;
                for (; i + 8 <= n; i += 8) {         // loads batched ahead of the in-order adds
                    TH v[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) v[u] = col[CS * (i + u)];
#pragma unroll
                    for (int u = 0; u < 8; ++u) sum += (T)v[u];
                }
                for (; i < n; ++i) sum += (T)col[CS * i];
                cs[j0 / G] = sum / (T)n;
            }
        }
        // broadcast to the group from the lane that summed it (no LDS image space)
        const int gb = c.g.lane & ~(G - 1);
        auto mc = [&](int j) { return __shfl(cs[j / G], gb + j % G); };
        const V3<T> m1 = vmk<T>(mc(0), mc(1), mc(2)), m2 = vmk<T>(mc(3), mc(4), mc(5));
        // max_i NORM2(p_i - m) = sqrt(max_i |p_i - m|^2): sqrt is monotone under correct rounding
        T r1 = -Tol<T>::BIG, r2 = -Tol<T>::BIG;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            int i = k * G + gl;
            const V3<T> da = vsub(c.AV(k), m1);
            const T ta = da.x * da.x + da.y * da.y + da.z * da.z;
            if (i < c.na && ta > r1) r1 = ta;
            const V3<T> db = vsub(c.BV(k), m2);
            const T tb = db.x * db.x + db.y * db.y + db.z * db.z;
            if (i < c.nb && tb > r2) r2 = tb;
        }
        r1 = tsqrt(gmax<G>(r1));
        r2 = tsqrt(gmax<G>(r2));
        GK_STAMP(SG_SPHERE);
        if (!c.g.unib(norm2(vsub(m1, m2)) <= r1 + r2 + T(1))) return PH_MISS;
        // Diagnostic quick reject (GJKEPA_AXIS_REJECT builds only): the axis between the hull
        // centres separates the hulls by more than kWarmMargin, so a pair the initial-simplex block
        // does not call a hit is answered "miss" without the tetrahedron loop.  NOT parity-safe:
        // the reference's loop can still report a hit on such a pair through isPointInSimplex's
        // on-face branch (:1246-1256), e.g. a unit cube vs the cube moved by (-1, 0, 2).
        if (try_axis) {
            const V3<T> d = vsub(m2, m1);
            T amax = -Tol<T>::BIG, bmin = Tol<T>::BIG;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int i = k * G + gl;
                const V3<T> pa = c.AV(k), pb = c.BV(k);
                const T ta = d.x * pa.x + d.y * pa.y + d.z * pa.z;
                const T tb = d.x * pb.x + d.y * pb.y + d.z * pb.z;
                if (i < c.na && ta > amax) amax = ta;
                if (i < c.nb && tb < bmin) bmin = tb;
            }
            amax = gmax<G>(amax);
            bmin = gmin<G>(bmin);
            const T margin = sizeof(T) == 8 ? T(kWarmMargin) : T(1e-4);
            axis_sep = c.g.unib(bmin - amax > margin * norm2(d));
        }
    }
    // --- initial simplex (:82-170)
    V3<T> s0 = O, s1 = O, s2 = O, s3 = O;   // fresh SAVE state: stale row 4 = 0
    uint32_t k0 = kStale, k1 = kStale, k2 = kStale, k3 = kStale;
    V3<T> dir;
    for (int iter = 1;; ++iter) {
        if (iter > 99) return PH_MISS;
        dir = vmk<T>((T)kDirTab[iter - 1][0], (T)kDirTab[iter - 1][1], (T)kDirTab[iter - 1][2]);
        s0 = support_pt(c, dir, k0);
        dir = vneg(dir);
        s1 = support_pt(c, dir, k1);
        if (!c.g.unib(allclose8(s0, s1))) break;
    }
    dir = vec_pl(O, s0, s1);
    s2 = support_pt(c, dir, k2);
    if (c.g.unib(allclose8(s2, s0) || allclose8(s2, s1))) return PH_MISS;
    dir = utzvec(cross(vsub(s1, s0), vsub(s2, s1)));
    const T vd = dot(vsub(O, s2), dir);
    bool enter = false;
    if (c.g.unib(fabs(vd) < Tol<T>::PT) && c.g.unib(inside_tri(s0, s1, s2, O))) enter = true;
    const int q = gl & 3;
    V3<T> nq = zero3<T>();   // this quad lane's raw face normal of the current simplex
    T mdq = 0;
    if (!enter) {
        if (c.g.unib(vd < T(0))) dir = vneg(dir);
        s3 = support_pt(c, dir, k3);
        const V3<T> n = uninml(s0, s1, s2);                         // DIST_PF_SIGN (:157)
        if (c.g.unib(is_zero_nml(n))) return GJKEPA_STATUS_DEGENERATE;
        if (c.g.unib(fabs(dot(vsub(s3, s0), n)) < Tol<T>::PT)) return PH_MISS;
        nq = quad_normal(q, s0, s1, s2, s3, mdq);
        if (c.g.unib(quad_inside(q, s0, s1, s2, s3, nq))) enter = true;
    }
    GK_STAMP(SG_INIT);
    // the quick reject answers only after the initial-simplex block: that block is where the
    // reference reports hits for separated tie-heavy hulls (origin on the initial triangle's plane)
    if (!enter && axis_sep) return PH_MISS;
    if (!enter) {
        // cycle history (:193-194): coordinate j < 12 of last1 / last2 lives on group lane j % G,
        // slot j / G
        constexpr int HS = (12 + G - 1) / G;
        T h1[HS], h2[HS];
#pragma unroll
        for (int t = 0; t < HS; ++t) { h1[t] = 0; h2[t] = 0; }
        const uint64_t lowg = G == 64 ? ~0ull : ((1ull << (G & 63)) - 1ull);
        const int sh = c.g.lane & ~(G - 1);
        for (int it = 1;; ++it) {                                        // :182-236
            gjk_it = it;
            if (it > 50) return PH_MISS;
#pragma unroll
            for (int t = 0; t < HS; ++t) {
                const int j = t * G + gl;
                h2[t] = h1[t];
                h1[t] = simplex_coord(j < 12 ? j : 0, s0, s1, s2, s3);
            }
            GK_STAMP(SG_CHK);
            update_simplex_c(c, nq, s0, s1, s2, s3, k0, k1, k2, k3);
            nq = quad_normal(q, s0, s1, s2, s3, mdq);
            GK_STAMP(SG_UPD);
            // :199-201 NORM2((s2-s1)x(s3-s2)) is face [1,2,3]'s |cross| (operands negated: same bits)
            if (c.g.unib(qbcast<2>(mdq) < Tol<T>::PT)) return PH_MISS;
            // :203 UNINML(s1,s2,s3) is then face [1,2,3]'s normal (|cross| >= 1e-8: never the zero case)
            const V3<T> n = vmk<T>(qbcast<2>(nq.x), qbcast<2>(nq.y), qbcast<2>(nq.z));
            if (c.g.unib(fabs(dot(vsub(s3, s0), n)) < Tol<T>::PT)) return PH_MISS;         // :203-206
            if (c.g.unib(quad_inside(q, s0, s1, s2, s3, nq))) break;                      // :210-216
            uint32_t e1 = 0, e2 = 0;                                                       // :219-234
#pragma unroll
            for (int t = 0; t < HS; ++t) {
                const int j = t * G + gl;
                const T cur = simplex_coord(j < 12 ? j : 0, s0, s1, s2, s3);
                e1 |= (uint32_t)((__ballot(fabs(cur - h1[t]) < Tol<T>::PT) >> sh) & lowg) << (t * G);
                e2 |= (uint32_t)((__ballot(fabs(cur - h2[t]) < Tol<T>::PT) >> sh) & lowg) << (t * G);
            }
            e1 &= 0xFFFu;
            e2 &= 0xFFFu;
            bool over = true;
#pragma unroll
            for (int p = 0; p < 4; ++p) over = over && (((e1 >> (3 * p)) & 7u) == 7u || ((e2 >> (3 * p)) & 7u) == 7u);
            if (c.g.unib(over)) return PH_MISS;
        }
        GK_STAMP(SG_CHK);
    }
    kc[0] = k0; kc[1] = k1; kc[2] = k2; kc[3] = k3;
    return PH_HIT;
}

// EPA_solu's polytope loop (:274-323) from the GJK simplex: 0 (depth, n filled), an error
// status or ST_DEFER; `diag_epa` gets (epa_iters << 8) | (faces << 16).
CTX_T DEV int epa_phase(CTX& c, const uint32_t* kc, T& depth, V3<T>& n, uint32_t& diag_epa, bool park = false,
                        ParkCtl pk = {}, const unsigned char* rec = nullptr, uint32_t* gjk_it = nullptr) {
    V3<T> s0 = zero3<T>(), s1 = s0, s2 = s0, s3 = s0;
    if (!rec) { s0 = decode_pt(c, kc[0]); s1 = decode_pt(c, kc[1]); s2 = decode_pt(c, kc[2]); s3 = decode_pt(c, kc[3]); }
    depth = 0;
    n = zero3<T>();
    int eit = 0, nf = 0;
    const int st = epa(c, s0, s1, s2, s3, depth, n, eit, nf, park, pk, rec, gjk_it);
    diag_epa = ((uint32_t)(eit & 0xff) << 8) | ((uint32_t)(nf & 0xffff) << 16);
    return st;
}

// EPA_solu's post-processing (:326-343) for EPA depth and normal n: nearest points, contact point
// (version_ 1/2/3) and contact type.  Returns -type (o13 filled) or an error status.
CTX_T DEV int contact_phase(CTX& c, T depth, V3<T> n, int version, T tol_ff, T* o13) {
    int st;
    int ia, ib;
    GK_STAMP(SE_TERM);
    // get_nearest_points (:326, :813-855): one pass of dots along n over both hulls, whose values
    // and maxima the contact point (v1, v2) and the contact type also use
    DotSet<T, K> D;
    support_dots(c, n, D, ia, ib);
    GK_STAMP(SE_NEAR);
    V3<T> pt = zero3<T>();
    // get_info_collisionType (:343) along the EPA normal depends only on these dots: taken before the
    // contact point, so the dots are dead during case_04 (the contact kernel's register peak)
    int type = (version == 1 || version == 2) ? collision_type(c, D, tol_ff) : 0;
    if (version == 1) st = contact_v1(c, n, D, pt);                       // :329-340
    else if (version == 2) st = contact_v2(c, D, pt);
    else if (version == 3) { V3<T> nw; st = contact_v3(c, n, pt, nw); n = nw; }
    else st = GJKEPA_STATUS_BAD_VERSION;
    GK_STAMP(SE_CONT);
    if (st) return st;
    if (version == 3) type = collision_type(c, n, tol_ff);             // along v3's replaced normal
    GK_STAMP(SE_TYPE);
    const V3<T> q1 = c.A(ia), q2 = c.B(ib);
    __builtin_amdgcn_wave_barrier();
    o13[0] = depth;
    o13[1] = n.x; o13[2] = n.y; o13[3] = n.z;
    o13[4] = pt.x; o13[5] = pt.y; o13[6] = pt.z;
    o13[7] = q1.x; o13[8] = q1.y; o13[9] = q1.z;
    o13[10] = q2.x; o13[11] = q2.y; o13[12] = q2.z;
    return -type;
}

// ---------------------------------------------------------------- kernels
// Hull load: coalesced SoA loads into registers (compute precision) and the LDS copy.
CTX_T DEV bool load_hulls(CTX& c, const TH* __restrict__ pa, const TH* __restrict__ pb) {
    const int gl = c.g.gl;
    bool nonfinite = false;
    // the hulls' largest |coordinate|: the fp32 support screen's bound, the fp32 certificate's scale
    constexpr bool kScreen = (ScreenOn<K>::value && sizeof(T) == 8 && sizeof(TH) == 4) || certify<T>();
    float ma = 0.0f, mb = 0.0f;     // largest |coordinate| (support screen bound; padding lanes hold 0)
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int i = k * G + gl;
        TH ax = 0, ay = 0, az = 0, bx = 0, by = 0, bz = 0;
        // slots past the count: zeros, or vertex 0 again (GJKEPA_PAD_V0, support_dots)
        const int ja = i < c.na ? i : 0, jb = i < c.nb ? i : 0;
        if (i < c.na || (GJKEPA_PAD_V0 && c.na > 0)) { ax = pa[ja]; ay = pa[c.na + ja]; az = pa[2 * c.na + ja]; }
        if (i < c.nb || (GJKEPA_PAD_V0 && c.nb > 0)) { bx = pb[jb]; by = pb[c.nb + jb]; bz = pb[2 * c.nb + jb]; }
        nonfinite = nonfinite || !isfinite(ax) || !isfinite(ay) || !isfinite(az) || !isfinite(bx) ||
                    !isfinite(by) || !isfinite(bz);
        if constexpr (kScreen) {
            ma = fmaxf(ma, fmaxf(fabsf((float)ax), fmaxf(fabsf((float)ay), fabsf((float)az))));
            mb = fmaxf(mb, fmaxf(fabsf((float)bx), fmaxf(fabsf((float)by), fabsf((float)bz))));
        }
        if constexpr (CTX::kRegHull) {
            c.ax[k] = (T)ax; c.ay[k] = (T)ay; c.az[k] = (T)az;
            c.bx[k] = (T)bx; c.by[k] = (T)by; c.bz[k] = (T)bz;
        }
#if GJKEPA_HULL_AOS
        c.L.hv[0][i] = HV<TH>{ax, ay, az, TH(0)};
        c.L.hv[1][i] = HV<TH>{bx, by, bz, TH(0)};
#else
        c.L.hx[0][i] = ax; c.L.hy[0][i] = ay; c.L.hz[0][i] = az;
        c.L.hx[1][i] = bx; c.L.hy[1][i] = by; c.L.hz[1][i] = bz;
#endif
    }
    if constexpr (kScreen) {
        c.vmax_a = gmax<G>(ma);
        c.vmax_b = gmax<G>(mb);
    }
    __builtin_amdgcn_wave_barrier();
    return c.g.any(nonfinite);
}

// record: 13 T fields, then int8 collision, type, status, reserved, uint32 diag, zero pad.
// Its 16 8-byte (f64) / 4-byte (f32) words are stored straight from registers, word j by group
// lane j % G.
template <int G, typename T> DEV void store_record(void* out, int64_t pair, int gl, const T* o13, int hit, int type,
                                                   int status, uint32_t diag) {
    const uint32_t flags = (uint32_t)(hit & 0xff) | ((uint32_t)(type & 0xff) << 8) | ((uint32_t)(status & 0xff) << 16);
#pragma unroll
    for (int j0 = 0; j0 < 16; j0 += G) {
        const int j = j0 + gl;
        if (j >= 16) break;
        T v = T(0);
#pragma unroll
        for (int i = 0; i < 13; ++i) v = (j == i) ? o13[i] : v;
        if constexpr (sizeof(T) == 8) {
            uint64_t word = __builtin_bit_cast(uint64_t, v);
            if (j == 13) word = (uint64_t)flags | ((uint64_t)diag << 32);
            if (j > 13) word = 0;
            reinterpret_cast<uint64_t*>(out)[pair * 16 + j] = word;
        } else {
            uint32_t word = __builtin_bit_cast(uint32_t, v);
            if (j == 13) word = flags;
            if (j == 14) word = diag;
            if (j == 15) word = 0;
            reinterpret_cast<uint32_t*>(out)[pair * 16 + j] = word;
        }
    }
}

// hull capacity (vertices) of EPA tier t
DEV constexpr int epa_hull_cap(int t) {
    return t == 0 ? GJKEPA_E0_G * GJKEPA_E0_K : t == 1 ? GJKEPA_E1_G * GJKEPA_E1_K : t == 2 ? GJKEPA_E2_G * GJKEPA_E2_K
         : t == 3 ? GJKEPA_E3_G * GJKEPA_E3_K : t == 4 ? GJKEPA_E4_G * GJKEPA_E4_K : GJKEPA_E5_G * GJKEPA_E5_K;
}
// polytope vertex capacity of EPA tier t
DEV constexpr int epa_vcap(int t) {
    return t == 0 ? GJKEPA_E0_VCAP : t == 1 ? GJKEPA_E1_VCAP : t == 2 ? GJKEPA_E2_VCAP : t == 3 ? GJKEPA_E3_VCAP
         : t == 4 ? GJKEPA_E4_VCAP : GJKEPA_E5_VCAP;
}
static_assert(GJKEPA_E5_G * GJKEPA_E5_K >= GJKEPA_MAX_HULL_VERTS, "the last EPA tier must hold every hull");
// smallest EPA tier >= t0 whose hull capacity holds nmax vertices and whose polytope capacity
// exceeds vc (a pair deferred by a tier with polytope capacity vc skips tiers no larger)
DEV int epa_tier_for(int nmax, int t0 = 0, int vc = 0) {
    for (int t = t0; t < GJKEPA_EPA_TIERS - 1; ++t)
        if (nmax <= epa_hull_cap(t) && epa_vcap(t) > vc) return t;
    return GJKEPA_EPA_TIERS - 1;
}

// Work distribution: runs of `claim` 64-pair chunks are handed out dynamically (one atomic per
// wave per run on this launch's counter, prefetched one run ahead), so the launch ends within
// about one run of its slowest wave.  Busy launches claim single chunks; launches that serve few
// pairs claim long runs so the scan is not bound by atomics on one address.  Inside a chunk, the wave ballots the pairs whose route byte matches this
// launch (one coalesced byte load) and hands them to its 64/G groups in pair order, one per group
// per round.  `route_code` < 0: every pair.  F(pair) runs for each pair the calling group receives.
// META: the pair metadata the callee needs first (hull counts and offsets) is loaded for every routed
// pair of the chunk at once (lane l: pair p0 + l) and handed to each group with ds_bpermute, so a
// round waits on one level of loads (the hulls) instead of three (pair -> hull -> vertices).
struct PairMeta { int na, nb; int64_t oa, ob; };
DEV int64_t shfl64(int64_t v, int src) {
    const int lo = __shfl((int)(uint32_t)(uint64_t)v, src), hi = __shfl((int)(uint32_t)((uint64_t)v >> 32), src);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
template <int G, bool META = false, typename F>
DEV void groups_take(const Grp<G>& grp, int64_t p0, uint64_t m, const int32_t* pairs, const int32_t* cnt,
                     const int64_t* off, F&& f) {
    constexpr int GPW = 64 / G;
    const int gid = grp.lane / G;
    PairMeta mine{0, 0, 0, 0};
    if constexpr (META) {
        if ((m >> grp.lane) & 1ull) {
            const int64_t p = p0 + grp.lane;
            const int32_t ha = pairs[2 * p], hb = pairs[2 * p + 1];
            mine.na = cnt[ha]; mine.nb = cnt[hb]; mine.oa = off[ha]; mine.ob = off[hb];
        }
    }
    while (m) {
        // group g takes the g-th lowest set bit of m
        uint64_t mm = m;
        for (int j = 0; j < gid && mm; ++j) mm &= mm - 1;
        const bool active = mm != 0;
        const int bit = active ? (int)__builtin_ctzll(mm) : 0;
        for (int j = 0; j < GPW && m; ++j) m &= m - 1;   // consume this round's GPW matches
        if constexpr (META) {
            PairMeta pm;
            pm.na = __shfl(mine.na, bit); pm.nb = __shfl(mine.nb, bit);
            pm.oa = shfl64(mine.oa, bit); pm.ob = shfl64(mine.ob, bit);
            if (active) f(p0 + bit, pm);
        } else {
            if (active) f(p0 + bit);
        }
    }
}
// 16-bit mask of this lane's 16 route bytes equal to code
DEV uint32_t match16(uint4 v, uint32_t code) {
    uint32_t m = 0;
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 16; ++i) m |= (((w[i >> 2] >> (8 * (i & 3))) & 0xffu) == code ? 1u : 0u) << i;
    return m;
}
// Work units of a launch (guided chunking): 64-pair chunks first, then the last `tail` pairs in
// units of SMALL pairs, so a wave that takes its last unit late holds a few pairs, not 64.  The
// tail covers about 64 pairs per workgroup of the grid (at most half the pairs).
struct Units {
    int64_t n_pairs, nbig, nunits;
    int small;
    DEV Units(int64_t n, int small_, bool whole_chunks = false) : n_pairs(n), small(small_) {
        int64_t tail = whole_chunks ? 0 : (int64_t)gridDim.x * 64;
        if (tail > n / 2) tail = n / 2;
        nbig = (n - tail) / 64;
        nunits = nbig + (n - nbig * 64 + small - 1) / small;
    }
    DEV void range(int64_t u, int64_t& p0, int& len) const {
        if (u < nbig) { p0 = u * 64; len = 64; }
        else { p0 = nbig * 64 + (u - nbig) * small; len = small; }
        if (p0 + len > n_pairs) len = (int)(n_pairs - p0);
    }
};
// Tail unit size: SMALL pairs, or one wave-round (64 / G pairs) when the launch has fewer than 8
// pairs per workgroup (a latency-bound batch, e.g. combined single-pair queries: spread the pairs
// over more waves instead of queueing them behind each other in one).
template <int G, int SMALL> DEV int tail_unit(int64_t n) {
    return n <= (int64_t)gridDim.x * 8 ? (64 / G < SMALL ? 64 / G : SMALL) : SMALL;
}

// Route tallies (workspace): each wave counts the pairs it routes per code in LDS and adds them to
// the launch-wide tallies once at its end; a later launch reads its own code's tally to pick dense
// (single-chunk claims) or sparse (runs of a.claim chunks) scheduling.
static __shared__ uint32_t s_tally[GJKEPA_WS_TALLY];
DEV void tally_begin() {
    if (lane_id() < GJKEPA_WS_TALLY) s_tally[lane_id()] = 0;
    __builtin_amdgcn_wave_barrier();
}
DEV void tally_route(uint8_t code) { if (code < GJKEPA_WS_TALLY) atomicAdd(&s_tally[code], 1u); }
DEV void tally_end(uint32_t* tally) {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
    const int l = lane_id();
    if (l < GJKEPA_WS_TALLY && s_tally[l]) atomicAdd(&tally[l], s_tally[l]);
}
// A tier's tally is final when its kernel starts (pairs are only routed to later launches): a tier
// nobody routed a pair to returns at once instead of scanning the route bytes.
DEV bool tier_empty(const uint32_t* tally, int route_code) {
    return route_code >= 0 && __builtin_amdgcn_readfirstlane(tally[route_code]) == 0;
}
DEV int pick_claim(const uint32_t* tally, int route_code, int64_t n_pairs, int claim) {
    if (route_code < 0 || claim <= 1) return claim;
    const uint32_t mine = __builtin_amdgcn_readfirstlane(tally[route_code]);
    return (int64_t)mine * 16 >= n_pairs ? 1 : claim;
}

template <int G, bool META = false, typename F>
DEV void for_each_routed_pair(const Grp<G>& grp, int64_t n_pairs, const uint8_t* __restrict__ route, int route_code,
                              uint32_t* ctr, int claim, bool unit_grid, F&& f, const int32_t* pairs = nullptr,
                              const int32_t* cnt = nullptr, const int64_t* off = nullptr) {
    // the first unit of workgroup b is unit b; later units come from the counter (offset by the
    // grid), so a launch with fewer units than workgroups issues no atomics at all.  unit_grid: the
    // launch has one workgroup per 64-pair chunk (dense launches only): a workgroup takes its own
    // chunk and leaves.
    const int64_t nchunks = (n_pairs + 63) / 64;
    uint32_t next = 0;
    if (unit_grid) {
        const int64_t u = blockIdx.x;
        if (u < nchunks) {
            const int64_t p0 = u * 64;
            const int len = n_pairs - p0 < 64 ? (int)(n_pairs - p0) : 64;
            const uint64_t m = route_code < 0 ? (len >= 64 ? ~0ull : ((1ull << len) - 1ull))
                                              : __ballot(grp.lane < len && (int)route[p0 + grp.lane] == route_code);
            groups_take<G, META>(grp, p0, m, pairs, cnt, off, f);
        }
        return;
    }
    if (claim <= 1 || route_code < 0) {
        const Units U(n_pairs, tail_unit<G, (64 / G > 8 ? 64 / G : 8)>(n_pairs));
        if ((int64_t)blockIdx.x < U.nunits && grp.lane == 0) next = gridDim.x + atomicAdd(ctr, 1u);
        int64_t u = blockIdx.x;
        while (u < U.nunits) {
            if (grp.lane == 0 && u != (int64_t)blockIdx.x) next = gridDim.x + atomicAdd(ctr, 1u);   // prefetch
            int64_t p0;
            int len;
            U.range(u, p0, len);
            uint64_t m;
            if (route_code < 0) {
                m = len >= 64 ? ~0ull : ((1ull << len) - 1ull);
            } else {
                const int64_t p = p0 + grp.lane;
                m = __ballot(grp.lane < len && (int)route[p] == route_code);
            }
            groups_take<G, META>(grp, p0, m, pairs, cnt, off, f);
            u = (int64_t)__builtin_amdgcn_readfirstlane(next);
        }
        return;
    }
    const int64_t nunits = (nchunks + 15) / 16;
    if ((int64_t)blockIdx.x < nunits && grp.lane == 0) next = gridDim.x + atomicAdd(ctr, 1u);
    // runs of 16 chunks: lane l loads route bytes [16 l, 16 l + 16) of the run in one 16-byte load
    for (int64_t run = blockIdx.x; run * 16 < nchunks; run = (int64_t)__builtin_amdgcn_readfirstlane(next)) {
        if (grp.lane == 0 && run != (int64_t)blockIdx.x) next = gridDim.x + atomicAdd(ctr, 1u);
        const int64_t q0 = run * 1024 + 16 * grp.lane;
        uint4 v = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
        if (q0 + 16 <= n_pairs) {
            v = *reinterpret_cast<const uint4*>(route + q0);
        } else {
            uint32_t w[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
            for (int i = 0; i < 16; ++i)
                if (q0 + i < n_pairs) w[i >> 2] = (w[i >> 2] & ~(0xffu << (8 * (i & 3)))) | ((uint32_t)route[q0 + i] << (8 * (i & 3)));
            v = make_uint4(w[0], w[1], w[2], w[3]);
        }
        const uint32_t mine = match16(v, (uint32_t)route_code);
        uint64_t lanes = __ballot(mine != 0);                 // lanes 4j..4j+3 hold chunk j of the run
        while (lanes) {
            const int j = (int)__builtin_ctzll(lanes) >> 2;
            lanes &= ~(0xFull << (4 * j));
            uint64_t m = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                m |= (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)mine, 4 * j + i) << (16 * i);
            groups_take<G, META>(grp, run * 1024 + 64 * j, m, pairs, cnt, off, f);
        }
    }
}

// GJK kernel: sphere pre-test + GJK.  Misses and errors get their final record here; hits park the
// simplex codes (5 words) in their own record slot and are routed to the smallest EPA tier that
// holds their hulls.  Tier 0 takes every pair; hulls above its capacity are routed to tier 1.
// WARM instantiations serve gjkepa_batch_warm_device (a.warm set); the plain ones carry no warm code.
template <typename TIn, typename T, int G, int K, int MINW, bool LH, bool WARM>
__global__ __launch_bounds__(64, MINW) void gjk_kernel(const gjkepa_gjk_args a) {
    static_assert(G >= 4, "the tetrahedron faces run on quads");
    using L_t = Lds<T, TIn, G, K, 0, 0>;
    extern __shared__ __align__(16) unsigned char smem[];
    const Grp<G> grp;
    L_t& L = *reinterpret_cast<L_t*>(smem + lds_stride<L_t, G>() * (grp.lane / G));
    const int gl = grp.gl;
    const TIn* verts = (const TIn*)a.verts;
    GK_GUARD(1, a.route_code);
    GK_STAMP_BEGIN();
    if (tier_empty(a.tally, a.route_code)) return;
    tally_begin();
    const int claim = pick_claim(a.tally, a.route_code, a.n_pairs, a.claim);
    auto body = [&](int64_t pair, const PairMeta& pm) {
        GK_STAMP(SG_ROUTE);
        Ctx<T, TIn, G, K, 0, 0, LH> c{L, grp};
        const int na = grp.uni(pm.na), nb = grp.uni(pm.nb);
        T o13[13];
#pragma unroll
        for (int i = 0; i < 13; ++i) o13[i] = T(0);
        uint8_t next = 0;
        if (na < 1 || nb < 1 || na > GJKEPA_MAX_HULL_VERTS || nb > GJKEPA_MAX_HULL_VERTS) {
            store_record<G, T>(a.out, pair, gl, o13, 0, 0, GJKEPA_STATUS_BAD_INPUT, 0u);
            if (WARM && gl < 4) a.warm[4 * pair + gl] = kStale;
        } else if (na > K * G || nb > K * G) {             // the smallest larger GJK tier that holds both
            next = (uint8_t)((na > nb ? na : nb) <= GJKEPA_G1_G * GJKEPA_G1_K ? GJKEPA_ROUTE_GJK1 : GJKEPA_ROUTE_GJK1 + 1);
        } else {
            c.na = na;
            c.nb = nb;
            const bool bad_in = load_hulls(c, verts + pm.oa, verts + pm.ob);
            GK_STAMP(SG_LOAD);
            if (bad_in) {
                store_record<G, T>(a.out, pair, gl, o13, 0, 0, GJKEPA_STATUS_BAD_INPUT, 0u);
                if (WARM && gl < 4) a.warm[4 * pair + gl] = kStale;
            } else {
                uint32_t kc[4];
                int gjk_it = 0;
                int r = PH_MISS;
                bool warm_hit = false;
                if constexpr (WARM) {    // a pair that missed last call runs the reference GJK again
                    if (a.warm[4 * pair] != kWarmMiss) warm_hit = warm_start(c, a.warm + 4 * pair, kc);
                }
                if (warm_hit) r = PH_HIT;
                else r = gjk_phase(c, kc, gjk_it, GJKEPA_AXIS_REJECT != 0);
                __builtin_amdgcn_wave_barrier();
                GK_STAMP(SG_CHK);
                if (WARM && gl < 4)     // this call's simplex seeds the next call; a miss mark; none for errors
                    a.warm[4 * pair + gl] = r == PH_HIT ? (gl == 0 ? kc[0] : gl == 1 ? kc[1] : gl == 2 ? kc[2] : kc[3])
                                          : (r == PH_MISS && gl == 0) ? kWarmMiss : kStale;
                if (r == PH_HIT) {
#pragma unroll
                    for (int j0 = 0; j0 < 6; j0 += G) {   // simplex codes, GJK iterations, no parked polytope
                        const int j = j0 + gl;
                        const uint32_t word = j == 0 ? kc[0] : j == 1 ? kc[1] : j == 2 ? kc[2] : j == 3 ? kc[3] : j == 4 ? (uint32_t)gjk_it : 0u;
                        if (j < 6) reinterpret_cast<uint32_t*>(a.out)[pair * (sizeof(T) == 8 ? 32 : 16) + j] = word;
                    }
                    next = (uint8_t)(GJKEPA_ROUTE_EPA0 + epa_tier_for(na > nb ? na : nb));
                } else if (r == PH_MISS) {
                    store_record<G, T>(a.out, pair, gl, o13, 0, 0, 0, 0u);
                } else if (certify<T>()) {                // fp32: GJK-phase error, recomputed in fp64
                    next = GJKEPA_ROUTE_REDO;
                } else {                                  // GJK-phase error (reference would STOP)
                    store_record<G, T>(a.out, pair, gl, o13, 1, 0, r, (uint32_t)(gjk_it & 0xff));
                }
            }
        }
        if (gl == 0) { a.route[pair] = next; tally_route(next); }
        __builtin_amdgcn_wave_barrier();
        GK_STAMP(SG_STORE);
    };
#if GJKEPA_GJK_META
    for_each_routed_pair<G, true>(grp, a.n_pairs, a.route, a.route_code, a.ctr, claim, false, body, a.pairs, a.hull_cnt,
                                  a.hull_off);
#else
    for_each_routed_pair<G>(grp, a.n_pairs, a.route, a.route_code, a.ctr, claim, false, [&](int64_t pair) {
        const int32_t ha = a.pairs[2 * pair], hb = a.pairs[2 * pair + 1];
        body(pair, PairMeta{a.hull_cnt[ha], a.hull_cnt[hb], a.hull_off[ha], a.hull_off[hb]});
    });
#endif
    GK_STAMP(SG_ROUTE);
    tally_end(a.tally);
    GK_STAMP_END();
}

DEV int contact_tier_for(int nmax) { return nmax <= GJKEPA_C0_G * GJKEPA_C0_K ? 0 : 1; }

// EPA kernel: the polytope loop for the pairs routed to this tier.  Depth, normal and the
// diagnostics are parked in their final record fields and the pair goes to its contact tier.  A
// polytope that outgrows the tier is routed to the next one (recomputed from the simplex codes).
// PR bit 0: park a polytope about to outgrow this tier (tier 3); bit 1: resume parked ones (tier 4).
template <typename TIn, typename T, int G, int K, int VC, int FC, int MINW, bool LH, int PR>
__global__ __launch_bounds__(64, MINW) void epa_kernel(const gjkepa_epa_args a) {
    using L_t = Lds<T, TIn, G, K, VC, FC>;
    extern __shared__ __align__(16) unsigned char smem[];
    const Grp<G> grp;
    L_t& L = *reinterpret_cast<L_t*>(smem + lds_stride<L_t, G>() * (grp.lane / G));
    const int gl = grp.gl;
    const TIn* verts = (const TIn*)a.verts;
    GK_GUARD(2, a.route_code);
    GK_STAMP_BEGIN();
    if (tier_empty(a.tally, a.route_code)) return;
    tally_begin();
    const int claim = pick_claim(a.tally, a.route_code, a.n_pairs, a.claim);
    for_each_routed_pair<G>(grp, a.n_pairs, a.route, a.route_code, a.ctr, claim, false, [&](int64_t pair) {
        GK_STAMP(SE_ROUTE);
        Ctx<T, TIn, G, K, VC, FC, LH> c{L, grp};
        const int32_t ha = a.pairs[2 * pair], hb = a.pairs[2 * pair + 1];
        c.na = grp.uni(a.hull_cnt[ha]);
        c.nb = grp.uni(a.hull_cnt[hb]);
        uint32_t* slot = reinterpret_cast<uint32_t*>(a.out) + pair * (sizeof(T) == 8 ? 32 : 16);
        uint32_t kc[4];
        kc[0] = slot[0]; kc[1] = slot[1]; kc[2] = slot[2]; kc[3] = slot[3];
        const uint32_t gjk_it = slot[4];
        load_hulls(c, verts + a.hull_off[ha], verts + a.hull_off[hb]);
        T depth;
        V3<T> n;
        uint32_t de = 0;
        GK_STAMP(SE_LOAD);
#ifdef GJKEPA_DIAG_GJK_ONLY   // timing ablation only (tools/build_variant.sh); never in the product build
        const int r = GJKEPA_STATUS_DEGENERATE;
        depth = 0; n = zero3<T>();
#else
        const uint32_t parked = (PR & 2) && a.park ? slot[5] : 0u;   // park slot + 1 (tiers 2, 3)
        uint32_t it_park = gjk_it;
        const ParkCtl pk{a.park, a.park_ctr, a.park_cap, gjk_it, slot};
        const bool can_park = (PR & 1) && a.park && a.next_code >= 0;
        const int r = (c.na > G * K || c.nb > G * K) ? ST_DEFER
                    : epa_phase(c, kc, depth, n, de, can_park, pk,
                                parked ? a.park + (size_t)(parked - 1) * GJKEPA_PARK_BYTES : nullptr, &it_park);
#endif
        __builtin_amdgcn_wave_barrier();
        const uint32_t diag = (gjk_it & 0xffu) | de;
        uint8_t next = 0;
        if ((r == ST_DEFER || r == ST_PARKED) && a.next_code >= 0) {   // next tier that holds the hulls
            next = (uint8_t)(GJKEPA_ROUTE_EPA0 + epa_tier_for(c.na > c.nb ? c.na : c.nb, a.next_code - GJKEPA_ROUTE_EPA0, VC));
        } else if (redo_status<T>(r, a.next_code < 0)) {   // fp32: not certified, recomputed in fp64
            next = GJKEPA_ROUTE_REDO;
        } else if (r == 0) {
            // park depth, normal (record fields 0..3) and diag; the contact tier finishes the record
            T* rec = reinterpret_cast<T*>(slot);
            if (gl < 4) rec[gl] = gl == 0 ? depth : gl == 1 ? n.x : gl == 2 ? n.y : n.z;
            if (gl == 4) slot[sizeof(T) == 8 ? 27 : 14] = diag;
            next = (uint8_t)(a.ct_base + contact_tier_for(c.na > c.nb ? c.na : c.nb));
        } else {                 // error status (last tier out of capacity: DEGENERATE): outputs zero, collision = 1
            T o13[13];
#pragma unroll
            for (int i = 0; i < 13; ++i) o13[i] = T(0);
            store_record<G, T>(a.out, pair, gl, o13, 1, 0, r == ST_DEFER ? GJKEPA_STATUS_DEGENERATE : r, diag);
        }
        if (gl == 0) { a.route[pair] = next; tally_route(next); }
        __builtin_amdgcn_wave_barrier();
        GK_STAMP(SE_STORE);
    });
    GK_STAMP(SE_ROUTE);
    tally_end(a.tally);
    GK_STAMP_END();
}

// Wave-uniform queue of the pairs routed to a launch, one work unit at a time (first unit
// static, later ones from the launch counter as in for_each_routed_pair).
struct PairQueue {
    const uint8_t* route;
    Units U;
    int64_t ch, p0;
    uint32_t* ctr;
    uint32_t next;
    uint64_t m;
    int code;
    bool done;
    DEV void load_chunk() {
        int len;
        U.range(ch, p0, len);
        const int64_t p = p0 + lane_id();
        m = __ballot(lane_id() < len && (int)route[p] == code);
    }
    DEV PairQueue(const uint8_t* route_, int64_t n, int small, int code_, uint32_t* ctr_)
        : route(route_), U(n, small), ch(blockIdx.x), p0(0), ctr(ctr_), next(0), m(0), code(code_), done(false) {
        if (ch < U.nunits) {
            if (lane_id() == 0) next = gridDim.x + atomicAdd(ctr, 1u);
            load_chunk();
        } else {
            done = true;
        }
    }
    // next pair in order, -1 when the launch has no more
    DEV int64_t pop() {
        while (!m && !done) {
            ch = (int64_t)__builtin_amdgcn_readfirstlane(next);
            if (ch >= U.nunits) { done = true; break; }
            if (lane_id() == 0) next = gridDim.x + atomicAdd(ctr, 1u);
            load_chunk();
        }
        if (!m) return -1;
        const int bit = (int)__builtin_ctzll(m);
        m &= m - 1;
        return p0 + bit;
    }
};

// EPA tier kernel with group refill: a group whose pair finished takes the next pair between
// two EPA iterations (once at least REFILL groups of the wave are idle), so a wave no longer
// runs every round to its slowest pair.  Results are the same as epa_kernel's.
template <typename TIn, typename T, int G, int K, int VC, int FC, int MINW, bool LH, int REFILL, int PR>
__global__ __launch_bounds__(64, MINW) void epa_kernel_refill(const gjkepa_epa_args a) {
    static_assert(!(PR & 2), "refill tiers do not resume parked polytopes");
    constexpr int R = (FC + G - 1) / G;
    constexpr int NG = 64 / G;
    using L_t = Lds<T, TIn, G, K, VC, FC>;
    extern __shared__ __align__(16) unsigned char smem[];
    const Grp<G> grp;
    L_t& L = *reinterpret_cast<L_t*>(smem + lds_stride<L_t, G>() * (grp.lane / G));
    const int gl = grp.gl;
    const int gid = grp.lane / G;
    const TIn* verts = (const TIn*)a.verts;
    GK_GUARD(3, a.route_code);
    GK_STAMP_BEGIN();
    if (tier_empty(a.tally, a.route_code)) return;
#if GJKEPA_E1_PRIO
    // EPA tier 1 serves the few polytopes that outgrew tier 0, restarted: on C2 it is the chain's tail,
    // beside the contact passes, so its waves take the SIMD's issue first
    if (a.route_code == GJKEPA_ROUTE_EPA0 + 1) __builtin_amdgcn_s_setprio(GJKEPA_E1_PRIO);
#endif
    tally_begin();
    PairQueue q(a.route, a.n_pairs, tail_unit<G, (2 * NG > 8 ? 2 * NG : 8)>(a.n_pairs), a.route_code, a.ctr);
    Ctx<T, TIn, G, K, VC, FC, LH> c{L, grp};
    EpaState<T, R> S;
    bool active = false;
    bool seeded = false;                 // iteration 1 set up by epa_seed: its support step is pending
    int64_t pair = 0;
    uint32_t gjk_it = 0;
    // final record / park / route for a pair whose EPA ended with status r
    auto finish = [&](int r, T depth, V3<T> n) {
        uint32_t* slot = reinterpret_cast<uint32_t*>(a.out) + pair * (sizeof(T) == 8 ? 32 : 16);
        const uint32_t diag = (gjk_it & 0xffu) | ((uint32_t)(S.iters & 0xff) << 8) | ((uint32_t)(S.nf & 0xffff) << 16);
        uint8_t next = 0;
        if ((r == ST_DEFER || r == ST_PARKED) && a.next_code >= 0) {
            next = (uint8_t)(GJKEPA_ROUTE_EPA0 + epa_tier_for(c.na > c.nb ? c.na : c.nb, a.next_code - GJKEPA_ROUTE_EPA0, VC));
        } else if (redo_status<T>(r, a.next_code < 0)) {   // fp32: not certified, recomputed in fp64
            next = GJKEPA_ROUTE_REDO;
        } else if (r == 0) {
            T* rec = reinterpret_cast<T*>(slot);
            if (gl < 4) rec[gl] = gl == 0 ? depth : gl == 1 ? n.x : gl == 2 ? n.y : n.z;
            if (gl == 4 % G) slot[sizeof(T) == 8 ? 27 : 14] = diag;
            next = (uint8_t)(a.ct_base + contact_tier_for(c.na > c.nb ? c.na : c.nb));
        } else {
            T o13[13];
#pragma unroll
            for (int i = 0; i < 13; ++i) o13[i] = T(0);
            store_record<G, T>(a.out, pair, gl, o13, 1, 0, r == ST_DEFER ? GJKEPA_STATUS_DEGENERATE : r, diag);
        }
        if (gl == 0) { a.route[pair] = next; tally_route(next); }
    };
    for (;;) {
        // refill idle groups (in group order) once enough of them are idle
        const uint64_t idle = __ballot(gl == 0 && !active);
        const int nidle = popc(idle);
        bool fresh = false;
        if (!q.done && (nidle >= REFILL || nidle == NG)) {
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                if ((idle >> (g * G)) & 1ull) {
                    const int64_t p = q.pop();
                    if (p >= 0 && gid == g) { pair = p; fresh = true; }
                }
            }
        }
        if (!__ballot(active || fresh)) break;
        GK_STAMP(SE_ROUTE);
        if (fresh) {
            const int32_t ha = a.pairs[2 * pair], hb = a.pairs[2 * pair + 1];
            c.na = a.hull_cnt[ha];
            c.nb = a.hull_cnt[hb];
            const uint32_t* slot = reinterpret_cast<const uint32_t*>(a.out) + pair * (sizeof(T) == 8 ? 32 : 16);
            uint32_t kc[4];
            kc[0] = slot[0]; kc[1] = slot[1]; kc[2] = slot[2]; kc[3] = slot[3];
            gjk_it = slot[4];
            load_hulls(c, verts + a.hull_off[ha], verts + a.hull_off[hb]);
            S.iters = 1; S.nf = 0;
            int r = ST_DEFER;
            seeded = false;
            if (c.na <= G * K && c.nb <= G * K) {
                const V3<T> s0 = decode_pt(c, kc[0]), s1 = decode_pt(c, kc[1]), s2 = decode_pt(c, kc[2]), s3 = decode_pt(c, kc[3]);
#if GJKEPA_EPA_SEED
                r = epa_seed(c, S, s0, s1, s2, s3);
                seeded = r == 0;
                if (r == ST_FALLBACK)
#endif
                    r = epa_begin(c, S, s0, s1, s2, s3);
            }
            __builtin_amdgcn_wave_barrier();
            active = r == 0;
            if (!active) finish(r, T(0), zero3<T>());
        }
        GK_STAMP(SE_LOAD);
        if (active) {
            // groups that closed an iteration (everything but the ones epa_seed just set up) take the
            // MINLOC / termination step; every continuing group then takes the support step together
            T depth = 0;
            V3<T> n = zero3<T>();
            int r = ST_CONT;
            if (!seeded) r = epa_close(c, S, depth, n);
            if constexpr ((PR & 1) != 0) {                 // park a polytope about to outgrow this tier
                if (r == ST_CONT && !seeded && a.park && a.next_code >= 0) {
                    const ParkCtl pk{a.park, a.park_ctr, a.park_cap, gjk_it,
                                     reinterpret_cast<uint32_t*>(a.out) + pair * (sizeof(T) == 8 ? 32 : 16)};
                    if (park_now(c, S, pk)) r = ST_PARKED;
                }
            }
            if (r == ST_CONT) r = epa_grow(c, S, seeded);
            seeded = false;
            __builtin_amdgcn_wave_barrier();
            if (r != ST_CONT) {
                finish(r, depth, n);
                active = false;
            }
        }
        GK_STAMP(SE_STORE);
    }
    GK_STAMP_END();
    tally_end(a.tally);
}

// One-wave query path (small batches, gjkepa_query's combined batches and its resident service):
// one wave per pair runs the sphere test, GJK, EPA and the contact features back to back, so a pair
// costs no tier chain.  Tuned for the latency of one pair on an otherwise idle wave: the hull
// register depth K (64K vertices per hull) is picked per pair from its larger hull, and EPA first
// runs with a small polytope (GJKEPA_Q_VCAP / GJKEPA_Q_FCAP: one face row per lane) and only on
// overflow restarts from the GJK simplex with the last EPA tier's polytope, as the tier chain's deferral
// does.  Same device functions as the tier kernels, so the records are the chain's bit for bit.
template <typename TIn, typename T, int K> using QLds = Lds<T, TIn, 64, K, GJKEPA_E5_VCAP, GJKEPA_E5_FCAP, true>;
template <typename TIn, typename T, int K> using QLdsS = Lds<T, TIn, 64, K, GJKEPA_Q_VCAP, GJKEPA_Q_FCAP, true>;
// RT: the record's field type (T, or float for the fp32 chain's fp64 redo).  Returns true when an fp32
// answer is not certified (certify<T>(): nothing stored; the caller recomputes the pair in fp64).
template <typename TIn, typename T, int K, typename RT = T>
DEV bool query_pair_k(unsigned char* smem, const Grp<64>& grp, const TIn* pa, const TIn* pb, int na, int nb,
                      int version, T tol_ff, void* out, int64_t pair) {
    using LB = QLds<TIn, T, K>;
    using LS = QLdsS<TIn, T, K>;
    static_assert(__builtin_offsetof(LB, u) == __builtin_offsetof(LS, u) && sizeof(LS) <= sizeof(LB),
                  "the two polytopes share the hull image");
    const int gl = grp.gl;
    Ctx<T, TIn, 64, K, GJKEPA_Q_VCAP, GJKEPA_Q_FCAP, 2> c{*reinterpret_cast<QLdsS<TIn, T, K>*>(smem), grp};
    T o13[13];
    RT o[13];
#pragma unroll
    for (int i = 0; i < 13; ++i) { o13[i] = T(0); o[i] = RT(0); }
    c.na = na;
    c.nb = nb;
    if (load_hulls(c, pa, pb)) {
        store_record<64, RT>(out, pair, gl, o, 0, 0, GJKEPA_STATUS_BAD_INPUT, 0u);
        return false;
    }
    uint32_t kc[4];
    int gjk_it = 0;
    int r = gjk_phase(c, kc, gjk_it, GJKEPA_AXIS_REJECT != 0);
    __builtin_amdgcn_wave_barrier();
    if (r == PH_MISS) {
        store_record<64, RT>(out, pair, gl, o, 0, 0, 0, 0u);
        return false;
    }
    if (r != PH_HIT) {                                   // GJK-phase error (reference would STOP)
        if (certify<T>()) return true;
        store_record<64, RT>(out, pair, gl, o, 1, 0, r, (uint32_t)(gjk_it & 0xff));
        return false;
    }
    T depth;
    V3<T> n;
    uint32_t de = 0;
    r = epa_phase(c, kc, depth, n, de);
    __builtin_amdgcn_wave_barrier();
    if (r == ST_DEFER) {                                 // small polytope full: the last tier's from the simplex
        Ctx<T, TIn, 64, K, GJKEPA_E5_VCAP, GJKEPA_E5_FCAP, 2> cb{*reinterpret_cast<QLds<TIn, T, K>*>(smem), grp};
        cb.na = na;
        cb.nb = nb;
        cb.vmax_a = c.vmax_a;
        cb.vmax_b = c.vmax_b;
        r = epa_phase(cb, kc, depth, n, de);
        __builtin_amdgcn_wave_barrier();
    }
    if (redo_status<T>(r, true)) return true;
    const uint32_t diag = ((uint32_t)gjk_it & 0xffu) | de;
    if (r != 0) {                                        // last tier out of capacity: DEGENERATE
        store_record<64, RT>(out, pair, gl, o, 1, 0, r == ST_DEFER ? GJKEPA_STATUS_DEGENERATE : r, diag);
        return false;
    }
    r = contact_phase(c, depth, n, version, tol_ff, o13);
    __builtin_amdgcn_wave_barrier();
    if (r < 0) {
#pragma unroll
        for (int i = 0; i < 13; ++i) o[i] = (RT)o13[i];
        store_record<64, RT>(out, pair, gl, o, 1, -r, 0, diag);
    } else {
        if (redo_status<T>(r, false)) return true;
        store_record<64, RT>(out, pair, gl, o, 1, 0, r, diag);
    }
    return false;
}

// one pair on this wave: hull depth from the larger hull; bad sizes answered BAD_INPUT.  An fp32 answer
// that is not certified is recomputed here in fp64 (records stay fp32): the redo launch's work, inline.
template <typename TIn, typename T, typename RT = T>
DEV void query_pair(unsigned char* smem, const Grp<64>& grp, const TIn* pa, const TIn* pb, int na, int nb,
                    int version, T tol_ff, void* out, int64_t pair) {
    const int nmax = na > nb ? na : nb;
    bool redo = false;
    if (na < 1 || nb < 1 || nmax > GJKEPA_MAX_HULL_VERTS) {
        RT o[13];
#pragma unroll
        for (int i = 0; i < 13; ++i) o[i] = RT(0);
        store_record<64, RT>(out, pair, grp.gl, o, 0, 0, GJKEPA_STATUS_BAD_INPUT, 0u);
    } else if (nmax <= 64) {
        redo = query_pair_k<TIn, T, 1, RT>(smem, grp, pa, pb, na, nb, version, tol_ff, out, pair);
    } else if (nmax <= 128) {
        redo = query_pair_k<TIn, T, 2, RT>(smem, grp, pa, pb, na, nb, version, tol_ff, out, pair);
    } else {
        redo = query_pair_k<TIn, T, GJKEPA_MAX_HULL_VERTS / 64, RT>(smem, grp, pa, pb, na, nb, version, tol_ff, out, pair);
    }
    if constexpr (certify<T>()) {
        if (redo) query_pair<TIn, double, RT>(smem, grp, pa, pb, na, nb, version, (double)tol_ff, out, pair);
    }
}

template <typename TIn, typename T>
__global__ __launch_bounds__(64, 1) void query_kernel(const gjkepa_epa_args a) {
    extern __shared__ __align__(16) unsigned char smem[];
    const Grp<64> grp;
    const int64_t pair = blockIdx.x;
    GK_GUARD(5, 0);
    if (pair >= a.n_pairs) return;
    const TIn* verts = (const TIn*)a.verts;
    const int32_t ha = a.pairs[2 * pair], hb = a.pairs[2 * pair + 1];
    const int na = grp.uni(a.hull_cnt[ha]), nb = grp.uni(a.hull_cnt[hb]);
    query_pair<TIn, T>(smem, grp, verts + a.hull_off[ha], verts + a.hull_off[hb], na, nb, a.version, (T)a.tol_ff,
                       a.out, pair);
}

// The fp32 chain's last launch: every pair routed GJKEPA_ROUTE_REDO (an fp32 answer that was not
// certified, or an fp32 error status) recomputed whole (GJK, EPA, contact features) in fp64 by one
// wave, stored as its fp32 record: the fp64 path's record rounded to fp32.  Few pairs (about 1 in
// 10^4 on C2 / C5), so one wave per pair and the sparse claim.
template <typename TIn>
__global__ __launch_bounds__(64, 1) void redo_kernel(const gjkepa_epa_args a) {
    extern __shared__ __align__(16) unsigned char smem[];
    const Grp<64> grp;
    const TIn* verts = (const TIn*)a.verts;
    GK_GUARD(7, a.route_code);
    if (tier_empty(a.tally, a.route_code)) return;
    const int claim = pick_claim(a.tally, a.route_code, a.n_pairs, a.claim);
    for_each_routed_pair<64>(grp, a.n_pairs, a.route, a.route_code, a.ctr, claim, false, [&](int64_t pair) {
        const int32_t ha = a.pairs[2 * pair], hb = a.pairs[2 * pair + 1];
        const int na = grp.uni(a.hull_cnt[ha]), nb = grp.uni(a.hull_cnt[hb]);
        query_pair<TIn, double, float>(smem, grp, verts + a.hull_off[ha], verts + a.hull_off[hb], na, nb, a.version,
                                       a.tol_ff, a.out, pair);
        if (grp.gl == 0) a.route[pair] = 0;
        __builtin_amdgcn_wave_barrier();
    });
}

// Resident query service (gjkepa_query, include/gjkepa.h): wave w serves request slot w of
// host-mapped memory.  It polls the slot's request line (one lane, system-scope acquire), answers a
// new request with query_pair straight from the slot (hull columns read once over the bus into
// LDS; the record stored into the slot) and publishes it with a system-scope release of `done`.
// Every wave leaves once the host sets its slot's stop word, or once no slot has been answered for
// idle_ticks (the first wave to see that marks the generation closing for the others and for the
// host, which relaunches the grid for the next request), so the grid always drains by itself.
DEV uint32_t uni32(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }

#if GK_IN(0)
__global__ __launch_bounds__(64, GJKEPA_SVC_MINW) void service_kernel(const gjkepa_svc_args a) {
    extern __shared__ __align__(16) unsigned char smem[];
    const Grp<64> grp;
    gjkepa_svc_slot* sl = a.slots + blockIdx.x;
    const uint32_t* hdr = &sl->req;
    uint32_t last = uni32(__hip_atomic_load(&sl->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    uint64_t seen = wall_clock64();
    const uint64_t born = seen;
    int empty = 0;
    for (;;) {
        // request line words 0, 1 (req, stop): relaxed system-scope reads (no cache invalidation
        // per poll); the acquire fence is paid once per new request
        uint32_t w = 0;
        if (grp.lane < 2) w = __hip_atomic_load(hdr + grp.lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint32_t req = uni32(w);
        const uint32_t stop = (uint32_t)__builtin_amdgcn_readlane((int)w, 1);
        if (req != last) {
            const uint64_t t_seen = wall_clock64();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // header and hulls are read after req
            GK_STAMP_BEGIN();
            uint32_t h = 0;
            if (grp.lane < 8) h = __hip_atomic_load(hdr + grp.lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            const int version = __builtin_amdgcn_readlane((int)h, 2);
            const int na = __builtin_amdgcn_readlane((int)h, 3), nb = __builtin_amdgcn_readlane((int)h, 4);
            const uint64_t tb = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)h, 6) |
                                ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)h, 7) << 32);
            const double tol = __builtin_bit_cast(double, tb);
            const int ca = na < 0 || na > GJKEPA_MAX_HULL_VERTS ? 0 : na;
            query_pair<double, double>(smem, grp, sl->v, sl->v + 3 * ca, na, nb, version, tol, sl->rec, 0);
            __builtin_amdgcn_wave_barrier();
            GK_STAMP_END();
            const uint64_t t_done = wall_clock64();
            if (grp.lane == 0) {
                sl->t_seen = t_seen;
                sl->t_done = t_done;
                __hip_atomic_store(&sl->done, req, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_fetch_max(&a.ctrl->last, t_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            last = req;
            seen = wall_clock64();
            empty = 0;
            continue;
        }
        if (stop) break;
        if (uni32(__hip_atomic_load(&a.ctrl->closing, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == a.gen) break;
        const uint64_t now = wall_clock64();
        const uint64_t g = __hip_atomic_load(&a.ctrl->last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t act = g > seen ? g : seen;
        // idle for idle_ticks, or resident for life_ticks (bounds how long work queued behind the grid
        // on a shared hardware queue can wait under steady traffic): drain; the next caller relaunches
        if ((now > act && now - act > a.idle_ticks) || (now > born && now - born > a.life_ticks)) {
            if (grp.lane == 0) {
                __hip_atomic_store(&a.ctrl->closing, a.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(a.host_closing, a.gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            break;
        }
        // a slot that just answered polls back to back; a quiet one about every microsecond, a
        // long-quiet one (callers take the lowest free slot) about every 8 microseconds
        if (++empty > 64) __builtin_amdgcn_s_sleep(32);
        if (empty > 4096) { __builtin_amdgcn_s_sleep(127); __builtin_amdgcn_s_sleep(127); }
    }
}
#endif  // GK_IN(0)

// Contact kernel: nearest points, contact point and contact type (:326-343) for every pair EPA
// finished, from the depth and normal it parked; writes the final record.
template <typename TIn, typename T, int G, int K, int MINW, bool LH>
__global__ __launch_bounds__(64, MINW) void contact_kernel(const gjkepa_epa_args a) {
    using L_t = Lds<T, TIn, G, K, 0, 1>;
    extern __shared__ __align__(16) unsigned char smem[];
    const Grp<G> grp;
    L_t& L = *reinterpret_cast<L_t*>(smem + lds_stride<L_t, G>() * (grp.lane / G));
    const int gl = grp.gl;
    const TIn* verts = (const TIn*)a.verts;
    GK_GUARD(4, a.route_code);
    GK_STAMP_BEGIN();
    if (tier_empty(a.tally, a.route_code)) return;
    tally_begin();
    const int claim = pick_claim(a.tally, a.route_code, a.n_pairs, a.claim);
    auto body = [&](int64_t pair, const PairMeta& pm) {
        GK_STAMP(SC_ROUTE);
        Ctx<T, TIn, G, K, 0, 1, LH> c{L, grp};
        c.na = grp.uni(pm.na);
        c.nb = grp.uni(pm.nb);
        const T* rec = reinterpret_cast<const T*>(a.out) + pair * 16;     // 16 T fields per record
        const T depth = rec[0];
        const V3<T> n = vmk<T>(rec[1], rec[2], rec[3]);
        const uint32_t diag = reinterpret_cast<const uint32_t*>(a.out)[pair * (sizeof(T) == 8 ? 32 : 16) + (sizeof(T) == 8 ? 27 : 14)];
        load_hulls(c, verts + pm.oa, verts + pm.ob);
        GK_STAMP(SC_LOAD);
        T o13[13];
#ifdef GJKEPA_DIAG_NO_CONTACT   // timing ablation only
        const int r = -1;
#pragma unroll
        for (int i = 0; i < 13; ++i) o13[i] = T(0);
#else
        const int r = contact_phase(c, depth, n, a.version, (T)a.tol_ff, o13);
#endif
        __builtin_amdgcn_wave_barrier();
        uint8_t next = 0;
        if (r < 0) {
            store_record<G, T>(a.out, pair, gl, o13, 1, -r, 0, diag);
        } else if (redo_status<T>(r, false)) {   // fp32: contact-phase error, recomputed in fp64
            next = GJKEPA_ROUTE_REDO;
        } else {                 // error status: outputs zero, collision = 1
#pragma unroll
            for (int i = 0; i < 13; ++i) o13[i] = T(0);
            store_record<G, T>(a.out, pair, gl, o13, 1, 0, r, diag);
        }
        if (gl == 0) { a.route[pair] = next; if (next) tally_route(next); }
        __builtin_amdgcn_wave_barrier();
        GK_STAMP(SC_STORE);
    };
#if GJKEPA_CONTACT_META
    for_each_routed_pair<G, true>(grp, a.n_pairs, a.route, a.route_code, a.ctr, claim, a.grid == GJKEPA_GRID_UNITS, body,
                                  a.pairs, a.hull_cnt, a.hull_off);
#else
    for_each_routed_pair<G>(grp, a.n_pairs, a.route, a.route_code, a.ctr, claim, a.grid == GJKEPA_GRID_UNITS, [&](int64_t pair) {
        const int32_t ha = a.pairs[2 * pair], hb = a.pairs[2 * pair + 1];
        body(pair, PairMeta{a.hull_cnt[ha], a.hull_cnt[hb], a.hull_off[ha], a.hull_off[hb]});
    });
#endif
    GK_STAMP(SC_ROUTE);
    tally_end(a.tally);
    GK_STAMP_END();
}

// Counter / tally reset at the head of a chain (one wave; the chain's first node).
#if GK_IN(0)
__global__ __launch_bounds__(64) void ws_reset_kernel(uint32_t* ws, int n32, uint32_t guard) {
#ifdef GJKEPA_DIAG_GUARD
    const uint32_t g_ = gjkepa_fold(gjkepa_mix(gjkepa_mix(0x72ull, (uint64_t)ws), (uint64_t)(int64_t)n32));
    if (g_ != guard) { guard_report(6u << 8, guard, g_); return; }
#endif
    (void)guard;
    for (int i = (int)threadIdx.x; i < n32; i += 64) ws[i] = 0u;
}
#endif  // GK_IN(0)

}  // namespace gk

// ---------------------------------------------------------------- host-side launch table
// The product build compiles this file once per part (Makefile: -DGK_PART=p), each object instantiating
// only its own kernels so the parts compile in parallel: 0 = chain reset, query service and the launch
// dispatchers, 1 = one-wave query path (fp64 compute), 2 = GJK tiers, 3 = contact tiers, 4 + t = EPA
// tier t, 10 = one-wave query path (fp32 compute), 11 = fp32 redo.
// Without GK_PART (diagnostic variant builds) one object holds every part.  The non-template kernels
// (chain reset, query service) are defined in part 0 only.
// the one-wave query path in fp32 compute (part 10)
hipError_t gk_launch_query_f32(int vert_dtype, const gjkepa_epa_args& a, hipStream_t s);
// EPA tier t's launcher, defined in part 4 + t
#define GK_EPA_DECL(t) hipError_t gk_launch_epa_##t(int vert_dtype, int precision, const gjkepa_epa_args& a, hipStream_t s);
GK_EPA_DECL(0) GK_EPA_DECL(1) GK_EPA_DECL(2) GK_EPA_DECL(3) GK_EPA_DECL(4) GK_EPA_DECL(5)
static_assert(GJKEPA_EPA_TIERS == 6, "one launcher per EPA tier");
namespace {

// no more workgroups than the launch has work units: 64-pair chunks, or one wave-round (64 / G
// pairs) each for a small batch (the kernels' tail_unit)
template <int G> int grid_cap(int64_t n_pairs, int grid) {
    const int64_t chunks = (n_pairs + 63) / 64, rounds = (n_pairs + 64 / G - 1) / (64 / G);
    const int64_t want = rounds <= (int64_t)grid * 8 / (64 / G) ? rounds : chunks;
    return (int)(want < 1 ? 1 : want < grid ? want : grid);
}
template <typename K_t> int grid_for(K_t kfn, size_t lds, int num_cus, int grid) {
    if (grid > 0) return grid;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, 64, lds) != hipSuccess || per_cu < 1) per_cu = 1;
    return per_cu * num_cus;
}

#if GK_IN(2)
template <typename TIn, typename T, int G, int K, int MINW, bool LH>
hipError_t launch_gjk(const gjkepa_gjk_args& a, hipStream_t s) {
    auto kfn = a.warm ? gk::gjk_kernel<TIn, T, G, K, MINW, LH, true> : gk::gjk_kernel<TIn, T, G, K, MINW, LH, false>;
    constexpr int GPW = 64 / G;
    const size_t lds = gk::lds_stride<gk::Lds<T, TIn, G, K, 0, 0>, G>() * GPW;
    int grid = grid_for(kfn, lds, a.num_cus, a.grid);
    grid = grid_cap<G>(a.n_pairs, grid);
    hipLaunchKernelGGL(kfn, dim3(grid), dim3(64), lds, s, a);
    return hipGetLastError();
}
template <typename TIn, typename T>
hipError_t gjk_any(int tier, const gjkepa_gjk_args& a, hipStream_t s) {
    static_assert(GJKEPA_GJK_TIERS == 3 && GJKEPA_G2_G * GJKEPA_G2_K >= GJKEPA_MAX_HULL_VERTS, "the last GJK tier holds every hull");
    return tier == 0 ? launch_gjk<TIn, T, GJKEPA_G0_G, GJKEPA_G0_K, GJKEPA_G0_MINW, (GJKEPA_G0_LH != 0)>(a, s)
         : tier == 1 ? launch_gjk<TIn, T, GJKEPA_G1_G, GJKEPA_G1_K, GJKEPA_G1_MINW, (GJKEPA_G1_LH != 0)>(a, s)
                     : launch_gjk<TIn, T, GJKEPA_G2_G, GJKEPA_G2_K, GJKEPA_G2_MINW, (GJKEPA_G2_LH != 0)>(a, s);
}
#endif

template <typename TIn, typename T, int G, int K, int VC, int FC, int MINW, bool LH, int REFILL = 0, int PR = 0>
hipError_t launch_epa(const gjkepa_epa_args& a, hipStream_t s) {
    auto kfn = [] {
        if constexpr (REFILL > 0) return gk::epa_kernel_refill<TIn, T, G, K, VC, FC, MINW, LH, REFILL, PR>;
        else return gk::epa_kernel<TIn, T, G, K, VC, FC, MINW, LH, PR>;
    }();
    constexpr int GPW = 64 / G;
    const size_t lds = gk::lds_stride<gk::Lds<T, TIn, G, K, VC, FC>, G>() * GPW;
    int grid = grid_for(kfn, lds, a.num_cus, a.grid);
    grid = grid_cap<G>(a.n_pairs, grid);
    hipLaunchKernelGGL(kfn, dim3(grid), dim3(64), lds, s, a);
    return hipGetLastError();
}

#define EPA_ARGS(t) GJKEPA_E##t##_G, GJKEPA_E##t##_K, GJKEPA_E##t##_VCAP, GJKEPA_E##t##_FCAP, GJKEPA_E##t##_MINW, \
                    (GJKEPA_E##t##_LH != 0)

#if GK_IN(3)
template <typename TIn, typename T, int G, int K, int MINW, bool LH>
hipError_t launch_contact(const gjkepa_epa_args& a, hipStream_t s) {
    auto kfn = gk::contact_kernel<TIn, T, G, K, MINW, LH>;
    constexpr int GPW = 64 / G;
    const size_t lds = gk::lds_stride<gk::Lds<T, TIn, G, K, 0, 1>, G>() * GPW;
    int grid;
    if (a.grid == GJKEPA_GRID_UNITS) {                  // one workgroup per 64-pair chunk (dense launches)
        grid = (int)((a.n_pairs + 63) / 64);
    } else {
        grid = grid_cap<G>(a.n_pairs, grid_for(kfn, lds, a.num_cus, a.grid));
    }
    hipLaunchKernelGGL(kfn, dim3(grid), dim3(64), lds, s, a);
    return hipGetLastError();
}
// tier 0: small hulls; 1: large hulls
template <typename TIn, typename T>
hipError_t contact_any(int tier, const gjkepa_epa_args& a, hipStream_t s) {
    if (tier == 0)
        return launch_contact<TIn, T, GJKEPA_C0_G, GJKEPA_C0_K, GJKEPA_C0_MINW, (GJKEPA_C0_LH != 0)>(a, s);
    return launch_contact<TIn, T, GJKEPA_C1_G, GJKEPA_C1_K, GJKEPA_C1_MINW, (GJKEPA_C1_LH != 0)>(a, s);
}
#endif

// EPA tier t over the four (storage, compute) combinations
#define GK_EPA_DEF(t, ...)                                                                                        \
    hipError_t gk_launch_epa_##t(int vert_dtype, int precision, const gjkepa_epa_args& a, hipStream_t s) {          \
        if (vert_dtype == GJKEPA_DTYPE_F32)                                                                         \
            return precision == GJKEPA_PREC_F64 ? launch_epa<float, double, __VA_ARGS__>(a, s)                      \
                                                : launch_epa<float, float, __VA_ARGS__>(a, s);                      \
        return precision == GJKEPA_PREC_F64 ? launch_epa<double, double, __VA_ARGS__>(a, s)                        \
                                            : launch_epa<double, float, __VA_ARGS__>(a, s);                         \
    }

}  // namespace

#if GK_IN(4)
GK_EPA_DEF(0, EPA_ARGS(0), GJKEPA_E0_REFILL)
#endif
#if GK_IN(5)
GK_EPA_DEF(1, EPA_ARGS(1), GJKEPA_E1_REFILL)
#endif
#if GK_IN(6)
GK_EPA_DEF(2, EPA_ARGS(2), GJKEPA_E2_REFILL, GJKEPA_PARK ? 1 : 0)     // parks
#endif
#if GK_IN(7)
GK_EPA_DEF(3, EPA_ARGS(3), 0, GJKEPA_PARK ? 1 : 0)                    // parks
#endif
#if GK_IN(8)
GK_EPA_DEF(4, EPA_ARGS(4), 0, GJKEPA_PARK ? 2 : 0)                    // resumes
#endif
#if GK_IN(9)
GK_EPA_DEF(5, EPA_ARGS(5))
#endif

#if GK_IN(0)
hipError_t gjkepa_launch_ws_reset(uint32_t* ws, int n32, hipStream_t s) {
    const uint32_t guard = gjkepa_fold(gjkepa_mix(gjkepa_mix(0x72ull, (uint64_t)ws), (uint64_t)(int64_t)n32));
    hipLaunchKernelGGL(gk::ws_reset_kernel, dim3(1), dim3(64), 0, s, ws, n32, guard);
    return hipGetLastError();
}
#ifdef GJKEPA_DIAG_GUARD
// diagnostic build only: the argument-guard report ([0] mismatches, [1] kernel id << 8 | route
// code of the last, [2] expected and [3] recomputed checksum), optionally cleared
extern "C" int gjkepa_diag_guard(uint32_t* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(gk::g_guard), sizeof(gk::g_guard)) != hipSuccess) return -1;
    if (reset) {
        uint32_t z[8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(gk::g_guard), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 8;
}
#endif

#ifdef GJKEPA_DIAG_STAMPS
// diagnostic build only: read (and optionally clear) the phase stamp totals
extern "C" int gjkepa_diag_stamps(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(gk::g_stamps), sizeof(gk::g_stamps)) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[gk::kStamps] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(gk::g_stamps), z, sizeof(z)) != hipSuccess) return -1;
    }
    return gk::kStamps;
}
#endif

hipError_t gjkepa_launch_service(const gjkepa_svc_args& a, int n_slots, hipStream_t s) {
    using L_t = gk::QLds<double, double, GJKEPA_MAX_HULL_VERTS / 64>;
    hipLaunchKernelGGL(gk::service_kernel, dim3((unsigned)n_slots), dim3(64), sizeof(L_t), s, a);
    return hipGetLastError();
}

hipError_t gjkepa_launch_epa(int tier, int vert_dtype, int precision, const gjkepa_epa_args& a, hipStream_t s) {
    switch (tier) {
        case 0: return gk_launch_epa_0(vert_dtype, precision, a, s);
        case 1: return gk_launch_epa_1(vert_dtype, precision, a, s);
        case 2: return gk_launch_epa_2(vert_dtype, precision, a, s);
        case 3: return gk_launch_epa_3(vert_dtype, precision, a, s);
        case 4: return gk_launch_epa_4(vert_dtype, precision, a, s);
        default: return gk_launch_epa_5(vert_dtype, precision, a, s);
    }
}
#endif

#if GK_IN(1) || GK_IN(10)
template <typename TIn, typename T> hipError_t launch_query(const gjkepa_epa_args& a, hipStream_t s) {
    // an fp32 query recomputes an uncertified pair in fp64 in place: room for the fp64 image
    using L_t = gk::QLds<TIn, double, GJKEPA_MAX_HULL_VERTS / 64>;
    auto kfn = gk::query_kernel<TIn, T>;
    hipLaunchKernelGGL(kfn, dim3((unsigned)a.n_pairs), dim3(64), sizeof(L_t), s, a);
    return hipGetLastError();
}
#endif
#if GK_IN(10)
hipError_t gk_launch_query_f32(int vert_dtype, const gjkepa_epa_args& a, hipStream_t s) {
    return vert_dtype == GJKEPA_DTYPE_F32 ? launch_query<float, float>(a, s) : launch_query<double, float>(a, s);
}
#endif
#if GK_IN(11)
template <typename TIn> hipError_t launch_redo(const gjkepa_epa_args& a, hipStream_t s) {
    using L_t = gk::QLds<TIn, double, GJKEPA_MAX_HULL_VERTS / 64>;
    auto kfn = gk::redo_kernel<TIn>;
    const int grid = grid_cap<64>(a.n_pairs, grid_for(kfn, sizeof(L_t), a.num_cus, a.grid));
    hipLaunchKernelGGL(kfn, dim3(grid), dim3(64), sizeof(L_t), s, a);
    return hipGetLastError();
}
hipError_t gjkepa_launch_redo(int vert_dtype, const gjkepa_epa_args& a, hipStream_t s) {
    return vert_dtype == GJKEPA_DTYPE_F32 ? launch_redo<float>(a, s) : launch_redo<double>(a, s);
}
#endif
#if GK_IN(1)
hipError_t gjkepa_launch_query(int vert_dtype, int precision, const gjkepa_epa_args& a, hipStream_t s) {
    if (precision != GJKEPA_PREC_F64) return gk_launch_query_f32(vert_dtype, a, s);
    return vert_dtype == GJKEPA_DTYPE_F32 ? launch_query<float, double>(a, s) : launch_query<double, double>(a, s);
}
#endif

#if GK_IN(2)
hipError_t gjkepa_launch_gjk(int tier, int vert_dtype, int precision, const gjkepa_gjk_args& a, hipStream_t s) {
    if (vert_dtype == GJKEPA_DTYPE_F32)
        return precision == GJKEPA_PREC_F64 ? gjk_any<float, double>(tier, a, s) : gjk_any<float, float>(tier, a, s);
    return precision == GJKEPA_PREC_F64 ? gjk_any<double, double>(tier, a, s) : gjk_any<double, float>(tier, a, s);
}

#endif

#if GK_IN(3)
hipError_t gjkepa_launch_contact(int tier, int vert_dtype, int precision, const gjkepa_epa_args& a, hipStream_t s) {
    if (vert_dtype == GJKEPA_DTYPE_F32)
        return precision == GJKEPA_PREC_F64 ? contact_any<float, double>(tier, a, s) : contact_any<float, float>(tier, a, s);
    return precision == GJKEPA_PREC_F64 ? contact_any<double, double>(tier, a, s) : contact_any<double, float>(tier, a, s);
}
#endif
