// gjkepa_kernel.h — host-side interface of the GJK and EPA kernels (internal, not the C-ABI).
//
// Three phases, each in tiers.  GJK tier 0 takes every pair (hulls up to G0*K0 vertices; larger
// hulls go to GJK tier 1).  Misses and errors are final after GJK; each hit is routed to the
// smallest EPA tier whose hull capacity holds it.  EPA parks depth and normal in the pair's
// record and routes it to the contact tier for its hull size (nearest points, contact point,
// contact type), which writes the final record.  An EPA tier that runs out of polytope capacity
// (VCAP vertices / FCAP faces) routes the pair to the next EPA tier, which
// recomputes it from the same GJK simplex; the last EPA tier holds the worst case the reference
// allows (6 + 2*99 EPA points, 2V-4 faces), so it never defers.  Which tier answered never
// changes a result.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

// GJK tiers: G lanes per pair (64/G pairs per wave), K vertices per lane per hull (hull <= G*K)
#ifndef GJKEPA_G0_G
#define GJKEPA_G0_G 4           // 16 pairs per wave: GJK is VALU-bound on group-uniform work
#endif
#ifndef GJKEPA_G0_K
#define GJKEPA_G0_K 8
#endif
#ifndef GJKEPA_G0_MINW
#define GJKEPA_G0_MINW 2        // __launch_bounds__ minimum waves per SIMD (caps VGPRs at 512/MINW)
#endif
// GJK tier 1: hulls of 33-128 vertices (C5, a quarter of C4); GJK tier 2: up to 256.  A pair goes to
// the smallest tier that holds its larger hull.  Tier 1 runs four pairs per wave at 16 lanes x 8
// vertices (K = 8 takes the fp32-screened support scan), despite 75 spilled VGPRs at three waves:
// A/B r6 (2 rounds, profiles/r06/ab_g1_tiers.txt) against 32 x 4 C4 45.76 -> 46.08, C5 25.59 -> 25.97;
// 64 x 2 lost (C4 -1.2%, C5 -2.9%)
#ifndef GJKEPA_G1_G
#define GJKEPA_G1_G 16
#endif
#ifndef GJKEPA_G1_K
#define GJKEPA_G1_K 8
#endif
#ifndef GJKEPA_G1_MINW
#define GJKEPA_G1_MINW 3
#endif
#ifndef GJKEPA_G2_G
#define GJKEPA_G2_G 32          // two pairs per wave (A/B on C4: 26.3 vs 25.5M queries/s at 64 lanes x 4)
#endif
#ifndef GJKEPA_G2_K
#define GJKEPA_G2_K 8
#endif
#ifndef GJKEPA_G2_MINW
#define GJKEPA_G2_MINW 3           // LDS hull frees the 96 VGPRs of register copies: three waves per SIMD
#endif
// EPA tiers: G, K as above, EPA polytope capacity VCAP vertices / FCAP faces
#ifndef GJKEPA_E0_G
#define GJKEPA_E0_G 16
#endif
#ifndef GJKEPA_E0_K
#define GJKEPA_E0_K 2
#endif
#ifndef GJKEPA_E0_VCAP
#define GJKEPA_E0_VCAP 40
#endif
#ifndef GJKEPA_E0_FCAP
#define GJKEPA_E0_FCAP 64
#endif
#ifndef GJKEPA_E0_MINW
#define GJKEPA_E0_MINW 3        // with GJKEPA_E0_LH: 168 VGPRs; with GJKEPA_EPA_HPACK the LDS holds 12 waves/CU
#endif
#ifndef GJKEPA_E0_REFILL
#define GJKEPA_E0_REFILL 2      // refill a wave's groups once this many are idle (0: per-round kernel)
#endif
#ifndef GJKEPA_E1_G
#define GJKEPA_E1_G 32
#endif
#ifndef GJKEPA_E1_K
#define GJKEPA_E1_K 1
#endif
#ifndef GJKEPA_E1_VCAP
#define GJKEPA_E1_VCAP 72
#endif
#ifndef GJKEPA_E1_FCAP
#define GJKEPA_E1_FCAP 128
#endif
#ifndef GJKEPA_E1_REFILL
#define GJKEPA_E1_REFILL 1      // tier 1 serves few, long pairs: refill a group as soon as it idles
#endif
#ifndef GJKEPA_E1_MINW
#define GJKEPA_E1_MINW 2
#endif
#ifndef GJKEPA_E2_G
#define GJKEPA_E2_G 32          // two pairs per wave for hulls of 33-128 vertices (configs C4, C5)
#endif
#ifndef GJKEPA_E2_K
#define GJKEPA_E2_K 4
#endif
#ifndef GJKEPA_E2_VCAP
#define GJKEPA_E2_VCAP 72       // polytope overflow goes on to tier 3 (A/B: 104 / 208 spills at 2 waves)
#endif
#ifndef GJKEPA_E2_FCAP
#define GJKEPA_E2_FCAP 128
#endif
#ifndef GJKEPA_E2_MINW
#define GJKEPA_E2_MINW 2
#endif
#ifndef GJKEPA_E2_REFILL
#define GJKEPA_E2_REFILL 1      // C4 EPA tier 2 14.5 -> 13.7 ms, C5 40.5 -> 40.0 ms
#endif
// EPA tier 3: hulls of 129-256 vertices, first with a small polytope (one face row per lane, four
// waves per SIMD); the ~16% of C4's large-hull pairs whose polytope outgrows it restart in tier 4
#ifndef GJKEPA_E3_G
#define GJKEPA_E3_G 64
#endif
#ifndef GJKEPA_E3_K
#define GJKEPA_E3_K 4
#endif
#ifndef GJKEPA_E3_VCAP
#define GJKEPA_E3_VCAP 40
#endif
#ifndef GJKEPA_E3_FCAP
#define GJKEPA_E3_FCAP 64
#endif
#ifndef GJKEPA_E3_MINW
#define GJKEPA_E3_MINW 4
#endif
#ifndef GJKEPA_E4_G
#define GJKEPA_E4_G 64
#endif
#ifndef GJKEPA_E4_K
#define GJKEPA_E4_K 4
#endif
#ifndef GJKEPA_E4_VCAP
#define GJKEPA_E4_VCAP 104
#endif
#ifndef GJKEPA_E4_FCAP
#define GJKEPA_E4_FCAP 208
#endif
#ifndef GJKEPA_E4_MINW
#define GJKEPA_E4_MINW 2
#endif
#ifndef GJKEPA_E5_G
#define GJKEPA_E5_G 64
#endif
#ifndef GJKEPA_E5_K
#define GJKEPA_E5_K 4
#endif
#ifndef GJKEPA_E5_VCAP
#define GJKEPA_E5_VCAP 208
#endif
#ifndef GJKEPA_E5_FCAP
#define GJKEPA_E5_FCAP 416
#endif
#ifndef GJKEPA_E5_MINW
#define GJKEPA_E5_MINW 1
#endif
// one-wave query path (query_kernel, the resident query service): EPA's first polytope
#ifndef GJKEPA_Q_VCAP
#define GJKEPA_Q_VCAP 40
#endif
#ifndef GJKEPA_Q_FCAP
#define GJKEPA_Q_FCAP 64
#endif
// contact-feature tiers (nearest points, contact point, contact type): G, K as above
#ifndef GJKEPA_C0_G
#define GJKEPA_C0_G 8
#endif
#ifndef GJKEPA_C0_K
#define GJKEPA_C0_K 4
#endif
#ifndef GJKEPA_C0_MINW
#define GJKEPA_C0_MINW 3        // A/B r5 (2 rounds): C2 162.7 -> 163.6 M/s, C4 / C5 unchanged (LDS allows 10 waves/CU)
#endif
#ifndef GJKEPA_C1_G
#define GJKEPA_C1_G 64
#endif
#ifndef GJKEPA_C1_K
#define GJKEPA_C1_K 4
#endif
#ifndef GJKEPA_C1_MINW
#define GJKEPA_C1_MINW 3        // A/B r5 (2 rounds): 2 -> 3 waves/SIMD C4 39.9 -> 40.6, C5 23.1 -> 23.5 M/s, C2 unchanged
#endif
#ifndef GJKEPA_EPA_SEED
#define GJKEPA_EPA_SEED 1           // refill tiers: a fresh pair's iteration 1 joins the common support step (epa_seed)
#endif
#ifndef GJKEPA_GJK_META
#define GJKEPA_GJK_META 1           // GJK tiers load every routed pair's hull counts / offsets once per chunk (0: per pair, A/B)
#endif
#ifndef GJKEPA_CONTACT_META
#define GJKEPA_CONTACT_META 1       // contact tiers load every routed pair's hull counts / offsets once per chunk (0: per pair, A/B)
#endif
#ifndef GJKEPA_E1_PRIO
#define GJKEPA_E1_PRIO 2            // wave priority (s_setprio) of EPA tier 1's waves (0: default; A/B r5: C2 +0.2%, C5 +0.6%)
#endif
#ifndef GJKEPA_HORIZON_W16
#define GJKEPA_HORIZON_W16 1        // horizon twin test on 16-bit edge windows (0: byte compares; A/B r5: C2 +0.6%, C4 +1.6%, C5 +2.2%)
#endif
#ifndef GJKEPA_SCREEN_SINGLE
#define GJKEPA_SCREEN_SINGLE 1      // fp32 support screen: a group's single candidate is the answer, no fp64 dot (A/B r5: C4 +1.0%, C2 +0.2%)
#endif
#ifndef GJKEPA_EPA_HPACK
#define GJKEPA_EPA_HPACK 1          // one-word horizon edges, FC / 2 of them, where keys fit 16 bits (0: A/B r5 C2 157.3 -> 162.7)
#endif
#ifndef GJKEPA_PAD_V0
#define GJKEPA_PAD_V0 1             // hull slots past the count hold vertex 0 again; support scans skip the mask
                                    // (A/B r6, 3 rounds: C2 +1.1%, C4 +1.6%, C5 +1.9%; 0: masked)
#endif
#ifndef GJKEPA_EMPTY_INF
#define GJKEPA_EMPTY_INF 1          // free polytope face slots carry a -inf distance; MINLOC without validity masks
                                    // (A/B r6, 3 rounds: C2 +3.4%, C4 +1.7%, C5 +2.7%; 0: masked scan)
#endif
#ifndef GJKEPA_DOTS_FMAX
#define GJKEPA_DOTS_FMAX 1          // support_dots' per-lane maximum on v_max_f64 (0: compare + selects, A/B)
#endif
#ifndef GJKEPA_EPA_PLACE
#define GJKEPA_EPA_PLACE 1          // EPA new faces built on the lane that owns their slot (0: staged in LDS, A/B)
#endif
#ifndef GJKEPA_LDS_SKEW
#define GJKEPA_LDS_SKEW 1           // pad LDS coordinate columns and skew group images across banks (0: A/B off)
#endif
#ifndef GJKEPA_HULL_AOS
#define GJKEPA_HULL_AOS 0           // 1: LDS hull copy as one (x, y, z, 0) 16-byte record per vertex (A/B: EPA tier 0 +13%, GJK +7%: bank conflicts)
#endif
#ifndef GJKEPA_SCREEN_MIN_K
#define GJKEPA_SCREEN_MIN_K 8       // fp32-screened support mapping in tiers with K >= this (fp64 compute,
#endif                              // fp32 storage); 0 = off
#ifndef GJKEPA_AXIS_REJECT
#define GJKEPA_AXIS_REJECT 0        // diagnostic A/B only, never the product build: GJK answers "miss"
                                    // when the centre axis separates the hulls.  Not parity-safe: the
                                    // reference's tetra loop reports hits on separated hulls through
                                    // isPointInSimplex's on-face branch (:1246-1256)
#endif
// Per tier: hull vertices read from the group's LDS copy (1) instead of held in registers (0).
// The LDS form frees 6K VGPRs per lane: EPA tier 0 then fits three waves per SIMD (168 VGPRs)
// without spills (C2: EPA tier 0 6.10 -> 5.26 ms); GJK tier 0 is +1% either way.  Measured and
// kept in registers: EPA tiers 1 / 2 at 3 waves (C2 tier 1 +8%, C5 tier 2 +15% slower: K = 4 support
// sums read 24 LDS values per step), contact tier 1 at 2 waves (+14%).
#ifndef GJKEPA_G0_LH
#define GJKEPA_G0_LH 1
#endif
#ifndef GJKEPA_G1_LH
#define GJKEPA_G1_LH 1
#endif
#ifndef GJKEPA_G2_LH
#define GJKEPA_G2_LH 1             // A/B r4 (2 rounds, with MINW 3): C4 39.07 -> 39.54, C2 -0.2%, C5 -0.4%
#endif
#ifndef GJKEPA_E0_LH
#define GJKEPA_E0_LH 1
#endif
#ifndef GJKEPA_E1_LH
#define GJKEPA_E1_LH 0
#endif
#ifndef GJKEPA_E2_LH
#define GJKEPA_E2_LH 0
#endif
#ifndef GJKEPA_E3_LH
#define GJKEPA_E3_LH 1
#endif
#ifndef GJKEPA_E4_LH
#define GJKEPA_E4_LH 1             // 152 VGPRs: LDS-bound at 11 waves/CU (C4: EPA tier 3 100.4 -> 90.6 ms)
#endif
#ifndef GJKEPA_E5_LH
#define GJKEPA_E5_LH 0
#endif
#ifndef GJKEPA_C0_LH
#define GJKEPA_C0_LH 1             // contact features read the hull from LDS (A/B r3: C4 +5% with the one-pass dots)
#endif
#ifndef GJKEPA_C1_LH
#define GJKEPA_C1_LH 1
#endif
#ifndef GJKEPA_CONTACT_OVERLAP
#define GJKEPA_CONTACT_OVERLAP 1    // each EPA tier's contact pass on a second stream, overlapping the later EPA tiers
#endif
#define GJKEPA_GJK_TIERS 3
#define GJKEPA_EPA_TIERS 6
#define GJKEPA_CONTACT_TIERS 2

// workspace: a 512-byte header of per-launch chunk counters, route tallies and the park counter, then
// one route byte per pair, then park slots (gjkepa_capi.cpp, gjkepa_workspace_bytes)
#define GJKEPA_WS_COUNTERS 40   // uint32 counters at the head of the workspace (one per launch of a chain)
// then GJKEPA_WS_TALLY uint32 route tallies (indexed by route code): every kernel adds the pairs it
// routes on; a launch whose own tally is at least 1/16 of the batch claims single chunks (dense),
// otherwise runs of `claim` chunks (sparse scan)
#define GJKEPA_WS_TALLY 48
// route byte per pair (workspace): which kernel owns the pair next
#define GJKEPA_ROUTE_DONE 0
#define GJKEPA_ROUTE_GJK1 1         // + GJK tier - 1 (tiers 1, 2)
#define GJKEPA_ROUTE_EPA0 0x10      // + EPA tier
#define GJKEPA_ROUTE_CT0 0x20       // + contact tier
// with GJKEPA_CONTACT_OVERLAP, the pairs EPA tier t finishes go to contact tier c under code CT(t) + c
#define GJKEPA_ROUTE_CT(t) (GJKEPA_ROUTE_CT0 + 2 * (t))
// fp32 compute: pairs whose fp32 answer is not certified (EPA's MINLOC distance dropped or its final
// support gap is open, or an fp32 error status) are recomputed whole in fp64 by the redo launch at
// the end of the chain (gjkepa_kernel.hip "fp32 certificate")
#define GJKEPA_ROUTE_REDO 0x2E

// Polytope parking.  EPA tiers 2 and 3 hand a pair whose polytope is about to outgrow them to tier 4
// with its polytope instead of its GJK simplex: the state at the start of an iteration (vertices,
// face slots with their vertex ids and creation keys, counters, the MINLOC direction) goes to a park
// slot in the workspace and tier 4 resumes from it, recomputing each face's plane from its vertices
// (the same arithmetic, so the same bits).  Results are those of a restart: the keys carry the face
// order, and a polytope does not depend on where its faces sit.  When the park slots run out a pair
// restarts from the simplex as before.
#ifndef GJKEPA_PARK
#define GJKEPA_PARK 1                 // 0: restart from the simplex (A/B)
#endif
#define GJKEPA_PARK_VC 72             // largest polytope parked: tier 2's (tier 3's is 40 / 64)
#define GJKEPA_PARK_FC 128
#define GJKEPA_PARK_HDR 128           // header: counters (64 B) and direction / distances (<= 64 B)
#define GJKEPA_PARK_BYTES (GJKEPA_PARK_HDR + 3 * 8 * GJKEPA_PARK_VC + 2 * 4 * GJKEPA_PARK_FC)   // 2880

// gjkepa_*_args::grid: > 0 explicit, 0 occupancy x CUs (looping workgroups), GJKEPA_GRID_UNITS one
// workgroup per work unit
#define GJKEPA_GRID_UNITS (-2)

struct gjkepa_gjk_args {
    const void* verts;
    const int64_t* hull_off;
    const int32_t* hull_cnt;
    const int32_t* pairs;
    int64_t n_pairs;
    uint8_t* route;             // [n_pairs]
    int route_code;             // pairs this launch serves: -1 = all (tier 0), else route code
    uint32_t* ctr;              // this launch's chunk counter (zero at launch)
    int claim;                  // 64-pair chunks taken per counter increment (sparse default)
    uint32_t* tally;            // pairs routed to each route code so far (GJKEPA_WS_TALLY entries)
    uint32_t* warm;             // optional [4 * n_pairs] warm-start simplex codes (in / out)
    void* out;                  // contact records (hits: simplex codes parked in their slot)
    int grid;                   // <= 0: occupancy x CUs
    int num_cus;
    uint32_t guard;             // gjkepa_guard_of(*this): checked at kernel entry in GJKEPA_DIAG_GUARD builds
};

struct gjkepa_epa_args {
    int version;
    double tol_ff;
    const void* verts;
    const int64_t* hull_off;
    const int32_t* hull_cnt;
    const int32_t* pairs;
    int64_t n_pairs;
    uint8_t* route;
    int route_code;             // GJKEPA_ROUTE_EPA0 + tier
    int next_code;              // route code for polytope overflow; -1 on the last tier
    int ct_base;                // route code base for the contact pass of the pairs this EPA tier finishes
    uint32_t* ctr;              // this launch's chunk counter (zero at launch)
    int claim;                  // 64-pair chunks taken per counter increment (sparse default)
    uint32_t* tally;            // pairs routed to each route code so far (GJKEPA_WS_TALLY entries)
    void* out;
    int grid;
    int num_cus;
    unsigned char* park;        // park slots (GJKEPA_PARK_BYTES each), nullptr: none
    uint32_t* park_ctr;         // park slots taken so far (workspace header)
    uint32_t park_cap;          // park slots available
    uint32_t guard;             // gjkepa_guard_of(*this): checked at kernel entry in GJKEPA_DIAG_GUARD builds
};

// Kernel-argument checksum over every field but `guard` (set by the host before each launch).  A
// GJKEPA_DIAG_GUARD build recomputes it at kernel entry: a kernel whose argument block does not
// match what the host enqueued records the mismatch in a device-global report
// (gjkepa_diag_guard) and returns without touching memory.
__host__ __device__ inline uint64_t gjkepa_mix(uint64_t h, uint64_t v) {
    h ^= v + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
    return h;
}
__host__ __device__ inline uint32_t gjkepa_fold(uint64_t h) { return (uint32_t)(h ^ (h >> 32)) | 1u; }
__host__ __device__ inline uint32_t gjkepa_guard_of(const gjkepa_gjk_args& a) {
    uint64_t h = 0x67ull;
    h = gjkepa_mix(h, (uint64_t)a.verts); h = gjkepa_mix(h, (uint64_t)a.hull_off); h = gjkepa_mix(h, (uint64_t)a.hull_cnt);
    h = gjkepa_mix(h, (uint64_t)a.pairs); h = gjkepa_mix(h, (uint64_t)a.n_pairs); h = gjkepa_mix(h, (uint64_t)a.route);
    h = gjkepa_mix(h, (uint64_t)(int64_t)a.route_code); h = gjkepa_mix(h, (uint64_t)a.ctr);
    h = gjkepa_mix(h, (uint64_t)(int64_t)a.claim); h = gjkepa_mix(h, (uint64_t)a.tally); h = gjkepa_mix(h, (uint64_t)a.warm);
    h = gjkepa_mix(h, (uint64_t)a.out); h = gjkepa_mix(h, (uint64_t)(int64_t)a.grid); h = gjkepa_mix(h, (uint64_t)(int64_t)a.num_cus);
    return gjkepa_fold(h);
}
__host__ __device__ inline uint32_t gjkepa_guard_of(const gjkepa_epa_args& a) {
    uint64_t h = 0x65ull;
    h = gjkepa_mix(h, (uint64_t)(int64_t)a.version); h = gjkepa_mix(h, __builtin_bit_cast(uint64_t, a.tol_ff));
    h = gjkepa_mix(h, (uint64_t)a.verts); h = gjkepa_mix(h, (uint64_t)a.hull_off); h = gjkepa_mix(h, (uint64_t)a.hull_cnt);
    h = gjkepa_mix(h, (uint64_t)a.pairs); h = gjkepa_mix(h, (uint64_t)a.n_pairs); h = gjkepa_mix(h, (uint64_t)a.route);
    h = gjkepa_mix(h, (uint64_t)(int64_t)a.route_code); h = gjkepa_mix(h, (uint64_t)(int64_t)a.next_code);
    h = gjkepa_mix(h, (uint64_t)(int64_t)a.ct_base); h = gjkepa_mix(h, (uint64_t)a.ctr);
    h = gjkepa_mix(h, (uint64_t)(int64_t)a.claim); h = gjkepa_mix(h, (uint64_t)a.tally); h = gjkepa_mix(h, (uint64_t)a.out);
    h = gjkepa_mix(h, (uint64_t)(int64_t)a.grid); h = gjkepa_mix(h, (uint64_t)(int64_t)a.num_cus);
    h = gjkepa_mix(h, (uint64_t)a.park); h = gjkepa_mix(h, (uint64_t)a.park_ctr); h = gjkepa_mix(h, (uint64_t)a.park_cap);
    return gjkepa_fold(h);
}

hipError_t gjkepa_launch_gjk(int tier, int vert_dtype, int precision, const gjkepa_gjk_args& a, hipStream_t s);
hipError_t gjkepa_launch_epa(int tier, int vert_dtype, int precision, const gjkepa_epa_args& a, hipStream_t s);
// contact tiers take the same argument block (route_code = GJKEPA_ROUTE_CT0 + tier; next_code unused)
hipError_t gjkepa_launch_contact(int tier, int vert_dtype, int precision, const gjkepa_epa_args& a, hipStream_t s);
// fp32 chain's last launch: the pairs routed GJKEPA_ROUTE_REDO, one wave each, GJK + EPA + contact in
// fp64, stored as fp32 records
hipError_t gjkepa_launch_redo(int vert_dtype, const gjkepa_epa_args& a, hipStream_t s);
// one-kernel path for small batches: one wave per pair (grid = n_pairs), GJK + EPA + contact features
hipError_t gjkepa_launch_query(int vert_dtype, int precision, const gjkepa_epa_args& a, hipStream_t s);
// the chain's counter / tally reset (n32 uint32 words from ws); a kernel node rather than a memset node
hipError_t gjkepa_launch_ws_reset(uint32_t* ws, int n32, hipStream_t s);

// ---- resident query service (gjkepa_query): a grid of one-wave workgroups, wave w serving request
// slot w, that polls host-mapped request slots and answers each posted pair with query_pair.  A
// slot's request line is written by the host (payload and header first, `req` last, release), its
// completion line by the device (record first, `done` last, release); each side polls the other's.
#ifndef GJKEPA_SVC_SLOTS
#define GJKEPA_SVC_SLOTS 64
#endif
// The service's waves run the full one-wave path (hulls up to GJKEPA_MAX_HULL_VERTS, polytope restarts);
// a lean variant (hulls <= 128, small polytope only, declining the rest) cost a lone call 2.3 us and a
// concurrent batch nothing less (A/B r5) and was removed in round 6.
#ifndef GJKEPA_SVC_MINW
#define GJKEPA_SVC_MINW 1
#endif
struct alignas(128) gjkepa_svc_slot {
    uint32_t req, stop;              // posted request's sequence number; nonzero: the serving wave exits
    int32_t version, na, nb, pad0;
    double tol_ff;
    uint32_t pad1[24];
    uint32_t done, pad2;             // sequence number of the last answered request
    uint64_t t_seen, t_done;         // device wall clock when it was seen / answered (GJKEPA_QUERY_STATS)
    uint32_t pad3[26];
    uint64_t rec[16];                // its gjkepa_contact_f64 record
    double v[3 * 2 * GJKEPA_MAX_HULL_VERTS];   // hull A columns (x, y, z), then hull B's
};
struct gjkepa_svc_ctrl {             // device memory, one per service
    uint32_t closing, pad;           // generation whose grid is draining
    uint64_t last;                   // wall clock of the latest answered request
};
struct gjkepa_svc_args {
    gjkepa_svc_slot* slots;          // device view of the host-mapped slots
    gjkepa_svc_ctrl* ctrl;
    uint32_t* host_closing;          // device view of a host-mapped word: generation that is draining
    uint32_t gen;                    // this grid's generation (nonzero)
    uint64_t idle_ticks;             // wall-clock ticks without a request anywhere before the grid drains
    uint64_t life_ticks;             // wall-clock ticks after which the grid drains even under traffic
};
hipError_t gjkepa_launch_service(const gjkepa_svc_args& a, int n_slots, hipStream_t s);
