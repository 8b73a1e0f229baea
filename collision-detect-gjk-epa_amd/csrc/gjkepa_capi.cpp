// gjkepa_capi.cpp — the C-ABI of include/gjkepa.h over the tiered HIP kernels.
//
// Host-buffer entries (gjkepa_query, gjkepa_batch) own per-device staging buffers that grow as
// needed and are reused; they are serialised per device by a mutex, so concurrent callers (the
// reference's `!$OMP PARALLEL DO ... CALL GJKEPA` pattern) are safe.  gjkepa_batch_device never
// allocates or synchronises: it enqueues a 256-byte counter / tally reset and the tier kernels (2 GJK +
// 5 EPA tiers, and the contact passes, forked onto a second stream for large batches); each kernel
// takes 64-pair chunks (or runs of 16) from its own counter.  gjkepa_hull_batch(_device) follow the
// same pattern for the batched convex-hull kernels (two tiers over one cloud list).
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdio>
#include <cstring>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/gjkepa.h"
#include "gjkepa_kernel.h"
#include "hull_kernel.h"
#include "broadphase_kernel.h"
#include "contacts_kernel.h"
#include "capi_internal.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
int hip_fail(hipError_t e, const char* what) {
    return fail(GJKEPA_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

constexpr int64_t kWsHeader = 512;      // counters, tallies, park slot counter (gjkepa_workspace_bytes)
constexpr int kWsParkWord = GJKEPA_WS_COUNTERS + GJKEPA_WS_TALLY;
// Workspace = header | one route byte per pair | park slots (GJKEPA_PARK_BYTES each, from the first
// 256-byte boundary after the route bytes).  gjkepa_workspace_bytes sizes the park area for one pair in
// kParkShare (C4 parks 9.2% of its pairs); whatever a caller provides beyond the route bytes is used.
constexpr int64_t kParkShare = 8;
int64_t ws_base(int64_t n) { return (kWsHeader + n + 255) / 256 * 256; }
constexpr int kSparseClaim = 16;
#ifndef GJKEPA_OVERLAP_MIN
#define GJKEPA_OVERLAP_MIN (1 << 16)
#endif
constexpr int64_t kOverlapMin = GJKEPA_OVERLAP_MIN;   // batches from this size fork the contact pass (enqueue)
#ifndef GJKEPA_FUSED_MAX
#define GJKEPA_FUSED_MAX 64
#endif
constexpr int64_t kFusedMax = GJKEPA_FUSED_MAX;       // batches up to this size run the one-kernel query path
#ifndef GJKEPA_DENSE_EPA_TIERS
#define GJKEPA_DENSE_EPA_TIERS 2   // EPA tiers below this always claim single chunks; the others start
#endif                             // sparse and switch to single chunks when their route tally is dense   // tiers that serve few pairs claim runs of 16 chunks (one 1-KB route load)

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = bytes + bytes / 4 + 4096;
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
};

struct HostBuf {                 // pinned host staging (one DMA each way for combined queries)
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        size_t want = bytes + bytes / 4 + 4096;
        hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e == hipSuccess) cap = want;
        return e;
    }
};

struct DeviceState {
    std::mutex mu;
    bool init = false;
    int num_cus = 0;
    hipStream_t stream = nullptr;
    DevBuf verts, off, cnt, pairs, out, ws;
    DevBuf h_foff, h_faces, h_nf, h_nv, h_st, h_hv, h_vi;   // gjkepa_hull_batch staging
    DevBuf b_pairs, b_count, b_ws;                          // gjkepa_broadphase staging
    DevBuf c_idx, c_hits, c_ws, c_n;                        // gjkepa_collide staging
    DevBuf q_blk, q_ws;                                     // combined gjkepa_query batches
    HostBuf q_host;
};

std::mutex g_table_mu;
std::vector<DeviceState*> g_dev;

DeviceState* device_state(int device, int* rc) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0) { *rc = fail(GJKEPA_E_NODEVICE, "no HIP device"); return nullptr; }
    if (device < 0 || device >= n) { *rc = fail(GJKEPA_E_ARG, "device index out of range"); return nullptr; }
    std::lock_guard<std::mutex> g(g_table_mu);
    if ((int)g_dev.size() < n) g_dev.resize((size_t)n, nullptr);
    if (!g_dev[(size_t)device]) g_dev[(size_t)device] = new DeviceState();
    *rc = 0;
    return g_dev[(size_t)device];
}

int num_cus_current() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) return 256;
    return cus;
}

// Second stream for the overlapped contact passes (GJKEPA_CONTACT_OVERLAP).  The pairs EPA tier t
// finishes carry the route codes GJKEPA_ROUTE_CT(t) + contact tier, and their contact pass is forked
// onto an internal stream as soon as tier t is done, so it runs beside EPA tiers t+1..4: on C2 the
// contact pass of EPA tier 0 (most of the hits) overlaps tier 1 (a few long pairs), on C5 that of
// tier 2 overlaps tier 3.  Every fork joins back into the caller's stream at the end of the chain;
// the two streams never touch the same pair.  The internal stream and its events belong to one
// (device, caller stream): callers on different streams never share them, so one caller's work
// never waits on another's contact passes, and an internal stream that joins a caller's graph
// capture (the fork / join events make it part of the capture) carries only that caller's work.
// Up to kForkMax caller streams get their own; further streams run the chain on one stream.
// (A/B: the other way round, later EPA tiers on a high-priority internal stream beside the contact
// pass, was 2.5% slower on C2.)
// Each fork point gets its own internal stream (GJKEPA_FORK_STREAMS 2; 1: one shared stream, the
// passes in order), so a small pass forked late does not queue behind the big pass of tier 0.  The
// internal streams run at the highest stream priority (GJKEPA_FORK_PRIO 1; 0 default, -1 lowest):
// the forked pass of EPA tier 0 is the C2 chain's critical path, while the EPA tiers beside it serve
// a few long pairs (A/B r3: C2 144.5 vs 143.9 M/s at the lowest priority; C4 / C5 unchanged).  The last fork
// point's pass runs on the caller's stream (GJKEPA_LAST_PASS_MAIN): nothing follows it to overlap.
#ifndef GJKEPA_FORK_MASK
#define GJKEPA_FORK_MASK 0x25
#endif
#ifndef GJKEPA_FORK_STREAMS
#define GJKEPA_FORK_STREAMS 2
#endif
#ifndef GJKEPA_FORK_PRIO
#define GJKEPA_FORK_PRIO 1
#endif
#ifndef GJKEPA_LAST_PASS_MAIN
#define GJKEPA_LAST_PASS_MAIN 1
#endif
struct Fork {
    std::mutex mu;
    hipStream_t s2[GJKEPA_EPA_TIERS] = {};       // internal stream of fork point t (all [0] if shared)
    hipEvent_t fork[GJKEPA_EPA_TIERS] = {}, join[GJKEPA_EPA_TIERS] = {};
    hipEvent_t part[8] = {};                     // fork of EPA tier 0's (0..3) / tier 2's (4..7) part i
    hipStream_t s3 = nullptr;                    // second stream for alternate parts (GJKEPA_EPA0_STREAMS 2)
    hipEvent_t fork3 = nullptr, join3 = nullptr;
    hipStream_t s4 = nullptr;                    // contact passes of the odd parts (GJKEPA_PART_PASS_STREAMS 2)
    hipEvent_t join4 = nullptr;
    hipEvent_t fork23 = nullptr, join23 = nullptr;   // EPA tier 3 on s3 beside tier 2 (GJKEPA_E23_STREAMS 2)
};
struct ForkKey {
    int dev;
    hipStream_t caller;
};
constexpr size_t kForkMax = 256;
std::mutex g_fork_mu;
std::vector<std::pair<ForkKey, Fork*>> g_fork;

// the fork state of (current device, caller stream s); *out = nullptr when the table is full
int fork_state(hipStream_t s, Fork** out) {
    *out = nullptr;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
    std::lock_guard<std::mutex> g(g_fork_mu);
    for (auto& kv : g_fork)
        if (kv.first.dev == dev && kv.first.caller == s) { *out = kv.second; return 0; }
    if (g_fork.size() >= kForkMax) return 0;
    Fork* f = new Fork();
    int least = 0, greatest = 0, prio = 0;
    if (GJKEPA_FORK_PRIO != 0 && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess)
        prio = GJKEPA_FORK_PRIO > 0 ? greatest : least;
    for (int t = 0; t < GJKEPA_EPA_TIERS && e == hipSuccess; ++t) {
        // a stream per fork point that forks (the first one only when shared)
        const bool forks = ((GJKEPA_FORK_MASK >> t) & 1) && !(GJKEPA_LAST_PASS_MAIN && t == GJKEPA_EPA_TIERS - 1);
        if (forks && (GJKEPA_FORK_STREAMS > 1 || !f->s2[0])) e = hipStreamCreateWithPriority(&f->s2[t], hipStreamNonBlocking, prio);
        else if (forks) f->s2[t] = f->s2[0];
        if (e == hipSuccess) e = hipEventCreateWithFlags(&f->fork[t], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&f->join[t], hipEventDisableTiming);
    }
    for (int i = 0; i < 8 && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&f->part[i], hipEventDisableTiming);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&f->s3, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&f->fork3, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&f->join3, hipEventDisableTiming);
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&f->s4, hipStreamNonBlocking, prio);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&f->join4, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&f->fork23, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&f->join23, hipEventDisableTiming);
    if (e != hipSuccess) {
        delete f;
        return hip_fail(e, "overlap stream / events");
    }
    g_fork.push_back({ForkKey{dev, s}, f});
    *out = f;
    return 0;
}

// hull capacity (vertices) of EPA tier t (gjkepa_kernel.hip: epa_hull_cap)
constexpr int epa_hull_cap(int t) {
    return t == 0 ? GJKEPA_E0_G * GJKEPA_E0_K : t == 1 ? GJKEPA_E1_G * GJKEPA_E1_K : t == 2 ? GJKEPA_E2_G * GJKEPA_E2_K
         : t == 3 ? GJKEPA_E3_G * GJKEPA_E3_K : t == 4 ? GJKEPA_E4_G * GJKEPA_E4_K : GJKEPA_E5_G * GJKEPA_E5_K;
}

// Fork points of an overlapped chain (bit t: a contact pass is forked after EPA tier t).  The pairs
// EPA tier t finishes go to the contact pass of the first fork point p >= t (route code
// GJKEPA_ROUTE_CT(p) + contact tier).  Default: after tier 0 (C2's hits), after tier 2 (C4 / C5's
// 33-128-vertex hulls, with tier 1's few overflow pairs) and after the last tier (tiers 3-5): three
// forks and five contact launches instead of one fork and up to two launches per tier, so the short
// tail of a C2 chain carries three fewer near-empty launches.
static_assert((GJKEPA_FORK_MASK >> (GJKEPA_EPA_TIERS - 1)) & 1, "the last EPA tier is a fork point");
constexpr int fork_point(int t) {          // first fork point >= t
    while (!((GJKEPA_FORK_MASK >> t) & 1)) ++t;
    return t;
}
// contact tiers a fork point's pass needs: 1 when every hull of its EPA tiers fits contact tier 0
constexpr int fork_contact_tiers(int p) {
    int cap = 0;
    for (int t = 0; t <= p; ++t)
        if (fork_point(t) == p && epa_hull_cap(t) > cap) cap = epa_hull_cap(t);
    return cap <= GJKEPA_C0_G * GJKEPA_C0_K ? 1 : GJKEPA_CONTACT_TIERS;
}
// EPA tier 0 in parts (GJKEPA_EPA0_PARTS; environment override for A/B): tier 0 runs over P
// consecutive pair ranges, one launch each, and the contact pass of part i is forked as soon as part i
// is done, so it runs beside the EPA of parts i+1.. instead of after all of tier 0 (C2's critical path
// was GJK 0 -> EPA 0 -> the whole contact pass).  Which launch answers a pair never changes its record.
#ifndef GJKEPA_EPA0_PARTS
#define GJKEPA_EPA0_PARTS 2       // A/B r4 (C2, 2 rounds): 1 part 149.7, 2 parts 150.7, 4 parts 145.5, 8 parts 113.8 M/s
#endif
constexpr int kPartsMax = 4;
int parts_env(const char* name, int dflt) {
    const char* e = std::getenv(name);
    const int v = e ? std::atoi(e) : dflt;
    return v < 1 ? 1 : v > kPartsMax ? kPartsMax : v;
}
// the parts alternate between the caller's stream and a second internal stream (2), so a part's tail
// overlaps the next part instead of idling the CUs it leaves (GJKEPA_EPA0_STREAMS, environment A/B)
#ifndef GJKEPA_EPA0_STREAMS
#define GJKEPA_EPA0_STREAMS 2     // A/B r4 (C2, 2 rounds, 2 parts): one stream 150.7, two streams 157.4 M/s
#endif
int epa0_streams() {
    static const int p = [] {
        const char* e = std::getenv("GJKEPA_EPA0_STREAMS");
        const int v = e ? std::atoi(e) : GJKEPA_EPA0_STREAMS;
        return v == 2 ? 2 : 1;
    }();
    return p;
}
// the contact passes of the odd parts on their own internal stream (2), so a part's pass starts when
// its EPA part ends instead of queueing behind the previous part's pass (GJKEPA_PART_PASS_STREAMS)
#ifndef GJKEPA_PART_PASS_STREAMS
#define GJKEPA_PART_PASS_STREAMS 1
#endif
int part_pass_streams() {
    static const int p = [] {
        const char* e = std::getenv("GJKEPA_PART_PASS_STREAMS");
        const int v = e ? std::atoi(e) : GJKEPA_PART_PASS_STREAMS;
        return v == 2 ? 2 : 1;
    }();
    return p;
}
// share of the pair range in EPA tier 0's first part when it runs in two (per mille; environment
// GJKEPA_EPA0_FIRST, A/B): the second part's contact pass is the chain's tail
#ifndef GJKEPA_EPA0_FIRST
#define GJKEPA_EPA0_FIRST 650      // A/B r4 (C2, 5 rounds): 500 157.6, 650 158.6, 700-750 158.5, 300 151.7 M/s
#endif
int epa0_first() {
    static const int p = [] {
        const char* e = std::getenv("GJKEPA_EPA0_FIRST");
        const int v = e ? std::atoi(e) : GJKEPA_EPA0_FIRST;
        return v < 100 ? 100 : v > 900 ? 900 : v;
    }();
    return p;
}
int epa0_parts() {
    static const int p = parts_env("GJKEPA_EPA0_PARTS", GJKEPA_EPA0_PARTS);
    return p;
}
// EPA tier 2 (hulls of 33-128 vertices: most of C5's pairs) in parts the same way (GJKEPA_EPA2_PARTS)
#ifndef GJKEPA_EPA2_PARTS
#define GJKEPA_EPA2_PARTS 1
#endif
int epa2_parts() {
    static const int p = parts_env("GJKEPA_EPA2_PARTS", GJKEPA_EPA2_PARTS);
    return p;
}
// launches of an overlapped chain: 2 GJK + the EPA tiers (tiers 0 and 2 in up to kPartsMax parts) +
// each fork point's contact pass (once per part); every launch owns one workspace counter
constexpr int overlap_launches() {
    int n = GJKEPA_GJK_TIERS + GJKEPA_EPA_TIERS + 2 * (kPartsMax - 1);
    for (int t = 0; t < GJKEPA_EPA_TIERS; ++t)
        if ((GJKEPA_FORK_MASK >> t) & 1) n += fork_contact_tiers(t) * (t == 0 || t == 2 ? kPartsMax : 1);
    return n;
}
static_assert(overlap_launches() + 1 <= GJKEPA_WS_COUNTERS, "workspace launch counters (+1: the fp32 redo launch)");
static_assert(GJKEPA_ROUTE_REDO < GJKEPA_WS_TALLY && GJKEPA_ROUTE_REDO > GJKEPA_ROUTE_CT(GJKEPA_EPA_TIERS - 1) + 1,
              "redo route code");
// The forked contact pass of EPA tier 0 (a dense launch) takes one workgroup per 64-pair chunk
// instead of an occupancy-sized grid of looping workgroups: a workgroup leaves when its chunk is
// done, so the EPA tiers launched beside the pass get wave slots as they free up instead of
// queueing behind the whole pass (C2: the empty EPA tier 2 launch waited 657 us behind it).
#ifndef GJKEPA_CONTACT_UNITS_GRID
#define GJKEPA_CONTACT_UNITS_GRID 1
#endif
// EPA tiers 2 (hulls of 33-128 vertices) and 3 (129-256, first pass) serve disjoint pairs: with 2 they
// run side by side, tier 3 on an internal stream forked after tier 1 and joined before tier 4, which
// resumes both tiers' parked polytopes.  Tier 2's overflow then goes straight to tier 4 (a restart in
// tier 3 would outgrow its 40-vertex polytope anyway; which tier answers never changes a record).
// Environment override GJKEPA_E23_STREAMS for A/B.
#ifndef GJKEPA_E23_STREAMS
#define GJKEPA_E23_STREAMS 1       // A/B r5 (C4, 2 rounds): in sequence 39.51 / 39.41, side by side 38.54 / 38.63 M/s; C5 within 0.2%
#endif
int e23_streams() {
    static const int p = [] {
        const char* e = std::getenv("GJKEPA_E23_STREAMS");
        const int v = e ? std::atoi(e) : GJKEPA_E23_STREAMS;
        return v == 2 ? 2 : 1;
    }();
    return p;
}

// Park slots.  Only EPA tiers 2 and 3 park (hulls above EPA tier 1's capacity), so the park area a
// batch can use is sized by its pairs with a hull above kParkMinHull vertices: gjkepa_workspace_bytes_for.
constexpr int kParkMinHull = epa_hull_cap(1);
static_assert(epa_hull_cap(0) <= kParkMinHull, "EPA tiers 0 and 1 never park");
int64_t ws_bytes_for(int64_t n_pairs, int64_t n_large) {
    return ws_base(n_pairs) + (n_large + kParkShare - 1) / kParkShare * GJKEPA_PARK_BYTES;
}
// pairs of a host-side pair list with a hull above kParkMinHull vertices
int64_t count_large(const int32_t* pairs, int64_t n_pairs, const int32_t* hull_cnt) {
    int64_t n = 0;
    for (int64_t k = 0; k < n_pairs; ++k)
        n += hull_cnt[pairs[2 * k]] > kParkMinHull || hull_cnt[pairs[2 * k + 1]] > kParkMinHull;
    return n;
}

// ---- per-launch timing (gjkepa_launch_timing; bench.py's dominant-kernel roofline) -------------------
// With timing on for the calling thread, each chain it enqueues records one event at its head on the
// caller's stream and two around every kernel launch, on the stream that launch goes to.
// gjkepa_launch_timing_read waits for them and reports each launch's start / end relative to its
// chain's head.  Timing events are barrier markers in the stream's queue; a launch's start is when the
// stream reached it (its previous work on that stream had finished).
struct TimedLaunch {
    gjkepa_launch_time info;
    hipEvent_t head, b, e;
};
struct Timing {
    bool on = false;
    int chain = -1;
    hipEvent_t head = nullptr;
    std::vector<hipStream_t> streams;        // this chain's streams, in order of first use (0: caller's)
    std::vector<TimedLaunch> launches;
    std::vector<hipEvent_t> pool;            // events no pending launch refers to
    std::vector<hipEvent_t> used;
    hipEvent_t get() {
        hipEvent_t ev = nullptr;
        if (!pool.empty()) {
            ev = pool.back();
            pool.pop_back();
        } else if (hipEventCreate(&ev) != hipSuccess) {
            return nullptr;
        }
        used.push_back(ev);
        return ev;
    }
};
constexpr size_t kTimingMax = 1 << 16;       // launches kept between two reads
static_assert(sizeof(gjkepa_launch_time) == 64, "gjkepa_launch_time layout (gjkepa.py LAUNCH_TIME)");
thread_local Timing g_tm;

// start a chain on caller stream s (no-op unless timing is on)
void timing_chain(hipStream_t s) {
    if (!g_tm.on || g_tm.launches.size() >= kTimingMax) return;
    g_tm.head = g_tm.get();
    if (!g_tm.head || hipEventRecord(g_tm.head, s) != hipSuccess) { g_tm.head = nullptr; return; }
    ++g_tm.chain;
    g_tm.streams.assign(1, s);
}
// launch f() on stream st, bracketed by timing events when on
template <typename F>
hipError_t timed(const char* kind, int tier, int part, int route_code, int64_t first, int64_t count, hipStream_t st,
                 F&& f) {
    if (!g_tm.on || !g_tm.head || g_tm.launches.size() >= kTimingMax) return f();
    TimedLaunch t{};
    std::snprintf(t.info.kernel, sizeof(t.info.kernel), "%s", kind);
    t.info.tier = tier;
    t.info.part = part;
    t.info.route_code = route_code;
    t.info.chain = g_tm.chain;
    int sid = 0;
    while (sid < (int)g_tm.streams.size() && g_tm.streams[(size_t)sid] != st) ++sid;
    if (sid == (int)g_tm.streams.size()) g_tm.streams.push_back(st);
    t.info.stream = sid;
    t.info.first_pair = first;
    t.info.n_pairs = count;
    t.head = g_tm.head;
    t.b = g_tm.get();
    t.e = g_tm.get();
    if (t.b) (void)hipEventRecord(t.b, st);
    const hipError_t e = f();
    if (t.e) (void)hipEventRecord(t.e, st);
    if (e == hipSuccess && t.b && t.e) g_tm.launches.push_back(t);
    return e;
}

int enqueue(int32_t version, double tol_ff, int32_t vert_dtype, int32_t precision, const void* verts,
            const int64_t* hull_off, const int32_t* hull_cnt, const int32_t* pairs, int64_t n_pairs,
            void* out, void* workspace, int64_t ws_bytes, hipStream_t s, int num_cus, uint32_t* warm = nullptr) {
    if (n_pairs == 0) return 0;
    // the header and the route bytes are required; park slots are used as far as the caller provides them
    if (ws_bytes < ws_base(n_pairs)) return fail(GJKEPA_E_WORKSPACE, "workspace too small");
    // workspace: per-launch chunk counters and route tallies (zeroed here), then one route byte per
    // pair (written by GJK tier 0 for every pair before any read)
    uint32_t* ctr = (uint32_t*)workspace;
    uint8_t* route = (uint8_t*)workspace + kWsHeader;
    const int64_t park_slots = ws_bytes > ws_base(n_pairs) ? (ws_bytes - ws_base(n_pairs)) / GJKEPA_PARK_BYTES : 0;
    hipError_t e;
    timing_chain(s);
    if (!warm && n_pairs <= kFusedMax) {                 // small batch: one launch, one wave per pair
        gjkepa_epa_args q{};
        q.version = version;
        q.tol_ff = tol_ff;
        q.verts = verts;
        q.hull_off = hull_off;
        q.hull_cnt = hull_cnt;
        q.pairs = pairs;
        q.n_pairs = n_pairs;
        q.out = out;
        q.num_cus = num_cus;
        q.guard = gjkepa_guard_of(q);
        if ((e = timed("query", 0, 0, -1, 0, n_pairs, s, [&] { return gjkepa_launch_query(vert_dtype, precision, q, s); })) !=
            hipSuccess)
            return hip_fail(e, "query kernel launch");
        return 0;
    }
    static_assert(sizeof(uint32_t) * (kWsParkWord + 1) <= kWsHeader, "workspace header");
    // counter / tally / park counter reset: a one-wave kernel rather than a memset, so a captured
    // chain is kernel nodes only
    if ((e = timed("reset", 0, 0, -1, 0, 0, s, [&] { return gjkepa_launch_ws_reset(ctr, kWsParkWord + 1, s); })) != hipSuccess)
        return hip_fail(e, "workspace counter reset");
    uint32_t* tally = ctr + GJKEPA_WS_COUNTERS;
    int launch = 0;
    gjkepa_gjk_args g{};
    g.verts = verts;
    g.hull_off = hull_off;
    g.hull_cnt = hull_cnt;
    g.pairs = pairs;
    g.n_pairs = n_pairs;
    g.route = route;
    g.tally = tally;
    g.warm = warm;
    g.out = out;
    g.num_cus = num_cus;
    g.route_code = -1;                                   // GJK tier 0: every pair
    g.ctr = ctr + launch++;
    g.claim = 1;
    g.guard = gjkepa_guard_of(g);
    if ((e = timed("gjk", 0, 0, -1, 0, n_pairs, s, [&] { return gjkepa_launch_gjk(0, vert_dtype, precision, g, s); })) !=
        hipSuccess)
        return hip_fail(e, "GJK tier 0 launch");
    for (int t = 1; t < GJKEPA_GJK_TIERS; ++t) {         // GJK tiers 1, 2: hulls above tier 0's capacity
        g.route_code = GJKEPA_ROUTE_GJK1 + t - 1;
        g.ctr = ctr + launch++;
        g.claim = kSparseClaim;
        g.guard = gjkepa_guard_of(g);
        if ((e = timed("gjk", t, 0, g.route_code, 0, n_pairs, s, [&] { return gjkepa_launch_gjk(t, vert_dtype, precision, g, s); })) !=
            hipSuccess)
            return hip_fail(e, "GJK tier launch");
    }
    gjkepa_epa_args a{};
    a.version = version;
    a.tol_ff = tol_ff;
    a.verts = verts;
    a.hull_off = hull_off;
    a.hull_cnt = hull_cnt;
    a.pairs = pairs;
    a.n_pairs = n_pairs;
    a.route = route;
    a.tally = tally;
    a.out = out;
    a.num_cus = num_cus;
    a.park = park_slots > 0 ? (unsigned char*)workspace + ws_base(n_pairs) : nullptr;
    a.park_ctr = ctr + kWsParkWord;
    a.park_cap = (uint32_t)(park_slots < (int64_t)UINT32_MAX ? park_slots : UINT32_MAX);
    // small batches (e.g. combined single-pair queries) keep one stream: the fork's events and extra
    // launches cost more latency than the overlap saves
    Fork* f = nullptr;
    int rc;
    if (GJKEPA_CONTACT_OVERLAP && n_pairs >= kOverlapMin && (rc = fork_state(s, &f))) return rc;
    const bool overlap = f != nullptr;
    // EPA tiers 2 and 3 side by side (not when a contact pass forks after tier 3)
    const bool e23 = overlap && e23_streams() == 2 && !((GJKEPA_FORK_MASK >> 3) & 1);
    const gjkepa_epa_args whole = a;                     // (a.pairs / route / out / n_pairs: a pair range below)
    int64_t r_first = 0;                                 // the pair range `a` points at
    auto range = [&](int64_t first, int64_t count) {     // point `a` at pairs [first, first + count)
        a.pairs = whole.pairs + 2 * first;
        a.route = whole.route + first;
        a.out = (unsigned char*)whole.out + first * (precision == GJKEPA_PREC_F64 ? 128 : 64);
        a.n_pairs = count;
        r_first = first;
    };
    auto epa_tier = [&](int t, hipStream_t es) -> int {  // EPA tier t on stream es; polytope overflow -> next
        a.route_code = GJKEPA_ROUTE_EPA0 + t;
        // beside tier 3, tier 2's overflow goes to tier 4 (tier 3 is running: its tally is final at its start)
        a.next_code = t == GJKEPA_EPA_TIERS - 1 ? -1 : GJKEPA_ROUTE_EPA0 + t + (e23 && t == 2 ? 2 : 1);
        a.ct_base = overlap ? GJKEPA_ROUTE_CT(fork_point(t)) : GJKEPA_ROUTE_CT0;
        a.ctr = ctr + launch++;
        a.claim = t < GJKEPA_DENSE_EPA_TIERS ? 1 : kSparseClaim;
        // the last tier (overflow of the 208-face polytope: rare) takes one workgroup per CU: its
        // one-wave-per-SIMD workgroups otherwise queue for dispatch behind a concurrent contact pass even
        // when the tier is empty (C5: an empty launch spanned 1.1 ms of the chain)
        a.grid = t == GJKEPA_EPA_TIERS - 1 ? num_cus : 0;
        a.guard = gjkepa_guard_of(a);
        hipError_t er = timed("epa", t, 0, a.route_code, r_first, a.n_pairs, es,
                              [&] { return gjkepa_launch_epa(t, vert_dtype, precision, a, es); });
        return er == hipSuccess ? 0 : hip_fail(er, "EPA tier launch");
    };
    // contact features of the EPA results under route codes base + contact tier (tiers 0..ntiers-1).
    // `single`: every launch claims single chunks.  A pass forked after one part of a parted tier must:
    // the other parts are still adding to the route tally its sparse/dense choice (pick_claim) reads.
    auto contact_tiers = [&](int base, int ntiers, hipStream_t cs, bool single, int part) -> int {
        for (int t = 0; t < ntiers; ++t) {
            a.route_code = base + t;
            a.next_code = -1;
            a.ctr = ctr + launch++;
            a.claim = (single || (t == 0 && base <= GJKEPA_ROUTE_CT(0))) ? 1 : kSparseClaim;
            // a forked dense pass (EPA tier 0's hits) takes one workgroup per chunk
            a.grid = GJKEPA_CONTACT_UNITS_GRID && cs != s && a.claim == 1 ? GJKEPA_GRID_UNITS : 0;
            a.guard = gjkepa_guard_of(a);
            hipError_t er = timed("contact", t, part, a.route_code, r_first, a.n_pairs, cs,
                                  [&] { return gjkepa_launch_contact(t, vert_dtype, precision, a, cs); });
            if (er != hipSuccess) return hip_fail(er, "contact tier launch");
        }
        return 0;
    };
    // fp32 compute: the pairs whose fp32 answer was not certified, recomputed in fp64 (after every
    // contact pass has joined the caller's stream; an empty launch returns at once)
    auto redo = [&]() -> int {
        if (precision != GJKEPA_PREC_F32) return 0;
        a.route_code = GJKEPA_ROUTE_REDO;
        a.next_code = -1;
        a.ctr = ctr + launch++;
        a.claim = kSparseClaim;
        a.grid = 0;
        a.guard = gjkepa_guard_of(a);
        hipError_t er = timed("redo", 0, 0, a.route_code, r_first, a.n_pairs, s,
                              [&] { return gjkepa_launch_redo(vert_dtype, a, s); });
        return er == hipSuccess ? 0 : hip_fail(er, "fp32 redo launch");
    };
    if (overlap) {
        std::lock_guard<std::mutex> lk(f->mu);
        constexpr int last = GJKEPA_EPA_TIERS - 1;
        bool forked[GJKEPA_EPA_TIERS] = {};
        // EPA tier t (a fork point that forks) in `parts` launches over consecutive pair ranges, alternately
        // on the caller's stream and an internal one, each range's contact pass forked when it is done
        bool used4 = false;
        auto parted = [&](int t, int parts) -> int {
            const int64_t chunks = (n_pairs + 63) / 64;
            const bool two = epa0_streams() == 2;
            if (two && ((e = hipEventRecord(f->fork3, s)) != hipSuccess || (e = hipStreamWaitEvent(f->s3, f->fork3, 0)) != hipSuccess))
                return hip_fail(e, "EPA part stream fork");
            for (int i = 0; i < parts; ++i) {
                int64_t c0 = chunks * i / parts, c1 = chunks * (i + 1) / parts;
                if (t == 0 && parts == 2) {                  // uneven halves (GJKEPA_EPA0_FIRST)
                    const int64_t cut = chunks * epa0_first() / 1000;
                    c0 = i == 0 ? 0 : cut;
                    c1 = i == 0 ? cut : chunks;
                }
                const int64_t first = c0 * 64, count = (c1 * 64 < n_pairs ? c1 * 64 : n_pairs) - first;
                if (count <= 0) continue;
                range(first, count);
                hipStream_t ps = two && (i & 1) ? f->s3 : s;
                a.route_code = GJKEPA_ROUTE_EPA0 + t;
                a.next_code = GJKEPA_ROUTE_EPA0 + t + 1;
                a.ct_base = GJKEPA_ROUTE_CT(fork_point(t));
                a.ctr = ctr + launch++;
                a.claim = t < GJKEPA_DENSE_EPA_TIERS ? 1 : kSparseClaim;
                a.grid = 0;
                a.guard = gjkepa_guard_of(a);
                if ((e = timed("epa", t, i, a.route_code, first, count, ps,
                               [&] { return gjkepa_launch_epa(t, vert_dtype, precision, a, ps); })) != hipSuccess)
                    return hip_fail(e, "EPA tier launch");
                hipEvent_t pe = f->part[(t == 0 ? 0 : kPartsMax) + i];
                hipStream_t cs = part_pass_streams() == 2 && (i & 1) ? f->s4 : f->s2[t];
                if ((e = hipEventRecord(pe, ps)) != hipSuccess || (e = hipStreamWaitEvent(cs, pe, 0)) != hipSuccess)
                    return hip_fail(e, "contact pass fork");
                if ((rc = contact_tiers(GJKEPA_ROUTE_CT(t), fork_contact_tiers(t), cs, true, i))) return rc;
                if (cs == f->s4) used4 = true;
            }
            if (two && ((e = hipEventRecord(f->join3, f->s3)) != hipSuccess || (e = hipStreamWaitEvent(s, f->join3, 0)) != hipSuccess))
                return hip_fail(e, "EPA part stream join");
            a = whole;
            r_first = 0;
            forked[t] = true;
            return 0;
        };
        for (int t = 0; t < GJKEPA_EPA_TIERS; ++t) {
            const bool forks = ((GJKEPA_FORK_MASK >> t) & 1) && !(GJKEPA_LAST_PASS_MAIN && t == last);
            if (e23 && t == 2) {
                // tier 3 on s3, forked here (after tier 1) and joined below before tier 4
                if ((e = hipEventRecord(f->fork23, s)) != hipSuccess || (e = hipStreamWaitEvent(f->s3, f->fork23, 0)) != hipSuccess)
                    return hip_fail(e, "EPA tier 3 stream fork");
                if ((rc = epa_tier(3, f->s3))) return rc;
                if ((e = hipEventRecord(f->join23, f->s3)) != hipSuccess) return hip_fail(e, "EPA tier 3 stream join");
            }
            if (e23 && t == 3) continue;                     // launched beside tier 2
            if (e23 && t == 4 && (e = hipStreamWaitEvent(s, f->join23, 0)) != hipSuccess)
                return hip_fail(e, "EPA tier 3 stream join");
            const int np = !forks ? 1 : t == 0 ? epa0_parts() : t == 2 && !e23 ? epa2_parts() : 1;
            if (np > 1) {
                if ((rc = parted(t, np))) return rc;
                continue;
            }
            if ((rc = epa_tier(t, s))) return rc;
            if (!((GJKEPA_FORK_MASK >> t) & 1)) continue;
            if (GJKEPA_LAST_PASS_MAIN && t == last) {
                if ((rc = contact_tiers(GJKEPA_ROUTE_CT(t), fork_contact_tiers(t), s, false, 0))) return rc;
                continue;
            }
            if ((e = hipEventRecord(f->fork[t], s)) != hipSuccess || (e = hipStreamWaitEvent(f->s2[t], f->fork[t], 0)) != hipSuccess)
                return hip_fail(e, "contact pass fork");
            if ((rc = contact_tiers(GJKEPA_ROUTE_CT(t), fork_contact_tiers(t), f->s2[t], false, 0))) return rc;
            forked[t] = true;
        }
        for (int t = 0; t < GJKEPA_EPA_TIERS; ++t) {      // join every internal stream used (last one per stream)
            if (!forked[t]) continue;
            bool later = false;
            for (int u = t + 1; u < GJKEPA_EPA_TIERS; ++u) later = later || (forked[u] && f->s2[u] == f->s2[t]);
            if (later) continue;
            if ((e = hipEventRecord(f->join[t], f->s2[t])) != hipSuccess || (e = hipStreamWaitEvent(s, f->join[t], 0)) != hipSuccess)
                return hip_fail(e, "contact pass join");
        }
        if (used4 && ((e = hipEventRecord(f->join4, f->s4)) != hipSuccess || (e = hipStreamWaitEvent(s, f->join4, 0)) != hipSuccess))
            return hip_fail(e, "contact pass join");
        return redo();
    }
    for (int t = 0; t < GJKEPA_EPA_TIERS; ++t)
        if ((rc = epa_tier(t, s))) return rc;
    if ((rc = contact_tiers(GJKEPA_ROUTE_CT0, GJKEPA_CONTACT_TIERS, s, false, 0))) return rc;
    return redo();
}

// select `device` and create its stream on first use (caller holds d->mu)
int init_device(DeviceState* d, int device) {
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    if (!d->init) {
        e = hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking);
        if (e != hipSuccess) return hip_fail(e, "hipStreamCreate");
        d->num_cus = num_cus_current();
        d->init = true;
    }
    return 0;
}

bool valid_enums(int32_t vert_dtype, int32_t precision) {
    return (vert_dtype == GJKEPA_DTYPE_F32 || vert_dtype == GJKEPA_DTYPE_F64) &&
           (precision == GJKEPA_PREC_F32 || precision == GJKEPA_PREC_F64);
}

}  // namespace

namespace gjkepa_internal {
int set_error(int code, const std::string& msg) { return fail(code, msg); }
}  // namespace gjkepa_internal

extern "C" {

int gjkepa_record_bytes(int32_t precision) {
    if (precision == GJKEPA_PREC_F64) return (int)sizeof(gjkepa_contact_f64);
    if (precision == GJKEPA_PREC_F32) return (int)sizeof(gjkepa_contact_f32);
    return GJKEPA_E_ARG;
}

int64_t gjkepa_workspace_bytes(int64_t n_pairs) {
    if (n_pairs < 0) return GJKEPA_E_ARG;
    return ws_bytes_for(n_pairs, n_pairs);
}

int64_t gjkepa_workspace_bytes_for(int64_t n_pairs, int64_t n_large_pairs) {
    if (n_pairs < 0 || n_large_pairs < 0 || n_large_pairs > n_pairs) return GJKEPA_E_ARG;
    return ws_bytes_for(n_pairs, n_large_pairs);
}

int gjkepa_launch_timing(int32_t enable) {
    const int prev = g_tm.on ? 1 : 0;
    g_tm.on = enable != 0;
    return prev;
}

int gjkepa_launch_timing_read(gjkepa_launch_time* out, int32_t max) {
    if (max < 0 || (max > 0 && !out)) return fail(GJKEPA_E_ARG, "bad timing buffer");
    int n = 0;
    hipError_t e = hipSuccess;
    for (const TimedLaunch& t : g_tm.launches) {
        if ((e = hipEventSynchronize(t.e)) != hipSuccess) break;
        if (n >= max) continue;
        out[n] = t.info;
        float a = 0.f, b = 0.f;
        if ((e = hipEventElapsedTime(&a, t.head, t.b)) != hipSuccess || (e = hipEventElapsedTime(&b, t.head, t.e)) != hipSuccess)
            break;
        out[n].start_ms = a;
        out[n].end_ms = b;
        ++n;
    }
    // every event of the read launches is free again (an unread tail is dropped with them)
    for (hipEvent_t ev : g_tm.used) (void)hipEventSynchronize(ev);
    g_tm.pool.insert(g_tm.pool.end(), g_tm.used.begin(), g_tm.used.end());
    g_tm.used.clear();
    g_tm.launches.clear();
    g_tm.head = nullptr;
    g_tm.chain = -1;
    return e == hipSuccess ? n : hip_fail(e, "launch timing events");
}

const char* gjkepa_last_error(void) { return g_err.c_str(); }

#ifndef GJKEPA_SRC_HASH
#define GJKEPA_SRC_HASH "unknown"
#endif
const char* gjkepa_version_string(void) {
    static char buf[800];
    std::snprintf(buf, sizeof(buf),
                  "gjkepa-mi355x gfx950 wave64; GJK tiers G/K = %d/%d, %d/%d, %d/%d; EPA tiers G/K/VCAP/FCAP = "
                  "%d/%d/%d/%d, %d/%d/%d/%d, %d/%d/%d/%d, %d/%d/%d/%d, %d/%d/%d/%d, %d/%d/%d/%d; contact tiers G/K = %d/%d, %d/%d; "
                  "waves/SIMD G%d%d%d E%d%d%d%d%d%d C%d%d; LDS-hull G%d%d%d E%d%d%d%d%d%d C%d%d; "
                  "-O3 -ffp-contract=off; src %s",
                  GJKEPA_G0_G, GJKEPA_G0_K, GJKEPA_G1_G, GJKEPA_G1_K, GJKEPA_G2_G, GJKEPA_G2_K, GJKEPA_E0_G, GJKEPA_E0_K, GJKEPA_E0_VCAP,
                  GJKEPA_E0_FCAP, GJKEPA_E1_G, GJKEPA_E1_K, GJKEPA_E1_VCAP, GJKEPA_E1_FCAP, GJKEPA_E2_G, GJKEPA_E2_K,
                  GJKEPA_E2_VCAP, GJKEPA_E2_FCAP, GJKEPA_E3_G, GJKEPA_E3_K, GJKEPA_E3_VCAP, GJKEPA_E3_FCAP,
                  GJKEPA_E4_G, GJKEPA_E4_K, GJKEPA_E4_VCAP, GJKEPA_E4_FCAP, GJKEPA_E5_G, GJKEPA_E5_K, GJKEPA_E5_VCAP,
                  GJKEPA_E5_FCAP, GJKEPA_C0_G, GJKEPA_C0_K, GJKEPA_C1_G,
                  GJKEPA_C1_K, GJKEPA_G0_MINW, GJKEPA_G1_MINW, GJKEPA_G2_MINW, GJKEPA_E0_MINW, GJKEPA_E1_MINW, GJKEPA_E2_MINW,
                  GJKEPA_E3_MINW, GJKEPA_E4_MINW, GJKEPA_E5_MINW, GJKEPA_C0_MINW, GJKEPA_C1_MINW, GJKEPA_G0_LH, GJKEPA_G1_LH, GJKEPA_G2_LH,
                  GJKEPA_E0_LH, GJKEPA_E1_LH, GJKEPA_E2_LH, GJKEPA_E3_LH, GJKEPA_E4_LH, GJKEPA_E5_LH, GJKEPA_C0_LH,
                  GJKEPA_C1_LH, GJKEPA_SRC_HASH);
    return buf;
}

int gjkepa_batch_device(int32_t version, double tol_ff, int32_t vert_dtype, int32_t precision,
                        const void* verts, const int64_t* hull_off, const int32_t* hull_cnt,
                        const int32_t* pairs, int64_t n_pairs, void* out, void* workspace,
                        int64_t workspace_bytes, void* stream) {
    const gjkepa_internal::Range range_("gjkepa_batch_device (chain enqueue)");
    if (n_pairs < 0 || !valid_enums(vert_dtype, precision)) return fail(GJKEPA_E_ARG, "bad n_pairs/dtype/precision");
    if (n_pairs > 0 && (!verts || !hull_off || !hull_cnt || !pairs || !out || !workspace))
        return fail(GJKEPA_E_ARG, "null pointer");
    if (n_pairs > INT32_MAX) return fail(GJKEPA_E_ARG, "n_pairs above 2^31-1");
    return enqueue(version, tol_ff, vert_dtype, precision, verts, hull_off, hull_cnt, pairs, n_pairs, out,
                   workspace, workspace_bytes, (hipStream_t)stream, num_cus_current());
}

int gjkepa_batch_warm_device(int32_t version, double tol_ff, int32_t vert_dtype, int32_t precision,
                             const void* verts, const int64_t* hull_off, const int32_t* hull_cnt,
                             const int32_t* pairs, int64_t n_pairs, void* out, void* workspace,
                             int64_t workspace_bytes, uint32_t* warm, void* stream) {
    const gjkepa_internal::Range range_("gjkepa_batch_warm_device (chain enqueue)");
    if (n_pairs < 0 || !valid_enums(vert_dtype, precision)) return fail(GJKEPA_E_ARG, "bad n_pairs/dtype/precision");
    if (n_pairs > 0 && (!verts || !hull_off || !hull_cnt || !pairs || !out || !workspace || !warm))
        return fail(GJKEPA_E_ARG, "null pointer");
    if (n_pairs > INT32_MAX) return fail(GJKEPA_E_ARG, "n_pairs above 2^31-1");
    return enqueue(version, tol_ff, vert_dtype, precision, verts, hull_off, hull_cnt, pairs, n_pairs, out,
                   workspace, workspace_bytes, (hipStream_t)stream, num_cus_current(), warm);
}

int gjkepa_batch(int32_t version, double tol_ff, int32_t vert_dtype, int32_t precision,
                 const void* verts, int64_t n_vert_scalars, const int64_t* hull_off,
                 const int32_t* hull_cnt, int64_t n_hulls, const int32_t* pairs, int64_t n_pairs,
                 void* out, int32_t device) {
    const gjkepa_internal::Range range_("gjkepa_batch (H2D, chain, D2H)");
    if (n_pairs < 0 || n_hulls < 0 || n_vert_scalars < 0 || !valid_enums(vert_dtype, precision))
        return fail(GJKEPA_E_ARG, "bad sizes/dtype/precision");
    if (n_pairs == 0) return 0;
    if (!verts || !hull_off || !hull_cnt || !pairs || !out) return fail(GJKEPA_E_ARG, "null pointer");
    if (n_pairs > INT32_MAX) return fail(GJKEPA_E_ARG, "n_pairs above 2^31-1");
    // host-side validation of the index structure (device code trusts it)
    for (int64_t k = 0; k < 2 * n_pairs; ++k)
        if (pairs[k] < 0 || pairs[k] >= n_hulls) return fail(GJKEPA_E_ARG, "pair references a missing hull");
    for (int64_t h = 0; h < n_hulls; ++h) {
        int64_t c = hull_cnt[h];
        if (c >= 1 && (hull_off[h] < 0 || hull_off[h] + 3 * c > n_vert_scalars))
            return fail(GJKEPA_E_ARG, "hull outside the vertex pool");
    }
    // park slots only for the pairs that can reach the parking EPA tiers
    const int64_t wsb = ws_bytes_for(n_pairs, count_large(pairs, n_pairs, hull_cnt));
    int rc = 0;
    DeviceState* d = device_state(device, &rc);
    if (!d) return rc;
    std::lock_guard<std::mutex> g(d->mu);
    if ((rc = init_device(d, device))) return rc;
    hipError_t e;
    const size_t esz = vert_dtype == GJKEPA_DTYPE_F32 ? 4 : 8;
    const size_t rec = (size_t)gjkepa_record_bytes(precision);
    if ((e = d->verts.ensure((size_t)n_vert_scalars * esz)) != hipSuccess ||
        (e = d->off.ensure((size_t)n_hulls * 8)) != hipSuccess ||
        (e = d->cnt.ensure((size_t)n_hulls * 4)) != hipSuccess ||
        (e = d->pairs.ensure((size_t)n_pairs * 8)) != hipSuccess ||
        (e = d->out.ensure((size_t)n_pairs * rec)) != hipSuccess ||
        (e = d->ws.ensure((size_t)wsb)) != hipSuccess)
        return hip_fail(e, "hipMalloc");
    hipStream_t s = d->stream;
    if ((e = hipMemcpyAsync(d->verts.p, verts, (size_t)n_vert_scalars * esz, hipMemcpyHostToDevice, s)) != hipSuccess ||
        (e = hipMemcpyAsync(d->off.p, hull_off, (size_t)n_hulls * 8, hipMemcpyHostToDevice, s)) != hipSuccess ||
        (e = hipMemcpyAsync(d->cnt.p, hull_cnt, (size_t)n_hulls * 4, hipMemcpyHostToDevice, s)) != hipSuccess ||
        (e = hipMemcpyAsync(d->pairs.p, pairs, (size_t)n_pairs * 8, hipMemcpyHostToDevice, s)) != hipSuccess)
        return hip_fail(e, "hipMemcpyAsync H2D");
    rc = enqueue(version, tol_ff, vert_dtype, precision, d->verts.p, (const int64_t*)d->off.p,
                 (const int32_t*)d->cnt.p, (const int32_t*)d->pairs.p, n_pairs, d->out.p, d->ws.p,
                 (int64_t)d->ws.cap, s, d->num_cus);
    if (rc) return rc;
    if ((e = hipMemcpyAsync(out, d->out.p, (size_t)n_pairs * rec, hipMemcpyDeviceToHost, s)) != hipSuccess)
        return hip_fail(e, "hipMemcpyAsync D2H");
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    return 0;
}

}  // extern "C"

namespace {

// Single-pair queries are combined across threads (the reference's `!$OMP PARALLEL DO ... CALL
// GJKEPA` pattern): a caller queues its pair; if no batch is being run, it becomes the leader, takes
// every queued pair with the same (version_, TOL_FF_), runs them as one gjkepa_batch and hands the
// records back; otherwise it waits.  While one batch is on the GPU the other threads' pairs queue
// up, so with T calling threads a round trip serves up to T pairs instead of one.
struct Query {
    int32_t version;
    double tol_ff;
    const double *p1, *p2;
    int32_t n1, n2;
    gjkepa_contact_f64 rec;
    int rc = 0;
    std::string err;             // gjkepa_last_error() of the batch, for the caller's thread
    bool done = false;
};
struct Combiner {
    std::mutex mu;
    std::condition_variable cv, cv_lead;
    std::vector<Query*> queue;
    int inflight = 0;            // callers inside gjkepa_query
    bool leader = false;
};
// A new leader waits up to this long for every caller inside gjkepa_query to queue its pair: the
// callers the previous batch just answered come back within microseconds, and one round trip
// costs far more than the wait.
constexpr auto kGatherWait = std::chrono::microseconds(40);

// GJKEPA_QUERY_STATS=1: batch count, mean batch size and mean round trip printed at exit (tuning aid)
struct QueryStats {
    std::atomic<int64_t> batches{0}, queries{0}, ns{0};
    bool on = std::getenv("GJKEPA_QUERY_STATS") != nullptr;
    ~QueryStats() {
        if (on && batches > 0)
            std::fprintf(stderr, "gjkepa_query: %lld batches, %.2f pairs/batch, %.1f us/batch\n", (long long)batches.load(),
                         (double)queries / (double)batches, 1e-3 * (double)ns / (double)batches);
    }
} g_qstats;
std::mutex g_comb_mu;
std::vector<Combiner*> g_comb;

Combiner* combiner(int device) {
    std::lock_guard<std::mutex> g(g_comb_mu);
    if ((int)g_comb.size() <= device) g_comb.resize((size_t)device + 1, nullptr);
    if (!g_comb[(size_t)device]) g_comb[(size_t)device] = new Combiner();
    return g_comb[(size_t)device];
}

// Run one batch of queued queries (all with the same version_ / TOL_FF_) on `device`.  The batch
// is packed straight into pinned host memory as [records | vertices | offsets | counts | pairs],
// copied to the device in one DMA, run, and its records copied back in one DMA.
int run_queries_on(DeviceState* d, std::vector<Query*>& qs, int device) {
    const size_t nq = qs.size();
    if (nq == 0) return 0;
    size_t nv = 0;
    for (Query* q : qs) nv += 3 * (size_t)(q->n1 + q->n2);
    int64_t nlarge = 0;                       // pairs that can park (ws_bytes_for)
    for (Query* q : qs) nlarge += q->n1 > kParkMinHull || q->n2 > kParkMinHull;
    const size_t rec = sizeof(gjkepa_contact_f64);
    const size_t o_v = nq * rec, o_off = o_v + 8 * (nv + 1), o_cnt = o_off + 8 * 2 * nq;
    const size_t o_pr = o_cnt + 4 * 2 * nq, total = o_pr + 4 * 2 * nq;
    std::lock_guard<std::mutex> g(d->mu);
    int rc = init_device(d, device);
    if (rc) return rc;
    hipError_t e;
    if ((e = d->q_host.ensure(total)) != hipSuccess || (e = d->q_blk.ensure(total)) != hipSuccess ||
        (e = d->q_ws.ensure((size_t)ws_bytes_for((int64_t)nq, nlarge))) != hipSuccess)
        return hip_fail(e, "query staging allocation");
    char* h = (char*)d->q_host.p;
    double* v = (double*)(h + o_v);
    int64_t* off = (int64_t*)(h + o_off);
    int32_t* cnt = (int32_t*)(h + o_cnt);
    int32_t* pr = (int32_t*)(h + o_pr);
    size_t o = 0;
    for (size_t j = 0; j < nq; ++j) {
        const Query* q = qs[j];
        off[2 * j] = (int64_t)o;
        cnt[2 * j] = q->n1;
        std::memcpy(v + o, q->p1, sizeof(double) * 3 * (size_t)q->n1);
        o += 3 * (size_t)q->n1;
        off[2 * j + 1] = (int64_t)o;
        cnt[2 * j + 1] = q->n2;
        std::memcpy(v + o, q->p2, sizeof(double) * 3 * (size_t)q->n2);
        o += 3 * (size_t)q->n2;
        pr[2 * j] = (int32_t)(2 * j);
        pr[2 * j + 1] = (int32_t)(2 * j + 1);
    }
    hipStream_t s = d->stream;
    char* dv = (char*)d->q_blk.p;
    if ((e = hipMemcpyAsync(dv + o_v, h + o_v, total - o_v, hipMemcpyHostToDevice, s)) != hipSuccess)
        return hip_fail(e, "hipMemcpyAsync H2D");
    rc = enqueue(qs[0]->version, qs[0]->tol_ff, GJKEPA_DTYPE_F64, GJKEPA_PREC_F64, dv + o_v, (const int64_t*)(dv + o_off),
                 (const int32_t*)(dv + o_cnt), (const int32_t*)(dv + o_pr), (int64_t)nq, dv, d->q_ws.p,
                 (int64_t)d->q_ws.cap, s, d->num_cus);
    if (rc) return rc;
    if ((e = hipMemcpyAsync(h, dv, o_v, hipMemcpyDeviceToHost, s)) != hipSuccess) return hip_fail(e, "hipMemcpyAsync D2H");
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    for (size_t j = 0; j < nq; ++j) std::memcpy(&qs[j]->rec, h + j * rec, rec);
    return 0;
}

void run_queries(std::vector<Query*>& qs, int device) {
    int rc = 0;
    DeviceState* d = device_state(device, &rc);
    if (d) rc = run_queries_on(d, qs, device);
    for (Query* q : qs) {
        q->rc = rc;
        if (rc) q->err = g_err;
    }
}

// ---- resident query service -----------------------------------------------------------------
// gjkepa_query's fast path: a persistent grid (service_kernel) polls GJKEPA_SVC_SLOTS request slots
// in host-mapped memory, one wave per slot.  A caller claims a free slot, writes its hull columns and
// header into it and posts the request's sequence number; the slot's wave answers it with the
// one-wave query path and posts the record back into the slot, which the caller polls.  No launch,
// copy or stream synchronisation per call: one bus read of the request line, one of the hulls and
// the record's write back.  The grid drains by itself after GJKEPA_SVC_IDLE_US without a request
// (or at process exit); the next caller relaunches it.  More concurrent callers than slots, and
// GJKEPA_QUERY_SERVICE=0, take the combining path above.
#ifndef GJKEPA_SVC_IDLE_US
#define GJKEPA_SVC_IDLE_US 2000
#endif
// longest residency of one grid, even under steady traffic: work that a later stream of the process
// puts on the grid's hardware queue waits at most this long (plus one call) behind it
#ifndef GJKEPA_SVC_LIFE_US
#define GJKEPA_SVC_LIFE_US 20000
#endif
struct Service {
    std::mutex mu;                            // launches
    int device = 0, ok = 0;                   // ok: 1 ready, -1 unavailable
    gjkepa_svc_slot* slots = nullptr;         // host view
    gjkepa_svc_slot* dslots = nullptr;        // device view
    gjkepa_svc_ctrl* ctrl = nullptr;          // device memory
    uint32_t* closing = nullptr;              // host-mapped word the draining grid writes its generation to
    uint32_t* dclosing = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t ev = nullptr;                  // recorded after each grid
    std::atomic<uint32_t> gen{0};             // generation of the latest grid (0: none launched)
    std::atomic<uint64_t> free_slots{~0ull >> (64 - GJKEPA_SVC_SLOTS)};
    uint32_t seq[GJKEPA_SVC_SLOTS] = {};      // last posted sequence number, owned by the slot's holder
    uint64_t idle_ticks = 0, life_ticks = 0;
    // grid size: slots 0..grid_n-1 have a wave.  Each launch sizes the grid to the slots claimed since
    // the previous one (callers take the lowest free slot, so that is the recent concurrency), in
    // steps of kSvcGridStep; a caller whose slot has no wave stops the grid and relaunches it larger.
    std::atomic<int> grid_n{0};
    std::atomic<int> hi{0};                   // highest slot + 1 claimed since the last launch
    // slots whose request a failed call left unanswered (a late wave could still read them): held out
    // of use until no grid runs, then marked answered and freed (release_stuck)
    std::atomic<uint64_t> stuck{0};
};
// a grid answering `slot` is not wanted: the service was turned off (gjkepa_query_service_set(0)) while
// the call was in flight; the caller goes through the combining path instead
constexpr int kSvcOff = 1;

// no grid is running (the caller holds sv->mu and has waited for the latest one): every stuck slot's
// request is marked answered, so a later wave (which starts from `done`) never reads it, and the slot
// is free again
void release_stuck(Service* sv) {
    uint64_t m = sv->stuck.exchange(0, std::memory_order_acq_rel);
    while (m) {
        const int k = __builtin_ctzll(m);
        m &= m - 1;
        __atomic_store_n(&sv->slots[k].done, __atomic_load_n(&sv->slots[k].req, __ATOMIC_ACQUIRE), __ATOMIC_RELEASE);
        sv->free_slots.fetch_or(1ull << k, std::memory_order_release);
    }
}
constexpr int kSvcGridStep = 8;
static_assert(GJKEPA_SVC_SLOTS >= 1 && GJKEPA_SVC_SLOTS <= 64, "service slot bitmap");
std::mutex g_svc_mu;
std::vector<Service*> g_svc;
bool g_svc_exit_hook = false;

void service_shutdown() {                     // atexit: every wave sees its stop word and leaves
    std::lock_guard<std::mutex> g(g_svc_mu);
    for (Service* sv : g_svc) {
        if (!sv || sv->ok != 1 || sv->gen.load() == 0) continue;
        for (int k = 0; k < GJKEPA_SVC_SLOTS; ++k) __atomic_store_n(&sv->slots[k].stop, 1u, __ATOMIC_RELEASE);
        (void)hipEventSynchronize(sv->ev);
    }
}

// on unless GJKEPA_QUERY_SERVICE=0; gjkepa_query_service_set() changes it at run time
std::atomic<int> g_svc_on{-1};
bool service_enabled() {
    int on = g_svc_on.load(std::memory_order_relaxed);
    if (on < 0) {
        const char* e = std::getenv("GJKEPA_QUERY_SERVICE");
        int want = !(e && e[0] == '0');
        g_svc_on.compare_exchange_strong(on, want);
        on = g_svc_on.load(std::memory_order_relaxed);
    }
    return on != 0;
}

// lock-free view of the services that are ready (per call: no mutex, no runtime query)
constexpr int kSvcDevMax = 64;
std::atomic<Service*> g_svc_ready[kSvcDevMax];
std::atomic<int> g_ndev{-1};

int device_count_cached() {
    int n = g_ndev.load(std::memory_order_relaxed);
    if (n < 0) {
        if (hipGetDeviceCount(&n) != hipSuccess || n < 0) n = 0;
        g_ndev.store(n, std::memory_order_relaxed);
    }
    return n;
}

// the device's service, set up on first use (nullptr: unavailable, the caller combines instead)
Service* service(int device) {
    if (device >= 0 && device < kSvcDevMax) {
        Service* r = g_svc_ready[device].load(std::memory_order_acquire);
        if (r) return r;
    }
    std::lock_guard<std::mutex> g(g_svc_mu);
    if ((int)g_svc.size() <= device) g_svc.resize((size_t)device + 1, nullptr);
    Service*& sv = g_svc[(size_t)device];
    if (sv) return sv->ok == 1 ? sv : nullptr;
    sv = new Service();
    sv->device = device;
    sv->ok = -1;
    if (hipSetDevice(device) != hipSuccess) return nullptr;
    void* h = nullptr;
    void* hc = nullptr;
    int rate_khz = 0;
    if (hipHostMalloc(&h, sizeof(gjkepa_svc_slot) * GJKEPA_SVC_SLOTS, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
        return nullptr;
    sv->slots = (gjkepa_svc_slot*)h;
    std::memset(h, 0, sizeof(gjkepa_svc_slot) * GJKEPA_SVC_SLOTS);
    if (hipHostMalloc(&hc, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return nullptr;
    sv->closing = (uint32_t*)hc;
    std::memset(hc, 0, 64);
    void* dv = nullptr;
    if (hipHostGetDevicePointer(&dv, h, 0) != hipSuccess) return nullptr;
    sv->dslots = (gjkepa_svc_slot*)dv;
    if (hipHostGetDevicePointer(&dv, hc, 0) != hipSuccess) return nullptr;
    sv->dclosing = (uint32_t*)dv;
    if (hipMalloc(&dv, sizeof(gjkepa_svc_ctrl)) != hipSuccess || hipMemset(dv, 0, sizeof(gjkepa_svc_ctrl)) != hipSuccess)
        return nullptr;
    sv->ctrl = (gjkepa_svc_ctrl*)dv;
    if (hipStreamCreateWithFlags(&sv->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&sv->ev, hipEventDisableTiming) != hipSuccess ||
        hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || rate_khz <= 0)
        return nullptr;
    sv->idle_ticks = (uint64_t)rate_khz * GJKEPA_SVC_IDLE_US / 1000;
    sv->life_ticks = (uint64_t)rate_khz * GJKEPA_SVC_LIFE_US / 1000;
    if (!g_svc_exit_hook) {
        std::atexit(service_shutdown);        // registered after the runtime's own: runs before its teardown
        g_svc_exit_hook = true;
    }
    sv->ok = 1;
    if (device < kSvcDevMax) g_svc_ready[device].store(sv, std::memory_order_release);
    return sv;
}

// make sure a grid that serves `slot` is running: relaunch when none was launched, the latest one is
// draining (it wrote its generation to `closing`), `check_done` and the latest one has finished, or
// the latest one has no wave for `slot` (it is stopped and relaunched larger)
int service_ensure(Service* sv, bool check_done, int slot) {
    const uint32_t g0 = sv->gen.load(std::memory_order_acquire);
    const bool small = g0 != 0 && slot >= sv->grid_n.load(std::memory_order_acquire);
    if (g0 != 0 && __atomic_load_n(sv->closing, __ATOMIC_ACQUIRE) != g0 && !check_done && !small) return 0;
    std::lock_guard<std::mutex> g(sv->mu);
    const uint32_t g1 = sv->gen.load(std::memory_order_relaxed);
    if (g1 != g0) return 0;                   // another caller relaunched meanwhile (a small one: next poll)
    hipError_t e;
    if (g1 != 0) {
        bool need = __atomic_load_n(sv->closing, __ATOMIC_ACQUIRE) == g1 || small;
        if (!need && check_done) {
            e = hipEventQuery(sv->ev);
            if (e != hipSuccess && e != hipErrorNotReady) return hip_fail(e, "query service");
            need = e == hipSuccess;
        }
        if (!need) return 0;
        // a grid too small for this slot leaves once its waves have answered what they hold
        if (small) for (int k = 0; k < GJKEPA_SVC_SLOTS; ++k) __atomic_store_n(&sv->slots[k].stop, 1u, __ATOMIC_RELEASE);
        e = hipEventSynchronize(sv->ev);
        if (small) for (int k = 0; k < GJKEPA_SVC_SLOTS; ++k) __atomic_store_n(&sv->slots[k].stop, 0u, __ATOMIC_RELEASE);
        if (e != hipSuccess) return hip_fail(e, "query service drain");
    }
    release_stuck(sv);                        // no grid runs here
    // turned off (gjkepa_query_service_set(0)) while a call was in flight: no relaunch; the grid has
    // drained, so the caller's slot is no longer read and it combines instead
    if (!service_enabled()) return kSvcOff;
    if ((e = hipSetDevice(sv->device)) != hipSuccess) return hip_fail(e, "hipSetDevice");
    uint32_t ng = g1 + 1;
    if (ng == 0) ng = 1;
    // size: the slots claimed since the last launch and now, and this one, rounded up to the step
    const uint64_t claimed = ~sv->free_slots.load(std::memory_order_acquire) & (~0ull >> (64 - GJKEPA_SVC_SLOTS));
    int want = sv->hi.exchange(claimed ? 64 - __builtin_clzll(claimed) : 0, std::memory_order_relaxed);
    const int now = claimed ? 64 - __builtin_clzll(claimed) : 0;
    want = want > now ? want : now;
    want = want > slot + 1 ? want : slot + 1;
    int n = (want + kSvcGridStep - 1) / kSvcGridStep * kSvcGridStep;
    n = n < kSvcGridStep ? kSvcGridStep : n > GJKEPA_SVC_SLOTS ? GJKEPA_SVC_SLOTS : n;
    gjkepa_svc_args a{sv->dslots, sv->ctrl, sv->dclosing, ng, sv->idle_ticks, sv->life_ticks};
    if ((e = gjkepa_launch_service(a, n, sv->stream)) != hipSuccess) return hip_fail(e, "query service launch");
    if ((e = hipEventRecord(sv->ev, sv->stream)) != hipSuccess) return hip_fail(e, "hipEventRecord");
    sv->grid_n.store(n, std::memory_order_release);
    sv->gen.store(ng, std::memory_order_release);
    return 0;
}

// GJKEPA_QUERY_STATS=1: calls served, mean round trip and mean device time per call, printed at exit
struct ServiceStats {
    std::atomic<int64_t> calls{0}, ns{0}, dev_ticks{0}, tick_khz{0};
    bool on = std::getenv("GJKEPA_QUERY_STATS") != nullptr;
    ~ServiceStats() {
        if (on && calls > 0 && tick_khz > 0)
            std::fprintf(stderr, "gjkepa_query service: %lld calls, %.2f us/call round trip, %.2f us/call on the device\n",
                         (long long)calls.load(), 1e-3 * (double)ns / (double)calls,
                         1e3 * (double)dev_ticks / (double)tick_khz / (double)calls);
    }
} g_sstats;

int service_claim(Service* sv) {
    uint64_t f = sv->free_slots.load(std::memory_order_relaxed);
    while (f) {
        const int k = __builtin_ctzll(f);
        if (sv->free_slots.compare_exchange_weak(f, f & ~(1ull << k), std::memory_order_acquire)) {
            int h = sv->hi.load(std::memory_order_relaxed);
            while (h < k + 1 && !sv->hi.compare_exchange_weak(h, k + 1, std::memory_order_relaxed)) {
            }
            return k;
        }
    }
    return -1;
}

// one pair through slot k; the record lands in *rec
int service_run(Service* sv, int k, int32_t version, double tol_ff, const double* p1, int32_t n1, const double* p2,
                int32_t n2, gjkepa_contact_f64* rec) {
    gjkepa_svc_slot* sl = &sv->slots[k];
    std::memcpy(sl->v, p1, sizeof(double) * 3 * (size_t)n1);
    std::memcpy(sl->v + 3 * (size_t)n1, p2, sizeof(double) * 3 * (size_t)n2);
    sl->version = version;
    sl->na = n1;
    sl->nb = n2;
    sl->tol_ff = tol_ff;
    uint32_t seq = sv->seq[k] + 1;
    if (seq == 0) seq = 1;
    sv->seq[k] = seq;
    __atomic_store_n(&sl->req, seq, __ATOMIC_RELEASE);
    // kSvcOff: no grid runs and none will be launched; an unanswered request is marked answered (the
    // slot's next wave starts from `done`), an answered one is returned as usual
    auto off = [&]() -> int {
        if (__atomic_load_n(&sl->done, __ATOMIC_ACQUIRE) == seq) return 0;
        __atomic_store_n(&sl->done, seq, __ATOMIC_RELEASE);
        return kSvcOff;
    };
    int rc = service_ensure(sv, false, k);
    if (rc == kSvcOff && (rc = off()) != 0) return rc;
    if (rc) return rc;
    const auto t0 = std::chrono::steady_clock::now();
    auto next_check = t0 + std::chrono::microseconds(200);
    bool yield = false;
    for (uint32_t spin = 1; __atomic_load_n(&sl->done, __ATOMIC_ACQUIRE) != seq; ++spin) {
        __builtin_ia32_pause();
        // after twice a typical round trip, give the core away between polls: with more calling
        // threads than cores, the threads whose answers have landed get to run
        if (yield) std::this_thread::yield();
        if ((spin & 63u) == 0) {
            const auto now = std::chrono::steady_clock::now();
            yield = now - t0 > std::chrono::microseconds(80);
            // a grid that reached its idle or lifetime limit marks itself closing: relaunch at once
            if ((rc = service_ensure(sv, false, k)) != 0) {
                if (rc == kSvcOff && (rc = off()) == 0) break;
                return rc;
            }
            if (now >= next_check) {              // the grid may have drained under this request
                if ((rc = service_ensure(sv, true, k)) != 0) {
                    if (rc == kSvcOff && (rc = off()) == 0) break;
                    return rc;
                }
                next_check = now + std::chrono::microseconds(200);
                if (now - t0 > std::chrono::seconds(30)) return fail(GJKEPA_E_HIP, "query service: no answer in 30 s");
            }
        }
    }
    std::memcpy(rec, sl->rec, sizeof(gjkepa_contact_f64));
    if (g_sstats.on) {
        g_sstats.calls += 1;
        g_sstats.ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
        g_sstats.dev_ticks += (int64_t)(sl->t_done - sl->t_seen);
        g_sstats.tick_khz = (int64_t)(sv->idle_ticks * 1000 / GJKEPA_SVC_IDLE_US);
    }
    return 0;
}

}  // namespace

extern "C" {

int gjkepa_query(int32_t version, double tol_ff, const double* p1, int32_t n1, const double* p2, int32_t n2,
                 int8_t* collision, int32_t* colli_type, double* nearest_points, double* collision_normal,
                 double* collision_point, double* penetration_depth, int32_t* status, int32_t device) {
    if (!p1 || !p2 || !collision || !colli_type || !nearest_points || !collision_normal || !collision_point ||
        !penetration_depth)
        return fail(GJKEPA_E_ARG, "null pointer");
    if (n1 < 0 || n2 < 0) return fail(GJKEPA_E_ARG, "negative vertex count");
    int rc = 0;
    Query me{version, tol_ff, p1, p2, n1, n2, {}};
    Service* sv = service_enabled() && n1 >= 1 && n2 >= 1 && n1 <= GJKEPA_MAX_HULL_VERTS && n2 <= GJKEPA_MAX_HULL_VERTS &&
                  device >= 0 && device < device_count_cached() ? service(device) : nullptr;
    const int slot = sv ? service_claim(sv) : -1;
    bool served = false;
    if (slot >= 0) {
        rc = service_run(sv, slot, version, tol_ff, p1, n1, p2, n2, &me.rec);
        // a request that may still be read by a late wave (no answer, or no grid launched) keeps its
        // slot out of use until no grid runs (release_stuck): the next holder would overwrite the hulls
        // under that wave
        if (rc == 0 || rc == kSvcOff || __atomic_load_n(&sv->slots[slot].done, __ATOMIC_ACQUIRE) == sv->seq[slot])
            sv->free_slots.fetch_or(1ull << slot, std::memory_order_release);
        else
            sv->stuck.fetch_or(1ull << slot, std::memory_order_release);
        if (rc != 0 && rc != kSvcOff) return rc;
        served = rc == 0;
    }
    if (!served && !device_state(device, &rc)) return rc;
    if (!served) {
    Combiner* cb = combiner(device);
    {
        std::unique_lock<std::mutex> lk(cb->mu);
        cb->queue.push_back(&me);
        ++cb->inflight;
        cb->cv_lead.notify_one();
        for (;;) {
            cb->cv.wait(lk, [&] { return me.done || !cb->leader; });
            if (me.done) break;
            cb->leader = true;                           // lead one batch: the queued pairs like the first
            const auto until = std::chrono::steady_clock::now() + kGatherWait;
            while ((int)cb->queue.size() < cb->inflight &&
                   cb->cv_lead.wait_until(lk, until) != std::cv_status::timeout) {
            }
            // the queued pairs with the first one's (version_, TOL_FF_), compared bit for bit (a NaN
            // TOL_FF_ joins its own batch); the first pair always leaves the queue
            std::vector<Query*> batch, rest;
            const Query* q0 = cb->queue[0];
            for (Query* q : cb->queue)
                (q == q0 || (q->version == q0->version && std::memcmp(&q->tol_ff, &q0->tol_ff, sizeof(double)) == 0)
                     ? batch : rest).push_back(q);
            cb->queue.swap(rest);
            lk.unlock();
            const auto t0 = std::chrono::steady_clock::now();
            run_queries(batch, device);
            if (g_qstats.on) {
                g_qstats.batches += 1;
                g_qstats.queries += (int64_t)batch.size();
                g_qstats.ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
            }
            lk.lock();
            for (Query* q : batch) q->done = true;
            cb->leader = false;
            cb->cv.notify_all();
        }
        --cb->inflight;
        rc = me.rc;
    }
    if (rc) return fail(rc, me.err);
    }
    const gjkepa_contact_f64& r = me.rec;
    *collision = r.collision;
    *colli_type = r.colli_type;
    // nearest_points_(2,3), Fortran column-major: (1,k) = p1, (2,k) = p2
    for (int k = 0; k < 3; ++k) {
        nearest_points[2 * k] = r.nearest_points[k];
        nearest_points[2 * k + 1] = r.nearest_points[3 + k];
        collision_normal[k] = r.collision_normal[k];
        collision_point[k] = r.collision_point[k];
    }
    *penetration_depth = r.penetration_depth;
    if (status) *status = r.status;
    return 0;
}

int gjkepa_query_service_stop(int32_t device) {
    std::vector<Service*> svs;
    {
        std::lock_guard<std::mutex> g(g_svc_mu);
        for (size_t d = 0; d < g_svc.size(); ++d)
            if (g_svc[d] && g_svc[d]->ok == 1 && (device < 0 || (size_t)device == d)) svs.push_back(g_svc[d]);
    }
    for (Service* sv : svs) {
        std::lock_guard<std::mutex> g(sv->mu);    // no relaunch while the grid drains
        const uint32_t gen = sv->gen.load(std::memory_order_acquire);
        if (gen == 0) continue;
        for (int k = 0; k < GJKEPA_SVC_SLOTS; ++k) __atomic_store_n(&sv->slots[k].stop, 1u, __ATOMIC_RELEASE);
        // every wave answers the request its slot holds, sees its stop word and leaves
        const hipError_t e = hipEventSynchronize(sv->ev);
        for (int k = 0; k < GJKEPA_SVC_SLOTS; ++k) __atomic_store_n(&sv->slots[k].stop, 0u, __ATOMIC_RELEASE);
        if (e == hipSuccess) release_stuck(sv);
        __atomic_store_n(sv->closing, gen, __ATOMIC_RELEASE);   // the next call relaunches
        if (e != hipSuccess) return hip_fail(e, "query service stop");
    }
    return 0;
}

int gjkepa_query_service_resident(int32_t device) {
    std::vector<Service*> svs;
    {
        std::lock_guard<std::mutex> g(g_svc_mu);
        for (size_t d = 0; d < g_svc.size(); ++d)
            if (g_svc[d] && g_svc[d]->ok == 1 && (device < 0 || (size_t)device == d)) svs.push_back(g_svc[d]);
    }
    int resident = 0;
    for (Service* sv : svs) {
        if (sv->gen.load(std::memory_order_acquire) == 0) continue;      // never launched
        const hipError_t e = hipEventQuery(sv->ev);                      // recorded after the latest grid
        if (e == hipErrorNotReady) resident = 1;
        else if (e != hipSuccess) return hip_fail(e, "query service state");
    }
    return resident;
}

int gjkepa_query_service_set(int32_t enabled) {
    const bool prev = service_enabled();
    g_svc_on.store(enabled ? 1 : 0, std::memory_order_relaxed);
    if (!enabled) {
        const int rc = gjkepa_query_service_stop(-1);
        if (rc) return rc;
    }
    return prev ? 1 : 0;
}

// ---- batched convex hulls (include/gjkepa.h) ------------------------------
int64_t gjkepa_hull_face_capacity(int32_t n_points) { return n_points >= 4 ? 2 * (int64_t)n_points - 4 : 0; }

int gjkepa_hull_batch_device(int32_t vert_dtype, const void* points, const int64_t* cloud_off,
                             const int32_t* cloud_cnt, int64_t n_clouds, const int64_t* face_off,
                             int32_t* faces, int32_t* n_faces, int32_t* n_verts, int8_t* status,
                             void* hull_verts, int32_t* vert_idx, void* stream) {
    if (n_clouds < 0 || (vert_dtype != GJKEPA_DTYPE_F32 && vert_dtype != GJKEPA_DTYPE_F64))
        return fail(GJKEPA_E_ARG, "bad n_clouds/dtype");
    if (n_clouds == 0) return 0;
    if (!points || !cloud_off || !cloud_cnt || !face_off || !faces || !n_faces || !n_verts || !status)
        return fail(GJKEPA_E_ARG, "null pointer");
    gjkepa_hull_args a{};
    a.points = points;
    a.cloud_off = cloud_off;
    a.cloud_cnt = cloud_cnt;
    a.n_clouds = n_clouds;
    a.face_off = face_off;
    a.faces = faces;
    a.n_faces = n_faces;
    a.n_verts = n_verts;
    a.status = status;
    a.hull_verts = hull_verts;
    a.vert_idx = vert_idx;
    a.num_cus = num_cus_current();
    hipError_t e = gjkepa_launch_hull(vert_dtype, a, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "hull kernel launch");
}

int gjkepa_hull_batch(int32_t vert_dtype, const void* points, int64_t n_point_scalars,
                      const int64_t* cloud_off, const int32_t* cloud_cnt, int64_t n_clouds,
                      const int64_t* face_off, int64_t n_face_slots, int32_t* faces,
                      int32_t* n_faces, int32_t* n_verts, int8_t* status,
                      void* hull_verts, int32_t* vert_idx, int32_t device) {
    if (n_clouds < 0 || n_point_scalars < 0 || n_face_slots < 0 ||
        (vert_dtype != GJKEPA_DTYPE_F32 && vert_dtype != GJKEPA_DTYPE_F64))
        return fail(GJKEPA_E_ARG, "bad sizes/dtype");
    if (n_clouds == 0) return 0;
    if (!points || !cloud_off || !cloud_cnt || !face_off || !faces || !n_faces || !n_verts || !status)
        return fail(GJKEPA_E_ARG, "null pointer");
    // host-side validation of the index structure (device code trusts it)
    for (int64_t c = 0; c < n_clouds; ++c) {
        const int64_t n = cloud_cnt[c];
        if (n < 4 || n > GJKEPA_HULL_MAX_POINTS) continue;      // answered with BAD_INPUT, nothing read
        if (cloud_off[c] < 0 || cloud_off[c] + 3 * n > n_point_scalars) return fail(GJKEPA_E_ARG, "cloud outside the point pool");
        if (face_off[c] < 0 || face_off[c] + gjkepa_hull_face_capacity((int32_t)n) > n_face_slots)
            return fail(GJKEPA_E_ARG, "cloud's face block outside the face buffer");
    }
    int rc = 0;
    DeviceState* d = device_state(device, &rc);
    if (!d) return rc;
    std::lock_guard<std::mutex> g(d->mu);
    if ((rc = init_device(d, device))) return rc;
    const size_t esz = vert_dtype == GJKEPA_DTYPE_F32 ? 4 : 8;
    const size_t pb = (size_t)n_point_scalars * esz, nc = (size_t)n_clouds;
    hipError_t e;
    if ((e = d->verts.ensure(pb)) != hipSuccess || (e = d->off.ensure(nc * 8)) != hipSuccess ||
        (e = d->cnt.ensure(nc * 4)) != hipSuccess || (e = d->h_foff.ensure(nc * 8)) != hipSuccess ||
        (e = d->h_faces.ensure((size_t)n_face_slots * 12 + 12)) != hipSuccess ||
        (e = d->h_nf.ensure(nc * 4)) != hipSuccess || (e = d->h_nv.ensure(nc * 4)) != hipSuccess ||
        (e = d->h_st.ensure(nc)) != hipSuccess ||
        (hull_verts && (e = d->h_hv.ensure(pb)) != hipSuccess) ||
        (vert_idx && (e = d->h_vi.ensure((size_t)n_point_scalars * 4)) != hipSuccess))
        return hip_fail(e, "hipMalloc");
    hipStream_t s = d->stream;
    if ((e = hipMemcpyAsync(d->verts.p, points, pb, hipMemcpyHostToDevice, s)) != hipSuccess ||
        (e = hipMemcpyAsync(d->off.p, cloud_off, nc * 8, hipMemcpyHostToDevice, s)) != hipSuccess ||
        (e = hipMemcpyAsync(d->cnt.p, cloud_cnt, nc * 4, hipMemcpyHostToDevice, s)) != hipSuccess ||
        (e = hipMemcpyAsync(d->h_foff.p, face_off, nc * 8, hipMemcpyHostToDevice, s)) != hipSuccess)
        return hip_fail(e, "hipMemcpyAsync H2D");
    rc = gjkepa_hull_batch_device(vert_dtype, d->verts.p, (const int64_t*)d->off.p, (const int32_t*)d->cnt.p,
                                  n_clouds, (const int64_t*)d->h_foff.p, (int32_t*)d->h_faces.p,
                                  (int32_t*)d->h_nf.p, (int32_t*)d->h_nv.p, (int8_t*)d->h_st.p,
                                  hull_verts ? d->h_hv.p : nullptr, vert_idx ? (int32_t*)d->h_vi.p : nullptr, s);
    if (rc) return rc;
    if ((e = hipMemcpyAsync(n_faces, d->h_nf.p, nc * 4, hipMemcpyDeviceToHost, s)) != hipSuccess ||
        (e = hipMemcpyAsync(n_verts, d->h_nv.p, nc * 4, hipMemcpyDeviceToHost, s)) != hipSuccess ||
        (e = hipMemcpyAsync(status, d->h_st.p, nc, hipMemcpyDeviceToHost, s)) != hipSuccess ||
        (e = hipStreamSynchronize(s)) != hipSuccess)
        return hip_fail(e, "hipMemcpyAsync D2H");
    // copy back only the written parts: each cloud's faces, hull vertices and vertex indices
    std::vector<int32_t> hf((size_t)n_face_slots * 3);
    std::vector<unsigned char> hh(hull_verts ? pb : 0);
    std::vector<int32_t> hi(vert_idx ? (size_t)n_point_scalars : 0);
    if ((e = hipMemcpyAsync(hf.data(), d->h_faces.p, hf.size() * 4, hipMemcpyDeviceToHost, s)) != hipSuccess ||
        (hull_verts && (e = hipMemcpyAsync(hh.data(), d->h_hv.p, pb, hipMemcpyDeviceToHost, s)) != hipSuccess) ||
        (vert_idx && (e = hipMemcpyAsync(hi.data(), d->h_vi.p, hi.size() * 4, hipMemcpyDeviceToHost, s)) != hipSuccess) ||
        (e = hipStreamSynchronize(s)) != hipSuccess)
        return hip_fail(e, "hipMemcpyAsync D2H");
    for (int64_t c = 0; c < n_clouds; ++c) {
        const int64_t nf = n_faces[c], nv = n_verts[c];
        if (nf) std::memcpy(faces + 3 * face_off[c], hf.data() + 3 * face_off[c], (size_t)nf * 12);
        if (nv && hull_verts)
            std::memcpy((unsigned char*)hull_verts + (size_t)cloud_off[c] * esz, hh.data() + (size_t)cloud_off[c] * esz,
                        (size_t)(3 * nv) * esz);
        if (nv && vert_idx) std::memcpy(vert_idx + cloud_off[c], hi.data() + cloud_off[c], (size_t)nv * 4);
    }
    return 0;
}

// ---- device broad phase (include/gjkepa.h) --------------------------------
int64_t gjkepa_broadphase_workspace_bytes(int64_t n_hulls, int64_t max_pairs) {
    if (n_hulls < 0 || max_pairs < 0 || n_hulls > INT32_MAX - 1 || max_pairs > INT32_MAX) return GJKEPA_E_ARG;
    const int64_t b = gjkepa_broadphase_ws_bytes(n_hulls, max_pairs);
    return b < 0 ? fail(GJKEPA_E_NODEVICE, "workspace query needs a HIP device") : b;
}

int gjkepa_broadphase_device(int32_t vert_dtype, const void* verts, const int64_t* hull_off, const int32_t* hull_cnt,
                             int64_t n_hulls, int32_t* pairs, int64_t max_pairs, int64_t* n_pairs, void* workspace,
                             int64_t workspace_bytes, void* stream) {
    if (n_hulls < 0 || max_pairs < 0 || n_hulls > INT32_MAX - 1 || max_pairs > INT32_MAX ||
        (vert_dtype != GJKEPA_DTYPE_F32 && vert_dtype != GJKEPA_DTYPE_F64))
        return fail(GJKEPA_E_ARG, "bad n_hulls/max_pairs/dtype");
    if (!n_pairs) return fail(GJKEPA_E_ARG, "null pointer");
    hipStream_t s = (hipStream_t)stream;
    hipError_t e;
    if (n_hulls == 0) {
        e = hipMemsetAsync(n_pairs, 0, 8, s);
        return e == hipSuccess ? 0 : hip_fail(e, "hipMemsetAsync");
    }
    if (!verts || !hull_off || !hull_cnt || !workspace || (max_pairs > 0 && !pairs)) return fail(GJKEPA_E_ARG, "null pointer");
    bool small = false;
    e = gjkepa_enqueue_broadphase(vert_dtype, verts, hull_off, hull_cnt, n_hulls, pairs, max_pairs, n_pairs, workspace,
                                  workspace_bytes, s, &small);
    if (e != hipSuccess) return hip_fail(e, "broad phase launch");
    return small ? fail(GJKEPA_E_WORKSPACE, "workspace too small") : 0;
}

int gjkepa_broadphase(int32_t vert_dtype, const void* verts, int64_t n_vert_scalars, const int64_t* hull_off,
                      const int32_t* hull_cnt, int64_t n_hulls, int32_t* pairs, int64_t max_pairs, int64_t* n_pairs,
                      int32_t device) {
    if (n_hulls < 0 || max_pairs < 0 || n_vert_scalars < 0 || n_hulls > INT32_MAX - 1 || max_pairs > INT32_MAX ||
        (vert_dtype != GJKEPA_DTYPE_F32 && vert_dtype != GJKEPA_DTYPE_F64))
        return fail(GJKEPA_E_ARG, "bad sizes/dtype");
    if (!n_pairs || (max_pairs > 0 && !pairs)) return fail(GJKEPA_E_ARG, "null pointer");
    *n_pairs = 0;
    if (n_hulls == 0) return 0;
    if (!verts || !hull_off || !hull_cnt) return fail(GJKEPA_E_ARG, "null pointer");
    for (int64_t h = 0; h < n_hulls; ++h) {
        const int64_t c = hull_cnt[h];
        if (c >= 1 && c <= GJKEPA_MAX_HULL_VERTS && (hull_off[h] < 0 || hull_off[h] + 3 * c > n_vert_scalars))
            return fail(GJKEPA_E_ARG, "hull outside the vertex pool");
    }
    int rc = 0;
    DeviceState* d = device_state(device, &rc);
    if (!d) return rc;
    std::lock_guard<std::mutex> g(d->mu);
    if ((rc = init_device(d, device))) return rc;
    const size_t esz = vert_dtype == GJKEPA_DTYPE_F32 ? 4 : 8;
    const int64_t wsb = gjkepa_broadphase_ws_bytes(n_hulls, max_pairs);
    if (wsb < 0) return fail(GJKEPA_E_HIP, "broad phase workspace query failed");
    hipError_t e;
    if ((e = d->verts.ensure((size_t)n_vert_scalars * esz)) != hipSuccess || (e = d->off.ensure((size_t)n_hulls * 8)) != hipSuccess ||
        (e = d->cnt.ensure((size_t)n_hulls * 4)) != hipSuccess || (e = d->b_pairs.ensure((size_t)max_pairs * 8 + 8)) != hipSuccess ||
        (e = d->b_count.ensure(8)) != hipSuccess || (e = d->b_ws.ensure((size_t)wsb)) != hipSuccess)
        return hip_fail(e, "hipMalloc");
    hipStream_t s = d->stream;
    if ((e = hipMemcpyAsync(d->verts.p, verts, (size_t)n_vert_scalars * esz, hipMemcpyHostToDevice, s)) != hipSuccess ||
        (e = hipMemcpyAsync(d->off.p, hull_off, (size_t)n_hulls * 8, hipMemcpyHostToDevice, s)) != hipSuccess ||
        (e = hipMemcpyAsync(d->cnt.p, hull_cnt, (size_t)n_hulls * 4, hipMemcpyHostToDevice, s)) != hipSuccess)
        return hip_fail(e, "hipMemcpyAsync H2D");
    rc = gjkepa_broadphase_device(vert_dtype, d->verts.p, (const int64_t*)d->off.p, (const int32_t*)d->cnt.p, n_hulls,
                                  (int32_t*)d->b_pairs.p, max_pairs, (int64_t*)d->b_count.p, d->b_ws.p,
                                  (int64_t)d->b_ws.cap, s);
    if (rc) return rc;
    if ((e = hipMemcpyAsync(n_pairs, d->b_count.p, 8, hipMemcpyDeviceToHost, s)) != hipSuccess ||
        (e = hipStreamSynchronize(s)) != hipSuccess)
        return hip_fail(e, "hipMemcpyAsync D2H");
    const int64_t m = *n_pairs < max_pairs ? *n_pairs : max_pairs;
    if (m > 0 && ((e = hipMemcpyAsync(pairs, d->b_pairs.p, (size_t)m * 8, hipMemcpyDeviceToHost, s)) != hipSuccess ||
                  (e = hipStreamSynchronize(s)) != hipSuccess))
        return hip_fail(e, "hipMemcpyAsync D2H");
    return 0;
}

// ---- contact-list compaction (include/gjkepa.h) ---------------------
int64_t gjkepa_compact_workspace_bytes(int64_t n_pairs) {
    if (n_pairs < 0 || n_pairs > INT32_MAX) return GJKEPA_E_ARG;
    const int64_t b = gjkepa_compact_ws_bytes(n_pairs);
    return b < 0 ? fail(GJKEPA_E_NODEVICE, "workspace query needs a HIP device") : b;
}

int gjkepa_compact_hits_device(int32_t precision, const void* records, int64_t n_pairs, int32_t* hit_idx, void* hits,
                               int64_t* n_hits, void* workspace, int64_t workspace_bytes, void* stream) {
    if (n_pairs < 0 || n_pairs > INT32_MAX || (precision != GJKEPA_PREC_F32 && precision != GJKEPA_PREC_F64))
        return fail(GJKEPA_E_ARG, "bad n_pairs/precision");
    if (!n_hits) return fail(GJKEPA_E_ARG, "null pointer");
    hipStream_t s = (hipStream_t)stream;
    hipError_t e;
    if (n_pairs == 0) {
        e = hipMemsetAsync(n_hits, 0, 8, s);
        return e == hipSuccess ? 0 : hip_fail(e, "hipMemsetAsync");
    }
    if (!records || !hit_idx || !workspace) return fail(GJKEPA_E_ARG, "null pointer");
    const int64_t need = gjkepa_compact_ws_bytes(n_pairs);
    if (need < 0) return fail(GJKEPA_E_HIP, "workspace query failed");
    if (workspace_bytes < need) return fail(GJKEPA_E_WORKSPACE, "workspace too small");
    const int rb = gjkepa_record_bytes(precision);
    const int flag = precision == GJKEPA_PREC_F64 ? (int)offsetof(gjkepa_contact_f64, collision)
                                                  : (int)offsetof(gjkepa_contact_f32, collision);
    e = gjkepa_enqueue_compact(records, n_pairs, rb, flag, hit_idx, hits, n_hits, workspace, s);
    return e == hipSuccess ? 0 : hip_fail(e, "compaction launch");
}

// ---- whole collision step: broad phase -> narrow phase -> hit list (host buffers) ---------------
int gjkepa_collide(int32_t version, double tol_ff, int32_t vert_dtype, int32_t precision, const void* verts,
                   int64_t n_vert_scalars, const int64_t* hull_off, const int32_t* hull_cnt, int64_t n_hulls,
                   int32_t* pairs, void* out, int64_t max_contacts, int64_t* n_contacts, int64_t* n_candidates,
                   int32_t device) {
    const gjkepa_internal::Range range_("gjkepa_collide (broad phase, chain, compaction)");
    if (n_hulls < 0 || max_contacts < 0 || n_vert_scalars < 0 || n_hulls > INT32_MAX - 1 || !valid_enums(vert_dtype, precision))
        return fail(GJKEPA_E_ARG, "bad sizes/dtype/precision");
    if (!n_contacts || (max_contacts > 0 && (!pairs || !out))) return fail(GJKEPA_E_ARG, "null pointer");
    *n_contacts = 0;
    if (n_candidates) *n_candidates = 0;
    if (n_hulls == 0) return 0;
    if (!verts || !hull_off || !hull_cnt) return fail(GJKEPA_E_ARG, "null pointer");
    for (int64_t h = 0; h < n_hulls; ++h) {
        const int64_t c = hull_cnt[h];
        if (c >= 1 && c <= GJKEPA_MAX_HULL_VERTS && (hull_off[h] < 0 || hull_off[h] + 3 * c > n_vert_scalars))
            return fail(GJKEPA_E_ARG, "hull outside the vertex pool");
    }
    int rc = 0;
    DeviceState* d = device_state(device, &rc);
    if (!d) return rc;
    std::lock_guard<std::mutex> g(d->mu);
    if ((rc = init_device(d, device))) return rc;
    const size_t esz = vert_dtype == GJKEPA_DTYPE_F32 ? 4 : 8;
    const size_t rec = (size_t)gjkepa_record_bytes(precision);
    hipStream_t s = d->stream;
    hipError_t e;
    if ((e = d->verts.ensure((size_t)n_vert_scalars * esz)) != hipSuccess || (e = d->off.ensure((size_t)n_hulls * 8)) != hipSuccess ||
        (e = d->cnt.ensure((size_t)n_hulls * 4)) != hipSuccess || (e = d->b_count.ensure(8)) != hipSuccess ||
        (e = d->c_n.ensure(8)) != hipSuccess)
        return hip_fail(e, "hipMalloc");
    if ((e = hipMemcpyAsync(d->verts.p, verts, (size_t)n_vert_scalars * esz, hipMemcpyHostToDevice, s)) != hipSuccess ||
        (e = hipMemcpyAsync(d->off.p, hull_off, (size_t)n_hulls * 8, hipMemcpyHostToDevice, s)) != hipSuccess ||
        (e = hipMemcpyAsync(d->cnt.p, hull_cnt, (size_t)n_hulls * 4, hipMemcpyHostToDevice, s)) != hipSuccess)
        return hip_fail(e, "hipMemcpyAsync H2D");
    // broad phase: a list of 8 candidates per hull first; one more pass at the exact size if it was cut
    int64_t cap = n_hulls * 8 > 1024 ? n_hulls * 8 : 1024, ncand = 0;
    for (int pass = 0; pass < 2; ++pass) {
        if (cap > INT32_MAX) return fail(GJKEPA_E_ARG, "candidate list above 2^31-1 pairs");
        const int64_t wsb = gjkepa_broadphase_ws_bytes(n_hulls, cap);
        if (wsb < 0) return fail(GJKEPA_E_HIP, "broad phase workspace query failed");
        if ((e = d->b_pairs.ensure((size_t)cap * 8 + 8)) != hipSuccess || (e = d->b_ws.ensure((size_t)wsb)) != hipSuccess)
            return hip_fail(e, "hipMalloc");
        rc = gjkepa_broadphase_device(vert_dtype, d->verts.p, (const int64_t*)d->off.p, (const int32_t*)d->cnt.p,
                                      n_hulls, (int32_t*)d->b_pairs.p, cap, (int64_t*)d->b_count.p, d->b_ws.p,
                                      (int64_t)d->b_ws.cap, s);
        if (rc) return rc;
        if ((e = hipMemcpyAsync(&ncand, d->b_count.p, 8, hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipStreamSynchronize(s)) != hipSuccess)
            return hip_fail(e, "hipMemcpyAsync D2H");
        if (ncand <= cap) break;
        cap = ncand;
    }
    if (n_candidates) *n_candidates = ncand;
    if (ncand == 0) return 0;
    // narrow phase on the device-resident list, then the dense hit list
    // park slots: the candidates can only reach the parking EPA tiers when some hull is above their
    // capacity (the pairs are on the device; the share is taken over every candidate then)
    bool large = false;
    for (int64_t h = 0; h < n_hulls && !large; ++h) large = hull_cnt[h] > kParkMinHull;
    const int64_t wsn = ws_bytes_for(ncand, large ? ncand : 0), wsc = gjkepa_compact_ws_bytes(ncand);
    if (wsc < 0) return fail(GJKEPA_E_HIP, "compaction workspace query failed");
    if ((e = d->out.ensure((size_t)ncand * rec)) != hipSuccess || (e = d->ws.ensure((size_t)wsn)) != hipSuccess ||
        (e = d->c_idx.ensure((size_t)ncand * 4)) != hipSuccess || (e = d->c_hits.ensure((size_t)ncand * rec)) != hipSuccess ||
        (e = d->c_ws.ensure((size_t)wsc)) != hipSuccess)
        return hip_fail(e, "hipMalloc");
    if ((rc = enqueue(version, tol_ff, vert_dtype, precision, d->verts.p, (const int64_t*)d->off.p,
                      (const int32_t*)d->cnt.p, (const int32_t*)d->b_pairs.p, ncand, d->out.p, d->ws.p,
                      (int64_t)d->ws.cap, s, d->num_cus)))
        return rc;
    const int flag = precision == GJKEPA_PREC_F64 ? (int)offsetof(gjkepa_contact_f64, collision)
                                                  : (int)offsetof(gjkepa_contact_f32, collision);
    if ((e = gjkepa_enqueue_compact(d->out.p, ncand, (int)rec, flag, (int32_t*)d->c_idx.p, d->c_hits.p,
                                    (int64_t*)d->c_n.p, d->c_ws.p, s)) != hipSuccess)
        return hip_fail(e, "compaction launch");
    int64_t nh = 0;
    if ((e = hipMemcpyAsync(&nh, d->c_n.p, 8, hipMemcpyDeviceToHost, s)) != hipSuccess ||
        (e = hipStreamSynchronize(s)) != hipSuccess)
        return hip_fail(e, "hipMemcpyAsync D2H");
    *n_contacts = nh;
    const int64_t m = nh < max_contacts ? nh : max_contacts;
    if (m > 0) {
        std::vector<int32_t> idx((size_t)m), cand((size_t)ncand * 2);
        if ((e = hipMemcpyAsync(idx.data(), d->c_idx.p, (size_t)m * 4, hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipMemcpyAsync(cand.data(), d->b_pairs.p, (size_t)ncand * 8, hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipMemcpyAsync(out, d->c_hits.p, (size_t)m * rec, hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipStreamSynchronize(s)) != hipSuccess)
            return hip_fail(e, "hipMemcpyAsync D2H");
        for (int64_t k = 0; k < m; ++k) {
            pairs[2 * k] = cand[2 * (size_t)idx[k]];
            pairs[2 * k + 1] = cand[2 * (size_t)idx[k] + 1];
        }
    }
    return 0;
}

}  // extern "C"
