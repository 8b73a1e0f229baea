// gjkepa_multi.cpp — multi-GPU entries of include/gjkepa.h (SURVEY.md §8 row e).
//
// Pairs are independent, so a job shards into contiguous blocks of pairs with no exchange during
// compute (gjkepa_shard_range).  Two ways to drive a node:
//   * one process, several devices (gjkepa_batch_multi; Fortran GJKEPA_BATCH(..., devices_)): the
//     reference's caller is one Fortran process whose parallelism is its own OpenMP loop
//     (GCLIB_GJKEPA.f90:9, :16, :55-60).  One host thread per device runs gjkepa_batch on that
//     device's shard; each shard's records are copied straight into the caller's array, which is
//     the gather.  Only the hulls a shard references travel to its device.
//   * one process per device (gjkepa_comm_* + gjkepa_allgather_records_device): each rank runs
//     gjkepa_batch_device on its shard and the fixed-size records are all-gathered in rank order
//     with one RCCL ncclAllGather over xGMI (config C3).
// RCCL is bound at run time: the RCCL already in the process (e.g. PyTorch's) or else /opt/rocm's
// librccl.so.1 loaded privately, so the library links against neither and a Python process uses
// the same RCCL as torch.distributed.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/gjkepa.h"
#include "capi_internal.h"

namespace {

using gjkepa_internal::set_error;

// ---- RCCL, bound at run time ---------------------------------------------------------------------
struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    const char* source = "";
    bool ok = false;
};

template <typename F> bool bind(void* h, const char* name, F& f) {
    f = reinterpret_cast<F>(dlsym(h, name));
    return f != nullptr;
}

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        // Prefer an RCCL the process already holds: one linked into the program (global scope), or
        // PyTorch's (its libtorch_hip NEEDs "librccl.so"; Python loads it RTLD_LOCAL, so only
        // RTLD_NOLOAD finds it).  Otherwise load ROCm's privately (RTLD_LOCAL), so it can never
        // interpose on another copy's symbols.
        void* h = nullptr;
        if (dlsym(RTLD_DEFAULT, "ncclCommInitRank")) { h = RTLD_DEFAULT; r.source = "process (global)"; }
        if (!h && (h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD))) r.source = "process (librccl.so)";
        if (!h && (h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD))) r.source = "process (librccl.so.1)";
        if (!h && (h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL))) r.source = "librccl.so.1";
        if (!h && (h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL))) r.source = "/opt/rocm/lib/librccl.so.1";
        if (!h) return;
        r.ok = bind(h, "ncclGetUniqueId", r.get_unique_id) && bind(h, "ncclCommInitRank", r.comm_init_rank) &&
               bind(h, "ncclCommDestroy", r.comm_destroy) && bind(h, "ncclAllGather", r.all_gather) &&
               bind(h, "ncclGetErrorString", r.error_string);
    });
    return r;
}

int nccl_fail(ncclResult_t e, const char* what) {
    const Rccl& r = rccl();
    return set_error(GJKEPA_E_COMM, std::string(what) + ": " + (r.error_string ? r.error_string(e) : "RCCL error"));
}

}  // namespace

struct gjkepa_comm {
    ncclComm_t comm = nullptr;
    int world = 0, rank = 0, device = 0;
};

extern "C" {

int gjkepa_shard_range(int64_t n_pairs, int32_t world, int32_t rank, int64_t* first, int64_t* count) {
    if (n_pairs < 0 || world < 1 || rank < 0 || rank >= world || !first || !count)
        return set_error(GJKEPA_E_ARG, "bad shard arguments");
    const int64_t base = n_pairs / world, extra = n_pairs % world;
    *first = rank * base + std::min<int64_t>(rank, extra);
    *count = base + (rank < extra ? 1 : 0);
    return 0;
}

int gjkepa_batch_multi(int32_t version, double tol_ff, int32_t vert_dtype, int32_t precision,
                       const void* verts, int64_t n_vert_scalars, const int64_t* hull_off,
                       const int32_t* hull_cnt, int64_t n_hulls, const int32_t* pairs, int64_t n_pairs,
                       void* out, const int32_t* devices, int32_t ndev) {
    const gjkepa_internal::Range range_("gjkepa_batch_multi (shards on devices)");
    if (ndev < 1 || !devices) return set_error(GJKEPA_E_ARG, "empty device list");
    if (n_pairs < 0 || n_hulls < 0 || n_vert_scalars < 0) return set_error(GJKEPA_E_ARG, "bad sizes");
    const int rb = gjkepa_record_bytes(precision);
    if (rb < 0 || (vert_dtype != GJKEPA_DTYPE_F32 && vert_dtype != GJKEPA_DTYPE_F64))
        return set_error(GJKEPA_E_ARG, "bad dtype/precision");
    if (n_pairs == 0) return 0;
    if (!verts || !hull_off || !hull_cnt || !pairs || !out) return set_error(GJKEPA_E_ARG, "null pointer");
    // the same argument checks as one gjkepa_batch call over the whole job, before any shard runs
    // (a shard's own call sees only its rebased slice of the pool)
    for (int64_t k = 0; k < 2 * n_pairs; ++k)
        if (pairs[k] < 0 || pairs[k] >= n_hulls) return set_error(GJKEPA_E_ARG, "pair references a missing hull");
    for (int64_t h = 0; h < n_hulls; ++h) {
        const int64_t c = hull_cnt[h];
        if (c >= 1 && (hull_off[h] < 0 || hull_off[h] + 3 * c > n_vert_scalars))
            return set_error(GJKEPA_E_ARG, "hull outside the vertex pool");
    }
    // A device may be listed more than once: its shards then run one after the other (gjkepa_batch
    // serialises the calls on one device), which also lets one GPU run any shard count.
    const size_t esz = vert_dtype == GJKEPA_DTYPE_F32 ? 4 : 8;
    std::vector<int> rc((size_t)ndev, 0);
    std::vector<std::string> msg((size_t)ndev);
    auto shard = [&](int s) {
        int64_t first = 0, count = 0;
        gjkepa_shard_range(n_pairs, ndev, s, &first, &count);
        if (count == 0) return;
        // the hulls this shard references: index range [hmin, hmax], vertex scalars [vlo, vhi)
        int32_t hmin = INT32_MAX, hmax = -1;
        for (int64_t k = 2 * first; k < 2 * (first + count); ++k) {
            hmin = std::min(hmin, pairs[k]);
            hmax = std::max(hmax, pairs[k]);
        }
        int64_t vlo = INT64_MAX, vhi = 0;
        for (int64_t h = hmin; h <= hmax; ++h) {
            const int64_t c = hull_cnt[h];
            if (c < 1) continue;                 // empty: answered BAD_INPUT, never read
            vlo = std::min(vlo, hull_off[h]);
            vhi = std::max(vhi, hull_off[h] + 3 * c);
        }
        if (vhi == 0) vlo = 0;
        const int64_t nh = (int64_t)hmax - hmin + 1;
        std::vector<int64_t> off((size_t)nh);
        std::vector<int32_t> prs((size_t)(2 * count));
        for (int64_t h = 0; h < nh; ++h) off[(size_t)h] = hull_off[hmin + h] - vlo;
        for (int64_t k = 0; k < 2 * count; ++k) prs[(size_t)k] = pairs[2 * first + k] - hmin;
        rc[(size_t)s] = gjkepa_batch(version, tol_ff, vert_dtype, precision, (const char*)verts + (size_t)vlo * esz,
                                     std::max<int64_t>(vhi - vlo, 0), off.data(), hull_cnt + hmin, nh, prs.data(),
                                     count, (char*)out + (size_t)first * (size_t)rb, devices[s]);
        if (rc[(size_t)s]) msg[(size_t)s] = gjkepa_last_error();
    };
    std::vector<std::thread> th;
    for (int s = 1; s < ndev; ++s) th.emplace_back(shard, s);
    shard(0);
    for (auto& t : th) t.join();
    for (int s = 0; s < ndev; ++s)
        if (rc[(size_t)s]) return set_error(rc[(size_t)s], "device " + std::to_string(devices[s]) + ": " + msg[(size_t)s]);
    return 0;
}

int gjkepa_comm_unique_id(void* id) {
    if (!id) return set_error(GJKEPA_E_ARG, "null pointer");
    const Rccl& r = rccl();
    if (!r.ok) return set_error(GJKEPA_E_COMM, "RCCL not available (librccl.so.1)");
    ncclUniqueId u;
    const ncclResult_t e = r.get_unique_id(&u);
    if (e != ncclSuccess) return nccl_fail(e, "ncclGetUniqueId");
    std::memcpy(id, &u, sizeof(u));
    return 0;
}

int gjkepa_comm_init(gjkepa_comm** comm, int32_t world, int32_t rank, const void* id, int32_t device) {
    if (!comm || !id || world < 1 || rank < 0 || rank >= world) return set_error(GJKEPA_E_ARG, "bad comm arguments");
    *comm = nullptr;
    const Rccl& r = rccl();
    if (!r.ok) return set_error(GJKEPA_E_COMM, "RCCL not available (librccl.so.1)");
    hipError_t he = hipSetDevice(device);
    if (he != hipSuccess) return set_error(GJKEPA_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(he));
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    gjkepa_comm* c = new gjkepa_comm();
    const ncclResult_t e = r.comm_init_rank(&c->comm, world, u, rank);
    if (e != ncclSuccess) {
        delete c;
        return nccl_fail(e, "ncclCommInitRank");
    }
    c->world = world;
    c->rank = rank;
    c->device = device;
    *comm = c;
    return 0;
}

int gjkepa_comm_destroy(gjkepa_comm* comm) {
    if (!comm) return 0;
    const Rccl& r = rccl();
    ncclResult_t e = ncclSuccess;
    if (r.ok && comm->comm) e = r.comm_destroy(comm->comm);
    delete comm;
    return e == ncclSuccess ? 0 : nccl_fail(e, "ncclCommDestroy");
}

int gjkepa_allgather_records_device(gjkepa_comm* comm, int32_t precision, const void* shard_records,
                                    void* all_records, int64_t count, void* stream) {
    const gjkepa_internal::Range range_("gjkepa_allgather_records_device (RCCL all-gather enqueue)");
    const int rb = gjkepa_record_bytes(precision);
    if (!comm || rb < 0 || count < 0) return set_error(GJKEPA_E_ARG, "bad allgather arguments");
    if (count == 0) return 0;
    if (!shard_records || !all_records) return set_error(GJKEPA_E_ARG, "null pointer");
    const ncclResult_t e = rccl().all_gather(shard_records, all_records, (size_t)count * (size_t)rb, ncclUint8,
                                             comm->comm, (hipStream_t)stream);
    return e == ncclSuccess ? 0 : nccl_fail(e, "ncclAllGather");
}

const char* gjkepa_comm_backend(void) {
    const Rccl& r = rccl();
    return r.ok ? r.source : "unavailable";
}

}  // extern "C"
