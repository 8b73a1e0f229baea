// synth.cpp — deterministic synthetic pair workloads (SURVEY.md §8d configs C2–C5).
//
// Counter-based SplitMix64: every value is a pure function of (seed, global pair index, draw
// number), so any shard [first_pair, first_pair + n_pairs) of a job reproduces exactly the pairs a
// single-GPU run of the whole job would see.  Vertices are unit vectors about the hull centre
// (every vertex extreme), hull A at the origin, hull B at u*r (u uniform on S^2, r ~ U[0, r_max]).
// All coordinates are rounded to fp32 so fp32 and fp64 pools hold the same numbers.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/gjkepa.h"

namespace {

inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

struct PairRng {
    uint64_t key;
    uint64_t ctr = 0;
    PairRng(uint64_t seed, int64_t pair) : key(splitmix64(seed ^ splitmix64((uint64_t)pair * 0xD1B54A32D192ED03ull + 1))) {}
    double u01() { return (double)(splitmix64(key + 0x9E3779B97F4A7C15ull * (++ctr)) >> 11) * 0x1.0p-53; }
};

constexpr double kTwoPi = 6.283185307179586476925286766559;

inline void unit_vec(PairRng& g, double* v) {
    double z = 2.0 * g.u01() - 1.0;
    double phi = kTwoPi * g.u01();
    double s = std::sqrt(std::fmax(0.0, 1.0 - z * z));
    v[0] = s * std::cos(phi);
    v[1] = s * std::sin(phi);
    v[2] = z;
}

inline int32_t draw_n(PairRng& g, int32_t n_min, int32_t n_max) {
    if (n_max <= n_min) return n_min;
    int32_t span = n_max - n_min + 1;
    int32_t k = (int32_t)(g.u01() * span);
    return n_min + (k >= span ? span - 1 : k);
}

}  // namespace

extern "C" int64_t gjkepa_synth_pairs(uint64_t seed, int64_t first_pair, int64_t n_pairs,
                                      int32_t n_min, int32_t n_max, double r_max,
                                      int32_t vert_dtype, void* verts,
                                      int64_t* hull_off, int32_t* hull_cnt, int32_t* pairs) {
    if (n_pairs < 0 || n_min < 1 || n_max < n_min || n_max > GJKEPA_MAX_HULL_VERTS) return GJKEPA_E_ARG;
    if (vert_dtype != GJKEPA_DTYPE_F32 && vert_dtype != GJKEPA_DTYPE_F64) return GJKEPA_E_ARG;
    // pass 1: sizes (first draws of every pair's stream)
    std::vector<int32_t> cnt((size_t)(2 * n_pairs));
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < n_pairs; ++k) {
        PairRng g(seed, first_pair + k);
        cnt[2 * k] = draw_n(g, n_min, n_max);
        cnt[2 * k + 1] = draw_n(g, n_min, n_max);
    }
    std::vector<int64_t> off((size_t)(2 * n_pairs) + 1);
    off[0] = 0;
    for (int64_t h = 0; h < 2 * n_pairs; ++h) off[h + 1] = off[h] + 3 * (int64_t)cnt[h];
    const int64_t total = off[2 * n_pairs];
    if (!verts) return total;
    if (!hull_off || !hull_cnt || !pairs) return GJKEPA_E_ARG;
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < n_pairs; ++k) {
        PairRng g(seed, first_pair + k);
        int32_t na = draw_n(g, n_min, n_max), nb = draw_n(g, n_min, n_max);
        double u[3];
        unit_vec(g, u);
        double r = r_max * g.u01();
        double c[3] = {u[0] * r, u[1] * r, u[2] * r};
        for (int side = 0; side < 2; ++side) {
            int32_t n = side ? nb : na;
            int64_t o = off[2 * k + side];
            for (int32_t i = 0; i < n; ++i) {
                double v[3];
                unit_vec(g, v);
                for (int d = 0; d < 3; ++d) {
                    float val = (float)(side ? v[d] + c[d] : v[d]);
                    if (vert_dtype == GJKEPA_DTYPE_F32) ((float*)verts)[o + (int64_t)d * n + i] = val;
                    else ((double*)verts)[o + (int64_t)d * n + i] = (double)val;
                }
            }
            hull_off[2 * k + side] = o;
            hull_cnt[2 * k + side] = n;
        }
        pairs[2 * k] = (int32_t)(2 * k);
        pairs[2 * k + 1] = (int32_t)(2 * k + 1);
    }
    return total;
}

// Point clouds for the batched hull module: cloud c has n ~ U{n_min..n_max}
// points, uniform in the unit ball (shape 0: mostly interior points, a raw scan-like cloud) or on
// the unit sphere (shape 1: every point extreme, the hull's worst case).  Same counter-based
// streams as the pairs (keyed by the global cloud index), coordinates rounded to fp32.
extern "C" int64_t gjkepa_synth_clouds(uint64_t seed, int64_t first_cloud, int64_t n_clouds,
                                       int32_t n_min, int32_t n_max, int32_t shape,
                                       int32_t vert_dtype, void* verts,
                                       int64_t* cloud_off, int32_t* cloud_cnt) {
    if (n_clouds < 0 || n_min < 1 || n_max < n_min || n_max > GJKEPA_HULL_MAX_POINTS || (shape != 0 && shape != 1))
        return GJKEPA_E_ARG;
    if (vert_dtype != GJKEPA_DTYPE_F32 && vert_dtype != GJKEPA_DTYPE_F64) return GJKEPA_E_ARG;
    std::vector<int32_t> cnt((size_t)n_clouds);
#pragma omp parallel for schedule(static)
    for (int64_t c = 0; c < n_clouds; ++c) {
        PairRng g(seed ^ 0xC10D5ull, first_cloud + c);
        cnt[c] = draw_n(g, n_min, n_max);
    }
    std::vector<int64_t> off((size_t)n_clouds + 1);
    off[0] = 0;
    for (int64_t c = 0; c < n_clouds; ++c) off[c + 1] = off[c] + 3 * (int64_t)cnt[c];
    const int64_t total = off[n_clouds];
    if (!verts) return total;
    if (!cloud_off || !cloud_cnt) return GJKEPA_E_ARG;
#pragma omp parallel for schedule(static)
    for (int64_t c = 0; c < n_clouds; ++c) {
        PairRng g(seed ^ 0xC10D5ull, first_cloud + c);
        const int32_t n = draw_n(g, n_min, n_max);
        const int64_t o = off[c];
        for (int32_t i = 0; i < n; ++i) {
            double v[3];
            unit_vec(g, v);
            const double r = shape == 0 ? std::cbrt(g.u01()) : 1.0;
            for (int d = 0; d < 3; ++d) {
                const float val = (float)(v[d] * r);
                if (vert_dtype == GJKEPA_DTYPE_F32) ((float*)verts)[o + (int64_t)d * n + i] = val;
                else ((double*)verts)[o + (int64_t)d * n + i] = (double)val;
            }
        }
        cloud_off[c] = o;
        cloud_cnt[c] = n;
    }
    return total;
}

// Scene for the broad phase: hull h has n ~ U{n_min..n_max} unit-sphere
// vertices about a centre uniform in [0, box)^3.  Streams keyed by the global hull index.
extern "C" int64_t gjkepa_synth_scene(uint64_t seed, int64_t first_hull, int64_t n_hulls,
                                      int32_t n_min, int32_t n_max, double box,
                                      int32_t vert_dtype, void* verts, int64_t* hull_off, int32_t* hull_cnt) {
    if (n_hulls < 0 || n_min < 1 || n_max < n_min || n_max > GJKEPA_MAX_HULL_VERTS || !(box >= 0.0)) return GJKEPA_E_ARG;
    if (vert_dtype != GJKEPA_DTYPE_F32 && vert_dtype != GJKEPA_DTYPE_F64) return GJKEPA_E_ARG;
    std::vector<int32_t> cnt((size_t)n_hulls);
#pragma omp parallel for schedule(static)
    for (int64_t h = 0; h < n_hulls; ++h) {
        PairRng g(seed ^ 0x5CE7Eull, first_hull + h);
        cnt[h] = draw_n(g, n_min, n_max);
    }
    std::vector<int64_t> off((size_t)n_hulls + 1);
    off[0] = 0;
    for (int64_t h = 0; h < n_hulls; ++h) off[h + 1] = off[h] + 3 * (int64_t)cnt[h];
    const int64_t total = off[n_hulls];
    if (!verts) return total;
    if (!hull_off || !hull_cnt) return GJKEPA_E_ARG;
#pragma omp parallel for schedule(static)
    for (int64_t h = 0; h < n_hulls; ++h) {
        PairRng g(seed ^ 0x5CE7Eull, first_hull + h);
        const int32_t n = draw_n(g, n_min, n_max);
        const double c[3] = {box * g.u01(), box * g.u01(), box * g.u01()};
        const int64_t o = off[h];
        for (int32_t i = 0; i < n; ++i) {
            double v[3];
            unit_vec(g, v);
            for (int d = 0; d < 3; ++d) {
                const float val = (float)(v[d] + c[d]);
                if (vert_dtype == GJKEPA_DTYPE_F32) ((float*)verts)[o + (int64_t)d * n + i] = val;
                else ((double*)verts)[o + (int64_t)d * n + i] = (double)val;
            }
        }
        hull_off[h] = o;
        hull_cnt[h] = n;
    }
    return total;
}
