/* Host sanitizer driver (ASan/UBSan on host code).  Built with
 * -fsanitize=address,undefined by tests/test_sanitizers.py together with the oracle restatement
 * (test infrastructure) and the product's host-side workload generators (csrc/synth.cpp), then
 * run over generated pair pools, point clouds and scenes: any out-of-bounds access, leak or
 * undefined behaviour aborts with a sanitizer report. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../include/gjkepa.h"
#include "../../oracle/gjkepa_oracle.h"

static int pairs_case(int n, int lo, int hi, double r) {
    int64_t total = gjkepa_synth_pairs(7, 0, n, lo, hi, r, GJKEPA_DTYPE_F64, NULL, NULL, NULL, NULL);
    double* v = malloc(sizeof(double) * (size_t)total);
    int64_t* off = malloc(sizeof(int64_t) * 2 * (size_t)n);
    int32_t* cnt = malloc(sizeof(int32_t) * 2 * (size_t)n);
    int32_t* prs = malloc(sizeof(int32_t) * 2 * (size_t)n);
    gjkepa_contact_f64* out = malloc(sizeof(gjkepa_contact_f64) * (size_t)n);
    gjkepa_synth_pairs(7, 0, n, lo, hi, r, GJKEPA_DTYPE_F64, v, off, cnt, prs);
    int hits = 0;
    for (int version = 1; version <= 3; ++version) {
        if (oracle_gjkepa_batch(version, 1.0, GJKEPA_DTYPE_F64, v, off, cnt, prs, n, out, 2)) return 1;
        for (int k = 0; k < n; ++k) hits += out[k].collision != 0;
    }
    printf("pairs %d (%d-%d verts, r %.1f): %d hits over 3 versions\n", n, lo, hi, r, hits);
    free(v); free(off); free(cnt); free(prs); free(out);
    return 0;
}

static int clouds_case(int n, int lo, int hi, int shape) {
    int64_t total = gjkepa_synth_clouds(9, 0, n, lo, hi, shape, GJKEPA_DTYPE_F32, NULL, NULL, NULL);
    float* v = malloc(sizeof(float) * (size_t)total);
    int64_t* off = malloc(sizeof(int64_t) * (size_t)n);
    int32_t* cnt = malloc(sizeof(int32_t) * (size_t)n);
    gjkepa_synth_clouds(9, 0, n, lo, hi, shape, GJKEPA_DTYPE_F32, v, off, cnt);
    int64_t* foff = malloc(sizeof(int64_t) * (size_t)n);
    int64_t slots = 0;
    for (int c = 0; c < n; ++c) { foff[c] = slots; slots += 2 * (int64_t)cnt[c] - 4; }
    int32_t* faces = malloc(sizeof(int32_t) * 3 * (size_t)slots);
    int32_t* nf = malloc(sizeof(int32_t) * (size_t)n);
    int32_t* nv = malloc(sizeof(int32_t) * (size_t)n);
    int8_t* st = malloc((size_t)n);
    float* hv = malloc(sizeof(float) * (size_t)total);
    int32_t* vi = malloc(sizeof(int32_t) * (size_t)total);
    if (oracle_hull_batch(GJKEPA_DTYPE_F32, v, off, cnt, n, foff, faces, nf, nv, st, hv, vi, 2)) return 1;
    int64_t tf = 0;
    for (int c = 0; c < n; ++c) tf += nf[c];
    printf("clouds %d (%d-%d pts, shape %d): %lld faces\n", n, lo, hi, shape, (long long)tf);
    free(v); free(off); free(cnt); free(foff); free(faces); free(nf); free(nv); free(st); free(hv); free(vi);
    return 0;
}

static int scene_case(int n, double box) {
    int64_t total = gjkepa_synth_scene(11, 0, n, 8, 48, box, GJKEPA_DTYPE_F64, NULL, NULL, NULL);
    double* v = malloc(sizeof(double) * (size_t)total);
    int64_t* off = malloc(sizeof(int64_t) * (size_t)n);
    int32_t* cnt = malloc(sizeof(int32_t) * (size_t)n);
    gjkepa_synth_scene(11, 0, n, 8, 48, box, GJKEPA_DTYPE_F64, v, off, cnt);
    int64_t found = 0;
    if (oracle_broadphase(GJKEPA_DTYPE_F64, v, off, cnt, n, NULL, 0, &found, 2)) return 1;
    int32_t* prs = malloc(sizeof(int32_t) * 2 * (size_t)(found + 1));
    if (oracle_broadphase(GJKEPA_DTYPE_F64, v, off, cnt, n, prs, found, &found, 2)) return 1;
    printf("scene %d hulls: %lld pairs\n", n, (long long)found);
    free(v); free(off); free(cnt); free(prs);
    return 0;
}

int main(void) {
    if (pairs_case(300, 32, 32, 2.5) || pairs_case(60, 8, 256, 2.5) || pairs_case(100, 32, 128, 0.3)) return 1;
    if (clouds_case(200, 4, 64, 0) || clouds_case(20, 200, 256, 1)) return 1;
    if (scene_case(2000, 20.0)) return 1;
    puts("sanitizers clean");
    return 0;
}
