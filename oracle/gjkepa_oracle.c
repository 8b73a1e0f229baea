/*
 * gjkepa_oracle.c — TEST INFRASTRUCTURE ONLY (see gjkepa_oracle.h).
 *
 * A from-scratch scalar fp64 restatement of the reference path in src/GCLIB_GJKEPA.f90
 * (xiejihong0306/collision-detect-GJK-EPA).  Every function cites the reference lines it follows.
 * It is the checker for the HIP kernels and the CPU baseline of bench.py; the product never
 * links it.  PARITY UNPINNED (reference unbuildable here, no reference tests): see DESIGN.md.
 *
 * Arithmetic contract (shared with the kernels so results can be compared bit for bit):
 *   dot(a,b)   = (a.x*b.x + a.y*b.y) + a.z*b.z      (DOT_PRODUCT, left to right)
 *   norm2(a)   = sqrt((a.x*a.x + a.y*a.y) + a.z*a.z) (NORM2)
 *   sums       = sequential in index order           (SUM)
 *   no FMA contraction (built with -ffp-contract=off), no fast-math.
 *
 * The one component the reference does not contain is the convex hull the EPA rebuilds every
 * iteration (GCLIB_QuickHull::QuickHull + GCLIB_DeHull::getHullMeshesVertex, used at :920,
 * :950; unvendored, no version pin).  It is re-supplied here with the published semantics of
 * QuickHull — the convex hull of (hull vertices ∪ new support point(s)) as outward triangles,
 * points within HULL_EPS of the hull dropped — computed incrementally (remove the faces the new
 * point sees, cone the horizon).  Face order (it only matters for exact MINLOC ties): surviving
 * faces keep their order, new faces follow in (visible-face order, edge 0..2) order.
 */
#include "gjkepa_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---- tolerances ---------------------------------------------------- */
#ifndef ORC_F32
#define TOL_PT   1.0e-8   /* coincidence / coplanar / collinear / on-plane / EPA convergence */
#define TOL_Z    1.0e-12  /* UTZVEC / UNINML / DIST_PF_SIGN zero */
#define TOL_ZO   1.0e-12  /* EPA orientation, origin-on-face (:905, :910, :935) */
#define TOL_POS  1.0e-15  /* IS_INSIDE_PF "positive" (:1306) */
#define HULL_EPS 1.0e-10  /* re-supplied QuickHull: visibility / coplanarity threshold */
#else
/* Diagnostic build (oracle/Makefile: libgjkepa_oracle_f32.so): the same restatement in fp32
 * arithmetic with the kernels' fp32 tolerances (csrc/gk_common.h Tol<float>), to study the fp32
 * compute path on the CPU.  Every `double` below this point is a float; records stay fp64 structs. */
#define TOL_PT   1.0e-6f
#define TOL_Z    1.0e-12f
#define TOL_ZO   1.0e-6f
#define TOL_POS  1.0e-15f
#define HULL_EPS 2.0e-6f
#define double float
#endif
typedef double oreal;     /* the narrow phase's arithmetic type (float in the ORC_F32 build) */
#define INIT_MAXIT 99     /* :86 */
#define GJK_MAXIT  50     /* :186 */
#define EPA_MAXIT  99     /* :299 */
#define SPHERE_TOL 1.0    /* :1172 */
#define SUPPORT_BAND 1.0e-1 /* :471-472, :792 */

/* Branch coverage (test infrastructure): the reference branches a pair took, as a bit mask per pair
 * (ORC_BR_* in gjkepa_oracle.h), collected in a thread-local word while the pair runs. */
static _Thread_local uint64_t g_cov;
#define COV(b) (g_cov |= (1ull << (b)))

#define OVCAP 1024
#define OFCAP 2048

typedef struct { double x, y, z; } v3;

static inline v3 mk(double x, double y, double z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
static inline v3 vsub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vadd(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vneg(v3 a) { return mk(-a.x, -a.y, -a.z); }
static inline v3 vscl(double s, v3 a) { return mk(s * a.x, s * a.y, s * a.z); }
static inline v3 vdiv(v3 a, double s) { return mk(a.x / s, a.y / s, a.z / s); }
static inline double dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline double norm2(v3 a) { return sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
static const v3 ORIGIN = {0.0, 0.0, 0.0};

/* CROSS_PRODUCT_3D (:1201-1212) */
static inline v3 cross(v3 a, v3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
/* UTZVEC (:1343-1352): unit vector, 0 if the norm is below 1e-12 */
static inline v3 utzvec(v3 a) {
    double md = norm2(a);
    if (md < TOL_Z) return ORIGIN;
    return vdiv(a, md);
}
/* UNINML (:1382-1394): unit normal of (v2-v1)x(v3-v2), 0 unless some |c_k| > 1e-12 */
static inline v3 uninml(v3 p1, v3 p2, v3 p3) {
    v3 c = cross(vsub(p2, p1), vsub(p3, p2));
    if (fabs(c.x) > TOL_Z || fabs(c.y) > TOL_Z || fabs(c.z) > TOL_Z) return vdiv(c, norm2(c));
    return ORIGIN;
}
static inline int is_zero_nml(v3 n) { return fabs(n.x) < TOL_Z && fabs(n.y) < TOL_Z && fabs(n.z) < TOL_Z; }
/* DIST_PF_SIGN (:1357-1377): signed distance of x to plane(p1,p2,p3); the reference STOPs on a
 * degenerate plane (:1369-1373) — reported here as a nonzero return (status DEGENERATE). */
static inline int dist_pf_sign(v3 x, v3 p1, v3 p2, v3 p3, double* r) {
    v3 n = uninml(p1, p2, p3);
    if (is_zero_nml(n)) return GJKEPA_STATUS_DEGENERATE;
    *r = dot(vsub(x, p1), n);
    return 0;
}
static inline int allclose8(v3 a, v3 b) {
    return fabs(a.x - b.x) < TOL_PT && fabs(a.y - b.y) < TOL_PT && fabs(a.z - b.z) < TOL_PT;
}

/* ---- hulls ---------------------------------------------------------------------------------- */
typedef struct { const double* p; int n; } hull_t;   /* REAL*8 p(n,3), column major */
static inline v3 hv(const hull_t* h, int i) { return mk(h->p[i], h->p[h->n + i], h->p[2 * h->n + i]); }

/* Fixed direction table GET_RANDOM_UNIT_VECTOR (:1578-1689) */
static const double DIRTAB[100][3] = {
#include "dirtab.inc"
};

/* support_mapping (:1030-1062): argmax_i d.p1_i, argmax_j (-d).p2_j, strict '>' (lowest index
 * wins ties), initial index 1 and value -HUGE. */
static v3 support(const hull_t* a, const hull_t* b, v3 d) {
    double m1 = -DBL_MAX, m2 = -DBL_MAX;
    int k1 = 0, k2 = 0;
    for (int i = 0; i < a->n; ++i) {
        double t = dot(d, hv(a, i));
        if (t > m1) { m1 = t; k1 = i; }
    }
    v3 nd = vneg(d);
    for (int i = 0; i < b->n; ++i) {
        double t = dot(nd, hv(b, i));
        if (t > m2) { m2 = t; k2 = i; }
    }
    return vsub(hv(a, k1), hv(b, k2));
}

/* mean of a hull, SUM(p(:,k)) / SIZE(p,1) (:1175-1176) */
static v3 hull_mean(const hull_t* h) {
    double sx = 0.0, sy = 0.0, sz = 0.0;
    for (int i = 0; i < h->n; ++i) { v3 p = hv(h, i); sx += p.x; sy += p.y; sz += p.z; }
    double n = (double)h->n;
    return mk(sx / n, sy / n, sz / n);
}

/* RoughCollisionDetection_SphericalEnvelope (:1165-1188) */
static int sphere_test(const hull_t* a, const hull_t* b) {
    v3 m1 = hull_mean(a), m2 = hull_mean(b);
    double r1 = -DBL_MAX, r2 = -DBL_MAX;
    for (int i = 0; i < a->n; ++i) { double t = norm2(vsub(hv(a, i), m1)); if (t > r1) r1 = t; }
    for (int i = 0; i < b->n; ++i) { double t = norm2(vsub(hv(b, i), m2)); if (t > r2) r2 = t; }
    return norm2(vsub(m1, m2)) <= r1 + r2 + SPHERE_TOL;
}

/* VEC_PL (:1423-1440): unit vector from C towards its foot D on line AB (the code's direction;
 * the comment at :1422 says the opposite). */
static v3 vec_pl(v3 C, v3 A, v3 B) {
    v3 AB = vsub(B, A), AC = vsub(C, A);
    double k = dot(AC, AB) / norm2(AB);
    v3 D = vadd(A, vscl(k, utzvec(AB)));
    return utzvec(vsub(D, C));
}

/* IS_INSIDE_PF (:1271-1337): point-in-polygon on the XY projection, XZ if no cross product is
 * positive; edge points count as inside. */
static int is_inside_pf(const v3* V, int nn, v3 P) {
    double cp[GJKEPA_MAX_HULL_VERTS + 4];
    for (int i = 0; i < nn; ++i) {
        int j = (i == nn - 1) ? 0 : i + 1;
        cp[i] = (V[j].x - V[i].x) * (P.y - V[i].y) - (V[j].y - V[i].y) * (P.x - V[i].x);
    }
    for (int i = 0; i < nn; ++i) if (fabs(cp[i]) < TOL_Z) cp[i] = 0.0;
    int anypos = 0;
    for (int i = 0; i < nn; ++i) if (cp[i] > TOL_POS) anypos = 1;
    if (!anypos) {
        COV(ORC_BR_IPF_XZ);
        for (int i = 0; i < nn; ++i) {
            int j = (i == nn - 1) ? 0 : i + 1;
            cp[i] = (V[j].x - V[i].x) * (P.z - V[i].z) - (V[j].z - V[i].z) * (P.x - V[i].x);
        }
    }
    for (int i = 0; i < nn; ++i) if (cp[0] * cp[i] < 0.0) return 0;
    return 1;
}

/* tetra faces of isPointInSimplex / update_simplex_GJK: idFc (:1227-1229, column-major fill) */
static const int IDFC[4][3] = {{0, 2, 3}, {0, 1, 3}, {0, 1, 2}, {1, 2, 3}};

static v3 centroid4(const v3* S) {   /* SUM(simplex_(:,k)) / 4.D0 (:1086, :1232) */
    return mk((((S[0].x + S[1].x) + S[2].x) + S[3].x) / 4.0,
              (((S[0].y + S[1].y) + S[2].y) + S[3].y) / 4.0,
              (((S[0].z + S[1].z) + S[2].z) + S[3].z) / 4.0);
}

/* isPointInSimplex (:1217-1265): 0 outside, 1 strictly inside (:1260), 2 the on-face branch */
static int is_point_in_simplex(v3 P, const v3* S) {
    v3 M = centroid4(S);
    v3 nml[4];
    double dist[4];
    for (int i = 0; i < 4; ++i) {
        v3 AB = vsub(S[IDFC[i][0]], S[IDFC[i][1]]);
        v3 BC = vsub(S[IDFC[i][1]], S[IDFC[i][2]]);
        nml[i] = utzvec(cross(AB, BC));
        if (dot(nml[i], vsub(S[i], M)) < 0.0) nml[i] = vneg(nml[i]);
    }
    for (int i = 0; i < 4; ++i) dist[i] = dot(vsub(S[i], P), nml[i]);
    for (int i = 0; i < 4; ++i) {
        if (fabs(dist[i]) < TOL_PT) {
            v3 V[3] = {S[IDFC[i][0]], S[IDFC[i][1]], S[IDFC[i][2]]};
            if (is_inside_pf(V, 3, P)) return 2;             /* on-face branch (:1246-1256) */
        }
    }
    return dist[0] > 0.0 && dist[1] > 0.0 && dist[2] > 0.0 && dist[3] > 0.0;
}

/* update_simplex_GJK (:1070-1157): drop the vertex opposite the face the origin is most
 * outside of, add the support along that face's outward normal. */
static void update_simplex(const hull_t* a, const hull_t* b, v3* S) {
    static const int REFV[4] = {0, 0, 0, 1};   /* vertex used for orientation / distance */
    v3 M = centroid4(S);
    v3 nml[4];
    double dst[4];
    for (int i = 0; i < 4; ++i) {
        v3 AB = vsub(S[IDFC[i][0]], S[IDFC[i][1]]);
        v3 BC = vsub(S[IDFC[i][1]], S[IDFC[i][2]]);
        nml[i] = utzvec(cross(AB, BC));
        if (dot(nml[i], vsub(S[REFV[i]], M)) < 0.0) nml[i] = vneg(nml[i]);
        dst[i] = dot(vneg(nml[i]), vsub(S[REFV[i]], ORIGIN));
    }
    int k = 0;                                   /* MAXLOC: first maximum */
    for (int i = 1; i < 4; ++i) if (dst[i] > dst[k]) k = i;
    v3 SM = support(a, b, nml[k]);
    v3 R[4] = {S[IDFC[k][0]], S[IDFC[k][1]], S[IDFC[k][2]], SM};
    memcpy(S, R, sizeof(R));
}

/* ---- re-supplied hull (GCLIB_QuickHull / GCLIB_DeHull semantics, see file header) ----------- */
typedef struct { int v[3]; v3 n; double sd, d; } face_t;   /* sd = DIST_PF_SIGN(O, face), d = |sd| */
typedef struct {
    v3 vert[OVCAP];
    int nv;
    face_t f[OFCAP];
    int nf;
    face_t tmp[OFCAP];
    int vis[OFCAP];
    int hu[OFCAP], hw[OFCAP];
    double d1[OFCAP], d2[OFCAP];
} hullbuf;

/* face record: plane normal UNINML of the stored (outward) order, DIST_PF_SIGN(O, face) and its
 * absolute value (the EPA face distance) */
static int make_face(const hullbuf* H, int a, int b, int c, face_t* f) {
    f->v[0] = a; f->v[1] = b; f->v[2] = c;
    v3 n = uninml(H->vert[a], H->vert[b], H->vert[c]);
    if (is_zero_nml(n)) return GJKEPA_STATUS_DEGENERATE;   /* :958-960 -> :1369-1373 */
    f->n = n;
    f->sd = dot(vsub(ORIGIN, H->vert[a]), n);
    f->d = fabs(f->sd);
    return 0;
}

/* Add vertex index k (already in H->vert) to the hull: faces with signed distance > HULL_EPS are
 * removed, the horizon is coned to k.  *changed = 0 when k is inside / on the hull.  The signed
 * distance of p from a face's plane is n.p - n.v0 = dot(p, n) + DIST_PF_SIGN(O, face): the plane
 * offset is the face's own origin distance, so the test needs no vertex coordinates. */
static int hull_add(hullbuf* H, int k, int* changed) {
    v3 p = H->vert[k];
    int nvis = 0;
    for (int f = 0; f < H->nf; ++f) {
        H->vis[f] = dot(p, H->f[f].n) + H->f[f].sd > HULL_EPS;
        nvis += H->vis[f];
    }
    *changed = nvis > 0;
    if (!nvis) return 0;
    int nh = 0;
    for (int f = 0; f < H->nf; ++f) {
        if (!H->vis[f]) continue;
        for (int e = 0; e < 3; ++e) {
            int u = H->f[f].v[e], w = H->f[f].v[(e + 1) % 3];
            int twin = 0;
            for (int g = 0; g < H->nf && !twin; ++g) {
                if (!H->vis[g]) continue;
                for (int e2 = 0; e2 < 3; ++e2)
                    if (H->f[g].v[e2] == w && H->f[g].v[(e2 + 1) % 3] == u) { twin = 1; break; }
            }
            if (!twin) { H->hu[nh] = u; H->hw[nh] = w; ++nh; }
        }
    }
    int nf2 = H->nf - nvis + nh;
    if (nf2 > OFCAP) return GJKEPA_STATUS_DEGENERATE;
    int m = 0;
    for (int f = 0; f < H->nf; ++f) if (!H->vis[f]) H->tmp[m++] = H->f[f];
    for (int h = 0; h < nh; ++h) {
        int st = make_face(H, H->hu[h], H->hw[h], k, &H->tmp[m++]);
        if (st) return st;
    }
    memcpy(H->f, H->tmp, sizeof(face_t) * (size_t)nf2);
    H->nf = nf2;
    return 0;
}

/* Hull of a small point set from scratch: first non-degenerate tetrahedron in list order (faces
 * in the EPA seed pattern of :279-293, each wound outward), then the other points in order. */
static int hull_build(hullbuf* H, const v3* P, int m) {
    H->nv = 0; H->nf = 0;
    for (int i = 0; i < m; ++i) H->vert[H->nv++] = P[i];
    int i0 = 0, i1 = -1, i2 = -1, i3 = -1;
    for (int j = 1; j < m; ++j) if (norm2(vsub(P[j], P[i0])) > HULL_EPS) { i1 = j; break; }
    if (i1 < 0) return GJKEPA_STATUS_DEGENERATE;
    v3 e1 = vsub(P[i1], P[i0]);
    double l1 = norm2(e1);
    for (int j = i1 + 1; j < m; ++j)
        if (norm2(cross(e1, vsub(P[j], P[i0]))) / l1 > HULL_EPS) { i2 = j; break; }
    if (i2 < 0) return GJKEPA_STATUS_DEGENERATE;
    v3 pn = utzvec(cross(e1, vsub(P[i2], P[i0])));
    for (int j = i2 + 1; j < m; ++j)
        if (fabs(dot(vsub(P[j], P[i0]), pn)) > HULL_EPS) { i3 = j; break; }
    if (i3 < 0) return GJKEPA_STATUS_DEGENERATE;
    int t[4] = {i0, i1, i2, i3};
    v3 T[4] = {P[i0], P[i1], P[i2], P[i3]};
    v3 cen = centroid4(T);
    static const int SEED[4][3] = {{0, 1, 2}, {0, 2, 3}, {0, 1, 3}, {1, 2, 3}};
    for (int f = 0; f < 4; ++f) {
        int a = t[SEED[f][0]], b = t[SEED[f][1]], c = t[SEED[f][2]];
        v3 n = cross(vsub(P[b], P[a]), vsub(P[c], P[b]));
        if (dot(n, vsub(P[a], cen)) < 0.0) { int s = b; b = c; c = s; }
        int st = make_face(H, a, b, c, &H->f[H->nf++]);
        if (st) return st;
    }
    for (int j = 0; j < m; ++j) {
        if (j == i0 || j == i1 || j == i2 || j == i3) continue;
        int ch, st = hull_add(H, j, &ch);
        if (st) return st;
    }
    return 0;
}

/* append point p and add it; drops it again if it does not change the hull */
static int hull_insert(hullbuf* H, v3 p) {
    if (H->nv >= OVCAP) return GJKEPA_STATUS_DEGENERATE;
    H->vert[H->nv] = p;
    int ch, st = hull_add(H, H->nv, &ch);
    if (st) return st;
    if (ch) H->nv++;
    else COV(ORC_BR_EPA_SWALLOW);                   /* QuickHull swallowed the point (:1005) */
    return 0;
}

static int cmp_dbl(const void* a, const void* b) {
    double x = *(const double*)a, y = *(const double*)b;
    return (x > y) - (x < y);
}

/* diagnostic: nonzero -> epa() prints one line per iteration to stderr (single-threaded use only) */
int oracle_epa_trace = 0;
/* fp32 certificate thresholds (ORC_F32 only; see gjkepa_kernel.hip "fp32 certificate"): the largest
 * drop of the polytope's MINLOC distance between iterations, relative to that distance, and the largest
 * support gap h_M(n) - depth at termination plus the fp32 evaluation noise of both terms
 * (oracle_cert_noise x (|A| + |B|), |A| the largest |coordinate| of hull A), relative to the depth. */
double oracle_cert_drop = 5e-7, oracle_cert_gap = 5e-7, oracle_cert_noise = 2.384185791015625e-07;   /* 4 x 2^-24 */
/* and the largest rounding error of the final face's unit normal (radians), bounded from its edges:
 * (2 sqrt3 u (|A|+|B|) (|e1|+|e2|) + 3 u |e1||e2|) / |e1 x e2| + 2u, u = 2^-24 */
double oracle_cert_angle = 5e-6;
static _Thread_local int g_cert;     /* bit 0: MINLOC drop, bit 1: termination gap, bit 3: origin not inside,
                                        bit 4: normal rounding bound */
static _Thread_local double g_cert_scale;   /* max |coordinate| of A + that of B */
#include <stdio.h>

/* EPA_solu loop (:274-323) with update_expandingPolytope_EPA (:863-1022). */
static int epa(const hull_t* A, const hull_t* B, const v3* S, hullbuf* H,
               double* depth, v3* normal, int* iters) {
    static const int SOUP[4][3] = {{0, 1, 2}, {0, 2, 3}, {0, 1, 3}, {1, 2, 3}};   /* :279-293 */
    int iter = 0;
    H->nv = 0;
    H->nf = 0;
    for (;;) {
        ++iter;
        *iters = iter;
        if (iter > EPA_MAXIT) { COV(ORC_BR_EPA_CAP); return GJKEPA_STATUS_EPA_MAXITER; }   /* :299-302 */
        int F1, ml = 0, st;
        double minv;
        v3 dir, a1, M;
        /* --- distances of the current polytope, MINLOC, outward direction (:888-910) --- */
        if (iter == 1) {
            F1 = 4;
            for (int f = 0; f < 4; ++f) {
                double r;
                st = dist_pf_sign(ORIGIN, S[SOUP[f][0]], S[SOUP[f][1]], S[SOUP[f][2]], &r);
                if (st) return st;
                H->d1[f] = fabs(r);
            }
            for (int f = 1; f < 4; ++f) if (H->d1[f] < H->d1[ml]) ml = f;
            dir = uninml(S[SOUP[ml][0]], S[SOUP[ml][1]], S[SOUP[ml][2]]);
            a1 = S[SOUP[ml][0]];
        } else {
            F1 = H->nf;
            for (int f = 0; f < F1; ++f) H->d1[f] = H->f[f].d;
            for (int f = 1; f < F1; ++f) if (H->d1[f] < H->d1[ml]) ml = f;
            dir = H->f[ml].n;
            a1 = H->vert[H->f[ml].v[0]];
        }
        minv = H->d1[ml];
        double dt = dot(vsub(a1, ORIGIN), dir);
        if (fabs(dt) < TOL_ZO) {                                                   /* :905-908 */
            COV(ORC_BR_EPA_CENTROID);
            double sx = 0.0, sy = 0.0, sz = 0.0;
            for (int j = 0; j < 3; ++j)
                for (int f = 0; f < F1; ++f) {
                    v3 q = (iter == 1) ? S[SOUP[f][j]] : H->vert[H->f[f].v[j]];
                    sx += q.x; sy += q.y; sz += q.z;
                }
            double cnt = (double)(F1 * 3);
            M = mk(sx / cnt, sy / cnt, sz / cnt);
            dt = dot(vsub(a1, M), dir);
        }
        if (dt <= -TOL_ZO) { dir = vneg(dir); COV(ORC_BR_EPA_FLIP); }               /* :910 */
        v3 sp = support(A, B, dir);                                                  /* :914 */
        int two = fabs(minv) < TOL_ZO;                                               /* :935 */
        if (two) COV(ORC_BR_EPA_TWO);
        /* --- hull of (polytope vertices + new point(s)) (:918-950) --- */
        if (iter == 1) {
            v3 P[6];
            int m = 0;
            for (int f = 0; f < 4; ++f)
                for (int j = 0; j < 3; ++j) {
                    v3 q = S[SOUP[f][j]];
                    int dup = 0;
                    for (int i = 0; i < m; ++i)
                        if (P[i].x == q.x && P[i].y == q.y && P[i].z == q.z) { dup = 1; break; }
                    if (!dup) P[m++] = q;
                }
            P[m++] = sp;
            if (two) P[m++] = support(A, B, vneg(dir));
            st = hull_build(H, P, m);
            if (st) return st;
        } else {
            st = hull_insert(H, sp);
            if (st) return st;
            if (two) {
                st = hull_insert(H, support(A, B, vneg(dir)));
                if (st) return st;
            }
        }
        /* --- new distances, MINLOC, orientation (:956-969) --- */
        int F2 = H->nf, ml2 = 0;
        for (int f = 0; f < F2; ++f) H->d2[f] = H->f[f].d;
        for (int f = 1; f < F2; ++f) if (H->d2[f] < H->d2[ml2]) ml2 = f;
        double minv2 = H->d2[ml2];
        v3 dir2 = H->f[ml2].n;
        if (dot(vsub(H->vert[H->f[ml2].v[0]], ORIGIN), dir2) < 0.0) dir2 = vneg(dir2);
        /* --- termination (:972-1015) --- */
        int stop;
        if (F1 == F2) {
            qsort(H->d1, (size_t)F1, sizeof(double), cmp_dbl);
            qsort(H->d2, (size_t)F2, sizeof(double), cmp_dbl);
            stop = 1;
            for (int f = 0; f < F1; ++f) if (!(fabs(H->d1[f] - H->d2[f]) < TOL_PT)) { stop = 0; break; }
            if (stop) COV(ORC_BR_EPA_STOP_EQUAL);
        } else {
            stop = F1 > F2;
            if (stop) COV(ORC_BR_EPA_STOP_SHRINK);
        }
        if (oracle_epa_trace)
            fprintf(stderr, "it %2d F1 %3d F2 %3d minv %.9g dir (%.7g %.7g %.7g) sp (%.7g %.7g %.7g) h %.9g minv2 %.9g stop %d\n",
                    iter, F1, F2, (double)minv, (double)dir.x, (double)dir.y, (double)dir.z, (double)sp.x,
                    (double)sp.y, (double)sp.z, (double)dot(sp, dir), (double)minv2, stop);
        {
            if (minv2 < minv - oracle_cert_drop * minv) g_cert |= 1;
            if (stop && !(dot(sp, dir) - minv2 + oracle_cert_noise * g_cert_scale <= oracle_cert_gap * minv2)) g_cert |= 2;
            if (stop) {
                int out = 0;
                for (int f = 0; f < F2; ++f) out |= !(H->f[f].sd < 0.0);
                if (out) g_cert |= 8;
                const v3 U = H->vert[H->f[ml2].v[0]], W = H->vert[H->f[ml2].v[1]], P = H->vert[H->f[ml2].v[2]];
                const v3 e1 = vsub(W, U), e2 = vsub(P, W), cr = cross(e1, e2);
                /* every operand a variable of the narrow phase's type: the same fp32 operations as the kernel */
                const double l1 = norm2(e1), l2 = norm2(e2), lc = norm2(cr), u = 5.9604644775390625e-08,
                             k = 3.4641016151377544, three = 3.0, two = 2.0;
                const double th = ((((k * u) * g_cert_scale) * (l1 + l2)) + (((three * u) * l1) * l2)) / lc + two * u;
                if (!(th <= oracle_cert_angle)) g_cert |= 16;
            }
        }
        if (stop) { *depth = minv2; *normal = dir2; return 0; }
    }
}

/* ---- contact features ----------------------------------------------------------------------- */
/* get_nearest_points (:813-855) */
static void nearest_points(const hull_t* a, const hull_t* b, v3 n, v3* q1, v3* q2) {
    double m1 = -DBL_MAX, m2 = -DBL_MAX;
    int k1 = 0, k2 = 0;
    for (int i = 0; i < a->n; ++i) { double t = dot(n, hv(a, i)); if (t > m1) { m1 = t; k1 = i; } }
    v3 nn = vneg(n);
    for (int i = 0; i < b->n; ++i) { double t = dot(nn, hv(b, i)); if (t > m2) { m2 = t; k2 = i; } }
    *q1 = hv(a, k1);
    *q2 = hv(b, k2);
}

/* get_info_collisionType (:353-413) */
static int collision_type(const hull_t* a, const hull_t* b, v3 n, double tol) {
    double mx = -DBL_MAX;
    int C = 0, D = 0;
    for (int i = 0; i < a->n; ++i) { double t = dot(n, hv(a, i)); if (t > mx) mx = t; }
    for (int i = 0; i < a->n; ++i) if (dot(n, hv(a, i)) > mx - tol) ++C;
    v3 nn = vneg(n);
    mx = -DBL_MAX;
    for (int i = 0; i < b->n; ++i) { double t = dot(nn, hv(b, i)); if (t > mx) mx = t; }
    for (int i = 0; i < b->n; ++i) if (dot(nn, hv(b, i)) > mx - tol) ++D;
    return (C >= 3 && D >= 3) ? 2 : 1;
}

/* two-deep "> max - 1e-8" scan of get_collisionPoint_01 (:722-732): ties update, so a later
 * near-tie wins and the running max can decrease.  idx[0] newest, idx[1] previous (-1 = none). */
static void scan_top2(const hull_t* h, v3 n, int idx[2]) {
    double mx = -DBL_MAX;
    idx[0] = -1; idx[1] = -1;
    for (int i = 0; i < h->n; ++i) {
        double t = dot(n, hv(h, i));
        if (t > mx - TOL_PT) { mx = t; idx[1] = idx[0]; idx[0] = i; }
    }
    if (idx[1] == -1) idx[1] = idx[0];
}

/* get_collisionPoint_01 (:700-806) */
static int contact_v1(const hull_t* a, const hull_t* b, v3 n, v3* res) {
    int i1[2], i2[2];
    scan_top2(a, n, i1);
    scan_top2(b, vneg(n), i2);
    if (i1[0] < 0 || i2[0] < 0) return GJKEPA_STATUS_DEGENERATE;   /* index 0: out of bounds */
    *res = ORIGIN;
    if (i1[0] == i1[1] && i2[0] == i2[1]) { *res = vdiv(vadd(hv(a, i1[0]), hv(b, i2[0])), 2.0); COV(ORC_BR_V1_MID); }
    if (i1[0] != i1[1] && i2[0] == i2[1]) { *res = hv(b, i2[0]); COV(ORC_BR_V1_B); }
    else if (i1[0] == i1[1] && i2[0] != i2[1]) { *res = hv(a, i1[0]); COV(ORC_BR_V1_A); }
    if (i1[0] != i1[1] && i2[0] != i2[1]) {
        COV(ORC_BR_V1_MEAN);
        double mx = -DBL_MAX;
        for (int i = 0; i < a->n; ++i) { double t = dot(n, hv(a, i)); if (t > mx) mx = t; }
        double sx = 0.0, sy = 0.0, sz = 0.0;
        int C = 0;
        for (int i = 0; i < a->n; ++i) {
            if (dot(n, hv(a, i)) > mx - SUPPORT_BAND) { v3 p = hv(a, i); sx += p.x; sy += p.y; sz += p.z; ++C; }
        }
        double c = (double)C;
        *res = mk(sx / c, sy / c, sz / c);
    }
    return 0;
}

/* FOOT_PL (:1492-1505) */
static v3 foot_pl(v3 P, v3 V1, v3 V2) {
    v3 u = utzvec(vsub(V2, V1));
    return vadd(V1, vscl(dot(vsub(P, V1), u), u));
}

/* FOOT_LL (:1446-1487): feet of the common perpendicular of lines P1Q1, P2Q2 */
static void foot_ll(v3 P1, v3 Q1, v3 P2, v3 Q2, v3* f1, v3* f2) {
    v3 d1 = vsub(Q1, P1), d2 = vsub(Q2, P2), r = vsub(P1, P2);
    double a = dot(d1, d1), b = dot(d1, d2), c = dot(d1, r), e = dot(d2, d2), f = dot(d2, r);
    double d = a * e - b * b;
    if (fabs(d) < TOL_Z) {
        COV(ORC_BR_FOOTLL_PARALLEL);
        *f1 = vdiv(vadd(P1, Q1), 2.0);
        *f2 = foot_pl(*f1, P2, Q2);
    } else {
        double s = (b * f - c * e) / d;
        double t = (a * f - b * c) / d;
        *f1 = vadd(P1, vscl(s, vsub(Q1, P1)));
        *f2 = vadd(P2, vscl(t, vsub(Q2, P2)));
    }
}

/* OVERLAP (:1399-1418) */
static int overlap(const v3* p, int n) {
    for (int i = 0; i < n - 1; ++i)
        for (int j = i + 1; j < n; ++j)
            if (fabs(p[i].x - p[j].x) > TOL_Z || fabs(p[i].y - p[j].y) > TOL_Z || fabs(p[i].z - p[j].z) > TOL_Z)
                return 0;
    return 1;
}

/* 2*ACOS(-1.0) in default (single) precision, promoted to REAL*8 (:1547) */
#define TWO_PI_SP ((double)(2.0f * 3.14159274101257324f))

/* SORT_CLOCK (:1513-1575): angular order about the centroid.  The reference leaves the result
 * undefined when all points coincide (returns before assigning); here the input is returned. */
static int sort_clock(const v3* p, int n, v3* o) {
    if (overlap(p, n)) { COV(ORC_BR_V2_OVERLAP); memcpy(o, p, sizeof(v3) * (size_t)n); return 0; }
    double sx = 0.0, sy = 0.0, sz = 0.0;
    for (int i = 0; i < n; ++i) { sx += p[i].x; sy += p[i].y; sz += p[i].z; }
    double dn = (double)n;
    v3 cen = mk(sx / dn, sy / dn, sz / dn);
    v3 nrm = cross(vsub(p[1], p[0]), vsub(p[2], p[0]));
    o[0] = p[0];
    for (int i = 1; i < n; ++i) {
        double mina = DBL_MAX;
        int idx = -1;
        for (int j = 0; j < n; ++j) {
            int seen = 0;
            for (int k = 0; k < i; ++k)
                if (p[j].x == o[k].x && p[j].y == o[k].y && p[j].z == o[k].z) { seen = 1; break; }
            if (seen) continue;
            v3 w1 = vsub(p[j], cen), w2 = vsub(o[i - 1], cen);
            double ang = atan2(dot(nrm, cross(w2, w1)), dot(w1, w2));
            ang = fmod(ang + TWO_PI_SP, TWO_PI_SP);   /* MODULO, positive arguments */
            if (ang < mina) { mina = ang; idx = j; }
        }
        if (idx < 0) return GJKEPA_STATUS_DEGENERATE;   /* duplicate points: out-of-bounds in ref */
        o[i] = p[idx];
    }
    return 0;
}

/* AddAllSupports (:509-529): vertices within `band` of the max along n, in index order */
static int support_set(const hull_t* h, v3 n, double band, v3* out) {
    double mx = -DBL_MAX;
    for (int i = 0; i < h->n; ++i) { double t = dot(n, hv(h, i)); if (t > mx) mx = t; }
    int c = 0;
    for (int i = 0; i < h->n; ++i) if (dot(n, hv(h, i)) > mx - band) out[c++] = hv(h, i);
    return c;
}

/* case_04 + branch_case_04 (:575-669): A has >= 3 supports, B exactly 2 */
static int contact_case04(const v3* A, int na, const v3* B, v3* res) {
    v3 srt[GJKEPA_MAX_HULL_VERTS];
    int st = sort_clock(A, na, srt);
    if (st) return st;
    int C = 0;
    for (int i = 0; i < 2; ++i) if (is_inside_pf(srt, na, B[i])) ++C;
    COV(C == 0 ? ORC_BR_V2_CASE04_1 : C == 1 ? ORC_BR_V2_CASE04_3 : ORC_BR_V2_CASE04_2);
    if (C == 0) {                                                   /* case_04_1 */
        double sx = 0.0, sy = 0.0, sz = 0.0;
        for (int i = 0; i < na; ++i) { sx += A[i].x; sy += A[i].y; sz += A[i].z; }
        double dn = (double)na;
        *res = foot_pl(mk(sx / dn, sy / dn, sz / dn), B[0], B[1]);
    } else {                                                        /* case_04_2 / case_04_3 */
        *res = vscl(0.5, vadd(B[0], B[1]));
    }
    return 0;
}

/* get_collisionPoint_02 (:457-696) */
static int contact_v2(const hull_t* a, const hull_t* b, v3 n, v3* res) {
    v3 s1[GJKEPA_MAX_HULL_VERTS], s2[GJKEPA_MAX_HULL_VERTS];
    int n1 = support_set(a, n, SUPPORT_BAND, s1);
    int n2 = support_set(b, vneg(n), SUPPORT_BAND, s2);
    *res = ORIGIN;
    if (n1 == 1 && n2 == 1) { *res = vdiv(vadd(s1[0], s2[0]), 2.0); COV(ORC_BR_V2_CASE01); }   /* case_01 */
    else if (n1 == 1 && n2 >= 2) { *res = s1[0]; COV(ORC_BR_V2_CASE02); }                    /* case_02 */
    else if (n1 >= 2 && n2 == 1) { *res = s2[0]; COV(ORC_BR_V2_CASE02B); }
    else if (n1 == 2 && n2 == 2) {                                         /* case_03 */
        COV(ORC_BR_V2_CASE03);
        v3 f1, f2;
        foot_ll(s1[0], s1[1], s2[0], s2[1], &f1, &f2);
        *res = vdiv(vadd(f1, f2), 2.0);
    } else if (n1 == 2 && n2 >= 3) { COV(ORC_BR_V2_CASE04); return contact_case04(s2, n2, s1, res); }
    else if (n1 >= 3 && n2 == 2) { COV(ORC_BR_V2_CASE04B); return contact_case04(s1, n1, s2, res); }
    else if (n1 >= 3 && n2 >= 3) {                                         /* case_05 */
        COV(ORC_BR_V2_CASE05);
        double sx = 0.0, sy = 0.0, sz = 0.0;
        for (int i = 0; i < n1; ++i) { sx += s1[i].x; sy += s1[i].y; sz += s1[i].z; }
        double dn = (double)n1;
        *res = mk(sx / dn, sy / dn, sz / dn);
    } else return GJKEPA_STATUS_DEGENERATE;                                /* :498-501 */
    return 0;
}

/* get_collisionPoint_03 (:426-452): contact on p2, z from p1's mean, normal projected on XY */
static int contact_v3(const hull_t* a, const hull_t* b, v3 n, v3* res, v3* nnew) {
    double mx = -DBL_MAX;
    int idx = -1;
    v3 nn = vneg(n);
    for (int i = 0; i < b->n; ++i) {
        double t = dot(nn, hv(b, i));
        if (t > mx - TOL_PT) { mx = t; idx = i; }
    }
    if (idx < 0) return GJKEPA_STATUS_DEGENERATE;
    double sz = 0.0;
    for (int i = 0; i < a->n; ++i) sz += hv(a, i).z;
    *res = hv(b, idx);
    res->z = sz / (double)(float)a->n;          /* REAL(SIZE(p1_,1)): default real */
    v3 q = mk(n.x, n.y, 0.0);
    double nq = norm2(q);
    *nnew = vdiv(q, nq);
    if (!(nq > 0.0)) COV(ORC_BR_V3_NAN);          /* n = +-z: 0/0 (:447) */
    return 0;
}

/* ---- GJKEPA (:39-239) ------------------------------------------------------------------------ */
static void zero_record(gjkepa_contact_f64* o) { memset(o, 0, sizeof(*o)); }

static int gjkepa_pair(int32_t version, double tol_ff, const hull_t* A, const hull_t* B,
                       hullbuf* H, gjkepa_contact_f64* out) {
    zero_record(out);
    if (A->n < 1 || B->n < 1 || A->n > GJKEPA_MAX_HULL_VERTS || B->n > GJKEPA_MAX_HULL_VERTS) {
        out->status = GJKEPA_STATUS_BAD_INPUT;
        return 0;
    }
    if (!sphere_test(A, B)) { COV(ORC_BR_SPHERE_MISS); return 0; }           /* :76-77 */
    v3 S[4] = {ORIGIN, ORIGIN, ORIGIN, ORIGIN};   /* fresh THREADPRIVATE SAVE state: row 4 = 0 */
    int st = 0, hit = 0, gjk_it = 0;
    /* --- initial simplex (:82-170) --- */
    int iter = 0;
    v3 dir;
    for (;;) {
        ++iter;
        if (iter > INIT_MAXIT) { COV(ORC_BR_INIT_CAP); return 0; }           /* :86-89 */
        if (iter > 1) COV(ORC_BR_INIT_RETRY);                                   /* :106-112 */
        dir = mk(DIRTAB[iter - 1][0], DIRTAB[iter - 1][1], DIRTAB[iter - 1][2]);
        S[0] = support(A, B, dir);
        dir = vneg(dir);
        S[1] = support(A, B, dir);
        if (!allclose8(S[0], S[1])) break;                                     /* :106-110 */
    }
    dir = vec_pl(ORIGIN, S[0], S[1]);                                          /* :116 */
    S[2] = support(A, B, dir);
    if (allclose8(S[2], S[0]) || allclose8(S[2], S[1])) { COV(ORC_BR_INIT_S3_COINCIDE); return 0; }   /* :123-127 */
    dir = utzvec(cross(vsub(S[1], S[0]), vsub(S[2], S[1])));                  /* :132-135 */
    v3 VO = vsub(ORIGIN, S[2]);
    double vd = dot(VO, dir);
    if (fabs(vd) < TOL_PT) {                                                   /* :140-148 */
        if (is_inside_pf(S, 3, ORIGIN)) { COV(ORC_BR_INIT_TRI_HIT); hit = 1; goto do_epa; }
        COV(ORC_BR_INIT_TRI_PLANE);
    }
    if (vd < 0.0) dir = vneg(dir);                                             /* :151 */
    S[3] = support(A, B, dir);                                                 /* :154 */
    {
        double r;
        st = dist_pf_sign(S[3], S[0], S[1], S[2], &r);                         /* :157 */
        if (st) goto fail;
        if (fabs(r) < TOL_PT) { COV(ORC_BR_INIT_COPLANAR); return 0; }
    }
    {
        int pis = is_point_in_simplex(ORIGIN, S);                              /* :164-170 */
        if (pis) { COV(pis == 2 ? ORC_BR_INIT_TETRA_ONFACE : ORC_BR_INIT_TETRA_HIT); hit = 1; goto do_epa; }
    }
    {
        v3 L1[4] = {ORIGIN, ORIGIN, ORIGIN, ORIGIN}, L2[4] = {ORIGIN, ORIGIN, ORIGIN, ORIGIN};
        iter = 0;
        for (;;) {                                                             /* :182-236 */
            ++iter;
            gjk_it = iter;
            if (iter > GJK_MAXIT) { COV(ORC_BR_LOOP_CAP); return 0; }
            memcpy(L2, L1, sizeof(L1));
            memcpy(L1, S, sizeof(L1));
            update_simplex(A, B, S);
            if (norm2(cross(vsub(S[1], S[0]), vsub(S[2], S[1]))) < TOL_PT) { COV(ORC_BR_LOOP_COLLINEAR); return 0; }   /* :199-201 */
            double r;
            st = dist_pf_sign(S[3], S[0], S[1], S[2], &r);                     /* :203 */
            if (st) { out->diag = (uint32_t)(gjk_it & 0xff); goto fail; }
            if (fabs(r) < TOL_PT) { COV(ORC_BR_LOOP_COPLANAR); return 0; }       /* :203-206 */
            const int pis = is_point_in_simplex(ORIGIN, S);                    /* :210-216 */
            if (pis) { COV(pis == 2 ? ORC_BR_LOOP_ONFACE : ORC_BR_LOOP_HIT); hit = 1; break; }
            int over = 1;                                                      /* :219-234 */
            for (int i = 0; i < 4; ++i) {
                if (!(allclose8(S[i], L1[i]) || allclose8(S[i], L2[i]))) { over = 0; break; }
            }
            if (over) { COV(ORC_BR_LOOP_CYCLE); return 0; }
        }
    }
do_epa:
    out->collision = 1;
    {
        double depth = 0.0;
        v3 n = ORIGIN, pt = ORIGIN, q1, q2;
        int eit = 0;
        g_cert = 0;
        {
            double ma = 0.0, mb = 0.0;
            for (int i = 0; i < 3 * A->n; ++i) { double t = fabs(A->p[i]); if (t > ma) ma = t; }
            for (int i = 0; i < 3 * B->n; ++i) { double t = fabs(B->p[i]); if (t > mb) mb = t; }
            g_cert_scale = ma + mb;
        }
        st = epa(A, B, S, H, &depth, &n, &eit);
#ifdef ORC_F32
        out->reserved = (int8_t)(g_cert | (st ? 4 : 0));   /* diagnostic build: certificate flags */
#endif
        out->diag = (uint32_t)(gjk_it & 0xff) | ((uint32_t)(eit & 0xff) << 8) |
                    ((uint32_t)(H->nf & 0xffff) << 16);
        if (st) goto fail;
        nearest_points(A, B, n, &q1, &q2);                                      /* :326 */
        if (version == 1) st = contact_v1(A, B, n, &pt);                        /* :329-340 */
        else if (version == 2) st = contact_v2(A, B, n, &pt);
        else if (version == 3) { v3 nn; st = contact_v3(A, B, n, &pt, &nn); n = nn; }
        else st = GJKEPA_STATUS_BAD_VERSION;
        if (st) goto fail;
        out->colli_type = (int8_t)collision_type(A, B, n, tol_ff);              /* :343 */
        COV(out->colli_type == 2 ? ORC_BR_TYPE2 : ORC_BR_TYPE1);
        out->penetration_depth = depth;
        out->collision_normal[0] = n.x; out->collision_normal[1] = n.y; out->collision_normal[2] = n.z;
        out->collision_point[0] = pt.x; out->collision_point[1] = pt.y; out->collision_point[2] = pt.z;
        out->nearest_points[0] = q1.x; out->nearest_points[1] = q1.y; out->nearest_points[2] = q1.z;
        out->nearest_points[3] = q2.x; out->nearest_points[4] = q2.y; out->nearest_points[5] = q2.z;
    }
    (void)hit;
    return 0;
fail: {
        if (st == GJKEPA_STATUS_DEGENERATE) COV(ORC_BR_DEGENERATE);
        if (st == GJKEPA_STATUS_BAD_VERSION) COV(ORC_BR_BAD_VERSION);
        uint32_t diag = out->diag;
        zero_record(out);
        out->collision = 1;
        out->status = (int8_t)st;
        out->diag = diag;
        return 0;
    }
}

/* ---- public oracle entries ------------------------------------------------------------------ */
#ifdef ORC_F32
#undef double
#endif
int oracle_gjkepa(int32_t version, double tol_ff,
                  const double* p1, int32_t n1, const double* p2, int32_t n2,
                  gjkepa_contact_f64* out) {
    if (!out || (!p1 && n1 > 0) || (!p2 && n2 > 0)) return GJKEPA_E_ARG;
    hullbuf* H = (hullbuf*)malloc(sizeof(hullbuf));
    if (!H) return GJKEPA_E_ARG;
#ifdef ORC_F32
    oreal* c1 = (oreal*)malloc(sizeof(oreal) * (3 * (size_t)n1 + 1));
    oreal* c2 = (oreal*)malloc(sizeof(oreal) * (3 * (size_t)n2 + 1));
    for (int i = 0; i < 3 * n1; ++i) c1[i] = (oreal)p1[i];
    for (int i = 0; i < 3 * n2; ++i) c2[i] = (oreal)p2[i];
    hull_t A = {c1, n1}, B = {c2, n2};
#else
    hull_t A = {p1, n1}, B = {p2, n2};
#endif
    gjkepa_pair(version, (oreal)tol_ff, &A, &B, H, out);
#ifdef ORC_F32
    free(c1); free(c2);
#endif
    free(H);
    return 0;
}

int oracle_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

int oracle_gjkepa_batch(int32_t version, double tol_ff, int32_t vert_dtype,
                        const void* verts, const int64_t* hull_off, const int32_t* hull_cnt,
                        const int32_t* pairs, int64_t n_pairs,
                        gjkepa_contact_f64* out, int32_t nthreads) {
    return oracle_gjkepa_batch_cov(version, tol_ff, vert_dtype, verts, hull_off, hull_cnt, pairs, n_pairs, out,
                                   NULL, nthreads);
}

int oracle_gjkepa_batch_cov(int32_t version, double tol_ff, int32_t vert_dtype,
                            const void* verts, const int64_t* hull_off, const int32_t* hull_cnt,
                            const int32_t* pairs, int64_t n_pairs,
                            gjkepa_contact_f64* out, uint64_t* cov, int32_t nthreads) {
    if (!verts || !hull_off || !hull_cnt || !pairs || !out || n_pairs < 0) return GJKEPA_E_ARG;
    if (vert_dtype != GJKEPA_DTYPE_F32 && vert_dtype != GJKEPA_DTYPE_F64) return GJKEPA_E_ARG;
    int nt = nthreads > 0 ? nthreads : oracle_max_threads();
    (void)nt;
#pragma omp parallel num_threads(nt)
    {
        hullbuf* H = (hullbuf*)malloc(sizeof(hullbuf));
        oreal* b1 = (oreal*)malloc(sizeof(oreal) * 3 * GJKEPA_MAX_HULL_VERTS);
        oreal* b2 = (oreal*)malloc(sizeof(oreal) * 3 * GJKEPA_MAX_HULL_VERTS);
#pragma omp for schedule(dynamic, 64)
        for (int64_t k = 0; k < n_pairs; ++k) {
            int32_t ha = pairs[2 * k], hb = pairs[2 * k + 1];
            int32_t na = hull_cnt[ha], nb = hull_cnt[hb];
            hull_t A, B;
            if (na < 1 || nb < 1 || na > GJKEPA_MAX_HULL_VERTS || nb > GJKEPA_MAX_HULL_VERTS) {
                zero_record(&out[k]);
                out[k].status = GJKEPA_STATUS_BAD_INPUT;
                if (cov) cov[k] = 1ull << ORC_BR_BAD_INPUT;
                continue;
            }
            if (vert_dtype == GJKEPA_DTYPE_F64 && sizeof(oreal) == sizeof(double)) {
                A.p = (const oreal*)verts + hull_off[ha];
                B.p = (const oreal*)verts + hull_off[hb];
            } else if (vert_dtype == GJKEPA_DTYPE_F64) {
                const double* fa = (const double*)verts + hull_off[ha];
                const double* fb = (const double*)verts + hull_off[hb];
                for (int i = 0; i < 3 * na; ++i) b1[i] = (oreal)fa[i];
                for (int i = 0; i < 3 * nb; ++i) b2[i] = (oreal)fb[i];
                A.p = b1;
                B.p = b2;
            } else {
                const float* fa = (const float*)verts + hull_off[ha];
                const float* fb = (const float*)verts + hull_off[hb];
                for (int i = 0; i < 3 * na; ++i) b1[i] = (oreal)fa[i];
                for (int i = 0; i < 3 * nb; ++i) b2[i] = (oreal)fb[i];
                A.p = b1;
                B.p = b2;
            }
            A.n = na;
            B.n = nb;
            g_cov = 0;
            gjkepa_pair(version, (oreal)tol_ff, &A, &B, H, &out[k]);
            if (cov) cov[k] = g_cov;
        }
        free(H); free(b1); free(b2);
    }
    return 0;
}

/* ==== batched convex hulls ==============================================
 * GCLIB_QuickHull::QuickHull + GCLIB_DeHull::getHullMeshesVertex as used at GCLIB_GJKEPA.f90:920,
 * :950 (unvendored, no version pin), with the algorithm fixed in include/gjkepa.h: QuickHull in
 * global furthest-point order, fp64, absolute epsilon GJKEPA_HULL_EPS, new faces in the removed
 * faces' slots (slot order) then appended.  hull_kernel.hip follows this operation for operation. */
#define QH_FCAP (2 * GJKEPA_HULL_MAX_POINTS - 4)
typedef struct {
    v3 p[GJKEPA_HULL_MAX_POINTS];
    int st[GJKEPA_HULL_MAX_POINTS];       /* assigned face slot, -1 = interior / processed */
    double dist[GJKEPA_HULL_MAX_POINTS];  /* distance above the assigned face */
    int fv[QH_FCAP][3];                   /* face vertex ids; fv[f][0] < 0: dead slot */
    v3 fn[QH_FCAP];                       /* UNINML of the stored (outward) order */
    int vis[QH_FCAP], vl[QH_FCAP], hu[QH_FCAP], hw[QH_FCAP], ns[QH_FCAP];
    unsigned char used[GJKEPA_HULL_MAX_POINTS];
} qhbuf;

/* signed distance of p above face f (the DIST_PF_SIGN recipe, :1357-1377) */
static inline double qh_dist(const qhbuf* Q, int f, v3 p) { return dot(vsub(p, Q->p[Q->fv[f][0]]), Q->fn[f]); }

static int qh_cloud(qhbuf* Q, int n, int32_t* faces, int32_t* nf_out, int32_t* vidx, int32_t* nv_out) {
    const double eps = GJKEPA_HULL_EPS;
    const int fcap = 2 * n - 4;
    *nf_out = 0; *nv_out = 0;
    for (int j = 0; j < n; ++j)
        if (!isfinite(Q->p[j].x) || !isfinite(Q->p[j].y) || !isfinite(Q->p[j].z)) return GJKEPA_STATUS_BAD_INPUT;
    /* 1. initial tetrahedron */
    int i0 = 0;
    for (int j = 1; j < n; ++j) if (Q->p[j].x < Q->p[i0].x) i0 = j;
    v3 p0 = Q->p[i0];
    int i1 = 0; double b = -1.0;
    for (int j = 0; j < n; ++j) { v3 d = vsub(Q->p[j], p0); double v = dot(d, d); if (v > b) { b = v; i1 = j; } }
    v3 e1 = vsub(Q->p[i1], p0);
    double l1 = norm2(e1);
    if (!(l1 > eps)) return GJKEPA_STATUS_DEGENERATE;
    int i2 = 0; b = -1.0;
    for (int j = 0; j < n; ++j) { v3 c = cross(e1, vsub(Q->p[j], p0)); double v = dot(c, c); if (v > b) { b = v; i2 = j; } }
    v3 pn = cross(e1, vsub(Q->p[i2], p0));
    double lp = norm2(pn);
    if (!(lp / l1 > eps)) return GJKEPA_STATUS_DEGENERATE;
    int i3 = 0; b = -1.0;
    for (int j = 0; j < n; ++j) { double v = fabs(dot(vsub(Q->p[j], p0), pn)); if (v > b) { b = v; i3 = j; } }
    if (!(b / lp > eps)) return GJKEPA_STATUS_DEGENERATE;
    const int t[4] = {i0, i1, i2, i3};
    v3 T[4] = {Q->p[i0], Q->p[i1], Q->p[i2], Q->p[i3]};
    v3 cen = centroid4(T);
    static const int SEED[4][3] = {{0, 1, 2}, {0, 2, 3}, {0, 1, 3}, {1, 2, 3}};
    for (int f = 0; f < 4; ++f) {
        int a = t[SEED[f][0]], bb = t[SEED[f][1]], c = t[SEED[f][2]];
        v3 nn = cross(vsub(Q->p[bb], Q->p[a]), vsub(Q->p[c], Q->p[bb]));
        if (dot(nn, vsub(Q->p[a], cen)) < 0.0) { int s = bb; bb = c; c = s; }
        Q->fv[f][0] = a; Q->fv[f][1] = bb; Q->fv[f][2] = c;
        Q->fn[f] = uninml(Q->p[a], Q->p[bb], Q->p[c]);
        if (is_zero_nml(Q->fn[f])) return GJKEPA_STATUS_DEGENERATE;
        Q->vis[f] = 0;
    }
    int hwm = 4;
    /* 2. initial assignment */
    for (int j = 0; j < n; ++j) {
        Q->st[j] = -1;
        if (j == i0 || j == i1 || j == i2 || j == i3) continue;
        double best = -DBL_MAX; int bf = -1;
        for (int f = 0; f < 4; ++f) { double d = qh_dist(Q, f, Q->p[j]); if (d > best) { best = d; bf = f; } }
        if (best > eps) { Q->st[j] = bf; Q->dist[j] = best; }
    }
    /* 3. furthest-point expansion */
    for (;;) {
        int eye = -1; double be = -DBL_MAX;
        for (int j = 0; j < n; ++j) if (Q->st[j] >= 0 && Q->dist[j] > be) { be = Q->dist[j]; eye = j; }
        if (eye < 0) break;
        v3 pe = Q->p[eye];
        int nvis = 0;
        for (int f = 0; f < hwm; ++f) {
            Q->vis[f] = Q->fv[f][0] >= 0 && qh_dist(Q, f, pe) > eps;
            if (Q->vis[f]) Q->vl[nvis++] = f;
        }
        int nh = 0;
        for (int j = 0; j < nvis; ++j) {
            const int* fv = Q->fv[Q->vl[j]];
            for (int e = 0; e < 3; ++e) {
                int u = fv[e], w = fv[(e + 1) % 3], twin = 0;
                for (int m = 0; m < nvis && !twin; ++m) {
                    const int* gv = Q->fv[Q->vl[m]];
                    twin = (gv[0] == w && gv[1] == u) || (gv[1] == w && gv[2] == u) || (gv[2] == w && gv[0] == u);
                }
                if (!twin) {
                    if (nh == fcap) return GJKEPA_STATUS_DEGENERATE;   /* cannot fit: see below */
                    Q->hu[nh] = u; Q->hw[nh] = w; ++nh;
                }
            }
        }
        if (nh == 0 || hwm + (nh > nvis ? nh - nvis : 0) > fcap) return GJKEPA_STATUS_DEGENERATE;
        for (int k = 0; k < nh; ++k) Q->ns[k] = k < nvis ? Q->vl[k] : hwm + (k - nvis);
        /* re-assign the points of removed faces among the new faces (needs the old vis flags) */
        v3 nnrm[QH_FCAP];
        for (int k = 0; k < nh; ++k) {
            nnrm[k] = uninml(Q->p[Q->hu[k]], Q->p[Q->hw[k]], pe);
            if (is_zero_nml(nnrm[k])) return GJKEPA_STATUS_DEGENERATE;
        }
        Q->st[eye] = -1;
        for (int j = 0; j < n; ++j) {
            if (Q->st[j] < 0 || !Q->vis[Q->st[j]]) continue;
            double best = -DBL_MAX; int bk = -1;
            for (int k = 0; k < nh; ++k) {
                double d = dot(vsub(Q->p[j], Q->p[Q->hu[k]]), nnrm[k]);
                if (d > best) { best = d; bk = k; }
            }
            if (best > eps) { Q->st[j] = Q->ns[bk]; Q->dist[j] = best; } else Q->st[j] = -1;
        }
        for (int j = 0; j < nvis; ++j) Q->vis[Q->vl[j]] = 0;
        for (int k = nh; k < nvis; ++k) Q->fv[Q->vl[k]][0] = -1;   /* removed slots left over */
        for (int k = 0; k < nh; ++k) {
            int s = Q->ns[k];
            Q->fv[s][0] = Q->hu[k]; Q->fv[s][1] = Q->hw[k]; Q->fv[s][2] = eye;
            Q->fn[s] = nnrm[k];
            Q->vis[s] = 0;
        }
        if (nh > nvis) hwm += nh - nvis;
    }
    /* output: live faces in slot order, then the referenced points in ascending order */
    int nf = 0;
    memset(Q->used, 0, sizeof(Q->used));
    for (int f = 0; f < hwm; ++f) {
        if (Q->fv[f][0] < 0) continue;
        for (int e = 0; e < 3; ++e) { faces[3 * nf + e] = Q->fv[f][e]; Q->used[Q->fv[f][e]] = 1; }
        ++nf;
    }
    int nv = 0;
    for (int j = 0; j < n; ++j) if (Q->used[j]) vidx[nv++] = j;
    *nf_out = nf; *nv_out = nv;
    return GJKEPA_STATUS_OK;
}

int oracle_hull_batch(int32_t vert_dtype, const void* points, const int64_t* cloud_off,
                      const int32_t* cloud_cnt, int64_t n_clouds, const int64_t* face_off,
                      int32_t* faces, int32_t* n_faces, int32_t* n_verts, int8_t* status,
                      void* hull_verts, int32_t* vert_idx, int32_t nthreads) {
    if (!points || !cloud_off || !cloud_cnt || !face_off || !faces || !n_faces || !n_verts || !status || n_clouds < 0)
        return GJKEPA_E_ARG;
    if (vert_dtype != GJKEPA_DTYPE_F32 && vert_dtype != GJKEPA_DTYPE_F64) return GJKEPA_E_ARG;
    int nt = nthreads > 0 ? nthreads : oracle_max_threads();
    (void)nt;
#pragma omp parallel num_threads(nt)
    {
        qhbuf* Q = (qhbuf*)malloc(sizeof(qhbuf));
        int32_t vi[GJKEPA_HULL_MAX_POINTS];
#pragma omp for schedule(dynamic, 16)
        for (int64_t c = 0; c < n_clouds; ++c) {
            const int n = cloud_cnt[c];
            int32_t nf = 0, nv = 0;
            int st = GJKEPA_STATUS_BAD_INPUT;
            if (n >= 4 && n <= GJKEPA_HULL_MAX_POINTS) {
                for (int j = 0; j < n; ++j) {
                    if (vert_dtype == GJKEPA_DTYPE_F64) {
                        const double* q = (const double*)points + cloud_off[c];
                        Q->p[j] = mk(q[j], q[n + j], q[2 * n + j]);
                    } else {
                        const float* q = (const float*)points + cloud_off[c];
                        Q->p[j] = mk((double)q[j], (double)q[n + j], (double)q[2 * n + j]);
                    }
                }
                st = qh_cloud(Q, n, faces + 3 * face_off[c], &nf, vi, &nv);
            }
            if (st != GJKEPA_STATUS_OK) { nf = 0; nv = 0; }
            n_faces[c] = nf; n_verts[c] = nv; status[c] = (int8_t)st;
            for (int k = 0; k < nv; ++k) {
                if (vert_idx) vert_idx[cloud_off[c] + k] = vi[k];
                if (!hull_verts) continue;
                if (vert_dtype == GJKEPA_DTYPE_F64) {
                    const double* q = (const double*)points + cloud_off[c];
                    double* h = (double*)hull_verts + cloud_off[c];
                    h[k] = q[vi[k]]; h[nv + k] = q[n + vi[k]]; h[2 * nv + k] = q[2 * n + vi[k]];
                } else {
                    const float* q = (const float*)points + cloud_off[c];
                    float* h = (float*)hull_verts + cloud_off[c];
                    h[k] = q[vi[k]]; h[nv + k] = q[n + vi[k]]; h[2 * nv + k] = q[2 * n + vi[k]];
                }
            }
        }
        free(Q);
    }
    return 0;
}

/* ==== broad phase ==========================================================
 * Every pair (a < b) of a hull pool passing RoughCollisionDetection_SphericalEnvelope (:1165-1188),
 * in ascending (a, b) order.  Centres / radii use sphere_test's arithmetic (hull_mean, max norm2);
 * candidates come from a uniform grid of cell size >= 2 r_max + 1 (27 neighbour cells), so the
 * search is complete, and every candidate is decided by the exact predicate. */
typedef struct { int64_t key; int32_t h; } bp_cell;
static int bp_cmp_cell(const void* x, const void* y) {
    const bp_cell *a = (const bp_cell*)x, *b = (const bp_cell*)y;
    return a->key < b->key ? -1 : a->key > b->key ? 1 : (a->h < b->h ? -1 : a->h > b->h);
}
static int bp_cmp_u64(const void* x, const void* y) {
    uint64_t a = *(const uint64_t*)x, b = *(const uint64_t*)y;
    return a < b ? -1 : a > b;
}

int oracle_broadphase(int32_t vert_dtype, const void* verts, const int64_t* hull_off, const int32_t* hull_cnt,
                      int64_t n_hulls, int32_t* pairs, int64_t max_pairs, int64_t* n_pairs, int32_t nthreads) {
    if (!verts || !hull_off || !hull_cnt || !n_pairs || n_hulls < 0 || max_pairs < 0 || (max_pairs > 0 && !pairs))
        return GJKEPA_E_ARG;
    if (vert_dtype != GJKEPA_DTYPE_F32 && vert_dtype != GJKEPA_DTYPE_F64) return GJKEPA_E_ARG;
    int nt = nthreads > 0 ? nthreads : oracle_max_threads();
    (void)nt;
    v3* m = (v3*)malloc(sizeof(v3) * (size_t)(n_hulls + 1));
    double* r = (double*)malloc(sizeof(double) * (size_t)(n_hulls + 1));
    unsigned char* ok = (unsigned char*)malloc((size_t)n_hulls + 1);
#pragma omp parallel num_threads(nt)
    {
        double* buf = (double*)malloc(sizeof(double) * 3 * GJKEPA_MAX_HULL_VERTS);
#pragma omp for schedule(static)
        for (int64_t h = 0; h < n_hulls; ++h) {
            const int n = hull_cnt[h];
            ok[h] = 0;
            if (n < 1 || n > GJKEPA_MAX_HULL_VERTS) continue;
            hull_t A;
            if (vert_dtype == GJKEPA_DTYPE_F64) {
                A.p = (const double*)verts + hull_off[h];
            } else {
                const float* f = (const float*)verts + hull_off[h];
                for (int i = 0; i < 3 * n; ++i) buf[i] = (double)f[i];
                A.p = buf;
            }
            A.n = n;
            m[h] = hull_mean(&A);
            double rr = -DBL_MAX;
            for (int i = 0; i < n; ++i) { double t = norm2(vsub(hv(&A, i), m[h])); if (t > rr) rr = t; }
            r[h] = rr;
            ok[h] = isfinite(m[h].x) && isfinite(m[h].y) && isfinite(m[h].z) && isfinite(rr);
        }
        free(buf);
    }
    double rmax = 0.0;
    for (int64_t h = 0; h < n_hulls; ++h) if (ok[h] && r[h] > rmax) rmax = r[h];
    const double cell = (2.0 * rmax + SPHERE_TOL) * (1.0 + 1e-9) + 1e-9;
    bp_cell* cells = (bp_cell*)malloc(sizeof(bp_cell) * (size_t)(n_hulls + 1));
    int64_t nc = 0;
    const int64_t B = 1 << 20;                  /* cell coordinates packed 21 bits each */
    for (int64_t h = 0; h < n_hulls; ++h) {
        if (!ok[h]) continue;
        int64_t ix = (int64_t)floor(m[h].x / cell) + B, iy = (int64_t)floor(m[h].y / cell) + B,
                iz = (int64_t)floor(m[h].z / cell) + B;
        cells[nc].key = (ix << 42) | (iy << 21) | iz;
        cells[nc].h = (int32_t)h;
        ++nc;
    }
    qsort(cells, (size_t)nc, sizeof(bp_cell), bp_cmp_cell);
    uint64_t* found = NULL;
    int64_t nfound = 0, cap = 0;
#pragma omp parallel num_threads(nt)
    {
        uint64_t* loc = NULL;
        int64_t nl = 0, cl = 0;
#pragma omp for schedule(dynamic, 256)
        for (int64_t s = 0; s < nc; ++s) {
            const int64_t key = cells[s].key;
            const int32_t a = cells[s].h;
            const int64_t ix = key >> 42, iy = (key >> 21) & ((1 << 21) - 1), iz = key & ((1 << 21) - 1);
            for (int dx = -1; dx <= 1; ++dx)
                for (int dy = -1; dy <= 1; ++dy)
                    for (int dz = -1; dz <= 1; ++dz) {
                        const int64_t k2 = ((ix + dx) << 42) | ((iy + dy) << 21) | (iz + dz);
                        int64_t lo = 0, hi = nc;                  /* first cell entry with key >= k2 */
                        while (lo < hi) { int64_t md = (lo + hi) / 2; if (cells[md].key < k2) lo = md + 1; else hi = md; }
                        for (int64_t t = lo; t < nc && cells[t].key == k2; ++t) {
                            const int32_t b = cells[t].h;
                            if (b <= a) continue;
                            if (!(norm2(vsub(m[a], m[b])) <= r[a] + r[b] + SPHERE_TOL)) continue;
                            if (nl == cl) { cl = cl ? 2 * cl : 1024; loc = (uint64_t*)realloc(loc, sizeof(uint64_t) * (size_t)cl); }
                            loc[nl++] = ((uint64_t)a << 32) | (uint32_t)b;
                        }
                    }
        }
#pragma omp critical
        {
            if (nfound + nl > cap) { cap = 2 * (nfound + nl) + 1024; found = (uint64_t*)realloc(found, sizeof(uint64_t) * (size_t)cap); }
            if (nl) memcpy(found + nfound, loc, sizeof(uint64_t) * (size_t)nl);
            nfound += nl;
        }
        free(loc);
    }
    qsort(found, (size_t)nfound, sizeof(uint64_t), bp_cmp_u64);
    for (int64_t k = 0; k < nfound && k < max_pairs; ++k) {
        pairs[2 * k] = (int32_t)(found[k] >> 32);
        pairs[2 * k + 1] = (int32_t)(found[k] & 0xffffffffu);
    }
    *n_pairs = nfound;
    free(found); free(cells); free(m); free(r); free(ok);
    return 0;
}
