"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU restatement (oracle/gjkepa_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this, and only as the
checker / CPU baseline.  Parity with the reference is unpinned (see gjkepa_oracle.h).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libgjkepa_oracle.so")

REC64 = np.dtype([
    ("penetration_depth", "<f8"), ("collision_normal", "<f8", (3,)), ("collision_point", "<f8", (3,)),
    ("nearest_points", "<f8", (6,)), ("collision", "i1"), ("colli_type", "i1"), ("status", "i1"),
    ("reserved", "i1"), ("diag", "<u4"), ("pad", "<u4", (4,)),
])

_lib = None


def build() -> str:
    subprocess.run(["make", "-C", _HERE, "-s"], check=True)
    return LIB_PATH


def load() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        lib = ctypes.CDLL(LIB_PATH)
        vp, i32, i64, dbl = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double
        lib.oracle_gjkepa.argtypes = [i32, dbl, vp, i32, vp, i32, vp]
        lib.oracle_gjkepa.restype = ctypes.c_int
        lib.oracle_gjkepa_batch.argtypes = [i32, dbl, i32, vp, vp, vp, vp, i64, vp, i32]
        lib.oracle_gjkepa_batch.restype = ctypes.c_int
        lib.oracle_max_threads.restype = ctypes.c_int
        _lib = lib
    return _lib


def gjkepa(version: int, tol_ff: float, p1, p2) -> np.ndarray:
    """One pair; p1, p2 are (n, 3).  Returns a REC64 record (0-d structured array)."""
    a = np.ascontiguousarray(np.asarray(p1, np.float64).T)
    b = np.ascontiguousarray(np.asarray(p2, np.float64).T)
    out = np.zeros(1, REC64)
    rc = load().oracle_gjkepa(int(version), float(tol_ff), a.ctypes.data, a.shape[1], b.ctypes.data, b.shape[1],
                              out.ctypes.data)
    assert rc == 0
    return out[0]


def gjkepa_batch(pool, version: int = 2, tol_ff: float = 1.0, nthreads: int = 0) -> np.ndarray:
    """Batch over a gjkepa.HullPool-like object (verts, hull_off, hull_cnt, pairs)."""
    verts = np.ascontiguousarray(pool.verts)
    code = 0 if verts.dtype == np.float32 else 1
    off = np.ascontiguousarray(pool.hull_off, np.int64)
    cnt = np.ascontiguousarray(pool.hull_cnt, np.int32)
    prs = np.ascontiguousarray(pool.pairs, np.int32).reshape(-1)
    n = prs.size // 2
    out = np.zeros(n, REC64)
    rc = load().oracle_gjkepa_batch(int(version), float(tol_ff), code, verts.ctypes.data, off.ctypes.data,
                                    cnt.ctypes.data, prs.ctypes.data, n, out.ctypes.data, int(nthreads))
    assert rc == 0
    return out


_lib32 = None


def gjkepa_batch_f32(pool, version: int = 2, tol_ff: float = 1.0, nthreads: int = 0) -> np.ndarray:
    """DIAGNOSTIC: the same restatement compiled in fp32 arithmetic with the kernels' fp32 tolerances
    (gjkepa_oracle.c ORC_F32), to study the fp32-compute path on the CPU.  REC64 records holding fp32
    values.  Not a parity reference for anything."""
    global _lib32
    if _lib32 is None:
        p = os.path.join(_HERE, "build", "libgjkepa_oracle_f32.so")
        if not os.path.exists(p):
            build()
        lib = ctypes.CDLL(p)
        lib.oracle_gjkepa_batch.argtypes = [ctypes.c_int32, ctypes.c_double, ctypes.c_int32, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                            ctypes.c_void_p, ctypes.c_int32]
        lib.oracle_gjkepa_batch.restype = ctypes.c_int
        _lib32 = lib
    verts = np.ascontiguousarray(pool.verts, np.float32)
    off = np.ascontiguousarray(pool.hull_off, np.int64)
    cnt = np.ascontiguousarray(pool.hull_cnt, np.int32)
    prs = np.ascontiguousarray(pool.pairs, np.int32).reshape(-1)
    n = prs.size // 2
    out = np.zeros(n, REC64)
    rc = _lib32.oracle_gjkepa_batch(int(version), float(tol_ff), 0, verts.ctypes.data, off.ctypes.data,
                                    cnt.ctypes.data, prs.ctypes.data, n, out.ctypes.data, int(nthreads))
    assert rc == 0
    return out


# ORC_BR_* bit names (gjkepa_oracle.h), in bit order
BRANCHES = [
    "SPHERE_MISS", "INIT_RETRY", "INIT_CAP", "INIT_S3_COINCIDE", "INIT_TRI_HIT", "INIT_TRI_PLANE",
    "INIT_COPLANAR", "INIT_TETRA_HIT", "INIT_TETRA_ONFACE", "LOOP_CAP", "LOOP_COLLINEAR", "LOOP_COPLANAR",
    "LOOP_HIT", "LOOP_ONFACE", "LOOP_CYCLE", "IPF_XZ", "EPA_CENTROID", "EPA_FLIP", "EPA_TWO", "EPA_SWALLOW",
    "EPA_STOP_EQUAL", "EPA_STOP_SHRINK", "EPA_CAP", "DEGENERATE", "BAD_VERSION", "BAD_INPUT",
    "V1_MID", "V1_B", "V1_A", "V1_MEAN", "V2_CASE01", "V2_CASE02", "V2_CASE02B", "V2_CASE03", "V2_CASE04",
    "V2_CASE04B", "V2_CASE04_1", "V2_CASE04_2", "V2_CASE04_3", "V2_CASE05", "V2_OVERLAP", "FOOTLL_PARALLEL",
    "V3_NAN", "TYPE1", "TYPE2",
]
BR = {name: i for i, name in enumerate(BRANCHES)}


def gjkepa_batch_cov(pool, version: int = 2, tol_ff: float = 1.0, nthreads: int = 0):
    """gjkepa_batch plus, per pair, the uint64 mask of reference branches taken (bit BR[name])."""
    verts = np.ascontiguousarray(pool.verts)
    code = 0 if verts.dtype == np.float32 else 1
    off = np.ascontiguousarray(pool.hull_off, np.int64)
    cnt = np.ascontiguousarray(pool.hull_cnt, np.int32)
    prs = np.ascontiguousarray(pool.pairs, np.int32).reshape(-1)
    n = prs.size // 2
    out = np.zeros(n, REC64)
    cov = np.zeros(n, np.uint64)
    lib = load()
    if not hasattr(lib, "_cov_typed"):
        vp, i32 = ctypes.c_void_p, ctypes.c_int32
        lib.oracle_gjkepa_batch_cov.argtypes = [i32, ctypes.c_double, i32, vp, vp, vp, vp, ctypes.c_int64, vp, vp, i32]
        lib.oracle_gjkepa_batch_cov.restype = ctypes.c_int
        lib._cov_typed = True
    rc = lib.oracle_gjkepa_batch_cov(int(version), float(tol_ff), code, verts.ctypes.data, off.ctypes.data,
                                     cnt.ctypes.data, prs.ctypes.data, n, out.ctypes.data, cov.ctypes.data,
                                     int(nthreads))
    assert rc == 0
    return out, cov


def branch_histogram(cov) -> dict:
    """{branch name: number of pairs that took it}."""
    cov = np.asarray(cov, np.uint64)
    return {name: int(((cov >> np.uint64(i)) & np.uint64(1)).sum()) for i, name in enumerate(BRANCHES)}


def max_threads() -> int:
    return int(load().oracle_max_threads())


def hull_face_offsets(cnt) -> np.ndarray:
    """Triangle offset of each cloud's face block: exclusive prefix sum of 2n - 4 (0 for n < 4)."""
    cap = np.where(np.asarray(cnt) >= 4, 2 * np.asarray(cnt, np.int64) - 4, 0)
    off = np.zeros(len(cap), np.int64)
    if len(cap) > 1:
        off[1:] = np.cumsum(cap)[:-1]
    return off


def hull_batch(verts, cloud_off, cloud_cnt, nthreads: int = 0) -> dict:
    """Convex hull of every cloud of a pool (gjkepa_hull_batch semantics).  Returns a dict with
    faces (int32 [sum(2n-4), 3]), face_off, n_faces, n_verts, status, hull_verts, vert_idx."""
    verts = np.ascontiguousarray(verts)
    code = 0 if verts.dtype == np.float32 else 1
    off = np.ascontiguousarray(cloud_off, np.int64)
    cnt = np.ascontiguousarray(cloud_cnt, np.int32)
    n = len(cnt)
    foff = hull_face_offsets(cnt)
    nslots = int(foff[-1] + max(2 * int(cnt[-1]) - 4, 0)) if n else 0
    faces = np.full((max(nslots, 1), 3), -1, np.int32)
    nf = np.zeros(n, np.int32)
    nv = np.zeros(n, np.int32)
    st = np.zeros(n, np.int8)
    hv = np.zeros_like(verts)
    vi = np.full(verts.size, -1, np.int32)
    lib = load()
    if not hasattr(lib, "_hull_typed"):
        vp = ctypes.c_void_p
        lib.oracle_hull_batch.argtypes = [ctypes.c_int32, vp, vp, vp, ctypes.c_int64, vp, vp, vp, vp, vp, vp, vp,
                                          ctypes.c_int32]
        lib.oracle_hull_batch.restype = ctypes.c_int
        lib._hull_typed = True
    rc = lib.oracle_hull_batch(code, verts.ctypes.data, off.ctypes.data, cnt.ctypes.data, n, foff.ctypes.data,
                               faces.ctypes.data, nf.ctypes.data, nv.ctypes.data, st.ctypes.data, hv.ctypes.data,
                               vi.ctypes.data, int(nthreads))
    assert rc == 0
    return dict(faces=faces[:nslots], face_off=foff, n_faces=nf, n_verts=nv, status=st, hull_verts=hv,
                vert_idx=vi)


def broadphase(verts, hull_off, hull_cnt, max_pairs: int = -1, nthreads: int = 0):
    """Every pair a < b passing the reference's sphere test, ascending (a, b).  Returns
    (pairs int32 [n, 2], n_found)."""
    verts = np.ascontiguousarray(verts)
    code = 0 if verts.dtype == np.float32 else 1
    off = np.ascontiguousarray(hull_off, np.int64)
    cnt = np.ascontiguousarray(hull_cnt, np.int32)
    lib = load()
    if not hasattr(lib, "_bp_typed"):
        vp = ctypes.c_void_p
        lib.oracle_broadphase.argtypes = [ctypes.c_int32, vp, vp, vp, ctypes.c_int64, vp, ctypes.c_int64, vp,
                                          ctypes.c_int32]
        lib.oracle_broadphase.restype = ctypes.c_int
        lib._bp_typed = True
    nf = np.zeros(1, np.int64)
    if max_pairs < 0:   # size query first
        assert lib.oracle_broadphase(code, verts.ctypes.data, off.ctypes.data, cnt.ctypes.data, cnt.size, None, 0,
                                     nf.ctypes.data, int(nthreads)) == 0
        max_pairs = int(nf[0])
    out = np.zeros((max(max_pairs, 1), 2), np.int32)
    assert lib.oracle_broadphase(code, verts.ctypes.data, off.ctypes.data, cnt.ctypes.data, cnt.size, out.ctypes.data,
                                 max_pairs, nf.ctypes.data, int(nthreads)) == 0
    return out[:min(max_pairs, int(nf[0]))], int(nf[0])
