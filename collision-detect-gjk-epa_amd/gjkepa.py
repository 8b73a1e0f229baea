"""Python host binding of the MI355X GJK/EPA C-ABI (include/gjkepa.h) via ctypes.

Mirrors the reference's operator interface: ``gjkepa(version, tol_ff, p1, p2)`` answers one
pair exactly like ``CALL GJKEPA(version_, TOL_FF_, p1_, p2_, ...)`` in
src/GCLIB_GJKEPA.f90:39-52 (same argument meaning; p1/p2 are (n, 3) vertex arrays) and returns
the reference's INTENT(OUT) arguments.  ``gjkepa_batch`` runs a pooled hull set; the
``*_device`` form takes device pointers (e.g. torch tensors on cuda) and an optional stream.

There is no CPU fallback: importing works without a GPU (so the library can be inspected),
but every compute call goes to libgjkepa_hip.so and fails loudly if it cannot run.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libgjkepa_hip.so")
FLIB_PATH = os.path.join(_HERE, "build", "libgclib_gjkepa.so")

STATUS_OK, STATUS_EPA_MAXITER, STATUS_DEGENERATE, STATUS_BAD_VERSION, STATUS_BAD_INPUT = 0, 1, 2, 3, 4
DTYPE_F32, DTYPE_F64 = 0, 1
PREC_F32, PREC_F64 = 0, 1
MAX_HULL_VERTS = 256

# exported symbols declared in include/gjkepa.h
EXPORTS = (
    "gjkepa_record_bytes", "gjkepa_query", "gjkepa_batch", "gjkepa_workspace_bytes",
    "gjkepa_batch_device", "gjkepa_last_error", "gjkepa_version_string", "gjkepa_synth_pairs",
    "gjkepa_hull_face_capacity", "gjkepa_hull_batch", "gjkepa_hull_batch_device", "gjkepa_synth_clouds",
    "gjkepa_broadphase_workspace_bytes", "gjkepa_broadphase", "gjkepa_broadphase_device", "gjkepa_synth_scene",
    "gjkepa_compact_workspace_bytes", "gjkepa_compact_hits_device", "gjkepa_batch_warm_device",
    "gjkepa_collide", "gjkepa_shard_range", "gjkepa_batch_multi", "gjkepa_comm_unique_id", "gjkepa_comm_init",
    "gjkepa_comm_destroy", "gjkepa_comm_backend", "gjkepa_allgather_records_device",
    "gjkepa_query_service_stop", "gjkepa_query_service_set", "gjkepa_query_service_resident", "gjkepa_workspace_bytes_for",
    "gjkepa_launch_timing", "gjkepa_launch_timing_read",
)
COMM_ID_BYTES = 128
# workspace header word counting the park slots a gjkepa_batch_device call took (diagnostics; csrc/
# gjkepa_capi.cpp kWsParkWord = GJKEPA_WS_COUNTERS + GJKEPA_WS_TALLY)
WS_COUNTERS, WS_TALLY = 40, 48   # gjkepa_kernel.h GJKEPA_WS_COUNTERS / GJKEPA_WS_TALLY (uint32 words)
WS_PARK_WORD = WS_COUNTERS + WS_TALLY
HULL_MAX_POINTS = 256

REC64 = np.dtype([
    ("penetration_depth", "<f8"), ("collision_normal", "<f8", (3,)), ("collision_point", "<f8", (3,)),
    ("nearest_points", "<f8", (6,)), ("collision", "i1"), ("colli_type", "i1"), ("status", "i1"),
    ("reserved", "i1"), ("diag", "<u4"), ("pad", "<u4", (4,)),
])
REC32 = np.dtype([
    ("penetration_depth", "<f4"), ("collision_normal", "<f4", (3,)), ("collision_point", "<f4", (3,)),
    ("nearest_points", "<f4", (6,)), ("collision", "i1"), ("colli_type", "i1"), ("status", "i1"),
    ("reserved", "i1"), ("diag", "<u4"), ("pad", "<u4"),
])
assert REC64.itemsize == 128 and REC32.itemsize == 64


def record_dtype(precision: int) -> np.dtype:
    return REC64 if precision == PREC_F64 else REC32


_lib = None


class GjkEpaError(RuntimeError):
    pass


def load(path: str | None = None) -> ctypes.CDLL:
    """Load libgjkepa_hip.so (built in-tree by ``make`` / __graft_entry__.build())."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("GJKEPA_LIB") or LIB_PATH
    try:
        # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so.7 (same soname as
        # /opt/rocm's).  Whichever loads first serves both, and torch's device init fails when it
        # finds the system runtime already mapped, so bring torch's in first when torch is present.
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(p):
        raise GjkEpaError(f"{p} not built; run `make -C collision-detect-gjk-epa_amd`")
    lib = ctypes.CDLL(p)
    c_i32, c_i64, c_dbl, c_vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p
    lib.gjkepa_record_bytes.argtypes = [c_i32]
    lib.gjkepa_record_bytes.restype = ctypes.c_int
    lib.gjkepa_workspace_bytes.argtypes = [c_i64]
    lib.gjkepa_workspace_bytes.restype = c_i64
    lib.gjkepa_last_error.restype = ctypes.c_char_p
    lib.gjkepa_version_string.restype = ctypes.c_char_p
    lib.gjkepa_query.argtypes = [c_i32, c_dbl, c_vp, c_i32, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32]
    lib.gjkepa_query.restype = ctypes.c_int
    lib.gjkepa_batch.argtypes = [c_i32, c_dbl, c_i32, c_i32, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_i32]
    lib.gjkepa_batch.restype = ctypes.c_int
    lib.gjkepa_batch_device.argtypes = [c_i32, c_dbl, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp]
    lib.gjkepa_batch_device.restype = ctypes.c_int
    lib.gjkepa_synth_pairs.argtypes = [ctypes.c_uint64, c_i64, c_i64, c_i32, c_i32, c_dbl, c_i32, c_vp, c_vp, c_vp, c_vp]
    lib.gjkepa_synth_pairs.restype = c_i64
    lib.gjkepa_hull_face_capacity.argtypes = [c_i32]
    lib.gjkepa_hull_face_capacity.restype = c_i64
    lib.gjkepa_hull_batch.argtypes = [c_i32, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                      c_vp, c_i32]
    lib.gjkepa_hull_batch.restype = ctypes.c_int
    lib.gjkepa_hull_batch_device.argtypes = [c_i32, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                             c_vp]
    lib.gjkepa_hull_batch_device.restype = ctypes.c_int
    lib.gjkepa_synth_clouds.argtypes = [ctypes.c_uint64, c_i64, c_i64, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp]
    lib.gjkepa_synth_clouds.restype = c_i64
    lib.gjkepa_broadphase_workspace_bytes.argtypes = [c_i64, c_i64]
    lib.gjkepa_broadphase_workspace_bytes.restype = c_i64
    lib.gjkepa_broadphase.argtypes = [c_i32, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_i32]
    lib.gjkepa_broadphase.restype = ctypes.c_int
    lib.gjkepa_broadphase_device.argtypes = [c_i32, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp]
    lib.gjkepa_broadphase_device.restype = ctypes.c_int
    lib.gjkepa_synth_scene.argtypes = [ctypes.c_uint64, c_i64, c_i64, c_i32, c_i32, c_dbl, c_i32, c_vp, c_vp, c_vp]
    lib.gjkepa_synth_scene.restype = c_i64
    lib.gjkepa_compact_workspace_bytes.argtypes = [c_i64]
    lib.gjkepa_compact_workspace_bytes.restype = c_i64
    lib.gjkepa_compact_hits_device.argtypes = [c_i32, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]
    lib.gjkepa_compact_hits_device.restype = ctypes.c_int
    lib.gjkepa_batch_warm_device.argtypes = [c_i32, c_dbl, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64,
                                             c_vp, c_vp]
    lib.gjkepa_batch_warm_device.restype = ctypes.c_int
    lib.gjkepa_collide.argtypes = [c_i32, c_dbl, c_i32, c_i32, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp,
                                   c_vp, c_i32]
    lib.gjkepa_collide.restype = ctypes.c_int
    lib.gjkepa_shard_range.argtypes = [c_i64, c_i32, c_i32, c_vp, c_vp]
    lib.gjkepa_shard_range.restype = ctypes.c_int
    lib.gjkepa_batch_multi.argtypes = [c_i32, c_dbl, c_i32, c_i32, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp,
                                       c_vp, c_i32]
    lib.gjkepa_batch_multi.restype = ctypes.c_int
    lib.gjkepa_comm_unique_id.argtypes = [c_vp]
    lib.gjkepa_comm_unique_id.restype = ctypes.c_int
    lib.gjkepa_comm_init.argtypes = [c_vp, c_i32, c_i32, c_vp, c_i32]
    lib.gjkepa_comm_init.restype = ctypes.c_int
    lib.gjkepa_comm_destroy.argtypes = [c_vp]
    lib.gjkepa_comm_destroy.restype = ctypes.c_int
    lib.gjkepa_comm_backend.restype = ctypes.c_char_p
    lib.gjkepa_allgather_records_device.argtypes = [c_vp, c_i32, c_vp, c_vp, c_i64, c_vp]
    lib.gjkepa_allgather_records_device.restype = ctypes.c_int
    lib.gjkepa_query_service_stop.argtypes = [c_i32]
    lib.gjkepa_query_service_stop.restype = ctypes.c_int
    lib.gjkepa_query_service_set.argtypes = [c_i32]
    lib.gjkepa_query_service_set.restype = ctypes.c_int
    lib.gjkepa_query_service_resident.argtypes = [c_i32]
    lib.gjkepa_query_service_resident.restype = ctypes.c_int
    lib.gjkepa_workspace_bytes_for.argtypes = [c_i64, c_i64]
    lib.gjkepa_workspace_bytes_for.restype = c_i64
    lib.gjkepa_launch_timing.argtypes = [c_i32]
    lib.gjkepa_launch_timing.restype = ctypes.c_int
    lib.gjkepa_launch_timing_read.argtypes = [c_vp, c_i32]
    lib.gjkepa_launch_timing_read.restype = ctypes.c_int
    if path is None:
        _lib = lib
    return lib


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().gjkepa_last_error().decode(errors="replace")
        raise GjkEpaError(f"{what} failed ({rc}): {msg}")


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


@dataclass
class Contact:
    """GJKEPA's INTENT(OUT) arguments (GCLIB_GJKEPA.f90:47-52) plus the status code."""
    collision: bool
    colli_type: int
    nearest_points: np.ndarray     # (2, 3): row 0 on p1, row 1 on p2
    collision_normal: np.ndarray   # (3,)
    collision_point: np.ndarray    # (3,)
    penetration_depth: float
    status: int


def gjkepa(version: int, tol_ff: float, p1, p2, device: int = 0) -> Contact:
    """One pair on the GPU; same arguments as the reference GJKEPA (p1, p2: (n, 3))."""
    lib = load()
    a = np.ascontiguousarray(np.asarray(p1, dtype=np.float64).T)   # column-major (n,3) = x[], y[], z[]
    b = np.ascontiguousarray(np.asarray(p2, dtype=np.float64).T)
    hit = np.zeros(1, np.int8)
    typ = np.zeros(1, np.int32)
    st = np.zeros(1, np.int32)
    npf = np.zeros(6)
    nrm = np.zeros(3)
    pt = np.zeros(3)
    dep = np.zeros(1)
    rc = lib.gjkepa_query(int(version), float(tol_ff), _ptr(a), a.shape[1], _ptr(b), b.shape[1],
                          _ptr(hit), _ptr(typ), _ptr(npf), _ptr(nrm), _ptr(pt), _ptr(dep), _ptr(st), int(device))
    _check(rc, "gjkepa_query")
    return Contact(bool(hit[0]), int(typ[0]), npf.reshape(3, 2).T.copy(), nrm, pt, float(dep[0]), int(st[0]))


def query_service_stop(device: int = -1) -> None:
    """Drain the resident grid behind gjkepa() (include/gjkepa.h): call before a device-wide
    synchronisation such as torch.cuda.synchronize() while single-pair calls may have run."""
    _check(load().gjkepa_query_service_stop(int(device)), "gjkepa_query_service_stop")


def query_service_resident(device: int = -1) -> bool:
    """Whether a resident service grid is still on the GPU (gjkepa_query_service_resident)."""
    rc = load().gjkepa_query_service_resident(int(device))
    _check(min(rc, 0), "gjkepa_query_service_resident")
    return rc == 1


def query_service_set(enabled: bool) -> bool:
    """Turn the resident query service on/off for later gjkepa() calls; returns the previous setting."""
    rc = load().gjkepa_query_service_set(1 if enabled else 0)
    if rc < 0:
        _check(rc, "gjkepa_query_service_set")
    return bool(rc)


@dataclass
class HullPool:
    """Pooled hulls: hull h = verts[off[h] : off[h] + 3*cnt[h]] as x[], y[], z[]."""
    verts: np.ndarray    # float32 or float64
    hull_off: np.ndarray  # int64
    hull_cnt: np.ndarray  # int32
    pairs: np.ndarray     # int32 (n_pairs, 2)

    @property
    def n_pairs(self) -> int:
        return int(self.pairs.shape[0])

    @property
    def dtype_code(self) -> int:
        return DTYPE_F32 if self.verts.dtype == np.float32 else DTYPE_F64

    def hull(self, h: int) -> np.ndarray:
        o, n = int(self.hull_off[h]), int(self.hull_cnt[h])
        return self.verts[o:o + 3 * n].reshape(3, n).T.astype(np.float64)

    def as_dtype(self, dt) -> "HullPool":
        return HullPool(self.verts.astype(dt), self.hull_off, self.hull_cnt, self.pairs)

    @staticmethod
    def from_pairs(pairs_list, dtype=np.float64) -> "HullPool":
        """Build a pool from a list of (p1, p2) (n,3) arrays."""
        chunks, off, cnt, pr = [], [], [], []
        o = 0
        for k, (a, b) in enumerate(pairs_list):
            for h in (a, b):
                h = np.asarray(h, dtype=np.float64).reshape(-1, 3)
                chunks.append(h.T.reshape(-1))
                off.append(o)
                cnt.append(h.shape[0])
                o += 3 * h.shape[0]
            pr.append((2 * k, 2 * k + 1))
        verts = np.concatenate(chunks).astype(dtype) if chunks else np.zeros(0, dtype)
        return HullPool(verts, np.asarray(off, np.int64), np.asarray(cnt, np.int32),
                        np.asarray(pr, np.int32).reshape(-1, 2))


def synth_pairs(seed: int, n_pairs: int, n_min: int = 32, n_max: int = 32, r_max: float = 2.5,
                first_pair: int = 0, dtype=np.float32) -> HullPool:
    """Deterministic synthetic workload: C2 = (32, 32, 2.5), C4 = (8, 256, 2.5),
    C5 = (32..128, 0.3)."""
    lib = load()
    code = DTYPE_F32 if np.dtype(dtype) == np.float32 else DTYPE_F64
    total = lib.gjkepa_synth_pairs(seed, first_pair, n_pairs, n_min, n_max, r_max, code, None, None, None, None)
    if total < 0:
        raise GjkEpaError("gjkepa_synth_pairs: bad arguments")
    verts = np.empty(total, dtype=dtype)
    off = np.empty(2 * n_pairs, np.int64)
    cnt = np.empty(2 * n_pairs, np.int32)
    prs = np.empty(2 * n_pairs, np.int32)
    lib.gjkepa_synth_pairs(seed, first_pair, n_pairs, n_min, n_max, r_max, code, _ptr(verts), _ptr(off), _ptr(cnt), _ptr(prs))
    return HullPool(verts, off, cnt, prs.reshape(-1, 2))


def gjkepa_batch(pool: HullPool, version: int = 2, tol_ff: float = 1.0, precision: int = PREC_F64,
                 device: int = 0) -> np.ndarray:
    """Host-buffer batch on the GPU; returns a structured array of contact records."""
    lib = load()
    out = np.zeros(pool.n_pairs, dtype=record_dtype(precision))
    verts = np.ascontiguousarray(pool.verts)
    off = np.ascontiguousarray(pool.hull_off, np.int64)
    cnt = np.ascontiguousarray(pool.hull_cnt, np.int32)
    prs = np.ascontiguousarray(pool.pairs, np.int32).reshape(-1)
    rc = lib.gjkepa_batch(int(version), float(tol_ff), pool.dtype_code, int(precision), _ptr(verts), verts.size,
                          _ptr(off), _ptr(cnt), cnt.size, _ptr(prs), pool.n_pairs, _ptr(out), int(device))
    _check(rc, "gjkepa_batch")
    return out


def workspace_bytes(n_pairs: int) -> int:
    return int(load().gjkepa_workspace_bytes(n_pairs))


PARK_MIN_HULL = 32   # pairs with a hull above this many vertices can reach the parking EPA tiers


def large_pairs(pool: HullPool) -> int:
    """Pairs of the pool with a hull above PARK_MIN_HULL vertices (gjkepa_workspace_bytes_for)."""
    c = pool.hull_cnt[pool.pairs.astype(np.int64)]
    return int((c.max(axis=1) > PARK_MIN_HULL).sum()) if pool.n_pairs else 0


def workspace_bytes_for(n_pairs: int, n_large_pairs: int) -> int:
    """Workspace with park slots only for the pairs that can park (include/gjkepa.h)."""
    b = int(load().gjkepa_workspace_bytes_for(int(n_pairs), int(n_large_pairs)))
    if b < 0:
        raise GjkEpaError("gjkepa_workspace_bytes_for: bad arguments")
    return b


# per-launch timing of the tier chain (include/gjkepa.h gjkepa_launch_time)
LAUNCH_TIME = np.dtype([
    ("kernel", "S16"), ("tier", "<i4"), ("part", "<i4"), ("route_code", "<i4"), ("chain", "<i4"),
    ("stream", "<i4"), ("pad", "<i4"), ("first_pair", "<i8"), ("n_pairs", "<i8"), ("start_ms", "<f4"),
    ("end_ms", "<f4"),
])
assert LAUNCH_TIME.itemsize == 64


def launch_timing(enable: bool) -> bool:
    """Record HIP events around every kernel launch of the chains this thread enqueues from now on;
    returns the previous setting."""
    return bool(load().gjkepa_launch_timing(1 if enable else 0))


def launch_timing_read(max_launches: int = 1 << 16) -> np.ndarray:
    """Wait for the recorded launches and return them (LAUNCH_TIME records, enqueue order)."""
    buf = np.zeros(max_launches, LAUNCH_TIME)
    n = load().gjkepa_launch_timing_read(_ptr(buf), max_launches)
    if n < 0:
        _check(n, "gjkepa_launch_timing_read")
    return buf[:n]


def gjkepa_batch_device(version: int, tol_ff: float, vert_dtype: int, precision: int, verts_ptr: int,
                        hull_off_ptr: int, hull_cnt_ptr: int, pairs_ptr: int, n_pairs: int, out_ptr: int,
                        ws_ptr: int, ws_bytes: int, stream: int = 0) -> None:
    """Device-resident batch (raw device pointers), asynchronous on `stream`."""
    rc = load().gjkepa_batch_device(int(version), float(tol_ff), int(vert_dtype), int(precision), verts_ptr,
                                    hull_off_ptr, hull_cnt_ptr, pairs_ptr, int(n_pairs), out_ptr, ws_ptr,
                                    int(ws_bytes), stream or None)
    _check(rc, "gjkepa_batch_device")


def gjkepa_batch_warm_device(version: int, tol_ff: float, vert_dtype: int, precision: int, verts_ptr: int,
                             hull_off_ptr: int, hull_cnt_ptr: int, pairs_ptr: int, n_pairs: int, out_ptr: int,
                             ws_ptr: int, ws_bytes: int, warm_ptr: int, stream: int = 0) -> None:
    """gjkepa_batch_device with a per-pair warm-start slot array (device uint32[4 * n_pairs], in/out;
    0xFFFFFFFF = none): persistent pairs whose last simplex still encloses the origin skip GJK."""
    rc = load().gjkepa_batch_warm_device(int(version), float(tol_ff), int(vert_dtype), int(precision), verts_ptr,
                                         hull_off_ptr, hull_cnt_ptr, pairs_ptr, int(n_pairs), out_ptr, ws_ptr,
                                         int(ws_bytes), warm_ptr, stream or None)
    _check(rc, "gjkepa_batch_warm_device")


# ---- multi-GPU (SURVEY.md §8 row e; include/gjkepa.h gjkepa_shard_range / _batch_multi / _comm_*) ------
def shard_range(n_pairs: int, world: int, rank: int) -> tuple[int, int]:
    """(first, count): the contiguous shard of pairs `rank` of `world` owns (the library's rule)."""
    first, count = ctypes.c_int64(), ctypes.c_int64()
    _check(load().gjkepa_shard_range(int(n_pairs), int(world), int(rank), ctypes.byref(first), ctypes.byref(count)),
           "gjkepa_shard_range")
    return first.value, count.value


def gjkepa_batch_multi(pool: HullPool, devices, version: int = 2, tol_ff: float = 1.0,
                       precision: int = PREC_F64) -> np.ndarray:
    """One process driving several devices: pool's pairs in contiguous shards, shard s on devices[s];
    returns every record in pair order (bit-identical to gjkepa_batch)."""
    lib = load()
    out = np.zeros(pool.n_pairs, dtype=record_dtype(precision))
    verts = np.ascontiguousarray(pool.verts)
    off = np.ascontiguousarray(pool.hull_off, np.int64)
    cnt = np.ascontiguousarray(pool.hull_cnt, np.int32)
    prs = np.ascontiguousarray(pool.pairs, np.int32).reshape(-1)
    dev = np.ascontiguousarray(devices, np.int32)
    rc = lib.gjkepa_batch_multi(int(version), float(tol_ff), pool.dtype_code, int(precision), _ptr(verts), verts.size,
                                _ptr(off), _ptr(cnt), cnt.size, _ptr(prs), pool.n_pairs, _ptr(out), _ptr(dev),
                                dev.size)
    _check(rc, "gjkepa_batch_multi")
    return out


class Comm:
    """RCCL communicator of the contact-record exchange, one process per device (config C3).
    Rank 0 calls ``Comm.unique_id()``; the caller broadcasts those bytes (e.g. torch.distributed);
    every rank then builds ``Comm(world, rank, uid, device)``."""

    def __init__(self, world: int, rank: int, uid: bytes, device: int):
        if len(uid) != COMM_ID_BYTES:
            raise GjkEpaError("unique id must be COMM_ID_BYTES bytes")
        self.world, self.rank, self.device = world, rank, device
        self._h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(bytes(uid), COMM_ID_BYTES)
        _check(load().gjkepa_comm_init(ctypes.byref(self._h), int(world), int(rank), buf, int(device)),
               "gjkepa_comm_init")

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(COMM_ID_BYTES)
        _check(load().gjkepa_comm_unique_id(buf), "gjkepa_comm_unique_id")
        return buf.raw

    @staticmethod
    def backend() -> str:
        return load().gjkepa_comm_backend().decode()

    def allgather_records(self, precision: int, shard_ptr: int, all_ptr: int, count: int, stream: int = 0) -> None:
        """Every rank's `count` records (device pointer) into all_ptr[world * count], rank order; async."""
        _check(load().gjkepa_allgather_records_device(self._h, int(precision), shard_ptr, all_ptr, int(count),
                                                      stream or None), "gjkepa_allgather_records_device")

    def close(self) -> None:
        if self._h:
            _check(load().gjkepa_comm_destroy(self._h), "gjkepa_comm_destroy")
            self._h = ctypes.c_void_p()


def version_string() -> str:
    return load().gjkepa_version_string().decode()


def source_hash() -> str:
    """The hash of the sources the loaded library was built from (Makefile SRCHASH)."""
    return version_string().rsplit("src ", 1)[-1].strip()


# ---- batched convex hulls (include/gjkepa.h gjkepa_hull_batch) ----------------
@dataclass
class CloudPool:
    """Pooled point clouds: cloud c = verts[off[c] : off[c] + 3*cnt[c]] as x[], y[], z[]."""
    verts: np.ndarray      # float32 or float64
    cloud_off: np.ndarray  # int64
    cloud_cnt: np.ndarray  # int32

    @property
    def n_clouds(self) -> int:
        return int(self.cloud_cnt.shape[0])

    @property
    def dtype_code(self) -> int:
        return DTYPE_F32 if self.verts.dtype == np.float32 else DTYPE_F64

    def cloud(self, c: int) -> np.ndarray:
        o, n = int(self.cloud_off[c]), int(self.cloud_cnt[c])
        return self.verts[o:o + 3 * n].reshape(3, n).T.astype(np.float64)

    @staticmethod
    def from_list(clouds, dtype=np.float64) -> "CloudPool":
        chunks, off, cnt, o = [], [], [], 0
        for p in clouds:
            p = np.asarray(p, dtype=np.float64).reshape(-1, 3)
            chunks.append(p.T.reshape(-1))
            off.append(o)
            cnt.append(p.shape[0])
            o += 3 * p.shape[0]
        verts = np.concatenate(chunks).astype(dtype) if chunks else np.zeros(0, dtype)
        return CloudPool(verts, np.asarray(off, np.int64), np.asarray(cnt, np.int32))


def hull_face_offsets(cloud_cnt) -> np.ndarray:
    """Triangle offset of each cloud's face block (exclusive prefix sum of 2n - 4, 0 for n < 4)."""
    cnt = np.asarray(cloud_cnt, np.int64)
    cap = np.where(cnt >= 4, 2 * cnt - 4, 0)
    off = np.zeros(len(cap), np.int64)
    if len(cap) > 1:
        off[1:] = np.cumsum(cap)[:-1]
    return off


def synth_clouds(seed: int, n_clouds: int, n_min: int = 64, n_max: int = 64, shape: int = 0,
                 first_cloud: int = 0, dtype=np.float32) -> CloudPool:
    """Deterministic synthetic clouds: uniform in the unit ball (shape 0) or on the sphere (shape 1)."""
    lib = load()
    code = DTYPE_F32 if np.dtype(dtype) == np.float32 else DTYPE_F64
    total = lib.gjkepa_synth_clouds(seed, first_cloud, n_clouds, n_min, n_max, shape, code, None, None, None)
    if total < 0:
        raise GjkEpaError("gjkepa_synth_clouds: bad arguments")
    verts = np.empty(total, dtype=dtype)
    off = np.empty(n_clouds, np.int64)
    cnt = np.empty(n_clouds, np.int32)
    lib.gjkepa_synth_clouds(seed, first_cloud, n_clouds, n_min, n_max, shape, code, _ptr(verts), _ptr(off), _ptr(cnt))
    return CloudPool(verts, off, cnt)


def hull_batch(pool: CloudPool, device: int = 0) -> dict:
    """Convex hull of every cloud on the GPU (host buffers, blocking).  Returns faces (int32
    [sum(2n-4), 3], cloud c's n_faces[c] triangles at face_off[c]), face_off, n_faces, n_verts,
    status, hull_verts (pool layout: cloud c's hull at cloud_off[c], stride n_verts[c]) and
    vert_idx (cloud c's hull vertex indices at cloud_off[c])."""
    lib = load()
    verts = np.ascontiguousarray(pool.verts)
    off = np.ascontiguousarray(pool.cloud_off, np.int64)
    cnt = np.ascontiguousarray(pool.cloud_cnt, np.int32)
    n = cnt.size
    foff = hull_face_offsets(cnt)
    nslots = int(foff[-1] + max(2 * int(cnt[-1]) - 4, 0)) if n else 0
    faces = np.full((max(nslots, 1), 3), -1, np.int32)
    nf = np.zeros(n, np.int32)
    nv = np.zeros(n, np.int32)
    st = np.zeros(n, np.int8)
    hv = np.zeros_like(verts)
    vi = np.full(verts.size, -1, np.int32)
    rc = lib.gjkepa_hull_batch(pool.dtype_code, _ptr(verts), verts.size, _ptr(off), _ptr(cnt), n, _ptr(foff), nslots,
                               _ptr(faces), _ptr(nf), _ptr(nv), _ptr(st), _ptr(hv), _ptr(vi), int(device))
    _check(rc, "gjkepa_hull_batch")
    return dict(faces=faces[:nslots], face_off=foff, n_faces=nf, n_verts=nv, status=st, hull_verts=hv, vert_idx=vi)


def hull_batch_device(vert_dtype: int, points_ptr: int, cloud_off_ptr: int, cloud_cnt_ptr: int, n_clouds: int,
                      face_off_ptr: int, faces_ptr: int, n_faces_ptr: int, n_verts_ptr: int, status_ptr: int,
                      hull_verts_ptr: int = 0, vert_idx_ptr: int = 0, stream: int = 0) -> None:
    """Device-resident hull batch (raw device pointers), asynchronous on `stream`."""
    rc = load().gjkepa_hull_batch_device(int(vert_dtype), points_ptr, cloud_off_ptr, cloud_cnt_ptr, int(n_clouds),
                                         face_off_ptr, faces_ptr, n_faces_ptr, n_verts_ptr, status_ptr,
                                         hull_verts_ptr or None, vert_idx_ptr or None, stream or None)
    _check(rc, "gjkepa_hull_batch_device")


def quickhull(points, device: int = 0):
    """GCLIB_QuickHull::QuickHull(points, polytope, info) as called at GCLIB_GJKEPA.f90:950:
    the hull of an (n, 3) cloud as a triangle soup polytope(F, 3, 3) (face, vertex, xyz), outward
    wound; info = the GJKEPA_STATUS_* code (0 = OK)."""
    p = np.asarray(points, np.float64).reshape(-1, 3)
    r = hull_batch(CloudPool.from_list([p]), device)
    nf = int(r["n_faces"][0])
    return p[r["faces"][:nf]], int(r["status"][0])


def hull_mesh_vertices(polytope) -> np.ndarray:
    """GCLIB_DeHull::getHullMeshesVertex(polytope, points, info) (GCLIB_GJKEPA.f90:920): the
    distinct vertices of a triangle soup, in order of first appearance (host-side; exact equality)."""
    v = np.asarray(polytope, np.float64).reshape(-1, 3)
    _, first = np.unique(v, axis=0, return_index=True)
    return v[np.sort(first)]


# ---- device broad phase (include/gjkepa.h gjkepa_broadphase) -----------------
def synth_scene(seed: int, n_hulls: int, n_min: int = 32, n_max: int = 32, box: float = 10.0,
                first_hull: int = 0, dtype=np.float32) -> HullPool:
    """Deterministic scene: unit-sphere hulls centred uniformly in [0, box)^3 (pairs left empty)."""
    lib = load()
    code = DTYPE_F32 if np.dtype(dtype) == np.float32 else DTYPE_F64
    total = lib.gjkepa_synth_scene(seed, first_hull, n_hulls, n_min, n_max, box, code, None, None, None)
    if total < 0:
        raise GjkEpaError("gjkepa_synth_scene: bad arguments")
    verts = np.empty(total, dtype=dtype)
    off = np.empty(n_hulls, np.int64)
    cnt = np.empty(n_hulls, np.int32)
    lib.gjkepa_synth_scene(seed, first_hull, n_hulls, n_min, n_max, box, code, _ptr(verts), _ptr(off), _ptr(cnt))
    return HullPool(verts, off, cnt, np.zeros((0, 2), np.int32))


def broadphase(pool: HullPool, max_pairs: int | None = None, device: int = 0):
    """Candidate pairs (a < b, ascending) passing the reference's sphere test, on the GPU.
    Returns (pairs int32 [n, 2], n_found); with max_pairs None the list is grown until it fits."""
    lib = load()
    verts = np.ascontiguousarray(pool.verts)
    off = np.ascontiguousarray(pool.hull_off, np.int64)
    cnt = np.ascontiguousarray(pool.hull_cnt, np.int32)
    cap = max_pairs if max_pairs is not None else max(16 * cnt.size, 1024)
    while True:
        out = np.zeros((max(cap, 1), 2), np.int32)
        nf = np.zeros(1, np.int64)
        rc = lib.gjkepa_broadphase(pool.dtype_code, _ptr(verts), verts.size, _ptr(off), _ptr(cnt), cnt.size, _ptr(out),
                                   cap, _ptr(nf), int(device))
        _check(rc, "gjkepa_broadphase")
        n = int(nf[0])
        if n <= cap or max_pairs is not None:
            return out[:min(n, cap)], n
        cap = n


def broadphase_workspace_bytes(n_hulls: int, max_pairs: int) -> int:
    return int(load().gjkepa_broadphase_workspace_bytes(n_hulls, max_pairs))


def broadphase_device(vert_dtype: int, verts_ptr: int, hull_off_ptr: int, hull_cnt_ptr: int, n_hulls: int,
                      pairs_ptr: int, max_pairs: int, n_pairs_ptr: int, ws_ptr: int, ws_bytes: int,
                      stream: int = 0) -> None:
    """Device-resident broad phase (raw device pointers), asynchronous on `stream`."""
    rc = load().gjkepa_broadphase_device(int(vert_dtype), verts_ptr, hull_off_ptr, hull_cnt_ptr, int(n_hulls),
                                         pairs_ptr, int(max_pairs), n_pairs_ptr, ws_ptr, int(ws_bytes), stream or None)
    _check(rc, "gjkepa_broadphase_device")


# ---- contact-list compaction ----------------------------------------
def compact_workspace_bytes(n_pairs: int) -> int:
    return int(load().gjkepa_compact_workspace_bytes(n_pairs))


def compact_hits_device(precision: int, records_ptr: int, n_pairs: int, hit_idx_ptr: int, hits_ptr: int,
                        n_hits_ptr: int, ws_ptr: int, ws_bytes: int, stream: int = 0) -> None:
    """Dense, order-preserving list of the hit pairs of a device-resident batch (indices, and the
    records when hits_ptr is non-zero); *n_hits is a device int64."""
    rc = load().gjkepa_compact_hits_device(int(precision), records_ptr, int(n_pairs), hit_idx_ptr, hits_ptr or None,
                                           n_hits_ptr, ws_ptr, int(ws_bytes), stream or None)
    _check(rc, "gjkepa_compact_hits_device")


def collide(pool: HullPool, version: int = 2, tol_ff: float = 1.0, precision: int = PREC_F64,
            max_contacts: int | None = None, device: int = 0):
    """The all-pairs GJKEPA loop over a hull pool in one call (broad phase, narrow phase, hit list).
    Returns (pairs int32 [n, 2] with a < b ascending, records of those hits, n_candidates)."""
    lib = load()
    verts = np.ascontiguousarray(pool.verts)
    off = np.ascontiguousarray(pool.hull_off, np.int64)
    cnt = np.ascontiguousarray(pool.hull_cnt, np.int32)
    cap = max_contacts if max_contacts is not None else max(4 * cnt.size, 1024)
    while True:
        prs = np.zeros((max(cap, 1), 2), np.int32)
        out = np.zeros(max(cap, 1), dtype=record_dtype(precision))
        nc = np.zeros(1, np.int64)
        ncand = np.zeros(1, np.int64)
        rc = lib.gjkepa_collide(int(version), float(tol_ff), pool.dtype_code, int(precision), _ptr(verts), verts.size,
                                _ptr(off), _ptr(cnt), cnt.size, _ptr(prs), _ptr(out), cap, _ptr(nc), _ptr(ncand),
                                int(device))
        _check(rc, "gjkepa_collide")
        n = int(nc[0])
        if n <= cap or max_contacts is not None:
            m = min(n, cap)
            return prs[:m], out[:m], int(ncand[0])
        cap = n
