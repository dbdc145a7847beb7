"""ctypes binding of the C-ABI in include/l5dhist.h (linkerd_amd/lib/libl5dhist.so).

This is the same boundary a JVM would bind through JNI.  There
is no fallback: if the HIP library is missing, importing the engine raises.
"""
from __future__ import annotations

import ctypes
import errno
import os
import re
import threading

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
# L5DH_LIB selects another build of the same library (A/B timing of kernel variants: tools/ab.sh)
LIB_PATH = os.environ.get("L5DH_LIB") or os.path.join(PKG_DIR, "lib", "libl5dhist.so")
SYNTH_PATH = os.path.join(PKG_DIR, "lib", "libl5dsynth.so")
HEADER_PATH = os.path.join(REPO_DIR, "include", "l5dhist.h")

NLIMITS = 1797
NBUCKETS = 1798
SUMMARY_FIELDS = ("count", "min", "max", "sum", "p50", "p90", "p95", "p99", "p9990", "p9999", "avg")
SUMMARY_DTYPE = np.dtype([(f, "<i8") for f in SUMMARY_FIELDS[:-1]] + [("avg", "<f8")])
BUCKET_COUNT_DTYPE = np.dtype([("lower", "<i4"), ("upper", "<i4"), ("count", "<i4")])

PARAM_TIMING = 1
PARAM_COLD_LIMIT = 2
PARAM_HOT_CHUNK = 3
PARAM_MAX_SEGMENTS = 4
PARAM_DIRECT_MAX = 6
PARAM_DIRECT_DIV = 7
PARAM_STAGE_SAMPLES = 9
PARAM_MAX_SLABS = 10
PARAM_MERGE_RCCL_1RANK = 11
PARAM_VARIANT = 12
PARAM_REGION_PCT = 13

MERGE_REDUCE_SCATTER = 0
MERGE_ALL_REDUCE = 1
UNIQUE_ID_BYTES = 128
OWN_STREAM = ctypes.c_void_p(-1 & (2 ** 64 - 1)).value  # L5DH_OWN_STREAM

K_COUNT, K_SCAN, K_BIN, K_ACCUM, K_HOT, K_COPY, K_BIN2, K_MERGE = range(8)
KERNEL_NAMES = ("count", "scan", "bin1", "accum", "hot", "copy", "bin2", "merge")


class NativeLibraryMissing(ImportError):
    pass


class L5dhError(RuntimeError):
    def __init__(self, code: int, where: str, detail: str = ""):
        self.code = code
        name = errno.errorcode.get(-code, str(code)) if code < 0 else str(code)
        super().__init__(f"{where} failed: {name} ({code}) {detail}".rstrip())


_lock = threading.Lock()
_lib = None

_c = ctypes
_vp = _c.c_void_p
SIGNATURES = {
    "l5dh_abi_version": (_c.c_int, []),
    "l5dh_open": (_c.c_int, [_c.POINTER(_vp), _c.c_uint32, _c.c_uint32]),
    "l5dh_close": (_c.c_int, [_vp]),
    "l5dh_limits": (_c.POINTER(_c.c_int32), [_c.POINTER(_c.c_size_t)]),
    "l5dh_ingest": (_c.c_int, [_vp, _vp, _vp, _c.c_size_t]),
    "l5dh_ingest_async": (_c.c_int, [_vp, _vp, _vp, _c.c_size_t, _c.POINTER(_c.c_uint64)]),
    "l5dh_ingest_wait": (_c.c_int, [_vp, _c.c_uint64]),
    "l5dh_snapshot": (_c.c_int, [_vp, _c.c_uint32, _c.c_uint32, _vp, _vp, _c.c_int]),
    "l5dh_peek": (_c.c_int, [_vp, _c.c_uint32, _vp, _c.c_size_t, _c.POINTER(_c.c_size_t)]),
    "l5dh_export_state": (_c.c_int, [_vp, _c.c_uint32, _c.c_uint32, _vp, _vp, _c.c_int]),
    "l5dh_summarize_dense": (_c.c_int, [_vp, _vp, _vp, _c.c_size_t, _vp]),
    "l5dh_sync": (_c.c_int, [_vp]),
    "l5dh_set_stream": (_c.c_int, [_vp, _vp]),
    "l5dh_wait_event": (_c.c_int, [_vp, _vp]),
    "l5dh_set_param": (_c.c_int, [_vp, _c.c_int, _c.c_int64]),
    "l5dh_kernel_time": (_c.c_int, [_vp, _c.c_int, _c.POINTER(_c.c_double), _c.POINTER(_c.c_int64), _c.c_int]),
    "l5dh_device": (_c.c_int, [_vp, _c.POINTER(_c.c_int)]),
    "l5dh_max_series": (_c.c_uint32, [_vp]),
    "l5dh_pin_alloc": (_c.c_int, [_c.c_size_t, _c.POINTER(_vp)]),
    "l5dh_pin_free": (_c.c_int, [_vp]),
    "l5dh_last_error": (_c.c_char_p, [_vp]),
    "l5dh_comm_unique_id": (_c.c_int, [_vp]),
    "l5dh_comm_init_rank": (_c.c_int, [_vp, _vp, _c.c_int, _c.c_int]),
    "l5dh_comm_init_all": (_c.c_int, [_c.POINTER(_vp), _c.c_int]),
    "l5dh_comm_init_loopback": (_c.c_int, [_c.POINTER(_vp), _c.c_int]),
    "l5dh_comm_destroy": (_c.c_int, [_vp]),
    "l5dh_merge": (_c.c_int, [_vp, _c.c_int, _vp, _vp, _vp, _c.POINTER(_c.c_uint32), _c.POINTER(_c.c_uint32)]),
    "l5dh_tile_totals": (_c.c_int, [_vp, _c.POINTER(_c.c_uint64), _c.c_size_t]),
    "l5dh_merge_bytes": (_c.c_int, [_vp, _c.POINTER(_c.c_uint64), _c.POINTER(_c.c_uint64), _c.POINTER(_c.c_uint64)]),
    "l5dh_partition_redos": (_c.c_int, [_vp, _c.POINTER(_c.c_uint64), _c.POINTER(_c.c_uint64),
                                        _c.POINTER(_c.c_uint64)]),
    "l5dh_merge_all": (_c.c_int, [_c.POINTER(_vp), _c.c_int, _c.c_int, _c.POINTER(_vp), _c.POINTER(_vp),
                                  _c.POINTER(_vp), _c.POINTER(_c.c_uint32), _c.POINTER(_c.c_uint32)]),
}


def engine_source_hash() -> str:
    """sha256 (16 hex) of the engine's kernel and host sources: ties committed
    profiles (PMC traffic) to the code they measured."""
    import hashlib
    h = hashlib.sha256()
    d = os.path.join(PKG_DIR, "csrc")
    for f in sorted(os.listdir(d)):
        if f.endswith((".hip", ".hpp", ".cpp")) and "synth" not in f:
            h.update(f.encode())
            h.update(open(os.path.join(d, f), "rb").read())
    return h.hexdigest()[:16]


def header_symbols(path: str = HEADER_PATH) -> list:
    """Function names declared in include/l5dhist.h."""
    text = open(path).read()
    return sorted(set(re.findall(r"\b(l5dh_[a-z_0-9]+)\s*\(", text)))


def load(path: str = LIB_PATH):
    """Load the HIP engine library; raises NativeLibraryMissing if absent."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        # One HIP runtime per process: torch ships libamdhip64.so with the same
        # soname as /opt/rocm's.  Loading torch first makes our DT_NEEDED resolve
        # to the already-mapped runtime instead of mapping a second one.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(path):
            raise NativeLibraryMissing(
                f"{path} not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                "(or make -C linkerd_amd/csrc); there is no CPU fallback")
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("L5DH_LIB") and not hasattr(lib, name):
                continue  # (an A/B build of an older revision: entry points it predates are absent)
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def limits() -> np.ndarray:
    lib = load()
    n = ctypes.c_size_t(0)
    p = lib.l5dh_limits(ctypes.byref(n))
    if not p or n.value != NLIMITS:
        raise L5dhError(-errno.EIO, "l5dh_limits")
    return np.ctypeslib.as_array(p, shape=(NLIMITS,)).copy()
