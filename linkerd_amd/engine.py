"""HistogramEngine: Python face of the C-ABI (one context = one GPU shard).

Mirrors what a JVM caller does through JNI: batched Stat.add (``ingest``) and
the timer-driven snapshot+reset (``snapshot``) of
AdminMetricsExportTelemeter.snapshotHistograms
(reference: telemetry/admin-metrics-export/.../AdminMetricsExportTelemeter.scala:154-162),
plus the RCCL fleet merge (``merge``).

Inputs may be numpy arrays (host) or torch tensors on the engine's GPU; outputs
go to numpy (host) or to caller-provided torch tensors (device).  Every buffer is
checked (dtype, device, size) before it reaches the library.  Calls that take a
device tensor first hand the library an event recorded on torch's current stream
(l5dh_wait_event), so the engine's kernels run after the torch work that produced
their inputs; calls with device outputs return once the outputs are written.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np

from . import _native as N

_NP_OF_TORCH = {"torch.int32": np.int32, "torch.uint32": np.uint32, "torch.int64": np.int64,
                "torch.float32": np.float32, "torch.float64": np.float64, "torch.uint8": np.uint8}


def _is_torch(x) -> bool:
    return hasattr(x, "data_ptr") and hasattr(x, "is_cuda")


def _numel(x) -> int:
    return int(x.size) if isinstance(x, np.ndarray) else int(x.numel())


class HistogramEngine:
    """Device-resident BucketedHistograms for ``max_series`` series on one GPU."""

    def __init__(self, max_series: int, device: int = 0):
        self._lib = N.load()
        self._ctx = ctypes.c_void_p()
        rc = self._lib.l5dh_open(ctypes.byref(self._ctx), int(max_series), 1 << int(device))
        if rc != 0:
            raise N.L5dhError(rc, "l5dh_open", f"max_series={max_series} device={device}")
        self.max_series = int(max_series)
        self.device = int(device)
        self._stream = None  # external stream handle the context runs on (None: its own)
        self._events = []
        self.nranks, self.rank = 1, 0

    # -- lifecycle -----------------------------------------------------------
    def close(self):
        if self._ctx:
            self._lib.l5dh_close(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, where: str):
        if rc != 0:
            msg = self._lib.l5dh_last_error(self._ctx)
            raise N.L5dhError(rc, where, msg.decode() if msg else "")

    # -- buffer checks -------------------------------------------------------
    def _buf(self, x, dtypes: Sequence, name: str, min_numel: int = 0, writable: bool = False) -> Optional[int]:
        """Raw pointer of a C-contiguous numpy array or torch tensor after checking
        dtype, device and size (ctypes passes no type information)."""
        if x is None:
            return None
        if isinstance(x, np.ndarray):
            if not x.flags["C_CONTIGUOUS"]:
                raise ValueError(f"{name}: array must be C-contiguous")
            if writable and not x.flags["WRITEABLE"]:
                raise ValueError(f"{name}: array is read-only")
            dt = x.dtype.type
        elif _is_torch(x):
            if not x.is_contiguous():
                raise ValueError(f"{name}: tensor must be contiguous")
            if x.is_cuda:
                if x.device.index != self.device:
                    raise ValueError(f"{name}: tensor on cuda:{x.device.index}, engine on cuda:{self.device}")
                self._order_after_torch()
            dt = _NP_OF_TORCH.get(str(x.dtype))
        else:
            raise TypeError(f"{name}: unsupported buffer type {type(x)!r}")
        if dt not in tuple(np.dtype(d).type for d in dtypes):
            raise TypeError(f"{name}: dtype {getattr(x, 'dtype', None)} not in {[np.dtype(d).name for d in dtypes]}")
        if _numel(x) < min_numel:
            raise ValueError(f"{name}: {_numel(x)} elements, at least {min_numel} needed")
        return x.data_ptr() if _is_torch(x) else x.ctypes.data

    def _order_after_torch(self):
        """Order the context's next work after everything queued on torch's current
        stream (an event handoff: no host synchronization)."""
        import torch
        cur = torch.cuda.current_stream(self.device)
        if self._stream is not None and int(self._stream) == cur.cuda_stream:
            return  # the context runs on that stream: already in order (a wait would only idle the GPU)
        ev = torch.cuda.Event()
        ev.record(cur)
        self._check(self._lib.l5dh_wait_event(self._ctx, ev.cuda_event), "l5dh_wait_event")
        self._events.append(ev)  # the handle must outlive the enqueued wait
        del self._events[:-4]

    def _range(self, first: int, count: Optional[int]):
        if count is None:
            count = self.max_series - first
        if first < 0 or count < 0 or first + count > self.max_series:
            raise ValueError(f"series range [{first}, {first + count}) outside [0, {self.max_series})")
        return first, count

    # -- hot path ---------------------------------------------------------------
    def ingest(self, series, values) -> None:
        """Batched Metric.Stat.add: values[i] into series[i] (u32 ids, f32 values)."""
        if isinstance(series, np.ndarray) and series.dtype != np.uint32:
            if series.size and (series.min() < 0 or series.max() >= 2 ** 32):
                raise ValueError("series ids must fit uint32")
            series = series.astype(np.uint32)
        if isinstance(values, np.ndarray) and values.dtype != np.float32:
            values = values.astype(np.float32)
        series = np.ascontiguousarray(series) if isinstance(series, np.ndarray) else series
        values = np.ascontiguousarray(values) if isinstance(values, np.ndarray) else values
        n = _numel(series)
        if n != _numel(values):
            raise ValueError("series and values differ in length")
        sp = self._buf(series, (np.uint32, np.int32), "series")
        vp = self._buf(values, (np.float32,), "values")
        self._check(self._lib.l5dh_ingest(self._ctx, sp, vp, n), "l5dh_ingest")

    def ingest_async(self, series, values) -> int:
        """l5dh_ingest_async: returns a ticket; the buffers must stay unchanged until
        ingest_wait(ticket) (host numpy buffers must stay referenced by the caller)."""
        for name, x, dts in (("series", series, (np.uint32, np.int32)), ("values", values, (np.float32,))):
            if isinstance(x, np.ndarray) and (x.dtype.type not in dts or not x.flags["C_CONTIGUOUS"]):
                raise TypeError(f"ingest_async: {name} must be C-contiguous {dts[0].__name__} (no conversion copy)")
        n = _numel(series)
        if n != _numel(values):
            raise ValueError("series and values differ in length")
        sp = self._buf(series, (np.uint32, np.int32), "series")
        vp = self._buf(values, (np.float32,), "values")
        t = ctypes.c_uint64(0)
        self._check(self._lib.l5dh_ingest_async(self._ctx, sp, vp, n, ctypes.byref(t)), "l5dh_ingest_async")
        return t.value

    def ingest_wait(self, ticket: int) -> None:
        self._check(self._lib.l5dh_ingest_wait(self._ctx, int(ticket)), "l5dh_ingest_wait")

    def snapshot(self, first: int = 0, count: Optional[int] = None, reset: bool = True,
                 with_counts: bool = False):
        """Summaries (numpy structured, HistogramSummary field order) and optional
        dense [count][1798] int32 bucket counts, for series [first, first+count)."""
        first, count = self._range(first, count)
        out = np.zeros(count, dtype=N.SUMMARY_DTYPE)
        counts = np.zeros((count, N.NBUCKETS), dtype=np.int32) if with_counts else None
        self._check(self._lib.l5dh_snapshot(self._ctx, first, count, out.ctypes.data,
                                            None if counts is None else counts.ctypes.data, int(reset)),
                    "l5dh_snapshot")
        return (out, counts) if with_counts else out

    def snapshot_into(self, summaries=None, counts=None, first: int = 0, count: Optional[int] = None,
                      reset: bool = True) -> None:
        """Snapshot into caller buffers (device tensors stay on the GPU).  summaries:
        int64 [count*11] (or the numpy summary dtype); counts: int32 [count][1798]."""
        first, count = self._range(first, count)
        sp = self._summ_buf(summaries, count, "summaries")
        cp = self._buf(counts, (np.int32,), "counts", count * N.NBUCKETS, writable=True)
        self._check(self._lib.l5dh_snapshot(self._ctx, first, count, sp, cp, int(reset)), "l5dh_snapshot")

    def _summ_buf(self, x, rows: int, name: str):
        if isinstance(x, np.ndarray) and x.dtype == N.SUMMARY_DTYPE:
            if x.size < rows or not x.flags["C_CONTIGUOUS"]:
                raise ValueError(f"{name}: needs {rows} contiguous summary records")
            return x.ctypes.data
        return self._buf(x, (np.int64,), name, rows * 11, writable=True)

    def peek(self, series: int) -> np.ndarray:
        """Metric.Stat.peek: non-empty buckets as (lower, upper, count)."""
        n = ctypes.c_size_t(0)
        self._check(self._lib.l5dh_peek(self._ctx, int(series), None, 0, ctypes.byref(n)), "l5dh_peek")
        out = np.zeros(n.value, dtype=N.BUCKET_COUNT_DTYPE)
        if n.value:
            self._check(self._lib.l5dh_peek(self._ctx, int(series), out.ctypes.data, n.value, ctypes.byref(n)),
                        "l5dh_peek")
        return out

    def export_state(self, first: int = 0, count: Optional[int] = None, reset: bool = False,
                     counts=None, totals=None):
        """Dense state for the fleet merge; fills caller buffers or returns numpy copies."""
        first, count = self._range(first, count)
        own = counts is None and totals is None
        if own:
            counts = np.zeros((count, N.NBUCKETS), dtype=np.int32)
            totals = np.zeros(count, dtype=np.int64)
        cp = self._buf(counts, (np.int32,), "counts", count * N.NBUCKETS, writable=True)
        tp = self._buf(totals, (np.int64,), "totals", count, writable=True)
        self._check(self._lib.l5dh_export_state(self._ctx, first, count, cp, tp, int(reset)), "l5dh_export_state")
        return (counts, totals) if own else None

    def summarize_dense(self, counts, totals, out=None):
        n = _numel(counts) // N.NBUCKETS
        if n * N.NBUCKETS != _numel(counts):
            raise ValueError("counts must hold whole rows of 1798 buckets")
        cp = self._buf(counts, (np.int32,), "counts")
        tp = self._buf(totals, (np.int64,), "totals", n)
        own = out is None
        if own:
            out = np.zeros(n, dtype=N.SUMMARY_DTYPE)
        op = self._summ_buf(out, n, "out")
        self._check(self._lib.l5dh_summarize_dense(self._ctx, cp, tp, n, op), "l5dh_summarize_dense")
        return out if own else None

    # -- fleet merge (RCCL) ------------------------------------------------------
    @staticmethod
    def comm_unique_id() -> bytes:
        lib = N.load()
        buf = ctypes.create_string_buffer(N.UNIQUE_ID_BYTES)
        rc = lib.l5dh_comm_unique_id(buf)
        if rc != 0:
            raise N.L5dhError(rc, "l5dh_comm_unique_id")
        return buf.raw

    def comm_init_rank(self, uid: bytes, nranks: int, rank: int) -> None:
        if len(uid) != N.UNIQUE_ID_BYTES:
            raise ValueError(f"unique id must be {N.UNIQUE_ID_BYTES} bytes")
        self._check(self._lib.l5dh_comm_init_rank(self._ctx, ctypes.create_string_buffer(uid, len(uid)),
                                                  int(nranks), int(rank)), "l5dh_comm_init_rank")
        self.nranks, self.rank = int(nranks), int(rank)

    @staticmethod
    def comm_init_all(engines: Sequence["HistogramEngine"]) -> None:
        arr = (ctypes.c_void_p * len(engines))(*[e._ctx.value for e in engines])
        rc = N.load().l5dh_comm_init_all(arr, len(engines))
        if rc != 0:
            engines[0]._check(rc, "l5dh_comm_init_all")
        for i, e in enumerate(engines):
            e.nranks, e.rank = len(engines), i

    @staticmethod
    def comm_init_loopback(engines: Sequence["HistogramEngine"]) -> None:
        """l5dh_comm_init_loopback: the engines (one device) as an n-rank group whose
        collectives are device copies -- the multi-rank merge path on one GPU (tests)."""
        arr = (ctypes.c_void_p * len(engines))(*[e._ctx.value for e in engines])
        rc = N.load().l5dh_comm_init_loopback(arr, len(engines))
        if rc != 0:
            engines[0]._check(rc, "l5dh_comm_init_loopback")
        for i, e in enumerate(engines):
            e.nranks, e.rank = len(engines), i

    @staticmethod
    def merge_all(engines: Sequence["HistogramEngine"], mode: int = N.MERGE_REDUCE_SCATTER, with_counts: bool = False):
        """l5dh_merge_all over an l5dh_comm_init_all / loopback group: per rank
        (first, count, summaries[, counts, totals]) as numpy."""
        n = len(engines)
        rows = engines[0].merge_rows(mode)
        outs = [np.zeros(rows, dtype=N.SUMMARY_DTYPE) for _ in engines]
        cnts = [np.zeros((rows, N.NBUCKETS), np.int32) for _ in engines] if with_counts else None
        tots = [np.zeros(rows, np.int64) for _ in engines] if with_counts else None
        ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p).value  # noqa: E731
        ctxs = (ctypes.c_void_p * n)(*[e._ctx.value for e in engines])
        o_arr = (ctypes.c_void_p * n)(*[ptr(o) for o in outs])
        c_arr = (ctypes.c_void_p * n)(*[ptr(c) for c in cnts]) if with_counts else None
        t_arr = (ctypes.c_void_p * n)(*[ptr(t) for t in tots]) if with_counts else None
        firsts, counts = (ctypes.c_uint32 * n)(), (ctypes.c_uint32 * n)()
        rc = N.load().l5dh_merge_all(ctxs, n, int(mode), o_arr, c_arr, t_arr, firsts, counts)
        if rc != 0:
            engines[0]._check(rc, "l5dh_merge_all")
        res = []
        for i in range(n):
            f, c = firsts[i], counts[i]
            item = (f, c, outs[i][:c])
            if with_counts:
                item += (cnts[i][:c], tots[i][:c])
            res.append(item)
        return res

    def comm_destroy(self) -> None:
        self._check(self._lib.l5dh_comm_destroy(self._ctx), "l5dh_comm_destroy")
        self.nranks, self.rank = 1, 0

    def merge_rows(self, mode: int = N.MERGE_REDUCE_SCATTER) -> int:
        """Rows each output of ``merge`` must hold."""
        per = -(-self.max_series // self.nranks)
        return per if mode == N.MERGE_REDUCE_SCATTER else self.max_series

    def merge(self, mode: int = N.MERGE_REDUCE_SCATTER, out=None, counts=None, totals=None):
        """Collective fleet merge (l5dh_merge): every rank's samples summed over RCCL,
        then this rank's rows summarized.  Returns (first, count[, summaries]) --
        summaries as numpy when ``out`` is None."""
        rows = self.merge_rows(mode)
        own = out is None
        if own:
            out = np.zeros(rows, dtype=N.SUMMARY_DTYPE)
        op = self._summ_buf(out, rows, "out")
        cp = self._buf(counts, (np.int32,), "counts", rows * N.NBUCKETS, writable=True)
        tp = self._buf(totals, (np.int64,), "totals", rows, writable=True)
        first, count = ctypes.c_uint32(0), ctypes.c_uint32(0)
        self._check(self._lib.l5dh_merge(self._ctx, int(mode), op, cp, tp, ctypes.byref(first), ctypes.byref(count)),
                    "l5dh_merge")
        return (first.value, count.value, out[:count.value]) if own else (first.value, count.value)

    def tile_totals(self) -> np.ndarray:
        """l5dh_tile_totals: records per 32-series tile of the last binned batch."""
        F = (self.max_series + 31) // 32
        out = np.zeros(F, np.uint64)
        self._check(self._lib.l5dh_tile_totals(self._ctx, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), F),
                    "l5dh_tile_totals")
        return out

    def partition_redos(self):
        """l5dh_partition_redos: (level-1 redos, level-2 redos, level-2 counting first
        passes) since open."""
        a, b, k = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        if not hasattr(self._lib, "l5dh_partition_redos"):  # (an older A/B build, L5DH_LIB)
            return 0, 0, 0
        self._check(self._lib.l5dh_partition_redos(self._ctx, ctypes.byref(a), ctypes.byref(b), ctypes.byref(k)),
                    "l5dh_partition_redos")
        return a.value, b.value, k.value

    def merge_bytes(self) -> dict:
        """l5dh_merge_bytes: dense / encoded / sent bytes of the last merge."""
        d, e, s = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
        self._check(self._lib.l5dh_merge_bytes(self._ctx, ctypes.byref(d), ctypes.byref(e), ctypes.byref(s)),
                    "l5dh_merge_bytes")
        return {"dense": d.value, "encoded": e.value, "sent": s.value}

    # -- plumbing -------------------------------------------------------------
    def sync(self):
        self._check(self._lib.l5dh_sync(self._ctx), "l5dh_sync")

    def set_stream(self, stream_handle: Optional[int]):
        """Run on an external hipStream_t handle (0: the legacy null stream, where
        torch's default stream work runs); None restores the context's own stream."""
        h = N.OWN_STREAM if stream_handle is None else int(stream_handle)
        self._check(self._lib.l5dh_set_stream(self._ctx, h), "l5dh_set_stream")
        self._stream = stream_handle

    def set_param(self, param: int, value: int):
        self._check(self._lib.l5dh_set_param(self._ctx, int(param), int(value)), "l5dh_set_param")

    def kernel_time(self, kernel_id: int, reset: bool = False):
        ms = ctypes.c_double(0)
        n = ctypes.c_int64(0)
        self._check(self._lib.l5dh_kernel_time(self._ctx, kernel_id, ctypes.byref(ms), ctypes.byref(n),
                                               int(reset)), "l5dh_kernel_time")
        return ms.value, n.value

    def kernel_times(self, reset: bool = False) -> dict:
        return {name: self.kernel_time(k, reset) for k, name in enumerate(N.KERNEL_NAMES)}
