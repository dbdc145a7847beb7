"""HistogramEngine: Python face of the C-ABI (one context = one GPU shard).

Mirrors what a JVM caller does through JNI: batched Stat.add (``ingest``) and
the timer-driven snapshot+reset (``snapshot``) of
AdminMetricsExportTelemeter.snapshotHistograms
(reference: telemetry/admin-metrics-export/.../AdminMetricsExportTelemeter.scala:154-162).

Inputs may be numpy arrays (host) or torch tensors on the engine's GPU; outputs
go to numpy (host) or to caller-provided torch tensors (device).
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from . import _native as N


def _ptr(x) -> Optional[int]:
    """Raw data pointer of a numpy array or a torch tensor (no copies)."""
    if x is None:
        return None
    if isinstance(x, np.ndarray):
        if not x.flags["C_CONTIGUOUS"]:
            raise ValueError("array must be C-contiguous")
        return x.ctypes.data
    if hasattr(x, "data_ptr"):
        if not x.is_contiguous():
            raise ValueError("tensor must be contiguous")
        return x.data_ptr()
    raise TypeError(f"unsupported buffer type {type(x)!r}")


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

    # -- hot path ---------------------------------------------------------------
    def ingest(self, series, values) -> None:
        """Batched Metric.Stat.add: values[i] into series[i] (u32 ids, f32 values)."""
        if isinstance(series, np.ndarray):
            series = np.ascontiguousarray(series, dtype=np.uint32)
        if isinstance(values, np.ndarray):
            values = np.ascontiguousarray(values, dtype=np.float32)
        n = _numel(series)
        if n != _numel(values):
            raise ValueError("series and values differ in length")
        self._check(self._lib.l5dh_ingest(self._ctx, _ptr(series), _ptr(values), n), "l5dh_ingest")

    def snapshot(self, first: int = 0, count: Optional[int] = None, reset: bool = True,
                 with_counts: bool = False):
        """Summaries (numpy structured, HistogramSummary field order) and optional
        dense [count][1798] int32 bucket counts, for series [first, first+count)."""
        if count is None:
            count = self.max_series - first
        out = np.zeros(count, dtype=N.SUMMARY_DTYPE)
        counts = np.zeros((count, N.NBUCKETS), dtype=np.int32) if with_counts else None
        self._check(self._lib.l5dh_snapshot(self._ctx, first, count, _ptr(out), _ptr(counts), int(reset)),
                    "l5dh_snapshot")
        return (out, counts) if with_counts else out

    def snapshot_into(self, summaries=None, counts=None, first: int = 0, count: Optional[int] = None,
                      reset: bool = True) -> None:
        """Snapshot into caller buffers (device tensors stay on the GPU)."""
        if count is None:
            count = self.max_series - first
        self._check(self._lib.l5dh_snapshot(self._ctx, first, count, _ptr(summaries), _ptr(counts), int(reset)),
                    "l5dh_snapshot")

    def peek(self, series: int) -> np.ndarray:
        """Metric.Stat.peek: non-empty buckets as (lower, upper, count)."""
        n = ctypes.c_size_t(0)
        self._check(self._lib.l5dh_peek(self._ctx, int(series), None, 0, ctypes.byref(n)), "l5dh_peek")
        out = np.zeros(n.value, dtype=N.BUCKET_COUNT_DTYPE)
        if n.value:
            self._check(self._lib.l5dh_peek(self._ctx, int(series), _ptr(out), n.value, ctypes.byref(n)),
                        "l5dh_peek")
        return out

    def export_state(self, first: int = 0, count: Optional[int] = None, reset: bool = False,
                     counts=None, totals=None):
        """Dense state for the fleet merge; fills caller buffers or returns numpy copies."""
        if count is None:
            count = self.max_series - first
        own = counts is None and totals is None
        if own:
            counts = np.zeros((count, N.NBUCKETS), dtype=np.int32)
            totals = np.zeros(count, dtype=np.int64)
        self._check(self._lib.l5dh_export_state(self._ctx, first, count, _ptr(counts), _ptr(totals), int(reset)),
                    "l5dh_export_state")
        return (counts, totals) if own else None

    def summarize_dense(self, counts, totals, out=None):
        n = _numel(counts) // N.NBUCKETS
        own = out is None
        if own:
            out = np.zeros(n, dtype=N.SUMMARY_DTYPE)
        self._check(self._lib.l5dh_summarize_dense(self._ctx, _ptr(counts), _ptr(totals), n, _ptr(out)),
                    "l5dh_summarize_dense")
        return out if own else None

    # -- plumbing -------------------------------------------------------------
    def sync(self):
        self._check(self._lib.l5dh_sync(self._ctx), "l5dh_sync")

    def set_stream(self, stream_handle: Optional[int]):
        self._check(self._lib.l5dh_set_stream(self._ctx, stream_handle), "l5dh_set_stream")

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
