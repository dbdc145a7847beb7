"""linkerd_amd -- MI355X-native engine for linkerd's latency-histogram hot path.

Drop-in for the arithmetic behind io.buoyant.telemetry.Metric.Stat
(reference: telemetry/core/src/main/scala/io/buoyant/telemetry/Metric.scala):
Stat.add samples are bucketized against finagle BucketedHistogram's 1797 limits
and summarized into HistogramSummary on the GPU, through the C-ABI in
include/l5dhist.h (linkerd_amd/lib/libl5dhist.so).

Modules:
  _native    ctypes binding of the C-ABI (raises if the HIP library is absent)
  engine     HistogramEngine (one context = one GPU shard)
  telemetry  MetricsTree / Metric.{Counter,Stat,Gauge} / HistogramSummary mirror
  prometheus PrometheusTelemeter text export from GPU summaries
  fleet      multi-GPU series sharding and the RCCL fleet merge
  synth      synthetic workloads C1-C4 of BASELINE.md
"""
from ._native import NLIMITS, NBUCKETS, SUMMARY_DTYPE, SUMMARY_FIELDS, L5dhError, NativeLibraryMissing  # noqa: F401

__all__ = ["NLIMITS", "NBUCKETS", "SUMMARY_DTYPE", "SUMMARY_FIELDS", "L5dhError", "NativeLibraryMissing"]


def HistogramEngine(*args, **kwargs):  # noqa: N802 - factory keeps import of the HIP lib lazy
    from .engine import HistogramEngine as _E
    return _E(*args, **kwargs)
