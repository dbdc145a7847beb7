/*
 * l5dhist.h -- C-ABI of the MI355X latency-histogram engine (drop-in boundary).
 *
 * The boundary replaces the per-Stat arithmetic behind
 * io.buoyant.telemetry.Metric.Stat (reference: telemetry/core/src/main/scala/
 * io/buoyant/telemetry/Metric.scala:22-70) with a batched, device-resident
 * engine.  A JNI shim binds these symbols one-to-one; the
 * Scala side keeps Metric.Stat / HistogramSummary unchanged so exporters
 * (Prometheus, InfluxDB, admin metrics.json) consume the summaries as-is.
 *
 * Conventions
 *  - Plain pointers and sizes only.  Any data pointer may be host memory
 *    (pageable or from l5dh_pin_alloc) or device memory (hipMalloc on the
 *    context's device); the library detects which.
 *  - Status codes: 0 = OK, negative errno otherwise (-EINVAL, -ENOMEM, -EIO,
 *    -ENODEV).  The HIP/RCCL error text of the last failure is kept in
 *    l5dh_last_error(ctx).  No C++ exception crosses the ABI.
 *  - Every entry point taking a context is thread-safe (one lock per context).
 *  - The library never retains a caller pointer after a call returns, except
 *    buffers from l5dh_pin_alloc, which it owns.
 *
 * Series ids are dense uint32 ids assigned when a Stat is created
 * (reference: MetricsTree.mkStat, MetricsTree.scala:85-93), 0 <= id < max_series.
 */
#ifndef L5DHIST_H
#define L5DHIST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define L5DH_ABI_VERSION 1
#define L5DH_NLIMITS 1797  /* BucketedHistogram.scala:42 (0.5% error => 1797 limits) */
#define L5DH_NBUCKETS 1798 /* counts = limits.length + 1 (upstream finagle-stats) */
#define L5DH_MAX_SERIES (1u << 20) /* per context (= per GPU); shard wider fleets */

typedef struct l5dh_ctx l5dh_ctx;

/* Metric.HistogramSummary (Metric.scala:76-88): same fields, same order, 88 B. */
typedef struct {
  int64_t count;
  int64_t min;
  int64_t max;
  int64_t sum;
  int64_t p50;
  int64_t p90;
  int64_t p95;
  int64_t p99;
  int64_t p9990;
  int64_t p9999;
  double avg;
} l5dh_summary;

/* finagle-core BucketAndCount(lowerLimit, upperLimit, count) */
typedef struct {
  int32_t lower;
  int32_t upper;
  int32_t count;
} l5dh_bucket_count;

/* Tunables for l5dh_set_param */
enum {
  L5DH_PARAM_TIMING = 1,      /* 1: record HIP events around every kernel launch */
  L5DH_PARAM_COLD_LIMIT = 2,  /* max records for the single-pass tile path (<= 65535) */
  L5DH_PARAM_HOT_CHUNK = 3,   /* records per work item on the split (hot-tile) path */
  L5DH_PARAM_MAX_SEGMENTS = 4, /* binned ingest batches kept before folding (1..8) */
  L5DH_PARAM_BIN_MODE = 5,     /* 0 auto, 1 single-level scatter, 2 two-level partition */
  L5DH_PARAM_DIRECT_MAX = 6,   /* tiles whose final records k_bin1 writes directly (0..255) */
  L5DH_PARAM_DIRECT_DIV = 7,   /* direct tiles average >= 1/div records per 8K-sample sub-chunk */
  L5DH_PARAM_SPLIT_MIN = 8     /* tiles laid out per half-tile have >= this many records per batch */
};

/* Kernel ids for l5dh_kernel_time */
enum {
  L5DH_K_COUNT = 0,  /* per-slab tile histogram of the batch */
  L5DH_K_SCAN = 1,   /* slab/tile offset scans and the snapshot plan */
  L5DH_K_BIN = 2,    /* level-1 partition by super-tile (or the single-level bin) */
  L5DH_K_ACCUM = 3,  /* LDS-private tile histograms + fused summary / dense flush */
  L5DH_K_HOT = 4,    /* split-tile init/finish and row summaries */
  L5DH_K_COPY = 5,   /* H2D/D2H staging copies */
  L5DH_K_BIN2 = 6,   /* level-2 partition (super-tile runs -> per-tile segments) */
  L5DH_K_NKERNELS = 7
};

/* Reference: BucketedHistogram() per Stat (MetricsTree.scala:88).  Opens a
 * context owning device state for max_series series on the single device
 * selected by device_mask (exactly one bit set; bit i = HIP device i). */
int l5dh_open(l5dh_ctx** out, uint32_t max_series, uint32_t device_mask);
int l5dh_close(l5dh_ctx* ctx);

/* Reference: BucketedHistogram.DefaultLimits (BucketedHistogram.scala:42-46).
 * Returns the 1797 limits (static storage); *n receives 1797. */
const int32_t* l5dh_limits(size_t* n);

/* Reference: Metric.Stat.add(Float) (Metric.scala:30-33), batched: adds
 * values[i] to series series[i] for i < n.  Integer-only effect, so order
 * independent.  Samples with out-of-range ids are dropped and the call
 * returns -EINVAL after ingesting the valid ones.  Returns once the batch is
 * binned on the device (no caller pointer is retained). */
int l5dh_ingest(l5dh_ctx* ctx, const uint32_t* series, const float* values, size_t n);

/* Reference: Metric.Stat.snapshot() + reset() per Stat as driven by
 * AdminMetricsExportTelemeter.snapshotHistograms (AdminMetricsExportTelemeter.scala:154-162),
 * batched over series [first, first+count).  out (nullable) receives one
 * l5dh_summary per series (Metric.scala:53-67); counts_out (nullable)
 * receives [count][1798] int32 bucket counts (what reset()/peek return, dense).
 * reset != 0 clears those series afterwards, atomically with the snapshot. */
int l5dh_snapshot(l5dh_ctx* ctx, uint32_t first, uint32_t count, l5dh_summary* out,
                  int32_t* counts_out, int reset);

/* Reference: Metric.Stat.peek (Metric.scala:35-37) -> Seq[BucketAndCount].
 * Writes up to cap non-empty buckets of one series; *n_out = number of
 * non-empty buckets (may exceed cap). */
int l5dh_peek(l5dh_ctx* ctx, uint32_t series, l5dh_bucket_count* out, size_t cap, size_t* n_out);

/* Dense export of current state for the fleet merge (sample-sharded config):
 * counts [count][1798] int32 and totals [count] int64 (nullable).  reset as
 * in l5dh_snapshot. */
int l5dh_export_state(l5dh_ctx* ctx, uint32_t first, uint32_t count, int32_t* counts,
                      int64_t* totals, int reset);

/* Summaries of externally held dense state (e.g. after an RCCL reduce-scatter
 * of exported counts): counts [n][1798] int32, totals [n] int64. */
int l5dh_summarize_dense(l5dh_ctx* ctx, const int32_t* counts, const int64_t* totals, size_t n,
                         l5dh_summary* out);

/* Wait for queued work; returns a deferred ingest error if any. */
int l5dh_sync(l5dh_ctx* ctx);
/* Use an external hipStream_t (e.g. torch's current stream); NULL restores the
 * context's own stream. */
int l5dh_set_stream(l5dh_ctx* ctx, void* hip_stream);
int l5dh_set_param(l5dh_ctx* ctx, int param, int64_t value);
/* Accumulated device time (ms) and launch count of one kernel id since the
 * last reset (requires L5DH_PARAM_TIMING=1). reset_after != 0 zeroes it. */
int l5dh_kernel_time(l5dh_ctx* ctx, int kernel_id, double* ms, int64_t* launches, int reset_after);
int l5dh_device(l5dh_ctx* ctx, int* hip_device);
uint32_t l5dh_max_series(l5dh_ctx* ctx);

/* Pinned host staging for the JNI side's per-thread DirectByteBuffers. */
int l5dh_pin_alloc(size_t bytes, void** out);
int l5dh_pin_free(void* p);

const char* l5dh_last_error(l5dh_ctx* ctx);
int l5dh_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif
