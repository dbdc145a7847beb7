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

#define L5DH_ABI_VERSION 3 /* 3: count-free partition (no bin-mode / split-min tunables); id errors from l5dh_sync only */
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
  L5DH_PARAM_HOT_CHUNK = 3,   /* max records per work item on the big-tile path, 1024..2^20 (fewer when CUs would idle) */
  L5DH_PARAM_MAX_SEGMENTS = 4, /* binned ingest batches kept before folding (1..8) */
  L5DH_PARAM_DIRECT_MAX = 6,   /* tiles whose final records level 1 writes directly (0..255) */
  L5DH_PARAM_DIRECT_DIV = 7,   /* direct tiles hold >= 1/div records per 8K samples of the batch */
  L5DH_PARAM_STAGE_SAMPLES = 9, /* device staging ring for small batches, in samples (0: off) */
  L5DH_PARAM_MAX_SLABS = 10,   /* ingest slabs (workgroups of the level-1 kernel), 1..512 */
  L5DH_PARAM_MERGE_RCCL_1RANK = 11, /* 1: run the RCCL collective even in a 1-rank communicator (tests) */
  L5DH_PARAM_REGION_PCT = 13,  /* capacity of the partition's regions in percent of the prediction (1..1000,
                                  default 100); a region that overflows is redone with exact sizes, so values
                                  below 100 exercise that path (tests) and cost time, never results */
  L5DH_PARAM_VARIANT = 12      /* kernel variant bits for same-context A/B timing (0: the default kernels;
                                  every variant computes the same results; bit 0: one-tile folds in u16 bins;
                                  bit 1: DMA copies of pinned host batches; bit 2: every ingest batch's
                                  capacity plan made as for a first interval, from its sample alone;
                                  other bits are ignored) */
};

/* Fleet-merge modes for l5dh_merge */
enum {
  L5DH_MERGE_REDUCE_SCATTER = 0, /* rank r receives the summed rows of its series slice */
  L5DH_MERGE_ALL_REDUCE = 1      /* every rank receives all summed rows */
};
#define L5DH_UNIQUE_ID_BYTES 128 /* = NCCL_UNIQUE_ID_BYTES */

/* Kernel ids for l5dh_kernel_time */
enum {
  L5DH_K_COUNT = 0,  /* (unused: the partition has no counting pass) */
  L5DH_K_SCAN = 1,   /* the batch sample, the partition plans and the snapshot plan */
  L5DH_K_BIN = 2,    /* level-1 partition by super-tile and direct half-tile (+ its redo) */
  L5DH_K_ACCUM = 3,  /* LDS-private tile histograms + fused summary / dense flush */
  L5DH_K_HOT = 4,    /* big-tile init/finish and row summaries */
  L5DH_K_COPY = 5,   /* H2D/D2H staging copies */
  L5DH_K_BIN2 = 6,   /* level-2 partition (super-tile regions -> 16-bit per-key records, + its redo) */
  L5DH_K_MERGE = 7,  /* the RCCL collective of l5dh_merge */
  L5DH_K_NKERNELS = 8
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
 * independent.
 *
 * Small batches (n <= half the staging ring, L5DH_PARAM_STAGE_SAMPLES) are
 * appended to a device staging ring and binned together when it fills or at
 * the next snapshot / peek / export / merge / sync; larger batches are binned
 * at once.  The call does not wait for the binning kernels: host buffers may
 * be reused as soon as it returns (their copy has completed); device buffers
 * may be reused once it returns when the context runs on its own stream, and
 * in stream order when it runs on a caller stream (l5dh_set_stream).
 *
 * Returns 0 once the batch is accepted (queued), otherwise an error and nothing
 * of the batch was queued.  Samples with out-of-range ids are dropped; the kernels
 * detect them asynchronously and l5dh_sync reports -EINVAL for them (a
 * later ingest never carries an earlier batch's error: an error from l5dh_ingest
 * means this batch was not queued -- or, for a batch above 2^30 samples, only its
 * leading 2^30-sample pieces were); all valid samples are ingested. */
int l5dh_ingest(l5dh_ctx* ctx, const uint32_t* series, const float* values, size_t n);

/* The same without waiting for the copy of host buffers: *ticket identifies the
 * call, and the caller keeps the buffers unchanged until l5dh_ingest_wait(ctx,
 * ticket) returns (a JNI thread double-buffers its pinned staging this way, so
 * the PCIe copy of one buffer overlaps the filling of the other).  Tickets grow;
 * waiting for a ticket also completes every earlier one.  Device buffers follow
 * l5dh_ingest's rules, with the ticket standing for "consumed". */
int l5dh_ingest_async(l5dh_ctx* ctx, const uint32_t* series, const float* values, size_t n, uint64_t* ticket);
int l5dh_ingest_wait(l5dh_ctx* ctx, uint64_t ticket);

/* Reference: Metric.Stat.snapshot() + reset() per Stat as driven by
 * AdminMetricsExportTelemeter.snapshotHistograms (AdminMetricsExportTelemeter.scala:154-162),
 * batched over series [first, first+count).  out (nullable) receives one
 * l5dh_summary per series (Metric.scala:53-67); counts_out (nullable)
 * receives [count][1798] int32 bucket counts (what reset()/peek return, dense).
 * reset != 0 clears those series afterwards, atomically with the snapshot.
 * The call returns once the outputs are written, except when every output given
 * is device memory and the context runs on a caller stream (l5dh_set_stream):
 * then the outputs are stream ordered on that stream (no host wait). */
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

/* Fleet merge over RCCL (xGMI): sample-sharded series (config C4) summed across
 * contexts on different GPUs.  One communicator per context, one rank per GPU:
 *  - multi-process (or one thread per context): rank 0 calls l5dh_comm_unique_id,
 *    the caller distributes the L5DH_UNIQUE_ID_BYTES bytes, every rank calls
 *    l5dh_comm_init_rank (collective: all ranks must call it);
 *  - one process holding several GPUs (e.g. a JVM): l5dh_comm_init_all over its
 *    contexts (distinct devices; rank i = ctxs[i]).
 * Every context of a communicator has the same max_series. */
int l5dh_comm_unique_id(void* id_out /* L5DH_UNIQUE_ID_BYTES */);
int l5dh_comm_init_rank(l5dh_ctx* ctx, const void* id, int nranks, int rank);
int l5dh_comm_init_all(l5dh_ctx** ctxs, int n);
/* Test transport: n contexts on ONE device form an n-rank group whose collectives are
 * device copies and reductions among their buffers (no RCCL), so the multi-rank merge
 * code -- per-destination slices, the size all-gather, the payload exchange, the
 * in-place local slice, the decode -- runs on a single GPU.  Such a group merges
 * through l5dh_merge_all only.  At most 64 ranks for every communicator kind
 * (the sparse reduce-scatter's sources): larger groups are rejected here, before
 * any merge consumes an interval. */
int l5dh_comm_init_loopback(l5dh_ctx** ctxs, int n);
int l5dh_comm_destroy(l5dh_ctx* ctx);

/* Reference: the snapshot of a series whose samples arrived on several hosts
 * must see their merged counts (AdminMetricsExportTelemeter.scala:154-162,
 * Metric.scala:39-67).  Collective (every rank of the communicator calls it):
 * each rank's pending samples and state are exported (whole range, reset), the
 * int32 counts [S][1798] and int64 totals [S] are summed with one RCCL
 * reduce-scatter (or all-reduce), and the rank summarizes the rows it received:
 * series [*first, *first + *count) (reduce-scatter: slice r of ceil(S/nranks)
 * rows; all-reduce: all S).  The reduce-scatter moves the rows sparse: each rank
 * sends each other rank the non-empty buckets of that rank's slice (one u32 per
 * bucket: bucket << 21 | count; larger counts take a second word) and the words per
 * row, and the totals go by one int64 reduce-scatter (l5dh_merge_bytes); the
 * all-reduce moves them dense.  out (nullable) receives *count l5dh_summary,
 * counts_out / totals_out (nullable) the summed rows.  Each output must hold
 * ceil(S/nranks) rows (reduce-scatter) or S rows (all-reduce).  Integer sums:
 * bit-exact and independent of the reduction order.  The export consumes the
 * rank's interval (as a resetting snapshot does) before the collective runs: if
 * the collective then fails (-EIO, l5dh_last_error), that interval is lost -- the
 * same outcome as a snapshot whose outputs are discarded. */
int l5dh_merge(l5dh_ctx* ctx, int mode, l5dh_summary* out, int32_t* counts_out, int64_t* totals_out,
               uint32_t* first, uint32_t* count);
/* The same for all contexts of an l5dh_comm_init_all communicator, from one
 * thread (the collectives are grouped).  Arrays are indexed like ctxs; any of
 * the output arrays (or their entries) may be NULL. */
int l5dh_merge_all(l5dh_ctx** ctxs, int n, int mode, l5dh_summary** outs, int32_t** counts_outs,
                   int64_t** totals_outs, uint32_t* firsts, uint32_t* counts);

/* Records per 32-series tile of the last binned ingest batch (out: >= ceil(max_series
 * / 32) entries; staged samples are binned first).  The load a series-sharded fleet
 * plans its next ranges from (linkerd_amd/fleet.py plan_shards). */
int l5dh_tile_totals(l5dh_ctx* ctx, uint64_t* out, size_t n);

/* Partition passes redone since l5dh_open because a capacity-planned region overflowed
 * (any pointer nullable): *level1 / *level2 = redos of the level-1 / level-2 partition
 * (each costs about one more pass of that level; results are exact either way).
 * *level2_counted = batches whose level-2 regions were known not to fit after level 1
 * (a moved load, a first interval): their first level-2 pass only counted the keys
 * (about 0.4 of a pass) and the second wrote exact regions -- not counted as redos. */
int l5dh_partition_redos(l5dh_ctx* ctx, uint64_t* level1, uint64_t* level2, uint64_t* level2_counted);

/* Bytes of the last l5dh_merge / l5dh_merge_all on this context (any pointer nullable):
 * *dense = the dense rows + totals a reduce-scatter would move ([S][1798] int32 +
 * [S] int64), *encoded = this rank's sparse encoding of them (non-empty buckets,
 * words per row, totals), *sent = what it sent to the other ranks. */
int l5dh_merge_bytes(l5dh_ctx* ctx, uint64_t* dense, uint64_t* encoded, uint64_t* sent);

/* Bin staged samples, wait for queued work; returns -EINVAL (once) if the device
 * found invalid series ids in any batch ingested since the last such report. */
int l5dh_sync(l5dh_ctx* ctx);
/* Run the context's work on an external hipStream_t, e.g. the caller's current
 * stream (torch's), so the context's kernels are ordered with the caller's work
 * on it; NULL selects the device's legacy default (null) stream.
 * L5DH_OWN_STREAM restores the context's own stream (the default). */
#define L5DH_OWN_STREAM ((void*)(intptr_t)-1)
int l5dh_set_stream(l5dh_ctx* ctx, void* hip_stream);
/* Order the context's next work after a caller's hipEvent_t (recorded on whatever
 * stream produced the device inputs, e.g. a torch.cuda.Event): the context's
 * stream waits for it on the device, the host does not. */
int l5dh_wait_event(l5dh_ctx* ctx, void* hip_event);
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
