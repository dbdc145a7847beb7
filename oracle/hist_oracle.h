/*
 * hist_oracle.h -- CPU ORACLE (test infrastructure only).
 *
 * A plain-C restatement of the reference's latency-histogram path, used ONLY
 * as the checker by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg.  Nothing in the product path (linkerd_amd/, the C-ABI
 * library) links, loads or calls this code.
 *
 * What it restates (citations relative to the reference checkout):
 *   - makeLimitsFor / DefaultLimits:
 *       telemetry/core/src/main/scala/com/twitter/finagle/stats/buoyant/BucketedHistogram.scala:25-46
 *   - Metric.Stat.add / peek / snapshot / reset / summary and HistogramSummary:
 *       telemetry/core/src/main/scala/io/buoyant/telemetry/Metric.scala:22-88
 *   - finagle-stats 6.45.0 BucketedHistogram.{add, percentile, minimum,
 *     maximum, average, bucketAndCounts, clear}.  That class lives in the
 *     third-party jar com.twitter:finagle-stats_2.12:6.45.0 (pinned at
 *     project/Deps.scala:18-19), which is NOT vendored in the reference; its
 *     published algorithm is restated here as spelled out in SURVEY.md §8a.
 *
 * Parity pinning: the restatement is pinned against the reference's own
 * known-answer tests P1-P4 (PrometheusTelemeterTest.scala:41-86,
 * InfluxDbTelemeterTest.scala:89-172, AdminMetricsExportTelemeterTest.scala:47-141)
 * and the fixture invariants P5 (admin/.../js/spec/fixtures/metrics.js).
 * Behaviour outside those pins (negative/NaN/Inf inputs, the overflow bucket,
 * Math.round ties at large counts) is "restated from upstream finagle-stats
 * 6.45 semantics; unverified against a JVM" -- parity unpinned there.
 */
#ifndef L5D_HIST_ORACLE_H
#define L5D_HIST_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define L5DO_NLIMITS 1797
#define L5DO_NBUCKETS 1798

typedef struct {
  int64_t count, min, max, sum, p50, p90, p95, p99, p9990, p9999;
  double avg;
} l5do_summary; /* field order of Metric.HistogramSummary, Metric.scala:76-88 */

typedef struct {
  int32_t lower, upper, count;
} l5do_bucket_count; /* finagle-core BucketAndCount(lowerLimit, upperLimit, count) */

typedef struct {
  int32_t counts[L5DO_NBUCKETS];
  int64_t num;
  int64_t total;
} l5do_hist; /* finagle-stats BucketedHistogram state (counts Int[], num Long, total Long) */

/* BucketedHistogram.scala:25-40 with error=0.005; returns number of limits written (1797). */
int l5do_make_limits(double error, int32_t* out, int cap);
const int32_t* l5do_default_limits(void);

int64_t l5do_java_f2l(float f);          /* Java (long) float cast: NaN->0, saturating, truncating */
int64_t l5do_java_round(double x);       /* java.lang.Math.round(double), JDK 8 semantics */
int l5do_bucket_of(int64_t v);           /* index that BucketedHistogram.add(v) increments */
int64_t l5do_midpoint(int b);            /* value reported for bucket b */

void l5do_hist_clear(l5do_hist* h);
void l5do_hist_add(l5do_hist* h, int64_t v);
void l5do_stat_add(l5do_hist* h, float value); /* Metric.Stat.add(Float): add(value.toLong) */
int64_t l5do_percentile(const l5do_hist* h, double p);
int64_t l5do_minimum(const l5do_hist* h);
int64_t l5do_maximum(const l5do_hist* h);
double l5do_average(const l5do_hist* h);
void l5do_summary_of(const l5do_hist* h, l5do_summary* out);
/* summary from a dense int32 count row + running total (num = sum of counts, 64-bit) */
void l5do_summary_of_counts(const int32_t* counts, int64_t total, l5do_summary* out);
size_t l5do_bucket_and_counts(const l5do_hist* h, l5do_bucket_count* out);

/* ---- batch drivers (tests and the cpu_baseline leg of bench.py) ---- */
/* Ingest a COO batch into S histograms with `threads` workers.  Workers
 * partition the series space (series % threads) and each Stat.add takes that
 * series' mutex, mirroring Metric.scala:30 (underlying.synchronized). */
int l5do_ingest(l5do_hist* hists, size_t nseries, const uint32_t* series,
                const float* values, size_t n, int threads);
/* Snapshot every series single-threaded (the DefaultTimer thread,
 * AdminMetricsExportTelemeter.scala:154-162): summary then optional reset. */
void l5do_snapshot_all(l5do_hist* hists, size_t nseries, l5do_summary* out, int reset);
/* Summaries of n dense int32 count rows + int64 totals (l5do_summary_of_counts per
 * row), rows split over `threads` workers.  Returns 0, or -3 on allocation failure. */
int l5do_summarize_counts_n(const int32_t* counts, const int64_t* totals, size_t n, l5do_summary* out,
                            int threads);
/* Copy dense counts/totals out. */
void l5do_export(const l5do_hist* hists, size_t nseries, int32_t* counts, int64_t* totals);
size_t l5do_hist_size(void);

#ifdef __cplusplus
}
#endif
#endif
