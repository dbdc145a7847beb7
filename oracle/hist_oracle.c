/*
 * hist_oracle.c -- CPU ORACLE (test infrastructure only; see hist_oracle.h).
 *
 * Plain C restatement of the reference's histogram path.  Every function cites
 * the reference line it follows.  Compiled with -ffp-contract=off so the FP64
 * arithmetic is the JVM's (strictfp-equivalent on x86-64 SSE2).
 */
#include "hist_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define INT32_MAXV 2147483647

/* BucketedHistogram.scala:25-40 (makeLimitsFor):
 *   build(maxValue=Int.MaxValue.toDouble, factor=1.0+(error*2), n=1.0):
 *     next = n*factor; stop when next >= maxValue
 *   values = build(...).map(_.toInt + 1).distinct;  result = Seq(1) ++ values */
int l5do_make_limits(double error, int32_t* out, int cap) {
  if (!(error > 0.0 && error <= 1.0)) return -1; /* require(error > 0.0 && error <= 1.0) */
  const double maxValue = (double)INT32_MAXV;
  const double factor = 1.0 + (error * 2);
  int n = 0;
  if (n < cap) out[n] = 1;
  n++;
  int32_t last = 0x7fffffff; /* .distinct over the mapped stream */
  int have_last = 0;
  double cur = 1.0;
  for (;;) {
    double next = cur * factor;
    if (next >= maxValue) break;
    int32_t v = (int32_t)next + 1; /* _.toInt + 1: truncation, next < 2^31 here */
    if (!have_last || v != last) {
      /* distinct over a non-decreasing sequence == drop consecutive repeats;
       * the prepended 1 is not part of the stream, so 2.. follow it. */
      if (n < cap) out[n] = v;
      n++;
      last = v;
      have_last = 1;
    }
    cur = next;
  }
  return n;
}

static int32_t g_limits[L5DO_NLIMITS];
static int g_limits_ready = 0;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static void init_limits(void) {
  /* DefaultErrorPercent = 0.005 (BucketedHistogram.scala:42-46) */
  int n = l5do_make_limits(0.005, g_limits, L5DO_NLIMITS);
  g_limits_ready = (n == L5DO_NLIMITS);
}
const int32_t* l5do_default_limits(void) {
  pthread_once(&g_once, init_limits);
  return g_limits_ready ? g_limits : NULL;
}

/* Metric.scala:32 `value.toLong` -- JLS 5.1.3 narrowing float->long:
 * NaN -> 0; values beyond the long range saturate; otherwise round toward zero. */
int64_t l5do_java_f2l(float f) {
  if (isnan(f)) return 0;
  if (f >= 9223372036854775808.0f) return INT64_MAX;
  if (f <= -9223372036854775808.0f) return INT64_MIN;
  return (int64_t)f;
}

/* java.lang.Math.round(double) (JDK 7+): closest long, ties toward +inf,
 * computed exactly (no floor(x+0.5) double-rounding). */
int64_t l5do_java_round(double x) {
  if (isnan(x)) return 0;
  if (x >= 9223372036854775807.0) return INT64_MAX;
  if (x <= -9223372036854775808.0) return INT64_MIN;
  double fl = floor(x);
  if (fabs(x) >= 4503599627370496.0) return (int64_t)x; /* already integral */
  double fr = x - fl;                                     /* exact for |x| < 2^52 */
  return (int64_t)fl + (fr >= 0.5 ? 1 : 0);
}

/* upstream BucketedHistogram.add(Long): if v >= Int.MaxValue -> last (overflow)
 * bucket; else i = Arrays.binarySearch(limits, v.toInt); idx = i>=0 ? i+1 : -i-1.
 * Both branches equal "number of limits <= key" (upper bound), restated here with
 * Java's binary search written out. */
int l5do_bucket_of(int64_t v) {
  const int32_t* L = l5do_default_limits();
  if (v >= INT32_MAXV) return L5DO_NLIMITS;
  int32_t key = (int32_t)(uint32_t)(uint64_t)v; /* Long.toInt: low 32 bits */
  /* java.util.Arrays.binarySearch0(int[], 0, len, key) */
  int low = 0, high = L5DO_NLIMITS - 1;
  while (low <= high) {
    int mid = (int)((unsigned)(low + high) >> 1);
    int32_t midVal = L[mid];
    if (midVal < key)
      low = mid + 1;
    else if (midVal > key)
      high = mid - 1;
    else
      return mid + 1; /* found: i >= 0 -> i + 1 */
  }
  return low; /* not found: -(low+1) -> -i-1 == low (insertion point) */
}

/* upstream midpoint of bucket b: 0 for b==0, Int.MaxValue for the overflow
 * bucket, else (limits(b-1) + limits(b)) / 2 in 64-bit (pinned by P5:
 * 3030 -> (3011+3042)/2 = 3026, metrics.js:2782-2794). */
int64_t l5do_midpoint(int b) {
  const int32_t* L = l5do_default_limits();
  if (b <= 0) return 0;
  if (b >= L5DO_NLIMITS) return INT32_MAXV;
  return ((int64_t)L[b - 1] + (int64_t)L[b]) / 2;
}

/* upstream clear(): Arrays.fill(counts, 0); num = 0; total = 0 */
void l5do_hist_clear(l5do_hist* h) { memset(h, 0, sizeof(*h)); }

/* upstream add(Long) */
void l5do_hist_add(l5do_hist* h, int64_t v) {
  int b;
  if (v >= INT32_MAXV) {
    h->total = (int64_t)((uint64_t)h->total + (uint64_t)INT32_MAXV);
    b = L5DO_NLIMITS;
  } else {
    h->total = (int64_t)((uint64_t)h->total + (uint64_t)v); /* Java long wraps */
    b = l5do_bucket_of(v);
  }
  h->counts[b] = (int32_t)((uint32_t)h->counts[b] + 1u); /* Java int wraps */
  h->num += 1;
}

/* Metric.scala:30-33: underlying.add(value.toLong) */
void l5do_stat_add(l5do_hist* h, float value) { l5do_hist_add(h, l5do_java_f2l(value)); }

/* upstream percentile(p): target = Math.round(p * num); walk the counts until the
 * running total reaches target; report the midpoint of that bucket; 0 when the
 * walk never starts (target == 0). */
int64_t l5do_percentile(const l5do_hist* h, double p) {
  int64_t target = l5do_java_round(p * (double)h->num);
  int64_t total = 0;
  int i = 0;
  while (i < L5DO_NBUCKETS && total < target) {
    total += h->counts[i];
    i++;
  }
  if (i == 0) return 0;
  if (i == L5DO_NBUCKETS) return INT32_MAXV;
  return l5do_midpoint(i - 1);
}

/* upstream minimum: midpoint of the first non-empty bucket (P5 pins midpoints) */
int64_t l5do_minimum(const l5do_hist* h) {
  if (h->num == 0) return 0;
  for (int i = 0; i < L5DO_NBUCKETS; i++)
    if (h->counts[i] > 0) return l5do_midpoint(i);
  return 0;
}

/* upstream maximum: Int.MaxValue if the overflow bucket is used, else midpoint
 * of the last non-empty bucket */
int64_t l5do_maximum(const l5do_hist* h) {
  if (h->num == 0) return 0;
  if (h->counts[L5DO_NBUCKETS - 1] > 0) return INT32_MAXV;
  for (int i = L5DO_NBUCKETS - 1; i >= 0; i--)
    if (h->counts[i] > 0) return l5do_midpoint(i);
  return 0;
}

/* upstream average: if (num == 0) 0.0 else total / num.toDouble */
double l5do_average(const l5do_hist* h) {
  if (h->num == 0) return 0.0;
  return (double)h->total / (double)h->num;
}

/* Metric.scala:53-67 (Stat.summary) */
void l5do_summary_of(const l5do_hist* h, l5do_summary* o) {
  o->count = h->num;
  o->min = l5do_minimum(h);
  o->max = l5do_maximum(h);
  o->sum = h->total;
  o->p50 = l5do_percentile(h, 0.50);
  o->p90 = l5do_percentile(h, 0.90);
  o->p95 = l5do_percentile(h, 0.95);
  o->p99 = l5do_percentile(h, 0.99);
  o->p9990 = l5do_percentile(h, 0.999);
  o->p9999 = l5do_percentile(h, 0.9999);
  o->avg = l5do_average(h);
}

void l5do_summary_of_counts(const int32_t* counts, int64_t total, l5do_summary* o) {
  l5do_hist h;
  memcpy(h.counts, counts, sizeof(h.counts));
  int64_t num = 0;
  for (int i = 0; i < L5DO_NBUCKETS; i++) num += (int64_t)(uint32_t)counts[i];
  h.num = num;
  h.total = total;
  l5do_summary_of(&h, o);
}

/* upstream bucketAndCounts: non-empty buckets as BucketAndCount(lower, upper, count),
 * lower = b==0 ? 0 : limits(b-1); upper = b < limits.length ? limits(b) : Int.MaxValue */
size_t l5do_bucket_and_counts(const l5do_hist* h, l5do_bucket_count* out) {
  const int32_t* L = l5do_default_limits();
  size_t n = 0;
  for (int b = 0; b < L5DO_NBUCKETS; b++) {
    if (h->counts[b] > 0) {
      if (out) {
        out[n].lower = b == 0 ? 0 : L[b - 1];
        out[n].upper = b < L5DO_NLIMITS ? L[b] : INT32_MAXV;
        out[n].count = h->counts[b];
      }
      n++;
    }
  }
  return n;
}

size_t l5do_hist_size(void) { return sizeof(l5do_hist); }

/* ---------------- batch drivers ---------------- */

typedef struct {
  l5do_hist* hists;
  pthread_mutex_t* locks;
  size_t nseries;
  const uint32_t* series;
  const float* values;
  size_t lo, hi;
  int bad;
} ingest_job;

static void* ingest_worker(void* arg) {
  ingest_job* j = (ingest_job*)arg;
  for (size_t i = j->lo; i < j->hi; i++) {
    uint32_t s = j->series[i];
    if (s >= j->nseries) {
      j->bad = 1;
      continue;
    }
    /* Metric.scala:30: underlying.synchronized { underlying.add(value.toLong) } */
    pthread_mutex_lock(&j->locks[s]);
    l5do_stat_add(&j->hists[s], j->values[i]);
    pthread_mutex_unlock(&j->locks[s]);
  }
  return NULL;
}

int l5do_ingest(l5do_hist* hists, size_t nseries, const uint32_t* series,
                const float* values, size_t n, int threads) {
  if (l5do_default_limits() == NULL) return -1;
  if (threads < 1) threads = 1;
  if (threads == 1) {
    int bad = 0;
    for (size_t i = 0; i < n; i++) {
      uint32_t s = series[i];
      if (s >= nseries) {
        bad = 1;
        continue;
      }
      l5do_stat_add(&hists[s], values[i]);
    }
    return bad ? -2 : 0;
  }
  pthread_mutex_t* locks = (pthread_mutex_t*)malloc(sizeof(pthread_mutex_t) * nseries);
  if (!locks) return -3;
  for (size_t s = 0; s < nseries; s++) pthread_mutex_init(&locks[s], NULL);
  pthread_t* tids = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  ingest_job* jobs = (ingest_job*)malloc(sizeof(ingest_job) * threads);
  size_t per = (n + threads - 1) / threads;
  for (int t = 0; t < threads; t++) {
    jobs[t].hists = hists;
    jobs[t].locks = locks;
    jobs[t].nseries = nseries;
    jobs[t].series = series;
    jobs[t].values = values;
    jobs[t].lo = (size_t)t * per < n ? (size_t)t * per : n;
    jobs[t].hi = jobs[t].lo + per < n ? jobs[t].lo + per : n;
    jobs[t].bad = 0;
    pthread_create(&tids[t], NULL, ingest_worker, &jobs[t]);
  }
  int bad = 0;
  for (int t = 0; t < threads; t++) {
    pthread_join(tids[t], NULL);
    bad |= jobs[t].bad;
  }
  for (size_t s = 0; s < nseries; s++) pthread_mutex_destroy(&locks[s]);
  free(locks);
  free(tids);
  free(jobs);
  return bad ? -2 : 0;
}

typedef struct {
  const int32_t* counts;
  const int64_t* totals;
  l5do_summary* out;
  size_t lo, hi;
} summary_job;

static void* summary_worker(void* arg) {
  summary_job* j = (summary_job*)arg;
  for (size_t s = j->lo; s < j->hi; s++)
    l5do_summary_of_counts(j->counts + s * L5DO_NBUCKETS, j->totals[s], &j->out[s]);
  return NULL;
}

/* Metric.scala:53-67 for n dense rows (each row independent: split over `threads`). */
int l5do_summarize_counts_n(const int32_t* counts, const int64_t* totals, size_t n, l5do_summary* out,
                            int threads) {
  if (threads < 1) threads = 1;
  if ((size_t)threads > n) threads = n ? (int)n : 1;
  pthread_t* tids = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  summary_job* jobs = (summary_job*)malloc(sizeof(summary_job) * threads);
  if (!tids || !jobs) {
    free(tids);
    free(jobs);
    return -3;
  }
  size_t per = (n + threads - 1) / threads;
  for (int t = 0; t < threads; t++) {
    jobs[t].counts = counts;
    jobs[t].totals = totals;
    jobs[t].out = out;
    jobs[t].lo = (size_t)t * per < n ? (size_t)t * per : n;
    jobs[t].hi = jobs[t].lo + per < n ? jobs[t].lo + per : n;
    pthread_create(&tids[t], NULL, summary_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; t++) pthread_join(tids[t], NULL);
  free(tids);
  free(jobs);
  return 0;
}

/* AdminMetricsExportTelemeter.scala:154-162: for each Stat, snapshot() then reset() */
void l5do_snapshot_all(l5do_hist* hists, size_t nseries, l5do_summary* out, int reset) {
  for (size_t s = 0; s < nseries; s++) {
    l5do_summary_of(&hists[s], &out[s]);
    if (reset) l5do_hist_clear(&hists[s]);
  }
}

void l5do_export(const l5do_hist* hists, size_t nseries, int32_t* counts, int64_t* totals) {
  for (size_t s = 0; s < nseries; s++) {
    if (counts) memcpy(counts + s * L5DO_NBUCKETS, hists[s].counts, sizeof(hists[s].counts));
    if (totals) totals[s] = hists[s].total;
  }
}
