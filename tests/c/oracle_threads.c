/*
 * oracle_threads.c -- sanitizer driver for the CPU oracle's multithreaded ingest
 * (oracle/hist_oracle.c l5do_ingest: worker threads + one mutex per series, the
 * restatement of Metric.Stat.add's per-Stat monitor, Metric.scala:30-33).
 * Built with -fsanitize=thread and with -fsanitize=address,undefined by
 * tests/test_sanitizers.py: 8 threads over a skewed batch (hot series contend on
 * their mutex) must give the single-thread counts, sums and summaries.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hist_oracle.h"

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint64_t next(void) {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return rng;
}

int main(void) {
  const size_t S = 300, n = 400000;
  uint32_t* series = malloc(n * 4);
  float* values = malloc(n * 4);
  for (size_t i = 0; i < n; ++i) {
    const uint64_t r = next();
    series[i] = (uint32_t)((r & 1) ? (r >> 1) % 4 : (r >> 1) % S); /* half the samples on 4 hot series */
    values[i] = (float)((next() >> 11) % 100000) * 0.37f;
  }
  series[7] = (uint32_t)S + 3; /* an invalid id: dropped and reported */
  l5do_hist* a = calloc(S, l5do_hist_size());
  l5do_hist* b = calloc(S, l5do_hist_size());
  const int ra = l5do_ingest(a, S, series, values, n, 1);
  const int rb = l5do_ingest(b, S, series, values, n, 8);
  if (ra != rb || ra == 0) {
    fprintf(stderr, "ingest status %d / %d\n", ra, rb);
    return 1;
  }
  if (memcmp(a, b, S * l5do_hist_size()) != 0) {
    fprintf(stderr, "8-thread state differs from 1-thread state\n");
    return 1;
  }
  l5do_summary* sa = calloc(S, sizeof(l5do_summary));
  l5do_summary* sb = calloc(S, sizeof(l5do_summary));
  l5do_snapshot_all(a, S, sa, 1);
  l5do_snapshot_all(b, S, sb, 1);
  if (memcmp(sa, sb, S * sizeof(l5do_summary)) != 0) return 1;
  free(series); free(values); free(a); free(b); free(sa); free(sb);
  puts("ok");
  return 0;
}
