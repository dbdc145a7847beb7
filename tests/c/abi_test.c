/*
 * abi_test.c -- a C caller of the C-ABI (include/l5dhist.h), linked against
 * linkerd_amd/lib/libl5dhist.so: the same sequence the JNI shim drives for the
 * Scala telemetry, without Python in between.
 *
 *   l5dh_abi_test --version                 prints the ABI version (no GPU needed)
 *   l5dh_abi_test <in.bin> <out.bin> <piece>
 *
 * in.bin: u64 S, u64 n, u32 series[n], f32 values[n].
 * Sequence: open -> limits -> pin_alloc staging -> ingest in `piece`-sample calls
 * (the staging buffer is refilled after every call) -> sync -> snapshot without
 * reset (summaries + dense counts) -> peek(series 0) -> merge (1-rank RCCL
 * communicator via comm_init_all, reduce-scatter) -> snapshot after the merge's
 * reset -> close.
 * out.bin: summaries[S] (88 B), counts[S][1798] (i32), u64 npeek, peek[npeek] (12 B),
 * merged summaries[S] (88 B), u64 merged first, u64 merged count, u64 count sum after.
 * tests/test_gpu_c_abi.py compares it with the oracle.
 */
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "l5dhist.h"

#define CHECK(expr)                                                                        \
  do {                                                                                     \
    int _r = (expr);                                                                       \
    if (_r != 0) {                                                                         \
      fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #expr, _r,             \
              ctx ? l5dh_last_error(ctx) : "");                                            \
      return 1;                                                                            \
    }                                                                                      \
  } while (0)

static int rd(FILE* f, void* p, size_t bytes) { return fread(p, 1, bytes, f) == bytes ? 0 : -EIO; }
static int wr(FILE* f, const void* p, size_t bytes) { return fwrite(p, 1, bytes, f) == bytes ? 0 : -EIO; }

int main(int argc, char** argv) {
  l5dh_ctx* ctx = NULL;
  if (argc == 2 && !strcmp(argv[1], "--version")) {
    printf("%d\n", l5dh_abi_version());
    return l5dh_abi_version() == L5DH_ABI_VERSION ? 0 : 1;
  }
  if (argc != 4) {
    fprintf(stderr, "usage: %s <in.bin> <out.bin> <piece> | --version\n", argv[0]);
    return 2;
  }
  const size_t piece = (size_t)strtoull(argv[3], NULL, 10);
  FILE* in = fopen(argv[1], "rb");
  if (!in) return 2;
  uint64_t S = 0, n = 0;
  CHECK(rd(in, &S, 8));
  CHECK(rd(in, &n, 8));
  uint32_t* series = malloc(n * 4 + 4);
  float* values = malloc(n * 4 + 4);
  CHECK(series && values ? 0 : -ENOMEM);
  CHECK(rd(in, series, n * 4));
  CHECK(rd(in, values, n * 4));
  fclose(in);

  size_t nl = 0;
  const int32_t* lim = l5dh_limits(&nl);
  CHECK(lim && nl == L5DH_NLIMITS && lim[112] == 113 && lim[113] == 115 ? 0 : -EIO);
  CHECK(l5dh_open(&ctx, (uint32_t)S, 1u));

  void *ps = NULL, *pv = NULL;
  CHECK(l5dh_pin_alloc(piece * 4, &ps));
  CHECK(l5dh_pin_alloc(piece * 4, &pv));
  for (uint64_t off = 0; off < n; off += piece) {
    const size_t m = n - off < piece ? (size_t)(n - off) : piece;
    memcpy(ps, series + off, m * 4);
    memcpy(pv, values + off, m * 4);
    CHECK(l5dh_ingest(ctx, ps, pv, m));
    memset(ps, 0xFF, m * 4); /* the call has copied the batch: reuse the buffer at once */
  }
  CHECK(l5dh_sync(ctx));

  l5dh_summary* summ = calloc(S, sizeof(l5dh_summary));
  int32_t* counts = calloc(S * L5DH_NBUCKETS, 4);
  l5dh_bucket_count* pk = calloc(L5DH_NBUCKETS, sizeof(l5dh_bucket_count));
  l5dh_summary* merged = calloc(S, sizeof(l5dh_summary));
  CHECK(summ && counts && pk && merged ? 0 : -ENOMEM);
  CHECK(l5dh_snapshot(ctx, 0, (uint32_t)S, summ, counts, 0));
  size_t npeek = 0;
  CHECK(l5dh_peek(ctx, 0, pk, L5DH_NBUCKETS, &npeek));

  l5dh_ctx* all[1] = {ctx};
  CHECK(l5dh_comm_init_all(all, 1));
  CHECK(l5dh_set_param(ctx, L5DH_PARAM_MERGE_RCCL_1RANK, 1)); /* run the RCCL reduce-scatter at one rank too */
  uint32_t first = 0, count = 0;
  CHECK(l5dh_merge(ctx, L5DH_MERGE_REDUCE_SCATTER, merged, NULL, NULL, &first, &count));
  l5dh_summary* after_summ = calloc(S, sizeof(l5dh_summary));
  CHECK(after_summ ? 0 : -ENOMEM);
  CHECK(l5dh_snapshot(ctx, 0, (uint32_t)S, after_summ, NULL, 0));  /* the merge exported with reset */
  uint64_t after = 0;
  for (uint64_t i = 0; i < S; ++i) after += (uint64_t)after_summ[i].count;

  FILE* out = fopen(argv[2], "wb");
  CHECK(out ? 0 : -EIO);
  CHECK(wr(out, summ, S * sizeof(l5dh_summary)));
  CHECK(wr(out, counts, S * L5DH_NBUCKETS * 4));
  const uint64_t np = npeek;
  CHECK(wr(out, &np, 8));
  CHECK(wr(out, pk, npeek * sizeof(l5dh_bucket_count)));
  CHECK(wr(out, merged, S * sizeof(l5dh_summary)));
  const uint64_t f64 = first, c64 = count;
  CHECK(wr(out, &f64, 8));
  CHECK(wr(out, &c64, 8));
  CHECK(wr(out, &after, 8));
  fclose(out);

  CHECK(l5dh_pin_free(ps));
  CHECK(l5dh_pin_free(pv));
  CHECK(l5dh_comm_destroy(ctx));
  CHECK(l5dh_close(ctx));
  ctx = NULL;
  free(series); free(values); free(summ); free(counts); free(pk); free(merged); free(after_summ);
  return 0;
}
