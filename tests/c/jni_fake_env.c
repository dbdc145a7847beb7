/*
 * jni_fake_env.c -- executes every JNI entry point of jni/src/main/native/l5dh_jni.c
 * (io.buoyant.telemetry.gpu.Native) without a JVM: a fake JNIEnv function table
 * (tests/jni_stub/jni.h) whose jobjects are plain C structs -- direct byte buffers,
 * int / byte / long arrays, strings -- and the call sequence GpuEngine.scala makes.
 * Inputs and outputs are raw little-endian files in a directory; the GPU test
 * (tests/test_gpu_jni.py) compares the outputs with the CPU oracle.
 *
 *   jni_fake_env <dir> <max_series> <n> <piece>
 * reads  <dir>/series.bin (n u32), <dir>/values.bin (n f32)
 * writes <dir>/limits.bin, summ.bin, counts.bin (the reset snapshot), summ2.bin (the
 * snapshot after it), peek.bin (12-B BucketAndCount of series 0..3, cap 2048 each,
 * with a u32 count before each), merge_rs_*.bin, merge_ar_*.bin, log.txt
 */
#define _POSIX_C_SOURCE 200809L
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "jni.h"
#include "l5dhist.h"

/* ---- fake objects ---- */
enum { K_DIRECT = 1, K_INTARR, K_BYTEARR, K_LONGARR, K_STRING };
typedef struct _jobject {
  int kind;
  void* addr;   /* direct buffer address / array elements / string bytes */
  jlong cap;    /* direct buffer capacity (bytes) */
  jsize len;    /* array length */
} FakeObj;

static int g_calls[16];  /* per-JNIEnv-function call counts (all must be exercised) */

static FakeObj* mkobj(int kind, void* addr, jlong cap, jsize len) {
  FakeObj* o = (FakeObj*)calloc(1, sizeof(FakeObj));
  o->kind = kind;
  o->addr = addr;
  o->cap = cap;
  o->len = len;
  return o;
}

static void* fk_GetDirectBufferAddress(JNIEnv* e, jobject o) {
  (void)e;
  g_calls[0]++;
  return o && o->kind == K_DIRECT ? o->addr : NULL;
}
static jobject fk_NewDirectByteBuffer(JNIEnv* e, void* p, jlong cap) {
  (void)e;
  g_calls[1]++;
  return mkobj(K_DIRECT, p, cap, 0);
}
static jintArray fk_NewIntArray(JNIEnv* e, jsize n) {
  (void)e;
  g_calls[2]++;
  return mkobj(K_INTARR, calloc((size_t)n + 1, 4), 0, n);
}
static void fk_SetIntArrayRegion(JNIEnv* e, jintArray a, jsize s, jsize n, const jint* v) {
  (void)e;
  g_calls[3]++;
  if (a->kind != K_INTARR || s < 0 || s + n > a->len) { fprintf(stderr, "SetIntArrayRegion out of bounds\n"); exit(3); }
  memcpy((jint*)a->addr + s, v, (size_t)n * 4);
}
static jbyteArray fk_NewByteArray(JNIEnv* e, jsize n) {
  (void)e;
  g_calls[4]++;
  return mkobj(K_BYTEARR, calloc((size_t)n + 1, 1), 0, n);
}
static void fk_SetByteArrayRegion(JNIEnv* e, jbyteArray a, jsize s, jsize n, const jbyte* v) {
  (void)e;
  g_calls[5]++;
  if (a->kind != K_BYTEARR || s < 0 || s + n > a->len) { fprintf(stderr, "SetByteArrayRegion out of bounds\n"); exit(3); }
  memcpy((jbyte*)a->addr + s, v, (size_t)n);
}
static void fk_GetByteArrayRegion(JNIEnv* e, jbyteArray a, jsize s, jsize n, jbyte* v) {
  (void)e;
  g_calls[6]++;
  if (a->kind != K_BYTEARR || s < 0 || s + n > a->len) { fprintf(stderr, "GetByteArrayRegion out of bounds\n"); exit(3); }
  memcpy(v, (jbyte*)a->addr + s, (size_t)n);
}
static void fk_GetLongArrayRegion(JNIEnv* e, jlongArray a, jsize s, jsize n, jlong* v) {
  (void)e;
  g_calls[7]++;
  if (a->kind != K_LONGARR || s < 0 || s + n > a->len) { fprintf(stderr, "GetLongArrayRegion out of bounds\n"); exit(3); }
  memcpy(v, (jlong*)a->addr + s, (size_t)n * 8);
}
static jsize fk_GetArrayLength(JNIEnv* e, jarray a) {
  (void)e;
  g_calls[8]++;
  return a->len;
}
static jstring fk_NewStringUTF(JNIEnv* e, const char* s) {
  (void)e;
  g_calls[9]++;
  char* c = strdup(s ? s : "");
  return mkobj(K_STRING, c, 0, (jsize)strlen(c));
}

static const struct JNINativeInterface_ g_table = {
    fk_GetDirectBufferAddress, fk_NewDirectByteBuffer, fk_NewIntArray,   fk_SetIntArrayRegion, fk_NewByteArray,
    fk_SetByteArrayRegion,     fk_GetByteArrayRegion,  fk_GetLongArrayRegion, fk_GetArrayLength, fk_NewStringUTF};

/* ---- the shim's entry points (l5dh_jni.c) ---- */
#define NATIVE(ret, name, ...) JNIEXPORT ret JNICALL Java_io_buoyant_telemetry_gpu_Native_##name(JNIEnv*, jclass, ##__VA_ARGS__)
NATIVE(jlong, open, jint, jint);
NATIVE(jint, close, jlong);
NATIVE(jintArray, limits);
NATIVE(jint, ingest, jlong, jobject, jobject, jint);
NATIVE(jlong, ingestAsync, jlong, jobject, jobject, jint);
NATIVE(jint, ingestWait, jlong, jlong);
NATIVE(jint, snapshot, jlong, jint, jint, jobject, jobject, jboolean);
NATIVE(jlong, peek, jlong, jint, jobject, jint);
NATIVE(jint, sync, jlong);
NATIVE(jint, setParam, jlong, jint, jlong);
NATIVE(jobject, pinAlloc, jlong);
NATIVE(jint, pinFree, jobject);
NATIVE(jbyteArray, commUniqueId);
NATIVE(jint, commInitRank, jlong, jbyteArray, jint, jint);
NATIVE(jint, commInitAll, jlongArray);
NATIVE(jint, merge, jlong, jint, jobject, jobject, jobject, jintArray);
NATIVE(jstring, lastError, jlong);

static JNIEnv g_env = &g_table;
static JNIEnv* env = &g_env;
static FILE* g_log;

#define CHECK(cond, ...)                        \
  do {                                          \
    if (!(cond)) {                              \
      fprintf(stderr, "FAILED %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);             \
      fprintf(stderr, "\n");                    \
      exit(1);                                  \
    }                                           \
  } while (0)

static void* read_file(const char* dir, const char* name, size_t bytes) {
  char p[4096];
  snprintf(p, sizeof p, "%s/%s", dir, name);
  FILE* f = fopen(p, "rb");
  CHECK(f, "open %s", p);
  void* b = malloc(bytes ? bytes : 1);
  CHECK(fread(b, 1, bytes, f) == bytes, "short read %s", p);
  fclose(f);
  return b;
}

static void write_file(const char* dir, const char* name, const void* b, size_t bytes) {
  char p[4096];
  snprintf(p, sizeof p, "%s/%s", dir, name);
  FILE* f = fopen(p, "wb");
  CHECK(f, "create %s", p);
  CHECK(fwrite(b, 1, bytes, f) == bytes, "short write %s", p);
  fclose(f);
}

static jobject direct(size_t bytes) {  /* ByteBuffer.allocateDirect */
  return mkobj(K_DIRECT, calloc(bytes ? bytes : 1, 1), (jlong)bytes, 0);
}

/* GpuEngine.Staging: two pinned pairs, double-buffered through ingestAsync/ingestWait */
static void ingest_async_pieces(jlong h, const uint32_t* s, const float* v, size_t n, size_t piece, jobject ids[2],
                                jobject vals[2]) {
  jlong ticket[2] = {0, 0};
  int cur = 0;
  for (size_t o = 0; o < n; o += piece) {
    const size_t m = n - o < piece ? n - o : piece;
    if (ticket[cur]) {
      CHECK(Java_io_buoyant_telemetry_gpu_Native_ingestWait(env, NULL, h, ticket[cur]) == 0, "ingestWait");
      ticket[cur] = 0;
    }
    memcpy(ids[cur]->addr, s + o, m * 4);
    memcpy(vals[cur]->addr, v + o, m * 4);
    const jlong t = Java_io_buoyant_telemetry_gpu_Native_ingestAsync(env, NULL, h, ids[cur], vals[cur], (jint)m);
    CHECK(t > 0, "ingestAsync returned %lld", (long long)t);
    ticket[cur] = t;
    cur ^= 1;
  }
  for (int k = 0; k < 2; ++k)
    if (ticket[k]) CHECK(Java_io_buoyant_telemetry_gpu_Native_ingestWait(env, NULL, h, ticket[k]) == 0, "ingestWait");
}

int main(int argc, char** argv) {
  if (argc != 5) {
    fprintf(stderr, "usage: %s <dir> <max_series> <n> <piece>\n", argv[0]);
    return 2;
  }
  const char* dir = argv[1];
  const int S = atoi(argv[2]);
  const size_t n = (size_t)atoll(argv[3]);
  const size_t piece = (size_t)atoll(argv[4]);
  char lp[4096];
  snprintf(lp, sizeof lp, "%s/log.txt", dir);
  g_log = fopen(lp, "w");
  uint32_t* series = (uint32_t*)read_file(dir, "series.bin", n * 4);
  float* values = (float*)read_file(dir, "values.bin", n * 4);

  /* open / limits / setParam */
  const jlong h = Java_io_buoyant_telemetry_gpu_Native_open(env, NULL, S, 0);
  CHECK(h > 0, "open returned %lld", (long long)h);
  jintArray lim = Java_io_buoyant_telemetry_gpu_Native_limits(env, NULL);
  CHECK(lim && lim->len == L5DH_NLIMITS, "limits");
  write_file(dir, "limits.bin", lim->addr, (size_t)lim->len * 4);
  CHECK(Java_io_buoyant_telemetry_gpu_Native_setParam(env, NULL, h, L5DH_PARAM_STAGE_SAMPLES, 1 << 20) == 0, "setParam");
  CHECK(Java_io_buoyant_telemetry_gpu_Native_setParam(env, NULL, h, 9999, 1) == -EINVAL, "setParam(unknown)");
  jstring e0 = Java_io_buoyant_telemetry_gpu_Native_lastError(env, NULL, h);
  fprintf(g_log, "lastError after a bad setParam: %s\n", (const char*)e0->addr);
  CHECK(e0->len > 0, "lastError text");

  /* pinned staging (pinAlloc): two pairs */
  jobject ids[2], vals[2];
  for (int k = 0; k < 2; ++k) {
    ids[k] = Java_io_buoyant_telemetry_gpu_Native_pinAlloc(env, NULL, (jlong)piece * 4);
    vals[k] = Java_io_buoyant_telemetry_gpu_Native_pinAlloc(env, NULL, (jlong)piece * 4);
    CHECK(ids[k] && vals[k] && ids[k]->cap == (jlong)piece * 4, "pinAlloc");
  }
  CHECK(Java_io_buoyant_telemetry_gpu_Native_pinAlloc(env, NULL, 0) == NULL, "pinAlloc(0) must fail");

  /* Stat.add, batched: the first half through ingestAsync pieces, the rest through ingest */
  const size_t half = n / 2;
  ingest_async_pieces(h, series, values, half, piece, ids, vals);
  for (size_t o = half; o < n; o += piece) {
    const size_t m = n - o < piece ? n - o : piece;
    memcpy(ids[0]->addr, series + o, m * 4);
    memcpy(vals[0]->addr, values + o, m * 4);
    CHECK(Java_io_buoyant_telemetry_gpu_Native_ingest(env, NULL, h, ids[0], vals[0], (jint)m) == 0, "ingest");
  }
  /* a batch with invalid ids: accepted, its invalid samples dropped, reported by sync once */
  {
    uint32_t* bs = (uint32_t*)ids[1]->addr;
    float* bv = (float*)vals[1]->addr;
    bs[0] = (uint32_t)S;
    bs[1] = (uint32_t)S + 100;
    bv[0] = bv[1] = 5.0f;
    CHECK(Java_io_buoyant_telemetry_gpu_Native_ingest(env, NULL, h, ids[1], vals[1], 2) == 0, "ingest(bad ids)");
    const jint r = Java_io_buoyant_telemetry_gpu_Native_sync(env, NULL, h);
    CHECK(r == -EINVAL, "sync after invalid ids returned %d", r);
    jstring e1 = Java_io_buoyant_telemetry_gpu_Native_lastError(env, NULL, h);
    fprintf(g_log, "lastError after invalid ids: %s\n", (const char*)e1->addr);
    CHECK(Java_io_buoyant_telemetry_gpu_Native_sync(env, NULL, h) == 0, "second sync");
  }

  /* peek (Metric.Stat.peek) of series 0..3: count, then up to 2048 entries each */
  {
    FILE* f;
    char p[4096];
    snprintf(p, sizeof p, "%s/peek.bin", dir);
    f = fopen(p, "wb");
    jobject pk = direct(2048 * 12);
    for (int s = 0; s < 4 && s < S; ++s) {
      const jlong k = Java_io_buoyant_telemetry_gpu_Native_peek(env, NULL, h, s, pk, 2048);
      CHECK(k >= 0 && k <= L5DH_NBUCKETS, "peek returned %lld", (long long)k);
      const uint32_t k32 = (uint32_t)k;
      fwrite(&k32, 4, 1, f);
      fwrite(pk->addr, 12, (size_t)k, f);
    }
    fclose(f);
    CHECK(Java_io_buoyant_telemetry_gpu_Native_peek(env, NULL, h, S, pk, 2048) == -EINVAL, "peek(out of range)");
  }

  /* snapshot(0, S, summaries, counts, reset) then the empty snapshot after it */
  {
    jobject out = direct((size_t)S * 88), cnt = direct((size_t)S * L5DH_NBUCKETS * 4);
    CHECK(Java_io_buoyant_telemetry_gpu_Native_snapshot(env, NULL, h, 0, S, out, cnt, 1) == 0, "snapshot(reset)");
    write_file(dir, "summ.bin", out->addr, (size_t)S * 88);
    write_file(dir, "counts.bin", cnt->addr, (size_t)S * L5DH_NBUCKETS * 4);
    jobject out2 = direct((size_t)S * 88);
    CHECK(Java_io_buoyant_telemetry_gpu_Native_snapshot(env, NULL, h, 0, S, out2, NULL, 0) == 0, "snapshot");
    write_file(dir, "summ2.bin", out2->addr, (size_t)S * 88);
  }

  /* fleet merge at one rank: commUniqueId + commInitRank + merge (the RCCL collective
   * forced in the 1-rank communicator), reduce-scatter */
  {
    ingest_async_pieces(h, series, values, n, piece, ids, vals);
    jbyteArray id = Java_io_buoyant_telemetry_gpu_Native_commUniqueId(env, NULL);
    CHECK(id && id->len == L5DH_UNIQUE_ID_BYTES, "commUniqueId");
    CHECK(Java_io_buoyant_telemetry_gpu_Native_commInitRank(env, NULL, h, id, 1, 0) == 0, "commInitRank");
    jbyteArray shortid = fk_NewByteArray(env, 16);  /* not a unique id: refused by the shim */
    CHECK(Java_io_buoyant_telemetry_gpu_Native_commInitRank(env, NULL, h, shortid, 1, 0) == -EINVAL, "short id");
    CHECK(Java_io_buoyant_telemetry_gpu_Native_setParam(env, NULL, h, L5DH_PARAM_MERGE_RCCL_1RANK, 1) == 0, "setParam");
    jobject out = direct((size_t)S * 88), cnt = direct((size_t)S * L5DH_NBUCKETS * 4), tot = direct((size_t)S * 8);
    jintArray range = fk_NewIntArray(env, 2);
    CHECK(Java_io_buoyant_telemetry_gpu_Native_merge(env, NULL, h, L5DH_MERGE_REDUCE_SCATTER, out, cnt, tot, range) == 0,
          "merge");
    const jint* r = (const jint*)range->addr;
    CHECK(r[0] == 0 && r[1] == S, "merge range %d %d", r[0], r[1]);
    write_file(dir, "merge_rs_summ.bin", out->addr, (size_t)S * 88);
    write_file(dir, "merge_rs_counts.bin", cnt->addr, (size_t)S * L5DH_NBUCKETS * 4);
    write_file(dir, "merge_rs_totals.bin", tot->addr, (size_t)S * 8);
  }

  /* a second context in an l5dh_comm_init_all communicator (one process, its GPUs):
   * commInitAll + merge(all-reduce) */
  {
    const jlong h2 = Java_io_buoyant_telemetry_gpu_Native_open(env, NULL, S, 0);
    CHECK(h2 > 0, "open(2)");
    ingest_async_pieces(h2, series, values, n, piece, ids, vals);
    jlongArray ctxs = mkobj(K_LONGARR, calloc(1, 8), 0, 1);
    ((jlong*)ctxs->addr)[0] = h2;
    CHECK(Java_io_buoyant_telemetry_gpu_Native_commInitAll(env, NULL, ctxs) == 0, "commInitAll");
    jobject out = direct((size_t)S * 88), cnt = direct((size_t)S * L5DH_NBUCKETS * 4);
    jintArray range = fk_NewIntArray(env, 2);
    CHECK(Java_io_buoyant_telemetry_gpu_Native_merge(env, NULL, h2, L5DH_MERGE_ALL_REDUCE, out, cnt, NULL, range) == 0,
          "merge(all-reduce)");
    write_file(dir, "merge_ar_summ.bin", out->addr, (size_t)S * 88);
    write_file(dir, "merge_ar_counts.bin", cnt->addr, (size_t)S * L5DH_NBUCKETS * 4);
    CHECK(Java_io_buoyant_telemetry_gpu_Native_close(env, NULL, h2) == 0, "close(2)");
  }

  for (int k = 0; k < 2; ++k) {
    CHECK(Java_io_buoyant_telemetry_gpu_Native_pinFree(env, NULL, ids[k]) == 0, "pinFree");
    CHECK(Java_io_buoyant_telemetry_gpu_Native_pinFree(env, NULL, vals[k]) == 0, "pinFree");
  }
  CHECK(Java_io_buoyant_telemetry_gpu_Native_close(env, NULL, h) == 0, "close");
  fprintf(g_log, "jnienv calls:");
  for (int k = 0; k < 10; ++k) fprintf(g_log, " %d", g_calls[k]);
  fprintf(g_log, "\n");
  fclose(g_log);
  printf("ok\n");
  return 0;
}
