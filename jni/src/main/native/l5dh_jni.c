/*
 * l5dh_jni.c -- JNI shim between the Scala telemetry (io.buoyant.telemetry.gpu.Native)
 * and the C-ABI of include/l5dhist.h.  One JNI method per entry point, no logic:
 * handles are jlong context pointers, data crosses as direct ByteBuffers (no copies
 * of staged samples or summaries), status codes pass through unchanged (<0: -errno).
 *
 * Reference interface replaced: io.buoyant.telemetry.Metric.Stat
 * (telemetry/core/src/main/scala/io/buoyant/telemetry/Metric.scala:22-70), driven by
 * MetricsTree.mkStat (MetricsTree.scala:85-93) and
 * AdminMetricsExportTelemeter.snapshotHistograms (AdminMetricsExportTelemeter.scala:154-162).
 *
 * Build (needs a JDK): make -C jni   (gcc -shared -fPIC -I$JAVA_HOME/include ... -ll5dhist)
 */
#include <jni.h>
#include <stdint.h>
#include <string.h>

#include "l5dhist.h"

#define CTX(h) ((l5dh_ctx*)(intptr_t)(h))
#define ADDR(b) ((b) ? (*env)->GetDirectBufferAddress(env, (b)) : NULL)

/* long open(int maxSeries, int device): context handle (> 0) or -errno */
JNIEXPORT jlong JNICALL Java_io_buoyant_telemetry_gpu_Native_open(JNIEnv* env, jclass k, jint maxSeries,
                                                                   jint device) {
  (void)env; (void)k;
  l5dh_ctx* c = NULL;
  const int rc = l5dh_open(&c, (uint32_t)maxSeries, 1u << (unsigned)device);
  return rc == 0 ? (jlong)(intptr_t)c : (jlong)rc;
}

JNIEXPORT jint JNICALL Java_io_buoyant_telemetry_gpu_Native_close(JNIEnv* env, jclass k, jlong ctx) {
  (void)env; (void)k;
  return l5dh_close(CTX(ctx));
}

/* int[] limits(): BucketedHistogram.DefaultLimits (1797 entries) */
JNIEXPORT jintArray JNICALL Java_io_buoyant_telemetry_gpu_Native_limits(JNIEnv* env, jclass k) {
  (void)k;
  size_t n = 0;
  const int32_t* l = l5dh_limits(&n);
  jintArray a = (*env)->NewIntArray(env, (jsize)n);
  if (a && l) (*env)->SetIntArrayRegion(env, a, 0, (jsize)n, (const jint*)l);
  return a;
}

/* ingest(ctx, ids: direct buffer of n u32, values: direct buffer of n f32, n): Stat.add batched */
JNIEXPORT jint JNICALL Java_io_buoyant_telemetry_gpu_Native_ingest(JNIEnv* env, jclass k, jlong ctx, jobject ids,
                                                                    jobject values, jint n) {
  (void)k;
  return l5dh_ingest(CTX(ctx), (const uint32_t*)ADDR(ids), (const float*)ADDR(values), (size_t)n);
}

/* long ingestAsync(ctx, ids, values, n): ticket (>= 0) or -errno; the buffers stay
 * untouched until ingestWait(ctx, ticket) (double-buffered per-thread staging) */
JNIEXPORT jlong JNICALL Java_io_buoyant_telemetry_gpu_Native_ingestAsync(JNIEnv* env, jclass k, jlong ctx, jobject ids,
                                                                          jobject values, jint n) {
  (void)k;
  uint64_t t = 0;
  const int rc = l5dh_ingest_async(CTX(ctx), (const uint32_t*)ADDR(ids), (const float*)ADDR(values), (size_t)n, &t);
  return rc == 0 ? (jlong)t : (jlong)rc;
}

JNIEXPORT jint JNICALL Java_io_buoyant_telemetry_gpu_Native_ingestWait(JNIEnv* env, jclass k, jlong ctx, jlong ticket) {
  (void)env; (void)k;
  return l5dh_ingest_wait(CTX(ctx), (uint64_t)ticket);
}

/* snapshot(ctx, first, count, out: count*88 B or null, counts: count*1798*4 B or null, reset) */
JNIEXPORT jint JNICALL Java_io_buoyant_telemetry_gpu_Native_snapshot(JNIEnv* env, jclass k, jlong ctx, jint first,
                                                                      jint count, jobject out, jobject counts,
                                                                      jboolean reset) {
  (void)k;
  return l5dh_snapshot(CTX(ctx), (uint32_t)first, (uint32_t)count, (l5dh_summary*)ADDR(out), (int32_t*)ADDR(counts),
                       reset ? 1 : 0);
}

/* peek(ctx, series, out: cap*12 B, cap): number of non-empty buckets (may exceed cap) or -errno */
JNIEXPORT jlong JNICALL Java_io_buoyant_telemetry_gpu_Native_peek(JNIEnv* env, jclass k, jlong ctx, jint series,
                                                                   jobject out, jint cap) {
  (void)k;
  size_t n = 0;
  const int rc = l5dh_peek(CTX(ctx), (uint32_t)series, (l5dh_bucket_count*)ADDR(out), (size_t)cap, &n);
  return rc == 0 ? (jlong)n : (jlong)rc;
}

JNIEXPORT jint JNICALL Java_io_buoyant_telemetry_gpu_Native_sync(JNIEnv* env, jclass k, jlong ctx) {
  (void)env; (void)k;
  return l5dh_sync(CTX(ctx));
}

JNIEXPORT jint JNICALL Java_io_buoyant_telemetry_gpu_Native_setParam(JNIEnv* env, jclass k, jlong ctx, jint param,
                                                                      jlong value) {
  (void)env; (void)k;
  return l5dh_set_param(CTX(ctx), (int)param, (int64_t)value);
}

/* ByteBuffer pinAlloc(bytes): pinned host staging owned by the library, or null */
JNIEXPORT jobject JNICALL Java_io_buoyant_telemetry_gpu_Native_pinAlloc(JNIEnv* env, jclass k, jlong bytes) {
  (void)k;
  void* p = NULL;
  if (bytes <= 0 || l5dh_pin_alloc((size_t)bytes, &p) != 0) return NULL;
  return (*env)->NewDirectByteBuffer(env, p, bytes);
}

JNIEXPORT jint JNICALL Java_io_buoyant_telemetry_gpu_Native_pinFree(JNIEnv* env, jclass k, jobject buf) {
  (void)k;
  return l5dh_pin_free(ADDR(buf));
}

/* byte[] commUniqueId(): rank 0 creates it, the caller distributes it */
JNIEXPORT jbyteArray JNICALL Java_io_buoyant_telemetry_gpu_Native_commUniqueId(JNIEnv* env, jclass k) {
  (void)k;
  uint8_t id[L5DH_UNIQUE_ID_BYTES];
  if (l5dh_comm_unique_id(id) != 0) return NULL;
  jbyteArray a = (*env)->NewByteArray(env, L5DH_UNIQUE_ID_BYTES);
  if (a) (*env)->SetByteArrayRegion(env, a, 0, L5DH_UNIQUE_ID_BYTES, (const jbyte*)id);
  return a;
}

JNIEXPORT jint JNICALL Java_io_buoyant_telemetry_gpu_Native_commInitRank(JNIEnv* env, jclass k, jlong ctx,
                                                                          jbyteArray id, jint nranks, jint rank) {
  (void)k;
  uint8_t buf[L5DH_UNIQUE_ID_BYTES];
  if (!id || (*env)->GetArrayLength(env, id) != L5DH_UNIQUE_ID_BYTES) return -22; /* -EINVAL */
  (*env)->GetByteArrayRegion(env, id, 0, L5DH_UNIQUE_ID_BYTES, (jbyte*)buf);
  return l5dh_comm_init_rank(CTX(ctx), buf, (int)nranks, (int)rank);
}

/* commInitAll(long[] ctxs): one process holding several GPUs */
JNIEXPORT jint JNICALL Java_io_buoyant_telemetry_gpu_Native_commInitAll(JNIEnv* env, jclass k, jlongArray ctxs) {
  (void)k;
  const jsize n = ctxs ? (*env)->GetArrayLength(env, ctxs) : 0;
  if (n <= 0 || n > 64) return -22;
  jlong h[64];
  l5dh_ctx* c[64];
  (*env)->GetLongArrayRegion(env, ctxs, 0, n, h);
  for (jsize i = 0; i < n; ++i) c[i] = CTX(h[i]);
  return l5dh_comm_init_all(c, (int)n);
}

/* merge(ctx, mode, out, counts, totals, range: int[2] {first, count}) -- collective */
JNIEXPORT jint JNICALL Java_io_buoyant_telemetry_gpu_Native_merge(JNIEnv* env, jclass k, jlong ctx, jint mode,
                                                                   jobject out, jobject counts, jobject totals,
                                                                   jintArray range) {
  (void)k;
  uint32_t first = 0, count = 0;
  const int rc = l5dh_merge(CTX(ctx), (int)mode, (l5dh_summary*)ADDR(out), (int32_t*)ADDR(counts),
                            (int64_t*)ADDR(totals), &first, &count);
  if (rc == 0 && range && (*env)->GetArrayLength(env, range) >= 2) {
    const jint r[2] = {(jint)first, (jint)count};
    (*env)->SetIntArrayRegion(env, range, 0, 2, r);
  }
  return rc;
}

JNIEXPORT jstring JNICALL Java_io_buoyant_telemetry_gpu_Native_lastError(JNIEnv* env, jclass k, jlong ctx) {
  (void)k;
  return (*env)->NewStringUTF(env, l5dh_last_error(CTX(ctx)));
}
