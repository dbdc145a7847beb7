package io.buoyant.telemetry.gpu;

import java.nio.ByteBuffer;

/**
 * JNI entry points of libl5dh_jni.so (jni/src/main/native/l5dh_jni.c), one per
 * C-ABI function of include/l5dhist.h.  Buffers are direct and little endian;
 * status codes are 0 or -errno.
 */
public final class Native {
  static { System.loadLibrary("l5dh_jni"); }

  private Native() {}

  public static final int SUMMARY_BYTES = 88;       // Metric.HistogramSummary: 10 x int64 + double
  public static final int BUCKET_COUNT_BYTES = 12;  // BucketAndCount(lower, upper, count)
  public static final int NBUCKETS = 1798;
  public static final int MERGE_REDUCE_SCATTER = 0;
  public static final int MERGE_ALL_REDUCE = 1;
  public static final int PARAM_STAGE_SAMPLES = 9;

  public static native long open(int maxSeries, int device);
  public static native int close(long ctx);
  public static native int[] limits();
  public static native int ingest(long ctx, ByteBuffer ids, ByteBuffer values, int n);
  public static native long ingestAsync(long ctx, ByteBuffer ids, ByteBuffer values, int n);
  public static native int ingestWait(long ctx, long ticket);
  public static native int snapshot(long ctx, int first, int count, ByteBuffer out, ByteBuffer counts, boolean reset);
  public static native long peek(long ctx, int series, ByteBuffer out, int cap);
  public static native int sync(long ctx);
  public static native int setParam(long ctx, int param, long value);
  public static native ByteBuffer pinAlloc(long bytes);
  public static native int pinFree(ByteBuffer buf);
  public static native byte[] commUniqueId();
  public static native int commInitRank(long ctx, byte[] id, int nranks, int rank);
  public static native int commInitAll(long[] ctxs);
  public static native int merge(long ctx, int mode, ByteBuffer out, ByteBuffer counts, ByteBuffer totals, int[] range);
  public static native String lastError(long ctx);
}
