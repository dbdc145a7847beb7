package io.buoyant.telemetry.gpu

import com.twitter.finagle.stats.BucketAndCount
import com.twitter.util.{Duration, Time}
import io.buoyant.telemetry.Metric.HistogramSummary
import java.nio.{ByteBuffer, ByteOrder}
import java.util.concurrent.ConcurrentLinkedQueue

/**
 * The histograms of up to `capacity` Stats on one MI355X (one l5dh context), for the
 * Scala telemetry.  Mirrors linkerd_amd/telemetry.py StatEngine (the tested Python
 * host side of the same C-ABI):
 *
 *  - `register` / `release` hand out dense series ids (MetricsTree.mkStat,
 *    MetricsTree.scala:85-93; MetricsTree.prune via MetricsPruningModule.scala:14-39);
 *    a released id is cleared on the GPU before it is reused.
 *  - `add` appends to the calling thread's pinned staging buffers (direct ByteBuffers
 *    over l5dh_pin_alloc memory), two per thread: a full buffer goes to the GPU with
 *    l5dh_ingest_async and the thread fills the other one while it is copied (it
 *    waits for that buffer's ticket before refilling it).
 *  - every read (summary / peek / reset / snapshotAll) flushes all staging buffers
 *    first, then makes ONE engine call, so a reset cannot lose a sample that another
 *    thread flushed in between (Metric.scala:44-51 holds one lock for the same reason).
 *
 * Statuses from the shim are 0 or -errno; failures throw IllegalStateException
 * with l5dh_last_error's text (the reference's Stat never fails, the GPU can).
 */
final class GpuEngine(val capacity: Int, device: Int = 0, batch: Int = 1 << 16) {
  private[this] val ctx: Long = {
    val h = Native.open(capacity, device)
    if (h <= 0) throw new IllegalStateException(s"l5dh_open(capacity=$capacity, device=$device) failed: $h")
    h
  }
  private[this] val limits: Array[Int] = Native.limits()
  private[this] val freeIds = new java.util.ArrayDeque[Integer]
  private[this] var nextId = 0
  private[this] val stagings = new ConcurrentLinkedQueue[Staging]
  // close(): `closed` is set first (no new operation starts, no thread gets a new
  // Staging); every call that passes `ctx` to native code runs under the read lock, and
  // the context is released under the write lock, so no call can use a freed context
  @volatile private[this] var closed = false
  private[this] var released = false // guarded by the write lock
  private[this] val rw = new java.util.concurrent.locks.ReentrantReadWriteLock
  private[this] val local = new ThreadLocal[Staging] {
    override def initialValue(): Staging = {
      if (closed) throw new IllegalStateException("GpuEngine is closed")
      val s = new Staging
      stagings.add(s)
      if (closed) { // close() may have freed the stagings it saw before this one was added
        stagings.remove(s)
        s.free()
        throw new IllegalStateException("GpuEngine is closed")
      }
      s
    }
  }

  /** A call on `ctx`: fails once close() has begun (`closing`: close's own flushes). */
  private[this] def onCtx[T](closing: Boolean = false)(body: => T): T = {
    val r = rw.readLock
    r.lock()
    try {
      if (released || (closed && !closing)) throw new IllegalStateException("GpuEngine is closed")
      body
    } finally r.unlock()
  }

  private[this] def check(rc: Long, what: String): Unit =
    if (rc < 0) throw new IllegalStateException(s"$what failed: $rc ${Native.lastError(ctx)}")

  private[this] def pinned(bytes: Long): ByteBuffer = {
    val b = Native.pinAlloc(bytes)
    if (b == null) throw new OutOfMemoryError(s"l5dh_pin_alloc($bytes)")
    b.order(ByteOrder.LITTLE_ENDIAN)
  }

  /** One thread's staged Stat.add calls: two pinned buffer pairs, double-buffered. */
  private final class Staging {
    private[this] val ids = Array(pinned(4L * batch), pinned(4L * batch))
    private[this] val values = Array(pinned(4L * batch), pinned(4L * batch))
    private[this] val ticket = Array(0L, 0L) // l5dh_ingest_async ticket of each pair (0: free)
    private[this] var cur = 0
    private[this] var n = 0
    private[this] var closed = false // the pinned buffers went back to the library (free)

    def add(id: Int, value: Float): Unit = synchronized {
      // a thread adding after (or racing with) close() must not write freed native memory
      if (closed || GpuEngine.this.closed) throw new IllegalStateException("GpuEngine is closed")
      ids(cur).putInt(4 * n, id)
      values(cur).putFloat(4 * n, value)
      n += 1
      if (n == batch) flushLocked(waitAll = false)
    }

    /** Everything staged reaches the library; returns once both buffers are free. */
    def flush(): Unit = synchronized { if (!closed) flushLocked(waitAll = true) }

    private[this] def flushLocked(waitAll: Boolean, closing: Boolean = false): Unit = onCtx(closing) {
      if (n > 0) {
        val m = n
        n = 0 // cleared first: a batch the library refused is dropped, never re-sent (no double count)
        val t = Native.ingestAsync(ctx, ids(cur), values(cur), m)
        check(t, "l5dh_ingest_async") // < 0: this batch was not queued (deferred id errors come from sync)
        ticket(cur) = t
        cur ^= 1
        // the other pair is refilled next: its copy must be done
        if (ticket(cur) != 0) { check(Native.ingestWait(ctx, ticket(cur)), "l5dh_ingest_wait"); ticket(cur) = 0 }
      }
      if (waitAll) for (k <- 0 to 1 if ticket(k) != 0) {
        check(Native.ingestWait(ctx, ticket(k)), "l5dh_ingest_wait")
        ticket(k) = 0
      }
    }

    /** After a final flush: the pinned buffers go back to the library. */
    def free(): Unit = synchronized {
      if (!closed) {
        closed = true // first: a failing flush still leaves the Staging closed
        try flushLocked(waitAll = true, closing = true)
        finally for (b <- ids ++ values) Native.pinFree(b)
      }
    }
  }

  def register(): Int = synchronized {
    if (!freeIds.isEmpty) freeIds.pop().intValue
    else if (nextId >= capacity) throw new IllegalStateException(s"histogram engine full: $capacity series")
    else { nextId += 1; nextId - 1 }
  }

  def release(id: Int): Unit = {
    flush()
    onCtx()(check(Native.snapshot(ctx, id, 1, null, null, true), "l5dh_snapshot(reset)"))
    synchronized { freeIds.push(id) }
  }

  def add(id: Int, value: Float): Unit = local.get.add(id, value)

  def flush(): Unit = {
    if (closed) throw new IllegalStateException("GpuEngine is closed")
    val it = stagings.iterator
    while (it.hasNext) it.next.flush()
  }

  private[this] def decode(b: ByteBuffer, i: Int): HistogramSummary = {
    val o = i * Native.SUMMARY_BYTES
    HistogramSummary(b.getLong(o), b.getLong(o + 8), b.getLong(o + 16), b.getLong(o + 24), b.getLong(o + 32),
      b.getLong(o + 40), b.getLong(o + 48), b.getLong(o + 56), b.getLong(o + 64), b.getLong(o + 72),
      b.getDouble(o + 80))
  }

  private[this] def buckets(row: ByteBuffer): Seq[BucketAndCount] = {
    val out = Seq.newBuilder[BucketAndCount]
    var b = 0
    while (b < Native.NBUCKETS) {
      val c = row.getInt(4 * b)
      if (c > 0) {
        val lower = if (b == 0) 0 else limits(b - 1)
        val upper = if (b < limits.length) limits(b) else Int.MaxValue
        out += BucketAndCount(lower, upper, c)
      }
      b += 1
    }
    out.result()
  }

  /** Metric.Stat.summary (Metric.scala:53-67) of one series, without reset. */
  def summary(id: Int): HistogramSummary = {
    flush()
    val b = ByteBuffer.allocateDirect(Native.SUMMARY_BYTES).order(ByteOrder.LITTLE_ENDIAN)
    onCtx()(check(Native.snapshot(ctx, id, 1, b, null, false), "l5dh_snapshot"))
    decode(b, 0)
  }

  /** Metric.Stat.peek (Metric.scala:35-37). */
  def peek(id: Int): Seq[BucketAndCount] = {
    flush()
    val row = ByteBuffer.allocateDirect(4 * Native.NBUCKETS).order(ByteOrder.LITTLE_ENDIAN)
    onCtx()(check(Native.snapshot(ctx, id, 1, null, row, false), "l5dh_snapshot(counts)"))
    buckets(row)
  }

  /** Metric.Stat.reset (Metric.scala:44-51): bucketAndCounts + clear in one call. */
  def reset(id: Int): Seq[BucketAndCount] = {
    flush()
    val row = ByteBuffer.allocateDirect(4 * Native.NBUCKETS).order(ByteOrder.LITTLE_ENDIAN)
    onCtx()(check(Native.snapshot(ctx, id, 1, null, row, true), "l5dh_snapshot(counts, reset)"))
    buckets(row)
  }

  /**
   * The batched AdminMetricsExportTelemeter.snapshotHistograms
   * (AdminMetricsExportTelemeter.scala:154-162): ONE fused GPU snapshot + reset of
   * every registered series; `f(id, summary)` is called per series id.
   */
  def snapshotAll(f: (Int, HistogramSummary) => Unit): Unit = {
    flush()
    val n = synchronized(nextId)
    if (n > 0) {
      val out = ByteBuffer.allocateDirect(n * Native.SUMMARY_BYTES).order(ByteOrder.LITTLE_ENDIAN)
      onCtx()(check(Native.snapshot(ctx, 0, n, out, null, true), "l5dh_snapshot(all, reset)"))
      var i = 0
      while (i < n) { f(i, decode(out, i)); i += 1 }
    }
  }

  /**
   * Flushes and frees every thread's staging (each one even when another fails), then
   * releases the context once every in-flight call on it has returned; the first
   * failure is rethrown after that.  Any later call fails with IllegalStateException.
   */
  def close(): Unit = {
    closed = true // first: no new call starts and no thread gets a new Staging
    var first: Throwable = null
    def keep(t: Throwable): Unit = if (first == null) first = t
    val it = stagings.iterator
    while (it.hasNext) {
      try it.next.free() // flushed, closed, its pinned buffers freed
      catch { case t: Throwable => keep(t) }
    }
    stagings.clear()
    val w = rw.writeLock
    w.lock() // every call that passed the closed check has returned
    try {
      if (!released) {
        try check(Native.sync(ctx), "l5dh_sync") // may report a deferred invalid-id -EINVAL (ABI 3)
        catch { case t: Throwable => keep(t) }
        released = true
        val rc = Native.close(ctx) // (no l5dh_last_error after this: the context is gone)
        if (rc < 0) keep(new IllegalStateException(s"l5dh_close failed: $rc"))
      }
    } finally w.unlock()
    if (first != null) throw first
  }
}

/**
 * The storage of one io.buoyant.telemetry.Metric.Stat on a GpuEngine, with the
 * Stat's public surface (Metric.scala:22-70): add, peek, snapshot, reset, summary,
 * snapshottedSummary, startingAt.  Metric is sealed, so the drop-in is Metric.Stat
 * delegating to one of these (INTEGRATION.md §2); exporters keep reading
 * snapshottedSummary unchanged.
 */
final class GpuStat(engine: GpuEngine) {
  @volatile private[this] var id: Int = engine.register()
  @volatile private[this] var summarySnapshot: HistogramSummary = null
  @volatile private[this] var resetTime: Time = Time.now

  def seriesId: Int = id
  def startingAt: Time = resetTime

  /**
   * A pruned Stat still accepts samples; they go nowhere (no exporter reads it).  The
   * id is read and the sample staged under this Stat's monitor (Metric.scala:30-33 holds
   * one per Stat), and `release` takes the id away under the same monitor: once it has,
   * no add can stage the old id, which the engine may hand to a new Stat.
   */
  def add(value: Float): Unit = synchronized { val i = id; if (i >= 0) engine.add(i, value) }

  def peek: Seq[BucketAndCount] = { val i = id; if (i >= 0) engine.peek(i) else Nil }

  def summary: HistogramSummary = {
    val i = id
    if (i >= 0) engine.summary(i) else HistogramSummary(0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0.0)
  }

  def snapshot(): HistogramSummary = { summarySnapshot = summary; summarySnapshot }

  def reset(): (Seq[BucketAndCount], Duration) = {
    val i = id
    val buckets = if (i >= 0) engine.reset(i) else Nil
    val now = Time.now
    val delta = now - resetTime
    resetTime = now
    (buckets, delta)
  }

  def snapshottedSummary: HistogramSummary = summarySnapshot

  /** Set by the batched snapshot driver (GpuEngine.snapshotAll). */
  def setSnapshot(s: HistogramSummary, at: Time): Unit = { summarySnapshot = s; resetTime = at }

  /** MetricsTree.prune: give the series id back. */
  def release(): Unit = synchronized {
    val i = id
    id = -1
    if (i >= 0) engine.release(i)
  }
}
