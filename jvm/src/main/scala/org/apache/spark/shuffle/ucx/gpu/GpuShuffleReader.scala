/*
 * GpuShuffleReader — UcxShuffleReader.read (spark_3_0/UcxShuffleReader.scala:74-200) for a GPU
 * shuffle.  The maps are the ones the MapOutputTracker lists for [startPartition,
 * endPartition) (:75-76), in map id order: the canonical per-reducer sequence.
 *
 * 1. Exchange barrier (multi-executor worlds): GpuExchangeCoordinator.awaitExchange -- the
 *    shuffle's collective has moved every executor's map outputs to the reducers' owners.
 * 2. If this executor owns the whole range (SgxNative.shuffleReducers), the work after the
 *    fetch runs on the GPU over HBM-resident blocks:
 *      declared "sum" aggregator (reduceByKey(_ + _): combineValuesByKey, or
 *        combineCombinersByKey after a map-side combine, :155-164)  -> readGrouped(AGG_SUM)
 *      declared "group" aggregator (groupByKey)                      -> readGrouped(AGG_GROUP)
 *      keyOrdering (sortByKey, :166-181)                             -> readSorted
 *      neither (deserializeStream, :137-145)                         -> readRecords
 * 3. Otherwise (Spark placed the task on another executor) the raw blocks of the range come
 *    from their owners over RPC (coordinator.fetchRemote), are imported into this executor's
 *    engine (SgxNative.importBlocks) and read on this GPU by the same calls as 2.
 *
 * Task metrics and cancellation follow the reference's reader (spark_3_0/UcxShuffleReader.scala):
 *   - incFetchWaitTime: the time blocked on the exchange barrier and on remote fetches (the
 *     reference times its progress() spin, :116-123);
 *   - incLocalBlocksFetched / incLocalBytesRead for blocks read from this executor's HBM,
 *     incRemoteBlocksFetched / incRemoteBytesRead for blocks fetched from their owners;
 *   - incRecordsRead per record handed to the task, merged into the task's metrics when the
 *     iterator completes (CompletionIterator + mergeShuffleReadMetrics, :148-153);
 *   - the result is an InterruptibleIterator (:155-156, :193-199), so a killed task stops at
 *     its next record, and a task killed while it waits for the exchange stops before the read.
 */
package org.apache.spark.shuffle.ucx.gpu

import java.nio.{ByteBuffer, ByteOrder}

import java.util.concurrent.TimeUnit

import org.apache.spark.{InterruptibleIterator, SparkEnv, TaskContext}
import org.apache.spark.shuffle.{ShuffleReadMetricsReporter, ShuffleReader}
import org.apache.spark.storage.ShuffleBlockId
import org.apache.spark.util.CompletionIterator
import org.apache.spark.util.collection.CompactBuffer

class GpuShuffleReader[K, C](engine: Long, handle: GpuShuffleHandle[K, _, C], startPartition: Int,
                             endPartition: Int, context: TaskContext,
                             coordinator: Option[GpuExchangeCoordinator],
                             readMetrics: ShuffleReadMetricsReporter,
                             mapRange: Option[(Int, Int)] = None) extends ShuffleReader[K, C] {
  private val dep = handle.dependency
  private val shuffleId = handle.shuffleId

  private def ids(blocks: Iterator[(_, Seq[(org.apache.spark.storage.BlockId, Long, Int)])]): Array[Long] =
    blocks.flatMap(_._2.map(_._1.asInstanceOf[ShuffleBlockId].mapId)).toArray.distinct.sorted

  /** The maps this read covers: those the MapOutputTracker lists for the partition range (and,
   *  for the AQE local reader, getReaderForRange's map index range). */
  private def mapIds: Array[Long] = mapRange match {
    case Some((m0, m1)) =>
      ids(SparkEnv.get.mapOutputTracker.getMapSizesByRange(shuffleId, m0, m1, startPartition, endPartition))
    case None =>
      ids(SparkEnv.get.mapOutputTracker.getMapSizesByExecutorId(shuffleId, startPartition, endPartition))
  }

  /** The shuffle's full map set (every partition): the exchange key every reduce task of the
   *  stage agrees on, whatever its own range.  Built once per map-output epoch on the executor
   *  (GpuExchangeCoordinator.allMapIds), not by every reduce task: listing every block of every
   *  partition costs M x R tuples. */
  private def allMapIds(coord: GpuExchangeCoordinator): Array[Long] =
    coord.allMapIds(shuffleId, SparkEnv.get.mapOutputTracker.getEpoch,
      ids(SparkEnv.get.mapOutputTracker.getMapSizesByExecutorId(shuffleId, 0, dep.partitioner.numPartitions)))

  /** A little-endian direct buffer of n bytes (a clear error past 2 GiB, no silent wrap). */
  private def le(n: Long): ByteBuffer = {
    if (n > Int.MaxValue - 8)
      throw new UnsupportedOperationException(
        s"a read of $n bytes of ONE partition exceeds one direct buffer (2 GiB)")
    ByteBuffer.allocateDirect(math.max(8L, n).toInt).order(ByteOrder.LITTLE_ENDIAN)
  }

  /** The largest result one engine call hands over (a direct buffer holds < 2 GiB). */
  private val maxChunkBytes: Long = SparkEnv.get.conf.getSizeAsBytes("spark.shuffle.ucx.gpu.readChunkBytes",
    (1L << 30).toString)

  /** The engine's size of a read of [a, b): what readGrouped / readSorted / readRecords would
   *  hand over (groups and values for an aggregation, bytes otherwise). */
  private def readSize(maps: Array[Long], a: Int, b: Int): Long =
    if (handle.agg != GpuUcxShuffleManager.NO_AGG) {
      val Array(groups, values, _) = SgxNative.readGrouped(engine, shuffleId, maps, a, b, handle.agg, null, null, null)
      8 * math.max(groups, values)
    } else if (dep.keyOrdering.isDefined) SgxNative.readSorted(engine, shuffleId, maps, a, b, null)
    else SgxNative.readRecords(engine, shuffleId, maps, a, b, null)

  /** [start, end) cut into partition sub-ranges whose results fit maxChunkBytes, read one after
   *  the other as the task consumes them: a range's sorted / grouped / plain result is the
   *  concatenation of its partitions' (a key lives in one partition; sortByKey's reader
   *  orders by partition, then key), so a large reduce task streams instead of failing on one
   *  2 GiB buffer.  A sub-range too large is halved; a single partition too large fails. */
  private def chunked(maps: Array[Long]): Iterator[Product2[K, C]] = {
    def ranges(a: Int, b: Int): Iterator[(Int, Int)] =
      if (b - a <= 1 || readSize(maps, a, b) <= maxChunkBytes) Iterator.single((a, b))
      else {
        val m = a + (b - a) / 2
        ranges(a, m) ++ ranges(m, b)
      }
    ranges(startPartition, endPartition).flatMap { case (a, b) => readOnGpu(maps, a, b) }
  }

  /** Blocks (map, reducer) of the range that hold bytes, and their bytes (the engine's lengths). */
  private def blockStats(maps: Array[Long]): (Long, Long) = {
    val nm = maps.length
    if (nm == 0 || endPartition <= startPartition) return (0L, 0L)
    val rs = (startPartition until endPartition).toArray
    val sizes = SgxNative.fetchBlocks(engine, shuffleId, rs.flatMap(_ => maps), rs.flatMap(r => Array.fill(nm)(r)), null)
    (sizes.count(_ > 0).toLong, sizes.sum)
  }

  private def timedWait[T](f: => T): T = {
    val t0 = System.nanoTime()
    try f finally readMetrics.incFetchWaitTime(TimeUnit.NANOSECONDS.toMillis(System.nanoTime() - t0))
  }

  override def read(): Iterator[Product2[K, C]] = {
    val maps = mapIds
    coordinator.foreach(c => timedWait(c.awaitExchange(shuffleId, allMapIds(c), handle.spec)))
    context.killTaskIfInterrupted()  // killed while it waited for the collective
    val local = coordinator.isEmpty || {
      val Array(r0, r1) = SgxNative.shuffleReducers(engine, shuffleId)
      r0 <= startPartition && endPartition <= r1
    }
    val records = if (local) {
      val (blocks, bytes) = blockStats(maps)
      readMetrics.incLocalBlocksFetched(blocks)
      readMetrics.incLocalBytesRead(bytes)
      chunked(maps)
    } else readRemote(maps, coordinator.get)
    // one per shuffled record; behind an aggregator readOnGpu counts the records it consumed
    val aggregated = handle.agg != GpuUcxShuffleManager.NO_AGG
    val counted = CompletionIterator[Product2[K, C], Iterator[Product2[K, C]]](
      if (aggregated) records else records.map { r => readMetrics.incRecordsRead(1); r },
      context.taskMetrics().mergeShuffleReadMetrics())
    new InterruptibleIterator[Product2[K, C]](context, counted)
  }

  private def readOnGpu(maps: Array[Long], a: Int, b: Int): Iterator[Product2[K, C]] = {
    if (handle.agg != GpuUcxShuffleManager.NO_AGG) {
      val sum = handle.agg == SgxNative.AGG_SUM
      val Array(groups, values, _) = SgxNative.readGrouped(engine, shuffleId, maps, a, b, handle.agg, null, null, null)
      val keys = le(groups * 8); val starts = le(groups * 8); val vals = le(values * 8)
      val Array(_, _, consumed) = SgxNative.readGrouped(engine, shuffleId, maps, a, b, handle.agg, keys, starts, vals)
      // the reference counts every shuffled record ahead of the aggregator, not its groups
      // (spark_3_0/UcxShuffleReader.scala:148-162)
      readMetrics.incRecordsRead(consumed)
      val k = keys.asLongBuffer(); val s = starts.asLongBuffer(); val v = vals.asLongBuffer()
      if (sum) {
        Iterator.tabulate(groups.toInt)(g => (k.get(g), v.get(g)).asInstanceOf[Product2[K, C]])
      } else {
        // groupByKey's combiner type is CompactBuffer[V], values in arrival order
        Iterator.tabulate(groups.toInt) { g =>
          val end = if (g + 1 < groups) s.get(g + 1) else values
          val buf = new CompactBuffer[Long]
          var i = s.get(g)
          while (i < end) { buf += v.get(i.toInt); i += 1 }
          (k.get(g), buf).asInstanceOf[Product2[K, C]]
        }
      }
    } else {
      val sorted = dep.keyOrdering.isDefined
      val bytes = if (sorted) SgxNative.readSorted(engine, shuffleId, maps, a, b, null)
                  else SgxNative.readRecords(engine, shuffleId, maps, a, b, null)
      val dst = le(bytes)
      if (sorted) SgxNative.readSorted(engine, shuffleId, maps, a, b, dst)
      else SgxNative.readRecords(engine, shuffleId, maps, a, b, dst)
      val recs = dst.asLongBuffer()
      Iterator.tabulate((bytes / 16).toInt)(i => (recs.get(2 * i), recs.get(2 * i + 1)).asInstanceOf[Product2[K, C]])
    }
  }

  /** Reducers this executor does not hold (Spark placed the task here): their raw blocks come
   *  from the owners over RPC -- one request per owner, its reducers of the range x every map,
   *  reducer-major (coordinator.fetchRemote, served from the owner's HBM) -- and are imported
   *  into this executor's engine (SgxNative.importBlocks), so the read runs on this GPU exactly
   *  as an owner's does: Kryo / LZ4 decode, sort, group, sum.  The reference's "any block from
   *  anywhere" (spark_3_0/UcxShuffleReader.scala:74-103), without Spark's CPU reader. */
  private def readRemote(maps: Array[Long], coord: GpuExchangeCoordinator): Iterator[Product2[K, C]] = {
    val owners = coord.rankRanges(shuffleId).toSeq.sortBy(_._2(0))
    val nm = maps.length
    val lengths = new Array[Long]((endPartition - startPartition) * nm)
    val pieces = owners.flatMap { case (rank, Array(a, b)) =>
      val lo = math.max(a, startPartition)
      val hi = math.min(b, endPartition)
      if (lo >= hi || nm == 0) None
      else {
        val rs = (lo until hi).toArray
        val got = timedWait(coord.fetchRemote(shuffleId, rank, rs.flatMap(_ => maps), rs.flatMap(r => Array.fill(nm)(r))))
        System.arraycopy(got.lengths, 0, lengths, (lo - startPartition) * nm, got.lengths.length)
        readMetrics.incRemoteBlocksFetched(got.lengths.count(_ > 0).toLong)
        readMetrics.incRemoteBytesRead(got.bytes.length.toLong)
        Some(got.bytes)
      }
    }
    val covered = owners.map { case (_, Array(a, b)) => math.max(0, math.min(b, endPartition) - math.max(a, startPartition)) }.sum
    if (covered != endPartition - startPartition)
      throw new SgxFetchException(s"the executors' reducer ranges do not cover [$startPartition, $endPartition) " +
                                  s"of shuffle $shuffleId")
    val buf = le(lengths.sum)
    pieces.foreach(p => buf.put(p))
    buf.flip()
    val id = SgxNative.importBlocks(engine, shuffleId, maps, startPartition, endPartition, buf, lengths)
    // every read copies its results out of HBM before returning: the import goes once the
    // last sub-range has been read (the iterator drains the chunks in order)
    var released = false
    def release(): Unit = if (!released) {
      released = true
      SgxNative.releaseImport(engine, shuffleId, id)
    }
    context.addTaskCompletionListener[Unit](_ => release())  // a killed task drops it too
    CompletionIterator[Product2[K, C], Iterator[Product2[K, C]]](chunked(maps), release())
  }
}
