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
 * 3. Otherwise (Spark placed the task on another executor) the raw blocks of the reducers
 *    this executor does not hold come from their owners over RPC (coordinator.fetchRemote),
 *    and the read runs on the CPU with Spark's own serializer stream, the dependency's real
 *    aggregator and an ExternalSorter -- what BlockStoreShuffleReader does, so the results
 *    are Spark's.
 */
package org.apache.spark.shuffle.ucx.gpu

import java.io.ByteArrayInputStream
import java.nio.{ByteBuffer, ByteOrder}

import org.apache.spark.{SparkEnv, TaskContext}
import org.apache.spark.serializer.KryoSerializer
import org.apache.spark.shuffle.{BaseShuffleHandle, ShuffleReader}
import org.apache.spark.storage.ShuffleBlockId
import org.apache.spark.util.CompletionIterator
import org.apache.spark.util.collection.{CompactBuffer, ExternalSorter}

class GpuShuffleReader[K, C](engine: Long, handle: GpuShuffleHandle[K, _, C], startPartition: Int,
                             endPartition: Int, context: TaskContext,
                             coordinator: Option[GpuExchangeCoordinator]) extends ShuffleReader[K, C] {
  private val dep = handle.dependency
  private val shuffleId = handle.shuffleId

  private def mapIds: Array[Long] =
    SparkEnv.get.mapOutputTracker
      .getMapSizesByExecutorId(shuffleId, startPartition, endPartition)
      .flatMap(_._2.map(_._1.asInstanceOf[ShuffleBlockId].mapId))
      .toArray.distinct.sorted

  /** A little-endian direct buffer of n bytes (a clear error past 2 GiB, no silent wrap). */
  private def le(n: Long): ByteBuffer = {
    if (n > Int.MaxValue - 8)
      throw new UnsupportedOperationException(
        s"a read of $n bytes exceeds one direct buffer: split the reduce task's partition range")
    ByteBuffer.allocateDirect(math.max(8L, n).toInt).order(ByteOrder.LITTLE_ENDIAN)
  }

  override def read(): Iterator[Product2[K, C]] = {
    val maps = mapIds
    coordinator.foreach(_.awaitExchange(shuffleId, maps))
    val local = coordinator.isEmpty || {
      val Array(r0, r1) = SgxNative.shuffleReducers(engine, shuffleId)
      r0 <= startPartition && endPartition <= r1
    }
    if (local) readOnGpu(maps) else readRemote(maps, coordinator.get)
  }

  private def readOnGpu(maps: Array[Long]): Iterator[Product2[K, C]] = {
    if (handle.agg != GpuUcxShuffleManager.NO_AGG) {
      val sum = handle.agg == SgxNative.AGG_SUM
      val Array(groups, values) = SgxNative.readGrouped(engine, shuffleId, maps, startPartition, endPartition,
                                                        handle.agg, null, null, null)
      val keys = le(groups * 8); val starts = le(groups * 8); val vals = le(values * 8)
      SgxNative.readGrouped(engine, shuffleId, maps, startPartition, endPartition, handle.agg, keys, starts, vals)
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
      val bytes = if (sorted) SgxNative.readSorted(engine, shuffleId, maps, startPartition, endPartition, null)
                  else SgxNative.readRecords(engine, shuffleId, maps, startPartition, endPartition, null)
      val dst = le(bytes)
      if (sorted) SgxNative.readSorted(engine, shuffleId, maps, startPartition, endPartition, dst)
      else SgxNative.readRecords(engine, shuffleId, maps, startPartition, endPartition, dst)
      val recs = dst.asLongBuffer()
      Iterator.tabulate((bytes / 16).toInt)(i => (recs.get(2 * i), recs.get(2 * i + 1)).asInstanceOf[Product2[K, C]])
    }
  }

  /** Blocks (map, r) of the range from their owners, deserialized and aggregated on the CPU. */
  private def readRemote(maps: Array[Long], coord: GpuExchangeCoordinator): Iterator[Product2[K, C]] = {
    val owners = coord.rankRanges(shuffleId)
    val kryo = dep.serializer.isInstanceOf[KryoSerializer]
    val blocks = (startPartition until endPartition).iterator.flatMap { r =>
      val rank = owners.collectFirst { case (k, Array(a, b)) if a <= r && r < b => k }
        .getOrElse(throw new SgxFetchException(s"no executor holds reducer $r of shuffle $shuffleId"))
      val got = coord.fetchRemote(shuffleId, rank, maps, Array.fill(maps.length)(r))
      var off = 0
      maps.indices.iterator.map { i =>
        val len = got.lengths(i).toInt
        val block = (ShuffleBlockId(shuffleId, maps(i), r), got.bytes, off, len)
        off += len
        block
      }
    }
    // empty blocks are never opened (Spark's fetcher drops zero-size blocks)
    val records: Iterator[Product2[Any, Any]] = blocks.filter(_._4 > 0).flatMap { case (id, bytes, off, len) =>
      if (kryo) {
        // Spark's own stream: LZ4 (spark.shuffle.compress) then the Kryo deserializer
        val wrapped = SparkEnv.get.serializerManager.wrapStream(id, new ByteArrayInputStream(bytes, off, len))
        dep.serializer.newInstance().deserializeStream(wrapped).asKeyValueIterator
      } else {
        // the engine's fixed 16 B codec: {key LE, value LE}
        val b = ByteBuffer.wrap(bytes, off, len).order(ByteOrder.LITTLE_ENDIAN)
        Iterator.fill(len / 16)((b.getLong, b.getLong))
      }
    }
    val aggregated: Iterator[Product2[K, C]] = dep.aggregator match {
      case Some(agg) if dep.mapSideCombine =>
        agg.combineCombinersByKey(records.asInstanceOf[Iterator[Product2[K, C]]], context)
      case Some(agg) =>
        agg.asInstanceOf[org.apache.spark.Aggregator[K, Any, C]]
          .combineValuesByKey(records.asInstanceOf[Iterator[Product2[K, Any]]], context)
      case None => records.asInstanceOf[Iterator[Product2[K, C]]]
    }
    dep.keyOrdering match {
      case Some(ord: Ordering[K @unchecked]) =>
        val sorter = new ExternalSorter[K, C, C](context, ordering = Some(ord), serializer = dep.serializer)
        sorter.insertAll(aggregated)
        CompletionIterator[Product2[K, C], Iterator[Product2[K, C]]](sorter.iterator, sorter.stop())
      case None => aggregated
    }
  }
}
