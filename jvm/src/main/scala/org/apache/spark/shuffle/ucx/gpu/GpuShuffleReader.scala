/*
 * GpuShuffleReader — UcxShuffleReader.read (spark_3_0/UcxShuffleReader.scala:74-200) for a
 * (Long, Long) dependency, with the work after the fetch done on the GPU:
 *   aggregator sum (reduceByKey: combineValuesByKey, or combineCombinersByKey after a
 *     map-side combine, :155-164)          -> SgxNative.readGrouped(AGG_SUM)
 *   aggregator group (groupByKey)          -> SgxNative.readGrouped(AGG_GROUP)
 *   keyOrdering (sortByKey, :166-181)      -> SgxNative.readSorted
 *   neither (deserializeStream, :137-145)  -> SgxNative.readRecords
 * The blocks come from the maps the MapOutputTracker lists for [startPartition,
 * endPartition) (:75-76), in map order: the canonical per-reducer sequence.
 */
package org.apache.spark.shuffle.ucx.gpu

import java.nio.{ByteBuffer, ByteOrder}

import org.apache.spark.{SparkEnv, TaskContext}
import org.apache.spark.shuffle.{BaseShuffleHandle, ShuffleReader}

class GpuShuffleReader[K, C](engine: Long, handle: BaseShuffleHandle[K, _, C], startPartition: Int,
                             endPartition: Int, context: TaskContext,
                             sumAggregator: Boolean) extends ShuffleReader[K, C] {
  private val dep = handle.dependency
  private val shuffleId = handle.shuffleId

  private def mapIds: Array[Long] =
    SparkEnv.get.mapOutputTracker
      .getMapSizesByExecutorId(shuffleId, startPartition, endPartition)
      .flatMap(_._2.map(_._1.asInstanceOf[org.apache.spark.storage.ShuffleBlockId].mapId))
      .toArray.distinct.sorted

  private def le(n: Long): ByteBuffer = ByteBuffer.allocateDirect(math.max(8L, n).toInt).order(ByteOrder.LITTLE_ENDIAN)

  override def read(): Iterator[Product2[K, C]] = {
    val maps = mapIds
    if (dep.aggregator.isDefined) {
      val agg = if (sumAggregator) SgxNative.AGG_SUM else SgxNative.AGG_GROUP
      val Array(groups, values) = SgxNative.readGrouped(engine, shuffleId, maps, startPartition, endPartition, agg,
                                                        null, null, null)
      val keys = le(groups * 8); val starts = le(groups * 8); val vals = le(values * 8)
      SgxNative.readGrouped(engine, shuffleId, maps, startPartition, endPartition, agg, keys, starts, vals)
      val k = keys.asLongBuffer(); val s = starts.asLongBuffer(); val v = vals.asLongBuffer()
      if (sumAggregator) {
        Iterator.tabulate(groups.toInt)(g => (k.get(g), v.get(g)).asInstanceOf[Product2[K, C]])
      } else {
        Iterator.tabulate(groups.toInt) { g =>
          val end = if (g + 1 < groups) s.get(g + 1) else values
          val buf = (s.get(g) until end).map(i => v.get(i.toInt))
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
}
