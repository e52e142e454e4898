/*
 * GpuShuffleWriter — what GpuUcxShuffleManager.getWriter returns for a (Long, Long)
 * dependency (replaces the SortShuffleWriter + NvkvShuffleMapOutputWriter pair the
 * reference builds at spark_3_0/UcxShuffleManager.scala:48-51 and
 * ucx/NvkvShuffleMapOutputWriter.scala:105-148).  Records are packed as 16 B {key LE,
 * value LE} into a pinned direct buffer and handed to the engine batch by batch
 * (SgxNative.mapAppend: the batches are Spark's spills, merged in order at mapCommit); the
 * partition id, histogram, scan, stable scatter, Kryo framing and LZ4 run on the GPU and the
 * map output stays in HBM.  commitAllPartitions' long[] is mapCommit's return value.
 */
package org.apache.spark.shuffle.ucx.gpu

import java.nio.{ByteBuffer, ByteOrder}

import org.apache.spark.SparkEnv
import org.apache.spark.scheduler.MapStatus
import org.apache.spark.shuffle.{BaseShuffleHandle, ShuffleWriter}

class GpuShuffleWriter[K, V](engine: Long, handle: BaseShuffleHandle[K, V, _], mapId: Long,
                             batchRecords: Int = 1 << 22) extends ShuffleWriter[K, V] {
  private val shuffleId = handle.shuffleId
  private val numPartitions = handle.dependency.partitioner.numPartitions
  private var mapStatus: MapStatus = _

  override def write(records: Iterator[Product2[K, V]]): Unit = {
    val buf = ByteBuffer.allocateDirect(batchRecords * 16).order(ByteOrder.LITTLE_ENDIAN)
    SgxNative.mapBegin(engine, shuffleId, mapId)
    var n = 0L
    def flush(): Unit = {
      if (n > 0) SgxNative.mapAppend(engine, shuffleId, mapId, buf, n, 16)
      buf.clear()
      n = 0
    }
    while (records.hasNext) {
      val r = records.next()
      buf.putLong(r._1.asInstanceOf[Long]).putLong(r._2.asInstanceOf[Long])
      n += 1
      if (n == batchRecords) flush()
    }
    flush()
    val lengths = SgxNative.mapCommit(engine, shuffleId, mapId, numPartitions)
    mapStatus = MapStatus(SparkEnv.get.blockManager.shuffleServerId, lengths, mapId)
  }

  override def stop(success: Boolean): Option[MapStatus] = if (success) Option(mapStatus) else None
}
