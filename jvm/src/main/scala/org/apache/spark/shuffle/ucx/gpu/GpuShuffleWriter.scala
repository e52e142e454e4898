/*
 * GpuShuffleWriter — what GpuUcxShuffleManager.getWriter returns for a GPU shuffle
 * (replaces the SortShuffleWriter + NvkvShuffleMapOutputWriter pair the reference builds at
 * spark_3_0/UcxShuffleManager.scala:48-51 and ucx/NvkvShuffleMapOutputWriter.scala:105-148).
 * Records are packed as 16 B {key LE, value LE} into a direct buffer and handed to the engine
 * batch by batch (SgxNative.mapAppend: the batches are Spark's spills, merged in order at
 * mapCommit); the partition id, histogram, scan, stable scatter, Kryo framing and LZ4 run on
 * the GPU and the map output stays in HBM.  commitAllPartitions' long[] is mapCommit's return
 * value, reported to the MapOutputTracker in the MapStatus.
 *
 * Index + data files: the reference's active writer never writes them either (its bytes go to
 * the DPU's NVKV store, NvkvShuffleMapOutputWriter.scala:115-148 commits no index).  With
 * spark.shuffle.ucx.gpu.writeIndexFiles=true the map output is also committed through
 * IndexShuffleBlockResolver's layout (SgxNative.writeIndex -> sgx_write_index: data file +
 * (R+1) big-endian offsets, tmp + rename, "an existing valid attempt wins",
 * IndexShuffleBlockResolver.scala:161-217), for external tools or a CPU reader; the lengths it
 * returns (the winning attempt's) are the ones reported.
 */
package org.apache.spark.shuffle.ucx.gpu

import java.io.File
import java.nio.{ByteBuffer, ByteOrder}

import org.apache.spark.{SparkConf, SparkEnv}
import org.apache.spark.scheduler.MapStatus
import org.apache.spark.shuffle.{BaseShuffleHandle, IndexShuffleBlockResolver, ShuffleBlockResolver,
  ShuffleWriteMetricsReporter, ShuffleWriter}
import org.apache.spark.storage.ShuffleIndexBlockId

class GpuShuffleWriter[K, V](engine: Long, handle: BaseShuffleHandle[K, V, _], mapId: Long, conf: SparkConf,
                             resolver: ShuffleBlockResolver, metrics: ShuffleWriteMetricsReporter,
                             batchRecords: Int = 1 << 22) extends ShuffleWriter[K, V] {
  private val shuffleId = handle.shuffleId
  private val numPartitions = handle.dependency.partitioner.numPartitions
  private var mapStatus: MapStatus = _

  override def write(records: Iterator[Product2[K, V]]): Unit = {
    val buf = ByteBuffer.allocateDirect(batchRecords * 16).order(ByteOrder.LITTLE_ENDIAN)
    SgxNative.mapBegin(engine, shuffleId, mapId)
    var n = 0L
    var total = 0L
    def flush(): Unit = {
      if (n > 0) SgxNative.mapAppend(engine, shuffleId, mapId, buf, n, 16)
      total += n
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
    var lengths = SgxNative.mapCommit(engine, shuffleId, mapId, numPartitions)
    if (conf.getBoolean("spark.shuffle.ucx.gpu.writeIndexFiles", false)) {
      val r = resolver.asInstanceOf[IndexShuffleBlockResolver]
      val data = r.getDataFile(shuffleId, mapId)
      // the index file sits next to the data file, named as Spark names it
      val index = new File(data.getParentFile, ShuffleIndexBlockId(shuffleId, mapId, 0).name)
      lengths = SgxNative.writeIndex(engine, shuffleId, mapId, index.getPath, data.getPath, numPartitions)
    }
    metrics.incRecordsWritten(total)
    metrics.incBytesWritten(lengths.sum)
    mapStatus = MapStatus(SparkEnv.get.blockManager.shuffleServerId, lengths, mapId)
  }

  override def stop(success: Boolean): Option[MapStatus] = if (success) Option(mapStatus) else None
}
