/*
 * GpuUcxShuffleManager — spark.shuffle.manager for the MI355X engine.  Keeps the reference's
 * plugin shape (spark_3_0/UcxShuffleManager.scala:25-80 over CommonUcxShuffleManager.scala:
 * 25-124: registerShuffle inherited from SortShuffleManager, getWriter / getReader dispatch,
 * unregisterShuffle, stop) and routes (Long, Long) dependencies with a hash or range
 * partitioner to the GPU; anything else falls back to SortShuffleManager's own writer and
 * reader.  One engine per executor (= per GPU: the executor's GPU ordinal in
 * spark.shuffle.ucx.gpu.device); the RCCL id of the exchange travels over
 * SgxNative.bootstrapServe / bootstrapJoin (or Spark RPC), replacing ExecutorAdded /
 * IntroduceAllExecutors.
 */
package org.apache.spark.shuffle.ucx.gpu

import java.nio.{ByteBuffer, ByteOrder}

import org.apache.spark.{HashPartitioner, RangePartitioner, ShuffleDependency, SparkConf, TaskContext}
import org.apache.spark.serializer.KryoSerializer
import org.apache.spark.shuffle._
import org.apache.spark.shuffle.sort.SortShuffleManager

class GpuUcxShuffleManager(conf: SparkConf, isDriver: Boolean) extends SortShuffleManager(conf) {
  private lazy val engine: Long = SgxNative.create(conf.getInt("spark.shuffle.ucx.gpu.device", 0),
    conf.getInt("spark.shuffle.ucx.gpu.numChunks", 0), 0, conf.getInt("spark.shuffle.ucx.gpu.commTimeoutMs", 0))
  private val onGpu = new java.util.concurrent.ConcurrentHashMap[Int, java.lang.Boolean]()

  private def isLongSum(dep: ShuffleDependency[_, _, _]): Boolean =
    dep.aggregator.exists(a => conf.get("spark.shuffle.ucx.gpu.sumAggregator." + dep.shuffleId, "false") == "true")

  override def registerShuffle[K, V, C](shuffleId: Int, dependency: ShuffleDependency[K, V, C]): ShuffleHandle = {
    val handle = super.registerShuffle(shuffleId, dependency)
    val gpu = dependency.partitioner match {
      case p: HashPartitioner =>
        SgxNative.registerShuffle(engine, shuffleId, p.numPartitions, SgxNative.PART_HASH, null, 0, true, 16)
        true
      case p: RangePartitioner[_, _] if dependency.keyOrdering.isDefined =>
        val bounds = p.rangeBounds.asInstanceOf[Array[Long]]
        val b = ByteBuffer.allocateDirect(math.max(8, bounds.length * 8)).order(ByteOrder.LITTLE_ENDIAN)
        bounds.foreach(b.putLong)
        SgxNative.registerShuffle(engine, shuffleId, p.numPartitions, SgxNative.PART_RANGE_I64, b, bounds.length,
                                  p.ascending, 16)
        true
      case _ => false
    }
    if (gpu) {
      if (dependency.serializer.isInstanceOf[KryoSerializer]) {
        SgxNative.setSerializer(engine, shuffleId, SgxNative.SER_KRYO)
        if (conf.getBoolean("spark.shuffle.compress", true))
          SgxNative.setCompression(engine, shuffleId, SgxNative.CODEC_LZ4,
                                   conf.getSizeAsBytes("spark.io.compression.lz4.blockSize", "32k").toInt)
      }
      if (dependency.mapSideCombine) SgxNative.setMapSideCombine(engine, shuffleId, SgxNative.AGG_SUM)
      // reducer placement of the exchange rounds: "even" (floor(r*P/R)) or "bytes" (ranges
      // balanced on the round's lengths, for skewed keys); the executor's range of a round
      // comes back from SgxNative.roundReducers for the scheduler's locality preferences
      if (conf.get("spark.shuffle.ucx.gpu.reducerPlacement", "even") == "bytes")
        SgxNative.setReducerPlacement(engine, shuffleId, SgxNative.PLACE_BYTES)
      onGpu.put(shuffleId, true)
    }
    handle
  }

  override def getWriter[K, V](handle: ShuffleHandle, mapId: Long, context: TaskContext,
                               metrics: ShuffleWriteMetricsReporter): ShuffleWriter[K, V] =
    if (onGpu.containsKey(handle.shuffleId))
      new GpuShuffleWriter[K, V](engine, handle.asInstanceOf[BaseShuffleHandle[K, V, _]], mapId)
    else super.getWriter(handle, mapId, context, metrics)

  override def getReader[K, C](handle: ShuffleHandle, startPartition: Int, endPartition: Int,
                               context: TaskContext, metrics: ShuffleReadMetricsReporter): ShuffleReader[K, C] =
    if (onGpu.containsKey(handle.shuffleId)) {
      val h = handle.asInstanceOf[BaseShuffleHandle[K, _, C]]
      new GpuShuffleReader[K, C](engine, h, startPartition, endPartition, context, isLongSum(h.dependency))
    } else super.getReader(handle, startPartition, endPartition, context, metrics)

  override def unregisterShuffle(shuffleId: Int): Boolean = {
    if (onGpu.remove(shuffleId) != null) SgxNative.unregisterShuffle(engine, shuffleId)
    super.unregisterShuffle(shuffleId)
  }

  override def stop(): Unit = {
    SgxNative.destroy(engine)
    super.stop()
  }
}
