/*
 * GpuUcxShuffleManager — spark.shuffle.manager for the MI355X engine.  Keeps the reference's
 * plugin shape (spark_3_0/UcxShuffleManager.scala:25-80 over CommonUcxShuffleManager.scala:
 * 25-124: registerShuffle inherited from SortShuffleManager, getWriter / getReader dispatch,
 * unregisterShuffle, stop) and routes a dependency to the GPU only when the engine computes
 * exactly what Spark would:
 *   - (Long, Long) records: dep.keyClassName and dep.valueClassName are long / java.lang.Long
 *     (the engine's 16 B record codec; anything else would throw ClassCastException in the
 *     writer);
 *   - a HashPartitioner, or a RangePartitioner over Long keys;
 *   - no aggregator, or one DECLARED with spark.shuffle.ucx.gpu.aggregator.<shuffleId> =
 *     "sum" (reduceByKey(_ + _) on Longs: the GPU sums with wrap-around, map-side combine
 *     allowed) or "group" (groupByKey: mapSideCombine must be false).  Spark cannot look
 *     inside an aggregator's closures, so an undeclared one -- reduceByKey(math.max),
 *     combineByKey(...) -- stays on the CPU path instead of being guessed.
 * Everything else falls back to SortShuffleManager's own writer and reader.
 *
 *   - a compressed Kryo shuffle only with spark.io.compression.codec = lz4 (the GPU frames
 *     lz4-java's LZ4BlockOutputStream; Spark's own readers unwrap with the configured codec).
 *
 * registerShuffle runs on the DRIVER (the ShuffleDependency constructor calls it): it only
 * decides, and puts the decision and the engine registration (GpuShuffleSpec) in the handle.
 * Each executor registers the shuffle with its own engine on first use (getWriter / getReader,
 * or the shuffle's GpuRunExchange on an executor that runs none of its tasks), so the engine
 * -- one per executor = per GPU, spark.shuffle.ucx.gpu.device -- never exists on the driver.  The exchange world (RCCL communicator, the collective per shuffle) is set up and
 * driven by GpuExchangeCoordinator.
 */
package org.apache.spark.shuffle.ucx.gpu

import java.nio.{ByteBuffer, ByteOrder}

import org.apache.spark.{HashPartitioner, Partitioner, RangePartitioner, ShuffleDependency, SparkConf, TaskContext}
import org.apache.spark.io.CompressionCodec
import org.apache.spark.serializer.KryoSerializer
import org.apache.spark.shuffle._
import org.apache.spark.shuffle.sort.{SortShuffleManager, SortShuffleWriter}

/** Everything an executor's engine needs to register a GPU shuffle (sgx_register_shuffle and
 *  the dependency properties), decided once on the driver.  It travels in the handle and in
 *  every GpuRunExchange, so an executor that never ran a task of the shuffle registers it
 *  before joining the shuffle's collective (instead of failing it). */
case class GpuShuffleSpec(shuffleId: Int, numPartitions: Int, kind: Int, bounds: Array[Long], ascending: Boolean,
                          kryo: Boolean, lz4Block: Int, combineSum: Boolean, writerUnsafe: Boolean,
                          placementBytes: Boolean)

/** A shuffle the GPU runs: same fields as BaseShuffleHandle, plus the declared aggregation and
 *  the engine registration. */
class GpuShuffleHandle[K, V, C](shuffleId: Int, dependency: ShuffleDependency[K, V, C], val agg: Int,
                                val spec: GpuShuffleSpec)
  extends BaseShuffleHandle[K, V, C](shuffleId, dependency)

object GpuUcxShuffleManager {
  val NO_AGG: Int = -1
  private val LONG_CLASSES = Set("long", "java.lang.Long")

  /** RangePartitioner keeps rangeBounds and ascending in private fields: read them by reflection. */
  private[gpu] def rangeField[T](p: RangePartitioner[_, _], name: String): T = {
    val f = classOf[RangePartitioner[_, _]].getDeclaredFields
      .find(f => f.getName == name || f.getName.endsWith("$$" + name))
      .getOrElse(throw new UnsupportedOperationException(s"RangePartitioner has no field $name"))
    f.setAccessible(true)
    f.get(p).asInstanceOf[T]
  }
}

class GpuUcxShuffleManager(conf: SparkConf, isDriver: Boolean) extends SortShuffleManager(conf) {
  import GpuUcxShuffleManager._

  @volatile private var engineCreated = false
  private lazy val engine: Long = {
    val e = SgxNative.create(conf.getInt("spark.shuffle.ucx.gpu.device", 0),
                             conf.getInt("spark.shuffle.ucx.gpu.numChunks", 0), 0,
                             conf.getInt("spark.shuffle.ucx.gpu.commTimeoutMs", 0))
    engineCreated = true
    e
  }
  private[gpu] lazy val coordinator = new GpuExchangeCoordinator(conf, isDriver, () => engine, ensureRegistered)
  if (conf.getInt("spark.shuffle.ucx.gpu.numExecutors", conf.getInt("spark.executor.instances", 1)) > 1)
    coordinator  // start the world's setup (driver endpoint / executor join) right away
  private val registered = new java.util.concurrent.ConcurrentHashMap[Int, java.lang.Boolean]()

  /** The declared aggregation of a dependency, NO_AGG for none, None if the GPU cannot run it. */
  private def gpuAgg(shuffleId: Int, dep: ShuffleDependency[_, _, _]): Option[Int] =
    if (dep.aggregator.isEmpty) Some(NO_AGG)
    else conf.get("spark.shuffle.ucx.gpu.aggregator." + shuffleId, "") match {
      case "sum" => Some(SgxNative.AGG_SUM)
      case "group" if !dep.mapSideCombine => Some(SgxNative.AGG_GROUP)
      case _ => None
    }

  private def gpuPartitioner(p: Partitioner, dep: ShuffleDependency[_, _, _]): Boolean = p match {
    case _: HashPartitioner => true
    case _: RangePartitioner[_, _] => dep.keyOrdering.isDefined  // Long keys: checked by the class names
    case _ => false
  }

  /** A compressed Kryo shuffle is framed with lz4-java's LZ4BlockOutputStream on the GPU, and
   *  Spark's own readers (remote reads, SortShuffleManager fallbacks) unwrap blocks with
   *  spark.io.compression.codec: the GPU path needs that codec to be lz4. */
  private def codecIsLz4: Boolean =
    CompressionCodec.getShortName(conf.get("spark.io.compression.codec", CompressionCodec.DEFAULT_COMPRESSION_CODEC)) ==
      "lz4"

  override def registerShuffle[K, V, C](shuffleId: Int, dependency: ShuffleDependency[K, V, C]): ShuffleHandle = {
    val longs = LONG_CLASSES(dependency.keyClassName) && LONG_CLASSES(dependency.valueClassName)
    val kryo = dependency.serializer.isInstanceOf[KryoSerializer]
    val codecOk = !kryo || !conf.getBoolean("spark.shuffle.compress", true) || codecIsLz4
    val agg = if (longs && codecOk && gpuPartitioner(dependency.partitioner, dependency)) gpuAgg(shuffleId, dependency)
              else None
    agg match {
      case Some(a) => new GpuShuffleHandle(shuffleId, dependency, a, specOf(shuffleId, dependency, a))
      case None => super.registerShuffle(shuffleId, dependency)
    }
  }

  /** Driver side: the engine registration of a GPU shuffle. */
  private def specOf(shuffleId: Int, dep: ShuffleDependency[_, _, _], agg: Int): GpuShuffleSpec = {
    val kryo = dep.serializer.isInstanceOf[KryoSerializer]
    val (kind, bounds, asc) = dep.partitioner match {
      case _: HashPartitioner => (SgxNative.PART_HASH, Array.empty[Long], true)
      case p: RangePartitioner[_, _] =>
        (SgxNative.PART_RANGE_I64, rangeField[Array[_]](p, "rangeBounds").map(_.asInstanceOf[Long]),
         rangeField[Boolean](p, "ascending"))
    }
    GpuShuffleSpec(
      shuffleId, dep.partitioner.numPartitions, kind, bounds, asc, kryo,
      if (kryo && conf.getBoolean("spark.shuffle.compress", true))
        conf.getSizeAsBytes("spark.io.compression.lz4.blockSize", "32k").toInt
      else 0,
      dep.mapSideCombine && agg == SgxNative.AGG_SUM,
      // the writer Spark's own handle would run (SortShuffleManager.registerShuffle; the
      // reference's getWriter, spark_3_0/UcxShuffleManager.scala:32-53): UnsafeShuffleWriter for
      // a SerializedShuffleHandle, whose fast spill merge keeps each spill's partition segment
      // as its own LZ4 stream (the batches GpuShuffleWriter appends are its spills)
      !SortShuffleWriter.shouldBypassMergeSort(conf, dep) && SortShuffleManager.canUseSerializedShuffle(dep) &&
        conf.getBoolean("spark.shuffle.unsafe.fastMergeEnabled", true),
      // reducer placement, fixed by the shuffle's first exchange: "even" (floor(r*P/R)) or
      // "bytes" (ranges balanced on the lengths, for skewed keys)
      conf.get("spark.shuffle.ucx.gpu.reducerPlacement", "even") == "bytes")
  }

  /** Executor side, once per shuffle: the shuffle's partitioner, serializer, codec, combine,
   *  map writer and reducer placement in this executor's engine -- from a task's handle, or
   *  from a GpuRunExchange on an executor that has not run a task of the shuffle yet. */
  private[gpu] def ensureRegistered(sp: GpuShuffleSpec): Unit = {
    if (registered.containsKey(sp.shuffleId)) return
    registered.synchronized {  // handles are per-task copies: lock the executor's table
      if (registered.containsKey(sp.shuffleId)) return
      if (sp.kind == SgxNative.PART_HASH) {
        SgxNative.registerShuffle(engine, sp.shuffleId, sp.numPartitions, SgxNative.PART_HASH, null, 0, true, 16)
      } else {
        val b = ByteBuffer.allocateDirect(math.max(8, sp.bounds.length * 8)).order(ByteOrder.LITTLE_ENDIAN)
        sp.bounds.foreach(b.putLong)
        SgxNative.registerShuffle(engine, sp.shuffleId, sp.numPartitions, sp.kind, b, sp.bounds.length, sp.ascending, 16)
      }
      if (sp.kryo) {
        SgxNative.setSerializer(engine, sp.shuffleId, SgxNative.SER_KRYO)
        if (sp.lz4Block > 0) SgxNative.setCompression(engine, sp.shuffleId, SgxNative.CODEC_LZ4, sp.lz4Block)
      }
      if (sp.combineSum) SgxNative.setMapSideCombine(engine, sp.shuffleId, SgxNative.AGG_SUM)
      if (sp.writerUnsafe) SgxNative.setMapWriter(engine, sp.shuffleId, SgxNative.WRITER_UNSAFE)
      if (sp.placementBytes) SgxNative.setReducerPlacement(engine, sp.shuffleId, SgxNative.PLACE_BYTES)
      registered.put(sp.shuffleId, true)
    }
  }

  private def ensureRegistered(h: GpuShuffleHandle[_, _, _]): Unit = ensureRegistered(h.spec)

  override def getWriter[K, V](handle: ShuffleHandle, mapId: Long, context: TaskContext,
                               metrics: ShuffleWriteMetricsReporter): ShuffleWriter[K, V] = handle match {
    case h: GpuShuffleHandle[K @unchecked, V @unchecked, _] =>
      ensureRegistered(h)
      new GpuShuffleWriter[K, V](engine, h, mapId, conf, shuffleBlockResolver, metrics)
    case _ => super.getWriter(handle, mapId, context, metrics)
  }

  override def getReader[K, C](handle: ShuffleHandle, startPartition: Int, endPartition: Int,
                               context: TaskContext, metrics: ShuffleReadMetricsReporter): ShuffleReader[K, C] =
    handle match {
      case h: GpuShuffleHandle[K @unchecked, _, C @unchecked] =>
        ensureRegistered(h)
        new GpuShuffleReader[K, C](engine, h, startPartition, endPartition, context,
                                   if (isWorld) Some(coordinator) else None, metrics)
      case _ => super.getReader(handle, startPartition, endPartition, context, metrics)
    }

  /** Spark 3.0's AQE local shuffle reader reads a map range (startMapIndex, endMapIndex) of a
   *  partition range.  The reference does not override it, so its local reads bypass UCX
   *  (SURVEY §8(b)); here a GPU shuffle's map outputs live in HBM (index files only with
   *  spark.shuffle.ucx.gpu.writeIndexFiles), so the range read goes through the same GPU reader
   *  restricted to those maps. */
  override def getReaderForRange[K, C](handle: ShuffleHandle, startMapIndex: Int, endMapIndex: Int,
                                       startPartition: Int, endPartition: Int, context: TaskContext,
                                       metrics: ShuffleReadMetricsReporter): ShuffleReader[K, C] =
    handle match {
      case h: GpuShuffleHandle[K @unchecked, _, C @unchecked] =>
        ensureRegistered(h)
        new GpuShuffleReader[K, C](engine, h, startPartition, endPartition, context,
                                   if (isWorld) Some(coordinator) else None, metrics,
                                   Some((startMapIndex, endMapIndex)))
      case _ => super.getReaderForRange(handle, startMapIndex, endMapIndex, startPartition, endPartition, context,
                                        metrics)
    }

  private def isWorld: Boolean =
    conf.getInt("spark.shuffle.ucx.gpu.numExecutors", conf.getInt("spark.executor.instances", 1)) > 1

  override def unregisterShuffle(shuffleId: Int): Boolean = {
    if (registered.remove(shuffleId) != null) SgxNative.unregisterShuffle(engine, shuffleId)
    super.unregisterShuffle(shuffleId)
  }

  override def stop(): Unit = {
    if (isWorld) coordinator.stop()
    if (engineCreated) SgxNative.destroy(engine)
    super.stop()
  }
}
