/*
 * GpuExchangeCoordinator — who calls the collective, and when.
 *
 * The engine's exchange (SgxNative.exchange -> sgx_exchange(e, shuffleId)) is a collective:
 * every executor of the exchange world must call it, in the same order, once its map tasks
 * of the shuffle are committed.  Spark has no such step -- the reference fetches every
 * block on demand, one UCX Active Message per block (spark_3_0/UcxShuffleReader.scala:74-103,
 * spark_3_0/UcxShuffleClient.scala:17-47, ucx/UcxWorkerWrapper.scala:96-186) -- so this
 * class adds one, over Spark RPC, shaped like the reference's rpc/ package
 * (rpc/UcxDriverRpcEndpoint.scala:21-42, rpc/UcxExecutorRpcEndpoint.scala:19-39):
 *
 *  1. World: each executor asks the driver to join (GpuExecutorJoin); the driver assigns
 *     ranks in join order and answers with the rank, the world size
 *     (spark.shuffle.ucx.gpu.numExecutors, default spark.executor.instances) and rank 0's
 *     host.  Rank 0 serves a fresh RCCL unique id on spark.shuffle.ucx.gpu.bootstrapPort
 *     (SgxNative.bootstrapServe), the others fetch it (bootstrapJoin), and every executor
 *     runs SgxNative.commInit -- all on the executor's one "comm" thread, so nothing else
 *     reaches the communicator before it exists.
 *  2. Exchange: the first reduce task of a shuffle on any executor (GpuShuffleReader.read)
 *     sends GpuExchangeRequest(shuffleId, the shuffle's full map id set as the
 *     MapOutputTracker lists it over ALL partitions, the shuffle's GpuShuffleSpec) to the
 *     driver and waits.  A reduce task only starts once its map stage has completed, so every
 *     executor's maps of those ids are committed by then, and every reduce task of the stage
 *     computes the same key (not its own range's non-empty blocks).  The driver
 *     de-duplicates (one exchange per shuffle and map set: a re-run map stage has new map ids
 *     and gets a new round with just the new maps) and sends GpuRunExchange to EVERY
 *     executor, in one global sequence (the driver endpoint is single-threaded; Spark RPC
 *     keeps a sender's messages to one receiver in order).  Each executor registers the
 *     shuffle from the spec if no task of it ran there yet, then runs SgxNative.exchange +
 *     SgxNative.sync on its comm thread, in that order, and completes the waiting readers.
 *     A rank that fails locally still joins the collective's first all-gather with an error
 *     mark (sgx_exchange), so all ranks fail the round together; each reports
 *     GpuExchangeFailed and the driver forgets the round, so a retried task starts a new one.
 *  3. Reads outside this executor's reducers (Spark placed the reduce task elsewhere):
 *     GpuShuffleReader asks the owners for the raw blocks over RPC (GpuFetchRemote, served
 *     from their HBM by SgxNative.fetchBlocks) and reads them on the CPU with Spark's own
 *     serializer, aggregator and sorter -- the reference's "any block from anywhere"
 *     contract, at RPC speed.  Owner-local reads are the fast path.
 *
 * The world is fixed for the application (like the RCCL communicator it builds): executors
 * lost or added under dynamic allocation are out of scope (INTEGRATION.md).
 */
package org.apache.spark.shuffle.ucx.gpu

import java.nio.ByteBuffer
import java.util.concurrent.{ConcurrentHashMap, TimeUnit}

import scala.collection.mutable
import scala.concurrent.{Await, Promise}
import scala.concurrent.duration.Duration

import org.apache.spark.{SparkConf, SparkEnv}
import org.apache.spark.internal.Logging
import org.apache.spark.rpc.{RpcCallContext, RpcEndpointRef, RpcEnv, ThreadSafeRpcEndpoint}
import org.apache.spark.util.{RpcUtils, ThreadUtils}

object GpuRpcMessages {
  /** executor -> driver (ask): join the exchange world; reply GpuRankAssigned. */
  case class GpuExecutorJoin(executorId: String, host: String, endpoint: RpcEndpointRef)
  case class GpuRankAssigned(rank: Int, nranks: Int, rootHost: String)
  /** executor -> driver (send): a reader needs shuffleId exchanged over this full map set. */
  case class GpuExchangeRequest(shuffleId: Int, maps: Seq[Long], spec: GpuShuffleSpec)
  /** driver -> every executor (send), one global sequence: run attempt `attempt` of the
   *  exchange now. */
  case class GpuRunExchange(shuffleId: Int, maps: Seq[Long], spec: GpuShuffleSpec, attempt: Int)
  /** executor -> driver (send): that attempt failed here; a new request starts a new round
   *  (a late report of an older attempt never cancels a newer one). */
  case class GpuExchangeFailed(shuffleId: Int, maps: Seq[Long], attempt: Int)
  /** executor -> driver (ask): every rank's endpoint; reply GpuPeers. */
  case object GpuPeersRequest
  case class GpuPeers(endpoints: Map[Int, RpcEndpointRef])
  /** executor -> executor (ask): the asked executor's reducer range of a shuffle (int[2]). */
  case class GpuRangeRequest(shuffleId: Int)
  /** executor -> executor (ask): raw blocks (map, reducer) the asker does not hold. */
  case class GpuFetchRemote(shuffleId: Int, mapIds: Array[Long], reduceIds: Array[Int])
  case class GpuRemoteBlocks(bytes: Array[Byte], lengths: Array[Long])
}

import GpuRpcMessages._

/** Driver side: rank assignment and the global exchange sequence. */
class GpuDriverEndpoint(override val rpcEnv: RpcEnv, nranks: Int) extends ThreadSafeRpcEndpoint with Logging {
  private val ranks = mutable.LinkedHashMap.empty[String, (Int, RpcEndpointRef)]
  private var rootHost: String = _
  private val done = mutable.HashMap.empty[(Int, Seq[Long]), Int]      // key -> attempt broadcast
  private val attempts = mutable.HashMap.empty[(Int, Seq[Long]), Int]

  override def receiveAndReply(context: RpcCallContext): PartialFunction[Any, Unit] = {
    case GpuExecutorJoin(execId, host, ep) =>
      val rank = ranks.get(execId).map(_._1).getOrElse {
        if (ranks.size >= nranks)
          throw new IllegalStateException(s"exchange world of $nranks executors is full (executor $execId)")
        ranks.size
      }
      ranks(execId) = (rank, ep)
      if (rank == 0) rootHost = host
      context.reply(GpuRankAssigned(rank, nranks, rootHost))
    case GpuPeersRequest =>
      context.reply(GpuPeers(ranks.values.map { case (r, ep) => r -> ep }.toMap))
  }

  override def receive: PartialFunction[Any, Unit] = {
    case GpuExchangeRequest(shuffleId, maps, spec) =>
      val key = (shuffleId, maps)
      if (!done.contains(key)) {
        val a = attempts.getOrElse(key, 0) + 1
        attempts(key) = a
        done(key) = a
        logInfo(s"exchange of shuffle $shuffleId (${maps.size} maps, attempt $a) on ${ranks.size} executors")
        // every rank, the same order: ranks in rank order, requests in arrival order
        ranks.values.toSeq.sortBy(_._1).foreach { case (_, ep) => ep.send(GpuRunExchange(shuffleId, maps, spec, a)) }
      }
    case GpuExchangeFailed(shuffleId, maps, attempt) =>
      if (done.get((shuffleId, maps)).contains(attempt)) done.remove((shuffleId, maps))
  }
}

/** Executor side: the communicator, the exchanges (on one comm thread) and remote blocks. */
class GpuExecutorEndpoint(override val rpcEnv: RpcEnv, engine: Long, coordinator: GpuExchangeCoordinator)
    extends ThreadSafeRpcEndpoint with Logging {
  override def receive: PartialFunction[Any, Unit] = {
    case GpuRunExchange(shuffleId, maps, spec, attempt) => coordinator.runExchange(shuffleId, maps, spec, attempt)
  }

  override def receiveAndReply(context: RpcCallContext): PartialFunction[Any, Unit] = {
    case GpuRangeRequest(shuffleId) =>
      context.reply(SgxNative.shuffleReducers(engine, shuffleId))
    case GpuFetchRemote(shuffleId, mapIds, reduceIds) =>
      val sizes = SgxNative.fetchBlocks(engine, shuffleId, mapIds, reduceIds, null)  // size query
      val total = sizes.sum
      if (total > Int.MaxValue - 1024)
        throw new IllegalArgumentException(s"remote fetch of $total bytes: split the request")
      val dst = ByteBuffer.allocateDirect(math.max(1L, total).toInt)
      SgxNative.fetchBlocks(engine, shuffleId, mapIds, reduceIds, dst)
      val out = new Array[Byte](total.toInt)
      dst.get(out)
      context.reply(GpuRemoteBlocks(out, sizes))
  }
}

class GpuExchangeCoordinator(conf: SparkConf, isDriver: Boolean, engine: () => Long,
                             register: GpuShuffleSpec => Unit) extends Logging {
  private val driverName = "SgxGpuShuffle_driver"
  private val nranks = conf.getInt("spark.shuffle.ucx.gpu.numExecutors", conf.getInt("spark.executor.instances", 1))
  private val port = conf.getInt("spark.shuffle.ucx.gpu.bootstrapPort", 13380)
  private val timeoutMs = conf.getInt("spark.shuffle.ucx.gpu.commTimeoutMs", 300000)
  // one thread runs commInit and every exchange, in message order
  private val comm = ThreadUtils.newDaemonSingleThreadExecutor("sgx-comm")
  private val exchanges = new ConcurrentHashMap[(Int, Seq[Long]), Promise[Unit]]()
  @volatile private var driverRef: RpcEndpointRef = _
  @volatile private var peers: Map[Int, RpcEndpointRef] = Map.empty
  private val ranges = new ConcurrentHashMap[(Int, Int), Array[Int]]()
  private val mapSets = new ConcurrentHashMap[Int, (Long, Array[Long])]()
  private val setup = Promise[Unit]()

  comm.submit(new Runnable {
    override def run(): Unit = try {
      while (SparkEnv.get == null) Thread.sleep(10)
      val env = SparkEnv.get
      if (isDriver) {
        env.rpcEnv.setupEndpoint(driverName, new GpuDriverEndpoint(env.rpcEnv, nranks))
      } else {
        while (env.blockManager.blockManagerId == null) Thread.sleep(5)
        val bm = env.blockManager.blockManagerId
        val me = env.rpcEnv.setupEndpoint(s"sgx-gpu-executor-${bm.executorId}",
                                          new GpuExecutorEndpoint(env.rpcEnv, engine(), GpuExchangeCoordinator.this))
        driverRef = RpcUtils.makeDriverRef(driverName, conf, env.rpcEnv)
        val a = driverRef.askSync[GpuRankAssigned](GpuExecutorJoin(bm.executorId, bm.host, me))
        val id = if (a.rank == 0) {
          val uid = SgxNative.uniqueId()
          // serve the id while this thread joins the communicator (commInit is collective)
          val server = new Thread(new Runnable {
            override def run(): Unit = SgxNative.bootstrapServe(port, a.nranks, uid, timeoutMs)
          }, "sgx-bootstrap")
          server.setDaemon(true)
          server.start()
          uid
        } else {
          SgxNative.bootstrapJoin(a.rootHost, port, a.rank, timeoutMs, new Array[Int](1))
        }
        SgxNative.commInit(engine(), a.nranks, a.rank, id)
        logInfo(s"GPU shuffle exchange world: rank ${a.rank} of ${a.nranks}")
      }
      setup.success(())
    } catch {
      case t: Throwable =>
        logError("GPU shuffle exchange setup failed", t)
        setup.failure(t)
    }
  })

  private def promise(key: (Int, Seq[Long])): Promise[Unit] = {
    val p = Promise[Unit]()
    val prev = exchanges.putIfAbsent(key, p)
    if (prev == null) p else prev
  }

  /** Called by GpuExecutorEndpoint for GpuRunExchange: queue the collective on the comm thread. */
  private[gpu] def runExchange(shuffleId: Int, maps: Seq[Long], spec: GpuShuffleSpec, attempt: Int): Unit = {
    val key = (shuffleId, maps)
    val p = promise(key)
    comm.submit(new Runnable {
      override def run(): Unit = try {
        try register(spec)  // an executor that ran no task of the shuffle still takes part
        catch {
          case t: Throwable =>
            // the round's collective still needs this executor: join its first all-gather
            // marked failed, so every rank fails the round now (sgx_exchange_fail)
            try SgxNative.exchangeFail(engine(), spec.numPartitions) catch { case _: Throwable => }
            throw t
        }
        SgxNative.exchange(engine(), shuffleId)
        SgxNative.sync(engine())
        p.trySuccess(())
      } catch {
        case t: Throwable =>
          // the report goes out BEFORE the promise is dropped: a reader of this executor that
          // asks again only finds no promise after the driver has the failure (Spark RPC keeps
          // one sender's messages to one receiver in order), so its GpuExchangeRequest starts
          // a new round instead of being dropped as a duplicate of the failed one
          driverRef.send(GpuExchangeFailed(shuffleId, maps, attempt))
          exchanges.remove(key, p)  // a later task may ask again
          p.tryFailure(t)
      }
    })
  }

  /** A reader's barrier: the shuffle's exchange over its full map set `allMaps` (sorted) has
   *  completed on this executor. */
  def awaitExchange(shuffleId: Int, allMaps: Array[Long], spec: GpuShuffleSpec): Unit = {
    Await.result(setup.future, Duration(timeoutMs, TimeUnit.MILLISECONDS))
    val maps: Seq[Long] = allMaps.toVector
    val key = (shuffleId, maps)
    val p = promise(key)
    if (!p.isCompleted) driverRef.send(GpuExchangeRequest(shuffleId, maps, spec))
    // A failed round has already dropped its promise (runExchange).  A timeout keeps it: the
    // round may only be slow (queued behind another exchange on the comm thread), and the
    // driver holds the key as broadcast, so a fresh promise would never be completed; the
    // next reader waits on this one, which the comm thread still completes.
    try Await.result(p.future, Duration(timeoutMs, TimeUnit.MILLISECONDS))
    catch {
      case t: Throwable =>
        throw new SgxFetchException(s"exchange of shuffle $shuffleId failed: ${t.getMessage}")
    }
  }

  /** The shuffle's full map id set for one map-output epoch, computed by the first reduce task
   *  of the executor that asks and reused by the others (listing every partition's blocks
   *  costs M x R tuples per call).  A new epoch (a map stage re-ran) recomputes it. */
  def allMapIds(shuffleId: Int, epoch: Long, compute: => Array[Long]): Array[Long] = {
    val cached = mapSets.get(shuffleId)
    if (cached != null && cached._1 == epoch) cached._2
    else {
      val ids = compute
      mapSets.put(shuffleId, (epoch, ids))
      ids
    }
  }

  /** [r0, r1) of every rank for a shuffle (asked once, cached): the owners of remote reads. */
  def rankRanges(shuffleId: Int): Map[Int, Array[Int]] = {
    if (peers.size < nranks) peers = driverRef.askSync[GpuPeers](GpuPeersRequest).endpoints
    peers.map { case (rank, ep) =>
      val r = ranges.computeIfAbsent((shuffleId, rank), _ => ep.askSync[Array[Int]](GpuRangeRequest(shuffleId)))
      rank -> r
    }
  }

  /** Raw blocks of reducers this executor does not hold, from their owners (RPC). */
  def fetchRemote(shuffleId: Int, rank: Int, mapIds: Array[Long], reduceIds: Array[Int]): GpuRemoteBlocks =
    peers(rank).askSync[GpuRemoteBlocks](GpuFetchRemote(shuffleId, mapIds, reduceIds))

  def stop(): Unit = comm.shutdownNow()
}
