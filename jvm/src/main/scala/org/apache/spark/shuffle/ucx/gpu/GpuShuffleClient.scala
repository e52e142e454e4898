/*
 * GpuShuffleClient — BlockStoreClient.fetchBlocks over the engine's HBM-resident blocks.
 * Replaces spark_3_0/UcxShuffleClient.scala:17-91: same signature, same recursive split in
 * halves (splitAt(length / 2)) above spark.shuffle.ucx.maxBlocksPerRequest (:53-58), same
 * "shuffle_<s>_<m>_<r>" parsing (:64).
 * Differences, by design:
 *   - one SgxNative.fetchBlocks per request (one gather launch on the GPU) instead of one
 *     synchronous UCX round trip per block with a progress() spin (:17-47);
 *   - a failed request reports onBlockFetchFailure for each of its blocks (the reference
 *     never calls it, :36-40), so Spark's FetchFailed / stage retry runs.
 * Mirrored in Python by sparkucx_amd.shuffle.UcxShuffleClient (tested there).
 */
package org.apache.spark.shuffle.ucx.gpu

import java.nio.ByteBuffer

import org.apache.spark.SparkConf
import org.apache.spark.network.buffer.NioManagedBuffer
import org.apache.spark.network.shuffle.{BlockFetchingListener, BlockStoreClient, DownloadFileManager}
import org.apache.spark.storage.{BlockId, ShuffleBlockId}

class GpuShuffleClient(engine: Long, conf: SparkConf) extends BlockStoreClient {
  private val maxBlocksPerRequest = conf.getInt("spark.shuffle.ucx.maxBlocksPerRequest", 50)

  override def fetchBlocks(host: String, port: Int, execId: String, blockIds: Array[String],
                           listener: BlockFetchingListener,
                           downloadFileManager: DownloadFileManager): Unit = {
    if (blockIds.length > maxBlocksPerRequest) {
      // the reference's split (UcxShuffleClient.scala:53-58): halve, recurse on both halves
      val (b1, b2) = blockIds.splitAt(blockIds.length / 2)
      fetchBlocks(host, port, execId, b1, listener, downloadFileManager)
      fetchBlocks(host, port, execId, b2, listener, downloadFileManager)
      return
    }
    val parsed = blockIds.map(id => BlockId(id).asInstanceOf[ShuffleBlockId])
    val shuffleId = parsed.head.shuffleId
    val mapIds = parsed.map(_.mapId)
    val reduceIds = parsed.map(_.reduceId)
    try {
      val sizes = SgxNative.fetchBlocks(engine, shuffleId, mapIds, reduceIds, null)  // size query
      if (sizes.sum > Int.MaxValue - 8) {
        // one direct buffer holds < 2 GiB: split the request (a single block that large fails)
        if (blockIds.length == 1)
          throw new SgxFetchException(s"block ${blockIds(0)} of ${sizes(0)} bytes exceeds one direct buffer")
        val (a, b) = blockIds.splitAt(blockIds.length / 2)
        fetchBlocks(host, port, execId, a, listener, downloadFileManager)
        fetchBlocks(host, port, execId, b, listener, downloadFileManager)
        return
      }
      val dst = ByteBuffer.allocateDirect(math.max(1L, sizes.sum).toInt)
      SgxNative.fetchBlocks(engine, shuffleId, mapIds, reduceIds, dst)
      var off = 0
      blockIds.indices.foreach { i =>
        val slice = dst.duplicate()
        slice.position(off).limit(off + sizes(i).toInt)
        listener.onBlockFetchSuccess(blockIds(i), new NioManagedBuffer(slice.slice()))
        off += sizes(i).toInt
      }
    } catch {
      case e: SgxFetchException => blockIds.foreach(listener.onBlockFetchFailure(_, e))
      case e: IllegalArgumentException => blockIds.foreach(listener.onBlockFetchFailure(_, e))
    }
  }

  override def close(): Unit = ()
}
