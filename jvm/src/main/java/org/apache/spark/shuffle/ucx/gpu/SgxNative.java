/*
 * SgxNative — the JNI surface of libsgxjni.so (jni/sgx_jni.c), one static native per C-ABI
 * entry point of include/sgx.h.  Source a maintainer adds to the reference tree next to
 * shuffle/compat/spark_3_0/ (this build image has no JDK; the shim itself is compile-checked
 * and driven by tests/test_jni_shim.py).
 *
 * Conventions: handles are the engine pointer as a long; host record / destination buffers
 * are direct ByteBuffers (pinned by the executor); arrays sized by a shuffle's partition
 * count take that count R as an argument.  Failures throw (see jni/sgx_jni.c):
 * IllegalArgumentException, IllegalStateException, IOException,
 * UnsupportedOperationException, OutOfMemoryError, SgxFetchException (missing block, RCCL
 * failure, timeout: turned into onBlockFetchFailure by GpuShuffleClient), RuntimeException.
 */
package org.apache.spark.shuffle.ucx.gpu;

import java.nio.ByteBuffer;

public final class SgxNative {
  static {
    System.loadLibrary("sgxjni");  // libsgxjni.so, linked against libsgx.so
  }

  private SgxNative() {}

  // partitioner kinds, serializers, codecs, aggregations (include/sgx.h enums)
  public static final int PART_HASH = 0, PART_RANGE_I64 = 1, PART_RANGE_BYTES10 = 2;
  public static final int SER_FIXED = 0, SER_KRYO = 1;
  public static final int CODEC_NONE = 0, CODEC_LZ4 = 1;
  public static final int AGG_GROUP = 0, AGG_SUM = 1;
  public static final int PLACE_EVEN = 0, PLACE_BYTES = 1;  // sgx_placement
  public static final int WRITER_SORT = 0, WRITER_UNSAFE = 1;  // sgx_map_writer

  // engine lifetime: CommonUcxShuffleManager.startUcxTransport / stop
  public static native long create(int device, int numChunks, int flags, int commTimeoutMs);
  public static native void destroy(long engine);
  public static native void releaseThread(long engine);

  // registerShuffle and the dependency's serializer / codec / map-side combine
  public static native void registerShuffle(long e, int shuffleId, int numPartitions, int kind,
                                            ByteBuffer bounds, long nbounds, boolean ascending,
                                            int recordBytes);
  public static native void setSerializer(long e, int shuffleId, int serializer);
  public static native void setCompression(long e, int shuffleId, int codec, int blockSize);
  public static native void setMapSideCombine(long e, int shuffleId, int agg);
  // the map writer of the shuffle's handle (WRITER_SORT / WRITER_UNSAFE; before the first write)
  public static native void setMapWriter(long e, int shuffleId, int writer);
  // reducer placement of the shuffle's exchange (PLACE_EVEN / PLACE_BYTES; before its first
  // exchange) and this executor's reducer range [r0, r1) of the shuffle (after it)
  public static native void setReducerPlacement(long e, int shuffleId, int placement);
  public static native int[] shuffleReducers(long e, int shuffleId);
  public static native int[] roundReducers(long e, int shuffleId, long mapId);
  public static native void unregisterShuffle(long e, int shuffleId);

  // getWriter().write(records) + commitAllPartitions(): long[R] partition lengths
  public static native long[] writeMap(long e, int shuffleId, long mapId, ByteBuffer records,
                                       long nrecords, int recordBytes, int numPartitions);
  // a map task whose records arrive in several batches (spills)
  public static native void mapBegin(long e, int shuffleId, long mapId);
  public static native void mapAppend(long e, int shuffleId, long mapId, ByteBuffer records,
                                      long nrecords, int recordBytes);
  public static native long[] mapCommit(long e, int shuffleId, long mapId, int numPartitions);

  // IndexShuffleBlockResolver
  public static native long[] writeIndex(long e, int shuffleId, long mapId, String indexPath,
                                         String dataPath, int numPartitions);
  public static native long[] checkIndexAndData(String indexPath, String dataPath, int blocks);
  public static native long[] indexBlockRange(String indexPath, int startReduce, int endReduce);

  // the exchange (ExecutorAdded / IntroduceAllExecutors replaced by the communicator id)
  public static native byte[] uniqueId();
  public static native void commInit(long e, int nranks, int rank, byte[] id);
  public static native void bootstrapServe(int port, int nranks, byte[] id, int timeoutMs);
  public static native byte[] bootstrapJoin(String host, int port, int rank, int timeoutMs,
                                            int[] nranksOut);
  // the shuffle's exchange, collective over every executor of the world (sgx_exchange: every
  // committed map of the shuffle this executor holds that no earlier exchange carried);
  // exchangeMaps: exactly these local maps (the pipelined form)
  public static native void exchange(long e, int shuffleId);
  public static native void exchangeMaps(long e, int shuffleId, long[] mapIds);
  // a round this executor cannot take part in: join it marked failed (every rank fails it)
  public static native void exchangeFail(long e, int numPartitions);
  // blocks of reducers [r0, r1) x mapIds fetched from their owners (reducer-major, map-minor
  // in a direct buffer): the reads then run over them on this GPU; returns the import id
  public static native long importBlocks(long e, int shuffleId, long[] mapIds, int r0, int r1, ByteBuffer data,
                                         long[] lengths);
  public static native void releaseImport(long e, int shuffleId, long importId);

  // fetchBlocksByBlockIds: blocks back to back in dst; returns their lengths (dst null = sizes)
  public static native long[] fetchBlocks(long e, int shuffleId, long[] mapIds, int[] reduceIds,
                                          ByteBuffer dst);
  public static native int progress(long e);
  public static native void sync(long e);

  // reduce side after the fetch (dst / buffers null = size query)
  public static native long readRecords(long e, int shuffleId, long[] mapIds, int startPartition,
                                        int endPartition, ByteBuffer dst);
  public static native long readSorted(long e, int shuffleId, long[] mapIds, int startPartition,
                                       int endPartition, ByteBuffer dst);
  public static native long[] readGrouped(long e, int shuffleId, long[] mapIds, int startPartition,
                                          int endPartition, int agg, ByteBuffer keys,
                                          ByteBuffer groupStarts, ByteBuffer values);
}
