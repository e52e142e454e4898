/*
 * sgx.h — C ABI of the MI355X-native shuffle engine (libsgx.so).
 *
 * This is the drop-in boundary behind SparkUCX's plugin API (ofirfarjun7/sparkucx,
 * Spark 3.0 profile).  Plain C types only: no torch, no HIP types in signatures.  Each
 * entry point names the reference interface it replaces (file:line relative to
 * /root/reference/src/main/scala/org/apache/spark/).  The JNI glue a maintainer adds on
 * the Scala side is shown in INTEGRATION.md.
 *
 * Conventions (mirror ShuffleTransport.scala:49-51,71 and the JVM exception mapping):
 *   - every int-returning call returns SGX_OK (0) or a negative SGX_ERR_* code;
 *     negative codes map to OperationStatus.FAILURE / a thrown exception on the JVM side;
 *   - sgx_last_error() returns a thread-local message for the last failure on this thread;
 *   - buffers passed in are caller-owned; map outputs and received blocks are engine-owned
 *     and live in HBM until sgx_unregister_shuffle / sgx_destroy;
 *   - one engine per GPU (= per executor).  The engine is thread-safe: every calling thread
 *     gets its own HIP stream and scratch buffers (the reference routes each calling thread
 *     to its own UCX worker, shuffle/ucx/UcxShuffleTransport.scala:277-296), so concurrent
 *     map tasks of one executor run side by side on the GPU; collectives (sgx_exchange) are
 *     issued by one thread at a time on the engine's exchange stream.
 */
#ifndef SGX_H
#define SGX_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SGX_ABI_VERSION 7

enum sgx_status {
    SGX_OK = 0,
    SGX_ERR_INVALID = -1,   /* IllegalArgumentException: bad argument / out-of-order use   */
    SGX_ERR_STATE = -2,     /* IllegalStateException: not registered / not initialised     */
    SGX_ERR_HIP = -3,       /* HIP runtime failure (RuntimeException)                      */
    SGX_ERR_COMM = -4,      /* RCCL failure (TransportError)                               */
    SGX_ERR_IO = -5,        /* IOException: index/data file commit                         */
    SGX_ERR_NOMEM = -6,     /* device or host allocation failed                            */
    SGX_ERR_NOT_FOUND = -7, /* block not registered (UcxShuffleTransport.scala:229-269)    */
    SGX_ERR_UNSUPPORTED = -8,
    SGX_ERR_TIMEOUT = -9    /* a bounded device spin gave up                               */
};

/* Partitioner kinds (the ShuffleDependency's partitioner). */
enum sgx_partitioner {
    SGX_PART_HASH = 0,          /* HashPartitioner: nonNegativeMod(Long.hashCode(k), R)    */
    SGX_PART_RANGE_I64 = 1,     /* RangePartitioner over signed-long keys                  */
    SGX_PART_RANGE_BYTES10 = 2  /* RangePartitioner over 10-byte unsigned keys (TeraSort)  */
};

/* Where a caller buffer lives.  SGX_MEM_DEVICE_RETAINED (sgx_map_append only): device memory
 * the caller keeps valid and unchanged until the map's partition lengths are known -- an
 * sgx_map_commit given out_partition_lengths has returned, or sgx_map_lengths / sgx_sync has
 * returned after an asynchronous commit -- because the commit's kernels read the batch in place
 * (no copy); elsewhere it means SGX_MEM_DEVICE. */
enum sgx_mem_kind { SGX_MEM_HOST = 0, SGX_MEM_DEVICE = 1, SGX_MEM_DEVICE_RETAINED = 2 };

typedef struct sgx_engine sgx_engine;

/* Kernel choices (every choice produces the same bytes; they differ in speed only). */
enum sgx_hist_mode { SGX_HIST_ATOMIC = 0,   /* one LDS atomic per record (default)            */
                     SGX_HIST_BALLOT = 1 }; /* wave-aggregated: peers by 64-lane ballots, the
                                               lowest peer adds popcount(peers) (16 B hash)   */
enum sgx_rank_mode { SGX_RANK_ORDERED = 0,  /* K4 ranks by lane-ordered LDS atomics (default) */
                     SGX_RANK_MATCH = 1 };  /* K4 ranks by ballot peer matching               */
enum sgx_flags {
    SGX_FLAG_NO_WRITE_COMBINING = 1,  /* hash K4 without on-chip line write-combining      */
    SGX_FLAG_NO_WIDE_STAGED = 2,      /* 100 B records: per-lane K4 instead of LDS-staged   */
    SGX_FLAG_SORT_ALL_DIGITS = 4,     /* sorted reads run every digit pass (no skipping)    */
    SGX_FLAG_DEBUG_SYNC = 8,          /* debugging: synchronise after every kernel and name the
                                         kernel in the error of a device fault (slow)         */
    SGX_FLAG_LZ4_LANE_DECODE = 16,    /* LZ4 reads decode every compressed frame one lane per
                                         frame (default: only from 32768 frames up)           */
    SGX_FLAG_NO_SPLIT_SCATTER = 32,   /* hash K4 with R > 1024: one lane-ordered pass instead
                                         of the two-level write-combining split               */
    SGX_FLAG_NO_BUCKET_SORT = 64,     /* sorted reads / map-side combine: LSD digit passes only
                                         (no key-window buckets sorted on chip)               */
    SGX_FLAG_ASSUME_LDS_DISORDER = 128, /* testing: act as if the engine-start LDS ordering
                                          check had failed (see sgx_lds_order_ok)             */
    SGX_FLAG_NO_PADDED_MAP = 256,     /* hash maps always take the two-pass map side (histogram
                                         + scan + scatter) instead of the single-pass padded
                                         write (sgx_map_layout)                                */
    SGX_FLAG_PAD_ANY_SIZE = 512,      /* testing: write maps of any size padded (default: from
                                         2^20 records up)                                      */
    SGX_FLAG_NO_SEG_WINDOW = 1024,    /* sorted reads of several partitions: the key window and
                                         the partitioner in two LSD passes instead of one
                                         segmented pass per partition                          */
    SGX_FLAG_NO_DEFERRED_APPEND = 2048, /* streaming maps: partition every sgx_map_append batch on
                                         arrival and gather them at the commit (the round-4 form)
                                         instead of one pass over all batches at the commit    */
    SGX_FLAG_NO_P2P_EXCHANGE = 4096,  /* exchange rounds move their bytes by grouped
                                         ncclSend / ncclRecv (RCCL) or the host all-to-all over
                                         contiguous map outputs, and a communicator keeps the
                                         map side two-pass; default: the direct peer gather
                                         (sgx_exchange) out of single-pass padded maps         */
    SGX_FLAG_NO_OVERLAP_WRITES = 8192, /* keep every padded write of a calling thread on one
                                         stream; default: consecutive writes alternate between
                                         two streams, so a write's sample and K4 start on the
                                         CUs the previous write's last K4 workgroups free (see
                                         sgx_set_overlap_writes)                              */
    SGX_FLAG_TEST_P2P_UNAVAILABLE = 16384 /* testing: this rank reports the direct peer gather's
                                         IPC mapping as unavailable; the exchange then falls
                                         back on every rank (see sgx_exchange)               */
};

typedef struct sgx_config {
    int32_t device;          /* HIP device ordinal for this executor                     */
    int32_t num_chunks;      /* map-side work chunks per batch (0 = one per CU)           */
    int32_t scatter_waves;   /* K4 geometry override (0 = auto): waves per workgroup       */
    int32_t scatter_items;   /* K4 geometry override (0 = auto): records per lane per tile */
    int32_t hist_mode;       /* enum sgx_hist_mode                                         */
    int32_t rank_mode;       /* enum sgx_rank_mode                                         */
    int32_t flags;           /* enum sgx_flags, or-ed                                      */
    int32_t comm_timeout_ms; /* bound on any wait for the exchange (0 = 300 s): a dead peer
                                aborts the communicator and fails with SGX_ERR_TIMEOUT
                                instead of spinning forever (UcxShuffleClient.scala:44-46) */
} sgx_config;

/* Overlapping consecutive map writes (default on; SGX_FLAG_NO_OVERLAP_WRITES at creation, or
 * this call at any time, from the next write on): a calling thread's padded writes alternate
 * between two streams, so the next write's sample and K4 fill the CUs the previous K4's last
 * workgroups leave idle (map throughput +1.3 % to +8 % at C1, by box).  With
 * it on, a K4's HIP-event interval or traced duration starts at its dispatch and includes the
 * wait for those CUs, so kernel-alone timings are taken with it off (bench.py's roofline). */
int sgx_set_overlap_writes(sgx_engine *e, int32_t on);

/* ---- engine lifetime: replaces CommonUcxShuffleManager.startUcxTransport
 *      (shuffle/ucx/CommonUcxShuffleManager.scala:67-100) and stop() (:111-124) ---- */
int sgx_create(const sgx_config *cfg, sgx_engine **out);
void sgx_destroy(sgx_engine *e);
/* Frees the calling thread's stream and scratch buffers (an executor thread that leaves the
 * pool); they are recreated on the thread's next call. */
int sgx_release_thread(sgx_engine *e);
const char *sgx_last_error(void);
int32_t sgx_abi_version(void);
/* Result of the engine-start device check (sgx_create runs it once, ~1 ms): 1 if same-address
 * LDS atomics issued back to back by one wave returned their old values in issue order, then
 * lane order, on this device -- the property the default ranking (SGX_RANK_ORDERED) and the
 * reduce side's sort passes rest on.  0 if it did not (or SGX_FLAG_ASSUME_LDS_DISORDER): the
 * engine then ranks every scatter by ballot peer matching (SGX_RANK_MATCH, the per-lane
 * kernels for sort passes and 100 B records) -- slower, same bytes.  -1 for a NULL engine. */
int32_t sgx_lds_order_ok(const sgx_engine *e);

/* ---- registerShuffle: SortShuffleManager.registerShuffle inherited at
 *      shuffle/ucx/CommonUcxShuffleManager.scala:25; the partitioner of the dependency.
 *      bounds: nbounds sorted keys (int64 for RANGE_I64, 10-byte rows for RANGE_BYTES10);
 *      num_partitions must be nbounds+1 for range kinds. record_bytes: 16 (Long,Long) or
 *      100 (TeraSort); the key is the first 8 (hash / range_i64) or 10 bytes. ---- */
int sgx_register_shuffle(sgx_engine *e, int32_t shuffle_id, int32_t num_partitions,
                         int32_t partitioner_kind, const void *bounds, int64_t nbounds,
                         int32_t ascending, int32_t record_bytes);
/* dep.serializer (ShuffleDependency; the writers built at spark_3_0/UcxShuffleManager.scala:
 * 37-51 serialize every record with it).  SGX_SER_FIXED: the engine's fixed-width record
 * codec (lengths = records x record_bytes).  SGX_SER_KRYO: Spark's KryoSerializer stream with
 * spark.shuffle.compress=false, for (Long, Long) 16 B records: per record
 * [0x09][zigzag varlong key][0x09][zigzag varlong value] (kryo.writeClassAndObject of two
 * java.lang.Long), framed on the GPU after the scatter; partition lengths, index offsets,
 * the data file, fetched blocks and exchanged bytes are then those of the Kryo stream, so
 * Spark's own reader deserializes them.  Set before the first sgx_write_map of the shuffle
 * (SGX_ERR_STATE after).  The reduce side (sgx_read_records / _sorted / _grouped) decodes the
 * fetched Kryo stream back to records on the GPU before sorting / grouping. */
enum sgx_serializer { SGX_SER_FIXED = 0, SGX_SER_KRYO = 1 };
int sgx_set_serializer(sgx_engine *e, int32_t shuffle_id, int32_t serializer);
/* spark.shuffle.compress=true, spark.io.compression.codec=lz4 (Spark 3.0.1 defaults): every
 * partition stream is wrapped on its own (ShufflePartitionPairsWriter.open ->
 * SerializerManager.wrapStream, invoked by the writers built at
 * spark_3_0/UcxShuffleManager.scala:37-51, bytes landing in NvkvShuffleMapOutputWriter's
 * PartitionWriterStream, ucx/NvkvShuffleMapOutputWriter.scala:228-246) in lz4-java's
 * LZ4BlockOutputStream(block_size, fast compressor, XXH32 seed 0x9747b28c).  Frames the
 * partition streams [part_offsets[r], part_offsets[r+1]) of stream_dev (device bytes, e.g. the
 * Kryo stream of sgx_map_data) on the GPU, byte-identical to lz4-java 1.7.1 / liblz4 1.9.x:
 * 32 KiB blocks by default, LZ4 or RAW per block, the 21-byte end mark per non-empty partition.
 * part_offsets: host int64[R+1]; out_lengths: caller-owned int64[R] (framed bytes per
 * partition; 0 for an empty partition, whose stream Spark never opens).  dst_dev NULL only
 * measures; otherwise the frames are written back to back into dst_dev (dst_cap bytes,
 * SGX_ERR_INVALID if too small, out_lengths still filled).  block_size in [64, 32768].
 * Synchronous. */
int sgx_lz4_frame_partitions(sgx_engine *e, const void *stream_dev, const int64_t *part_offsets,
                             int32_t num_partitions, int32_t block_size, void *dst_dev, int64_t dst_cap,
                             int64_t *out_lengths);
/* The same compression as a shuffle property: with SGX_CODEC_LZ4 every map output of the
 * shuffle publishes its LZ4-framed partition streams (block_size, 32768 = Spark's default)
 * instead of the raw Kryo stream -- partition lengths, index offsets, data file, fetched and
 * exchanged blocks are then the bytes Spark writes with spark.shuffle.compress=true.  Needs
 * SGX_SER_KRYO (set first); set before the first sgx_write_map (SGX_ERR_STATE after).  The
 * reduce-side reads (sgx_read_records / _sorted / _grouped) fetch the frames, decompress them
 * on the GPU and decode the Kryo stream. */
enum sgx_codec { SGX_CODEC_NONE = 0, SGX_CODEC_LZ4 = 1 };
int sgx_set_compression(sgx_engine *e, int32_t shuffle_id, int32_t codec, int32_t block_size);
/* The reduce side of the same codec (lz4-java LZ4BlockInputStream, what
 * SerializerManager.wrapStream does to each fetched block before deserialization,
 * spark_3_0/UcxShuffleReader.scala:137-145): framed_dev holds any number of LZ4-framed
 * partition streams back to back (e.g. the blocks of sgx_fetch_blocks); their decompressed
 * bytes are written back to back into dst_dev.  *out_bytes = decompressed size; dst_dev NULL
 * only measures.  Headers, lengths, block contents (LZ4_decompress_safe bounds) and every
 * XXH32 are checked: SGX_ERR_INVALID on a malformed or corrupt stream.  Synchronous. */
int sgx_lz4_unframe(sgx_engine *e, const void *framed_dev, int64_t framed_bytes, void *dst_dev, int64_t dst_cap,
                    int64_t *out_bytes);
/* The same over fetched blocks whose extents are known (stream_lens[nstreams], summing to the
 * buffer's bytes; each one LZ4 stream, e.g. one partition block of one map): the frame walks run
 * one per stream in parallel instead of one serial walk over the whole buffer.  The reduce-side
 * reads (sgx_read_*) of a compressed shuffle decode this way. */
int sgx_lz4_unframe_streams(sgx_engine *e, const void *framed_dev, const int64_t *stream_lens, int64_t nstreams,
                            void *dst_dev, int64_t dst_cap, int64_t *out_bytes);
/* dep.mapSideCombine with dep.aggregator (reduceByKey: Spark's default is mapSideCombine =
 * true; the writer built at spark_3_0/UcxShuffleManager.scala:48-51 then runs
 * ExternalSorter.insertAll with the aggregator, and the reader merges combiners with
 * combineCombinersByKey, spark_3_0/UcxShuffleReader.scala:158-161).  SGX_AGG_SUM on (Long,
 * Long) records: every map output holds one record {key, wrapping sum of the map's values of
 * key} per distinct key, partitioned by the shuffle's partitioner, keys ascending within a
 * partition (Spark's PartitionedAppendOnlyMap iteration order is unspecified; this is the
 * canonical order the parity tests compare).  Set before the first write (SGX_ERR_STATE
 * after).  sgx_read_grouped(SGX_AGG_SUM) on such a shuffle is combineCombinersByKey. */
int sgx_set_map_side_combine(sgx_engine *e, int32_t shuffle_id, int32_t agg);
/* The map writer Spark runs for the shuffle's handle.  SortShuffleManager.registerShuffle
 * (inherited, shuffle/ucx/CommonUcxShuffleManager.scala:25) gives a dependency with a
 * relocatable serializer (Kryo), no map-side combine and more partitions than
 * spark.shuffle.sort.bypassMergeThreshold (200) a SerializedShuffleHandle, and the reference's
 * getWriter (spark_3_0/UcxShuffleManager.scala:32-53) runs UnsafeShuffleWriter for it; every
 * other handle gets SortShuffleWriter.  SGX_WRITER_SORT (the default): a map's spills are
 * merged into ONE serialized -- and compressed -- stream per partition (ExternalSorter).
 * SGX_WRITER_UNSAFE: UnsafeShuffleWriter with its fast spill merge
 * (spark.shuffle.unsafe.fastMergeEnabled, LZ4 being a concatenable codec): each spill's
 * partition segment is its own LZ4 stream (DiskBlockObjectWriter.commitAndGet per partition)
 * and a partition's segments are concatenated in spill order.  The two differ only for a
 * compressed Kryo map written in several batches (sgx_map_append); Spark's reader
 * (LZ4BlockInputStream with concatenation) and sgx_read_* decode both.  Set before the first
 * write; SGX_ERR_STATE together with map-side combine (Spark never gives such a dependency a
 * SerializedShuffleHandle). */
enum sgx_map_writer { SGX_WRITER_SORT = 0, SGX_WRITER_UNSAFE = 1 };
int sgx_set_map_writer(sgx_engine *e, int32_t shuffle_id, int32_t writer);

/* Reducer placement of a shuffle's exchange (sgx_exchange).  SGX_PLACE_EVEN (the default):
 * rank j holds the reducers r with floor(r * P / R) == j.  SGX_PLACE_BYTES: contiguous reducer
 * ranges that balance the bytes each rank receives (sgx_balanced_ranges over the all-gathered
 * lengths of the shuffle's first exchange round, the same on every rank), for skewed keys
 * (config C3: Zipf(1.1) puts most of the head of the distribution on rank 0 under the even
 * split).  Which ranks run which reduce tasks is the engine's choice -- Spark's scheduler
 * places reduce tasks itself (UcxShuffleReader.scala:74-103 reads whichever partition range
 * it is given); the canonical per-reducer sequences do not change.  The ranges are fixed by
 * the shuffle's first exchange round and hold for every later round, so all blocks of a
 * reducer land on one rank: set the placement before the first sgx_exchange (SGX_ERR_STATE
 * after). */
enum sgx_placement { SGX_PLACE_EVEN = 0, SGX_PLACE_BYTES = 1 };
int sgx_set_reducer_placement(sgx_engine *e, int32_t shuffle_id, int32_t placement);
/* The reducers [*r0, *r1) this rank holds for shuffle_id (fixed by its first exchange round;
 * SGX_ERR_STATE before it).  The executor's reduce tasks for these partitions read locally;
 * INTEGRATION.md shows how the JVM side turns them into preferred locations. */
int sgx_shuffle_reducers(sgx_engine *e, int32_t shuffle_id, int32_t *r0, int32_t *r1);
/* The same, looked up through the exchange round that carried map_id (the map of any rank). */
int sgx_round_reducers(sgx_engine *e, int32_t shuffle_id, int64_t map_id, int32_t *r0, int32_t *r1);
/* unregisterShuffle: CommonUcxShuffleManager.scala:103-106 -> removeShuffle
 * (CommonUcxShuffleBlockResolver.scala:63-71). Frees the shuffle's HBM. */
int sgx_unregister_shuffle(sgx_engine *e, int32_t shuffle_id);

/* ---- getWriter(...).write(records) + ShuffleMapOutputWriter.commitAllPartitions
 *      (spark_3_0/UcxShuffleManager.scala:32-53; ucx/NvkvShuffleMapOutputWriter.scala:
 *      105-148): partition ids + histogram + scan + stable scatter on the GPU.  The map
 *      output stays in HBM, engine-owned.  out_partition_lengths: caller-owned int64[R],
 *      in BYTES (Spark's long[] lengths).  If NULL the call is asynchronous: lengths are
 *      available from sgx_map_lengths after sgx_sync. ---- */
int sgx_write_map(sgx_engine *e, int32_t shuffle_id, int64_t map_id, const void *records,
                  int64_t nrecords, int32_t record_bytes, int32_t mem_kind,
                  int64_t *out_partition_lengths);
int sgx_map_lengths(sgx_engine *e, int32_t shuffle_id, int64_t map_id, int64_t *out_lengths);
/* Streaming map output: the map task's records arrive as any number of batches (Spark's
 * writer sees unbounded partition streams and merges spills in spill order,
 * ucx/NvkvShuffleMapOutputWriter.scala:106-113,228-246).  sgx_map_begin opens the map.
 * sgx_map_append hands over one batch: a host batch is copied into HBM, a SGX_MEM_DEVICE
 * batch is copied within HBM, a SGX_MEM_DEVICE_RETAINED batch stays where it is (the caller
 * keeps it until the map's lengths are known: see sgx_mem_kind).  sgx_map_commit then partitions ALL batches in one
 * pass, exactly as sgx_write_map partitions one contiguous batch (the padded single-pass
 * write when sgx_write_map would take it): every batch is cut into chunks of
 * its own and a chunk table replaces the contiguous input.  The result is byte-identical to
 * sgx_write_map of all batches concatenated; LZ4 framing applies as for sgx_write_map.
 * Shuffles the one-pass commit does not cover (map-side combine, R > 1024 under a hash
 * partitioner, 16 B records under a RangePartitioner, SGX_FLAG_NO_DEFERRED_APPEND, an engine
 * whose lane-ordered ranking check failed) partition every batch on arrival and concatenate
 * the batches per partition at the commit (one gather launch), with the same bytes.
 * out_lengths as sgx_write_map (may be NULL).  A map holds < 2^32 records. */
int sgx_map_begin(sgx_engine *e, int32_t shuffle_id, int64_t map_id);
int sgx_map_append(sgx_engine *e, int32_t shuffle_id, int64_t map_id, const void *records, int64_t nrecords,
                   int32_t record_bytes, int32_t mem_kind);
int sgx_map_commit(sgx_engine *e, int32_t shuffle_id, int64_t map_id, int64_t *out_partition_lengths);
/* Device pointer + byte size of a map output (partition-contiguous data; a padded map's
 * contiguous copy is built on the first call, see sgx_map_layout). */
int sgx_map_data(sgx_engine *e, int32_t shuffle_id, int64_t map_id, void **out_dev_ptr,
                 int64_t *out_bytes);
/* How the engine holds a written map (waits for its kernels).  A fixed-codec HashPartitioner
 * map of 16 B records (R > 1024 through the two-level split), or a 100 B TeraSort map under
 * its RangePartitioner, written by sgx_write_map (or committed from sgx_map_append batches)
 * on an engine with no communicator at all (none: a one-rank or host-collective communicator
 * counts, so every multi-executor deployment takes the two-pass write), is written in ONE pass
 * over its records: a sampled
 * histogram sizes a line-aligned sub-bin per (partition, chunk) stream, the stable scatter
 * writes every stream into its sub-bin, and a scan of the streams' true counts gives the
 * partition lengths and index offsets -- the same lengths, offsets and per-block bytes as the
 * two-pass write, with gaps between the streams in HBM (SGX_LAYOUT_PADDED).  Block fetches
 * gather the streams directly; exchange sends, sgx_map_data and index files use a contiguous
 * copy built once on first use.  A stream longer than its sub-bin (keys not spread like the
 * sample) makes the write redo the map with the two-pass kernels on the device
 * (SGX_LAYOUT_CONTIGUOUS), and the shuffle's later maps skip the padded attempt.  A Kryo
 * shuffle's (Long, Long) map under a HashPartitioner is written the same way and its serializer
 * reads the records from the sub-bins: what it publishes (the Kryo stream) is contiguous, and
 * SGX_LAYOUT_SERIALIZED_PADDED says only how the records got there.  Maps of other shuffles
 * are always SGX_LAYOUT_CONTIGUOUS. */
enum sgx_layout { SGX_LAYOUT_CONTIGUOUS = 0, SGX_LAYOUT_PADDED = 1, SGX_LAYOUT_SERIALIZED_PADDED = 2 };
int sgx_map_layout(sgx_engine *e, int32_t shuffle_id, int64_t map_id, int32_t *out_layout);

/* ---- IndexShuffleBlockResolver.writeIndexFileAndCommit (IndexShuffleBlockResolver.scala:
 *      161-217): writes the map output as data file + index file ((R+1) big-endian int64
 *      offsets), atomically via tmp+rename; an existing valid attempt wins and its lengths
 *      are returned in out_lengths (may be NULL). ---- */
int sgx_write_index(sgx_engine *e, int32_t shuffle_id, int64_t map_id, const char *index_path,
                    const char *data_path, int64_t *out_lengths);
/* Host-only helpers (no GPU needed): checkIndexAndDataFile (:110-149) and the
 * getBlockData offset lookup (:219-262). */
int sgx_check_index_and_data(const char *index_path, const char *data_path, int32_t blocks,
                             int64_t *out_lengths);
int sgx_index_block_range(const char *index_path, int32_t start_reduce, int32_t end_reduce,
                          int64_t *out_offset, int64_t *out_length);

/* ---- reduce-side exchange: replaces the per-block UCX AM fetch path
 *      (ucx/UcxWorkerWrapper.scala:96-186, spark_3_0/UcxShuffleClient.scala:17-91) with one
 *      lengths all-gather + one grouped all-to-all over xGMI per shuffle.  Call
 *      sgx_comm_init once per engine (the unique id travels over the host's control plane,
 *      which replaces the ExecutorAdded/IntroduceAllExecutors RPC in the rpc/ package). ---- */
int sgx_get_unique_id(uint8_t out_id[128]);
/* Host control plane for the id (§8(f) row 4; replaces the ExecutorAdded /
 * IntroduceAllExecutors RPC of rpc/UcxDriverRpcEndpoint.scala:21-42 and
 * rpc/UcxExecutorRpcEndpoint.scala:19-39): rank 0 serves `id` on TCP `port` until ranks
 * 1..nranks-1 have each fetched it once (SGX_ERR_TIMEOUT after timeout_ms); rank r joins
 * host:port, retrying until the server is up, and receives the id and the world size.
 * No GPU is touched: the id may travel on Spark RPC instead. */
int sgx_bootstrap_serve(int32_t port, int32_t nranks, const uint8_t id[128], int32_t timeout_ms);
int sgx_bootstrap_join(const char *host, int32_t port, int32_t rank, int32_t timeout_ms, uint8_t out_id[128],
                       int32_t *out_nranks);
int sgx_comm_init(sgx_engine *e, int32_t nranks, int32_t rank, const uint8_t id[128]);
/* Host collective backend (the fake exchange backend of SURVEY §4, and the path for ranks
 * that share one GPU, which RCCL refuses): the exchange runs exactly as over RCCL -- counts
 * all-gather, sgx_plan_exchange, all-to-all of the partition-contiguous map output into the
 * [source][my reducers] receive layout, block fetches from HBM -- but the two collectives are
 * the caller's functions over host memory (the map output is staged device -> host and the
 * received bytes host -> device).  Return 0 on success; anything else fails the exchange with
 * SGX_ERR_COMM.  allgather: every rank contributes `bytes` bytes, recv receives nranks * bytes,
 * rank-major.  alltoallv: byte counts / displacements, as ncclAllToAllv. */
typedef struct sgx_host_comm {
    void *user;
    int (*allgather)(void *user, const void *send, int64_t bytes, void *recv);
    int (*alltoallv)(void *user, const void *send, const int64_t *send_counts, const int64_t *send_displs,
                     void *recv, const int64_t *recv_counts, const int64_t *recv_displs);
} sgx_host_comm;
int sgx_comm_init_host(sgx_engine *e, int32_t nranks, int32_t rank, const sgx_host_comm *comm);
int sgx_comm_size(sgx_engine *e, int32_t *nranks, int32_t *rank);
/* The exchange of shuffle_id (sgx_exchange(e, shuffle_id)), collective: every
 * rank calls it, in the same order relative to its other exchanges, once its map tasks of the
 * shuffle are committed.  Each rank contributes every committed map output of the shuffle it
 * holds that no earlier exchange carried -- any number, none included: Spark's map tasks land
 * on executors independently -- and afterwards every rank holds its reducers' blocks
 * (sgx_shuffle_reducers) of every map of every rank.  Steps: an all-gather of each rank's map
 * count with its first map's {map id, R lengths} (a second all-gather of every map's, only
 * when some rank holds more than one), then ONE grouped exchange of the
 * partition-contiguous map outputs (already grouped by destination: no pack step) into this
 * rank's receive buffer, laid out [source rank][its maps][my reducers].  Asynchronous on the
 * engine's exchange stream; completes at sgx_sync (fetches and reads wait for it on the GPU).
 * Calling it again after more maps were written runs another round with just those maps (the
 * reducer ranges stay those of the first round).  Map ids must be unique across ranks. */
int sgx_exchange(sgx_engine *e, int32_t shuffle_id);
/* The same collective with exactly the listed local maps (n >= 0; 0 = this rank contributes
 * nothing this round): a pipelined writer exchanges map k while it writes map k + 1. */
int sgx_exchange_maps(sgx_engine *e, int32_t shuffle_id, const int64_t *map_ids, int64_t n);
/* A rank that cannot take part in an exchange round of a shuffle with num_partitions
 * reducers (it failed before sgx_exchange: e.g. registering the shuffle) joins the round's
 * first all-gather anyway, marked failed with `code` (< 0), so every rank's sgx_exchange of
 * that round fails at once with SGX_ERR_STATE instead of waiting in the collective for it
 * until the timeout.  A rank whose own sgx_exchange fails locally (an open map, a failed
 * write) marks the round the same way by itself.  Returns `code`. */
int sgx_exchange_fail(sgx_engine *e, int32_t num_partitions, int32_t code);

/* ---- ShuffleTransport.fetchBlocksByBlockIds (ucx/ShuffleTransport.scala:154-156) /
 *      BlockStoreClient.fetchBlocks (spark_3_0/UcxShuffleClient.scala:49-91): copy blocks
 *      (map_ids[i], reduce_ids[i]) back to back into the caller-owned dst (dst_mem_kind).
 *      out_lengths[i] = bytes of block i.  Blocks come from local map outputs or from data
 *      received by sgx_exchange. Fails with SGX_ERR_NOT_FOUND for an unknown block and
 *      SGX_ERR_INVALID if dst_cap is too small (nothing partial is reported as success). */
int sgx_fetch_blocks(sgx_engine *e, int32_t shuffle_id, const int64_t *map_ids,
                     const int32_t *reduce_ids, int64_t n, void *dst, int64_t dst_cap,
                     int32_t dst_mem_kind, int64_t *out_lengths);

/* ShuffleTransport.progress (ShuffleTransport.scala:158-165): non-blocking; returns 1 when
 * all submitted work is complete, 0 while some is in flight. sgx_sync blocks until done. */
int sgx_progress(sgx_engine *e);
int sgx_sync(sgx_engine *e);

/* ---- blocks fetched from elsewhere: a reduce task Spark placed on an executor that does not
 *      own its reducers (the reference's reader takes any block from anywhere,
 *      spark_3_0/UcxShuffleReader.scala:74-103) fetches their raw blocks from the owners and
 *      imports them into its own engine; sgx_read_records / _sorted / _grouped and
 *      sgx_fetch_blocks then run over them on this GPU as over exchanged blocks.  data: the
 *      blocks (map_ids[j], r) for r in [start, end), j in [0, nmaps), back to back in the
 *      canonical order -- reducer-major, then map (what sgx_fetch_blocks returns for that
 *      list) -- in host or device memory (mem_kind); lengths[(r - start) * nmaps + j] their
 *      bytes (published bytes: fixed records, or Kryo / LZ4 frames).  Copied: the caller's
 *      buffer may be freed on return.  *out_import_id names the import for
 *      sgx_release_import, which frees its HBM (the read's results stay valid). ---- */
int sgx_import_blocks(sgx_engine *e, int32_t shuffle_id, const int64_t *map_ids, int64_t nmaps,
                      int32_t start_partition, int32_t end_partition, const void *data, int32_t mem_kind,
                      const int64_t *lengths, int64_t *out_import_id);
int sgx_release_import(sgx_engine *e, int32_t shuffle_id, int64_t import_id);

/* ---- reduce side after the fetch: UcxShuffleReader.read (spark_3_0/UcxShuffleReader.scala:
 *      137-191).  Input = the blocks (map_ids[0..nmaps) x reducers [start, end)) this engine
 *      holds (local map outputs or blocks received by sgx_exchange), taken in the canonical
 *      order (reducer-major, then map order, then record order).
 *
 * sgx_read_sorted: dep.keyOrdering (sortByKey, TeraSort's reduce side; ExternalSorter with an
 * ordering, :166-181): every reducer's records sorted STABLY by key -- signed Long for 16 B
 * records, the 10-byte unsigned big-endian key for 100 B records -- written back to back,
 * reducer-major, into dst (dst_mem_kind).  *out_bytes = total bytes; dst NULL with dst_cap 0
 * is a size query.  LSD radix passes of the map side's own partition kernels (8-bit digits)
 * plus one pass by the shuffle's partitioner (skipped for an ascending RangePartitioner,
 * whose partition order is key order).  SGX_ERR_UNSUPPORTED for other record widths. */
int sgx_read_sorted(sgx_engine *e, int32_t shuffle_id, const int64_t *map_ids, int64_t nmaps,
                    int32_t start_partition, int32_t end_partition, void *dst, int64_t dst_cap,
                    int32_t dst_mem_kind, int64_t *out_bytes);

/* sgx_read_records: no aggregator, no key ordering -- the records of reducers [start, end)
 * in the canonical order (what the reader's deserializeStream(...).asKeyValueIterator
 * yields, :137-145), back to back into dst.  For a fixed-codec shuffle this is the fetched
 * blocks; for a Kryo shuffle the fetched Kryo stream is decoded to 16 B (Long, Long) records
 * on the GPU (SGX_ERR_INVALID if it is not a Kryo stream of Long pairs).  dst NULL with
 * dst_cap 0 is a size query. */
int sgx_read_records(sgx_engine *e, int32_t shuffle_id, const int64_t *map_ids, int64_t nmaps,
                     int32_t start_partition, int32_t end_partition, void *dst, int64_t dst_cap,
                     int32_t dst_mem_kind, int64_t *out_bytes);

/* sgx_read_grouped: dep.aggregator with mapSideCombine = false (Aggregator.combineValuesByKey,
 * :155-164) on (Long, Long) records.  Groups are emitted in ascending key order per reducer
 * (Spark's hash-map iteration order is unspecified; this is the canonical order the parity
 * tests compare), values of a group in the canonical arrival order.
 *   SGX_AGG_GROUP (groupByKey): keys[G], group_starts[G] (index of the group's first value),
 *                               values[N] (every value, grouped).
 *   SGX_AGG_SUM   (reduceByKey(_ + _)): keys[G], values[G] = wrapping Long sums;
 *                               group_starts may be NULL.
 * Capacities in elements: cap_groups for keys / group_starts, cap_values for values.  A call
 * with keys NULL and both capacities 0 only reports *out_groups / *out_values.  Output memory
 * kind: mem_kind (all three arrays). */
enum sgx_agg { SGX_AGG_GROUP = 0, SGX_AGG_SUM = 1 };
int sgx_read_grouped(sgx_engine *e, int32_t shuffle_id, const int64_t *map_ids, int64_t nmaps,
                     int32_t start_partition, int32_t end_partition, int32_t agg, int64_t *keys,
                     int64_t *group_starts, int64_t *values, int64_t cap_groups, int64_t cap_values,
                     int32_t mem_kind, int64_t *out_groups, int64_t *out_values);
/* The records the calling thread's last sgx_read_records / _sorted / _grouped consumed, before
 * any aggregation: the reference's reader counts incRecordsRead once per shuffled record ahead
 * of combineValuesByKey / combineCombinersByKey (spark_3_0/UcxShuffleReader.scala:148-162), so
 * an aggregated read reports these, not its groups. */
int sgx_last_read_records(sgx_engine *e, int64_t *out_records);

/* ---- RangePartitioner's bounds from the data (Spark 3.0.1 RangePartitioner: the
 *      rangeBounds initialiser, RangePartitioner.sketch and RangePartitioner.determineBounds;
 *      the partitioner is built where the dependency is, UcxShuffleManager.scala:50).
 * batches[i] (nrecords[i] records of record_bytes, memory kind mem_kind) is input partition i
 * of the RDD; keys are signed Longs (16 B records) or 10-byte unsigned keys (100 B records).
 * sampleSize = min(sample_points_per_partition * num_partitions, 1e6),
 * k = ceil(3 * sampleSize / nbatches) keys per partition by reservoir sampling with
 * XORShiftRandom(byteswap32(i ^ (rdd_id << 16))) -- rdd_id is the id of rdd.map(_._1), the
 * RDD sketch runs on -- on the GPU, every record's draw in parallel by GF(2) jump-ahead.  A
 * partition with fraction * n > k (fraction = min(sampleSize / numItems, 1)) is re-sampled as
 * Spark does: RDD.sample(false, fraction, byteswap32(-parent_rdd_id - 1)) over the imbalanced
 * partitions (parent_rdd_id: the id of the pair RDD the partitioner is built from), i.e. per
 * partition a BernoulliSampler seeded from java.util.Random's nextLong -- gap sampling on the
 * host when fraction <= 0.4, one draw per record on the GPU otherwise -- weighted
 * (1 / fraction).toFloat.  Then determineBounds on the host.  Writes up to num_partitions - 1
 * bounds (int64 or 10-byte keys) to out_bounds (host) and their count to *out_nbounds (fewer
 * when keys repeat; the shuffle then has *out_nbounds + 1 partitions). */
int sgx_range_bounds(sgx_engine *e, const void *const *batches, const int64_t *nrecords, int32_t nbatches,
                     int32_t record_bytes, int32_t mem_kind, int32_t num_partitions, int32_t rdd_id,
                     int32_t parent_rdd_id, int32_t sample_points_per_partition, void *out_bounds,
                     int32_t *out_nbounds);

/* ---- MemoryPool (memory/MemoryPool.scala:22-147): the BufferAllocator of the fetch contract
 *      (ShuffleTransport.scala:113).  Blocks come in power-of-two size classes from 4 KiB
 *      (spark.shuffle.ucx.memory.minBufferSize), pinned host memory (SGX_MEM_HOST: DMA-able)
 *      or HBM (SGX_MEM_DEVICE); sgx_pool_put returns a block (MemoryBlock.close()) to its
 *      class's free list, sgx_pool_preallocate fills a class ahead of time
 *      (spark.shuffle.ucx.memory.preAllocateBuffers, :141-147).  Thread-safe; freed with the
 *      engine. ---- */
int sgx_pool_get(sgx_engine *e, int64_t size, int32_t mem_kind, void **out_ptr, int64_t *out_capacity);
int sgx_pool_put(sgx_engine *e, void *ptr);
int sgx_pool_preallocate(sgx_engine *e, int64_t size, int32_t count, int32_t mem_kind);
int sgx_pool_stats(sgx_engine *e, int64_t *out_allocated_bytes, int64_t *out_idle_bytes);

/* ---- measurement: HIP-event times of the last write_map / exchange stages, and
 *      accumulated per-stage sums since the last reset (index = enum sgx_stage). ---- */
/* SGX_STAGE_REGROUP times the fetch-side gather kernel (blocks into request order). */
enum sgx_stage { SGX_STAGE_HIST = 0, SGX_STAGE_SCAN = 1, SGX_STAGE_SCATTER = 2,
                 SGX_STAGE_ALLGATHER = 3, SGX_STAGE_ALLTOALL = 4, SGX_STAGE_REGROUP = 5,
                 SGX_STAGE_SORT = 6, SGX_STAGE_GROUP = 7, SGX_STAGE_SERIALIZE = 8,
                 SGX_STAGE_DESERIALIZE = 9, SGX_STAGE_COMBINE = 10, SGX_STAGE_COMPRESS = 11,
                 SGX_STAGE_DECOMPRESS = 12, SGX_NUM_STAGES = 13 };
/* SGX_STAGE_SORT times sgx_read_sorted's radix + partitioner passes (the fetch gather is
 * REGROUP), SGX_STAGE_GROUP the grouping / summing kernels of sgx_read_grouped,
 * SGX_STAGE_COMBINE the map-side combine of sgx_write_map (sort + sum + repartition),
 * SGX_STAGE_SERIALIZE the Kryo framing kernel of sgx_write_map (SGX_SER_KRYO),
 * SGX_STAGE_DESERIALIZE the Kryo decoder of the reduce-side reads, SGX_STAGE_COMPRESS the LZ4
 * block kernel of a compressed map output (spark.shuffle.compress), SGX_STAGE_DECOMPRESS the
 * LZ4 block decoder of the reduce side (frame walks excluded). */
int sgx_stats_reset(sgx_engine *e);
/* out_ms[SGX_NUM_STAGES] summed milliseconds, out_count[SGX_NUM_STAGES] launches. */
int sgx_stats_get(sgx_engine *e, double *out_ms, int64_t *out_count);
/* Bytes the exchange rounds moved since sgx_stats_reset: out[0] to other ranks, out[1] kept
 * by this rank (its own reducers' blocks), out[2] rounds -- the blocks' lengths exactly, with
 * no sub-bin slack, whether a map was written padded or contiguous. */
int sgx_exchange_bytes(sgx_engine *e, int64_t out[3]);

/* ---- pure-host exchange planning (exported for tests of the multi-GPU logic) ----
 * lengths_all: [P][R] per-rank partition lengths in bytes.  Writes, for `rank`:
 * send_counts/send_displs[P] and recv_counts/recv_displs[P] in bytes, and the regroup
 * copy list (src offset in the receive buffer, dst offset in the per-reducer output,
 * bytes), ordered by reducer then source rank; *n_items in: capacity, out: count.
 * item_bytes: max bytes per copy item (0 = unlimited). */
int sgx_plan_exchange(const int64_t *lengths_all, int32_t P, int32_t R, int32_t rank,
                      int64_t item_bytes, int64_t *send_counts, int64_t *send_displs,
                      int64_t *recv_counts, int64_t *recv_displs, int64_t *items,
                      int64_t *n_items);
/* sgx_plan_exchange for explicit contiguous reducer ranges: rank j holds [bounds[j],
 * bounds[j + 1]) (bounds[P + 1], bounds[0] = 0, non-decreasing, bounds[P] = R). */
int sgx_plan_exchange_ranges(const int64_t *lengths_all, int32_t P, int32_t R, int32_t rank,
                             const int32_t *bounds, int64_t item_bytes, int64_t *send_counts,
                             int64_t *send_displs, int64_t *recv_counts, int64_t *recv_displs,
                             int64_t *items, int64_t *n_items);
/* The per-shuffle exchange's plan: rank j contributes maps_per_rank[j] maps, lengths_all
 * [M][R] source-rank-major.  send_counts/send_displs[P]: this rank's maps' bytes of each
 * destination's reducers, packed [destination][map]; recv_counts/recv_displs[P]: the bytes
 * from each source rank, [source rank][its maps][my reducers]; block_off[M][nmine] (may be
 * NULL): where block (map m, my reducer r) lands in the receive buffer. */
int sgx_plan_exchange_maps(const int64_t *lengths_all, const int64_t *maps_per_rank, int32_t P, int32_t R,
                           int32_t rank, const int32_t *bounds, int64_t *send_counts, int64_t *send_displs,
                           int64_t *recv_counts, int64_t *recv_displs, int64_t *block_off);
/* Byte-balanced placement: bounds[P + 1] of P contiguous reducer ranges minimising the largest
 * per-rank total of sum_j lengths_all[j][r] (binary search on the bound + greedy cuts; a
 * round with no bytes gets the even split).  Deterministic: every rank computes the same. */
int sgx_balanced_ranges(const int64_t *lengths_all, int32_t P, int32_t R, int32_t *bounds);
/* The even placement's bounds[P + 1] (floor(r * P / R) == j). */
int sgx_even_ranges(int32_t P, int32_t R, int32_t *bounds);
/* Apply a regroup copy list (items[n][3] host array, as produced by sgx_plan_exchange)
 * from src_dev to dst_dev with the K5 kernel; synchronous. */
int sgx_copy_items(sgx_engine *e, const void *src_dev, void *dst_dev, const int64_t *items,
                   int64_t n_items, int32_t align);
/* Reducer ownership: floor(r * P / R). */
int32_t sgx_reducer_owner(int32_t reduce_id, int32_t num_partitions, int32_t nranks);

/* ---- synthetic input generators (bench/test plumbing; the same definitions as the
 *      oracle's). dst is device memory. ---- */
int sgx_gen_uniform16(sgx_engine *e, void *dst_dev, int64_t n, uint64_t seed, int64_t value_base);
int sgx_gen_zipf16(sgx_engine *e, void *dst_dev, int64_t n, uint64_t seed, int64_t value_base,
                   const double *cdf_host, int64_t K);
int sgx_gen_terasort100(sgx_engine *e, void *dst_dev, int64_t n, uint64_t seed, int64_t index_base);
/* Device memory helpers for hosts without their own allocator (bench/tests). */
int sgx_device_alloc(sgx_engine *e, int64_t bytes, void **out);
int sgx_device_free(sgx_engine *e, void *p);
int sgx_memcpy(sgx_engine *e, void *dst, const void *src, int64_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* SGX_H */
