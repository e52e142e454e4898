/*
 * shuffle_oracle.h — CPU restatement of the Spark 3.0.1 map-side shuffle semantics.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may link or call this library, and only as the checker / the
 * reported CPU baseline.  The product library (sparkucx_amd/libsgx.so) never links it.
 *
 * PARITY STATUS: the reference ships no tests or golden vectors for this path and its
 * arithmetic lives in the un-vendored spark-core 3.0.1 (pom.xml:80,90-95).  This
 * restatement is pinned by the known-answer tests of SURVEY.md §8(c) and cross-checked
 * against the independent Python restatement oracle/spark_semantics.py.
 */
#ifndef SHUFFLE_ORACLE_H
#define SHUFFLE_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Java Long.hashCode: (int)(v ^ (v >>> 32)). */
int32_t orc_java_long_hash(int64_t v);
/* Spark Utils.nonNegativeMod(x, mod). */
int32_t orc_non_negative_mod(int32_t x, int32_t mod);
/* HashPartitioner.getPartition for a java.lang.Long key. */
int32_t orc_hash_partition(int64_t key, int32_t num_partitions);
/* RangePartitioner.getPartition, signed-long keys (bounds: nb sorted longs). */
int32_t orc_range_partition_i64(int64_t key, const int64_t *bounds, int32_t nb, int32_t ascending);
/* RangePartitioner.getPartition, klen-byte unsigned-lexicographic keys. */
int32_t orc_range_partition_bytes(const uint8_t *key, int32_t klen, const uint8_t *bounds,
                                  int32_t nb, int32_t ascending);

/* Partitioner kinds (mirror include/sgx.h). */
enum { ORC_PART_HASH = 0, ORC_PART_RANGE_I64 = 1, ORC_PART_RANGE_BYTES10 = 2 };

/* Partition ids for n records of record_bytes each (key = first 8 bytes LE for HASH /
 * RANGE_I64; first 10 bytes for RANGE_BYTES10). */
void orc_partition_ids(const void *records, int64_t n, int32_t record_bytes, int32_t kind,
                       int32_t num_partitions, const void *bounds, int32_t nbounds,
                       int32_t ascending, int32_t *pids);

/* Stable group-by-partition (counting sort): out gets records in partition order, input
 * order within a partition; counts[num_partitions] = records per partition. */
void orc_stable_scatter(const void *records, int64_t n, int32_t record_bytes, const int32_t *pids,
                        int32_t num_partitions, void *out, int64_t *counts);

/* Whole map-side write (partition ids + stable scatter), multi-threaded over nthreads
 * (nthreads <= 1: single-threaded).  counts[num_partitions] in records. */
int orc_map_write(const void *records, int64_t n, int32_t record_bytes, int32_t kind,
                  int32_t num_partitions, const void *bounds, int32_t nbounds, int32_t ascending,
                  void *out, int64_t *counts, int32_t nthreads);

/* IndexShuffleBlockResolver index: (nparts+1) big-endian int64 offsets into out[]. */
void orc_index_bytes(const int64_t *lengths, int32_t nparts, uint8_t *out);
/* checkIndexAndDataFile: 0 and lengths[] filled if consistent, else -1. */
int orc_check_index(const uint8_t *index, int64_t index_len, int64_t data_len, int32_t blocks,
                    int64_t *lengths);

/* Synthetic generators (the build's definitions). */
uint64_t orc_splitmix64_at(uint64_t seed, uint64_t i);
void orc_gen_uniform16(void *records, int64_t n, uint64_t seed, int64_t value_base);
void orc_gen_terasort100(void *records, int64_t n, uint64_t seed, int64_t index_base);
/* Zipf(s) over ranks 1..K by inverse CDF: cdf[K] (doubles, cdf[K-1]==1) precomputed. */
void orc_zipf_cdf(double s, int64_t K, double *cdf);
void orc_gen_zipf16(void *records, int64_t n, uint64_t seed, int64_t value_base, const double *cdf,
                    int64_t K);

#ifdef __cplusplus
}
#endif
#endif
