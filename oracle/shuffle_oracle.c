/*
 * shuffle_oracle.c — CPU restatement of Spark 3.0.1 map-side shuffle semantics.
 *
 * TEST INFRASTRUCTURE ONLY (see shuffle_oracle.h).  Pure C99 + pthreads, built by
 * oracle/Makefile into oracle/liboracle.so.  Each function cites what it restates:
 *   - java.lang.Long.hashCode (JDK 8)                       -> orc_java_long_hash
 *   - org.apache.spark.util.Utils.nonNegativeMod (3.0.1)    -> orc_non_negative_mod
 *   - HashPartitioner.getPartition (3.0.1), called per record by the SortShuffleWriter
 *     that spark_3_0/UcxShuffleManager.scala:48-51 builds     -> orc_hash_partition
 *   - RangePartitioner.getPartition (3.0.1) + JDK Arrays.binarySearch -> orc_range_*
 *   - ExternalSorter / ShuffleInMemorySorter stable grouping -> orc_stable_scatter
 *   - IndexShuffleBlockResolver.scala:161-217 (index) and :110-149 (validation)
 */
#include "shuffle_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

int32_t orc_java_long_hash(int64_t v) {
    uint64_t u = (uint64_t)v;
    return (int32_t)(uint32_t)(u ^ (u >> 32));
}

int32_t orc_non_negative_mod(int32_t x, int32_t mod) {
    int32_t raw = x % mod; /* C99 '%' truncates toward zero, as Java's does */
    return raw + (raw < 0 ? mod : 0);
}

int32_t orc_hash_partition(int64_t key, int32_t num_partitions) {
    return orc_non_negative_mod(orc_java_long_hash(key), num_partitions);
}

/* JDK 8 Arrays.binarySearch0(long[], 0, len, key). */
static int32_t java_binary_search_i64(const int64_t *a, int32_t len, int64_t key) {
    int32_t low = 0, high = len - 1;
    while (low <= high) {
        int32_t mid = (int32_t)(((uint32_t)low + (uint32_t)high) >> 1);
        int64_t mv = a[mid];
        if (mv < key) low = mid + 1;
        else if (mv > key) high = mid - 1;
        else return mid;
    }
    return -(low + 1);
}

int32_t orc_range_partition_i64(int64_t key, const int64_t *bounds, int32_t nb, int32_t ascending) {
    int32_t p = 0;
    if (nb <= 128) {
        while (p < nb && key > bounds[p]) p++; /* ordering.gt(k, rangeBounds(partition)) */
    } else {
        p = java_binary_search_i64(bounds, nb, key);
        if (p < 0) p = -p - 1;
        if (p > nb) p = nb;
    }
    return ascending ? p : nb - p;
}

static int cmp_bytes(const uint8_t *a, const uint8_t *b, int32_t klen) {
    for (int32_t i = 0; i < klen; i++) {
        if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
    }
    return 0;
}

/* Arrays.binarySearch(Object[], key, Comparator) — same loop, comparator form. */
int32_t orc_range_partition_bytes(const uint8_t *key, int32_t klen, const uint8_t *bounds,
                                  int32_t nb, int32_t ascending) {
    int32_t p = 0;
    if (nb <= 128) {
        while (p < nb && cmp_bytes(key, bounds + (int64_t)p * klen, klen) > 0) p++;
    } else {
        int32_t low = 0, high = nb - 1;
        p = -1;
        int found = 0;
        while (low <= high) {
            int32_t mid = (int32_t)(((uint32_t)low + (uint32_t)high) >> 1);
            int c = cmp_bytes(bounds + (int64_t)mid * klen, key, klen);
            if (c < 0) low = mid + 1;
            else if (c > 0) high = mid - 1;
            else { p = mid; found = 1; break; }
        }
        if (!found) p = low; /* -(-(low+1)) - 1 */
        if (p > nb) p = nb;
    }
    return ascending ? p : nb - p;
}

static inline int64_t load_i64le(const uint8_t *p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
    return (int64_t)v;
}

static inline int32_t pid_of(const uint8_t *rec, int32_t kind, int32_t R, const void *bounds,
                             int32_t nb, int32_t asc) {
    switch (kind) {
    case ORC_PART_HASH: return orc_hash_partition(load_i64le(rec), R);
    case ORC_PART_RANGE_I64: return orc_range_partition_i64(load_i64le(rec), (const int64_t *)bounds, nb, asc);
    default: return orc_range_partition_bytes(rec, 10, (const uint8_t *)bounds, nb, asc);
    }
}

void orc_partition_ids(const void *records, int64_t n, int32_t record_bytes, int32_t kind,
                       int32_t num_partitions, const void *bounds, int32_t nbounds,
                       int32_t ascending, int32_t *pids) {
    const uint8_t *r = (const uint8_t *)records;
    for (int64_t i = 0; i < n; i++)
        pids[i] = pid_of(r + i * record_bytes, kind, num_partitions, bounds, nbounds, ascending);
}

void orc_stable_scatter(const void *records, int64_t n, int32_t record_bytes, const int32_t *pids,
                        int32_t num_partitions, void *out, int64_t *counts) {
    int64_t *cursor = (int64_t *)calloc((size_t)num_partitions, sizeof(int64_t));
    memset(counts, 0, sizeof(int64_t) * (size_t)num_partitions);
    for (int64_t i = 0; i < n; i++) counts[pids[i]]++;
    int64_t run = 0;
    for (int32_t p = 0; p < num_partitions; p++) { cursor[p] = run; run += counts[p]; }
    const uint8_t *src = (const uint8_t *)records;
    uint8_t *dst = (uint8_t *)out;
    for (int64_t i = 0; i < n; i++) {
        int64_t d = cursor[pids[i]]++;
        memcpy(dst + d * record_bytes, src + i * record_bytes, (size_t)record_bytes);
    }
    free(cursor);
}

/* ---- multi-threaded map write (the CPU baseline) --------------------------------- */
typedef struct {
    const uint8_t *src; uint8_t *dst; int64_t begin, end; int32_t rb, kind, R, nb, asc;
    const void *bounds; int32_t *pids; int64_t *hist; /* hist[R] per thread */
    int64_t *cursor;                                   /* cursor[R] per thread */
} mt_task;

static void *mt_hist(void *arg) {
    mt_task *t = (mt_task *)arg;
    memset(t->hist, 0, sizeof(int64_t) * (size_t)t->R);
    for (int64_t i = t->begin; i < t->end; i++) {
        int32_t p = pid_of(t->src + i * t->rb, t->kind, t->R, t->bounds, t->nb, t->asc);
        t->pids[i] = p;
        t->hist[p]++;
    }
    return NULL;
}

static void *mt_scatter(void *arg) {
    mt_task *t = (mt_task *)arg;
    const int32_t rb = t->rb;
    for (int64_t i = t->begin; i < t->end; i++) {
        int64_t d = t->cursor[t->pids[i]]++;
        memcpy(t->dst + d * rb, t->src + i * rb, (size_t)rb);
    }
    return NULL;
}

int orc_map_write(const void *records, int64_t n, int32_t record_bytes, int32_t kind,
                  int32_t num_partitions, const void *bounds, int32_t nbounds, int32_t ascending,
                  void *out, int64_t *counts, int32_t nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (n < (int64_t)nthreads * 1024) nthreads = 1;
    const int32_t R = num_partitions;
    int32_t *pids = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    mt_task *tasks = (mt_task *)calloc((size_t)nthreads, sizeof(mt_task));
    int64_t *hist = (int64_t *)calloc((size_t)nthreads * R, sizeof(int64_t));
    int64_t *cur = (int64_t *)calloc((size_t)nthreads * R, sizeof(int64_t));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    if (!pids || !tasks || !hist || !cur || !th) return -1;
    for (int32_t t = 0; t < nthreads; t++) {
        mt_task *k = &tasks[t];
        k->src = (const uint8_t *)records; k->dst = (uint8_t *)out;
        k->begin = n * t / nthreads; k->end = n * (t + 1) / nthreads;
        k->rb = record_bytes; k->kind = kind; k->R = R; k->nb = nbounds; k->asc = ascending;
        k->bounds = bounds; k->pids = pids; k->hist = hist + (int64_t)t * R; k->cursor = cur + (int64_t)t * R;
    }
    for (int32_t t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, mt_hist, &tasks[t]);
    mt_hist(&tasks[0]);
    for (int32_t t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
    /* exclusive scan, partition-major then thread-major: stable across threads */
    int64_t run = 0;
    for (int32_t p = 0; p < R; p++) {
        int64_t c = 0;
        for (int32_t t = 0; t < nthreads; t++) {
            cur[(int64_t)t * R + p] = run;
            run += hist[(int64_t)t * R + p];
            c += hist[(int64_t)t * R + p];
        }
        counts[p] = c;
    }
    for (int32_t t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, mt_scatter, &tasks[t]);
    mt_scatter(&tasks[0]);
    for (int32_t t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
    free(pids); free(tasks); free(hist); free(cur); free(th);
    return 0;
}

/* ---- IndexShuffleBlockResolver layout --------------------------------------------- */
static void store_be64(uint8_t *p, int64_t v) {
    uint64_t u = (uint64_t)v;
    for (int i = 7; i >= 0; i--) { p[i] = (uint8_t)(u & 0xFF); u >>= 8; }
}
static int64_t load_be64(const uint8_t *p) {
    uint64_t u = 0;
    for (int i = 0; i < 8; i++) u = (u << 8) | p[i];
    return (int64_t)u;
}

void orc_index_bytes(const int64_t *lengths, int32_t nparts, uint8_t *out) {
    int64_t off = 0;
    store_be64(out, off);
    for (int32_t i = 0; i < nparts; i++) {
        off += lengths[i];
        store_be64(out + 8 * (int64_t)(i + 1), off);
    }
}

int orc_check_index(const uint8_t *index, int64_t index_len, int64_t data_len, int32_t blocks,
                    int64_t *lengths) {
    if (index_len != ((int64_t)blocks + 1) * 8) return -1;
    int64_t off = load_be64(index);
    if (off != 0) return -1;
    int64_t sum = 0;
    for (int32_t i = 0; i < blocks; i++) {
        int64_t nx = load_be64(index + 8 * (int64_t)(i + 1));
        lengths[i] = nx - off;
        sum += lengths[i];
        off = nx;
    }
    return data_len == sum ? 0 : -1;
}

/* ---- generators --------------------------------------------------------------------- */
uint64_t orc_splitmix64_at(uint64_t seed, uint64_t i) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static void store_le64(uint8_t *p, uint64_t v) {
    for (int i = 0; i < 8; i++) { p[i] = (uint8_t)(v & 0xFF); v >>= 8; }
}

void orc_gen_uniform16(void *records, int64_t n, uint64_t seed, int64_t value_base) {
    uint8_t *r = (uint8_t *)records;
    for (int64_t i = 0; i < n; i++) {
        store_le64(r + 16 * i, orc_splitmix64_at(seed, (uint64_t)i));
        store_le64(r + 16 * i + 8, (uint64_t)(value_base + i));
    }
}

void orc_gen_terasort100(void *records, int64_t n, uint64_t seed, int64_t index_base) {
    uint8_t *r = (uint8_t *)records;
    for (int64_t i = 0; i < n; i++) {
        uint8_t *rec = r + 100 * i;
        uint8_t tmp[8];
        store_le64(rec, orc_splitmix64_at(seed, 2 * (uint64_t)i));
        store_le64(tmp, orc_splitmix64_at(seed, 2 * (uint64_t)i + 1));
        rec[8] = tmp[0]; rec[9] = tmp[1];
        store_le64(rec + 10, (uint64_t)(index_base + i));
        for (int j = 18; j < 100; j++) rec[j] = (uint8_t)((uint64_t)(index_base + i) + (uint64_t)j);
    }
}

void orc_zipf_cdf(double s, int64_t K, double *cdf) {
    double h = 0.0;
    for (int64_t k = 1; k <= K; k++) { h += pow((double)k, -s); cdf[k - 1] = h; }
    for (int64_t k = 0; k < K; k++) cdf[k] /= h;
    cdf[K - 1] = 1.0;
}

void orc_gen_zipf16(void *records, int64_t n, uint64_t seed, int64_t value_base, const double *cdf,
                    int64_t K) {
    uint8_t *r = (uint8_t *)records;
    for (int64_t i = 0; i < n; i++) {
        double u = (double)(orc_splitmix64_at(seed, (uint64_t)i) >> 11) * 0x1.0p-53;
        int64_t lo = 0, hi = K - 1; /* first k with cdf[k] > u */
        while (lo < hi) {
            int64_t mid = (lo + hi) >> 1;
            if (cdf[mid] > u) hi = mid; else lo = mid + 1;
        }
        store_le64(r + 16 * i, (uint64_t)(lo + 1));
        store_le64(r + 16 * i + 8, (uint64_t)(value_base + i));
    }
}
