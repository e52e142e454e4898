/*
 * sgx_jni.c — the JNI shim between the Scala plugin classes (jvm/) and libsgx.so
 * (include/sgx.h).  Built against the JDK's <jni.h> into libsgxjni.so, which links
 * libsgx.so:
 *
 *   cc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *      jni/sgx_jni.c -Lsparkucx_amd -lsgx -Wl,-rpath,'$ORIGIN' -o libsgxjni.so
 *
 * This image has no JDK: the CPU suite compiles this file against jni/stub/jni.h (a minimal
 * hand-written stand-in for syntax checking and for a fake JNIEnv in tests, NOT a JDK
 * header) and drives the natives that need no GPU (tests/test_jni_shim.py).
 *
 * Every native forwards to one C-ABI call.  Arrays sized by the shuffle's partition count
 * are allocated from the R the caller passes (the Scala side keeps the dependency's
 * numPartitions); host records / destinations are direct ByteBuffers (pinned by the
 * executor's allocator).  A negative SGX_ERR_* becomes a Java exception carrying
 * sgx_last_error():
 *   SGX_ERR_INVALID      java.lang.IllegalArgumentException
 *   SGX_ERR_STATE        java.lang.IllegalStateException
 *   SGX_ERR_IO           java.io.IOException
 *   SGX_ERR_UNSUPPORTED  java.lang.UnsupportedOperationException
 *   SGX_ERR_NOMEM        java.lang.OutOfMemoryError
 *   SGX_ERR_NOT_FOUND, SGX_ERR_COMM, SGX_ERR_TIMEOUT
 *                        org.apache.spark.shuffle.ucx.gpu.SgxFetchException -- the client
 *                        turns it into BlockFetchingListener.onBlockFetchFailure, so Spark's
 *                        FetchFailed / stage retry runs (the reference never reports a failed
 *                        fetch, spark_3_0/UcxShuffleClient.scala:36-40)
 *   anything else        java.lang.RuntimeException
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "sgx.h"

#define JNI_FN(name) Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_##name

static const char *exception_class(int rc) {
    switch (rc) {
    case SGX_ERR_INVALID: return "java/lang/IllegalArgumentException";
    case SGX_ERR_STATE: return "java/lang/IllegalStateException";
    case SGX_ERR_IO: return "java/io/IOException";
    case SGX_ERR_UNSUPPORTED: return "java/lang/UnsupportedOperationException";
    case SGX_ERR_NOMEM: return "java/lang/OutOfMemoryError";
    case SGX_ERR_NOT_FOUND:
    case SGX_ERR_COMM:
    case SGX_ERR_TIMEOUT: return "org/apache/spark/shuffle/ucx/gpu/SgxFetchException";
    default: return "java/lang/RuntimeException";
    }
}

/* throws and returns nonzero when rc is an error */
static int check(JNIEnv *env, int rc) {
    if (rc >= 0) return 0;
    jclass cls = (*env)->FindClass(env, exception_class(rc));
    if (cls) (*env)->ThrowNew(env, cls, sgx_last_error());
    return 1;
}

static int throw_arg(JNIEnv *env, const char *msg) {
    jclass cls = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
    if (cls) (*env)->ThrowNew(env, cls, msg);
    return 1;
}

static sgx_engine *E(jlong h) { return (sgx_engine *)(intptr_t)h; }

/* a long[] of map ids as a C array (n + 1 entries, so an empty list is not NULL); free() it */
static int64_t *map_list(JNIEnv *env, jlongArray maps, jsize *n) {
    *n = (*env)->GetArrayLength(env, maps);
    int64_t *m = (int64_t *)calloc((size_t)*n + 1, sizeof(int64_t));
    if (m) (*env)->GetLongArrayRegion(env, maps, 0, *n, (jlong *)m);
    return m;
}

/* direct buffer -> (pointer, capacity in bytes); NULL buffer -> (NULL, 0) */
static int direct(JNIEnv *env, jobject buf, void **p, int64_t *cap) {
    *p = NULL;
    *cap = 0;
    if (!buf) return 0;
    *p = (*env)->GetDirectBufferAddress(env, buf);
    *cap = (int64_t)(*env)->GetDirectBufferCapacity(env, buf);
    if (!*p || *cap < 0) return throw_arg(env, "records / destination must be a direct ByteBuffer");
    return 0;
}

static jlongArray long_array(JNIEnv *env, const int64_t *v, jsize n) {
    jlongArray out = (*env)->NewLongArray(env, n);
    if (out && n) (*env)->SetLongArrayRegion(env, out, 0, n, (const jlong *)v);
    return out;
}

/* long[R] scratch for partition lengths (heap: R may be large) */
static int64_t *lengths_buf(JNIEnv *env, jint R) {
    if (R < 1) {
        throw_arg(env, "numPartitions must be positive");
        return NULL;
    }
    int64_t *p = (int64_t *)calloc((size_t)R, sizeof(int64_t));
    if (!p) {
        jclass cls = (*env)->FindClass(env, "java/lang/OutOfMemoryError");
        if (cls) (*env)->ThrowNew(env, cls, "partition lengths");
    }
    return p;
}

/* ---- engine lifetime: CommonUcxShuffleManager.startUcxTransport / stop ---- */
JNIEXPORT jlong JNICALL JNI_FN(create)(JNIEnv *env, jclass c, jint device, jint numChunks, jint flags,
                                       jint commTimeoutMs) {
    (void)c;
    sgx_config cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.device = device;
    cfg.num_chunks = numChunks;
    cfg.flags = flags;
    cfg.comm_timeout_ms = commTimeoutMs;
    sgx_engine *e = NULL;
    if (check(env, sgx_create(&cfg, &e))) return 0;
    return (jlong)(intptr_t)e;
}

JNIEXPORT void JNICALL JNI_FN(destroy)(JNIEnv *env, jclass c, jlong e) {
    (void)env;
    (void)c;
    sgx_destroy(E(e));
}

JNIEXPORT void JNICALL JNI_FN(releaseThread)(JNIEnv *env, jclass c, jlong e) {
    (void)c;
    check(env, sgx_release_thread(E(e)));
}

/* ---- registerShuffle and the dependency's properties ---- */
JNIEXPORT void JNICALL JNI_FN(registerShuffle)(JNIEnv *env, jclass c, jlong e, jint sid, jint R, jint kind,
                                               jobject bounds, jlong nbounds, jboolean ascending, jint rb) {
    (void)c;
    void *b;
    int64_t cap;
    if (direct(env, bounds, &b, &cap)) return;
    check(env, sgx_register_shuffle(E(e), sid, R, kind, b, nbounds, ascending ? 1 : 0, rb));
}

JNIEXPORT void JNICALL JNI_FN(setSerializer)(JNIEnv *env, jclass c, jlong e, jint sid, jint ser) {
    (void)c;
    check(env, sgx_set_serializer(E(e), sid, ser));
}

JNIEXPORT void JNICALL JNI_FN(setCompression)(JNIEnv *env, jclass c, jlong e, jint sid, jint codec, jint block) {
    (void)c;
    check(env, sgx_set_compression(E(e), sid, codec, block));
}

JNIEXPORT void JNICALL JNI_FN(setMapSideCombine)(JNIEnv *env, jclass c, jlong e, jint sid, jint agg) {
    (void)c;
    check(env, sgx_set_map_side_combine(E(e), sid, agg));
}

/* the map writer of the shuffle's handle (SGX_WRITER_SORT / SGX_WRITER_UNSAFE) */
JNIEXPORT void JNICALL JNI_FN(setMapWriter)(JNIEnv *env, jclass c, jlong e, jint sid, jint writer) {
    (void)c;
    check(env, sgx_set_map_writer(E(e), sid, writer));
}

JNIEXPORT void JNICALL JNI_FN(unregisterShuffle)(JNIEnv *env, jclass c, jlong e, jint sid) {
    (void)c;
    check(env, sgx_unregister_shuffle(E(e), sid));
}

/* ---- getWriter().write(records) + commitAllPartitions(): long[R] lengths ---- */
JNIEXPORT jlongArray JNICALL JNI_FN(writeMap)(JNIEnv *env, jclass c, jlong e, jint sid, jlong mapId,
                                              jobject records, jlong n, jint rb, jint R) {
    (void)c;
    void *p;
    int64_t cap;
    if (direct(env, records, &p, &cap)) return NULL;
    if (n < 0 || n * (int64_t)rb > cap) {
        throw_arg(env, "records buffer holds fewer than nrecords records");
        return NULL;
    }
    int64_t *len = lengths_buf(env, R);
    if (!len) return NULL;
    jlongArray out = NULL;
    if (!check(env, sgx_write_map(E(e), sid, mapId, p, n, rb, SGX_MEM_HOST, len))) out = long_array(env, len, R);
    free(len);
    return out;
}

/* streaming map output: one call per spill, then the commit */
JNIEXPORT void JNICALL JNI_FN(mapBegin)(JNIEnv *env, jclass c, jlong e, jint sid, jlong mapId) {
    (void)c;
    check(env, sgx_map_begin(E(e), sid, mapId));
}

JNIEXPORT void JNICALL JNI_FN(mapAppend)(JNIEnv *env, jclass c, jlong e, jint sid, jlong mapId, jobject records,
                                         jlong n, jint rb) {
    (void)c;
    void *p;
    int64_t cap;
    if (direct(env, records, &p, &cap)) return;
    if (n < 0 || n * (int64_t)rb > cap) {
        throw_arg(env, "records buffer holds fewer than nrecords records");
        return;
    }
    check(env, sgx_map_append(E(e), sid, mapId, p, n, rb, SGX_MEM_HOST));
}

JNIEXPORT jlongArray JNICALL JNI_FN(mapCommit)(JNIEnv *env, jclass c, jlong e, jint sid, jlong mapId, jint R) {
    (void)c;
    int64_t *len = lengths_buf(env, R);
    if (!len) return NULL;
    jlongArray out = NULL;
    if (!check(env, sgx_map_commit(E(e), sid, mapId, len))) out = long_array(env, len, R);
    free(len);
    return out;
}

/* ---- IndexShuffleBlockResolver ---- */
JNIEXPORT jlongArray JNICALL JNI_FN(writeIndex)(JNIEnv *env, jclass c, jlong e, jint sid, jlong mapId,
                                                jstring index, jstring data, jint R) {
    (void)c;
    int64_t *len = lengths_buf(env, R);
    if (!len) return NULL;
    const char *ip = (*env)->GetStringUTFChars(env, index, NULL);
    const char *dp = (*env)->GetStringUTFChars(env, data, NULL);
    jlongArray out = NULL;
    if (ip && dp && !check(env, sgx_write_index(E(e), sid, mapId, ip, dp, len))) out = long_array(env, len, R);
    if (ip) (*env)->ReleaseStringUTFChars(env, index, ip);
    if (dp) (*env)->ReleaseStringUTFChars(env, data, dp);
    free(len);
    return out;
}

/* checkIndexAndDataFile: the lengths, or null when index and data do not match */
JNIEXPORT jlongArray JNICALL JNI_FN(checkIndexAndData)(JNIEnv *env, jclass c, jstring index, jstring data,
                                                       jint blocks) {
    (void)c;
    if (blocks < 0) {
        throw_arg(env, "blocks must be >= 0");
        return NULL;
    }
    int64_t *len = (int64_t *)calloc((size_t)blocks + 1, sizeof(int64_t));
    const char *ip = (*env)->GetStringUTFChars(env, index, NULL);
    const char *dp = (*env)->GetStringUTFChars(env, data, NULL);
    jlongArray out = NULL;
    if (len && ip && dp) {
        const int rc = sgx_check_index_and_data(ip, dp, blocks, len);
        if (rc == SGX_OK) out = long_array(env, len, blocks);
        else if (rc != SGX_ERR_NOT_FOUND) check(env, rc);
    }
    if (ip) (*env)->ReleaseStringUTFChars(env, index, ip);
    if (dp) (*env)->ReleaseStringUTFChars(env, data, dp);
    free(len);
    return out;
}

/* getBlockData's offset lookup: {offset, length} */
JNIEXPORT jlongArray JNICALL JNI_FN(indexBlockRange)(JNIEnv *env, jclass c, jstring index, jint start, jint end) {
    (void)c;
    const char *ip = (*env)->GetStringUTFChars(env, index, NULL);
    int64_t r[3] = {0, 0, 0};
    jlongArray out = NULL;
    if (ip && !check(env, sgx_index_block_range(ip, start, end, &r[0], &r[1]))) out = long_array(env, r, 2);
    if (ip) (*env)->ReleaseStringUTFChars(env, index, ip);
    return out;
}

/* ---- the exchange: communicator id, bootstrap, collective push ---- */
JNIEXPORT jbyteArray JNICALL JNI_FN(uniqueId)(JNIEnv *env, jclass c) {
    (void)c;
    uint8_t id[128];
    if (check(env, sgx_get_unique_id(id))) return NULL;
    jbyteArray out = (*env)->NewByteArray(env, 128);
    if (out) (*env)->SetByteArrayRegion(env, out, 0, 128, (const jbyte *)id);
    return out;
}

static int id_bytes(JNIEnv *env, jbyteArray id, uint8_t out[128]) {
    if (!id || (*env)->GetArrayLength(env, id) != 128) return throw_arg(env, "the communicator id is 128 bytes");
    (*env)->GetByteArrayRegion(env, id, 0, 128, (jbyte *)out);
    return 0;
}

JNIEXPORT void JNICALL JNI_FN(commInit)(JNIEnv *env, jclass c, jlong e, jint nranks, jint rank, jbyteArray id) {
    (void)c;
    uint8_t b[128];
    if (id_bytes(env, id, b)) return;
    check(env, sgx_comm_init(E(e), nranks, rank, b));
}

JNIEXPORT void JNICALL JNI_FN(bootstrapServe)(JNIEnv *env, jclass c, jint port, jint nranks, jbyteArray id,
                                              jint timeoutMs) {
    (void)c;
    uint8_t b[128];
    if (id_bytes(env, id, b)) return;
    check(env, sgx_bootstrap_serve(port, nranks, b, timeoutMs));
}

/* returns the id; nranksOut[0] = the world size */
JNIEXPORT jbyteArray JNICALL JNI_FN(bootstrapJoin)(JNIEnv *env, jclass c, jstring host, jint port, jint rank,
                                                   jint timeoutMs, jintArray nranksOut) {
    (void)c;
    uint8_t id[128];
    int32_t nr = 0;
    const char *hp = (*env)->GetStringUTFChars(env, host, NULL);
    if (!hp) return NULL;
    const int rc = sgx_bootstrap_join(hp, port, rank, timeoutMs, id, &nr);
    (*env)->ReleaseStringUTFChars(env, host, hp);
    if (check(env, rc)) return NULL;
    if (nranksOut && (*env)->GetArrayLength(env, nranksOut) >= 1)
        (*env)->SetIntArrayRegion(env, nranksOut, 0, 1, (const jint *)&nr);
    jbyteArray out = (*env)->NewByteArray(env, 128);
    if (out) (*env)->SetByteArrayRegion(env, out, 0, 128, (const jbyte *)id);
    return out;
}

/* the shuffle's exchange (collective: every executor calls it, see GpuExchangeCoordinator) */
JNIEXPORT void JNICALL JNI_FN(exchange)(JNIEnv *env, jclass c, jlong e, jint sid) {
    (void)c;
    check(env, sgx_exchange(E(e), sid));
}

/* the pipelined form: exactly these local maps (an empty array contributes nothing) */
JNIEXPORT void JNICALL JNI_FN(exchangeMaps)(JNIEnv *env, jclass c, jlong e, jint sid, jlongArray maps) {
    (void)c;
    jsize n;
    int64_t *m = map_list(env, maps, &n);
    if (!m) return;
    const int rc = sgx_exchange_maps(E(e), sid, m, n);
    free(m);
    check(env, rc);
}

/* a round this executor cannot take part in (it failed before the exchange): join its first
 * all-gather marked failed, so every rank fails the round together (sgx_exchange_fail) */
JNIEXPORT void JNICALL JNI_FN(exchangeFail)(JNIEnv *env, jclass c, jlong e, jint numPartitions) {
    (void)c;
    check(env, sgx_exchange_fail(E(e), numPartitions, SGX_ERR_STATE));
}

/* the executor's reducers [r0, r1) of the shuffle (fixed by its first exchange): int[2] */
JNIEXPORT jintArray JNICALL JNI_FN(shuffleReducers)(JNIEnv *env, jclass c, jlong e, jint sid) {
    (void)c;
    int32_t r[2] = {0, 0};
    if (check(env, sgx_shuffle_reducers(E(e), sid, &r[0], &r[1]))) return NULL;
    jintArray out = (*env)->NewIntArray(env, 2);
    if (out) (*env)->SetIntArrayRegion(env, out, 0, 2, (const jint *)r);
    return out;
}

JNIEXPORT void JNICALL JNI_FN(setReducerPlacement)(JNIEnv *env, jclass c, jlong e, jint sid, jint placement) {
    (void)c;
    check(env, sgx_set_reducer_placement(E(e), sid, placement));
}

/* the executor's reducers [r0, r1) for the exchange round that carried mapId: int[2] */
JNIEXPORT jintArray JNICALL JNI_FN(roundReducers)(JNIEnv *env, jclass c, jlong e, jint sid, jlong mapId) {
    (void)c;
    int32_t r[2] = {0, 0};
    if (check(env, sgx_round_reducers(E(e), sid, mapId, &r[0], &r[1]))) return NULL;
    jintArray out = (*env)->NewIntArray(env, 2);
    if (out) (*env)->SetIntArrayRegion(env, out, 0, 2, (const jint *)r);
    return out;
}

/* ---- fetchBlocksByBlockIds: blocks back to back into dst; returns long[n] lengths.  dst null
 *      (or too small) with a SGX_ERR_INVALID is a size query: the lengths are still returned. */
JNIEXPORT jlongArray JNICALL JNI_FN(fetchBlocks)(JNIEnv *env, jclass c, jlong e, jint sid, jlongArray mapIds,
                                                 jintArray reduceIds, jobject dst) {
    (void)c;
    const jsize n = (*env)->GetArrayLength(env, mapIds);
    if ((*env)->GetArrayLength(env, reduceIds) != n) {
        throw_arg(env, "mapIds and reduceIds differ in length");
        return NULL;
    }
    void *p;
    int64_t cap;
    if (direct(env, dst, &p, &cap)) return NULL;
    int64_t *m = (int64_t *)calloc((size_t)n + 1, sizeof(int64_t));
    int32_t *r = (int32_t *)calloc((size_t)n + 1, sizeof(int32_t));
    int64_t *len = (int64_t *)calloc((size_t)n + 1, sizeof(int64_t));
    jlongArray out = NULL;
    if (m && r && len) {
        (*env)->GetLongArrayRegion(env, mapIds, 0, n, (jlong *)m);
        (*env)->GetIntArrayRegion(env, reduceIds, 0, n, (jint *)r);
        const int rc = sgx_fetch_blocks(E(e), sid, m, r, n, p, cap, SGX_MEM_HOST, len);
        if (rc == SGX_OK || (rc == SGX_ERR_INVALID && !p)) out = long_array(env, len, n);
        else check(env, rc);
    }
    free(m);
    free(r);
    free(len);
    return out;
}

/* blocks fetched from the reducers' owners (reducer-major, map-minor in `data`, a direct
 * buffer; lengths in the same order) handed to this executor's engine: the reads then run
 * over them on this GPU (sgx_import_blocks).  Returns the import id for releaseImport. */
JNIEXPORT jlong JNICALL JNI_FN(importBlocks)(JNIEnv *env, jclass c, jlong e, jint sid, jlongArray mapIds, jint r0,
                                             jint r1, jobject data, jlongArray lengths) {
    (void)c;
    jsize n, nl;
    void *p;
    int64_t cap;
    if (direct(env, data, &p, &cap)) return 0;
    int64_t *m = map_list(env, mapIds, &n);
    int64_t *len = map_list(env, lengths, &nl);
    int64_t id = 0;
    if (m && len) {
        if ((int64_t)nl != (int64_t)n * (r1 - r0)) {
            throw_arg(env, "one length per (reducer, map) block");
        } else {
            int64_t total = 0;
            for (jsize i = 0; i < nl; ++i) total += len[i];
            if (total > cap) throw_arg(env, "lengths exceed the data buffer");
            else check(env, sgx_import_blocks(E(e), sid, m, n, r0, r1, p, SGX_MEM_HOST, len, &id));
        }
    }
    free(m);
    free(len);
    return (jlong)id;
}

JNIEXPORT void JNICALL JNI_FN(releaseImport)(JNIEnv *env, jclass c, jlong e, jint sid, jlong importId) {
    (void)c;
    check(env, sgx_release_import(E(e), sid, importId));
}

JNIEXPORT jint JNICALL JNI_FN(progress)(JNIEnv *env, jclass c, jlong e) {
    (void)c;
    const int rc = sgx_progress(E(e));
    check(env, rc);
    return rc;
}

JNIEXPORT void JNICALL JNI_FN(sync)(JNIEnv *env, jclass c, jlong e) {
    (void)c;
    check(env, sgx_sync(E(e)));
}

/* ---- reduce side after the fetch ---- */

/* readRecords / readSorted: bytes written (dst null = size query) */
JNIEXPORT jlong JNICALL JNI_FN(readRecords)(JNIEnv *env, jclass c, jlong e, jint sid, jlongArray maps, jint start,
                                            jint end, jobject dst) {
    (void)c;
    void *p;
    int64_t cap, bytes = 0;
    jsize n;
    if (direct(env, dst, &p, &cap)) return -1;
    int64_t *m = map_list(env, maps, &n);
    if (!m) return -1;
    const int rc = sgx_read_records(E(e), sid, m, n, start, end, p, cap, SGX_MEM_HOST, &bytes);
    free(m);
    return check(env, rc) ? -1 : bytes;
}

JNIEXPORT jlong JNICALL JNI_FN(readSorted)(JNIEnv *env, jclass c, jlong e, jint sid, jlongArray maps, jint start,
                                           jint end, jobject dst) {
    (void)c;
    void *p;
    int64_t cap, bytes = 0;
    jsize n;
    if (direct(env, dst, &p, &cap)) return -1;
    int64_t *m = map_list(env, maps, &n);
    if (!m) return -1;
    const int rc = sgx_read_sorted(E(e), sid, m, n, start, end, p, cap, SGX_MEM_HOST, &bytes);
    free(m);
    return check(env, rc) ? -1 : bytes;
}

/* readGrouped: {groups, values, records}; agg 0 = groupByKey (keys, groupStarts, values), 1 = sum
 * (keys, sums in values); records = the shuffled records the aggregation consumed (the reader's
 * incRecordsRead).  Null buffers with their capacities 0 = size query. */
JNIEXPORT jlongArray JNICALL JNI_FN(readGrouped)(JNIEnv *env, jclass c, jlong e, jint sid, jlongArray maps,
                                                 jint start, jint end, jint agg, jobject keys, jobject starts,
                                                 jobject values) {
    (void)c;
    void *kp, *sp, *vp;
    int64_t kc, sc, vc;
    if (direct(env, keys, &kp, &kc) || direct(env, starts, &sp, &sc) || direct(env, values, &vp, &vc)) return NULL;
    jsize n;
    int64_t *m = map_list(env, maps, &n);
    if (!m) return NULL;
    int64_t r[3] = {0, 0, 0};
    /* group_starts receives as many entries as keys: the smaller buffer bounds both */
    const int64_t cap_groups = kp ? (sp && sc < kc ? sc : kc) / 8 : 0, cap_values = vp ? vc / 8 : 0;
    const int rc = sgx_read_grouped(E(e), sid, m, n, start, end, agg, (int64_t *)kp, (int64_t *)sp, (int64_t *)vp,
                                    cap_groups, cap_values, SGX_MEM_HOST, &r[0], &r[1]);
    free(m);
    if (check(env, rc) || check(env, sgx_last_read_records(E(e), &r[2]))) return NULL;
    return long_array(env, r, 3);
}
