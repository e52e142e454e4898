/*
 * A fake JNIEnv (over jni/stub/jni.h) for driving the JNI shim jni/sgx_jni.c from ctypes on a
 * host without a JVM or a GPU (tests/test_jni_shim.py).  Java objects are small tagged
 * structs; ThrowNew records the exception class and message.  Only the natives that need no
 * device are exercised here; the device paths are the same one-line forwards and run under
 * the GPU suite through the Python binding.
 */
#include <jni.h>
#include <stdlib.h>
#include <string.h>

enum { K_LONGS = 1, K_INTS, K_BYTES, K_STRING, K_DIRECT };
typedef struct {
    int kind;
    jsize n;
    void *data;
    jlong cap;
} obj;

static char g_exc_class[256], g_exc_msg[1024];

static jclass find_class(JNIEnv *env, const char *name) {
    (void)env;
    return (jclass)name;
}
static jint throw_new(JNIEnv *env, jclass cls, const char *msg) {
    (void)env;
    strncpy(g_exc_class, (const char *)cls, sizeof g_exc_class - 1);
    strncpy(g_exc_msg, msg ? msg : "", sizeof g_exc_msg - 1);
    return 0;
}
static void *direct_addr(JNIEnv *env, jobject b) {
    (void)env;
    obj *o = (obj *)b;
    return o && o->kind == K_DIRECT ? o->data : NULL;
}
static jlong direct_cap(JNIEnv *env, jobject b) {
    (void)env;
    obj *o = (obj *)b;
    return o && o->kind == K_DIRECT ? o->cap : -1;
}
static jsize array_len(JNIEnv *env, jarray a) {
    (void)env;
    return ((obj *)a)->n;
}
static obj *new_obj(int kind, jsize n, size_t elem) {
    obj *o = (obj *)calloc(1, sizeof(obj));
    o->kind = kind;
    o->n = n;
    o->data = calloc((size_t)n + 1, elem);
    return o;
}
static jlongArray new_longs(JNIEnv *env, jsize n) {
    (void)env;
    return new_obj(K_LONGS, n, 8);
}
static void set_longs(JNIEnv *env, jlongArray a, jsize s, jsize n, const jlong *b) {
    (void)env;
    memcpy((jlong *)((obj *)a)->data + s, b, (size_t)n * 8);
}
static void get_longs(JNIEnv *env, jlongArray a, jsize s, jsize n, jlong *b) {
    (void)env;
    memcpy(b, (jlong *)((obj *)a)->data + s, (size_t)n * 8);
}
static jintArray new_ints(JNIEnv *env, jsize n) {
    (void)env;
    return new_obj(K_INTS, n, 4);
}
static void get_ints(JNIEnv *env, jintArray a, jsize s, jsize n, jint *b) {
    (void)env;
    memcpy(b, (jint *)((obj *)a)->data + s, (size_t)n * 4);
}
static void set_ints(JNIEnv *env, jintArray a, jsize s, jsize n, const jint *b) {
    (void)env;
    memcpy((jint *)((obj *)a)->data + s, b, (size_t)n * 4);
}
static jbyteArray new_bytes(JNIEnv *env, jsize n) {
    (void)env;
    return new_obj(K_BYTES, n, 1);
}
static void set_bytes(JNIEnv *env, jbyteArray a, jsize s, jsize n, const jbyte *b) {
    (void)env;
    memcpy((jbyte *)((obj *)a)->data + s, b, (size_t)n);
}
static void get_bytes(JNIEnv *env, jbyteArray a, jsize s, jsize n, jbyte *b) {
    (void)env;
    memcpy(b, (jbyte *)((obj *)a)->data + s, (size_t)n);
}
static const char *utf(JNIEnv *env, jstring s, jboolean *c) {
    (void)env;
    if (c) *c = 0;
    return (const char *)((obj *)s)->data;
}
static void release_utf(JNIEnv *env, jstring s, const char *p) {
    (void)env;
    (void)s;
    (void)p;
}

static const struct JNINativeInterface_ g_table = {
    NULL,      find_class, throw_new, direct_addr, direct_cap, array_len, new_longs, set_longs,
    get_longs, get_ints,   set_ints,  new_ints,    new_bytes,  set_bytes, get_bytes, utf,      release_utf};
static JNIEnv g_env = &g_table;

/* natives of jni/sgx_jni.c (declared here: the shim has no header of its own) */
jlongArray Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_checkIndexAndData(JNIEnv *, jclass, jstring, jstring, jint);
jlongArray Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_indexBlockRange(JNIEnv *, jclass, jstring, jint, jint);
jlongArray Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_writeMap(JNIEnv *, jclass, jlong, jint, jlong, jobject, jlong,
                                                                   jint, jint);
jlongArray Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_fetchBlocks(JNIEnv *, jclass, jlong, jint, jlongArray,
                                                                      jintArray, jobject);
jbyteArray Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_bootstrapJoin(JNIEnv *, jclass, jstring, jint, jint, jint,
                                                                        jintArray);
void Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_bootstrapServe(JNIEnv *, jclass, jint, jint, jbyteArray, jint);
void Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_exchange(JNIEnv *, jclass, jlong, jint);
void Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_exchangeMaps(JNIEnv *, jclass, jlong, jint, jlongArray);
void Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_setMapWriter(JNIEnv *, jclass, jlong, jint, jint);
jintArray Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_shuffleReducers(JNIEnv *, jclass, jlong, jint);
jlong Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_importBlocks(JNIEnv *, jclass, jlong, jint, jlongArray, jint, jint,
                                                                   jobject, jlongArray);
void Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_exchangeFail(JNIEnv *, jclass, jlong, jint);

static obj *jstr(const char *s) {
    obj *o = (obj *)calloc(1, sizeof(obj));
    o->kind = K_STRING;
    o->data = (void *)s;
    return o;
}

/* ---- entry points for ctypes: return a value, and the pending exception (class, message) ---- */
const char *fake_exception_class(void) { return g_exc_class; }
const char *fake_exception_message(void) { return g_exc_msg; }
void fake_clear(void) {
    g_exc_class[0] = 0;
    g_exc_msg[0] = 0;
}

/* checkIndexAndData: number of lengths copied to out, -1 for Java null */
int fake_check_index(const char *index, const char *data, int blocks, int64_t *out) {
    obj *r = (obj *)Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_checkIndexAndData(&g_env, NULL, jstr(index),
                                                                                     jstr(data), blocks);
    if (!r) return -1;
    memcpy(out, r->data, (size_t)r->n * 8);
    return r->n;
}

int fake_index_block_range(const char *index, int start, int end, int64_t *out2) {
    obj *r = (obj *)Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_indexBlockRange(&g_env, NULL, jstr(index), start,
                                                                                   end);
    if (!r) return -1;
    memcpy(out2, r->data, 16);
    return 0;
}

/* writeMap with an engine handle, a direct buffer of `cap` bytes and R partitions */
int fake_write_map(int64_t engine, void *records, int64_t cap, int64_t n, int R) {
    obj buf = {K_DIRECT, 0, records, cap};
    obj *r = (obj *)Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_writeMap(&g_env, NULL, engine, 1, 0, &buf, n, 16, R);
    return r ? r->n : -1;
}

int fake_fetch_mismatched(int64_t engine) {
    obj *m = new_obj(K_LONGS, 3, 8), *r = new_obj(K_INTS, 2, 4);
    obj *res = (obj *)Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_fetchBlocks(&g_env, NULL, engine, 1, m, r, NULL);
    return res ? res->n : -1;
}

/* importBlocks of 2 maps x reducers [0, r1) with nlen lengths of 16 B each over a direct
 * buffer of cap bytes: the import id, or -1 (an exception is pending) */
int64_t fake_import_blocks(int64_t engine, void *data, int64_t cap, int r1, int nlen) {
    obj buf = {K_DIRECT, 0, data, cap};
    obj *m = new_obj(K_LONGS, 2, 8), *l = new_obj(K_LONGS, nlen, 8);
    ((int64_t *)m->data)[0] = 1;
    ((int64_t *)m->data)[1] = 2;
    for (int i = 0; i < nlen; ++i) ((int64_t *)l->data)[i] = 16;
    const jlong id = Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_importBlocks(&g_env, NULL, engine, 1, m, 0, r1,
                                                                                   &buf, l);
    return g_exc_class[0] ? -1 : id;
}

int fake_exchange_fail(int64_t engine, int R) {
    Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_exchangeFail(&g_env, NULL, engine, R);
    return 0;
}

int fake_exchange(int64_t engine) {
    Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_exchange(&g_env, NULL, engine, 1);
    return 0;
}

int fake_set_map_writer(int64_t engine, int writer) {
    Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_setMapWriter(&g_env, NULL, engine, 1, writer);
    return 0;
}

/* exchangeMaps with n map ids 0..n-1 (an empty array included) */
int fake_exchange_maps(int64_t engine, int n) {
    obj *m = new_obj(K_LONGS, n, 8);
    for (int i = 0; i < n; ++i) ((int64_t *)m->data)[i] = i;
    Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_exchangeMaps(&g_env, NULL, engine, 1, m);
    return 0;
}

/* shuffleReducers: 0 and r0, r1 in out2, or -1 for Java null (an exception is pending) */
int fake_shuffle_reducers(int64_t engine, int32_t *out2) {
    obj *r = (obj *)Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_shuffleReducers(&g_env, NULL, engine, 1);
    if (!r) return -1;
    memcpy(out2, r->data, 8);
    return 0;
}

/* bootstrapJoin against nothing listening: the timeout must surface as SgxFetchException */
int fake_bootstrap_join(const char *host, int port, int rank, int timeout_ms, uint8_t *id_out, int *nranks_out) {
    obj *nr = new_obj(K_INTS, 1, 4);
    obj *r = (obj *)Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_bootstrapJoin(&g_env, NULL, jstr(host), port, rank,
                                                                                 timeout_ms, nr);
    if (!r) return -1;
    memcpy(id_out, r->data, 128);
    *nranks_out = *(jint *)nr->data;
    return 0;
}

void fake_bootstrap_serve(int port, int nranks, const uint8_t *id, int timeout_ms) {
    obj *b = new_obj(K_BYTES, 128, 1);
    memcpy(b->data, id, 128);
    Java_org_apache_spark_shuffle_ucx_gpu_SgxNative_bootstrapServe(&g_env, NULL, port, nranks, b, timeout_ms);
}
