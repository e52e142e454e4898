/*
 * jni/stub/jni.h — NOT the JDK's jni.h.  A minimal hand-written stand-in with just the
 * types and JNIEnv functions jni/sgx_jni.c uses, so the shim can be compile-checked in an
 * image without a JDK and driven by a fake JNIEnv in the CPU tests (tests/test_jni_shim.py).
 * The function table here is NOT laid out like the JVM's; a real build uses
 * $JAVA_HOME/include/jni.h (see the build line in jni/sgx_jni.c).
 */
#ifndef SGX_JNI_STUB_H
#define SGX_JNI_STUB_H
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef jint jsize;
typedef void *jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jlongArray;
typedef jarray jintArray;
typedef jarray jbyteArray;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;

struct JNINativeInterface_ {
    void *ctx; /* the fake environment's state (tests) */
    jclass (*FindClass)(JNIEnv *env, const char *name);
    jint (*ThrowNew)(JNIEnv *env, jclass cls, const char *msg);
    void *(*GetDirectBufferAddress)(JNIEnv *env, jobject buf);
    jlong (*GetDirectBufferCapacity)(JNIEnv *env, jobject buf);
    jsize (*GetArrayLength)(JNIEnv *env, jarray a);
    jlongArray (*NewLongArray)(JNIEnv *env, jsize n);
    void (*SetLongArrayRegion)(JNIEnv *env, jlongArray a, jsize start, jsize n, const jlong *buf);
    void (*GetLongArrayRegion)(JNIEnv *env, jlongArray a, jsize start, jsize n, jlong *buf);
    void (*GetIntArrayRegion)(JNIEnv *env, jintArray a, jsize start, jsize n, jint *buf);
    void (*SetIntArrayRegion)(JNIEnv *env, jintArray a, jsize start, jsize n, const jint *buf);
    jintArray (*NewIntArray)(JNIEnv *env, jsize n);
    jbyteArray (*NewByteArray)(JNIEnv *env, jsize n);
    void (*SetByteArrayRegion)(JNIEnv *env, jbyteArray a, jsize start, jsize n, const jbyte *buf);
    void (*GetByteArrayRegion)(JNIEnv *env, jbyteArray a, jsize start, jsize n, jbyte *buf);
    const char *(*GetStringUTFChars)(JNIEnv *env, jstring s, jboolean *is_copy);
    void (*ReleaseStringUTFChars)(JNIEnv *env, jstring s, const char *chars);
};

#endif
