/*
 * jni.h — TEST-ONLY stand-in for the JDK header, used by
 * tests/test_jni_shim.py to compile jni/gdist_jni.c where no JDK exists (this
 * image). It declares only what the shim uses, with the JNI specification's
 * types and function signatures (JNI 21: jni.h's JNINativeInterface_); the
 * function table is filled by tests/jni_harness/fake_jvm.c, a minimal
 * in-process "JVM" of arrays, strings and a pending exception. The shim is
 * built for a real JVM with the JDK's own jni.h (jni/Makefile).
 */
#ifndef GDIST_TEST_JNI_H
#define GDIST_TEST_JNI_H
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_FALSE 0
#define JNI_TRUE 1

typedef int32_t jint;
typedef int64_t jlong;
typedef signed char jbyte;
typedef unsigned char jboolean;
typedef double jdouble;
typedef jint jsize;

struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jobjectArray;
typedef jarray jbyteArray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jarray jdoubleArray;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
    jclass (JNICALL* FindClass)(JNIEnv* env, const char* name);
    jint (JNICALL* ThrowNew)(JNIEnv* env, jclass clazz, const char* msg);
    jboolean (JNICALL* ExceptionCheck)(JNIEnv* env);
    void (JNICALL* DeleteLocalRef)(JNIEnv* env, jobject obj);
    jsize (JNICALL* GetArrayLength)(JNIEnv* env, jarray array);
    jobject (JNICALL* GetObjectArrayElement)(JNIEnv* env, jobjectArray array, jsize index);
    const char* (JNICALL* GetStringUTFChars)(JNIEnv* env, jstring str, jboolean* isCopy);
    void (JNICALL* ReleaseStringUTFChars)(JNIEnv* env, jstring str, const char* chars);
    void (JNICALL* GetByteArrayRegion)(JNIEnv* env, jbyteArray array, jsize start, jsize len, jbyte* buf);
    void (JNICALL* GetIntArrayRegion)(JNIEnv* env, jintArray array, jsize start, jsize len, jint* buf);
    void (JNICALL* GetLongArrayRegion)(JNIEnv* env, jlongArray array, jsize start, jsize len, jlong* buf);
    void (JNICALL* GetDoubleArrayRegion)(JNIEnv* env, jdoubleArray array, jsize start, jsize len, jdouble* buf);
    void (JNICALL* SetIntArrayRegion)(JNIEnv* env, jintArray array, jsize start, jsize len, const jint* buf);
    void (JNICALL* SetLongArrayRegion)(JNIEnv* env, jlongArray array, jsize start, jsize len, const jlong* buf);
    void (JNICALL* SetDoubleArrayRegion)(JNIEnv* env, jdoubleArray array, jsize start, jsize len,
                                         const jdouble* buf);
};
#endif
