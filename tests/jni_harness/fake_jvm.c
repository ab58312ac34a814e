/*
 * fake_jvm.c — TEST-ONLY in-process stand-in for the JVM side of JNI, so
 * tests/test_jni_shim.py can call the natives of jni/gdist_jni.c through
 * ctypes. Objects are heap records (arrays of one primitive kind, object
 * arrays, strings, classes); a region call outside an array throws
 * ArrayIndexOutOfBoundsException as the JVM does; ThrowNew leaves one pending
 * exception (class name + message) that the test reads and clears. Local
 * references are counted so the test can see DeleteLocalRef pairing.
 */
#include <stdlib.h>
#include <string.h>

#include "jni.h"

enum { K_BYTE = 1, K_INT, K_LONG, K_DOUBLE, K_OBJECT, K_STRING, K_CLASS };

struct _jobject {
    int kind;
    jsize len;
    void* data;          /* elements; K_STRING / K_CLASS: the NUL-terminated text */
};

static char g_exc_class[256];
static char g_exc_msg[4096];
static int g_pending = 0;
static long g_local_refs = 0;  /* GetObjectArrayElement minus DeleteLocalRef */

static void throw_(const char* cls, const char* msg) {
    if (g_pending) return;   /* the first exception stays pending, as in the JVM */
    g_pending = 1;
    strncpy(g_exc_class, cls, sizeof g_exc_class - 1);
    strncpy(g_exc_msg, msg ? msg : "", sizeof g_exc_msg - 1);
}

static size_t elem(int kind) {
    switch (kind) {
        case K_BYTE: return 1;
        case K_INT: return 4;
        case K_LONG: case K_DOUBLE: return 8;
        case K_OBJECT: return sizeof(jobject);
        default: return 1;
    }
}

static jobject new_obj(int kind, jsize len, const void* init) {
    jobject o = calloc(1, sizeof *o);
    o->kind = kind;
    o->len = len;
    size_t bytes = kind == K_STRING || kind == K_CLASS ? (size_t)len + 1 : (size_t)len * elem(kind);
    o->data = calloc(bytes ? bytes : 1, 1);
    if (init) memcpy(o->data, init, bytes);
    return o;
}

static int region_ok(jarray a, int kind, jsize start, jsize len) {
    if (!a || a->kind != kind) { throw_("java/lang/NullPointerException", "array"); return 0; }
    if (start < 0 || len < 0 || (int64_t)start + len > a->len) {
        throw_("java/lang/ArrayIndexOutOfBoundsException", "region");
        return 0;
    }
    return 1;
}

static jclass JNICALL FindClass(JNIEnv* env, const char* name) {
    (void)env;
    return new_obj(K_CLASS, (jsize)strlen(name), name);
}
static jint JNICALL ThrowNew(JNIEnv* env, jclass c, const char* msg) {
    (void)env;
    throw_((const char*)c->data, msg);
    return 0;
}
static jboolean JNICALL ExceptionCheck(JNIEnv* env) { (void)env; return g_pending ? JNI_TRUE : JNI_FALSE; }
static void JNICALL DeleteLocalRef(JNIEnv* env, jobject o) { (void)env; (void)o; g_local_refs--; }
static jsize JNICALL GetArrayLength(JNIEnv* env, jarray a) { (void)env; return a ? a->len : 0; }
static jobject JNICALL GetObjectArrayElement(JNIEnv* env, jobjectArray a, jsize i) {
    (void)env;
    if (!region_ok(a, K_OBJECT, i, 1)) return NULL;
    g_local_refs++;
    return ((jobject*)a->data)[i];
}
static const char* JNICALL GetStringUTFChars(JNIEnv* env, jstring s, jboolean* copy) {
    (void)env;
    if (copy) *copy = JNI_FALSE;
    return (const char*)s->data;
}
static void JNICALL ReleaseStringUTFChars(JNIEnv* env, jstring s, const char* c) { (void)env; (void)s; (void)c; }

#define REGION(Name, Kind, T, dir)                                                                  \
    static void JNICALL Name(JNIEnv* env, jarray a, jsize start, jsize len, dir T* buf) {           \
        (void)env;                                                                                  \
        if (!region_ok(a, Kind, start, len)) return;                                                \
        GDIST_COPY_##dir(a, buf, start, len, T);                                                    \
    }
#define GDIST_COPY_(a, buf, start, len, T) memcpy(buf, (T*)(a)->data + (start), (size_t)(len) * sizeof(T))
#define GDIST_COPY_const(a, buf, start, len, T) memcpy((T*)(a)->data + (start), buf, (size_t)(len) * sizeof(T))
REGION(GetByteArrayRegion, K_BYTE, jbyte, )
REGION(GetIntArrayRegion, K_INT, jint, )
REGION(GetLongArrayRegion, K_LONG, jlong, )
REGION(GetDoubleArrayRegion, K_DOUBLE, jdouble, )
REGION(SetIntArrayRegion, K_INT, jint, const)
REGION(SetLongArrayRegion, K_LONG, jlong, const)
REGION(SetDoubleArrayRegion, K_DOUBLE, jdouble, const)

static const struct JNINativeInterface_ g_table = {
    FindClass, ThrowNew, ExceptionCheck, DeleteLocalRef, GetArrayLength, GetObjectArrayElement,
    GetStringUTFChars, ReleaseStringUTFChars, GetByteArrayRegion, GetIntArrayRegion, GetLongArrayRegion,
    GetDoubleArrayRegion,
    SetIntArrayRegion, SetLongArrayRegion, SetDoubleArrayRegion,
};
static JNIEnv g_env = &g_table;

/* ---- the test's side (ctypes) ---------------------------------------------- */
JNIEXPORT JNIEnv* fj_env(void) { return &g_env; }
JNIEXPORT jobject fj_array(int kind, jsize len, const void* init) { return new_obj(kind, len, init); }
JNIEXPORT void* fj_data(jobject o) { return o->data; }
JNIEXPORT jobject fj_string(const char* s) { return new_obj(K_STRING, (jsize)strlen(s), s); }
JNIEXPORT void fj_set_element(jobject arr, jsize i, jobject v) { ((jobject*)arr->data)[i] = v; }
JNIEXPORT int fj_pending(void) { return g_pending; }
JNIEXPORT const char* fj_exception_class(void) { return g_pending ? g_exc_class : ""; }
JNIEXPORT const char* fj_exception_message(void) { return g_pending ? g_exc_msg : ""; }
JNIEXPORT void fj_clear(void) { g_pending = 0; g_exc_class[0] = g_exc_msg[0] = 0; }
JNIEXPORT long fj_local_refs(void) { return g_local_refs; }
