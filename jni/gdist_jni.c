/*
 * gdist_jni.c — JNI shim between the Java host (org.theseed.genome.distance)
 * and libgdist.so (include/gdist.h). Build where a JDK exists (jni/Makefile);
 * this image has none, so tests/test_jni_shim.py checks every gdist_* call
 * here against the declarations of include/gdist.h instead.
 *
 * Rules kept by every native:
 *   - no JVM array is held (GetPrimitiveArrayCritical) across a library call:
 *     inputs are copied into native buffers (Get*ArrayRegion) first and
 *     outputs copied back (Set*ArrayRegion) after, so a long GPU call never
 *     stalls the JVM's garbage collector;
 *   - status codes map to the exceptions the reference throws for the same
 *     failures: EINVAL -> IllegalArgumentException, ENOMEM ->
 *     OutOfMemoryError, EDEVICE / ECOMM -> IllegalStateException, with
 *     gdist_last_error() as the message;
 *   - every GetObjectArrayElement's local reference is deleted in the loop
 *     (thousands of genomes would overflow the local frame).
 * Handles are the library's pointers carried as Java longs.
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "gdist.h"

#define JFN(name) Java_org_theseed_genome_distance_gpu_GpuKmerSets_##name

static void throw_for(JNIEnv* env, int rc) {
    const char* cls = rc == GDIST_EINVAL ? "java/lang/IllegalArgumentException"
                    : rc == GDIST_ENOMEM ? "java/lang/OutOfMemoryError"
                                         : "java/lang/IllegalStateException";
    jclass c = (*env)->FindClass(env, cls);
    if (c) (*env)->ThrowNew(env, c, gdist_last_error());
}

static void throw_oom(JNIEnv* env) {
    jclass c = (*env)->FindClass(env, "java/lang/OutOfMemoryError");
    if (c) (*env)->ThrowNew(env, c, "native buffer");
}

static void throw_arg(JNIEnv* env, const char* msg) {
    jclass c = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
    if (c) (*env)->ThrowNew(env, c, msg);
}

/* the number of sets of a collection (-1 with the exception thrown) */
static int64_t nsets_of(JNIEnv* env, const gdist_sets* s) {
    int kind = 0, k = 0;
    int64_t n = 0, total = 0;
    int rc = gdist_sets_info(s, &kind, &k, &n, &total);
    if (rc) { throw_for(env, rc); return -1; }
    return n;
}

/* an array argument shorter than the collection it describes: the library
 * writes (or reads) one element per set, so it is refused up front */
static int too_short(JNIEnv* env, jarray a, int64_t n, const char* what) {
    if (a && (int64_t)(*env)->GetArrayLength(env, a) >= n) return 0;
    throw_arg(env, what);
    return 1;
}

#define CTX(h) ((gdist_ctx*)(intptr_t)(h))
#define SETS(h) ((gdist_sets*)(intptr_t)(h))

/* ---- context ------------------------------------------------------------ */
JNIEXPORT jlong JNICALL JFN(nCtxCreate)(JNIEnv* env, jclass c, jint device) {
    gdist_ctx* ctx = NULL;
    int rc = gdist_ctx_create(device, &ctx);
    if (rc) { throw_for(env, rc); return 0; }
    return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNICALL JFN(nCtxDestroy)(JNIEnv* env, jclass c, jlong ctx) {
    int rc = gdist_ctx_destroy(CTX(ctx));
    if (rc) throw_for(env, rc);
}

JNIEXPORT void JNICALL JFN(nSetOption)(JNIEnv* env, jclass c, jlong ctx, jstring name, jlong value) {
    const char* n = (*env)->GetStringUTFChars(env, name, NULL);
    if (!n) return;
    int rc = gdist_ctx_set_option(CTX(ctx), n, (int64_t)value);
    (*env)->ReleaseStringUTFChars(env, name, n);
    if (rc) throw_for(env, rc);
}

/* ---- kmer sets: KmerType.createKmers / new GenomeKmers / new ProteinKmers - */
/* The byte arrays of seqs as one buffer + int64 offsets (n + 1), copied out
 * with GetByteArrayRegion (no array pinned across a library call). Returns
 * the element count, -1 with an exception pending. */
static jsize gather_seqs(JNIEnv* env, jobjectArray seqs, char** blob_out, int64_t** off_out) {
    const jsize n = (*env)->GetArrayLength(env, seqs);
    int64_t* off = malloc(((size_t)n + 1) * sizeof(int64_t));
    if (!off) { throw_oom(env); return -1; }
    off[0] = 0;
    for (jsize i = 0; i < n; i++) {
        jbyteArray a = (*env)->GetObjectArrayElement(env, seqs, i);
        off[i + 1] = off[i] + (a ? (*env)->GetArrayLength(env, a) : 0);
        if (a) (*env)->DeleteLocalRef(env, a);
    }
    char* blob = malloc((size_t)off[n] + 1);
    if (!blob) { free(off); throw_oom(env); return -1; }
    for (jsize i = 0; i < n; i++) {
        jbyteArray a = (*env)->GetObjectArrayElement(env, seqs, i);
        if (a) {
            (*env)->GetByteArrayRegion(env, a, 0, (jsize)(off[i + 1] - off[i]), (jbyte*)blob + off[i]);
            (*env)->DeleteLocalRef(env, a);
            if ((*env)->ExceptionCheck(env)) { free(blob); free(off); return -1; }
        }
    }
    *blob_out = blob;
    *off_out = off;
    return n;
}

JNIEXPORT jlong JNICALL JFN(nPack)(JNIEnv* env, jclass c, jlong ctx, jint kind, jint k, jint flags,
                                   jobjectArray seqs) {
    char* blob = NULL;
    int64_t* off = NULL;
    const jsize n = gather_seqs(env, seqs, &blob, &off);
    if (n < 0) return 0;
    gdist_sets* s = NULL;
    int rc = gdist_sets_pack(CTX(ctx), kind, k, (unsigned)flags, blob, off, n, &s);
    free(blob);
    free(off);
    if (rc) { throw_for(env, rc); return 0; }
    return (jlong)(intptr_t)s;
}

/* more sequences packed into an existing collection (a genome cache that
 * packs each genome once): the index of the first new set */
JNIEXPORT jlong JNICALL JFN(nAppend)(JNIEnv* env, jclass c, jlong ctx, jlong sets, jobjectArray seqs) {
    char* blob = NULL;
    int64_t* off = NULL;
    const jsize n = gather_seqs(env, seqs, &blob, &off);
    if (n < 0) return 0;
    int64_t first = 0;
    int rc = gdist_sets_append(CTX(ctx), SETS(sets), blob, off, n, &first);
    free(blob);
    free(off);
    if (rc) { throw_for(env, rc); return 0; }
    return (jlong)first;
}

JNIEXPORT jlong JNICALL JFN(nConcat)(JNIEnv* env, jclass c, jlong a, jlong b) {
    gdist_sets* s = NULL;
    int rc = gdist_sets_concat(SETS(a), SETS(b), &s);
    if (rc) { throw_for(env, rc); return 0; }
    return (jlong)(intptr_t)s;
}

JNIEXPORT void JNICALL JFN(nFree)(JNIEnv* env, jclass c, jlong sets) {
    int rc = gdist_sets_free(SETS(sets));
    if (rc) throw_for(env, rc);
}

JNIEXPORT jlong JNICALL JFN(nSize)(JNIEnv* env, jclass c, jlong sets) {
    int kind = 0, k = 0;
    int64_t n = 0, total = 0;
    int rc = gdist_sets_info(SETS(sets), &kind, &k, &n, &total);
    if (rc) { throw_for(env, rc); return 0; }
    return (jlong)n;
}

/* SequenceKmers.size() of every set */
JNIEXPORT void JNICALL JFN(nSizes)(JNIEnv* env, jclass c, jlong sets, jlongArray out) {
    const int64_t n = nsets_of(env, SETS(sets));
    if (n < 0 || too_short(env, out, n, "out shorter than the number of sets")) return;
    int64_t* v = malloc(((size_t)n + 1) * sizeof(int64_t));
    if (!v) { throw_oom(env); return; }
    int rc = gdist_sets_sizes(SETS(sets), v);
    if (!rc) (*env)->SetLongArrayRegion(env, out, 0, (jsize)n, (const jlong*)v);
    free(v);
    if (rc) throw_for(env, rc);
}

JNIEXPORT void JNICALL JFN(nBuildBitsets)(JNIEnv* env, jclass c, jlong sets, jint flags) {
    int rc = gdist_sets_build_bitsets(SETS(sets), (unsigned)flags);
    if (rc) throw_for(env, rc);
}

JNIEXPORT jint JNICALL JFN(nPrepare)(JNIEnv* env, jclass c, jlong ctx, jlong sets, jint method, jdouble pairs) {
    int chosen = 0;
    int rc = gdist_sets_prepare(CTX(ctx), SETS(sets), method, pairs, &chosen, NULL, NULL);
    if (rc) { throw_for(env, rc); return 0; }
    return chosen;
}

/* ---- distances: FastaDistanceProcessor / GenomeProcessor row blocks ------ */
/* out[(i - r0) * ld + (j - c0)] = distance; (r1 - r0) * ld doubles */
JNIEXPORT void JNICALL JFN(nMatrix)(JNIEnv* env, jclass c, jlong ctx, jlong sets, jlong r0, jlong r1, jlong c0,
                                    jlong c1, jint method, jint flags, jdoubleArray out, jint ld) {
    const int64_t cells = (int64_t)(r1 - r0) * (int64_t)ld;
    if (cells < 0 || (*env)->GetArrayLength(env, out) < cells) {
        jclass e = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
        if (e) (*env)->ThrowNew(env, e, "output array smaller than (r1 - r0) * ld");
        return;
    }
    double* d = malloc((size_t)(cells ? cells : 1) * sizeof(double));
    if (!d) { throw_oom(env); return; }
    /* untouched entries (j <= i with GDIST_UPPER_TRIANGLE) keep the array's values */
    (*env)->GetDoubleArrayRegion(env, out, 0, (jsize)cells, d);
    if ((*env)->ExceptionCheck(env)) { free(d); return; }
    int rc = gdist_intersect_matrix(CTX(ctx), SETS(sets), r0, r1, c0, c1, method, (unsigned)flags, NULL, d, ld);
    if (!rc) (*env)->SetDoubleArrayRegion(env, out, 0, (jsize)cells, d);
    free(d);
    if (rc) throw_for(env, rc);
}

/* NULL with an exception pending (out of memory, or the copy failed) */
static int64_t* copy_cols(JNIEnv* env, jlongArray cols, jsize* n) {
    *n = (*env)->GetArrayLength(env, cols);
    int64_t* cl = malloc(((size_t)*n + 1) * sizeof(int64_t));
    if (!cl) { throw_oom(env); return NULL; }
    (*env)->GetLongArrayRegion(env, cols, 0, *n, (jlong*)cl);
    if ((*env)->ExceptionCheck(env)) { free(cl); return NULL; }
    return cl;
}

/* anyMatch(d <= maxDist): DistanceRepsProcessor.java:190, FastaDistanceRepsProcessor.java:124-128 */
JNIEXPORT jboolean JNICALL JFN(nAnyLe)(JNIEnv* env, jclass c, jlong ctx, jlong sets, jlong q, jlongArray cols,
                                       jdouble t) {
    jsize n = 0;
    int64_t* cl = copy_cols(env, cols, &n);
    if (!cl) return JNI_FALSE;
    int32_t hit = 0;
    int rc = gdist_row_query(CTX(ctx), SETS(sets), q, cl, n, GDIST_QUERY_ANY_LE, t, NULL, &hit, NULL, NULL);
    free(cl);
    if (rc) { throw_for(env, rc); return JNI_FALSE; }
    return hit ? JNI_TRUE : JNI_FALSE;
}

/* reduce(NULL_RESULT, merge) argmin: DistanceRepsProcessor.java:238-239; returns the
 * position in cols (-1: none below 1.0), bestD[0] = its distance */
JNIEXPORT jint JNICALL JFN(nArgmin)(JNIEnv* env, jclass c, jlong ctx, jlong sets, jlong q, jlongArray cols,
                                    jdoubleArray bestD) {
    jsize n = 0;
    int64_t* cl = copy_cols(env, cols, &n);
    if (!cl) return -1;
    int64_t idx = -1;
    double d = 1.0;
    int rc = gdist_row_query(CTX(ctx), SETS(sets), q, cl, n, GDIST_QUERY_ARGMIN, 1.0, NULL, NULL, &idx, &d);
    free(cl);
    if (rc) { throw_for(env, rc); return -1; }
    if (bestD && (*env)->GetArrayLength(env, bestD) > 0) (*env)->SetDoubleArrayRegion(env, bestD, 0, 1, &d);
    return (jint)idx;
}

/* distances of query q to cols (a Measurer's row: MethodTableProcessor.java:261-275) */
JNIEXPORT void JNICALL JFN(nRow)(JNIEnv* env, jclass c, jlong ctx, jlong sets, jlong q, jlongArray cols,
                                 jdoubleArray out) {
    jsize n = 0;
    int64_t* cl = copy_cols(env, cols, &n);
    if (!cl) return;
    if (too_short(env, out, n, "out shorter than cols")) { free(cl); return; }
    double* d = malloc(((size_t)n + 1) * sizeof(double));
    if (!d) { free(cl); throw_oom(env); return; }
    int rc = gdist_row_query(CTX(ctx), SETS(sets), q, cl, n, GDIST_QUERY_ALL, 1.0, d, NULL, NULL, NULL);
    if (!rc) (*env)->SetDoubleArrayRegion(env, out, 0, n, d);
    free(cl);
    free(d);
    if (rc) throw_for(env, rc);
}

/* greedy representatives, both passes (DistanceRepsProcessor.java:185-262) */
JNIEXPORT jlong JNICALL JFN(nGreedyReps)(JNIEnv* env, jclass c, jlong ctx, jlong sets, jdouble t,
                                         jlongArray tieRank, jintArray isRep, jlongArray repOf,
                                         jdoubleArray repDist) {
    const int64_t n = nsets_of(env, SETS(sets));
    if (n < 0 || too_short(env, isRep, n, "isRep shorter than the number of sets") ||
        (tieRank && too_short(env, tieRank, n, "tieRank shorter than the number of sets")) ||
        (repOf && too_short(env, repOf, n, "repOf shorter than the number of sets")) ||
        (repDist && too_short(env, repDist, n, "repDist shorter than the number of sets")))
        return 0;
    int64_t* tr = tieRank ? malloc(((size_t)n + 1) * sizeof(int64_t)) : NULL;
    int32_t* ir = malloc(((size_t)n + 1) * sizeof(int32_t));
    int64_t* ro = repOf ? malloc(((size_t)n + 1) * sizeof(int64_t)) : NULL;
    double* rd = repDist ? malloc(((size_t)n + 1) * sizeof(double)) : NULL;
    if (!ir || (tieRank && !tr) || (repOf && !ro) || (repDist && !rd)) {
        free(tr); free(ir); free(ro); free(rd);
        throw_oom(env);
        return 0;
    }
    if (tr) {
        (*env)->GetLongArrayRegion(env, tieRank, 0, (jsize)n, (jlong*)tr);
        if ((*env)->ExceptionCheck(env)) { free(tr); free(ir); free(ro); free(rd); return 0; }
    }
    int64_t nreps = 0;
    int rc = gdist_greedy_reps(CTX(ctx), SETS(sets), GDIST_METHOD_AUTO, t, tr, ir, ro, rd, &nreps);
    if (!rc) {
        (*env)->SetIntArrayRegion(env, isRep, 0, (jsize)n, (const jint*)ir);
        if (ro) (*env)->SetLongArrayRegion(env, repOf, 0, (jsize)n, (const jlong*)ro);
        if (rd) (*env)->SetDoubleArrayRegion(env, repDist, 0, (jsize)n, rd);
    }
    free(tr); free(ir); free(ro); free(rd);
    if (rc) { throw_for(env, rc); return 0; }
    return (jlong)nreps;
}

/* ---- MinHash: hashSet(width) and Sketch.distance (WidthProcessor.java:178-185) */
JNIEXPORT jlong JNICALL JFN(nSketch)(JNIEnv* env, jclass c, jlong ctx, jlong sets, jint width) {
    gdist_sets* sk = NULL;
    int rc = gdist_sketch_build(CTX(ctx), SETS(sets), width, &sk);
    if (rc) { throw_for(env, rc); return 0; }
    return (jlong)(intptr_t)sk;
}

/* a sketch collection from signatures (Sketch.getSignature of each sketch of
 * a Bucket, TuningProcessor.java:114-119): off[nsets + 1], sigs[off[nsets]],
 * each signature ascending */
JNIEXPORT jlong JNICALL JFN(nSketchUpload)(JNIEnv* env, jclass c, jlong ctx, jint width, jlongArray off,
                                           jintArray sigs) {
    const jsize n1 = (*env)->GetArrayLength(env, off);
    if (n1 < 1) {
        jclass e = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
        if (e) (*env)->ThrowNew(env, e, "off needs nsets + 1 entries");
        return 0;
    }
    int64_t* o = malloc((size_t)n1 * sizeof(int64_t));
    if (!o) { throw_oom(env); return 0; }
    (*env)->GetLongArrayRegion(env, off, 0, n1, (jlong*)o);
    if ((*env)->ExceptionCheck(env)) { free(o); return 0; }
    const int64_t total = o[n1 - 1];
    if (total < 0 || (*env)->GetArrayLength(env, sigs) < total) {
        free(o);
        jclass e = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
        if (e) (*env)->ThrowNew(env, e, "sigs shorter than off[nsets]");
        return 0;
    }
    int32_t* v = malloc(((size_t)total + 1) * sizeof(int32_t));
    if (!v) { free(o); throw_oom(env); return 0; }
    (*env)->GetIntArrayRegion(env, sigs, 0, (jsize)total, (jint*)v);
    if ((*env)->ExceptionCheck(env)) { free(o); free(v); return 0; }
    gdist_sets* sk = NULL;
    int rc = gdist_sketch_upload(CTX(ctx), width, (int64_t)n1 - 1, o, v, &sk);
    free(o);
    free(v);
    if (rc) { throw_for(env, rc); return 0; }
    return (jlong)(intptr_t)sk;
}

/* the total number of codes (hashes, for a sketch collection) */
JNIEXPORT jlong JNICALL JFN(nTotal)(JNIEnv* env, jclass c, jlong sets) {
    int kind = 0, k = 0;
    int64_t n = 0, total = 0;
    int rc = gdist_sets_info(SETS(sets), &kind, &k, &n, &total);
    if (rc) { throw_for(env, rc); return 0; }
    return (jlong)total;
}

/* the signatures of a sketch collection (Sketch.getSignature of each set,
 * SketchProcessor.java:88): off[nsets + 1] and sigs[total], ascending ints */
JNIEXPORT void JNICALL JFN(nSketchDownload)(JNIEnv* env, jclass c, jlong sk, jlongArray off, jintArray sigs) {
    int kind = 0, k = 0;
    int64_t n = 0, total = 0;
    int rc = gdist_sets_info(SETS(sk), &kind, &k, &n, &total);
    if (rc) { throw_for(env, rc); return; }
    if (too_short(env, off, n + 1, "off shorter than the number of sets + 1") ||
        too_short(env, sigs, total, "sigs shorter than the collection's hashes"))
        return;
    int64_t* o = malloc(((size_t)n + 1) * sizeof(int64_t));
    int32_t* v = malloc(((size_t)total + 1) * sizeof(int32_t));
    if (!o || !v) { free(o); free(v); throw_oom(env); return; }
    rc = gdist_sketch_download(SETS(sk), o, v);
    if (!rc) {
        (*env)->SetLongArrayRegion(env, off, 0, (jsize)(n + 1), (const jlong*)o);
        if (!(*env)->ExceptionCheck(env)) (*env)->SetIntArrayRegion(env, sigs, 0, (jsize)total, (const jint*)v);
    }
    free(o);
    free(v);
    if (rc) throw_for(env, rc);
}

JNIEXPORT void JNICALL JFN(nSketchMatrix)(JNIEnv* env, jclass c, jlong ctx, jlong sk, jlong r0, jlong r1, jlong c0,
                                          jlong c1, jint flags, jdoubleArray out, jint ld) {
    const int64_t cells = (int64_t)(r1 - r0) * (int64_t)ld;
    if (cells < 0 || (*env)->GetArrayLength(env, out) < cells) {
        jclass e = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
        if (e) (*env)->ThrowNew(env, e, "output array smaller than (r1 - r0) * ld");
        return;
    }
    double* d = malloc((size_t)(cells ? cells : 1) * sizeof(double));
    if (!d) { throw_oom(env); return; }
    (*env)->GetDoubleArrayRegion(env, out, 0, (jsize)cells, d);
    if ((*env)->ExceptionCheck(env)) { free(d); return; }
    int rc = gdist_sketch_matrix(CTX(ctx), SETS(sk), r0, r1, c0, c1, (unsigned)flags, NULL, d, ld);
    if (!rc) (*env)->SetDoubleArrayRegion(env, out, 0, (jsize)cells, d);
    free(d);
    if (rc) throw_for(env, rc);
}
