/*
 * skml_jni.c -- JNI shim binding the reference's Java surface to libskml.so (include/skml.h).
 *
 * Built only where a JDK exists (jni/Makefile; this repo's image has none, so CI here only
 * syntax-checks it, tests/test_jni_shim.py).  Every native below is one call (or two) into the C
 * ABI; the Java side is the classes under jni/java/org/dma/sketchml/hip/.
 *
 * Memory: Java arrays are pinned with Get<Type>ArrayCritical for the duration of one C call and
 * handed to the host entry points (skml_dense_encode_host_f32 / _f64, ...), which stage them
 * through library-owned pinned buffers.  Dense payloads live in Java byte[]s
 * (header, splits, packed codes); sparse payloads are library-owned device objects behind a
 * long handle, freed by freeSparse (HipSparseVectorCompressor.close / a Cleaner).
 * A critical region holds off the JVM's garbage collector for the length of the call (the
 * host-path encode of 2^26 floats: 6-9 ms); the alternative, Get<Type>ArrayRegion
 * into the library's pinned staging, adds a second full host copy of the array, so the shim keeps
 * the critical regions and states the cost here.
 *
 * Errors: a non-zero status becomes the reference's unchecked exception:
 * SKML_E_NAN -> QuantileSketchException("Encounter NaN value") (HeapQuantileSketch.java:75-76);
 * a partition-number error -> QuantileSketchException; everything else -> SketchMLException with
 * skml_last_error().
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "skml.h"

#define CLS_SKETCHML "org/dma/sketchml/sketch/base/SketchMLException"
#define CLS_QSKETCH "org/dma/sketchml/sketch/sketch/quantile/QuantileSketchException"

static int throw_status(JNIEnv* env, int st) {
    if (st == SKML_OK) return 0;
    const char* msg = st == SKML_E_NAN ? "Encounter NaN value" : skml_last_error();
    const char* cls = (st == SKML_E_NAN || (msg && strstr(msg, "partition number"))) ? CLS_QSKETCH : CLS_SKETCHML;
    jclass k = (*env)->FindClass(env, cls);
    if (k) (*env)->ThrowNew(env, k, msg ? msg : "libskml error");
    return 1;
}

static skml_ctx* CTX(jlong h) { return (skml_ctx*)(uintptr_t)h; }

static void fill_params(skml_params* p, jint bins, jboolean dedup, jlong seed, jint parallelism) {
    skml_params_default(p);
    p->bin_num = bins;
    p->dedup = dedup ? 1 : 0;
    p->seed = seed;
    p->parallelism = parallelism > 1 ? parallelism : 1;
}

/* A Java byte[] holding exactly the `written` payload bytes of a host encode. */
static jbyteArray to_byte_array(JNIEnv* env, const uint8_t* buf, size_t len) {
    jbyteArray out = (*env)->NewByteArray(env, (jsize)len);
    if (out) (*env)->SetByteArrayRegion(env, out, 0, (jsize)len, (const jbyte*)buf);
    return out;
}

/* GetPrimitiveArrayCritical may return NULL (out of memory): throw OutOfMemoryError unless the JVM
 * already has an exception pending.  Returns 1 when the caller must bail out. */
static int pin_failed(JNIEnv* env, const void* a, const void* b) {
    if (a && b) return 0;
    if (!(*env)->ExceptionCheck(env)) {
        jclass k = (*env)->FindClass(env, "java/lang/OutOfMemoryError");
        if (k) (*env)->ThrowNew(env, k, "cannot pin a Java array for the GPU codec");
    }
    return 1;
}

/* ---------------------------------------------------------------- context */
JNIEXPORT jlong JNICALL Java_org_dma_sketchml_hip_HipCodec_ctxCreate(JNIEnv* env, jclass cls, jint device) {
    (void)cls;
    skml_ctx* ctx = NULL;
    if (throw_status(env, skml_ctx_create(device, SKML_STREAM_OWN, &ctx))) return 0;
    return (jlong)(uintptr_t)ctx;
}

JNIEXPORT void JNICALL Java_org_dma_sketchml_hip_HipCodec_ctxDestroy(JNIEnv* env, jclass cls, jlong ctx) {
    (void)env;
    (void)cls;
    skml_ctx_destroy(CTX(ctx));
}

/* ---------------------------------------------------------------- dense: QuantileQuantizer */
/* byte[] encodeDense(long ctx, float[] x, int binNum, boolean dedup, long seed, int parallelism) */
JNIEXPORT jbyteArray JNICALL Java_org_dma_sketchml_hip_HipCodec_encodeDense(JNIEnv* env, jclass cls, jlong ctx,
                                                                          jfloatArray xs, jint bins,
                                                                          jboolean dedup, jlong seed,
                                                                          jint parallelism) {
    (void)cls;
    skml_params p;
    fill_params(&p, bins, dedup, seed, parallelism);
    const jsize n = (*env)->GetArrayLength(env, xs);
    size_t cap = 0, wrote = 0;
    if (throw_status(env, skml_dense_encode_host_f32(CTX(ctx), NULL, n, &p, NULL, 0, &cap))) return NULL;
    uint8_t* buf = (uint8_t*)malloc(cap ? cap : 1);
    if (!buf) return NULL;
    float* x = (float*)(*env)->GetPrimitiveArrayCritical(env, xs, NULL);
    if (pin_failed(env, x, buf)) {
        free(buf);
        return NULL;
    }
    int st = skml_dense_encode_host_f32(CTX(ctx), x, n, &p, buf, cap, &wrote);
    (*env)->ReleasePrimitiveArrayCritical(env, xs, x, JNI_ABORT);
    jbyteArray out = st ? NULL : to_byte_array(env, buf, wrote);
    free(buf);
    throw_status(env, st);
    return out;
}

/* byte[] encodeDenseF64(long ctx, double[] x, int binNum, boolean dedup, long seed, int parallelism):
 * the reference's double[] itself (QuantileQuantizer.quantize(double[]), no rounding). */
JNIEXPORT jbyteArray JNICALL Java_org_dma_sketchml_hip_HipCodec_encodeDenseF64(JNIEnv* env, jclass cls, jlong ctx,
                                                                             jdoubleArray xs, jint bins,
                                                                             jboolean dedup, jlong seed,
                                                                             jint parallelism) {
    (void)cls;
    skml_params p;
    fill_params(&p, bins, dedup, seed, parallelism);
    const jsize n = (*env)->GetArrayLength(env, xs);
    size_t cap = 0, wrote = 0;
    if (throw_status(env, skml_dense_encode_host_f64(CTX(ctx), NULL, n, &p, NULL, 0, &cap))) return NULL;
    uint8_t* buf = (uint8_t*)malloc(cap ? cap : 1);
    if (!buf) return NULL;
    double* x = (double*)(*env)->GetPrimitiveArrayCritical(env, xs, NULL);
    if (pin_failed(env, x, buf)) {
        free(buf);
        return NULL;
    }
    int st = skml_dense_encode_host_f64(CTX(ctx), x, n, &p, buf, cap, &wrote);
    (*env)->ReleasePrimitiveArrayCritical(env, xs, x, JNI_ABORT);
    jbyteArray out = st ? NULL : to_byte_array(env, buf, wrote);
    free(buf);
    throw_status(env, st);
    return out;
}

/* byte[] encodeDenseUniformF64(long ctx, double[] x, int binNum): UniformQuantizer.quantize(double[])
 * (quantization/UniformQuantizer.java:21-45) through the host entry point with
 * params.quant_type = SKML_UNIFORM, i.e. skml_dense_encode_uniform_f64 on the device copy. */
JNIEXPORT jbyteArray JNICALL Java_org_dma_sketchml_hip_HipCodec_encodeDenseUniformF64(JNIEnv* env, jclass cls,
                                                                                    jlong ctx, jdoubleArray xs,
                                                                                    jint bins) {
    (void)cls;
    skml_params p;
    fill_params(&p, bins, JNI_FALSE, 0, 1);
    p.quant_type = SKML_UNIFORM;
    const jsize n = (*env)->GetArrayLength(env, xs);
    size_t cap = 0, wrote = 0;
    if (throw_status(env, skml_dense_encode_host_f64(CTX(ctx), NULL, n, &p, NULL, 0, &cap))) return NULL;
    uint8_t* buf = (uint8_t*)malloc(cap ? cap : 1);
    if (!buf) return NULL;
    double* x = (double*)(*env)->GetPrimitiveArrayCritical(env, xs, NULL);
    if (pin_failed(env, x, buf)) {
        free(buf);
        return NULL;
    }
    int st = skml_dense_encode_host_f64(CTX(ctx), x, n, &p, buf, cap, &wrote);
    (*env)->ReleasePrimitiveArrayCritical(env, xs, x, JNI_ABORT);
    jbyteArray out = st ? NULL : to_byte_array(env, buf, wrote);
    free(buf);
    throw_status(env, st);
    return out;
}

/* void decodeDense(long ctx, byte[] payload, float[] out)  (DenseVectorCompressor.java:84-91) */
JNIEXPORT void JNICALL Java_org_dma_sketchml_hip_HipCodec_decodeDense(JNIEnv* env, jclass cls, jlong ctx,
                                                                    jbyteArray payload, jfloatArray out) {
    (void)cls;
    const jsize len = (*env)->GetArrayLength(env, payload), n = (*env)->GetArrayLength(env, out);
    void* pl = (*env)->GetPrimitiveArrayCritical(env, payload, NULL);
    float* o = pl ? (float*)(*env)->GetPrimitiveArrayCritical(env, out, NULL) : NULL;
    if (pin_failed(env, pl, o)) {
        if (pl) (*env)->ReleasePrimitiveArrayCritical(env, payload, pl, JNI_ABORT);
        return;
    }
    int st = skml_dense_decode_host_f32(CTX(ctx), pl, (size_t)len, o, n);
    (*env)->ReleasePrimitiveArrayCritical(env, out, o, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, payload, pl, JNI_ABORT);
    throw_status(env, st);
}

/* void decodeDenseF64(long ctx, byte[] payload, double[] out) */
JNIEXPORT void JNICALL Java_org_dma_sketchml_hip_HipCodec_decodeDenseF64(JNIEnv* env, jclass cls, jlong ctx,
                                                                       jbyteArray payload, jdoubleArray out) {
    (void)cls;
    const jsize len = (*env)->GetArrayLength(env, payload), n = (*env)->GetArrayLength(env, out);
    void* pl = (*env)->GetPrimitiveArrayCritical(env, payload, NULL);
    double* o = pl ? (double*)(*env)->GetPrimitiveArrayCritical(env, out, NULL) : NULL;
    if (pin_failed(env, pl, o)) {
        if (pl) (*env)->ReleasePrimitiveArrayCritical(env, payload, pl, JNI_ABORT);
        return;
    }
    int st = skml_dense_decode_host_f64(CTX(ctx), pl, (size_t)len, o, n);
    (*env)->ReleasePrimitiveArrayCritical(env, out, o, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, payload, pl, JNI_ABORT);
    throw_status(env, st);
}

/* void getBins(byte[] payload, int[] out): Quantizer.getBins() (Quantizer.java:163-165) */
JNIEXPORT void JNICALL Java_org_dma_sketchml_hip_HipCodec_getBins(JNIEnv* env, jclass cls, jbyteArray payload,
                                                                jintArray out) {
    (void)cls;
    const jsize len = (*env)->GetArrayLength(env, payload), n = (*env)->GetArrayLength(env, out);
    void* pl = (*env)->GetPrimitiveArrayCritical(env, payload, NULL);
    jint* o = pl ? (jint*)(*env)->GetPrimitiveArrayCritical(env, out, NULL) : NULL;
    if (pin_failed(env, pl, o)) {
        if (pl) (*env)->ReleasePrimitiveArrayCritical(env, payload, pl, JNI_ABORT);
        return;
    }
    int st = skml_dense_bins_host(pl, (size_t)len, (int32_t*)o, n);
    (*env)->ReleasePrimitiveArrayCritical(env, out, o, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, payload, pl, JNI_ABORT);
    throw_status(env, st);
}

/* double[] info(byte[] payload): {binNum, n, zeroIdx, min, max, splits[0..binNum-2]} */
JNIEXPORT jdoubleArray JNICALL Java_org_dma_sketchml_hip_HipCodec_info(JNIEnv* env, jclass cls, jbyteArray payload) {
    (void)cls;
    const jsize len = (*env)->GetArrayLength(env, payload);
    skml_dense_header h;
    double* sp = (double*)malloc(sizeof(double) * SKML_MAX_BINS);
    if (!sp) return NULL;
    void* pl = (*env)->GetPrimitiveArrayCritical(env, payload, NULL);
    if (pin_failed(env, pl, pl)) {
        free(sp);
        return NULL;
    }
    int st = skml_dense_info_host(pl, (size_t)len, &h, sp, SKML_MAX_BINS);
    (*env)->ReleasePrimitiveArrayCritical(env, payload, pl, JNI_ABORT);
    jdoubleArray out = NULL;
    if (!st) {
        const jsize ns = h.bin_num - 1;
        out = (*env)->NewDoubleArray(env, 5 + ns);
        if (out) {
            const jdouble head[5] = {(double)h.bin_num, (double)h.n, (double)h.zero_idx, h.min, h.max};
            (*env)->SetDoubleArrayRegion(env, out, 0, 5, head);
            (*env)->SetDoubleArrayRegion(env, out, 5, ns, sp);
        }
    }
    free(sp);
    throw_status(env, st);
    return out;
}

/* void timesBy(byte[] payload, double x): Quantizer.timesBy (Quantizer.java:119-124), in place */
JNIEXPORT void JNICALL Java_org_dma_sketchml_hip_HipCodec_timesBy(JNIEnv* env, jclass cls, jbyteArray payload,
                                                                jdouble x) {
    (void)cls;
    const jsize len = (*env)->GetArrayLength(env, payload);
    void* pl = (*env)->GetPrimitiveArrayCritical(env, payload, NULL);
    if (pin_failed(env, pl, pl)) return;
    int st = skml_dense_times_by_host(pl, (size_t)len, x);
    (*env)->ReleasePrimitiveArrayCritical(env, payload, pl, 0);
    throw_status(env, st);
}

/* ---------------------------------------------------------------- sparse: GroupedMinMaxSketch */
static void throw_class(JNIEnv* env, const char* cls, const char* msg) {
    jclass k = (*env)->FindClass(env, cls);
    if (k) (*env)->ThrowNew(env, k, msg);
}

/* long encodeSparse(long ctx, int[] keys, double[] vals, int binNum, int groupNum, int rowNum,
 *                   double colRatio, long seed, long hashSeed, boolean uniform, int parallelism):
 * the reference's double values themselves (skml_sparse_encode_kv_host_f64: the quantizer sketches
 * and bins the doubles, SparseVectorCompressor.java:52-67, SketchGradient.scala:35-48). */
JNIEXPORT jlong JNICALL Java_org_dma_sketchml_hip_HipCodec_encodeSparse(JNIEnv* env, jclass cls, jlong ctx,
                                                                      jintArray keys, jdoubleArray vals, jint bins,
                                                                      jint groups, jint rows, jdouble ratio,
                                                                      jlong seed, jlong hash_seed,
                                                                      jboolean uniform, jint parallelism) {
    (void)cls;
    const jsize n = (*env)->GetArrayLength(env, keys);
    if ((*env)->GetArrayLength(env, vals) != n) {
        throw_class(env, CLS_SKETCHML, "Lengths of key array and value array do not match");
        return 0;
    }
    skml_params p;
    fill_params(&p, bins, JNI_TRUE, seed, parallelism);
    p.group_num = groups;
    p.row_num = rows;
    p.col_ratio = ratio;
    p.hash_seed = hash_seed;
    p.quant_type = uniform ? SKML_UNIFORM : SKML_QUANTILE;
    skml_sparse* s = NULL;
    jint* k = (jint*)(*env)->GetPrimitiveArrayCritical(env, keys, NULL);
    double* v = k ? (double*)(*env)->GetPrimitiveArrayCritical(env, vals, NULL) : NULL;
    if (pin_failed(env, k, v)) {
        if (k) (*env)->ReleasePrimitiveArrayCritical(env, keys, k, JNI_ABORT);
        return 0;
    }
    int st = skml_sparse_encode_kv_host_f64(CTX(ctx), (const int32_t*)k, v, n, &p, &s);
    (*env)->ReleasePrimitiveArrayCritical(env, vals, v, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, keys, k, JNI_ABORT);
    if (throw_status(env, st)) return 0;
    return (jlong)(uintptr_t)s;
}

/* void decodeSparse(long ctx, long sparse, int[] keys, double[] vals): restore + Sort.merge +
 * quantValues[bin] in double (SparseVectorCompressor.decompressSparse, :118-126).  Both arrays must
 * hold the payload's nnz entries (skml_sparse_nnz): checked before anything is written. */
JNIEXPORT void JNICALL Java_org_dma_sketchml_hip_HipCodec_decodeSparse(JNIEnv* env, jclass cls, jlong ctx,
                                                                     jlong sp, jintArray keys, jdoubleArray vals) {
    (void)cls;
    int64_t nnz = 0;
    if (throw_status(env, skml_sparse_nnz((const skml_sparse*)(uintptr_t)sp, &nnz))) return;
    if ((int64_t)(*env)->GetArrayLength(env, keys) < nnz || (int64_t)(*env)->GetArrayLength(env, vals) < nnz) {
        throw_class(env, CLS_SKETCHML, "decodeSparse: key / value arrays shorter than the payload's nnz");
        return;
    }
    jint* k = (jint*)(*env)->GetPrimitiveArrayCritical(env, keys, NULL);
    double* v = k ? (double*)(*env)->GetPrimitiveArrayCritical(env, vals, NULL) : NULL;
    if (pin_failed(env, k, v)) {
        if (k) (*env)->ReleasePrimitiveArrayCritical(env, keys, k, JNI_ABORT);
        return;
    }
    int st = skml_sparse_decode_host_f64(CTX(ctx), (const skml_sparse*)(uintptr_t)sp, (int32_t*)k, v);
    (*env)->ReleasePrimitiveArrayCritical(env, vals, v, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, keys, k, 0);
    throw_status(env, st);
}

JNIEXPORT jint JNICALL Java_org_dma_sketchml_hip_HipCodec_sparseNnz(JNIEnv* env, jclass cls, jlong sp) {
    (void)cls;
    int64_t n = 0;
    if (throw_status(env, skml_sparse_nnz((const skml_sparse*)(uintptr_t)sp, &n))) return 0;
    return (jint)n;
}

/* double[] sparseValues(long sparse, int binNum): SparseVectorCompressor.quantValues */
JNIEXPORT jdoubleArray JNICALL Java_org_dma_sketchml_hip_HipCodec_sparseValues(JNIEnv* env, jclass cls, jlong sp,
                                                                             jint bins) {
    (void)cls;
    skml_dense_header h;
    if (throw_status(env, skml_sparse_quant_info((const skml_sparse*)(uintptr_t)sp, &h, NULL, 0))) return NULL;
    const jint nb = h.bin_num < bins ? h.bin_num : bins;
    double* v = (double*)malloc(sizeof(double) * (nb > 0 ? nb : 1));
    if (!v) return NULL;
    jdoubleArray out = NULL;
    if (!throw_status(env, skml_sparse_values((const skml_sparse*)(uintptr_t)sp, v, nb))) {
        out = (*env)->NewDoubleArray(env, nb);
        if (out) (*env)->SetDoubleArrayRegion(env, out, 0, nb, v);
    }
    free(v);
    return out;
}

/* void sparseTimesBy(long sparse, double x): SparseVectorCompressor.timesBy (:128-134) */
JNIEXPORT void JNICALL Java_org_dma_sketchml_hip_HipCodec_sparseTimesBy(JNIEnv* env, jclass cls, jlong sp, jdouble x) {
    (void)cls;
    throw_status(env, skml_sparse_times_by((skml_sparse*)(uintptr_t)sp, x));
}

/* byte[] writeSparse(long ctx, long sparse): GroupedMinMaxSketch.writeObject field stream */
JNIEXPORT jbyteArray JNICALL Java_org_dma_sketchml_hip_HipCodec_writeSparse(JNIEnv* env, jclass cls, jlong ctx,
                                                                          jlong sp) {
    (void)cls;
    size_t need = 0;
    if (throw_status(env, skml_sparse_serialize(CTX(ctx), (const skml_sparse*)(uintptr_t)sp, NULL, 0, &need)))
        return NULL;
    uint8_t* buf = (uint8_t*)malloc(need ? need : 1);
    if (!buf) return NULL;
    int st = skml_sparse_serialize(CTX(ctx), (const skml_sparse*)(uintptr_t)sp, buf, need, &need);
    jbyteArray out = st ? NULL : to_byte_array(env, buf, need);
    free(buf);
    throw_status(env, st);
    return out;
}

/* long readSparse(long ctx, byte[] stream, double[] quantValues): GroupedMinMaxSketch.readObject */
JNIEXPORT jlong JNICALL Java_org_dma_sketchml_hip_HipCodec_readSparse(JNIEnv* env, jclass cls, jlong ctx,
                                                                    jbyteArray data, jdoubleArray qv) {
    (void)cls;
    const jsize len = (*env)->GetArrayLength(env, data);
    const jsize nq = qv ? (*env)->GetArrayLength(env, qv) : 0;
    skml_sparse* s = NULL;
    void* d = (*env)->GetPrimitiveArrayCritical(env, data, NULL);
    double* q = (d && qv) ? (double*)(*env)->GetPrimitiveArrayCritical(env, qv, NULL) : NULL;
    if (pin_failed(env, d, qv ? (const void*)q : d)) {
        if (d) (*env)->ReleasePrimitiveArrayCritical(env, data, d, JNI_ABORT);
        return 0;
    }
    int st = skml_sparse_deserialize(CTX(ctx), (const uint8_t*)d, (size_t)len, q, nq, &s);
    if (q) (*env)->ReleasePrimitiveArrayCritical(env, qv, q, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, data, d, JNI_ABORT);
    if (throw_status(env, st)) return 0;
    return (jlong)(uintptr_t)s;
}

JNIEXPORT void JNICALL Java_org_dma_sketchml_hip_HipCodec_freeSparse(JNIEnv* env, jclass cls, jlong sp) {
    (void)env;
    (void)cls;
    skml_sparse_free((skml_sparse*)(uintptr_t)sp);
}

/* ---------------------------------------------------------------- DeltaAdaptiveEncoder */
/* long[] deltaEncode(long ctx, int[] keys):
 *   {numIntervals, flagKind, nFlagBits, nDeltaBits, nFlagWords, nDeltaWords, flagWords..., deltaWords...}
 * (BitSet.toLongArray layout of the two streams, DeltaAdaptiveEncoder.java:148-170) */
JNIEXPORT jlongArray JNICALL Java_org_dma_sketchml_hip_HipCodec_deltaEncode(JNIEnv* env, jclass cls, jlong ctx,
                                                                          jintArray keys) {
    (void)cls;
    const jsize n = (*env)->GetArrayLength(env, keys);
    const int64_t cap = ((int64_t)n * 33 + 63) / 64 + 1;
    uint64_t* fw = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)cap);
    uint64_t* dw = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)cap);
    if (!fw || !dw) {
        free(fw);
        free(dw);
        return NULL;
    }
    int32_t m = 0, kind = 0;
    int64_t nfb = 0, ndb = 0;
    jint* k = (jint*)(*env)->GetPrimitiveArrayCritical(env, keys, NULL);
    if (pin_failed(env, k, k)) {
        free(fw);
        free(dw);
        return NULL;
    }
    int st = skml_delta_encode_host(CTX(ctx), (const int32_t*)k, n, &m, &kind, &nfb, &ndb, fw, dw, cap);
    (*env)->ReleasePrimitiveArrayCritical(env, keys, k, JNI_ABORT);
    jlongArray out = NULL;
    if (!st) {
        /* toLongArray trims trailing zero words */
        int64_t nf = (nfb + 63) / 64, nd = (ndb + 63) / 64;
        while (nf > 0 && fw[nf - 1] == 0) nf--;
        while (nd > 0 && dw[nd - 1] == 0) nd--;
        out = (*env)->NewLongArray(env, (jsize)(6 + nf + nd));
        if (out) {
            const jlong head[6] = {m, kind, nfb, ndb, nf, nd};
            (*env)->SetLongArrayRegion(env, out, 0, 6, head);
            (*env)->SetLongArrayRegion(env, out, 6, (jsize)nf, (const jlong*)fw);
            (*env)->SetLongArrayRegion(env, out, (jsize)(6 + nf), (jsize)nd, (const jlong*)dw);
        }
    }
    free(fw);
    free(dw);
    throw_status(env, st);
    return out;
}

/* int[] deltaDecode(long ctx, int size, int numIntervals, boolean flagKind, long[] flagWords, long[] deltaWords) */
JNIEXPORT jintArray JNICALL Java_org_dma_sketchml_hip_HipCodec_deltaDecode(JNIEnv* env, jclass cls, jlong ctx,
                                                                         jint size, jint m, jboolean kind,
                                                                         jlongArray flags, jlongArray deltas) {
    (void)cls;
    const jsize nf = (*env)->GetArrayLength(env, flags), nd = (*env)->GetArrayLength(env, deltas);
    jintArray out = (*env)->NewIntArray(env, size);
    if (!out || size <= 0) return out;
    jlong* f = (jlong*)(*env)->GetPrimitiveArrayCritical(env, flags, NULL);
    jlong* d = f ? (jlong*)(*env)->GetPrimitiveArrayCritical(env, deltas, NULL) : NULL;
    jint* o = d ? (jint*)(*env)->GetPrimitiveArrayCritical(env, out, NULL) : NULL;
    if (pin_failed(env, f, d) || pin_failed(env, o, o)) {
        if (d) (*env)->ReleasePrimitiveArrayCritical(env, deltas, d, JNI_ABORT);
        if (f) (*env)->ReleasePrimitiveArrayCritical(env, flags, f, JNI_ABORT);
        return NULL;
    }
    int st = skml_delta_decode_host(CTX(ctx), size, m, kind ? 1 : 0, (const uint64_t*)f, nf, (const uint64_t*)d, nd,
                                    (int32_t*)o);
    (*env)->ReleasePrimitiveArrayCritical(env, out, o, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, deltas, d, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, flags, f, JNI_ABORT);
    if (throw_status(env, st)) return NULL;
    return out;
}
