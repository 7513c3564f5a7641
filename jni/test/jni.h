/*
 * jni.h -- SYNTAX-CHECK STAND-IN, test infrastructure only (tests/test_jni_shim.py).
 *
 * This image has no JDK.  To still type-check jni/skml_jni.c against include/skml.h here, this
 * header declares the subset of the JNI 1.8 C interface the shim uses, with the JDK's names,
 * types and call shapes ((*env)->Fn(env, ...)).  It is never used to build a library; the real
 * build (jni/Makefile) takes $(JAVA_HOME)/include/jni.h.
 */
#ifndef SKML_TEST_JNI_H
#define SKML_TEST_JNI_H
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_ABORT 2

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef uint16_t jchar;
typedef int16_t jshort;
typedef float jfloat;
typedef double jdouble;
typedef jint jsize;

struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jthrowable;
typedef jobject jarray;
typedef jarray jbyteArray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jarray jfloatArray;
typedef jarray jdoubleArray;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
    jclass (*FindClass)(JNIEnv* env, const char* name);
    jint (*ThrowNew)(JNIEnv* env, jclass clazz, const char* msg);
    jsize (*GetArrayLength)(JNIEnv* env, jarray array);
    jbyteArray (*NewByteArray)(JNIEnv* env, jsize len);
    jintArray (*NewIntArray)(JNIEnv* env, jsize len);
    jlongArray (*NewLongArray)(JNIEnv* env, jsize len);
    jdoubleArray (*NewDoubleArray)(JNIEnv* env, jsize len);
    void (*SetByteArrayRegion)(JNIEnv* env, jbyteArray array, jsize start, jsize len, const jbyte* buf);
    void (*SetLongArrayRegion)(JNIEnv* env, jlongArray array, jsize start, jsize len, const jlong* buf);
    void (*SetDoubleArrayRegion)(JNIEnv* env, jdoubleArray array, jsize start, jsize len, const jdouble* buf);
    void* (*GetPrimitiveArrayCritical)(JNIEnv* env, jarray array, jboolean* isCopy);
    void (*ReleasePrimitiveArrayCritical)(JNIEnv* env, jarray array, void* carray, jint mode);
    jboolean (*ExceptionCheck)(JNIEnv* env);
};
#endif
