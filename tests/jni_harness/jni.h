/*
 * jni.h -- TEST INFRASTRUCTURE: the subset of the JNI C interface (Java Native Interface Specification, "JNI Types and
 * Data Structures" / "JNI Functions") that jni/ngsep_gpu_jni.c uses, so the shim compiles and runs in this image, which
 * has no JDK.  The function-table layout is this harness's own (a JVM's jni.h orders ~230 slots); calls go through
 * (*env)->Name(env, ...) exactly as against the real header.  tests/jni_harness/harness.c implements the functions.
 */
#ifndef NGSEP_TEST_JNI_H
#define NGSEP_TEST_JNI_H
#include <stdarg.h>
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef double jdouble;
typedef jint jsize;
typedef struct _jobject* jobject;
typedef jobject jclass, jstring, jarray, jthrowable;
typedef jarray jintArray, jlongArray, jbyteArray, jdoubleArray, jobjectArray;
typedef struct _jmethodID* jmethodID;
typedef struct _jfieldID* jfieldID;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;
struct JNINativeInterface_ {
    jclass (*FindClass)(JNIEnv*, const char*);
    jint (*ThrowNew)(JNIEnv*, jclass, const char*);
    jstring (*NewStringUTF)(JNIEnv*, const char*);
    const char* (*GetStringUTFChars)(JNIEnv*, jstring, jboolean*);
    void (*ReleaseStringUTFChars)(JNIEnv*, jstring, const char*);
    jsize (*GetArrayLength)(JNIEnv*, jarray);
    jobjectArray (*NewObjectArray)(JNIEnv*, jsize, jclass, jobject);
    jobject (*GetObjectArrayElement)(JNIEnv*, jobjectArray, jsize);
    void (*SetObjectArrayElement)(JNIEnv*, jobjectArray, jsize, jobject);
    jbyteArray (*NewByteArray)(JNIEnv*, jsize);
    jlongArray (*NewLongArray)(JNIEnv*, jsize);
    jint* (*GetIntArrayElements)(JNIEnv*, jintArray, jboolean*);
    void (*ReleaseIntArrayElements)(JNIEnv*, jintArray, jint*, jint);
    jlong* (*GetLongArrayElements)(JNIEnv*, jlongArray, jboolean*);
    void (*ReleaseLongArrayElements)(JNIEnv*, jlongArray, jlong*, jint);
    void (*SetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, const jbyte*);
    void (*SetLongArrayRegion)(JNIEnv*, jlongArray, jsize, jsize, const jlong*);
    void* (*GetPrimitiveArrayCritical)(JNIEnv*, jarray, jboolean*);
    void (*ReleasePrimitiveArrayCritical)(JNIEnv*, jarray, void*, jint);
    jmethodID (*GetStaticMethodID)(JNIEnv*, jclass, const char*, const char*);
    jobject (*CallStaticObjectMethod)(JNIEnv*, jclass, jmethodID, ...);
    jbyte* (*GetByteArrayElements)(JNIEnv*, jbyteArray, jboolean*);
    void (*ReleaseByteArrayElements)(JNIEnv*, jbyteArray, jbyte*, jint);
    jfieldID (*GetStaticFieldID)(JNIEnv*, jclass, const char*, const char*);
    jobject (*GetStaticObjectField)(JNIEnv*, jclass, jfieldID);
    jmethodID (*GetMethodID)(JNIEnv*, jclass, const char*, const char*);
    jobject (*CallObjectMethod)(JNIEnv*, jobject, jmethodID, ...);
};
#endif
