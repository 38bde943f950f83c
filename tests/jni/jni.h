/*
 * SUBSET of the JNI interface, for the tests only: it declares the types and the JNIEnv functions that
 * integration/jni/mpi_HipIntracomm.c calls, with their JNI 1.8 signatures, so the shim is compiled with
 * -Wall -Werror in this JDK-less image (tests/test_integration.py) and executed against the functional
 * stand-in tests/jni/fakejvm.c, which fills this table (tests/test_gpu_jni.py). The table's layout is
 * NOT the JDK's: a maintainer builds the shim against $JAVA_HOME/include.
 */
#ifndef MPJX_TEST_JNI_H
#define MPJX_TEST_JNI_H
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef jint jsize;
typedef struct _jobject *jobject;
typedef jobject jclass;
typedef jobject jarray;
typedef jarray jbyteArray;
typedef jarray jintArray;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;

struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv *env, const char *name);
  jint (*ThrowNew)(JNIEnv *env, jclass clazz, const char *msg);
  jboolean (*ExceptionCheck)(JNIEnv *env);
  jsize (*GetArrayLength)(JNIEnv *env, jarray array);
  void (*GetByteArrayRegion)(JNIEnv *env, jbyteArray array, jsize start, jsize len, jbyte *buf);
  void (*SetByteArrayRegion)(JNIEnv *env, jbyteArray array, jsize start, jsize len, const jbyte *buf);
  void (*GetIntArrayRegion)(JNIEnv *env, jintArray array, jsize start, jsize len, jint *buf);
  jint *(*GetIntArrayElements)(JNIEnv *env, jintArray array, jboolean *isCopy);
  void (*ReleaseIntArrayElements)(JNIEnv *env, jintArray array, jint *elems, jint mode);
  void *(*GetPrimitiveArrayCritical)(JNIEnv *env, jarray array, jboolean *isCopy);
  void (*ReleasePrimitiveArrayCritical)(JNIEnv *env, jarray array, void *carray, jint mode);
  void *(*GetDirectBufferAddress)(JNIEnv *env, jobject buf);
  jlong (*GetDirectBufferCapacity)(JNIEnv *env, jobject buf);
};
#endif
