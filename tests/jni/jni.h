/* jni.h -- TEST INFRASTRUCTURE ONLY: a stand-in for the JDK's jni.h (no JDK in this image) with
 * just the types and JNIEnv functions electionguard-remote_amd/jvm/src/main/c/eg_hip_jni.c uses,
 * so tests/jni/jni_harness.c can compile that file unchanged and execute every JNI function.
 * The function-table layout is this file's own (not the JDK's); the harness supplies the
 * implementations.  Never used to build the shipped JNI library. */
#ifndef EG_TEST_JNI_H
#define EG_TEST_JNI_H
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
#define JNI_FALSE 0
#define JNI_TRUE 1
typedef double jdouble;
typedef jint jsize;

typedef struct eg_test_jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jbyteArray;
typedef jarray jlongArray;
typedef jarray jdoubleArray;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv* env, const char* name);
  jint (*ThrowNew)(JNIEnv* env, jclass cls, const char* msg);
  jsize (*GetArrayLength)(JNIEnv* env, jarray a);
  void (*GetByteArrayRegion)(JNIEnv* env, jbyteArray a, jsize start, jsize len, jbyte* buf);
  void (*SetByteArrayRegion)(JNIEnv* env, jbyteArray a, jsize start, jsize len, const jbyte* buf);
  jbyte* (*GetByteArrayElements)(JNIEnv* env, jbyteArray a, jboolean* is_copy);
  void (*ReleaseByteArrayElements)(JNIEnv* env, jbyteArray a, jbyte* elems, jint mode);
  jlong* (*GetLongArrayElements)(JNIEnv* env, jlongArray a, jboolean* is_copy);
  void (*ReleaseLongArrayElements)(JNIEnv* env, jlongArray a, jlong* elems, jint mode);
  jstring (*NewStringUTF)(JNIEnv* env, const char* utf);
  jdoubleArray (*NewDoubleArray)(JNIEnv* env, jsize len);
  void (*SetDoubleArrayRegion)(JNIEnv* env, jdoubleArray a, jsize start, jsize len, const jdouble* buf);
};
#endif
