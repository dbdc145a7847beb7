/* TEST STUB, not a JDK header: the declarations of <jni.h> that
 * jni/src/main/native/l5dh_jni.c uses, with the JDK's C calling shape
 * ((*env)->Fn(env, ...)), so tests/test_jni_shim.py can syntax-check the shim
 * against include/l5dhist.h in an image without a JDK.  Real builds use the
 * JDK's jni.h (jni/Makefile). */
#ifndef L5DH_TEST_JNI_STUB_H
#define L5DH_TEST_JNI_STUB_H
#include <stdint.h>
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef jint jsize;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jintArray;
typedef jarray jbyteArray;
typedef jarray jlongArray;
struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;
struct JNINativeInterface_ {
  void* (*GetDirectBufferAddress)(JNIEnv*, jobject);
  jobject (*NewDirectByteBuffer)(JNIEnv*, void*, jlong);
  jintArray (*NewIntArray)(JNIEnv*, jsize);
  void (*SetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, const jint*);
  jbyteArray (*NewByteArray)(JNIEnv*, jsize);
  void (*SetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, const jbyte*);
  void (*GetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, jbyte*);
  void (*GetLongArrayRegion)(JNIEnv*, jlongArray, jsize, jsize, jlong*);
  jsize (*GetArrayLength)(JNIEnv*, jarray);
  jstring (*NewStringUTF)(JNIEnv*, const char*);
};
#endif
