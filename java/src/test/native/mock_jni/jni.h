/* Minimal JNI surface for testing the JNI layer (java/src/main/native/cylon_jni.cpp) without a JDK:
 * the types and the JNIEnv members that layer calls, with JNIEnv's members implemented by the test
 * harness (jni_mock_test.cpp) over plain C++ objects.  Not a JVM: only what cylon_jni.cpp uses. */
#ifndef CYLON_MOCK_JNI_H_
#define CYLON_MOCK_JNI_H_
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

typedef int32_t jint;
typedef int64_t jlong;
typedef uint8_t jboolean;
typedef double jdouble;
typedef jint jsize;

struct _jobject {
  virtual ~_jobject() {}
};
typedef _jobject *jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jobjectArray;
typedef jobject jintArray;
typedef jobject jlongArray;
struct _jmethodID;
typedef _jmethodID *jmethodID;

struct JNIEnv {
  const char *GetStringUTFChars(jstring s, jboolean *is_copy);
  void ReleaseStringUTFChars(jstring s, const char *c);
  jstring NewStringUTF(const char *c);
  jclass FindClass(const char *name);
  jclass GetObjectClass(jobject o);
  jmethodID GetMethodID(jclass cls, const char *name, const char *sig);
  jobject NewObject(jclass cls, jmethodID ctor, ...);
  jboolean CallBooleanMethod(jobject o, jmethodID m, ...);
  void DeleteLocalRef(jobject o);
  jsize GetArrayLength(jobject a);
  void GetIntArrayRegion(jintArray a, jsize start, jsize len, jint *buf);
  void GetLongArrayRegion(jlongArray a, jsize start, jsize len, jlong *buf);
  jobject GetObjectArrayElement(jobjectArray a, jsize i);
};
#endif
