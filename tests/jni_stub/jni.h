/* Test-only stand-in for <jni.h> (no JDK in this image): the subset of the JNI C++ interface that
 * opencv-msegment_amd/jni/msegment_jni.cpp uses, with the JDK's type hierarchy and the same
 * member-function signatures as the JDK header's inline wrappers, so a name, type or argument
 * mistake in the shim fails to compile here as it would against a real JDK.  The member functions
 * are defined by the mock environment in mock_env.cpp (tests/test_jni_shim.py). */
#ifndef MSEG_TEST_JNI_STUB_H
#define MSEG_TEST_JNI_STUB_H
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef jint jsize;

class _jobject {};
class _jclass : public _jobject {};
class _jstring : public _jobject {};
class _jarray : public _jobject {};
class _jbyteArray : public _jarray {};
class _jintArray : public _jarray {};
class _jobjectArray : public _jarray {};
typedef _jobject* jobject;
typedef _jclass* jclass;
typedef _jstring* jstring;
typedef _jarray* jarray;
typedef _jbyteArray* jbyteArray;
typedef _jintArray* jintArray;
typedef _jobjectArray* jobjectArray;

struct JNIEnv_ {
  jsize GetArrayLength(jarray array);
  void GetByteArrayRegion(jbyteArray array, jsize start, jsize len, jbyte* buf);
  void SetByteArrayRegion(jbyteArray array, jsize start, jsize len, const jbyte* buf);
  void GetIntArrayRegion(jintArray array, jsize start, jsize len, jint* buf);
  void SetIntArrayRegion(jintArray array, jsize start, jsize len, const jint* buf);
  jstring NewStringUTF(const char* utf);
  jboolean ExceptionCheck();
  void* GetPrimitiveArrayCritical(jarray array, jboolean* isCopy);
  void ReleasePrimitiveArrayCritical(jarray array, void* carray, jint mode);
  jobject GetObjectArrayElement(jobjectArray array, jsize index);
  void DeleteLocalRef(jobject obj);
};
typedef JNIEnv_ JNIEnv;
#endif
