// Compile-check stub of the parts of <jni.h> the JNI shim uses (no JDK in the build container).
// Member signatures follow the JNI C++ API; only type-checking depends on this file — the real
// shim is compiled against the JDK's header (oap_mllib_amd/build.py, JAVA_HOME).
#pragma once
#include <cstdint>
typedef int32_t jint;
typedef int64_t jlong;
typedef double jdouble;
typedef uint8_t jboolean;
typedef jint jsize;
class _jobject {};
typedef _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jthrowable;
typedef jobject jarray;
typedef jarray jdoubleArray;
struct _jfieldID;
typedef _jfieldID* jfieldID;
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
struct JNIEnv {
  jclass FindClass(const char*);
  jint ThrowNew(jclass, const char*);
  jclass GetObjectClass(jobject);
  jfieldID GetFieldID(jclass, const char*, const char*);
  void SetIntField(jobject, jfieldID, jint);
  void SetLongField(jobject, jfieldID, jlong);
  void SetDoubleField(jobject, jfieldID, jdouble);
  jstring NewStringUTF(const char*);
  const char* GetStringUTFChars(jstring, jboolean*);
  void ReleaseStringUTFChars(jstring, const char*);
  void GetDoubleArrayRegion(jdoubleArray, jsize, jsize, jdouble*);
  jdoubleArray NewDoubleArray(jsize);
  void SetDoubleArrayRegion(jdoubleArray, jsize, jsize, const jdouble*);
  void* GetDirectBufferAddress(jobject);
};
