// Compile-check stub of the parts of <jni.h> the JNI shim uses (no JDK in the build container).
// Member signatures follow the JNI C++ API; the real shim is compiled against the JDK's header
// (oap_mllib_amd/build.py, JAVA_HOME).  tests/native/jni_harness.cpp defines these members with
// a recording, type-checking fake VM so the shim's entry points run in the test suite.
#pragma once
#include <cstdint>
typedef int32_t jint;
typedef int64_t jlong;
typedef double jdouble;
typedef float jfloat;
typedef uint8_t jboolean;
typedef jint jsize;
class _jobject {
 public:
  virtual ~_jobject() = default;
};
typedef _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jthrowable;
typedef jobject jarray;
typedef jarray jdoubleArray;
typedef jarray jfloatArray;
typedef jarray jlongArray;
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
  jsize GetArrayLength(jarray);
  void GetDoubleArrayRegion(jdoubleArray, jsize, jsize, jdouble*);
  void GetFloatArrayRegion(jfloatArray, jsize, jsize, jfloat*);
  void GetLongArrayRegion(jlongArray, jsize, jsize, jlong*);
  jdoubleArray NewDoubleArray(jsize);
  void SetDoubleArrayRegion(jdoubleArray, jsize, jsize, const jdouble*);
  void* GetDirectBufferAddress(jobject);
  jlong GetDirectBufferCapacity(jobject);
  jobject NewDirectByteBuffer(void*, jlong);
};
