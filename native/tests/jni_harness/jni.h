// Test-only stand-in for a JDK's <jni.h>: the subset of the JNI C++ API that
// native/jni/srml_jni.cpp uses, backed by host objects, so the shim can be compiled and executed
// without a JVM (native/tests/jni_shim_test.cpp). Array pinning has copy semantics (what HotSpot
// does for Get<Type>ArrayElements): a missing copy-back or a release with the wrong mode shows up
// as a wrong result, and leaked pins are counted.
#ifndef SRML_TEST_JNI_H_
#define SRML_TEST_JNI_H_

#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_COMMIT 1
#define JNI_ABORT 2

typedef int32_t jint;
typedef int64_t jlong;
typedef double jdouble;
typedef uint8_t jboolean;
typedef jint jsize;

struct _jobject {
  virtual ~_jobject() = default;
};
struct _jclass : _jobject {
  std::string name;
};
struct _jstring : _jobject {
  std::string s;
};
struct _jarray : _jobject {};
struct _jdoubleArray : _jarray {
  std::vector<double> v;
};
typedef _jobject* jobject;
typedef _jclass* jclass;
typedef _jstring* jstring;
typedef _jarray* jarray;
typedef _jdoubleArray* jdoubleArray;

struct JNIEnv_ {
  std::string exception_class, exception_msg;  // pending exception (last ThrowNew)
  int pins = 0;                                // Get...Elements without a matching Release
  std::vector<std::unique_ptr<_jobject>> heap;

  template <class T>
  T* own(T* o) {
    heap.emplace_back(o);
    return o;
  }
  jclass FindClass(const char* name) {
    auto* c = own(new _jclass);
    c->name = name;
    return c;
  }
  jint ThrowNew(jclass c, const char* msg) {
    exception_class = c->name;
    exception_msg = msg;
    return 0;
  }
  jdoubleArray NewDoubleArray(jsize n) {
    if (n < 0) return nullptr;
    auto* a = own(new _jdoubleArray);
    a->v.assign((size_t)n, 0.0);
    return a;
  }
  jsize GetArrayLength(jarray a) { return (jsize)static_cast<_jdoubleArray*>(a)->v.size(); }
  jdouble* GetDoubleArrayElements(jdoubleArray a, jboolean* is_copy) {
    if (is_copy) *is_copy = 1;
    double* p = new double[a->v.size() + 1];
    if (!a->v.empty()) std::memcpy(p, a->v.data(), a->v.size() * sizeof(double));
    ++pins;
    return p;
  }
  void ReleaseDoubleArrayElements(jdoubleArray a, jdouble* p, jint mode) {
    if (mode != JNI_ABORT && !a->v.empty()) std::memcpy(a->v.data(), p, a->v.size() * sizeof(double));
    if (mode != JNI_COMMIT) {
      delete[] p;
      --pins;
    }
  }
  jstring NewStringUTF(const char* s) {
    auto* o = own(new _jstring);
    o->s = s ? s : "";
    return o;
  }
};
typedef JNIEnv_ JNIEnv;

#endif  // SRML_TEST_JNI_H_
