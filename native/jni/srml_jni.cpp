// JNI shim over the C ABI (reference rapidsml_jni.cpp + the JNI half of rapidsml_jni.cu).
// Built only when a JDK's jni.h is available (see native/CMakeLists.txt, SRML_BUILD_JNI).
// Java side: jvm/src/main/java/com/amd/spark/ml/linalg/JniSRML.java.
#include <jni.h>

#include <string>

#include "srml/srml.h"

namespace {
void throw_status(JNIEnv* env, const char* what, int rc) {
  jclass cls = env->FindClass("java/lang/RuntimeException");
  if (cls) env->ThrowNew(cls, (std::string(what) + " failed with status " + std::to_string(rc)).c_str());
}

struct DoubleArray {
  JNIEnv* env;
  jdoubleArray arr;
  jdouble* p;
  DoubleArray(JNIEnv* e, jdoubleArray a) : env(e), arr(a), p(a ? e->GetDoubleArrayElements(a, nullptr) : nullptr) {}
  ~DoubleArray() {
    if (p) env->ReleaseDoubleArrayElements(arr, p, 0);
  }
};
}  // namespace

extern "C" {

// C (rows x k) = X (rows x n) . P (n x k), row-major host arrays (N2/N6 dgemmWithColumnViewPtr)
JNIEXPORT jdoubleArray JNICALL Java_com_amd_spark_ml_linalg_JniSRML_dgemm(JNIEnv* env, jclass, jdoubleArray x,
                                                                          jlong rows, jint n, jdoubleArray pc,
                                                                          jint k, jint device) {
  DoubleArray X(env, x), P(env, pc);
  jdoubleArray out = env->NewDoubleArray((jsize)(rows * k));
  DoubleArray C(env, out);
  // row-major C = X P  <=>  column-major C^T = P^T X^T
  const int rc = srml_capi_dgemm(0, 0, k, (int)rows, n, 1.0, P.p, k, X.p, n, 0.0, C.p, k, device);
  if (rc) throw_status(env, "dgemm", rc);
  return out;
}

// X^T X of a rows x cols row-major matrix (N3/N7 dgemmCov; returns the covariance instead of UB)
JNIEXPORT jdoubleArray JNICALL Java_com_amd_spark_ml_linalg_JniSRML_dgemmCov(JNIEnv* env, jclass, jdoubleArray x,
                                                                             jlong rows, jint cols, jint device) {
  DoubleArray X(env, x);
  jdoubleArray out = env->NewDoubleArray(cols * cols);
  DoubleArray C(env, out);
  const int rc = srml_capi_dgemm_cov(X.p, rows, cols, C.p, device);
  if (rc) throw_status(env, "dgemmCov", rc);
  return out;
}

// (N5 calSVD) U column-major m x m, S descending square roots of the eigenvalues
JNIEXPORT void JNICALL Java_com_amd_spark_ml_linalg_JniSRML_calSVD(JNIEnv* env, jclass, jint m, jdoubleArray a,
                                                                   jdoubleArray u, jdoubleArray s, jint device) {
  DoubleArray A(env, a), U(env, u), S(env, s);
  const int rc = srml_capi_cal_svd(A.p, m, U.p, S.p, device);
  if (rc) throw_status(env, "calSVD", rc);
}

// (N8 accumulateCov, implemented)
JNIEXPORT void JNICALL Java_com_amd_spark_ml_linalg_JniSRML_accumulateCov(JNIEnv* env, jclass, jdoubleArray acc,
                                                                          jdoubleArray c) {
  DoubleArray A(env, acc), C(env, c);
  srml_capi_accumulate_cov(A.p, C.p, env->GetArrayLength(acc));
}
}
