// JNI shim over the C ABI (reference rapidsml_jni.cpp + the JNI half of rapidsml_jni.cu).
// Java side: jvm/src/main/java/com/amd/spark/ml/linalg/JniSRML.java. Built by native/CMakeLists.txt
// when a JDK's jni.h exists; native/tests/jni_shim_test.cpp compiles this same file against a
// test-only JNIEnv (native/tests/jni_harness/jni.h) and runs every entry point on the GPU.
#include <jni.h>

#include <string>

#include "srml/srml.h"

namespace {
void throw_status(JNIEnv* env, const char* what, int rc) {
  jclass cls = env->FindClass("java/lang/RuntimeException");
  if (cls) env->ThrowNew(cls, (std::string(what) + " failed with status " + std::to_string(rc)).c_str());
}

void throw_arg(JNIEnv* env, const std::string& msg) {
  jclass cls = env->FindClass("java/lang/IllegalArgumentException");
  if (cls) env->ThrowNew(cls, msg.c_str());
}

// Pinned view of a Java double[]; released with mode 0 (copy back) or JNI_ABORT (read-only use).
struct DoubleArray {
  JNIEnv* env;
  jdoubleArray arr;
  jdouble* p;
  jint mode;
  DoubleArray(JNIEnv* e, jdoubleArray a, bool read_only)
      : env(e), arr(a), p(a ? e->GetDoubleArrayElements(a, nullptr) : nullptr), mode(read_only ? JNI_ABORT : 0) {}
  ~DoubleArray() {
    if (p) env->ReleaseDoubleArrayElements(arr, p, mode);
  }
  jsize size() const { return arr ? env->GetArrayLength(arr) : 0; }
};
}  // namespace

extern "C" {

// C (rows x k, row-major) = X (rows x n, row-major) . P (n x k, column-major = Spark DenseMatrix
// values) (N2/N6 dgemmWithColumnViewPtr). Column-major view: C^T (k x rows) = P^T X^T.
JNIEXPORT jdoubleArray JNICALL Java_com_amd_spark_ml_linalg_JniSRML_dgemm(JNIEnv* env, jclass, jdoubleArray x,
                                                                          jlong rows, jint n, jdoubleArray pc,
                                                                          jint k, jint device) {
  DoubleArray X(env, x, true), P(env, pc, true);
  if ((jlong)X.size() < rows * n || P.size() < n * k) {
    throw_arg(env, "dgemm: array shorter than rows*n or n*k");
    return nullptr;
  }
  jdoubleArray out = env->NewDoubleArray((jsize)(rows * k));
  if (!out) return nullptr;
  if (rows == 0 || k == 0) return out;
  DoubleArray C(env, out, false);
  const int rc = srml_capi_dgemm(1, 0, k, (int)rows, n, 1.0, P.p, n, X.p, n, 0.0, C.p, k, device);
  if (rc) throw_status(env, "dgemm", rc);
  return out;
}

// X^T X of a rows x cols row-major matrix (N3/N7 dgemmCov; returns the covariance instead of UB)
JNIEXPORT jdoubleArray JNICALL Java_com_amd_spark_ml_linalg_JniSRML_dgemmCov(JNIEnv* env, jclass, jdoubleArray x,
                                                                             jlong rows, jint cols, jint device) {
  DoubleArray X(env, x, true);
  if ((jlong)X.size() < rows * cols) {
    throw_arg(env, "dgemmCov: array shorter than rows*cols");
    return nullptr;
  }
  jdoubleArray out = env->NewDoubleArray(cols * cols);
  if (!out) return nullptr;
  DoubleArray C(env, out, false);
  const int rc = srml_capi_dgemm_cov(X.p, rows, cols, C.p, device);
  if (rc) throw_status(env, "dgemmCov", rc);
  return out;
}

// (N5 calSVD) U column-major m x m, S descending square roots of the eigenvalues
JNIEXPORT void JNICALL Java_com_amd_spark_ml_linalg_JniSRML_calSVD(JNIEnv* env, jclass, jint m, jdoubleArray a,
                                                                   jdoubleArray u, jdoubleArray s, jint device) {
  DoubleArray A(env, a, true), U(env, u, false), S(env, s, false);
  if (A.size() < m * m || U.size() < m * m || S.size() < m) {
    throw_arg(env, "calSVD: array shorter than m*m / m");
    return;
  }
  const int rc = srml_capi_cal_svd(A.p, m, U.p, S.p, device);
  if (rc) throw_status(env, "calSVD", rc);
}

// (N8 accumulateCov, implemented)
JNIEXPORT void JNICALL Java_com_amd_spark_ml_linalg_JniSRML_accumulateCov(JNIEnv* env, jclass, jdoubleArray acc,
                                                                          jdoubleArray c) {
  DoubleArray A(env, acc, false), C(env, c, true);
  if (A.size() != C.size()) {
    throw_arg(env, "accumulateCov: length mismatch");
    return;
  }
  srml_capi_accumulate_cov(A.p, C.p, A.size());
}

JNIEXPORT jstring JNICALL Java_com_amd_spark_ml_linalg_JniSRML_version(JNIEnv* env, jclass) {
  return env->NewStringUTF(srml_capi_version());
}
}
