/*
 * JNI entry points of libsrml_jni.so (native/jni/srml_jni.cpp) over the MI355X C ABI.
 * Parity with the reference's JniRAPIDSML (jvm/src/main/java/com/nvidia/spark/ml/linalg/
 * JniRAPIDSML.java:26-78): the shared library is extracted from the jar (or found on
 * java.library.path) and loaded once.
 */
package com.amd.spark.ml.linalg;

import java.io.File;
import java.io.IOException;
import java.io.InputStream;
import java.nio.file.Files;
import java.nio.file.StandardCopyOption;

public final class JniSRML {
  private static volatile boolean loaded = false;

  private JniSRML() {}

  public static synchronized void load() {
    if (loaded) {
      return;
    }
    try {
      System.loadLibrary("srml_jni");
    } catch (UnsatisfiedLinkError e) {
      String res = "/" + System.getProperty("os.arch") + "/" + System.getProperty("os.name") + "/libsrml_jni.so";
      try (InputStream in = JniSRML.class.getResourceAsStream(res)) {
        if (in == null) {
          throw new UnsatisfiedLinkError("libsrml_jni.so not found on java.library.path nor at " + res);
        }
        File tmp = File.createTempFile("libsrml_jni", ".so");
        tmp.deleteOnExit();
        Files.copy(in, tmp.toPath(), StandardCopyOption.REPLACE_EXISTING);
        System.load(tmp.getAbsolutePath());
      } catch (IOException io) {
        throw new UnsatisfiedLinkError("cannot extract libsrml_jni.so: " + io);
      }
    }
    loaded = true;
  }

  /** C (rows x k) = X (rows x n) . P (n x k); row-major host arrays. */
  public static native double[] dgemm(double[] x, long rows, int n, double[] pc, int k, int device);

  /** X^T X (cols x cols) of a rows x cols row-major matrix. */
  public static native double[] dgemmCov(double[] x, long rows, int cols, int device);

  /** Eigendecomposition of a symmetric m x m matrix: U column-major (descending), S = sqrt(eigenvalues). */
  public static native void calSVD(int m, double[] a, double[] u, double[] s, int device);

  /** acc += c (element-wise). */
  public static native void accumulateCov(double[] acc, double[] c);
}
