/*
 * JNI entry points of libsrml_jni.so (native/jni/srml_jni.cpp) over the MI355X C ABI (libsrml.so).
 * Parity with the reference's JniRAPIDSML (jvm/src/main/java/com/nvidia/spark/ml/linalg/
 * JniRAPIDSML.java:26-78): the shared libraries are found on java.library.path or extracted from
 * the jar (/<os.arch>/<os.name>/, where the Maven build bundles them) and loaded once.
 * libsrml.so (the gfx950 kernels) is loaded first so the shim's DT_NEEDED entry resolves from the
 * same temporary directory.
 */
package com.amd.spark.ml.linalg;

import java.io.File;
import java.io.IOException;
import java.io.InputStream;
import java.nio.file.Files;
import java.nio.file.StandardCopyOption;

public final class JniSRML {
  private static volatile boolean loaded = false;
  private static volatile Throwable loadError = null;

  private JniSRML() {}

  /** Loads the native libraries; throws UnsatisfiedLinkError when they are unavailable. */
  public static synchronized void load() {
    if (loaded) {
      return;
    }
    if (loadError != null) {
      throw new UnsatisfiedLinkError("libsrml_jni unavailable: " + loadError);
    }
    try {
      try {
        System.loadLibrary("srml");
        System.loadLibrary("srml_jni");
      } catch (UnsatisfiedLinkError e) {
        File dir = Files.createTempDirectory("srml_native").toFile();
        dir.deleteOnExit();
        System.load(extract("libsrml.so", dir));
        System.load(extract("libsrml_jni.so", dir));
      }
      loaded = true;
    } catch (Throwable t) {
      loadError = t;
      throw (t instanceof UnsatisfiedLinkError) ? (UnsatisfiedLinkError) t
          : new UnsatisfiedLinkError("cannot load libsrml_jni: " + t);
    }
  }

  /** True when the native path can be used (loads on first call; never throws). */
  public static boolean isAvailable() {
    try {
      load();
      return true;
    } catch (Throwable t) {
      return false;
    }
  }

  private static String extract(String name, File dir) throws IOException {
    String res = "/" + System.getProperty("os.arch") + "/" + System.getProperty("os.name") + "/" + name;
    try (InputStream in = JniSRML.class.getResourceAsStream(res)) {
      if (in == null) {
        throw new UnsatisfiedLinkError(name + " not found on java.library.path nor at " + res);
      }
      File out = new File(dir, name);
      out.deleteOnExit();
      Files.copy(in, out.toPath(), StandardCopyOption.REPLACE_EXISTING);
      return out.getAbsolutePath();
    }
  }

  /** C (rows x k) = X (rows x n) . P (n x k); row-major host arrays; P column-major like Spark's DenseMatrix. */
  public static native double[] dgemm(double[] x, long rows, int n, double[] pc, int k, int device);

  /** X^T X (cols x cols) of a rows x cols row-major matrix. */
  public static native double[] dgemmCov(double[] x, long rows, int cols, int device);

  /** Eigendecomposition of a symmetric m x m matrix: U column-major (descending), S = sqrt(eigenvalues). */
  public static native void calSVD(int m, double[] a, double[] u, double[] s, int device);

  /** acc += c (element-wise). */
  public static native void accumulateCov(double[] acc, double[] c);

  /** Version string of the native library (for diagnostics). */
  public static native String version();
}
