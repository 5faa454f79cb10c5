/*
 * Scala facade over JniSRML (reference RAPIDSML.scala:27-157: cov, gemm, calSVD, accumulateCov).
 * The device id comes from the task's "gpu" resource (Spark GPU scheduling), else 0 — the
 * reference's `TaskContext.get().resources()("gpu")` rule (RapidsPCA.scala:130-134).
 */
package com.amd.spark.ml.linalg

import org.apache.spark.TaskContext

object SRML {

  /** GPU ordinal of the running task (0 in local mode / on the driver). */
  def taskDevice: Int = {
    val tc = TaskContext.get()
    if (tc == null) 0
    else tc.resources().get("gpu").flatMap(_.addresses.headOption).map(_.toInt).getOrElse(0)
  }

  /** True when libsrml_jni.so (and libsrml.so under it) can be loaded in this JVM. */
  def available: Boolean = JniSRML.isAvailable()

  /** Uncentred X^T X (cols x cols, symmetric) of one block of rows (rows x cols, row-major). */
  def cov(rows: Array[Double], numRows: Long, numCols: Int, device: Int = taskDevice): Array[Double] = {
    JniSRML.load()
    JniSRML.dgemmCov(rows, numRows, numCols, device)
  }

  /** rows (numRows x n, row-major) . pc (n x k, column-major as in Spark's DenseMatrix) -> numRows x k row-major. */
  def gemm(rows: Array[Double], numRows: Long, n: Int, pc: Array[Double], k: Int,
           device: Int = taskDevice): Array[Double] = {
    JniSRML.load()
    JniSRML.dgemm(rows, numRows, n, pc, k, device)
  }

  /** (U column-major, S descending = sqrt(eigenvalues)) of a symmetric m x m matrix. */
  def calSVD(m: Int, a: Array[Double], device: Int = taskDevice): (Array[Double], Array[Double]) = {
    JniSRML.load()
    val u = new Array[Double](m * m)
    val s = new Array[Double](m)
    JniSRML.calSVD(m, a, u, s, device)
    (u, s)
  }

  /** acc += c, returns acc. */
  def accumulateCov(acc: Array[Double], c: Array[Double]): Array[Double] = {
    require(acc.length == c.length, s"length mismatch ${acc.length} vs ${c.length}")
    if (JniSRML.isAvailable()) JniSRML.accumulateCov(acc, c)
    else {
      var i = 0
      while (i < acc.length) { acc(i) += c(i); i += 1 }
    }
    acc
  }
}
