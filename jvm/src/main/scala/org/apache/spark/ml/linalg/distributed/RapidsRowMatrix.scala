/*
 * Distributed row matrix whose covariance and eigendecomposition run on MI355X through the C ABI.
 *
 * Parity: reference RapidsRowMatrix (jvm/src/main/scala/org/apache/spark/ml/linalg/distributed/
 * RapidsRowMatrix.scala:30-141): per-partition X^T X on the GPU, reduced, then `calSVD` in a
 * one-task job on an executor GPU. Differences by design:
 *  - mean centring is implemented (the reference's `meanCentering` was a TODO): each partition
 *    also returns its row count and column sums, and C = (X^T X - m mu mu^T) / (m - 1), the
 *    sample covariance Spark's RowMatrix.computePrincipalComponents uses;
 *  - rows are read as Spark vectors or numeric arrays (no spark-rapids ColumnarRdd / cudf), in
 *    blocks of `blockRows` rows so a partition never has to fit in one host array, and the
 *    partial Grams are combined with treeAggregate (depth 2) instead of a driver reduce;
 *  - without the native library (no GPU on this host) the same math runs on the CPU (Breeze),
 *    so the class is usable in CPU-only test JVMs.
 */
package org.apache.spark.ml.linalg.distributed

import breeze.linalg.{eigSym, DenseMatrix => BDM}
import com.amd.spark.ml.linalg.SRML
import org.apache.spark.internal.Logging
import org.apache.spark.ml.linalg.{DenseMatrix, DenseVector, Vector => MLVector}
import org.apache.spark.sql.DataFrame

import scala.collection.mutable

class RapidsRowMatrix(val rowsDf: DataFrame, val meanCentering: Boolean, private val nCols: Int,
                      val blockRows: Int = 8192) extends Logging with Serializable {

  def numCols: Int = nCols

  /** Top-k principal components (n x k, column-major) and the explained-variance ratios. */
  def computePrincipalComponentsAndExplainedVariance(k: Int): (DenseMatrix, DenseVector) = {
    val n = nCols
    require(k > 0 && k <= n, s"k = $k out of range (0, n = $n]")
    val cov = computeCovariance()
    val (u, s) = eigen(cov, n)
    val eig = s.map(x => x * x) // calSVD returns sqrt(eigenvalues)
    val total = eig.sum
    val ev = if (total > 0) eig.map(_ / total) else eig
    (new DenseMatrix(n, k, java.util.Arrays.copyOfRange(u, 0, n * k)),
      new DenseVector(java.util.Arrays.copyOfRange(ev, 0, k)))
  }

  /** Covariance (n x n, row-major == column-major: symmetric) of the rows. */
  def computeCovariance(): Array[Double] = {
    val n = nCols
    val bs = blockRows
    val zero = (0L, new Array[Double](n), new Array[Double](n * n))
    val (m, sums, xtx) = rowsDf.rdd.mapPartitions { it =>
      val useGpu = SRML.available
      val dev = SRML.taskDevice
      val buf = new Array[Double](bs * n)
      val sum = new Array[Double](n)
      val acc = new Array[Double](n * n)
      var count = 0L
      var r = 0
      def flush(): Unit = if (r > 0) {
        val blk = if (r == bs) buf else java.util.Arrays.copyOf(buf, r * n)
        val c = if (useGpu) SRML.cov(blk, r, n, dev) else RapidsRowMatrix.cpuGram(blk, r, n)
        SRML.accumulateCov(acc, c)
        r = 0
      }
      it.foreach { row =>
        RapidsRowMatrix.copyRow(row.get(0), buf, r * n, n)
        var j = 0
        val off = r * n
        while (j < n) { sum(j) += buf(off + j); j += 1 }
        r += 1
        count += 1
        if (r == bs) flush()
      }
      flush()
      Iterator.single((count, sum, acc))
    }.treeAggregate(zero)(
      (a, b) => RapidsRowMatrix.merge(a, b),
      (a, b) => RapidsRowMatrix.merge(a, b),
      2)
    require(m > 0, "PCA needs at least one row")
    val denom = math.max(m - 1, 1).toDouble
    val out = new Array[Double](n * n)
    if (meanCentering) {
      val mu = sums.map(_ / m)
      var i = 0
      while (i < n) {
        var j = 0
        while (j < n) { out(i * n + j) = (xtx(i * n + j) - m * mu(i) * mu(j)) / denom; j += 1 }
        i += 1
      }
    } else {
      var i = 0
      while (i < n * n) { out(i) = xtx(i) / denom; i += 1 }
    }
    out
  }

  /** (U column-major, S = sqrt(eigenvalues) descending): one-task job on an executor GPU, like the
   *  reference; falls back to Breeze's eigSym when no native library is loadable there. */
  private def eigen(cov: Array[Double], n: Int): (Array[Double], Array[Double]) = {
    val sc = rowsDf.sparkSession.sparkContext
    val res = sc.parallelize(Seq(0), 1).mapPartitions { _ =>
      Iterator.single(if (SRML.available) SRML.calSVD(n, cov) else RapidsRowMatrix.cpuEig(cov, n))
    }.collect()
    res.head
  }
}

object RapidsRowMatrix {

  /** Copy one row (ml Vector or numeric array) into buf[off, off + n). */
  def copyRow(v: Any, buf: Array[Double], off: Int, n: Int): Unit = v match {
    case vec: MLVector =>
      require(vec.size == n, s"row has ${vec.size} features, expected $n")
      java.util.Arrays.fill(buf, off, off + n, 0.0)
      vec.foreachActive((i, x) => buf(off + i) = x)
    case a: mutable.WrappedArray[_] =>
      require(a.length == n, s"row has ${a.length} features, expected $n")
      var j = 0
      while (j < n) {
        buf(off + j) = a(j) match {
          case d: Double => d
          case f: Float => f.toDouble
          case x: Number => x.doubleValue()
        }
        j += 1
      }
    case s: Seq[_] => copyRow(mutable.WrappedArray.make[Any](s.toArray[Any]), buf, off, n)
    case null => throw new IllegalArgumentException("null feature row")
    case other => throw new IllegalArgumentException(s"unsupported feature type ${other.getClass}")
  }

  def numColsOf(v: Any): Int = v match {
    case vec: MLVector => vec.size
    case a: Seq[_] => a.length
    case other => throw new IllegalArgumentException(s"unsupported feature type ${other.getClass}")
  }

  private[distributed] def merge(a: (Long, Array[Double], Array[Double]),
                                 b: (Long, Array[Double], Array[Double])): (Long, Array[Double], Array[Double]) = {
    SRML.accumulateCov(a._2, b._2)
    SRML.accumulateCov(a._3, b._3)
    (a._1 + b._1, a._2, a._3)
  }

  /** CPU X^T X of a row-major block (fallback when no GPU library is loadable). */
  def cpuGram(x: Array[Double], rows: Int, n: Int): Array[Double] = {
    val g = new Array[Double](n * n)
    var r = 0
    while (r < rows) {
      val off = r * n
      var i = 0
      while (i < n) {
        val xi = x(off + i)
        if (xi != 0.0) {
          var j = 0
          while (j < n) { g(i * n + j) += xi * x(off + j); j += 1 }
        }
        i += 1
      }
      r += 1
    }
    g
  }

  /** CPU calSVD equivalent: descending eigenpairs, sqrt eigenvalues, max-|x| entry positive. */
  def cpuEig(a: Array[Double], n: Int): (Array[Double], Array[Double]) = {
    val es = eigSym(new BDM[Double](n, n, a.clone()))
    val order = (0 until n).sortBy(i => -es.eigenvalues(i))
    val u = new Array[Double](n * n)
    val s = new Array[Double](n)
    order.zipWithIndex.foreach { case (src, dst) =>
      s(dst) = math.sqrt(math.max(es.eigenvalues(src), 0.0))
      var big = 0
      var i = 0
      while (i < n) {
        if (math.abs(es.eigenvectors(i, src)) > math.abs(es.eigenvectors(big, src))) big = i
        i += 1
      }
      val sign = if (es.eigenvectors(big, src) < 0) -1.0 else 1.0
      i = 0
      while (i < n) { u(dst * n + i) = sign * es.eigenvectors(i, src); i += 1 }
    }
    (u, s)
  }
}
