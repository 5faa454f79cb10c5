/*
 * Drop-in Spark ML PCA backed by the MI355X C ABI (reference com.nvidia.spark.ml.feature.PCA +
 * RapidsPCA / RapidsRowMatrix, jvm/src/main/scala/...:27-230). Differences by design: the
 * covariance IS mean-centred (the reference left a TODO and used X^T X), and the explained
 * variance uses eigenvalues / trace like Spark (the reference divided sqrt(eigenvalues)).
 */
package com.amd.spark.ml.feature

import com.amd.spark.ml.linalg.SRML
import org.apache.spark.ml.feature.{PCA => SparkPCA, PCAModel}
import org.apache.spark.ml.linalg.{DenseMatrix, DenseVector, Vector => MLVector}
import org.apache.spark.ml.util.Identifiable
import org.apache.spark.sql.{Dataset, Row}

class PCA(override val uid: String) extends SparkPCA(uid) {

  def this() = this(Identifiable.randomUID("pca"))

  override def fit(dataset: Dataset[_]): PCAModel = {
    val k = $(this.k)
    val rows = dataset.select($(inputCol)).rdd.map {
      case Row(v: MLVector) => v.toArray
      case Row(a: Seq[_]) => a.map(_.toString.toDouble).toArray
    }
    val n = rows.first().length
    // per partition: (count, column sums, X^T X) on the GPU, reduced on the driver
    val (m, sums, xtx) = rows.mapPartitions { it =>
      val buf = it.toArray
      val flat = buf.flatten
      val s = new Array[Double](n)
      buf.foreach(r => { var j = 0; while (j < n) { s(j) += r(j); j += 1 } })
      Iterator((buf.length.toLong, s, if (buf.isEmpty) new Array[Double](n * n) else SRML.cov(flat, buf.length, n)))
    }.treeReduce { case ((m1, s1, c1), (m2, s2, c2)) =>
      (m1 + m2, s1.zip(s2).map { case (a, b) => a + b }, SRML.accumulateCov(c1, c2))
    }
    val mean = sums.map(_ / m)
    val cov = Array.tabulate(n * n) { idx =>
      val i = idx / n
      val j = idx % n
      (xtx(idx) - m * mean(i) * mean(j)) / math.max(m - 1, 1)
    }
    val (u, s) = SRML.calSVD(n, cov)
    val eig = s.map(x => x * x)
    val total = eig.sum
    val pc = new DenseMatrix(n, k, u.slice(0, n * k), false)
    val ev = new DenseVector(eig.take(k).map(_ / total))
    copyValues(new PCAModel(uid, pc, ev).setParent(this))
  }
}
