/*
 * Drop-in PCA class name for Spark applications (reference com.nvidia.spark.ml.feature.PCA,
 * jvm/src/main/scala/com/nvidia/spark/ml/feature/PCA.scala:27-37): swap the import
 * `org.apache.spark.ml.feature.PCA` for `com.amd.spark.ml.feature.PCA` and the fit / transform run
 * on MI355X (org.apache.spark.ml.feature.RapidsPCA).
 */
package com.amd.spark.ml.feature

import org.apache.spark.ml.feature.RapidsPCA
import org.apache.spark.ml.util.{DefaultParamsReadable, Identifiable}

class PCA(override val uid: String) extends RapidsPCA(uid) {

  def this() = this(Identifiable.randomUID("pca"))
}

object PCA extends DefaultParamsReadable[PCA] {
  override def load(path: String): PCA = super.load(path)
}
