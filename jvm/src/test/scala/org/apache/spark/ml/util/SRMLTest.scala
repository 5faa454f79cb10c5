/*
 * Local-session base for the JVM tests (reference jvm/src/test/scala/org/apache/spark/ml/util/
 * RapidsMLTest.scala:21-33). No spark-rapids plugin: the native path is the JNI library, so the
 * session only needs local[2] and a small shuffle-partition count.
 */
package org.apache.spark.ml.util

import org.apache.spark.SparkConf
import org.apache.spark.sql.test.SharedSparkSession

trait SRMLTest extends org.apache.spark.SparkFunSuite with SharedSparkSession with TempDirectory {

  override protected def sparkConf: SparkConf = super.sparkConf
    .set("spark.master", "local[2]")
    .set("spark.sql.shuffle.partitions", "2")
    .set("spark.rocm.ml.uvm.enabled", "false")
}
