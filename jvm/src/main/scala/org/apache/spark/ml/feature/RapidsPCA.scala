/*
 * PCA estimator / model whose fit (covariance + eigendecomposition) and transform (projection)
 * run on MI355X through the C ABI (libsrml.so via libsrml_jni.so).
 *
 * Parity: reference RapidsPCA / RapidsPCAModel (jvm/src/main/scala/org/apache/spark/ml/feature/
 * RapidsPCA.scala:34-230): `meanCentering` param, fit through RapidsRowMatrix, model transform
 * on the GPU with a CPU fallback, parquet persistence of (pc, explainedVariance).
 * Differences by design (MI355X-first, no spark-rapids / cudf on ROCm):
 *  - transform batches `transformBatchRows` rows of a partition into one row-major host block
 *    and projects it with ONE device GEMM per block (the reference registered a cudf columnar
 *    RapidsUDF that only worked under the spark-rapids plugin, RapidsPCA.scala:128-165);
 *  - the output column is a Spark ML vector (drop-in for org.apache.spark.ml.feature.PCAModel)
 *    and the input may be a vector or a numeric array column;
 *  - `meanCentering` is honoured (centred sample covariance, Spark RowMatrix semantics);
 *  - the saved data layout equals Spark's PCAModel (pc, explainedVariance), and `cpu()` returns
 *    an org.apache.spark.ml.feature.PCAModel.
 */
package org.apache.spark.ml.feature

import com.amd.spark.ml.linalg.SRML
import org.apache.hadoop.fs.Path
import org.apache.spark.ml._
import org.apache.spark.ml.attribute.AttributeGroup
import org.apache.spark.ml.linalg._
import org.apache.spark.ml.linalg.distributed.RapidsRowMatrix
import org.apache.spark.ml.param._
import org.apache.spark.ml.util._
import org.apache.spark.sql._
import org.apache.spark.sql.types._

trait RapidsPCAParams extends PCAParams {

  /** Whether to centre the data before the covariance (default true). @group param */
  final val meanCentering: BooleanParam =
    new BooleanParam(this, "meanCentering", "whether to apply mean centering")

  /** Rows per device GEMM in fit (covariance blocks) and transform. @group expertParam */
  final val transformBatchRows: IntParam = new IntParam(this, "transformBatchRows",
    "rows per device GEMM block in fit and transform", ParamValidators.gt(0))

  setDefault(meanCentering -> true, transformBatchRows -> 8192)

  def getMeanCentering: Boolean = $(meanCentering)

  def getTransformBatchRows: Int = $(transformBatchRows)

  /** Input: vector or array<double|float>; output: vector of size k. */
  protected def validateAndTransformSchemaAnyInput(schema: StructType): StructType = {
    val inType = schema($(inputCol)).dataType
    inType match {
      case _: VectorUDT =>
      case ArrayType(DoubleType, _) | ArrayType(FloatType, _) =>
      case other => throw new IllegalArgumentException(
        s"Column ${$(inputCol)} must be a vector or array<double|float>, got ${other.catalogString}")
    }
    require(!schema.fieldNames.contains($(outputCol)), s"Output column ${$(outputCol)} already exists.")
    StructType(schema.fields :+ new AttributeGroup($(outputCol), $(k)).toStructField())
  }
}

class RapidsPCA(override val uid: String)
  extends Estimator[RapidsPCAModel] with RapidsPCAParams with DefaultParamsWritable {

  def this() = this(Identifiable.randomUID("pca"))

  def setInputCol(value: String): this.type = set(inputCol, value)

  def setOutputCol(value: String): this.type = set(outputCol, value)

  def setK(value: Int): this.type = set(k, value)

  def setMeanCentering(value: Boolean): this.type = set(meanCentering, value)

  def setTransformBatchRows(value: Int): this.type = set(transformBatchRows, value)

  override def fit(dataset: Dataset[_]): RapidsPCAModel = {
    transformSchema(dataset.schema, logging = true)
    val input = dataset.select($(inputCol))
    val first = input.head()
    val numCols = RapidsRowMatrix.numColsOf(first.get(0))
    require($(k) <= numCols, s"source vector size $numCols must be no less than k=${$(k)}")
    val mat = new RapidsRowMatrix(input.toDF(), $(meanCentering), numCols, $(transformBatchRows))
    val (pc, explainedVariance) = mat.computePrincipalComponentsAndExplainedVariance($(k))
    copyValues(new RapidsPCAModel(uid, pc, explainedVariance).setParent(this))
  }

  override def transformSchema(schema: StructType): StructType = validateAndTransformSchemaAnyInput(schema)

  override def copy(extra: ParamMap): RapidsPCA = defaultCopy(extra)
}

object RapidsPCA extends DefaultParamsReadable[RapidsPCA] {
  override def load(path: String): RapidsPCA = super.load(path)
}

/**
 * @param pc                principal components (n x k), one component per column
 * @param explainedVariance proportion of variance explained by each component
 */
class RapidsPCAModel(override val uid: String, val pc: DenseMatrix, val explainedVariance: DenseVector)
  extends Model[RapidsPCAModel] with RapidsPCAParams with MLWritable {

  import RapidsPCAModel._

  def setInputCol(value: String): this.type = set(inputCol, value)

  def setOutputCol(value: String): this.type = set(outputCol, value)

  def setTransformBatchRows(value: Int): this.type = set(transformBatchRows, value)

  /** Project every row on the components: one device GEMM per block of `transformBatchRows` rows. */
  override def transform(dataset: Dataset[_]): DataFrame = {
    val outSchema = transformSchema(dataset.schema, logging = true)
    val df = dataset.toDF()
    val inIdx = df.schema.fieldIndex($(inputCol))
    val n = pc.numRows
    val kk = pc.numCols
    val bcPc = df.sparkSession.sparkContext.broadcast(pc.toArray) // column-major n x k
    val bs = $(transformBatchRows)
    val rdd = df.rdd.mapPartitions { it =>
      val useGpu = SRML.available
      val dev = SRML.taskDevice
      val p = bcPc.value
      it.grouped(bs).flatMap { grp =>
        val rows = grp.length
        val buf = new Array[Double](rows * n)
        var r = 0
        grp.foreach { row => RapidsRowMatrix.copyRow(row.get(inIdx), buf, r * n, n); r += 1 }
        val out = if (useGpu) SRML.gemm(buf, rows, n, p, kk, dev) else cpuProject(buf, rows, n, p, kk)
        grp.iterator.zipWithIndex.map { case (row, i) =>
          Row.fromSeq(row.toSeq :+ Vectors.dense(java.util.Arrays.copyOfRange(out, i * kk, (i + 1) * kk)))
        }
      }
    }
    df.sparkSession.createDataFrame(rdd, outSchema)
  }

  override def transformSchema(schema: StructType): StructType = validateAndTransformSchemaAnyInput(schema)

  /** Spark's own model (CPU transform), same components / variances / params. */
  def cpu(): PCAModel = {
    val m = new PCAModel(uid, pc, explainedVariance)
    m.set(m.k, $(k)).set(m.inputCol, $(inputCol)).set(m.outputCol, $(outputCol))
  }

  override def copy(extra: ParamMap): RapidsPCAModel = {
    val copied = new RapidsPCAModel(uid, pc, explainedVariance)
    copyValues(copied, extra).setParent(parent)
  }

  override def write: MLWriter = new RapidsPCAModelWriter(this)

  override def toString: String = s"RapidsPCAModel: uid=$uid, k=${$(k)}"
}

object RapidsPCAModel extends MLReadable[RapidsPCAModel] {

  /** rows (rows x n, row-major) . pc (n x k, column-major) on the CPU (fallback path). */
  private[feature] def cpuProject(x: Array[Double], rows: Int, n: Int, p: Array[Double], k: Int): Array[Double] = {
    val out = new Array[Double](rows * k)
    var r = 0
    while (r < rows) {
      var c = 0
      while (c < k) {
        var s = 0.0
        var j = 0
        while (j < n) { s += x(r * n + j) * p(c * n + j); j += 1 }
        out(r * k + c) = s
        c += 1
      }
      r += 1
    }
    out
  }

  override def read: MLReader[RapidsPCAModel] = new RapidsPCAModelReader

  override def load(path: String): RapidsPCAModel = super.load(path)

  private case class Data(pc: DenseMatrix, explainedVariance: DenseVector)

  private[RapidsPCAModel] class RapidsPCAModelWriter(instance: RapidsPCAModel) extends MLWriter {
    override protected def saveImpl(path: String): Unit = {
      DefaultParamsWriter.saveMetadata(instance, path, sc)
      val dataPath = new Path(path, "data").toString
      sparkSession.createDataFrame(Seq(Data(instance.pc, instance.explainedVariance)))
        .repartition(1).write.parquet(dataPath)
    }
  }

  private class RapidsPCAModelReader extends MLReader[RapidsPCAModel] {
    private val className = classOf[RapidsPCAModel].getName

    override def load(path: String): RapidsPCAModel = {
      val metadata = DefaultParamsReader.loadMetadata(path, sc, className)
      val dataPath = new Path(path, "data").toString
      val Row(pc: DenseMatrix, explainedVariance: DenseVector) =
        sparkSession.read.parquet(dataPath).select("pc", "explainedVariance").head()
      val model = new RapidsPCAModel(metadata.uid, pc, explainedVariance)
      metadata.getAndSetParams(model)
      model
    }
  }
}
