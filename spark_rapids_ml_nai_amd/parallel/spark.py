"""Spark integration: barrier-mode fit stage, per-batch transform, stage-level scheduling.

Reference: ``_CumlCaller._call_cuml_fit_func`` / ``_train_udf`` (``core.py:622-787``) runs the
algorithm closure in ``mapInPandas(...).rdd.barrier().mapPartitions`` tasks, bootstraps NCCL by
sending the unique id through ``BarrierTaskContext.allGather`` (``common/cuml_context.py:35-124``)
and yields the model attributes from rank 0. Here the same stage runs our worker closure:

* rendezvous: every task ``allGather``s ``host:port`` (rank 0 binds a free port); rank 0 hosts the
  ``torch.distributed`` TCP store and the group comes up on RCCL (``"nccl"``) over xGMI / RoCE,
  or gloo for CPU tasks. Only this tiny bootstrap blob goes through the driver — every numeric
  exchange (partition sizes, moments, forests, kNN partials) is a device collective;
* device: the task's ``gpu`` resource address (cluster) or ``partitionId % device_count`` (local);
* ingest is Arrow end to end (``mapInArrow``): the partition's ``RecordBatch``es are wrapped into
  one table without copying, ``array<float>`` / VectorUDT values buffers are viewed as 2-D numpy
  arrays (no per-row Python objects, the reference's ``np.array(list(pdf[...]))`` at core.py:733),
  then -> ``HostPartition`` -> device (pinned staging) exactly like the Spark-free paths, so the same
  ``_fit_worker`` runs; transform builds its output columns as Arrow arrays the same way;
* failure: an exception aborts the communicator (``ncclCommAbort``), the barrier stage fails and
  Spark retries it as a whole (reference semantics);
* stage-level scheduling (``core.py:901-1004``): training tasks ask for a whole GPU and more than
  half the executor cores so that two training tasks never share an executor.

pyspark is optional: importing this module never requires it; the worker entry point works with
any object offering ``partitionId() / allGather(str) / barrier()`` (tests drive it with a
multi-process stand-in for ``BarrierTaskContext``).
"""
from __future__ import annotations

import os
import socket
from datetime import timedelta
from typing import Any, Callable, Dict, Iterable, Iterator, List, Optional, Tuple

import cloudpickle


def spark_available() -> bool:
    try:
        import pyspark  # noqa: F401

        return True
    except Exception:  # noqa: BLE001
        return False


def is_spark_dataframe(obj: Any) -> bool:
    mod = type(obj).__module__
    return mod.startswith("pyspark.sql") and type(obj).__name__ in ("DataFrame",)


# ------------------------------------------------------------------------------------------
# stage-level scheduling (pure decision logic, reference core.py:901-1004)
# ------------------------------------------------------------------------------------------
def _ver(v: str) -> Tuple[int, ...]:
    out = []
    for p in v.split(".")[:3]:
        digits = "".join(ch for ch in p if ch.isdigit())
        out.append(int(digits) if digits else 0)
    return tuple(out + [0] * (3 - len(out)))


def stage_level_scheduling_plan(spark_version: str, conf: Dict[str, Optional[str]], master: str,
                                spark_plugins: str = "", rapids_sql_enabled: str = "true",
                                reasons: Optional[List[str]] = None) -> Optional[Tuple[int, float]]:
    """(task_cores, task_gpus) for the training stage, or None to leave scheduling alone.
    ``reasons`` (optional list) receives the decision in words, as the reference logs it
    (``core.py:906-1004``)."""
    why = reasons if reasons is not None else []
    if master.startswith("local[") or master == "local":
        why.append("Stage level scheduling is not needed in local mode (%s)." % master)
        return None
    if _ver(spark_version) < (3, 4, 0):
        why.append("Stage level scheduling requires spark version 3.4.0+ (found %s)." % spark_version)
        return None
    standalone = master.startswith("spark://") or master.startswith("local-cluster")
    if (3, 4, 0) <= _ver(spark_version) < (3, 5, 1) and not standalone:
        why.append("Stage level scheduling on spark %s is supported only on standalone or local-cluster mode."
                   % spark_version)
        return None
    cores, gpus = conf.get("spark.executor.cores"), conf.get("spark.executor.resource.gpu.amount")
    if cores is None or gpus is None:
        why.append("Stage level scheduling requires spark.executor.cores and "
                   "spark.executor.resource.gpu.amount to be set.")
        return None
    if int(cores) == 1:
        why.append("Stage level scheduling is skipped: spark.executor.cores = 1 leaves nothing to reserve.")
        return None
    if float(gpus) > 1:
        why.append("Stage level scheduling is skipped: more than one GPU per executor "
                   "(spark.executor.resource.gpu.amount = %s)." % gpus)
        return None
    task_gpus = conf.get("spark.task.resource.gpu.amount")
    if task_gpus is not None and float(task_gpus) == float(gpus):
        why.append("Stage level scheduling is skipped: spark.task.resource.gpu.amount already equals the "
                   "executor's GPU amount, so a training task owns its GPU.")
        return None
    plugin_sql = "SQLPlugin" in (spark_plugins or "") and (rapids_sql_enabled or "true").lower() == "true"
    task_cores = int(cores) if plugin_sql else int(cores) // 2 + 1
    why.append("Training tasks require the resource(cores=%d, gpu=1.0)%s." %
               (task_cores, " (the SQL plugin is on: all executor cores)" if plugin_sql else ""))
    return task_cores, 1.0


def _try_stage_level_scheduling(rdd: Any, spark: Any) -> Any:
    from ..utils.log import get_logger

    sc = spark.sparkContext
    conf = {k: sc.getConf().get(k) for k in ("spark.executor.cores", "spark.executor.resource.gpu.amount",
                                             "spark.task.resource.gpu.amount")}
    reasons: List[str] = []
    plan = stage_level_scheduling_plan(spark.version, conf, sc.master, spark.conf.get("spark.plugins", ""),
                                       spark.conf.get("spark.rapids.sql.enabled", "true"), reasons)
    log = get_logger("stage_level_scheduling")
    for r in reasons:
        log.info(r)
    if plan is None:
        return rdd
    from pyspark.resource.profile import ResourceProfileBuilder  # type: ignore
    from pyspark.resource.requests import TaskResourceRequests  # type: ignore

    treqs = TaskResourceRequests().cpus(plan[0]).resource("gpu", plan[1])
    return rdd.withResources(ResourceProfileBuilder().require(treqs).build)


# ------------------------------------------------------------------------------------------
# worker side
# ------------------------------------------------------------------------------------------
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("", 0))
        return int(s.getsockname()[1])


def _local_ip() -> str:
    try:
        with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as s:
            s.connect(("10.255.255.255", 1))
            return s.getsockname()[0]
    except OSError:
        return "127.0.0.1"


def _task_device(task_ctx: Any, use_gpu: bool) -> Any:
    import torch

    if not use_gpu:
        return torch.device("cpu")
    addr = None
    try:
        res = task_ctx.resources()
        if "gpu" in res and res["gpu"].addresses:
            addr = int(res["gpu"].addresses[0])
    except Exception:  # noqa: BLE001 - stand-in contexts / local mode
        addr = None
    n = torch.cuda.device_count()
    if addr is None:
        addr = task_ctx.partitionId() % max(n, 1)
    return torch.device("cuda", addr % max(n, 1))


def init_barrier_group(task_ctx: Any, use_gpu: bool, timeout_s: float = 1800.0) -> Any:
    """torch.distributed bootstrap through the barrier allGather; returns a WorkerContext."""
    import torch
    import torch.distributed as dist

    from .context import WorkerContext

    rank = task_ctx.partitionId()
    host = os.environ.get("SRML_RENDEZVOUS_HOST") or _local_ip()
    port = _free_port() if rank == 0 else 0
    infos = task_ctx.allGather("%s:%d" % (host, port))
    world = len(infos)
    master_host, master_port = infos[0].rsplit(":", 1)
    device = _task_device(task_ctx, use_gpu)
    if device.type == "cuda":
        torch.cuda.set_device(device)
        from .context import bind_numa_local

        bind_numa_local(device)
    store = dist.TCPStore(master_host, int(master_port), world, is_master=(rank == 0),
                          timeout=timedelta(seconds=timeout_s))
    from .comm import comm_timeout

    dist.init_process_group("nccl" if device.type == "cuda" else "gloo", store=store, rank=rank, world_size=world,
                            timeout=timedelta(seconds=comm_timeout(timeout_s)),
                            **({"device_id": device} if device.type == "cuda" else {}))
    return WorkerContext.from_process_group(device)


def batches_to_table(batches: Iterable[Any], vector_cols: List[str], allow_empty: bool = False) -> Any:
    """Arrow ``RecordBatch``es (``mapInArrow``) — or pandas frames from older callers — of one
    partition -> ONE Arrow table without copying the column buffers (vector structs tagged as
    VectorUDT so the ingest reads their values buffers directly). An empty partition raises like
    the reference's fit UDF, or gives None with ``allow_empty``."""
    import pyarrow as pa

    from ..core.dataframe import vector_field

    rbs, tables = [], []
    for b in batches:
        if isinstance(b, pa.RecordBatch):
            rbs.append(b)
        elif isinstance(b, pa.Table):
            tables.append(b)
        else:  # pandas.DataFrame
            tables.append(pa.Table.from_pandas(b, preserve_index=False))
    if rbs:
        nonempty = [b for b in rbs if b.num_rows > 0] or rbs[:1]
        tables.append(pa.Table.from_batches(nonempty))
    if not tables:
        if allow_empty:
            return None
        raise RuntimeError("A worker received no data. Please increase amount of data or use fewer workers.")
    t = pa.concat_tables(tables) if len(tables) > 1 else tables[0]
    fields = [vector_field(f.name) if f.name in vector_cols else f for f in t.schema]
    return pa.Table.from_arrays(t.columns, schema=pa.schema(fields))


def spark_worker_entry(task_ctx: Any, batches: Iterable[Any], payload: bytes) -> Iterator[Any]:
    """Body of one barrier fit task (reference ``_train_udf``, core.py:694-779): Arrow batches in,
    one ``RecordBatch`` with the pickled model attributes out (rank 0)."""
    import pyarrow as pa

    from ..core.base import _fit_worker
    from ..core.dataframe import DataFrame
    from .context import use_context

    est, fit_fn, params, float32, vector_cols, use_gpu, *rest = cloudpickle.loads(payload)
    if rest and rest[0]:
        os.environ["SRML_UVM"] = "1"  # spark.rocm.ml.uvm.enabled: managed-memory ingest
    if len(rest) > 1 and rest[1]:
        os.environ["SRML_COMM"] = rest[1]  # spark.rocm.ml.comm: rccl | oneshot | auto
    ctx = init_barrier_group(task_ctx, use_gpu)
    try:
        table = batches_to_table(batches, vector_cols)
        hp = est._host_partition(DataFrame([table]))
        with use_context(ctx):
            res = _fit_worker(ctx, (hp, fit_fn, params, float32))
        ctx.comm.barrier()
    except BaseException:
        ctx.comm.abort()
        raise
    import torch.distributed as dist

    dist.destroy_process_group()
    if task_ctx.partitionId() == 0:
        yield pa.RecordBatch.from_pydict({"result": pa.array([cloudpickle.dumps(res)], type=pa.binary())})


def barrier_job_entry(task_ctx: Any, batches: Iterable[Any], payload: bytes) -> Iterator[Any]:
    """Body of one task of a generic barrier job (``spark_barrier_job``): bring up the rank's
    communicator, run ``fn(ctx, table, extra)`` on the partition's Arrow table (None when the
    partition is empty) and emit either its record batches or, for a collecting job, one row
    with the pickled ``(rank, result)``."""
    import pyarrow as pa

    from .context import use_context

    fn, extra, vector_cols, use_gpu, env, collect = cloudpickle.loads(payload)
    os.environ.update(env)
    ctx = init_barrier_group(task_ctx, use_gpu)
    try:
        table = batches_to_table(batches, vector_cols, allow_empty=True)
        with use_context(ctx):
            res = fn(ctx, table, extra)
            if collect:
                out = [pa.RecordBatch.from_pydict({"result": pa.array([cloudpickle.dumps((ctx.rank, res))],
                                                                      type=pa.binary())})]
            else:
                out = list(res)
        ctx.comm.barrier()
    except BaseException:
        ctx.comm.abort()
        raise
    import torch.distributed as dist

    dist.destroy_process_group()
    yield from out


def _worker_env(spark: Any) -> Dict[str, str]:
    """Driver-side settings every barrier task applies before it touches the device."""
    env = {"SRML_COMM": spark_comm_mode(spark)}
    if str(spark.conf.get("spark.rocm.ml.uvm.enabled", "false")).lower() == "true":
        env["SRML_UVM"] = "1"
    return env


def spark_barrier_job(sdf: Any, fn: Callable, extra: Any, out_schema: Any = None) -> Any:
    """Run ``fn(ctx, table, extra)`` in ONE barrier task per partition of ``sdf`` (one rank per GPU,
    RCCL bootstrapped through ``allGather``) — the shape of the reference's kNN / DBSCAN / UMAP
    jobs (``knn.py:558-624``, ``clustering.py:940-998``, ``umap.py:959-1077``).

    ``out_schema`` None: every rank's return value is collected to the driver (list in rank order).
    Otherwise ``fn`` yields Arrow record batches of that schema and the result is a DataFrame
    (computed lazily by Spark, like any other; nothing is collected)."""
    from .context import gpu_available

    spark = sdf.sparkSession
    sdf_u, vec = _unwrap_vectors(sdf)
    use_gpu = os.environ.get("SRML_FORCE_CPU", "0") != "1" and (gpu_available() or _cluster_has_gpus(spark))
    collect = out_schema is None
    payload = cloudpickle.dumps((fn, extra, vec, use_gpu, _worker_env(spark), collect))

    def _task(it: Iterator[Any]) -> Iterator[Any]:
        from pyspark import BarrierTaskContext  # type: ignore

        return barrier_job_entry(BarrierTaskContext.get(), it, payload)

    schema = "result binary" if collect else out_schema
    try:
        out = sdf_u.mapInArrow(_task, schema=schema, barrier=True)  # Spark >= 3.5
        rdd = None
    except TypeError:  # older Spark: barrier RDD over the mapped frame
        out = None
        rdd = sdf_u.mapInArrow(_task, schema=schema).rdd.barrier().mapPartitions(lambda x: x)
    if collect:
        rows = out.collect() if out is not None else rdd.collect()
        res = sorted((cloudpickle.loads(r["result"]) for r in rows), key=lambda t: t[0])
        return [r for _, r in res]
    return out if out is not None else spark.createDataFrame(rdd, out_schema)


def spark_map_partitions(sdf: Any, fn: Callable, extra: Any, out_schema: Any) -> Any:
    """Non-barrier per-partition job: ``fn(ctx, table, extra)`` yields record batches, on the task's
    pinned device (reference ``_transform_evaluate_internal``, core.py:1318-1417)."""
    sdf_u, vec = _unwrap_vectors(sdf)
    blob = cloudpickle.dumps((fn, extra, vec))

    def _run(it: Iterator[Any]) -> Iterator[Any]:
        import torch

        from pyspark import TaskContext  # type: ignore

        from .context import WorkerContext, gpu_available, use_context

        f, ex, vcols = cloudpickle.loads(blob)
        tc = TaskContext.get()
        dev = _task_device(tc, gpu_available()) if tc is not None else torch.device("cpu")
        ctx = WorkerContext.single(dev)
        table = batches_to_table(it, vcols, allow_empty=True)
        with use_context(ctx):
            yield from f(ctx, table, ex)

    return sdf_u.mapInArrow(_run, schema=out_schema)


# ------------------------------------------------------------------------------------------
# driver side
# ------------------------------------------------------------------------------------------
def _unwrap_vectors(sdf: Any) -> Tuple[Any, List[str]]:
    from pyspark.ml.linalg import VectorUDT  # type: ignore
    from pyspark.sql import functions as F  # type: ignore

    vec = [f.name for f in sdf.schema.fields if isinstance(f.dataType, VectorUDT)]
    for c in vec:
        sdf = sdf.withColumn(c, F.unwrap_udt(F.col(c)))
    return sdf, vec


def run_spark_fit(est: Any, sdf: Any, fit_fn: Callable, params: Dict[str, Any]) -> Any:
    from pyspark.sql import SparkSession  # type: ignore

    from .context import gpu_available

    spark = SparkSession.getActiveSession()
    nw = est.num_workers
    col, cols = est._get_input_columns()
    keep = list(cols or [col])
    if est._fit_uses_label():
        keep.append(est.getOrDefault("labelCol"))
    keep += [c for c in est._fit_extra_cols() if c in sdf.columns]
    sdf = sdf.select(*keep)
    if sdf.rdd.getNumPartitions() != nw:
        sdf = sdf.repartition(nw)
    sdf, vec = _unwrap_vectors(sdf)
    use_gpu = os.environ.get("SRML_FORCE_CPU", "0") != "1" and (gpu_available() or _cluster_has_gpus(spark))
    uvm = str(spark.conf.get("spark.rocm.ml.uvm.enabled", "false")).lower() == "true"
    payload = cloudpickle.dumps((est, fit_fn, params, est._float32_inputs, vec, use_gpu, uvm, spark_comm_mode(spark)))

    def _train(it: Iterator[Any]) -> Iterator[Any]:
        from pyspark import BarrierTaskContext  # type: ignore

        return spark_worker_entry(BarrierTaskContext.get(), it, payload)

    rdd = sdf.mapInArrow(_train, schema="result binary").rdd.barrier().mapPartitions(lambda x: x)
    rdd = _try_stage_level_scheduling(rdd, spark)
    rows = rdd.collect()
    return cloudpickle.loads(rows[0]["result"])


def spark_comm_mode(spark: Any) -> str:
    """``spark.rocm.ml.comm`` (rccl | oneshot | auto; default: the driver's ``SRML_COMM`` or rccl),
    validated on the driver so a typo fails before any barrier task starts."""
    from .oneshot import MODES

    mode = str(spark.conf.get("spark.rocm.ml.comm", os.environ.get("SRML_COMM", "rccl"))).lower()
    if mode not in MODES:
        raise ValueError("spark.rocm.ml.comm must be one of %s, got %r" % (MODES, mode))
    return mode


def _cluster_has_gpus(spark: Any) -> bool:
    return spark.sparkContext.getConf().get("spark.executor.resource.gpu.amount") is not None


def spark_transform(model: Any, sdf: Any) -> Any:
    """Per-batch transform with the model's device predict function (reference ``_transform``,
    core.py:1419-1435 / 1537-1557): one model construction per task, pinned device per task,
    Arrow in / Arrow out (``mapInArrow``): outputs are appended as Arrow columns (2-D results as
    ``list<double>`` over the flat values buffer), never as per-row Python lists."""
    import numpy as np
    import pyarrow as pa

    from ..core.dataframe import DataFrame, dense_to_list_array

    out_fields = model._spark_output_fields(sdf)
    if _vector_columns(sdf):
        # Spark < 4 cannot move a VectorUDT through Arrow: pass the features as arrays through a
        # scalar-iterator pandas UDF and keep every original column (reference core.py:1537-1557)
        return _spark_transform_udf(model, sdf, out_fields)
    sdf_u, vec = _unwrap_vectors(sdf)
    blob = cloudpickle.dumps((_task_model(model, sdf), vec))
    model._spark_closure_bytes = len(blob)

    def _predict(it: Iterator[Any]) -> Iterator[Any]:
        import torch

        from pyspark import TaskContext  # type: ignore

        from .context import WorkerContext, gpu_available

        m, vcols = cloudpickle.loads(blob)
        tc = TaskContext.get()
        dev = _task_device(tc, gpu_available()) if tc is not None else torch.device("cpu")
        ctx = WorkerContext.single(dev)
        construct, predict = m._get_transform_func(None)
        state = construct(ctx)
        for rb in it:
            if rb.num_rows == 0:
                continue
            table = batches_to_table([rb], vcols)
            X = m._transform_features(DataFrame([table]))
            res = predict(state, X, ctx)
            cols, names = list(rb.columns), list(rb.schema.names)
            for k, v in res.items():
                v = np.asarray(v)
                cols.append(dense_to_list_array(v.astype(np.float64)) if v.ndim == 2 else pa.array(v.astype(np.float64)))
                names.append(k)
            yield pa.RecordBatch.from_arrays(cols, names=names)

    schema = sdf_u.schema
    from pyspark.sql.types import StructType  # type: ignore

    out_schema = StructType(list(schema.fields) + out_fields)
    out = sdf_u.mapInArrow(_predict, schema=out_schema)
    return _wrap_vector_outputs(model, out, out_fields, False)


def _task_model(model: Any, sdf: Any) -> Any:
    """What the transform tasks unpickle: the model itself, or — for models holding training
    data (UMAP: embedding + raw rows) — a light copy whose arrays travel as chunked Spark
    broadcasts (``_spark_task_model``), so the task closure stays small at any data size."""
    hook = getattr(model, "_spark_task_model", None)
    return hook(sdf.sparkSession) if hook is not None else model


def collect_arrow(sdf: Any) -> Any:
    """The rows of ``sdf`` on the driver as ONE Arrow table (Spark 4 ``toArrow``, the Arrow
    collection behind ``toPandas`` on older versions, or a pandas round trip)."""
    import pyarrow as pa

    if hasattr(sdf, "toArrow"):
        return sdf.toArrow()
    if hasattr(sdf, "_collect_as_arrow"):
        rbs = sdf._collect_as_arrow()
        return pa.Table.from_batches(rbs) if rbs else None
    return pa.Table.from_pandas(sdf.toPandas(), preserve_index=False)


def _vector_columns(sdf: Any) -> List[str]:
    try:
        from pyspark.ml.linalg import VectorUDT  # type: ignore
    except Exception:  # noqa: BLE001
        return []
    return [f.name for f in sdf.schema.fields if isinstance(f.dataType, VectorUDT)]


def _wrap_vector_outputs(model: Any, out: Any, out_fields: List[Any], input_is_vector: bool) -> Any:
    """Vector-typed outputs travel as list<double>; Spark wraps them as VectorUDT (array_to_vector)
    so pyspark evaluators / VectorAssembler consume them directly (reference core.py:1559-1610)."""
    names = [f.name for f in out_fields]
    to_vec = [c for c in model._spark_vector_output_cols(input_is_vector) if c in names]
    if to_vec:
        from pyspark.ml.functions import array_to_vector  # type: ignore
        from pyspark.sql import functions as F  # type: ignore

        for c in to_vec:
            out = out.withColumn(c, array_to_vector(F.col(c)))
    return out


def _spark_transform_udf(model: Any, sdf: Any, out_fields: List[Any]) -> Any:
    """Transform of a frame holding VectorUDT columns: ``withColumn`` of a scalar-iterator pandas UDF
    over ``struct(vector_to_array(features))`` returning a struct of the outputs, expanded into
    columns — every input column (vectors included) is kept as it was."""
    import numpy as np
    import pandas as pd
    import pyarrow as pa

    from pyspark.ml.functions import vector_to_array  # type: ignore
    from pyspark.sql import functions as F  # type: ignore
    from pyspark.sql.functions import pandas_udf  # type: ignore
    from pyspark.sql.types import StructType  # type: ignore

    from ..core.dataframe import DataFrame

    col, cols = model._transform_input_cols()
    vec = _vector_columns(sdf)
    dt = "float32" if getattr(model, "_float32_inputs", True) else "float64"
    inputs = [vector_to_array(F.col(c), dt).alias(c) if c in vec else F.col(c) for c in ([col] if col else cols)]
    blob = cloudpickle.dumps(_task_model(model, sdf))
    model._spark_closure_bytes = len(blob)

    def _udf(it: Iterator[pd.DataFrame]) -> Iterator[pd.DataFrame]:
        import torch

        from pyspark import TaskContext  # type: ignore

        from .context import WorkerContext, gpu_available

        m = cloudpickle.loads(blob)
        tc = TaskContext.get()
        dev = _task_device(tc, gpu_available()) if tc is not None else torch.device("cpu")
        ctx = WorkerContext.single(dev)
        construct, predict = m._get_transform_func(None)
        state = construct(ctx)
        for pdf in it:
            table = pa.Table.from_pandas(pdf, preserve_index=False)
            res = predict(state, m._transform_features(DataFrame([table])), ctx) if table.num_rows else {}
            yield pd.DataFrame({k: (list(np.asarray(v, np.float64)) if np.ndim(v) == 2 else np.asarray(v, np.float64))
                                for k, v in res.items()})

    _udf.__annotations__ = {"it": Iterator[pd.DataFrame], "return": Iterator[pd.DataFrame]}
    predict_udf = pandas_udf(_udf, returnType=StructType(out_fields))
    tmp = "__srml_out"
    out = sdf.withColumn(tmp, predict_udf(F.struct(*inputs)))
    for f in out_fields:
        out = out.withColumn(f.name, F.col("%s.%s" % (tmp, f.name)))
    out = out.drop(tmp)
    return _wrap_vector_outputs(model, out, out_fields, bool(col) and col in vec)
