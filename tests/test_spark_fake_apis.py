"""Spark-DataFrame reach of the APIs beyond fit/transform (reference knn.py:558-749 / 1154-1427,
clustering.py:1013-1091, umap.py:830-1077, tuning.py:39-177, core.py:1559-1610), executed against
the test-only pyspark stand-in (tests/fakespark): barrier jobs run one spawned process per
partition over gloo. Each result is checked against an oracle: brute-force numpy for kNN, the
in-process fit for DBSCAN, pyspark's own generic CrossValidator loop on the same folds. What only
a real cluster can show (JVM planning, Arrow IPC, UDT handling of a real Spark) is parity unpinned."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = [pytest.mark.dist, pytest.mark.slow]


@pytest.fixture(scope="module")
def result():
    env = dict(os.environ, SRML_FORCE_CPU="1", OMP_NUM_THREADS="2",
               PYTHONPATH=os.pathsep.join([os.path.join(ROOT, "tests", "fakespark"), ROOT]))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "spark_fake_apis_driver.py")], env=env,
                       capture_output=True, text=True, timeout=1500, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-5000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")][-1]
    return json.loads(line[len("RESULT "):])


def test_exact_knn_barrier_job(result):
    assert result["knn_rows"] == 50 and result["knn_sorted"]
    assert result["knn_exact_frac"] == 1.0 and result["knn_dist_err"] < 1e-4
    assert result["join_columns"] == ["item_df", "query_df", "d"] and result["join_rows"] == 50 * 4


def test_ann_barrier_job(result):
    # nprobe == nlist probes every list: the IVF search must return the exact neighbours
    assert result["ann_rows"] == 50 and result["ann_recall_vs_exact"] >= 0.999
    assert result["ann_join_rows"] == 50 * 4


def test_dbscan_spark_transform(result):
    assert result["dbscan_rows"] == 400
    assert set(result["dbscan_columns"]) == {"features", "unique_id", "prediction"}
    assert result["dbscan_nclusters"] == result["dbscan_nclusters_local"] == 3


def test_umap_spark_fit_transform(result):
    assert result["umap_embedding_shape"] == [300, 2]
    assert result["umap_transform_columns"] == ["features", "embedding"] and result["umap_transform_rows"] == 300


def test_umap_spark_chunked(result):
    """Reference tests/test_umap.py:333-377: tiny limits force several fit batches and broadcasts;
    the result equals the in-process fit / transform and no training data rides in the closure."""
    assert result["umap_fit_batches"] == 5  # 300 rows / maxRecordsPerBatch 64
    assert result["umap_chunked_fit_equal"]
    assert result["umap_broadcasts"] == [2, 4] and result["umap_new_broadcasts"] == 6
    assert result["umap_new_broadcasts_2nd"] == 6  # reused, not re-broadcast
    assert result["umap_closure_bytes"] < result["umap_raw_bytes"]
    assert result["umap_chunked_transform_maxdiff"] < 1e-4


def test_vector_udt_outputs(result):
    assert result["lr_types"]["probability"] == result["lr_types"]["rawPrediction"] == "VectorUDT"
    assert result["lr_types"]["features"] == "ArrayType"
    # a VectorUDT input keeps its type (pandas-UDF path) and predicts the same labels
    assert result["lr_vec_types"]["features"] == "VectorUDT" and result["lr_vec_pred_match"]
    assert result["pca_vec_out"] == "VectorUDT" and result["pca_arr_out"] == "ArrayType"


def test_cross_validator_is_pyspark_and_matches_generic(result):
    assert result["cv_is_pyspark"] and result["cv_model_is_pyspark"]
    for fast, gen in (("cv_avg", "cv_generic_avg"), ("cvc_f1", "cvc_f1_generic"),
                      ("cvc_logLoss", "cvc_logLoss_generic")):
        assert result[fast] == pytest.approx(result[gen], rel=1e-9, abs=1e-12), fast
