"""ML persistence with the reference's on-disk layout.

Estimator: ``<path>/metadata/part-00000`` = one JSON line (Spark ``DefaultParamsWriter``
fields: class, timestamp, sparkVersion, uid, paramMap, defaultParamMap) plus
``_cuml_params``, ``_num_workers``, ``_float32_inputs`` (reference ``core.py:249-288``).
Model: the same metadata plus ``<path>/data/part-00000`` holding ONE JSON line of model
attributes (``core.py:291-336``); ``Model._from_row`` rebuilds it. Large numeric attributes
(UMAP embeddings, raw data) are written as ``.npy`` side files instead of JSON
(reference ``umap.py:1262-1327``).
"""
from __future__ import annotations

import importlib
import json
import os
import shutil
import threading
import time
from typing import Any, Dict, Optional, Type

import numpy as np

SPARK_VERSION_TAG = "3.5.0"  # metadata compatibility tag (no Spark needed)
_save_state = threading.local()


def _jsonable(v: Any) -> Any:
    if isinstance(v, np.ndarray):
        return v.tolist()
    if isinstance(v, (np.floating, np.integer, np.bool_)):
        return v.item()
    if isinstance(v, dict):
        return {str(k): _jsonable(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_jsonable(x) for x in v]
    return v


def _write_text(path: str, text: str) -> None:
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "part-00000"), "w") as f:
        f.write(text + "\n")
    open(os.path.join(path, "_SUCCESS"), "w").close()


def _read_text(path: str) -> str:
    with open(os.path.join(path, "part-00000")) as f:
        return f.read().strip()


def param_map_json(instance: Any) -> Dict[str, Any]:
    return {
        "paramMap": {p.name: _jsonable(v) for p, v in instance._paramMap.items()},
        "defaultParamMap": {p.name: _jsonable(v) for p, v in instance._defaultParamMap.items()},
    }


class MLWriter:
    def __init__(self, instance: Any) -> None:
        self.instance = instance
        self.shouldOverwrite = False

    def overwrite(self) -> "MLWriter":
        self.shouldOverwrite = True
        return self

    def option(self, key: str, value: Any) -> "MLWriter":
        return self

    def session(self, spark: Any) -> "MLWriter":
        return self

    def save(self, path: str) -> None:
        """Write the instance to ``path``.

        In an SPMD job (torchrun: every rank holds the same fitted model) only rank 0 writes, the
        way the reference's Spark driver is the only writer (``core.py:249-336``); the other ranks
        wait for rank 0's outcome (one object broadcast) and raise the same error if it failed, so
        a ``load`` on any rank after ``save`` returns sees the complete directory. A barrier opens
        the save, so no rank is still reading an earlier model at the path when rank 0 replaces it.
        The directory is written under a temporary sibling name and renamed into place, so a
        reader never sees a half-written model."""
        from ..parallel.context import current_context, spmd_active, spmd_context

        if not spmd_active() or getattr(_save_state, "nested", False):
            # single process, or a sub-model written from inside rank 0's save (CrossValidatorModel's
            # bestModel): plain local write, no collective
            self._save_local(path)
            return
        ctx = current_context() or spmd_context()
        # the save is a collective: every rank has arrived (so no rank is still reading an earlier
        # model at this path) before rank 0 replaces the directory
        ctx.comm.barrier()
        err = None
        if ctx.rank == 0:
            _save_state.nested = True
            try:
                self._save_local(path)
            except Exception as e:  # noqa: BLE001 - re-raised below, on every rank
                err = (type(e).__name__, str(e))
            finally:
                _save_state.nested = False
        err = ctx.comm.broadcast_object(err, src=0)
        if err is not None:
            kind, msg = err
            raise (IOError if kind in ("OSError", "IOError", "FileExistsError", "PermissionError")
                   else RuntimeError)("model save on rank 0 failed: %s: %s" % (kind, msg))

    def _save_local(self, path: str) -> None:
        path = os.path.abspath(path)
        if os.path.exists(path) and not self.shouldOverwrite:
            raise IOError("Path %s already exists. Use write().overwrite().save(path)." % path)
        parent = os.path.dirname(path)
        os.makedirs(parent, exist_ok=True)
        tmp = os.path.join(parent, ".%s.tmp-%d-%d" % (os.path.basename(path), os.getpid(), time.monotonic_ns()))
        try:
            self.saveImpl(tmp)
            if os.path.exists(path):
                shutil.rmtree(path)
            os.rename(tmp, path)
        finally:
            if os.path.exists(tmp):
                shutil.rmtree(tmp, ignore_errors=True)

    def _metadata(self, extra: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
        inst = self.instance
        md = {
            "class": inst.__class__.__module__ + "." + inst.__class__.__name__,
            "timestamp": int(round(time.time() * 1000)),
            "sparkVersion": SPARK_VERSION_TAG,
            "uid": inst.uid,
        }
        md.update(param_map_json(inst))
        md.update(extra or {})
        return md

    def saveImpl(self, path: str) -> None:
        raise NotImplementedError


class EstimatorWriter(MLWriter):
    def saveImpl(self, path: str) -> None:
        inst = self.instance
        md = self._metadata(
            {
                "_cuml_params": _jsonable(inst._backend_params),
                "_num_workers": inst._num_workers,
                "_float32_inputs": inst._float32_inputs,
            }
        )
        _write_text(os.path.join(path, "metadata"), json.dumps(md))


class ModelWriter(MLWriter):
    def saveImpl(self, path: str) -> None:
        inst = self.instance
        md = self._metadata(
            {
                "_cuml_params": _jsonable(inst._backend_params),
                "_num_workers": inst._num_workers,
                "_float32_inputs": inst._float32_inputs,
            }
        )
        _write_text(os.path.join(path, "metadata"), json.dumps(md))
        attrs = inst._get_model_attributes()
        arrays = {k: v for k, v in attrs.items() if isinstance(v, np.ndarray) and v.size > 65536}
        plain = {k: v for k, v in attrs.items() if k not in arrays}
        data_path = os.path.join(path, "data")
        _write_text(data_path, json.dumps(_jsonable(plain)))
        for k, v in arrays.items():
            np.save(os.path.join(data_path, k + ".npy"), v, allow_pickle=False)
        if arrays:
            with open(os.path.join(data_path, "_npy_attrs.json"), "w") as f:
                json.dump(sorted(arrays), f)


def _load_class(name: str) -> Type:
    mod, _, cls = name.rpartition(".")
    return getattr(importlib.import_module(mod), cls)


def _apply_params(inst: Any, md: Dict[str, Any]) -> None:
    for name, v in md.get("defaultParamMap", {}).items():
        if inst.hasParam(name):
            inst._defaultParamMap[inst.getParam(name)] = v
    for name, v in md.get("paramMap", {}).items():
        if inst.hasParam(name):
            inst._set(**{name: v})
    if "_cuml_params" in md:
        inst._backend_params = md["_cuml_params"]
    inst._num_workers = md.get("_num_workers")
    inst._float32_inputs = md.get("_float32_inputs", True)


class MLReader:
    def __init__(self, cls: Type) -> None:
        self.cls = cls

    def session(self, spark: Any) -> "MLReader":
        return self

    def load(self, path: str) -> Any:
        raise NotImplementedError


class EstimatorReader(MLReader):
    def load(self, path: str) -> Any:
        md = json.loads(_read_text(os.path.join(path, "metadata")))
        cls = self.cls if self.cls is not None else _load_class(md["class"])
        inst = cls()
        inst._resetUid(md["uid"])
        _apply_params(inst, md)
        return inst


class ModelReader(MLReader):
    def load(self, path: str) -> Any:
        md = json.loads(_read_text(os.path.join(path, "metadata")))
        data_path = os.path.join(path, "data")
        attrs = json.loads(_read_text(data_path))
        npy_list = os.path.join(data_path, "_npy_attrs.json")
        if os.path.exists(npy_list):
            with open(npy_list) as f:
                for k in json.load(f):
                    attrs[k] = np.load(os.path.join(data_path, k + ".npy"), allow_pickle=False)
        cls = self.cls if self.cls is not None else _load_class(md["class"])
        inst = cls._from_row(attrs)
        inst._resetUid(md["uid"])
        _apply_params(inst, md)
        return inst


class MLWritable:
    def write(self) -> MLWriter:
        raise NotImplementedError

    def save(self, path: str) -> None:
        self.write().save(path)


class MLReadable:
    @classmethod
    def read(cls) -> MLReader:
        raise NotImplementedError

    @classmethod
    def load(cls, path: str) -> Any:
        return cls.read().load(path)
