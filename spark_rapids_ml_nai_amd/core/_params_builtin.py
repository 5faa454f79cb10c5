"""Built-in implementation of the ``pyspark.ml.param`` API (``Param``, ``Params``,
``TypeConverters``, ``keyword_only``): same method names and semantics (defaults vs. user-set
values, ``copy(extra)``, ``extractParamMap``, ``explainParams``, ``_resetUid``), used when pyspark
is not importable (or ``SRML_PYSPARK=0``). ``core/params.py`` picks pyspark's classes instead when
pyspark is present, so estimators then ARE ``pyspark.ml`` Params/Estimators/Models.
"""
from __future__ import annotations

import copy as _copy
import functools
import uuid
from typing import Any, Callable, Dict, List, Optional, TypeVar, Union

import numpy as np

# --------------------------------------------------------------------------------------
# TypeConverters
# --------------------------------------------------------------------------------------
class TypeConverters:
    """Same converters (and error behaviour) as ``pyspark.ml.param.TypeConverters``."""

    @staticmethod
    def _is_numeric(value: Any) -> bool:
        return isinstance(value, (int, float, np.integer, np.floating)) and not isinstance(
            value, bool
        )

    @staticmethod
    def _is_integer(value: Any) -> bool:
        return TypeConverters._is_numeric(value) and float(value).is_integer()

    @staticmethod
    def _can_convert_to_list(value: Any) -> bool:
        return isinstance(value, (list, tuple, np.ndarray, range)) or hasattr(value, "toArray")

    @staticmethod
    def identity(value: Any) -> Any:
        return value

    @staticmethod
    def toList(value: Any) -> List:
        if type(value) == list:
            return value
        if TypeConverters._can_convert_to_list(value):
            if hasattr(value, "toArray"):
                return list(value.toArray())
            return list(value)
        raise TypeError("Could not convert %s to list" % value)

    @staticmethod
    def toListFloat(value: Any) -> List[float]:
        v = TypeConverters.toList(value)
        if all(TypeConverters._is_numeric(x) for x in v):
            return [float(x) for x in v]
        raise TypeError("Could not convert %s to list of floats" % value)

    @staticmethod
    def toListListFloat(value: Any) -> List[List[float]]:
        return [TypeConverters.toListFloat(x) for x in TypeConverters.toList(value)]

    @staticmethod
    def toListInt(value: Any) -> List[int]:
        v = TypeConverters.toList(value)
        if all(TypeConverters._is_integer(x) for x in v):
            return [int(x) for x in v]
        raise TypeError("Could not convert %s to list of ints" % value)

    @staticmethod
    def toListString(value: Any) -> List[str]:
        v = TypeConverters.toList(value)
        if all(isinstance(x, str) for x in v):
            return [str(x) for x in v]
        raise TypeError("Could not convert %s to list of strings" % value)

    @staticmethod
    def toVector(value: Any) -> Any:
        from .linalg import Vectors

        if hasattr(value, "toArray") and hasattr(value, "size"):
            return value
        if TypeConverters._can_convert_to_list(value):
            v = TypeConverters.toList(value)
            if all(TypeConverters._is_numeric(x) for x in v):
                return Vectors.dense(v)
        raise TypeError("Could not convert %s to vector" % value)

    @staticmethod
    def toMatrix(value: Any) -> Any:
        if hasattr(value, "toArray") and hasattr(value, "numRows"):
            return value
        raise TypeError("Could not convert %s to matrix" % value)

    @staticmethod
    def toFloat(value: Any) -> float:
        if TypeConverters._is_numeric(value):
            return float(value)
        raise TypeError("Could not convert %s to float" % value)

    @staticmethod
    def toInt(value: Any) -> int:
        if TypeConverters._is_integer(value):
            return int(value)
        raise TypeError("Could not convert %s to int" % value)

    @staticmethod
    def toString(value: Any) -> str:
        if isinstance(value, str):
            return value
        if isinstance(value, np.str_):
            return str(value)
        raise TypeError("Could not convert %s to string type" % type(value))

    @staticmethod
    def toBoolean(value: Any) -> bool:
        if type(value) == bool or isinstance(value, np.bool_):
            return bool(value)
        raise TypeError("Boolean Param requires value of type bool. Found %s." % type(value))


# --------------------------------------------------------------------------------------
# Param / Params
# --------------------------------------------------------------------------------------
class _Dummy:
    uid = "undefined"


class Param:
    """A param with self-contained documentation (pyspark.ml.param.Param equivalent)."""

    def __init__(
        self,
        parent: Any,
        name: str,
        doc: str,
        typeConverter: Optional[Callable[[Any], Any]] = None,
    ) -> None:
        if not isinstance(parent, _Dummy) and not hasattr(parent, "uid"):
            raise TypeError("Parent must be a Params object but got %s" % type(parent))
        self.parent = parent.uid
        self.name = str(name)
        self.doc = str(doc)
        self.typeConverter = TypeConverters.identity if typeConverter is None else typeConverter

    def _copy_new_parent(self, parent: Any) -> "Param":
        if self.parent == "undefined":
            param = _copy.copy(self)
            param.parent = parent.uid
            return param
        raise ValueError("Cannot copy from non-dummy parent %s." % parent)

    def __str__(self) -> str:
        return str(self.parent) + "__" + self.name

    def __repr__(self) -> str:
        return "Param(parent=%r, name=%r, doc=%r)" % (self.parent, self.name, self.doc)

    def __hash__(self) -> int:
        return hash(str(self))

    def __eq__(self, other: Any) -> bool:
        if isinstance(other, Param):
            return self.parent == other.parent and self.name == other.name
        return False


def keyword_only(func: Callable) -> Callable:
    """Only allow keyword arguments; stores them in ``self._input_kwargs`` (pyspark semantics)."""

    @functools.wraps(func)
    def wrapper(self: Any, *args: Any, **kwargs: Any) -> Any:
        if len(args) > 0:
            raise TypeError("Method %s forces keyword arguments." % func.__name__)
        self._input_kwargs = kwargs
        return func(self, **kwargs)

    return wrapper


class Params:
    """Components that take parameters (pyspark.ml.param.Params equivalent)."""

    @staticmethod
    def _dummy() -> _Dummy:
        return _Dummy()

    def __init__(self) -> None:
        self.uid = self._randomUID()
        self._paramMap: Dict[Param, Any] = {}
        self._defaultParamMap: Dict[Param, Any] = {}
        self._params: Optional[List[Param]] = None
        self._copy_params()

    @classmethod
    def _randomUID(cls) -> str:
        return cls.__name__ + "_" + uuid.uuid4().hex[-12:]

    def _copy_params(self) -> None:
        cls = type(self)
        src_name_attrs = [(x, getattr(cls, x)) for x in dir(cls)]
        src_params = [(n, a) for n, a in src_name_attrs if isinstance(a, Param)]
        for name, param in src_params:
            setattr(self, name, param._copy_new_parent(self))

    @property
    def params(self) -> List[Param]:
        if self._params is None:
            self._params = [
                getattr(self, x)
                for x in dir(self)
                if x != "params" and not isinstance(getattr(type(self), x, None), property)
                and isinstance(getattr(self, x), Param)
            ]
        return self._params

    def explainParam(self, param: Union[str, Param]) -> str:
        param = self._resolveParam(param)
        values = []
        if self.isDefined(param):
            if param in self._defaultParamMap:
                values.append("default: %s" % self._defaultParamMap[param])
            if param in self._paramMap:
                values.append("current: %s" % self._paramMap[param])
        else:
            values.append("undefined")
        return "%s: %s (%s)" % (param.name, param.doc, ", ".join(values))

    def explainParams(self) -> str:
        return "\n".join([self.explainParam(p) for p in self.params])

    def getParam(self, paramName: str) -> Param:
        param = getattr(self, paramName, None)
        if isinstance(param, Param):
            return param
        raise ValueError("Cannot find param with name %s." % paramName)

    def hasParam(self, paramName: str) -> bool:
        if isinstance(paramName, str):
            p = getattr(self, paramName, None)
            return isinstance(p, Param)
        raise TypeError("hasParam(): paramName must be a string")

    def isSet(self, param: Union[str, Param]) -> bool:
        return self._resolveParam(param) in self._paramMap

    def hasDefault(self, param: Union[str, Param]) -> bool:
        return self._resolveParam(param) in self._defaultParamMap

    def isDefined(self, param: Union[str, Param]) -> bool:
        return self.isSet(param) or self.hasDefault(param)

    def getOrDefault(self, param: Union[str, Param]) -> Any:
        param = self._resolveParam(param)
        if param in self._paramMap:
            return self._paramMap[param]
        if param in self._defaultParamMap:
            return self._defaultParamMap[param]
        raise KeyError("Param %s is not set and has no default." % param.name)

    def extractParamMap(self, extra: Optional[Dict[Param, Any]] = None) -> Dict[Param, Any]:
        if extra is None:
            extra = dict()
        paramMap = self._defaultParamMap.copy()
        paramMap.update(self._paramMap)
        paramMap.update(extra)
        return paramMap

    def copy(self: "P_", extra: Optional[Dict[Param, Any]] = None) -> "P_":
        if extra is None:
            extra = dict()
        that = _copy.copy(self)
        that._paramMap = {}
        that._defaultParamMap = {}
        return self._copyValues(that, extra)

    def set(self, param: Param, value: Any) -> None:
        self._shouldOwn(param)
        try:
            value = param.typeConverter(value)
        except ValueError as e:
            raise ValueError('Invalid param value given for param "%s". %s' % (param.name, e))
        self._paramMap[param] = value

    def _shouldOwn(self, param: Param) -> None:
        if not (self.uid == param.parent and self.hasParam(param.name)):
            raise ValueError("Param %r does not belong to %r." % (param, self))

    def _resolveParam(self, param: Union[str, Param]) -> Param:
        if isinstance(param, Param):
            self._shouldOwn(param)
            return param
        if isinstance(param, str):
            return self.getParam(param)
        raise TypeError("Cannot resolve %r as a param." % param)

    def clear(self, param: Param) -> None:
        if self.isSet(param):
            del self._paramMap[self._resolveParam(param)]

    def _set(self: "P_", **kwargs: Any) -> "P_":
        for param, value in kwargs.items():
            p = getattr(self, param)
            if value is not None:
                try:
                    value = p.typeConverter(value)
                except TypeError as e:
                    raise TypeError('Invalid param value given for param "%s". %s' % (p.name, e))
            self._paramMap[p] = value
        return self

    def _clear(self, param: Param) -> None:
        self.clear(param)

    def _setDefault(self: "P_", **kwargs: Any) -> "P_":
        for param, value in kwargs.items():
            p = getattr(self, param)
            if value is not None and not isinstance(value, dict):
                try:
                    value = p.typeConverter(value)
                except TypeError as e:
                    raise TypeError(
                        'Invalid default param value given for param "%s". %s' % (p.name, e)
                    )
            self._defaultParamMap[p] = value
        return self

    def _copyValues(self, to: "P_", extra: Optional[Dict[Param, Any]] = None) -> "P_":
        paramMap = self._paramMap.copy()
        if isinstance(extra, dict):
            for param, value in extra.items():
                if isinstance(param, Param):
                    paramMap[param] = value
                else:
                    raise TypeError("Expecting a valid instance of Param, but received: %s" % param)
        elif extra is not None:
            raise TypeError("Expecting a dict, but received an object of type %s." % type(extra))
        for param in self.params:
            if param in self._defaultParamMap and to.hasParam(param.name):
                to._defaultParamMap[to.getParam(param.name)] = self._defaultParamMap[param]
            if param in paramMap and to.hasParam(param.name):
                to._set(**{param.name: paramMap[param]})
        return to

    def _resetUid(self: "P_", newUid: Any) -> "P_":
        newUid = str(newUid)
        self.uid = newUid
        newDefaultParamMap = dict()
        newParamMap = dict()
        for param in self.params:
            newParam = _copy.copy(param)
            newParam.parent = newUid
            if param in self._defaultParamMap:
                newDefaultParamMap[newParam] = self._defaultParamMap[param]
            if param in self._paramMap:
                newParamMap[newParam] = self._paramMap[param]
            param.parent = newUid
        self._defaultParamMap = newDefaultParamMap
        self._paramMap = newParamMap
        return self


P_ = TypeVar("P_", bound=Params)
