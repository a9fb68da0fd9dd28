"""Spark-SQL compatible data types and schemas.

Covers the types the reference lab exercises (``integer``, ``double`` and ML ``vector``, see
``DataQuality4MachineLearningApp.java:72,81,114`` printSchema calls) plus the rest of the CSV
type-inference lattice (null -> int -> long -> decimal -> double -> timestamp ->
boolean -> string).  Each type knows its physical device representation (torch dtype).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch

__all__ = [
    "DataType", "NullType", "BooleanType", "IntegerType", "LongType", "FloatType", "DoubleType",
    "StringType", "TimestampType", "DecimalType", "VectorUDT", "StructField", "StructType",
    "DataTypes", "parse_type_name", "is_numeric", "wider_numeric",
]


class DataType:
    _type_name = "data"
    _simple = "data"
    torch_dtype: Optional[torch.dtype] = None

    def typeName(self) -> str:
        return self._type_name

    def simpleString(self) -> str:
        return self._simple

    def __eq__(self, other):
        return type(self) is type(other)

    def __hash__(self):
        return hash(type(self).__name__)

    def __repr__(self):
        return type(self).__name__ + "()"


class NullType(DataType):
    _type_name = "null"
    _simple = "null"
    torch_dtype = torch.float64


class BooleanType(DataType):
    _type_name = "boolean"
    _simple = "boolean"
    torch_dtype = torch.bool


class IntegerType(DataType):
    _type_name = "integer"
    _simple = "int"
    torch_dtype = torch.int32


class LongType(DataType):
    _type_name = "long"
    _simple = "bigint"
    torch_dtype = torch.int64


class FloatType(DataType):
    _type_name = "float"
    _simple = "float"
    torch_dtype = torch.float32


class DoubleType(DataType):
    _type_name = "double"
    _simple = "double"
    torch_dtype = torch.float64


class StringType(DataType):
    _type_name = "string"
    _simple = "string"
    torch_dtype = None  # host-resident python list


class TimestampType(DataType):
    _type_name = "timestamp"
    _simple = "timestamp"
    torch_dtype = torch.int64  # microseconds since epoch


class DecimalType(DataType):
    """Integers too long for ``long`` (CSV inference lattice).  Stored as float64 on device."""

    def __init__(self, precision: int = 38, scale: int = 0):
        self.precision, self.scale = precision, scale

    _type_name = "decimal"
    torch_dtype = torch.float64

    def simpleString(self):
        return f"decimal({self.precision},{self.scale})"

    def typeName(self):
        return f"decimal({self.precision},{self.scale})"

    def __eq__(self, other):
        return isinstance(other, DecimalType) and (self.precision, self.scale) == (other.precision, other.scale)

    def __hash__(self):
        return hash(("decimal", self.precision, self.scale))


class VectorUDT(DataType):
    """``org.apache.spark.ml.linalg.VectorUDT``.  Physically a feature-major ``[d, n]`` tensor."""

    _type_name = "vector"
    _simple = "vector"
    torch_dtype = torch.float64


@dataclass
class StructField:
    name: str
    dataType: DataType
    nullable: bool = True
    metadata: Dict = field(default_factory=dict)

    def simpleString(self):
        return f"{self.name}:{self.dataType.simpleString()}"


class StructType:
    def __init__(self, fields: Optional[List[StructField]] = None):
        self.fields: List[StructField] = list(fields or [])
        self._index = None  # name -> field (first occurrence), built on demand

    def add(self, name, dataType, nullable=True, metadata=None):
        self.fields.append(StructField(name, dataType, nullable, metadata or {}))
        self._index = None
        return self

    def _idx(self):
        if self._index is None or len(self._index[1]) != len(self.fields):
            d = {}
            for f in self.fields:
                d.setdefault(f.name, f)
            self._index = (d, [f.name for f in self.fields], {k.lower(): k for k in reversed(list(d))})
        return self._index

    @property
    def names(self):
        # (a copy: callers may mutate it; the index tuple keeps its own list)
        return self._idx()[1][:]

    def fieldNames(self):
        return self.names

    def has(self, name) -> bool:
        return name in self._idx()[0]

    def resolve_ci(self, name):
        """Exact name if present, else the case-insensitive match (first field), else None."""
        d, _, lower = self._idx()
        if name in d:
            return name
        return lower.get(name.lower())

    def __getitem__(self, key):
        if isinstance(key, int):
            return self.fields[key]
        f = self._idx()[0].get(key)
        if f is None:
            raise KeyError(key)
        return f

    def __iter__(self):
        return iter(self.fields)

    def __len__(self):
        return len(self.fields)

    def __eq__(self, other):
        return isinstance(other, StructType) and [(f.name, f.dataType, f.nullable) for f in self.fields] == \
            [(f.name, f.dataType, f.nullable) for f in other.fields]

    def simpleString(self):
        return "struct<" + ",".join(f.simpleString() for f in self.fields) + ">"

    def treeString(self) -> str:
        """``StructType.treeString`` as printed by ``Dataset.printSchema``."""
        lines = ["root"]
        for f in self.fields:
            lines.append(f" |-- {f.name}: {f.dataType.typeName()} (nullable = {'true' if f.nullable else 'false'})")
        return "\n".join(lines) + "\n"

    def __repr__(self):
        return f"StructType({self.fields!r})"


class DataTypes:
    """Mirror of ``org.apache.spark.sql.types.DataTypes`` singletons (used at
    ``DataQuality4MachineLearningApp.java:47,49`` to declare UDF return types)."""

    NullType = NullType()
    BooleanType = BooleanType()
    IntegerType = IntegerType()
    LongType = LongType()
    FloatType = FloatType()
    DoubleType = DoubleType()
    StringType = StringType()
    TimestampType = TimestampType()


_NAMES = {
    "int": IntegerType, "integer": IntegerType, "bigint": LongType, "long": LongType,
    "double": DoubleType, "float": FloatType, "real": FloatType, "string": StringType,
    "boolean": BooleanType, "bool": BooleanType, "timestamp": TimestampType,
}


def parse_type_name(name: str) -> DataType:
    n = name.strip().lower()
    if n.startswith("decimal"):
        inner = n[len("decimal"):].strip("() ")
        if inner:
            p, _, s = inner.partition(",")
            return DecimalType(int(p), int(s or 0))
        return DecimalType(10, 0)
    if n not in _NAMES:
        raise ValueError(f"DataType {name} is not supported.")
    return _NAMES[n]()


_RANK = {BooleanType: 0, IntegerType: 1, LongType: 2, FloatType: 3, DecimalType: 4, DoubleType: 5}


def is_numeric(t: DataType) -> bool:
    return type(t) in (IntegerType, LongType, FloatType, DoubleType, DecimalType)


def wider_numeric(a: DataType, b: DataType) -> DataType:
    """Binary-operator type coercion (int op double -> double, etc.)."""
    if isinstance(a, NullType):
        return b
    if isinstance(b, NullType):
        return a
    ra, rb = _RANK.get(type(a), 5), _RANK.get(type(b), 5)
    if isinstance(a, FloatType) and isinstance(b, (LongType, DecimalType)) or \
            isinstance(b, FloatType) and isinstance(a, (LongType, DecimalType)):
        return DoubleType()
    if isinstance(a, DecimalType) or isinstance(b, DecimalType):
        return DoubleType() if max(ra, rb) >= 5 else (a if ra >= rb else b)
    return a if ra >= rb else b
