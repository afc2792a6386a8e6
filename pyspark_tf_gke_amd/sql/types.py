"""Spark SQL data types (the subset the reference's DataFrames carry: health.csv columns are
strings, integers/longs and doubles; ML adds vectors)."""
from __future__ import annotations

import torch


class DataType:
    simple = "unknown"
    torch_dtype = None

    def simpleString(self):  # noqa: N802 (pyspark naming)
        return self.simple

    def typeName(self):  # noqa: N802
        return self.simple

    def __repr__(self):
        return type(self).__name__ + "()"

    def __eq__(self, other):
        return type(self) is type(other)

    def __hash__(self):
        return hash(type(self).__name__)


class StringType(DataType):
    simple = "string"
    torch_dtype = torch.int32  # dictionary codes


class IntegerType(DataType):
    simple = "int"
    torch_dtype = torch.int32


class LongType(DataType):
    simple = "bigint"
    torch_dtype = torch.int64


class DoubleType(DataType):
    simple = "double"
    torch_dtype = torch.float64


class FloatType(DataType):
    simple = "float"
    torch_dtype = torch.float32


class BooleanType(DataType):
    simple = "boolean"
    torch_dtype = torch.bool


class TimestampType(DataType):
    simple = "timestamp"
    torch_dtype = torch.int64


class VectorUDT(DataType):
    simple = "vector"
    torch_dtype = torch.float32


class StructField:
    def __init__(self, name: str, dataType: DataType, nullable: bool = True):  # noqa: N803
        self.name, self.dataType, self.nullable = name, dataType, nullable

    def __repr__(self):
        return f"StructField('{self.name}', {self.dataType!r}, {self.nullable})"


class StructType:
    def __init__(self, fields=None):
        self.fields = list(fields or [])

    def add(self, name, dataType, nullable=True):  # noqa: N803
        self.fields.append(StructField(name, dataType, nullable))
        return self

    @property
    def names(self):
        return [f.name for f in self.fields]

    def __iter__(self):
        return iter(self.fields)

    def __len__(self):
        return len(self.fields)

    def __getitem__(self, k):
        if isinstance(k, str):
            for f in self.fields:
                if f.name == k:
                    return f
            raise KeyError(k)
        return self.fields[k]

    def simpleString(self):  # noqa: N802
        return "struct<" + ",".join(f"{f.name}:{f.dataType.simple}" for f in self.fields) + ">"

    def treeString(self) -> str:  # noqa: N802
        lines = ["root"]
        for f in self.fields:
            lines.append(f" |-- {f.name}: {f.dataType.simple} (nullable = {str(f.nullable).lower()})")
        return "\n".join(lines) + "\n"

    def __repr__(self):
        return f"StructType({self.fields!r})"


NUMERIC = (IntegerType, LongType, DoubleType, FloatType, BooleanType)


def from_torch(dt: torch.dtype) -> DataType:
    return {torch.int32: IntegerType(), torch.int64: LongType(), torch.float64: DoubleType(),
            torch.float32: FloatType(), torch.bool: BooleanType(), torch.uint8: BooleanType()}[dt]
